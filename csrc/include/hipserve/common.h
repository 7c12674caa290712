// hipserve — common device helpers for gfx950 (CDNA4, wave64).
//
// Everything here is written for MI355X directly: 64-lane wavefronts, 16-byte
// vector memory ops, bf16 <-> f32 via the native gfx950 converts.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define HS_DEVICE __device__ __forceinline__
#define HS_HOST_DEVICE __host__ __device__ __forceinline__

namespace hipserve {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// 16-byte vector register types (8 x bf16 as raw 16-bit lanes)
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

HS_DEVICE float bf16_to_f32(unsigned short x) {
  return __uint_as_float(static_cast<unsigned int>(x) << 16);
}

// Round-to-nearest-even; on gfx950 -O3 lowers to v_cvt_pk_bf16_f32 (NaN-safe).
HS_DEVICE unsigned short f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(unsigned short, b);
}

HS_DEVICE unsigned int pack_bf16x2(float lo, float hi) {
  return static_cast<unsigned int>(f32_to_bf16(lo)) |
         (static_cast<unsigned int>(f32_to_bf16(hi)) << 16);
}

// ---- wave64 reductions (xor butterflies over all 64 lanes) ----
// Wave reductions on the DPP crossbar: quad swaps, half-row and row mirrors (every lane
// then holds its 16-lane row's result), the row broadcasts 15 / 31 (lane 63 holds the
// wave's), and a readlane to broadcast it — six VALU steps instead of six dependent
// ds_bpermute round trips through the LDS crossbar. The result is wave-uniform.
template <int kCtrl, int kRowMask, bool kMax>
HS_DEVICE float dpp_step(float x) {
  const float y = __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, x), __builtin_bit_cast(int, x), kCtrl, kRowMask, 0xf,
                                         false));
  return kMax ? fmaxf(x, y) : x + y;
}
template <bool kMax>
HS_DEVICE float wave_reduce(float v) {
  // masked-off rows keep `old` = x: for the sum those rows must add 0, so the broadcast
  // steps use the explicit select below instead of dpp_step
  v = dpp_step<0xB1, 0xf, kMax>(v);   // quad_perm [1, 0, 3, 2]
  v = dpp_step<0x4E, 0xf, kMax>(v);   // quad_perm [2, 3, 0, 1]
  v = dpp_step<0x141, 0xf, kMax>(v);  // row_half_mirror
  v = dpp_step<0x140, 0xf, kMax>(v);  // row_mirror
  if constexpr (kMax) {
    v = dpp_step<0x142, 0xa, true>(v);  // row_bcast:15 -> rows 1, 3
    v = dpp_step<0x143, 0xc, true>(v);  // row_bcast:31 -> rows 2, 3
  } else {
    const float b15 = __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xa, 0xf, false));
    v += b15;  // rows 1, 3 (+0 elsewhere)
    const float b31 = __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xc, 0xf, false));
    v += b31;  // rows 2, 3
  }
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
HS_DEVICE float wave_sum(float v) { return wave_reduce<false>(v); }
HS_DEVICE float wave_max(float v) { return wave_reduce<true>(v); }

// Block-wide sum for blockDim.x <= 1024 (16 waves). `scratch` needs >= 16 floats.
HS_DEVICE float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? scratch[lane] : 0.f;
  r = wave_sum(r);
  __syncthreads();
  return r;
}

HS_DEVICE float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = (lane < nw) ? scratch[lane] : -INFINITY;
  r = wave_max(r);
  __syncthreads();
  return r;
}

// per-token dynamic e4m3 copy of a bf16 row for the W8A8 decode GEMM (fp8_decode.hip) and the FP8 prefill GEMM,
// bit-identical to act_quant_fp8 (prefill_gemm.hip) on the same bf16 values: xs = amax /
// 448 (1 for a zero row), q = sat(x * (448 / amax)) with the same conversions
HS_DEVICE uint2 e4m3_8(const u16x8 o, float inv) {
  float f[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = __builtin_amdgcn_fmed3f(bf16_to_f32(o[e]) * inv, -448.f, 448.f);
  uint2 r;
  r.x = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  r.x = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], (int)r.x, true);
  r.y = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  r.y = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], (int)r.y, true);
  return r;
}

// ---- paged KV cache elements: bf16 (unsigned short) or OCP e4m3 (unsigned char) ----
// The e4m3 cache (--kv-cache-dtype fp8) holds K / V with a per-tensor scale of 1 (vLLM's
// fp8 KV cache without calibrated scales): writers round the bf16 value to e4m3 (RNE,
// saturated to +-448), readers widen e4m3 -> bf16 exactly (v_cvt_scalef32_pk_bf16_fp8),
// so attention math is unchanged and only the stored K / V lose precision.
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
template <typename KV> struct KvVec;  // 8 cache elements in registers
template <> struct KvVec<unsigned short> { using T = u16x8; };
template <> struct KvVec<unsigned char> { using T = u32x2; };

HS_DEVICE u16x8 kv_widen8(const u16x8 v) { return v; }
// two e4m3 in the low 16 bits of w -> two bf16 (exact). The high pair goes through a shift
// rather than the instruction's word select: with op_sel the paged decode kernel read wrong
// keys on the GPU although a standalone probe of the same builtin matched (round 6)
HS_DEVICE unsigned kv_widen2(unsigned w) {
  return __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.f, false));
}
HS_DEVICE u16x8 kv_widen8(const u32x2 v) {
  const u32x4 r{kv_widen2(v[0]), kv_widen2(v[0] >> 16), kv_widen2(v[1]), kv_widen2(v[1] >> 16)};
  return __builtin_bit_cast(u16x8, r);
}
// 4 elements (the v1 prefill attention's V^T runs)
HS_DEVICE u16x4 kv_widen4(const u16x4 v) { return v; }
HS_DEVICE u16x4 kv_widen4(const unsigned v) {
  const u32x2 r{kv_widen2(v), kv_widen2(v >> 16)};
  return __builtin_bit_cast(u16x4, r);
}
HS_DEVICE unsigned char e4m3_1(unsigned short bf) {
  const float f = __builtin_amdgcn_fmed3f(bf16_to_f32(bf), -448.f, 448.f);
  return (unsigned char)((unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(f, 0.f, 0, false) & 0xff);
}
// 8 consecutive elements (16-byte bf16 / 8-byte e4m3 store)
HS_DEVICE void kv_store8(unsigned short* p, const u16x8 v) { *reinterpret_cast<u16x8*>(p) = v; }
HS_DEVICE void kv_store8(unsigned char* p, const u16x8 v) {
  const uint2 r = e4m3_8(v, 1.f);
  *reinterpret_cast<u32x2*>(p) = u32x2{r.x, r.y};
}
HS_DEVICE void kv_store1(unsigned short* p, unsigned short bf) { *p = bf; }
HS_DEVICE void kv_store1(unsigned char* p, unsigned short bf) { *p = e4m3_1(bf); }
template <typename KV>
HS_DEVICE typename KvVec<KV>::T kv_load8(const KV* p) {
  return *reinterpret_cast<const typename KvVec<KV>::T*>(p);
}
template <typename KV>
HS_DEVICE typename KvVec<KV>::T kv_load8_nt(const KV* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const typename KvVec<KV>::T*>(p));
}

template <int VPT, int NT>
HS_DEVICE void row_e4m3(const u16x8 (&ov)[VPT], int nvec, int row, int N, unsigned char* __restrict__ out8,
                        float* __restrict__ xs8, float* scratch) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
    if (threadIdx.x + i * NT < nvec)
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf16_to_f32(ov[i][j])));
  __syncthreads();  // scratch was the norm's reduction buffer
  amax = block_max(amax, scratch);
  const float inv = amax > 0.f ? 448.f / amax : 1.f;
  if (threadIdx.x == 0) xs8[row] = amax > 0.f ? amax / 448.f : 1.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) *reinterpret_cast<uint2*>(out8 + (long)row * N + idx * 8) = e4m3_8(ov[i], inv);
  }
}

HS_HOST_DEVICE int cdiv(int a, int b) { return (a + b - 1) / b; }

// SiLU(gate) * up on 8 bf16 lanes, fp32 math, one bf16 rounding (shared by the
// standalone silu_and_mul kernel and the decode GEMM's fused x staging, so both
// paths are bit-identical).
HS_DEVICE unsigned short silu_mul1(unsigned short g, unsigned short u) {
  const float gf = bf16_to_f32(g);
  const float s = gf / (1.f + __expf(-gf));
  return f32_to_bf16(s * bf16_to_f32(u));
}
HS_DEVICE u16x8 silu_mul8(const u16x8 g, const u16x8 u) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = silu_mul1(g[j], u[j]);
  return o;
}

// tanh-GELU(gate) * up (Gemma GeGLU, HF "gelu_pytorch_tanh"):
// 0.5 x (1 + tanh(y)) = x * sigmoid(2y), y = sqrt(2/pi) (x + 0.044715 x^3).
HS_DEVICE unsigned short gelu_mul1(unsigned short g, unsigned short u) {
  const float x = bf16_to_f32(g);
  const float y2 = 1.5957691216057308f * (x + 0.044715f * x * x * x);
  return f32_to_bf16(x / (1.f + __expf(-y2)) * bf16_to_f32(u));
}
HS_DEVICE u16x8 gelu_mul8(const u16x8 g, const u16x8 u) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = gelu_mul1(g[j], u[j]);
  return o;
}

// Row-norm launch policy shared by every RMSNorm-family kernel (norm.hip,
// decode_fused.hip) so they reduce in the same order and stay bit-identical:
// 512 threads from 4096 columns up (more loads in flight on the 1-row-per-CU
// decode shapes), 256 below.
HS_HOST_DEVICE int norm_threads(int hidden) { return hidden >= 4096 ? 512 : 256; }

// Bijective XCD-aware block remap (MI355X: 8 XCDs, blocks dealt round-robin).
// Blocks that share operand panels end up on the same XCD's L2.
HS_DEVICE int xcd_remap(int bid, int nwg) {
  constexpr int kXcd = 8;
  if (nwg < kXcd) return bid;
  const int q = nwg / kXcd, r = nwg % kXcd;
  const int xcd = bid % kXcd;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kXcd;
}

// Sum of S split-K slices of 8 consecutive fp32 partials (p, p + slice, ...),
// accumulated in slice order 0, 1, 2, ... into (lo, hi). Loads go out in batches
// of 8 slices with no branch or use between them: a plain load-add loop over a
// runtime S compiles to one s_waitcnt per slice — S serial HBM round trips
// (~0.7 us each), which is what made the decode split-K epilogues ~5.7 us at
// S = 8. Slices past S re-read slice S-1 (a cache hit, discarded).
constexpr int kSliceBatch = 8;

// RoPE rotation of the pair (a, b) by (c, s) with a FIXED rounding sequence (one
// explicit FMA each, never left to -ffp-contract): every kernel that rotates q / k
// (rope_cache, splitk_rope_cache, the fused decode attention) agrees bit for bit.
HS_DEVICE void rope_rot(float a, float b, float c, float s, float& ra, float& rb) {
  ra = __builtin_fmaf(a, c, -(b * s));
  rb = __builtin_fmaf(b, c, a * s);
}

HS_DEVICE void sum_slices8(f32x4& lo, f32x4& hi, const float* __restrict__ p, long slice, int S) {
  for (int s0 = 0; s0 < S; s0 += kSliceBatch) {
    f32x4 a[kSliceBatch], b[kSliceBatch];
#pragma unroll
    for (int j = 0; j < kSliceBatch; ++j) {
      const float* q = p + min(s0 + j, S - 1) * slice;
      a[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q));
      b[j] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q + 4));
    }
    if (s0 == 0) {
      lo = a[0];
      hi = b[0];
    } else {
      lo += a[0];
      hi += b[0];
    }
#pragma unroll
    for (int j = 1; j < kSliceBatch; ++j) {
      if (s0 + j < S) {
        lo += a[j];
        hi += b[j];
      }
    }
  }
}

}  // namespace hipserve
