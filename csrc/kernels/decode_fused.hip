// Split-K partial reductions fused with the op that follows them in a decode
// layer (SURVEY §3.F hot loop, K2/K3 fused into K6/K7/K9's epilogue).
//
// The decode GEMMs (decode_gemm.hip, DG_PARTIAL) leave fp32 partials
// ws[S, M, N]; instead of a reduce kernel followed by a separate elementwise
// kernel (each ~5 us at decode sizes, almost all of it launch + dependent-load
// latency, profiles/r1_bench_llama3_8b_v3_trace.md), ONE kernel sums the slices
// and applies the next op:
//   * splitk_add_rmsnorm: o_proj / down_proj -> residual add -> RMSNorm
//     (the next layer's input_layernorm, or the final norm);
//   * splitk_rope_cache:  qkv_proj -> RoPE on q, k -> q back into the qkv buffer,
//     k / v into the paged cache.
// Both round exactly where the unfused chain rounds (bf16 after the sum, bf16
// residual), so the fused and unfused decode paths are bit-identical.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

// sum over S slices of 8 consecutive fp32 partials (batched loads, common.h),
// rounded to bf16 like the unfused reduce output, returned as fp32
// x = bf16(x + b) for 8 bf16 bias values (torch's bf16 add of the bias vector)
HS_DEVICE void add_bias8(float (&x)[8], const unsigned short* __restrict__ b) {
  const u16x8 v = *reinterpret_cast<const u16x8*>(b);
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = bf16_to_f32(f32_to_bf16(x[j] + bf16_to_f32(v[j])));
}

// 8 bf16 values -> f16 in the quantised decode GEMM's staging pair order
// {0, 2, 1, 3, 4, 6, 5, 7} (gguf_mfma.hip kX16): bf16 -> fp32 exact, -> f16 round to
// nearest — the conversion the GEMM would otherwise run in every workgroup
HS_DEVICE u16x8 f16_pairs8(const u16x8 v) {
  constexpr int ord[8] = {0, 2, 1, 3, 4, 6, 5, 7};
  u16x8 h;
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = __builtin_bit_cast(unsigned short, static_cast<_Float16>(bf16_to_f32(v[ord[j]])));
  return h;
}

HS_DEVICE void sum8_bf16(float (&o)[8], const float* __restrict__ p, long slice, int S) {
  f32x4 lo, hi;
  sum_slices8(lo, hi, p, slice, S);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = bf16_to_f32(f32_to_bf16(lo[j]));
    o[j + 4] = bf16_to_f32(f32_to_bf16(hi[j]));
  }
}

template <int NT, int VPT, bool kWF32>
__global__ __launch_bounds__(NT) void splitk_add_rmsnorm_kernel(unsigned short* __restrict__ out,
                                                                 unsigned short* __restrict__ residual,
                                                                 const float* __restrict__ ws, int S,
                                                                 const void* __restrict__ weight, int M, int N,
                                                                 float eps, unsigned short* __restrict__ out16,
                                                                 unsigned char* __restrict__ out8,
                                                                 float* __restrict__ xs8) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = N >> 3;
  const long slice = (long)M * N;
  // the norm weight and the residual do not depend on the reduction: issue their
  // loads first and keep them raw, so no s_waitcnt sits in front of the partials
  f32x4 wf[VPT][2];
  u16x8 wb[VPT], res[VPT];
  u16x8* rr = reinterpret_cast<u16x8*>(residual + (long)row * N);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      if constexpr (kWF32) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(weight) + idx * 2;
        wf[i][0] = wp[0];
        wf[i][1] = wp[1];
      } else {
        wb[i] = reinterpret_cast<const u16x8*>(weight)[idx];
      }
      res[i] = rr[idx];
    }
  }
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float h[8];
      sum8_bf16(h, ws + (long)row * N + idx * 8, slice, S);
      u16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        r[j] = f32_to_bf16(h[j] + bf16_to_f32(res[i][j]));
        v[i][j] = bf16_to_f32(r[j]);
        ss += v[i][j] * v[i][j];
      }
      rr[idx] = r;
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / N + eps);
  u16x8* orow = reinterpret_cast<u16x8*>(out + (long)row * N);
  u16x8 ov[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float wj;
        if constexpr (kWF32) wj = wf[i][j >> 2][j & 3];
        else wj = bf16_to_f32(wb[i][j]);
        o[j] = f32_to_bf16(v[i][j] * inv * wj);
      }
      orow[idx] = o;
      ov[i] = o;
      if (out16 != nullptr) reinterpret_cast<u16x8*>(out16 + (long)row * N)[idx] = f16_pairs8(o);
    }
  }
  if (out8 != nullptr) row_e4m3<VPT, NT>(ov, nvec, row, N, out8, xs8, scratch);
}

template <bool kWF32>
static void add_rmsnorm_t(void* out, void* residual, const float* ws, int S, const void* w, int M, int N, float eps,
                          hipStream_t s, unsigned short* o16, unsigned char* o8, float* x8) {
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  const int nvec = N / 8;
  if (norm_threads(N) == 256) {
    if (nvec <= 256) splitk_add_rmsnorm_kernel<256, 1, kWF32><<<M, 256, 0, s>>>(o, r, ws, S, w, M, N, eps, o16, o8, x8);
    else splitk_add_rmsnorm_kernel<256, 2, kWF32><<<M, 256, 0, s>>>(o, r, ws, S, w, M, N, eps, o16, o8, x8);
  } else {
    if (nvec <= 512) splitk_add_rmsnorm_kernel<512, 1, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, w, M, N, eps, o16, o8, x8);
    else if (nvec <= 1024) splitk_add_rmsnorm_kernel<512, 2, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, w, M, N, eps, o16, o8, x8);
    else splitk_add_rmsnorm_kernel<512, 4, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, w, M, N, eps, o16, o8, x8);
  }
}

void launch_splitk_add_rmsnorm(void* out, void* residual, const float* ws, int S, const void* w, bool weight_f32,
                               int M, int N, float eps, hipStream_t s, void* out16, void* out8, float* xs8) {
  if (M <= 0) return;
  auto* o16 = static_cast<unsigned short*>(out16);
  auto* o8 = static_cast<unsigned char*>(out8);
  if (weight_f32) add_rmsnorm_t<true>(out, residual, ws, S, w, M, N, eps, s, o16, o8, xs8);
  else add_rmsnorm_t<false>(out, residual, ws, S, w, M, N, eps, s, o16, o8, xs8);
}

// Sandwich-norm epilogue (Gemma-3: post-attention / post-feedforward RMSNorm on the
// projection output BEFORE the residual add): h = bf16(sum_s ws); p = bf16(RMSNorm(h)
// * w_post); residual = bf16(p + residual); out = RMSNorm(residual) * w_next — the
// unfused chain splitk_reduce -> rmsnorm -> fused_add_rmsnorm in one kernel, with each
// norm reduced in the row-norm kernels' order (same thread -> element map), so the
// result is bit-identical.
template <bool kWF32>
HS_DEVICE void norm_w8(float (&w)[8], const void* __restrict__ weight, int idx) {
  if constexpr (kWF32) {
    const f32x4* wp = reinterpret_cast<const f32x4*>(weight) + idx * 2;
    const f32x4 w0 = wp[0], w1 = wp[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = w0[j];
      w[j + 4] = w1[j];
    }
  } else {
    const u16x8 wv = reinterpret_cast<const u16x8*>(weight)[idx];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = bf16_to_f32(wv[j]);
  }
}

template <int NT, int VPT, bool kWF32>
__global__ __launch_bounds__(NT) void splitk_post_add_rmsnorm_kernel(unsigned short* __restrict__ out,
                                                                      unsigned short* __restrict__ residual,
                                                                      const float* __restrict__ ws, int S,
                                                                      const void* __restrict__ w_post,
                                                                      const void* __restrict__ w_next, int M, int N,
                                                                      float eps, unsigned short* __restrict__ out16,
                                                                      unsigned char* __restrict__ out8,
                                                                      float* __restrict__ xs8) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = N >> 3;
  const long slice = (long)M * N;
  u16x8 res[VPT];
  u16x8* rr = reinterpret_cast<u16x8*>(residual + (long)row * N);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) res[i] = rr[idx];
  }
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      sum8_bf16(v[i], ws + (long)row * N + idx * 8, slice, S);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv1 = rsqrtf(ss / N + eps);
  float ss2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float w[8];
      norm_w8<kWF32>(w, w_post, idx);
      u16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = bf16_to_f32(f32_to_bf16(v[i][j] * inv1 * w[j]));
        r[j] = f32_to_bf16(p + bf16_to_f32(res[i][j]));
        v[i][j] = bf16_to_f32(r[j]);
        ss2 += v[i][j] * v[i][j];
      }
      rr[idx] = r;
    }
  }
  ss2 = block_sum(ss2, scratch);
  const float inv2 = rsqrtf(ss2 / N + eps);
  u16x8* orow = reinterpret_cast<u16x8*>(out + (long)row * N);
  u16x8 ov[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float w[8];
      norm_w8<kWF32>(w, w_next, idx);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(v[i][j] * inv2 * w[j]);
      orow[idx] = o;
      ov[i] = o;
      if (out16 != nullptr) reinterpret_cast<u16x8*>(out16 + (long)row * N)[idx] = f16_pairs8(o);
    }
  }
  if (out8 != nullptr) row_e4m3<VPT, NT>(ov, nvec, row, N, out8, xs8, scratch);
}

template <bool kWF32>
static void post_add_rmsnorm_t(void* out, void* residual, const float* ws, int S, const void* wp, const void* wn,
                               int M, int N, float eps, hipStream_t s, unsigned short* o16, unsigned char* o8,
                               float* x8) {
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  const int nvec = N / 8;
  if (norm_threads(N) == 256) {
    if (nvec <= 256) splitk_post_add_rmsnorm_kernel<256, 1, kWF32><<<M, 256, 0, s>>>(o, r, ws, S, wp, wn, M, N, eps, o16, o8, x8);
    else splitk_post_add_rmsnorm_kernel<256, 2, kWF32><<<M, 256, 0, s>>>(o, r, ws, S, wp, wn, M, N, eps, o16, o8, x8);
  } else {
    if (nvec <= 512) splitk_post_add_rmsnorm_kernel<512, 1, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, wp, wn, M, N, eps, o16, o8, x8);
    else if (nvec <= 1024) splitk_post_add_rmsnorm_kernel<512, 2, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, wp, wn, M, N, eps, o16, o8, x8);
    else splitk_post_add_rmsnorm_kernel<512, 4, kWF32><<<M, 512, 0, s>>>(o, r, ws, S, wp, wn, M, N, eps, o16, o8, x8);
  }
}

void launch_splitk_post_add_rmsnorm(void* out, void* residual, const float* ws, int S, const void* w_post,
                                    const void* w_next, bool weight_f32, int M, int N, float eps, hipStream_t s,
                                    void* out16, void* out8, float* xs8) {
  if (M <= 0) return;
  auto* o16 = static_cast<unsigned short*>(out16);
  auto* o8 = static_cast<unsigned char*>(out8);
  if (weight_f32) post_add_rmsnorm_t<true>(out, residual, ws, S, w_post, w_next, M, N, eps, s, o16, o8, xs8);
  else post_add_rmsnorm_t<false>(out, residual, ws, S, w_post, w_next, M, N, eps, s, o16, o8, xs8);
}

// The rope_cache kernel (rope_cache.hip) reading its input from the split-K
// partials instead of a bf16 qkv row. Work item = one 8-wide chunk: (q/k head,
// chunk) pairs first, then the v chunks; 64-thread workgroups over
// (token, item block) so a 64-token decode batch spreads over ~450 workgroups
// instead of 64 (the partial reads are per-CU-bandwidth bound at one WG per token).
//
// Family extras, bit-identical to the unfused chain (GEMM -> bias add -> qk_rmsnorm ->
// rope_cache): bias (Qwen2: bf16 [N], added to the bf16-rounded sum and rounded
// again) and per-head q/k RMSNorm (Qwen3: fp32 weights [D]; a head's lanes are
// consecutive, its sum of squares is reduced in qk_rmsnorm_vec_kernel's order: each
// lane's two chunks (d and d + D/2) are the kernel's first xor pair, then xor 4, 2, 1).
template <int kMode, bool kNorm, typename KV>
__global__ __launch_bounds__(64) void splitk_rope_cache_kernel(
    unsigned short* __restrict__ qkv, long qkv_stride, const float* __restrict__ ws, int S,
    const long* __restrict__ positions, const long* __restrict__ slots, const float* __restrict__ cos_sin,
    KV* __restrict__ k_cache, KV* __restrict__ v_cache, int T, int nq, int nkv, int D,
    int block_size, const unsigned short* __restrict__ bias, const float* __restrict__ qw,
    const float* __restrict__ kw, float eps) {
  const int t = blockIdx.x;
  const int it = blockIdx.y * 64 + threadIdx.x;
  const int half = D / 2;
  const int qk_chunks = kMode == 0 ? half / 8 : D / 8;  // work items per q/k head
  const int n_qk = (nq + nkv) * qk_chunks;
  const int n_v = nkv * (D / 8);
  if (it >= n_qk + n_v) return;
  const long pos = positions[t];
  const long slot = slots[t];
  const int N = (nq + 2 * nkv) * D;
  const long slice = (long)T * N;
  const float* wrow = ws + (long)t * N;
  const float* cs = cos_sin + pos * D;
  unsigned short* row = qkv + t * qkv_stride;
  const long blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? (int)(slot % block_size) : 0;

  if (it >= n_qk) {  // V: transposed cache block (tokens contiguous per d)
    if (slot < 0) return;
    const int iv = it - n_qk, kh = iv / (D / 8), c = iv % (D / 8);
    float x[8];
    sum8_bf16(x, wrow + (nq + nkv) * D + kh * D + c * 8, slice, S);
    if (bias != nullptr) add_bias8(x, bias + (nq + nkv) * D + kh * D + c * 8);
    KV* vc = v_cache + (blk * nkv + kh) * (long)D * block_size + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) kv_store1(vc + (c * 8 + j) * block_size, f32_to_bf16(x[j]));
    return;
  }
  const int h = it / qk_chunks, c = it % qk_chunks;
  if (h >= nq && slot < 0) return;
  if constexpr (kMode == 0) {
    float x[8], y[8];
    sum8_bf16(x, wrow + h * D + c * 8, slice, S);
    sum8_bf16(y, wrow + h * D + half + c * 8, slice, S);
    if (bias != nullptr) {
      add_bias8(x, bias + h * D + c * 8);
      add_bias8(y, bias + h * D + half + c * 8);
    }
    if constexpr (kNorm) {
      float ss = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
#pragma unroll
      for (int j = 0; j < 8; ++j) s2 += y[j] * y[j];
      ss += s2;
      for (int o = qk_chunks / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float inv = rsqrtf(ss / D + eps);
      const float* nw = h < nq ? qw : kw;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        x[j] = bf16_to_f32(f32_to_bf16(x[j] * inv * nw[c * 8 + j]));
        y[j] = bf16_to_f32(f32_to_bf16(y[j] * inv * nw[half + c * 8 + j]));
      }
    }
    u16x8 va, vb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float co = cs[c * 8 + j], si = cs[half + c * 8 + j];
      float ra, rb;
      rope_rot(x[j], y[j], co, si, ra, rb);
      va[j] = f32_to_bf16(ra);
      vb[j] = f32_to_bf16(rb);
    }
    if (h < nq) {
      *reinterpret_cast<u16x8*>(row + h * D + c * 8) = va;
      *reinterpret_cast<u16x8*>(row + h * D + half + c * 8) = vb;
    } else {
      KV* dst = k_cache + ((blk * nkv + (h - nq)) * block_size + off) * (long)D;
      kv_store8(dst + c * 8, va);
      kv_store8(dst + half + c * 8, vb);
    }
  } else {
    float x[8];
    sum8_bf16(x, wrow + h * D + c * 8, slice, S);
    if (bias != nullptr) add_bias8(x, bias + h * D + c * 8);
    u16x8 v;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int i = c * 4 + p;
      const float co = cs[i], si = cs[half + i];
      float ra, rb;
      rope_rot(x[2 * p], x[2 * p + 1], co, si, ra, rb);
      v[2 * p] = f32_to_bf16(ra);
      v[2 * p + 1] = f32_to_bf16(rb);
    }
    if (h < nq) *reinterpret_cast<u16x8*>(row + h * D + c * 8) = v;
    else kv_store8(k_cache + ((blk * nkv + (h - nq)) * block_size + off) * (long)D + c * 8, v);
  }
}

template <typename KV>
static void splitk_rope_cache_t(unsigned short* q, long qkv_stride, const float* ws, int S, const long* positions,
                                const long* slots, const float* cos_sin, KV* kc, KV* vc, int T, int nq, int nkv,
                                int D, int block_size, int mode, hipStream_t s, const unsigned short* b,
                                const float* qw, const float* kw, float eps) {
  const int qk_chunks = mode == 0 ? D / 16 : D / 8;
  const int items = (nq + nkv) * qk_chunks + nkv * (D / 8);
  const dim3 grid(T, (items + 63) / 64);
  if (mode == 0 && qw != nullptr)
    splitk_rope_cache_kernel<0, true, KV><<<grid, 64, 0, s>>>(q, qkv_stride, ws, S, positions, slots, cos_sin, kc,
                                                               vc, T, nq, nkv, D, block_size, b, qw, kw, eps);
  else if (mode == 0)
    splitk_rope_cache_kernel<0, false, KV><<<grid, 64, 0, s>>>(q, qkv_stride, ws, S, positions, slots, cos_sin, kc,
                                                                vc, T, nq, nkv, D, block_size, b, nullptr, nullptr,
                                                                eps);
  else
    splitk_rope_cache_kernel<1, false, KV><<<grid, 64, 0, s>>>(q, qkv_stride, ws, S, positions, slots, cos_sin, kc,
                                                                vc, T, nq, nkv, D, block_size, b, nullptr, nullptr,
                                                                eps);
}

void launch_splitk_rope_cache(void* qkv, long qkv_stride, const float* ws, int S, const long* positions,
                              const long* slots, const float* cos_sin, void* k_cache, void* v_cache, int T, int nq,
                              int nkv, int D, int block_size, int mode, hipStream_t s, const void* bias,
                              const float* qw, const float* kw, float eps, bool kv_f8) {
  if (T <= 0) return;
  auto* q = static_cast<unsigned short*>(qkv);
  auto* b = static_cast<const unsigned short*>(bias);
  if (kv_f8)
    splitk_rope_cache_t(q, qkv_stride, ws, S, positions, slots, cos_sin, static_cast<unsigned char*>(k_cache),
                        static_cast<unsigned char*>(v_cache), T, nq, nkv, D, block_size, mode, s, b, qw, kw, eps);
  else
    splitk_rope_cache_t(q, qkv_stride, ws, S, positions, slots, cos_sin, static_cast<unsigned short*>(k_cache),
                        static_cast<unsigned short*>(v_cache), T, nq, nkv, D, block_size, mode, s, b, qw, kw, eps);
}

// GLU over the split-K partials of a merged [gate | up] projection in the plain
// (non-interleaved) layout — the GGUF decode GEMM's output (gguf_mfma.hip):
// act[m, j] = act(bf16(sum_s gate)) * bf16(sum_s up), bit-identical to the reduce
// followed by silu_and_mul / gelu_and_mul. grid (M, ceil(I / 2048)), 8 per thread.
template <bool kGelu>
__global__ __launch_bounds__(256) void splitk_glu_kernel(unsigned short* __restrict__ act, long act_stride,
                                                         const float* __restrict__ ws, int S, int M, int I,
                                                         unsigned short* __restrict__ act16) {
  const int m = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c * 8 >= I) return;
  const long N = 2L * I, slice = (long)M * N;
  float g[8], u[8];
  sum8_bf16(g, ws + m * N + c * 8, slice, S);
  sum8_bf16(u, ws + m * N + I + c * 8, slice, S);
  u16x8 gb, ub;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gb[j] = f32_to_bf16(g[j]);
    ub[j] = f32_to_bf16(u[j]);
  }
  const u16x8 o = kGelu ? gelu_mul8(gb, ub) : silu_mul8(gb, ub);
  *reinterpret_cast<u16x8*>(act + m * act_stride + c * 8) = o;
  if (act16 != nullptr) *reinterpret_cast<u16x8*>(act16 + m * act_stride + c * 8) = f16_pairs8(o);
}

void launch_splitk_glu(void* act, long act_stride, const float* ws, int S, int M, int I, bool gelu, hipStream_t s,
                       void* act16) {
  if (M <= 0) return;
  const dim3 grid(M, (I / 8 + 255) / 256);
  auto* a = static_cast<unsigned short*>(act);
  auto* a16 = static_cast<unsigned short*>(act16);
  if (gelu) splitk_glu_kernel<true><<<grid, 256, 0, s>>>(a, act_stride, ws, S, M, I, a16);
  else splitk_glu_kernel<false><<<grid, 256, 0, s>>>(a, act_stride, ws, S, M, I, a16);
}

}  // namespace hipserve
