// RMSNorm and fused residual-add + RMSNorm.
//
// One 256/512-thread workgroup per token row (norm_threads, common.h); each lane owns VPT 16-byte vectors of
// the row, held in registers between the sum-of-squares pass and the scale
// pass, so the row is read from HBM exactly once and written once.
// fp32 accumulation, bf16 I/O. Weight may be bf16 (HF checkpoints) or fp32
// (GGUF stores norm weights as F32).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

// Token-id source of the gather mode (embedding lookup fused into the first
// RMSNorm of a decode step): id = src[row] >= 0 ? tok[src[row]] : ids[row]
// (tok = the previous graph step's sampled ids, src = this step's row in it:
// the decode lookahead of model_runner.py; src == nullptr: ids only).
struct GatherIds {
  const long* ids;
  const long* src;
  const long* tok;
  float scale;  // embedding multiplier (Gemma: sqrt(hidden) rounded to bf16), 1 = none
};

// kGather: x is the embedding table, row r reads table row id(r) (GatherIds), scales
// it by gi.scale (bf16(row * scale), as a bf16 tensor times a float scalar rounds) and
// also writes that row to `residual` (the layer-0 residual stream): one kernel
// instead of the id select + embedding gather + scale + residual copy + RMSNorm chain,
// with the same per-row arithmetic as the plain RMSNorm (bit-identical output).
template <int NT, int VPT, bool kAdd, bool kWF32, bool kGather = false>
__global__ __launch_bounds__(NT) void rmsnorm_kernel(
    unsigned short* __restrict__ out, unsigned short* __restrict__ residual,
    const unsigned short* __restrict__ x, const void* __restrict__ weight,
    int hidden, long x_stride, long out_stride, float eps, GatherIds gi = GatherIds{},
    unsigned char* __restrict__ out8 = nullptr, float* __restrict__ xs8 = nullptr) {
  static_assert(!(kAdd && kGather), "gather mode writes the residual, it does not add to it");
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const int nvec = hidden >> 3;
  long xrow = row;
  if constexpr (kGather) {
    const long sr = gi.src != nullptr ? gi.src[row] : -1;
    xrow = sr >= 0 ? gi.tok[sr] : gi.ids[row];
  }
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + xrow * x_stride);
  u16x8* rr = (kAdd || kGather) ? reinterpret_cast<u16x8*>(residual + (long)row * hidden) : nullptr;
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      u16x8 a = xr[idx];
      if constexpr (kAdd) {
        u16x8 b = rr[idx];
        u16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f = bf16_to_f32(a[j]) + bf16_to_f32(b[j]);
          s[j] = f32_to_bf16(f);
          v[i][j] = bf16_to_f32(s[j]);  // normalise the bf16-rounded residual
        }
        rr[idx] = s;
      } else {
        if constexpr (kGather) {
          if (gi.scale != 1.f) {
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = f32_to_bf16(bf16_to_f32(a[j]) * gi.scale);
          }
          rr[idx] = a;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf16_to_f32(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / hidden + eps);
  u16x8* orow = reinterpret_cast<u16x8*>(out + row * out_stride);
  u16x8 ov[VPT];
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float w[8];
      if constexpr (kWF32) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(weight) + idx * 2;
        f32x4 w0 = wp[0], w1 = wp[1];
#pragma unroll
        for (int j = 0; j < 4; ++j) { w[j] = w0[j]; w[j + 4] = w1[j]; }
      } else {
        u16x8 wv = reinterpret_cast<const u16x8*>(weight)[idx];
#pragma unroll
        for (int j = 0; j < 8; ++j) w[j] = bf16_to_f32(wv[j]);
      }
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(v[i][j] * inv * w[j]);
      orow[idx] = o;
      ov[i] = o;
    }
  }
  // optional per-token e4m3 copy (the FP8 W8A8 GEMM's input, = act_quant_fp8 of out)
  if (out8 != nullptr) row_e4m3<VPT, NT>(ov, nvec, row, hidden, out8, xs8, scratch);
}

template <bool kAdd, bool kWF32>
static void launch_rmsnorm_t(unsigned short* out, unsigned short* residual,
                             const unsigned short* x, const void* w, int rows,
                             int hidden, long x_stride, long out_stride, float eps,
                             hipStream_t s, unsigned char* o8, float* x8) {
  const int nvec = hidden / 8;
  dim3 grid(rows);
  if (norm_threads(hidden) == 256) {  // hidden < 4096: nvec < 512
    if (nvec <= 256)
      rmsnorm_kernel<256, 1, kAdd, kWF32><<<grid, 256, 0, s>>>(out, residual, x, w, hidden, x_stride, out_stride, eps, GatherIds{}, o8, x8);
    else
      rmsnorm_kernel<256, 2, kAdd, kWF32><<<grid, 256, 0, s>>>(out, residual, x, w, hidden, x_stride, out_stride, eps, GatherIds{}, o8, x8);
  } else {
    if (nvec <= 512)
      rmsnorm_kernel<512, 1, kAdd, kWF32><<<grid, 512, 0, s>>>(out, residual, x, w, hidden, x_stride, out_stride, eps, GatherIds{}, o8, x8);
    else if (nvec <= 1024)
      rmsnorm_kernel<512, 2, kAdd, kWF32><<<grid, 512, 0, s>>>(out, residual, x, w, hidden, x_stride, out_stride, eps, GatherIds{}, o8, x8);
    else
      rmsnorm_kernel<512, 4, kAdd, kWF32><<<grid, 512, 0, s>>>(out, residual, x, w, hidden, x_stride, out_stride, eps, GatherIds{}, o8, x8);
  }
}

// Per-head RMSNorm of the q and k heads inside the merged qkv rows, in place
// (Qwen3 / Gemma-3 q_norm, k_norm; applied before RoPE). One wave per
// (token, head), D <= 256 on 4 elements per lane; fp32 weights [D] (Gemma's
// 1 + w folded in at load).
__global__ __launch_bounds__(256) void qk_rmsnorm_kernel(unsigned short* __restrict__ qkv, long stride,
                                                         const float* __restrict__ qw,
                                                         const float* __restrict__ kw, int T, int nq, int nkv,
                                                         int D, float eps) {
  const int nh = nq + nkv;
  const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (long)T * nh) return;
  const int t = (int)(item / nh), h = (int)(item % nh);
  const int lane = threadIdx.x & 63;
  unsigned short* p = qkv + (long)t * stride + (long)h * D;
  const float* w = h < nq ? qw : kw;
  float v[4];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = lane + 64 * i;
    v[i] = d < D ? bf16_to_f32(p[d]) : 0.f;
    ss += v[i] * v[i];
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / D + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d = lane + 64 * i;
    if (d < D) p[d] = f32_to_bf16(v[i] * inv * w[d]);
  }
}

// Vector form for D = 8 * LPH (64 / 128 / 256): LPH lanes per head, one 16-byte
// load per lane, 64 / LPH heads per wave, the sum of squares reduced over the
// head's lane group with xor shuffles.
template <int LPH>
__global__ __launch_bounds__(256) void qk_rmsnorm_vec_kernel(unsigned short* __restrict__ qkv, long stride,
                                                             const float* __restrict__ qw,
                                                             const float* __restrict__ kw, int T, int nq, int nkv,
                                                             float eps) {
  constexpr int D = 8 * LPH, HPW = 64 / LPH;
  const int nh = nq + nkv;
  const int lane = threadIdx.x & 63;
  const long item = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * HPW + lane / LPH;
  const bool valid = item < (long)T * nh;
  const long it = valid ? item : 0;
  const int t = (int)(it / nh), h = (int)(it % nh);
  const int c = lane % LPH;
  u16x8* p = reinterpret_cast<u16x8*>(qkv + (long)t * stride + (long)h * D) + c;
  const u16x8 v = *p;
  float f[8], ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f[j] = bf16_to_f32(v[j]);
    ss += f[j] * f[j];
  }
#pragma unroll
  for (int o = LPH / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
  const float inv = rsqrtf(ss / D + eps);
  const f32x4* wp = reinterpret_cast<const f32x4*>(h < nq ? qw : kw) + 2 * c;
  const f32x4 w0 = wp[0], w1 = wp[1];
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = f32_to_bf16(f[j] * inv * w0[j]);
    o[j + 4] = f32_to_bf16(f[j + 4] * inv * w1[j]);
  }
  if (valid) *p = o;
}

void launch_qk_rmsnorm(void* qkv, long stride, const float* qw, const float* kw, int T, int nq, int nkv, int D,
                       float eps, hipStream_t s) {
  const long items = (long)T * (nq + nkv);
  if (items <= 0) return;
  auto* q = static_cast<unsigned short*>(qkv);
  const bool vec = stride % 8 == 0 && (D == 64 || D == 128 || D == 256);
  if (vec) {
    const int hpw = 64 / (D / 8);  // heads per wave
    const long waves = (items + hpw - 1) / hpw;
    const dim3 grid((unsigned)((waves + 3) / 4));
    if (D == 64) qk_rmsnorm_vec_kernel<8><<<grid, 256, 0, s>>>(q, stride, qw, kw, T, nq, nkv, eps);
    else if (D == 128) qk_rmsnorm_vec_kernel<16><<<grid, 256, 0, s>>>(q, stride, qw, kw, T, nq, nkv, eps);
    else qk_rmsnorm_vec_kernel<32><<<grid, 256, 0, s>>>(q, stride, qw, kw, T, nq, nkv, eps);
    return;
  }
  qk_rmsnorm_kernel<<<dim3((unsigned)((items + 3) / 4)), dim3(256), 0, s>>>(q, stride, qw, kw, T, nq, nkv, D, eps);
}

template <bool kWF32>
static void launch_embed_rmsnorm_t(unsigned short* out, unsigned short* residual, const unsigned short* table,
                                   const void* w, int rows, int hidden, float eps, GatherIds gi, hipStream_t s,
                                   unsigned char* o8, float* x8) {
  const int nvec = hidden / 8;
  dim3 grid(rows);
  const long xs = hidden;
  if (norm_threads(hidden) == 256) {
    if (nvec <= 256)
      rmsnorm_kernel<256, 1, false, kWF32, true><<<grid, 256, 0, s>>>(out, residual, table, w, hidden, xs, hidden, eps, gi, o8, x8);
    else
      rmsnorm_kernel<256, 2, false, kWF32, true><<<grid, 256, 0, s>>>(out, residual, table, w, hidden, xs, hidden, eps, gi, o8, x8);
  } else {
    if (nvec <= 512)
      rmsnorm_kernel<512, 1, false, kWF32, true><<<grid, 512, 0, s>>>(out, residual, table, w, hidden, xs, hidden, eps, gi, o8, x8);
    else if (nvec <= 1024)
      rmsnorm_kernel<512, 2, false, kWF32, true><<<grid, 512, 0, s>>>(out, residual, table, w, hidden, xs, hidden, eps, gi, o8, x8);
    else
      rmsnorm_kernel<512, 4, false, kWF32, true><<<grid, 512, 0, s>>>(out, residual, table, w, hidden, xs, hidden, eps, gi, o8, x8);
  }
}

void launch_embed_rmsnorm(void* out, void* residual, const void* table, const long* ids, const long* src,
                          const long* tok, const void* w, bool weight_f32, int rows, int hidden, float eps,
                          hipStream_t s, float scale, void* out8, float* xs8) {
  if (rows <= 0) return;
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  auto* t = static_cast<const unsigned short*>(table);
  auto* o8 = static_cast<unsigned char*>(out8);
  const GatherIds gi{ids, src, tok, scale};
  if (weight_f32) launch_embed_rmsnorm_t<true>(o, r, t, w, rows, hidden, eps, gi, s, o8, xs8);
  else launch_embed_rmsnorm_t<false>(o, r, t, w, rows, hidden, eps, gi, s, o8, xs8);
}

void launch_rmsnorm(void* out, void* residual, const void* x, const void* w,
                    bool weight_f32, int rows, int hidden, long x_stride,
                    long out_stride, float eps, hipStream_t s, void* out8, float* xs8) {
  auto* o8 = static_cast<unsigned char*>(out8);
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  auto* xi = static_cast<const unsigned short*>(x);
  if (residual) {
    if (weight_f32) launch_rmsnorm_t<true, true>(o, r, xi, w, rows, hidden, x_stride, out_stride, eps, s, o8, xs8);
    else launch_rmsnorm_t<true, false>(o, r, xi, w, rows, hidden, x_stride, out_stride, eps, s, o8, xs8);
  } else {
    if (weight_f32) launch_rmsnorm_t<false, true>(o, r, xi, w, rows, hidden, x_stride, out_stride, eps, s, o8, xs8);
    else launch_rmsnorm_t<false, false>(o, r, xi, w, rows, hidden, x_stride, out_stride, eps, s, o8, xs8);
  }
}

}  // namespace hipserve
