// Skinny bf16 GEMM for decode batches (SURVEY K6/K7/K9 at M <= 64):
//   out[M, N] = x[M, K] . W[N, K]^T      (W row-major [N][K], fp32 accumulate)
//
// Decode GEMMs are HBM-bound weight streams. gfx950 mapping:
//  * out^T = W . x^T on v_mfma_f32_16x16x32_bf16: A = 16 W rows, B = x^T with up
//    to 4 m-tiles of 16 rows, so each W fragment feeds MT MFMAs;
//  * the k order inside each 256-k chunk is permuted so every lane streams 128
//    CONTIGUOUS bytes of its W row (8 x 16-byte loads; a row's 4 lane groups cover
//    512 B) straight into VGPRs — weights are read once, never staged in LDS
//    (guide: GEMV / M<=16 weight streams);
//  * KW waves of a workgroup split K and are reduced through LDS at the end, so
//    small-N projections (o_proj N=4096) still put >= 8 waves on every CU without
//    a split-K global reduction;
//  * RT row tiles per wave share every x fragment (halves x re-reads for large K);
//  * one chunk of W is always in flight ahead of the MFMAs (register double buffer).
// hipBLASLt stays the path for shapes where it is faster (chosen by autotune in
// hipserve/ops/gemm.py).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

template <int MT, int RT, int KW>
__global__ __launch_bounds__(64 * KW) void skinny_gemm_kernel(
    unsigned short* __restrict__ out, const unsigned short* __restrict__ x, long x_stride,
    const unsigned short* __restrict__ w, long out_stride, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [KW][RT*MT][64][4]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * (16 * RT);
  const int kw = K / KW;             // multiple of 256 (host-checked)
  const int k0 = wave * kw, k1 = k0 + kw;
  const unsigned short* wr[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) wr[r] = w + (long)min(n0 + 16 * r + c, N - 1) * K + 64 * g;
  const unsigned short* xr[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xr[t] = x + (long)min(16 * t + c, M - 1) * x_stride + 64 * g;

  f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  u16x8 a[RT][8], an[RT][8];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int s = 0; s < 8; ++s) a[r][s] = *reinterpret_cast<const u16x8*>(wr[r] + k0 + 8 * s);

  for (int kk = k0; kk < k1; kk += 256) {
    const int kn = kk + 256;
    if (kn < k1) {
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int s = 0; s < 8; ++s) an[r][s] = *reinterpret_cast<const u16x8*>(wr[r] + kn + 8 * s);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xr[t] + kk + 8 * s);
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[r][s]),
                                                               __builtin_bit_cast(bf16x8, b), acc[r][t], 0, 0, 0);
      }
    }
    if (kn < k1) {
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int s = 0; s < 8; ++s) a[r][s] = an[r][s];
    }
  }

  if constexpr (KW > 1) {
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int t = 0; t < MT; ++t)
        *reinterpret_cast<f32x4*>(red + (((wave * RT + r) * MT + t) * 64 + lane) * 4) = acc[r][t];
    __syncthreads();
    // wave w reduces tiles (r, t) with (r*MT + t) % KW == w
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        if ((r * MT + t) % KW != wave) continue;
        f32x4 s = {0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < KW; ++q) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(red + (((q * RT + r) * MT + t) * 64 + lane) * 4);
          s += v;
        }
        acc[r][t] = s;
      }
  }
  // C layout: col m = 16t + c, rows n = n0 + 16r + 4g + j
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if (KW > 1 && (r * MT + t) % KW != wave) continue;
      const int m = 16 * t + c;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + 16 * r + 4 * g + j;
        if (n < N) out[m * out_stride + n] = f32_to_bf16(acc[r][t][j]);
      }
    }
}

template <int MT, int RT, int KW>
static void launch_t(void* out, const void* x, long x_stride, const void* w, long out_stride, int M, int N,
                     int K, hipStream_t s) {
  dim3 grid((N + 16 * RT - 1) / (16 * RT)), block(64 * KW);
  const size_t smem = KW > 1 ? (size_t)KW * RT * MT * 64 * 4 * sizeof(float) : 0;
  skinny_gemm_kernel<MT, RT, KW><<<grid, block, smem, s>>>(
      static_cast<unsigned short*>(out), static_cast<const unsigned short*>(x), x_stride,
      static_cast<const unsigned short*>(w), out_stride, M, N, K);
}

template <int MT>
static bool launch_mt(void* out, const void* x, long x_stride, const void* w, long out_stride, int M, int N,
                      int K, int rt, int kw, hipStream_t s) {
#define HS_SK(RT_, KW_) \
  if (rt == RT_ && kw == KW_) { launch_t<MT, RT_, KW_>(out, x, x_stride, w, out_stride, M, N, K, s); return true; }
  HS_SK(1, 1) HS_SK(1, 2) HS_SK(1, 4) HS_SK(1, 8) HS_SK(1, 16)
  HS_SK(2, 1) HS_SK(2, 2) HS_SK(2, 4) HS_SK(2, 8)
#undef HS_SK
  return false;
}

// Returns false when (rt, kw) is not a compiled configuration.
bool launch_skinny_gemm(void* out, const void* x, long x_stride, const void* w, long out_stride, int M,
                        int N, int K, int rt, int kw, hipStream_t s) {
  if (M <= 16) return launch_mt<1>(out, x, x_stride, w, out_stride, M, N, K, rt, kw, s);
  if (M <= 32) return launch_mt<2>(out, x, x_stride, w, out_stride, M, N, K, rt, kw, s);
  return launch_mt<4>(out, x, x_stride, w, out_stride, M, N, K, rt, kw, s);
}

}  // namespace hipserve
