// Decode GEMM v3 for the weight-streaming regime (SURVEY K6/K7/K9, M <= 64):
//   out[M, N] = x[M, K] . W[N, K]^T      (bf16 in/out, fp32 accumulate)
//
// Why not the skinny kernel (one x read per 16 W rows): at M = 64 the activation
// re-reads from L2 (M/16 = 4x the weight bytes) throttle the HBM stream. Here
//  * a workgroup owns NW = 16*RT*NWAVES weight rows and one K slice; the x slice
//    [16*MT, 256] for the current 256-k step is staged in LDS (double-buffered,
//    528 B rows = conflict-free ds_read_b128) and shared by all waves, so L2->CU
//    activation traffic drops to M/NW of the weight bytes;
//  * MFMA k order is permuted so that each 16-byte load instruction of a wave
//    covers 16 rows x 64 contiguous bytes (4 lane groups side by side) rather than
//    64 scattered 16-byte pieces; two 256-k steps (512 B per row each) are kept
//    in flight in a VGPR ring ahead of the MFMAs — weights are read exactly once;
//  * out^T = W . x^T on v_mfma_f32_16x16x32_bf16: each W fragment feeds MT MFMAs
//    and each LDS x fragment feeds RT MFMAs;
//  * small-N projections (o_proj / down N = 4096 -> 32 workgroups of 128 rows) are
//    split over K into S slices so the grid covers all 256 CUs; slices write fp32
//    partials [S, M, N] and `splitk_reduce` sums them (a kernel boundary instead of
//    cross-XCD fences: the 8 L2s are not coherent with each other mid-kernel).
//  * blockIdx -> (slice, tile) is slice-major so the 8 XCDs (round-robin dispatch)
//    each walk disjoint weight rows of one slice.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int DG_LDS_ROW = 264;  // 256 + 8 bf16 pad -> 528 B row stride

template <int MT, int RT, int NWAVES>
__global__ __launch_bounds__(64 * NWAVES) void decode_gemm_kernel(
    unsigned short* __restrict__ out, long out_stride, float* __restrict__ ws,
    const unsigned short* __restrict__ x, long x_stride, const unsigned short* __restrict__ w,
    int M, int N, int K, int S, int tiles) {
  constexpr int NW = 16 * RT * NWAVES;
  constexpr int XR = 16 * MT;                 // x rows staged (padded M)
  constexpr int NT = 64 * NWAVES;             // threads
  constexpr int XPASS = XR * 32 / NT;         // 16-byte x loads per thread per step
  __shared__ __attribute__((aligned(16))) unsigned short xs[2][XR * DG_LDS_ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int split = blockIdx.x / tiles, tile = blockIdx.x - split * tiles;
  const int ks = K / S, k0 = split * ks, nsteps = ks / 256;
  const int nbase = tile * NW + wave * 16 * RT;

  const unsigned short* wr[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) wr[r] = w + (long)min(nbase + 16 * r + c, N - 1) * K + k0 + 8 * g;

  // x staging: thread -> (row, 16-byte column chunk)
  u16x8 xv[XPASS];
  auto load_x = [&](int step) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      xv[p] = row < M ? *reinterpret_cast<const u16x8*>(x + (long)row * x_stride + k0 + step * 256 + col)
                      : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      *reinterpret_cast<u16x8*>(&xs[buf][row * DG_LDS_ROW + col]) = xv[p];
    }
  };

  f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weights: 3-deep register ring (two 256-k steps in flight while one is consumed);
  // x: LDS double buffer, one step ahead
  u16x8 a0[RT][8], a1[RT][8], a2[RT][8];
  auto load_w = [&](u16x8 (&dst)[RT][8], int step) {
    if (step < nsteps) {
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int s = 0; s < 8; ++s) dst[r][s] = *reinterpret_cast<const u16x8*>(wr[r] + step * 256 + 32 * s);
    }
  };
  auto body = [&](u16x8 (&cur)[RT][8], u16x8 (&refill)[RT][8], int st) {
    const int buf = st & 1;
    const bool more = st + 1 < nsteps;
    load_w(refill, st + 2);
    if (more) load_x(st + 1);
    const unsigned short* xb = &xs[buf][c * DG_LDS_ROW + 8 * g];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xb + 16 * t * DG_LDS_ROW + 32 * s);
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cur[r][s]),
                                                               __builtin_bit_cast(bf16x8, b), acc[r][t], 0, 0, 0);
      }
    }
    if (more) store_x(buf ^ 1);
    __syncthreads();
  };
  load_w(a0, 0);
  load_w(a1, 1);
  load_x(0);
  store_x(0);
  __syncthreads();
  for (int st = 0; st < nsteps; st += 3) {
    body(a0, a2, st);
    if (st + 1 < nsteps) body(a1, a0, st + 1);
    if (st + 2 < nsteps) body(a2, a1, st + 2);
  }

  // C: col m = 16t + c, rows n = nbase + 16r + 4g + j
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int n = nbase + 16 * r + 4 * g;
    if (n >= N) continue;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + c;
      if (m >= M) continue;
      if (S == 1) {
        uint2 v;
        v.x = pack_bf16x2(acc[r][t][0], acc[r][t][1]);
        v.y = pack_bf16x2(acc[r][t][2], acc[r][t][3]);
        *reinterpret_cast<uint2*>(out + (long)m * out_stride + n) = v;
      } else {
        *reinterpret_cast<f32x4*>(ws + ((long)split * M + m) * N + n) = acc[r][t];
      }
    }
  }
}

// out[m, n] = bf16(sum_s ws[s, m, n]); 8 columns per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(unsigned short* __restrict__ out, long out_stride,
                                                            const float* __restrict__ ws, int M, int N, int S) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= (long)M * N) return;
  const int m = i / N, n = i - (long)m * N;
  f32x4 lo = *reinterpret_cast<const f32x4*>(ws + i), hi = *reinterpret_cast<const f32x4*>(ws + i + 4);
  for (int s = 1; s < S; ++s) {
    lo += *reinterpret_cast<const f32x4*>(ws + (long)s * M * N + i);
    hi += *reinterpret_cast<const f32x4*>(ws + (long)s * M * N + i + 4);
  }
  u32x4 o;
  o[0] = pack_bf16x2(lo[0], lo[1]);
  o[1] = pack_bf16x2(lo[2], lo[3]);
  o[2] = pack_bf16x2(hi[0], hi[1]);
  o[3] = pack_bf16x2(hi[2], hi[3]);
  *reinterpret_cast<u32x4*>(out + (long)m * out_stride + n) = o;
}

template <int MT, int RT>
static void dg_launch(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                      int N, int K, int S, hipStream_t s) {
  constexpr int NWAVES = 4, NW = 16 * RT * NWAVES;
  const int tiles = (N + NW - 1) / NW;
  decode_gemm_kernel<MT, RT, NWAVES><<<tiles * S, 64 * NWAVES, 0, s>>>(
      static_cast<unsigned short*>(out), out_stride, ws, static_cast<const unsigned short*>(x), x_stride,
      static_cast<const unsigned short*>(w), M, N, K, S, tiles);
  if (S > 1) {
    const long n8 = (long)M * N / 8;
    splitk_reduce_kernel<<<(n8 + 255) / 256, 256, 0, s>>>(static_cast<unsigned short*>(out), out_stride, ws, M, N,
                                                          S);
  }
}

bool launch_decode_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                        int N, int K, int rt, int S, hipStream_t s) {
#define HS_DG(MT_)                                                                   \
  if (rt == 1) { dg_launch<MT_, 1>(out, out_stride, ws, x, x_stride, w, M, N, K, S, s); return true; } \
  if (rt == 2) { dg_launch<MT_, 2>(out, out_stride, ws, x, x_stride, w, M, N, K, S, s); return true; } \
  return false;
  if (M <= 16) { HS_DG(1) }
  if (M <= 32) { HS_DG(2) }
  HS_DG(4)
#undef HS_DG
}

}  // namespace hipserve
