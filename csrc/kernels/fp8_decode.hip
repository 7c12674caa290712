// FP8 W8A8 decode GEMM (SURVEY K6/K7 for the FP8-Dynamic checkpoints at M <= 256):
//   ws[s, m, n] = (sum over K slice s of xq[m, k] . wq[n, k]) * xs[m] * rs[n] / 256
// xq / xs: per-token dynamic e4m3 activations (act_quant_fp8, prefill_gemm.hip), wq / rs:
// the per-channel e4m3 weight in the decode tiled layout (ops/quant.py
// QuantPart.from_fp8: 16-byte piece (row n, k 16 c) of 128-k tile kt at
// [(n >> 4) nsb + kt / 2] 4096 + (c & 3) 1024 + (kt & 1) 512 + (c >> 2) 256 + (n & 15) 16).
// The fp32 partials feed the fused decode epilogues (splitk_rope_cache /
// splitk_add_rmsnorm / splitk_glu / splitk_post_add_rmsnorm) or splitk_reduce.
//
// Why: the W8A16 quantised decode GEMM (gguf_mfma.hip) converts every weight byte to
// f16 in VALU and runs f16 MFMAs; at 64 sequences that body sits at 2-3 TB/s of FP8
// bytes. Here the weights go straight from HBM into v_mfma_scale_f32_16x16x128_f8f6f4
// operands (unit E8M0 scales; the per-row / per-token scales are applied once in the
// epilogue): no dequant VALU, one MFMA per 2 KiB of weights per m-tile, so the body is
// a weight stream like the bf16 decode GEMM (decode_gemm.hip), whose structure it
// follows:
//  * a workgroup = 8 waves x 16 weight rows (128 rows) and one K slice of NSTEPS
//    256-k steps, fully unrolled (hipcc then counts every vmcnt exactly);
//  * weights: per step a wave loads 4 KiB (64 B per lane: 4 x 16-byte pieces, each
//    instruction 4 runs of 256 contiguous bytes) two steps ahead in a 3-deep VGPR ring,
//    non-temporal (read once);
//  * x: the step's [16 MT, 256] e4m3 slice is staged through registers into a 2-slot
//    LDS ring shared by the 8 waves (one x read per workgroup, not per wave);
//  * MFMA operands (32 bytes per lane): A = weight rows (lane row n & 15, chunks q and
//    q + 4 of the 128-k tile, q = lane >> 4), B = x rows with the same k chunks, so
//    the lane -> k permutation matches on both sides; the result lane holds 4
//    consecutive n of one m (f32x4 partial stores).
// Multi-part weights (q | k | v, gate | up) are up to 4 parts stacked along N; a wave's
// 16 rows always lie in one part (part rows % 16 == 0).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int FD_LDS_ROW = 272;  // 256 e4m3 + 16 B pad

template <int MT, int NSTEPS>
__global__ __launch_bounds__(512) void fp8_decode_kernel(float* __restrict__ ws, const unsigned char* __restrict__ xq,
                                                         PgF8 W, int M, int N, int K, int tiles) {
  constexpr int XR = 16 * MT;                          // staged x rows (padded M)
  constexpr int XPASS = (XR * 16 + 511) / 512;         // 16-byte x loads per thread per step
  __shared__ __attribute__((aligned(16))) unsigned char xs_lds[2][XR * FD_LDS_ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, q = lane >> 4;
  const int split = blockIdx.x / tiles, tile = blockIdx.x - split * tiles;
  const int nsb = K >> 8;
  const int sb0 = split * NSTEPS;
  const int n0 = tile * 128 + wave * 16;  // this wave's first output row
  const bool active = n0 < N;

  // the wave's part and its 4096-byte block row
  const unsigned char* wb = W.p[0].q;
  const float* rsp = W.p[0].rs;
  int nl = min(n0, N - 16);
  {
    int col = 0;
#pragma unroll
    for (int i = 0; i < kPgF8Parts; ++i) {
      if (i < W.n && nl >= col && nl < col + W.p[i].rows) {
        wb = W.p[i].q;
        rsp = W.p[i].rs;
        nl -= col;
        col = 1 << 30;  // found: later parts do not match
      } else if (i < W.n) {
        col += W.p[i].rows;
      }
    }
  }
  const unsigned char* wrow = wb + ((long)(nl >> 4) * nsb + sb0) * 4096 + q * 1024 + c * 16;

  // x staging: thread -> (row, 16-byte chunk of the 256-byte step slice)
  u32x4 xv[XPASS];
  auto load_x = [&](int st) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * 512 + tid;
      if (XR * 16 % 512 == 0 || idx < XR * 16) {
        const int row = idx >> 4, ch = idx & 15;
        // rows >= M are clamped (they only feed output columns that are never stored)
        xv[p] = *reinterpret_cast<const u32x4*>(xq + (long)min(row, M - 1) * K + (long)(sb0 + st) * 256 + ch * 16);
      }
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * 512 + tid;
      if (XR * 16 % 512 == 0 || idx < XR * 16) {
        const int row = idx >> 4, ch = idx & 15;
        *reinterpret_cast<u32x4*>(&xs_lds[buf][row * FD_LDS_ROW + ch * 16]) = xv[p];
      }
    }
  };

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight ring: [slot][piece (h, s) = 2 h + s] — piece (h, s) of the lane: 128-k tile
  // half h of the step, chunk q + 4 s
  u32x4 ring[3][4];
  auto load_w = [&](int slot, int st) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
      ring[slot][p] = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4*>(wrow + (long)st * 4096 + (p >> 1) * 512 + (p & 1) * 256));
  };

  // prologue: x(0) -> LDS[0]; x(1) in registers; W(0), W(1) in flight
  load_x(0);
  store_x(0);
  if (NSTEPS > 1) load_x(1);
  load_w(0, 0);
  if (NSTEPS > 1) load_w(1, 1);
  __syncthreads();
#pragma unroll
  for (int st = 0; st < NSTEPS; ++st) {
    if (st + 1 < NSTEPS) store_x((st + 1) % 2);  // x(st+1), loaded during step st-1
    if (st + 2 < NSTEPS) {
      load_x(st + 2);
      load_w((st + 2) % 3, st + 2);
    }
    const unsigned char* xb = &xs_lds[st % 2][c * FD_LDS_ROW + q * 16];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const u32x4 w0 = ring[st % 3][2 * h], w1 = ring[st % 3][2 * h + 1];
      const i32x8 a = i32x8{(int)w0[0], (int)w0[1], (int)w0[2], (int)w0[3], (int)w1[0], (int)w1[1], (int)w1[2], (int)w1[3]};
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u32x4 b0 = *reinterpret_cast<const u32x4*>(xb + 16 * t * FD_LDS_ROW + h * 128);
        const u32x4 b1 = *reinterpret_cast<const u32x4*>(xb + 16 * t * FD_LDS_ROW + h * 128 + 64);
        const i32x8 b = i32x8{(int)b0[0], (int)b0[1], (int)b0[2], (int)b0[3], (int)b1[0], (int)b1[1], (int)b1[2], (int)b1[3]};
        acc[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[t], 0, 0, 0, 127, 0, 127);
      }
    }
    // pin this step's MFMAs before the barrier: left free, hipcc sank every step's
    // MFMAs to the end of the unrolled loop and kept all weight / x fragments live
#pragma unroll
    for (int t = 0; t < MT; ++t) asm volatile("" : "+v"(acc[t]));
    if (st + 1 < NSTEPS) __syncthreads();
  }

  if (!active) return;
  // lane: rows n = n0 + 4 q + j (j = 0..3), column m = 16 t + c
  const f32x4 rsv = *reinterpret_cast<const f32x4*>(rsp + nl + 4 * q);
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + c;
    if (m >= M) continue;
    const float sx = W.xs[m] * (1.f / 256.f);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = acc[t][j] * (sx * rsv[j]);
    *reinterpret_cast<f32x4*>(ws + ((long)split * M + m) * N + n0 + 4 * q) = o;
  }
}

template <int MT>
static bool fd_launch(float* ws, const unsigned char* xq, const PgF8& W, int M, int N, int K, int S, hipStream_t s) {
  const int tiles = (N + 127) / 128, steps = (K >> 8) / S;
  const dim3 grid(tiles * S);
#define FD_CASE(n)                                                                                   \
  case n:                                                                                            \
    fp8_decode_kernel<MT, n><<<grid, 512, 0, s>>>(ws, xq, W, M, N, K, tiles);                        \
    return true;
  switch (steps) {
    FD_CASE(1) FD_CASE(2) FD_CASE(3) FD_CASE(4) FD_CASE(6) FD_CASE(7) FD_CASE(8) FD_CASE(12) FD_CASE(14)
    FD_CASE(16) FD_CASE(21)
    default: return false;
  }
#undef FD_CASE
}

bool fp8_decode_steps_ok(int steps) {
  switch (steps) {
    case 1: case 2: case 3: case 4: case 6: case 7: case 8: case 12: case 14: case 16: case 21: return true;
    default: return false;
  }
}

// M <= 256: the decode graph buckets above 64 rows (max_num_seqs 256, the chart default)
// stream the weight once too — 8 / 16 x-tiles per wave (acc 32 / 64 VGPRs; the x slice
// ring is 70 / 139 KiB of LDS, so 2 / 1 workgroups per CU) instead of the prefill GEMM,
// whose few 256-row tiles left most of the chip idle at these row counts
bool launch_fp8_decode_gemm(float* ws, const void* xq, const PgF8& W, int M, int N, int K, int S, hipStream_t s) {
  if (M < 1 || M > 256 || K % 256 || S < 1 || (K >> 8) % S || N % 16) return false;
  for (int i = 0; i < W.n; ++i)
    if (W.p[i].rows % 16) return false;
  auto* x = static_cast<const unsigned char*>(xq);
  if (M <= 16) return fd_launch<1>(ws, x, W, M, N, K, S, s);
  if (M <= 32) return fd_launch<2>(ws, x, W, M, N, K, S, s);
  if (M <= 64) return fd_launch<4>(ws, x, W, M, N, K, S, s);
  if (M <= 128) return fd_launch<8>(ws, x, W, M, N, K, S, s);
  return fd_launch<16>(ws, x, W, M, N, K, S, s);
}

}  // namespace hipserve
