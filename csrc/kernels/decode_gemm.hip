// Decode GEMM v3 for the weight-streaming regime (SURVEY K6/K7/K9, M <= 64):
//   out[M, N] = x[M, K] . W[N, K]^T      (bf16 in/out, fp32 accumulate)
//
// Why not the skinny kernel (one x read per 16 W rows): at M = 64 the activation
// re-reads from L2 (M/16 = 4x the weight bytes) throttle the HBM stream. Here
//  * a workgroup owns NW = 128 weight rows and one K slice; the x slice
//    [16*MT, 256] for the current 256-k step is staged in LDS (3-deep ring,
//    528 B rows = conflict-free ds_read_b128) and shared by all waves, so L2->CU
//    activation traffic drops to M/NW of the weight bytes;
//  * MFMA k order is permuted so that each 16-byte load instruction of a wave
//    covers 16 rows x 64 contiguous bytes (4 lane groups side by side) rather than
//    64 scattered 16-byte pieces; two 256-k steps (512 B per row each) are kept
//    in flight in a VGPR ring ahead of the MFMAs (non-temporal: read once) —
//    and they are issued AFTER the next x slice so the in-order vmcnt wait before
//    the LDS store does not drain them;
//  * out^T = W . x^T on v_mfma_f32_16x16x32_bf16: each W fragment feeds MT MFMAs
//    and each LDS x fragment feeds RT MFMAs;
//  * small-N projections (o_proj / down N = 4096 -> 32 workgroups of 128 rows) are
//    split over K into S slices so the grid covers all 256 CUs; slices write fp32
//    partials [S, M, N] and `splitk_reduce` sums them (a kernel boundary instead of
//    cross-XCD fences: the 8 L2s are not coherent with each other mid-kernel).
//  * blockIdx -> (slice, tile) is slice-major so the 8 XCDs (round-robin dispatch)
//    each walk disjoint weight rows of one slice.
//  * kGlu (merged gate|up projection, packed with pack_decode_weight(glu=true):
//    each 128-row tile holds 64 gate rows then the 64 matching up rows): with
//    S == 1 the epilogue exchanges the up half through LDS and writes
//    act = silu(gate) * up [M, N/2] directly — no [M, N] gate|up round trip and
//    no separate silu_and_mul launch. S > 1 partials go to splitk_reduce_glu.
//  * ws != nullptr: fp32 partials [S, M, N] are written even for S == 1 and no
//    reduce kernel is launched when DG_PARTIAL is set — the caller's fused
//    epilogue (decode_fused.hip: residual add + RMSNorm, RoPE + KV write) sums them.
//  * kPacked: the weight is pre-shuffled ONCE at load time into the exact order the
//    waves consume it, [N/128][K/256][8 row groups][8 k-slots][64 lanes][8]
//    (pack_decode_weight below). Every 16-byte-per-lane load instruction then reads
//    1 KiB of contiguous memory and a workgroup streams one contiguous region
//    (64 KiB per 256-k step) — the access pattern of a memcpy, instead of 128
//    rows x 512 B pieces scattered over 128 DRAM pages per step. Rows past N are
//    zero padding (N is rounded up to 128 in the packed copy).
//  * kMoe (Mixtral decode experts): blockIdx.y is one expert-sorted tile of 16*MT
//    slots from moe_align (moe.hip); the workgroup streams THAT expert's weight
//    (w + e * w_estride) and stages the tile's x rows through the slot list
//    (row = pair / gather_k for the token-indexed w13 input, row = slot for the
//    slot-indexed w2 input). Padding slots (-1) read row 0 and are never stored;
//    output rows / partial rows are slot-indexed. Tiles of absent experts exit.
#include <cstdlib>

#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int DG_LDS_ROW = 264;  // 256 + 8 bf16 pad -> 528 B row stride

struct MoeTiles {
  const int* slots;        // [tiles_cap * 16 * MT] pair index per slot, -1 = padding
  const int* tile_expert;  // [tiles_cap] expert of each tile, -1 = unused tile
  int gather_k;            // > 0: x row = pair / gather_k; 0: x row = slot
  long w_estride;          // elements between consecutive experts' weights
};

template <int MT, int RT, int NWAVES, int NSTEPS, bool kPacked, bool kGlu, bool kMoe = false>
__global__ __launch_bounds__(64 * NWAVES) void decode_gemm_kernel(
    unsigned short* __restrict__ out, long out_stride, float* __restrict__ ws,
    const unsigned short* __restrict__ x, long x_stride, const unsigned short* __restrict__ w,
    int M, int N, int K, int S, int tiles, MoeTiles moe = MoeTiles{}) {
  constexpr int NW = 16 * RT * NWAVES;
  constexpr int XR = 16 * MT;                 // x rows staged (padded M)
  constexpr int NT = 64 * NWAVES;             // threads
  constexpr int XPASS = XR * 32 / NT;         // 16-byte x loads per thread per step
  // x ring in LDS: 2 slots suffice (x(st+1) is stored at the start of step st into the
  // slot x(st-1) used, after the barrier that ended step st-1); at M = 64 that is
  // 68 KB instead of 101 KB, so two workgroups fit per CU
  __shared__ __attribute__((aligned(16))) unsigned short xs[2][XR * DG_LDS_ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int split = blockIdx.x / tiles, tile = blockIdx.x - split * tiles;
  constexpr int nsteps = NSTEPS;  // K slice = 256 * NSTEPS, fully unrolled: straight-line
                                  // code lets hipcc count every vmcnt exactly
  const int k0 = split * 256 * NSTEPS;
  const int nbase = tile * NW + wave * 16 * RT;
  int mrow0 = 0;  // kMoe: first slot of this expert tile
  if constexpr (kMoe) {
    const int e = moe.tile_expert[blockIdx.y];
    if (e < 0) return;
    w += (long)e * moe.w_estride;
    mrow0 = blockIdx.y * XR;
  }

  const unsigned short* wr[RT];
  // packed: [128-row tile][kstep][row group][slot s][lane][8]; a 64-row workgroup
  // (NW = 64) streams half the row groups of one packed tile
  constexpr int PT = 128 / NW;
  static_assert(!kGlu || PT == 1, "the GLU epilogue pairs the two halves of a 128-row tile");
  if constexpr (kPacked) {
    const int ptile = tile / PT, prg0 = (tile - ptile * PT) * (NW / 16);
    const unsigned short* wp = w + ((long)ptile * (K >> 8) + (long)split * NSTEPS) * 32768 + lane * 8;
#pragma unroll
    for (int r = 0; r < RT; ++r) wr[r] = wp + (long)(prg0 + wave * RT + r) * (8 * 512);
  } else {
#pragma unroll
    for (int r = 0; r < RT; ++r) wr[r] = w + (long)min(nbase + 16 * r + c, N - 1) * K + k0 + 8 * g;
  }

  // x staging: thread -> (row, 16-byte column chunk)
  u16x8 xv[XPASS];
  [[maybe_unused]] const unsigned short* xg[XPASS];  // kMoe: gathered row pointers
  if constexpr (kMoe) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      const int slot = mrow0 + row, pr = moe.slots[slot];
      const long xrow = pr < 0 ? 0 : (moe.gather_k > 0 ? pr / moe.gather_k : slot);
      xg[p] = x + xrow * x_stride + k0 + col;
    }
  }
  auto load_x = [&](int step) {
    if constexpr (kMoe) {
#pragma unroll
      for (int p = 0; p < XPASS; ++p) xv[p] = *reinterpret_cast<const u16x8*>(xg[p] + step * 256);
      return;
    }
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      // rows >= M are clamped, not zeroed: they only feed output columns m >= M,
      // which are never stored, and a per-lane select around a load makes hipcc
      // branch and drain vmcnt(0) — the whole weight prefetch — every step
      const unsigned short* xp = x + (long)min(row, M - 1) * x_stride + k0 + step * 256 + col;
      xv[p] = *reinterpret_cast<const u16x8*>(xp);
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

  // Both operands run two 256-k steps ahead, issued in the order x(st+2), W(st+2)
  // every step, so each in-order vmcnt wait (x into LDS one step ahead, W for the
  // MFMAs) leaves the younger step's loads in flight: weights in a 3-deep VGPR
  // ring, x through registers into a 3-deep LDS ring.
  u16x8 ring[3][RT][8];
  auto load_w = [&](int slot, int step) {
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int s = 0; s < 8; ++s)
        ring[slot][r][s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(
            kPacked ? wr[r] + (long)step * 32768 + 512 * s : wr[r] + step * 256 + 32 * s));
  };
  // prologue: x(0) -> LDS[0]; x(1) in registers; W(0), W(1) in flight
  load_x(0);
  store_x(0);
  if (nsteps > 1) load_x(1);
  load_w(0, 0);
  if (nsteps > 1) load_w(1, 1);
  __syncthreads();
#pragma unroll
  for (int st = 0; st < nsteps; ++st) {
    if (st + 1 < nsteps) store_x((st + 1) % 2);  // x(st+1), loaded during step st-1
    if (st + 2 < nsteps) {
      load_x(st + 2);
      load_w((st + 2) % 3, st + 2);
    }
    const unsigned short* xb = &xs[st % 2][c * DG_LDS_ROW + 8 * g];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xb + 16 * t * DG_LDS_ROW + 32 * s);
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ring[st % 3][r][s]),
                                                               __builtin_bit_cast(bf16x8, b), acc[r][t], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps) __syncthreads();
  }

  // output row of MFMA column m = 16t + c: slot-indexed for kMoe
  bool mok[MT];
  int orow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + c;
    if constexpr (kMoe) {
      orow[t] = mrow0 + m;
      mok[t] = moe.slots[orow[t]] >= 0;
    } else {
      orow[t] = m;
      mok[t] = m < M;
    }
  }
  if constexpr (kGlu) {
    if (ws == nullptr) {
      // row group rg = wave*RT + r: 0-3 gate rows, 4-7 the matching up rows
      constexpr int EW = 16 * MT;  // exchange row width (fp32)
      float* ex = reinterpret_cast<float*>(&xs[0][0]);
      __syncthreads();  // every wave is done reading the x ring
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int rg = wave * RT + r;
        if (rg < 4) continue;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ex[((rg - 4) * 16 + 4 * g + j) * EW + 16 * t + c] = bf16_to_f32(f32_to_bf16(acc[r][t][j]));
      }
      __syncthreads();
      const int I = N >> 1;
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int rg = wave * RT + r;
        if (rg >= 4) continue;
        const int col = tile * 64 + rg * 16 + 4 * g;  // act column of j = 0
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          if (!mok[t]) continue;
          unsigned short o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            o[j] = silu_mul1(f32_to_bf16(acc[r][t][j]),
                             f32_to_bf16(ex[(rg * 16 + 4 * g + j) * EW + 16 * t + c]));
          uint2 v;
          v.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          v.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          if (col < I) *reinterpret_cast<uint2*>(out + (long)orow[t] * out_stride + col) = v;
        }
      }
      return;
    }
  }
  // C: col m = 16t + c, rows n = nbase + 16r + 4g + j
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    const int n = nbase + 16 * r + 4 * g;
    if (n >= N) continue;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      if (!mok[t]) continue;
      if (ws == nullptr) {
        uint2 v;
        v.x = pack_bf16x2(acc[r][t][0], acc[r][t][1]);
        v.y = pack_bf16x2(acc[r][t][2], acc[r][t][3]);
        *reinterpret_cast<uint2*>(out + (long)orow[t] * out_stride + n) = v;
      } else {
        *reinterpret_cast<f32x4*>(ws + ((long)split * M + orow[t]) * N + n) = acc[r][t];
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
  f32x4 lo, hi;
  sum_slices8(lo, hi, ws + i, (long)M * N, S);
  u32x4 o;
  o[0] = pack_bf16x2(lo[0], lo[1]);
  o[1] = pack_bf16x2(lo[2], lo[3]);
  o[2] = pack_bf16x2(hi[0], hi[1]);
  o[3] = pack_bf16x2(hi[2], hi[3]);
  *reinterpret_cast<u32x4*>(out + (long)m * out_stride + n) = o;
}

// GLU split-K reduce: partial columns are in the interleaved packed order
// (tile t: 64 gate columns then their 64 up columns); act[m, 64t + i] =
// silu(bf16(sum gate)) * bf16(sum up). 8 act columns per thread.
__global__ __launch_bounds__(256) void splitk_reduce_glu_kernel(unsigned short* __restrict__ out, long out_stride,
                                                                const float* __restrict__ ws, int M, int N, int S) {
  const int I = N >> 1;
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= (long)M * I) return;
  const int m = i / I, a = i - (long)m * I;
  const long gc = (long)(a >> 6) * 128 + (a & 63);  // gate column in the partials
  const float* pg = ws + (long)m * N + gc;
  f32x4 g0 = *reinterpret_cast<const f32x4*>(pg), g1 = *reinterpret_cast<const f32x4*>(pg + 4);
  f32x4 u0 = *reinterpret_cast<const f32x4*>(pg + 64), u1 = *reinterpret_cast<const f32x4*>(pg + 68);
  for (int s = 1; s < S; ++s) {
    const float* q = pg + (long)s * M * N;
    g0 += *reinterpret_cast<const f32x4*>(q);
    g1 += *reinterpret_cast<const f32x4*>(q + 4);
    u0 += *reinterpret_cast<const f32x4*>(q + 64);
    u1 += *reinterpret_cast<const f32x4*>(q + 68);
  }
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = silu_mul1(f32_to_bf16(g0[j]), f32_to_bf16(u0[j]));
    o[j + 4] = silu_mul1(f32_to_bf16(g1[j]), f32_to_bf16(u1[j]));
  }
  *reinterpret_cast<u16x8*>(out + (long)m * out_stride + a) = o;
}

void launch_splitk_reduce(void* out, long out_stride, const float* ws, int M, int N, int S, hipStream_t s) {
  const long n8 = (long)M * N / 8;
  if (n8 <= 0) return;
  splitk_reduce_kernel<<<(n8 + 255) / 256, 256, 0, s>>>(static_cast<unsigned short*>(out), out_stride, ws, M, N, S);
}

// rt 1: 8 waves x 1 row group, 2: 4 waves x 2 (both 128 weight rows per workgroup);
// 3: 4 waves x 1 (64 rows: twice the workgroups at the same K split, for projections
// whose 128-row tiles do not fill the chip without more split-K partials)
template <int MT, int RT, int NSTEPS, bool kPacked, bool kGlu, int NWAVES = RT == 1 ? 8 : 4>
static void dg_launch(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                      int N, int K, int S, int flags, hipStream_t s) {
  constexpr int NW = 16 * RT * NWAVES;
  const int tiles = (N + NW - 1) / NW;
  decode_gemm_kernel<MT, RT, NWAVES, NSTEPS, kPacked, kGlu><<<tiles * S, 64 * NWAVES, 0, s>>>(
      static_cast<unsigned short*>(out), out_stride, ws, static_cast<const unsigned short*>(x), x_stride,
      static_cast<const unsigned short*>(w), M, N, K, S, tiles);
  if (ws != nullptr && !(flags & DG_PARTIAL)) {
    if (kGlu) {
      const long n8 = (long)M * (N / 2) / 8;
      splitk_reduce_glu_kernel<<<(n8 + 255) / 256, 256, 0, s>>>(static_cast<unsigned short*>(out), out_stride, ws,
                                                                 M, N, S);
      return;
    }
    const long n8 = (long)M * N / 8;
    splitk_reduce_kernel<<<(n8 + 255) / 256, 256, 0, s>>>(static_cast<unsigned short*>(out), out_stride, ws, M, N,
                                                          S);
  }
}

template <int MT, int RT, bool kPacked, bool kGlu, int NWAVES = RT == 1 ? 8 : 4>
static bool dg_steps(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M, int N,
                     int K, int S, int flags, hipStream_t s) {
  const int nsteps = K / S / 256;
#define DG_CASE(NS)                                                                                       \
  case NS:                                                                                                \
    dg_launch<MT, RT, NS, kPacked, kGlu, NWAVES>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s); \
    return true;
  switch (nsteps) {
    DG_CASE(1) DG_CASE(2) DG_CASE(4) DG_CASE(7) DG_CASE(8) DG_CASE(16)
    // K = 3072 (Phi-3, Llama-3.2-3B) and K = 5376 (Gemma-3-27B) in one K slice
    DG_CASE(12) DG_CASE(21)
    default: return false;
  }
#undef DG_CASE
}

template <bool kPacked, bool kGlu>
static bool dg_dispatch(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                        int N, int K, int rt, int S, int flags, hipStream_t s) {
  if (M <= 16) {
    if (rt == 1) return dg_steps<1, 1, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
    if (rt == 2) return dg_steps<1, 2, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
  } else if (M <= 32) {
    if (rt == 1) return dg_steps<2, 1, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
    if (rt == 2) return dg_steps<2, 2, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
  } else {
    if (rt == 1) return dg_steps<4, 1, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
    if (rt == 2) return dg_steps<4, 2, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
    if constexpr (!kGlu) {  // 64-row workgroups (33-64 rows: the decode batch of the headline load)
      if (rt == 3) return dg_steps<4, 1, kPacked, kGlu, 4>(out, out_stride, ws, x, x_stride, w, M, N, K, S, flags, s);
    }
  }
  return false;
}

// K slice per workgroup = K / S must be 256 * {1, 2, 4, 7, 8, 12, 16, 21}; false otherwise.
// packed: w is the pack_decode_weight layout (N rounded up to 128 rows).
bool launch_decode_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                        int N, int K, int rt, int S, bool packed, int flags, hipStream_t s) {
  if (flags & DG_GLU) {  // gate|up interleaved packing -> act = silu(gate) * up
    return packed && N % 128 == 0 &&
           dg_dispatch<true, true>(out, out_stride, ws, x, x_stride, w, M, N, K, rt, S, flags, s);
  }
  return packed ? dg_dispatch<true, false>(out, out_stride, ws, x, x_stride, w, M, N, K, rt, S, flags, s)
                : dg_dispatch<false, false>(out, out_stride, ws, x, x_stride, w, M, N, K, rt, S, flags, s);
}

// ---- MoE decode experts (kMoe): one 128-row weight tile x one expert tile per workgroup.
template <int MT, int NSTEPS, bool kPacked, bool kGlu>
static void moe_dg_launch(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w,
                          const MoeTiles& mt, int tiles_cap, int N, int K, int S, hipStream_t s) {
  const int tiles = (N + 127) / 128;  // RT = 1, 8 waves: 128 weight rows per workgroup
  dim3 grid(tiles * S, tiles_cap);
  decode_gemm_kernel<MT, 1, 8, NSTEPS, kPacked, kGlu, true><<<grid, 512, 0, s>>>(
      static_cast<unsigned short*>(out), out_stride, ws, static_cast<const unsigned short*>(x), x_stride,
      static_cast<const unsigned short*>(w), tiles_cap * 16 * MT, N, K, S, tiles, mt);
}

template <int MT, bool kPacked, bool kGlu>
static bool moe_dg_steps(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w,
                         const MoeTiles& mt, int tiles_cap, int N, int K, int S, hipStream_t s) {
  switch (K / S / 256) {
    case 1: moe_dg_launch<MT, 1, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 2: moe_dg_launch<MT, 2, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 4: moe_dg_launch<MT, 4, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 7: moe_dg_launch<MT, 7, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 8: moe_dg_launch<MT, 8, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 16: moe_dg_launch<MT, 16, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    // small-expert MoE (Qwen3-MoE: expert width 768 / 1536 -> w2 K in one slice)
    case 3: moe_dg_launch<MT, 3, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    case 6: moe_dg_launch<MT, 6, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s); return true;
    default: return false;
  }
}

template <bool kPacked, bool kGlu>
static bool moe_dg_tile(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w,
                        const MoeTiles& mt, int tiles_cap, int tile, int N, int K, int S, hipStream_t s) {
  if (tile == 16) return moe_dg_steps<1, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s);
  if (tile == 32) return moe_dg_steps<2, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s);
  if (tile == 64) return moe_dg_steps<4, kPacked, kGlu>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, N, K, S, s);
  return false;
}

// Expert GEMM over moe_align tiles. ws == nullptr: bf16 out[slot, N] (glu: act[slot, N/2]
// from the gate/up-interleaved packing, S must be 1); else fp32 partials
// ws[S, tiles_cap * tile, N] (summed by moe_combine_partial). w: [E] x (packed or
// row-major [N, K]) with w_estride elements per expert. K / S = 256 * {1,2,3,4,6,7,8,16}.
// ---- small-expert MoE decode (Qwen3-MoE: 128 experts of width 768, K <= 2048):
// the expert tile's x rows [16*MT, K] are gathered into LDS ONCE and stay
// resident while the workgroup streams `tpw` consecutive 128-row weight tiles of
// its expert (packed layout: one contiguous region per tile), so the per-tile
// prologue of the streaming kernel above (expert lookup, x gather, pipeline
// fill) is paid once per tpw tiles and the weight stream never drains between
// tiles: a flat (tile, 256-k step) loop with a 3-deep VGPR ring, unrolled by 3
// so every ring slot is a static register set. Epilogue per finished tile:
// bf16 rows (w2) or the SiLU-GLU of the gate/up-interleaved tile (w13).
// Measured (Qwen3-30B-A3B decode, B = 64, all 128 experts active): w13 805 MB in
// 117 us (6.9 TB/s), w2 403 MB in 63 us (6.4 TB/s) — the same HBM-bound time as
// the per-tile streaming kernel with a third of the workgroups.
constexpr int XRES_MAX_LDS = 72 * 1024;

template <int MT, bool kGlu>
__global__ __launch_bounds__(512) void moe_xres_kernel(unsigned short* __restrict__ out, long out_stride,
                                                       const unsigned short* __restrict__ x, long x_stride,
                                                       const unsigned short* __restrict__ w, MoeTiles moe, int N,
                                                       int K, int tpw) {
  constexpr int XR = 16 * MT;
  extern __shared__ __attribute__((aligned(16))) unsigned short xres[];  // [XR][K + 8], then GLU exchange
  const int e = moe.tile_expert[blockIdx.y];
  if (e < 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int KS = K >> 8, LROW = K + 8;
  const int ntiles = (N + 127) >> 7;
  const int t0 = blockIdx.x * tpw;
  const int ntl = min(tpw, ntiles - t0);
  if (ntl <= 0) return;
  const int mrow0 = blockIdx.y * XR;
  // gather the tile's x rows (padding slots read row 0; never stored)
  const int kv = K >> 3;
  for (int idx = tid; idx < XR * kv; idx += 512) {
    const int row = idx / kv, col = (idx - row * kv) * 8;
    const int slot = mrow0 + row, pr = moe.slots[slot];
    const long xrow = pr < 0 ? 0 : (moe.gather_k > 0 ? pr / moe.gather_k : slot);
    *reinterpret_cast<u16x8*>(&xres[row * LROW + col]) = *reinterpret_cast<const u16x8*>(x + xrow * x_stride + col);
  }
  bool mok[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) mok[t] = moe.slots[mrow0 + 16 * t + c] >= 0;
  // this wave's 16-row group of every (tile, k step) chunk: 64 KiB apart, contiguous
  const unsigned short* wb = w + (long)e * moe.w_estride + (long)t0 * KS * 32768 + wave * 4096 + lane * 8;
  const int total = ntl * KS;
  u16x8 ring[3][8];
  auto load_w = [&](u16x8(&r)[8], int f) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
      r[s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wb + (long)f * 32768 + 512 * s));
  };
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float* ex = reinterpret_cast<float*>(&xres[XR * LROW]);  // kGlu: [4][16][XR] fp32

  auto epilogue = [&](int tile) {
    if constexpr (kGlu) {
      if (wave >= 4) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ex[((wave - 4) * 16 + 4 * g + j) * XR + 16 * t + c] = bf16_to_f32(f32_to_bf16(acc[t][j]));
      }
      __syncthreads();
      if (wave < 4) {
        const int col = tile * 64 + wave * 16 + 4 * g;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          if (!mok[t]) continue;
          unsigned short o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            o[j] = silu_mul1(f32_to_bf16(acc[t][j]), f32_to_bf16(ex[(wave * 16 + 4 * g + j) * XR + 16 * t + c]));
          uint2 v;
          v.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          v.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          if (col < (N >> 1)) *reinterpret_cast<uint2*>(out + (long)(mrow0 + 16 * t + c) * out_stride + col) = v;
        }
      }
      __syncthreads();  // exchange buffer reused by the next tile
    } else {
      const int n = tile * 128 + wave * 16 + 4 * g;
      if (n < N) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          if (!mok[t]) continue;
          uint2 v;
          v.x = pack_bf16x2(acc[t][0], acc[t][1]);
          v.y = pack_bf16x2(acc[t][2], acc[t][3]);
          *reinterpret_cast<uint2*>(out + (long)(mrow0 + 16 * t + c) * out_stride + n) = v;
        }
      }
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  auto compute = [&](const u16x8(&r)[8], int step) {
    const unsigned short* xb = &xres[c * LROW + step * 256 + 8 * g];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xb + 16 * t * LROW + 32 * s);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, r[s]),
                                                         __builtin_bit_cast(bf16x8, b), acc[t], 0, 0, 0);
      }
  };

  load_w(ring[0], 0);
  if (total > 1) load_w(ring[1], 1);
  __syncthreads();  // x resident
  // flat (tile, step) stream; slot of chunk f is f % 3, loads run two chunks ahead
  for (int f = 0; f < total; f += 3) {
    if (f + 2 < total) load_w(ring[2], f + 2);
    compute(ring[0], f % KS);
    if (f % KS == KS - 1) epilogue(t0 + f / KS);
    if (f + 1 >= total) break;
    if (f + 3 < total) load_w(ring[0], f + 3);
    compute(ring[1], (f + 1) % KS);
    if ((f + 1) % KS == KS - 1) epilogue(t0 + (f + 1) / KS);
    if (f + 2 >= total) break;
    if (f + 4 < total) load_w(ring[1], f + 4);
    compute(ring[2], (f + 2) % KS);
    if ((f + 2) % KS == KS - 1) epilogue(t0 + (f + 2) / KS);
  }
}

static size_t xres_lds(int MT, int K, bool glu) {
  return (size_t)16 * MT * (K + 8) * 2 + (glu ? (size_t)4 * 16 * 16 * MT * 4 : 0);
}

// true when the x-resident kernel took the launch (packed, bf16 out, MT <= 2, x fits)
static bool try_moe_xres(void* out, long out_stride, const void* x, long x_stride, const void* w,
                         const MoeTiles& mt, int tiles_cap, int tile, int N, int K, bool glu, hipStream_t s) {
  const int MT = tile / 16;
  if (MT > 2 || K % 256 != 0 || xres_lds(MT, K, glu) > XRES_MAX_LDS || getenv("HIPSERVE_MOE_NO_XRES")) return false;
  const int ntiles = (N + 127) / 128;
  const long tile_bytes = 128L * K * 2;
  // >= ~512 KiB of weights per workgroup, but keep >= 512 workgroups in flight
  long want = (512L * 1024 + tile_bytes - 1) / tile_bytes;
  int tpw = (int)(want < 1 ? 1 : (want > ntiles ? ntiles : want));
  while (tpw > 1 && (long)((ntiles + tpw - 1) / tpw) * tiles_cap < 512) --tpw;
  const dim3 grid((ntiles + tpw - 1) / tpw, tiles_cap);
  const size_t lds = xres_lds(MT, K, glu);
  auto* o = static_cast<unsigned short*>(out);
  auto* xi = static_cast<const unsigned short*>(x);
  auto* wi = static_cast<const unsigned short*>(w);
#define XRES_LAUNCH(mt_, glu_)                                                                             \
  do {                                                                                                     \
    static bool attr = [] {  /* dynamic LDS above 64 KiB (gfx950: 160 KiB per CU) */                       \
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&moe_xres_kernel<mt_, glu_>),                \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, XRES_MAX_LDS) == hipSuccess;   \
    }();                                                                                                   \
    (void)attr;                                                                                            \
    moe_xres_kernel<mt_, glu_><<<grid, 512, lds, s>>>(o, out_stride, xi, x_stride, wi, mt, N, K, tpw);       \
  } while (0)
  if (MT == 1) {
    if (glu) XRES_LAUNCH(1, true); else XRES_LAUNCH(1, false);
  } else {
    if (glu) XRES_LAUNCH(2, true); else XRES_LAUNCH(2, false);
  }
#undef XRES_LAUNCH
  return true;
}

bool launch_moe_decode_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w,
                            long w_estride, const int* slots, const int* tile_expert, int tiles_cap, int tile,
                            int gather_k, int N, int K, int S, bool packed, bool glu, hipStream_t s) {
  const MoeTiles mt{slots, tile_expert, gather_k, w_estride};
  if (packed && ws == nullptr && S == 1 && (!glu || N % 128 == 0) &&
      try_moe_xres(out, out_stride, x, x_stride, w, mt, tiles_cap, tile, N, K, glu, s))
    return true;
  if (glu) {
    return packed && ws == nullptr && S == 1 && N % 128 == 0 &&
           moe_dg_tile<true, true>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, tile, N, K, S, s);
  }
  return packed ? moe_dg_tile<true, false>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, tile, N, K, S, s)
                : moe_dg_tile<false, false>(out, out_stride, ws, x, x_stride, w, mt, tiles_cap, tile, N, K, S, s);
}

// W[N, K] row-major -> packed [ceil(N/128)][K/256][8][8][64][8] (zero rows past N).
// glu: W is a merged [gate; up] weight (N % 128 == 0) packed gate/up-interleaved per tile.
// One thread per packed 16-byte piece: reads 16 B of a weight row, writes 16 B.
__global__ __launch_bounds__(256) void pack_decode_weight_kernel(unsigned short* __restrict__ out,
                                                                 const unsigned short* __restrict__ w, int N, int K,
                                                                 long pieces, int glu) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= pieces) return;
  // blockIdx.y: one matrix of a stacked batch (MoE experts), packed back to back
  out += (long)blockIdx.y * pieces * 8;
  w += (long)blockIdx.y * N * K;
  // piece index = ((((tile * KS + kstep) * 8 + rg) * 8 + s) * 64 + lane)
  const int lane = i & 63, sl = (i >> 6) & 7, rg = (i >> 9) & 7;
  const long ts = i >> 12;
  const int KS = K >> 8;
  const int kstep = ts % KS;
  const long tile = ts / KS;
  const int g = lane >> 4, c = lane & 15;
  long n = tile * 128 + rg * 16 + c;
  if (glu) {  // tile = 64 gate rows [64t, 64t+64) then the up rows N/2 + [64t, 64t+64)
    const int i = rg * 16 + c;
    n = i < 64 ? tile * 64 + i : (N >> 1) + tile * 64 + (i - 64);
  }
  const long k = (long)kstep * 256 + 32 * sl + 8 * g;
  u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  if (n < N) v = *reinterpret_cast<const u16x8*>(w + n * K + k);
  *reinterpret_cast<u16x8*>(out + i * 8) = v;
}

void launch_pack_decode_weight(void* out, const void* w, int N, int K, bool glu, hipStream_t s, int batch) {
  const long tiles = (N + 127) / 128;
  const long pieces = tiles * (K / 256) * 8 * 8 * 64;
  if (batch <= 0) return;
  pack_decode_weight_kernel<<<dim3((pieces + 255) / 256, batch), 256, 0, s>>>(
      static_cast<unsigned short*>(out), static_cast<const unsigned short*>(w), N, K, pieces, glu ? 1 : 0);
}

}  // namespace hipserve
