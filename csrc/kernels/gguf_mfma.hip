// GGUF decode GEMM v2 — dequant in registers at ~2 VALU ops per
// weight, f16 MFMA, weights in a tiled layout built once at load.
//
// Why v1 (gguf.hip qgemm) ran at 0.7-2 TB/s of quantised bytes:
//  * a 64-row workgroup re-read the whole x K-slice for 64 rows of ~4.5-bit
//    weights (x traffic 3.6x the weight traffic at M = 64);
//  * split-K workgroups read 144-210 B pieces of rows 2-8 KB apart: partial cache
//    lines, fetched again by the neighbouring K slice on another XCD;
//  * dequant cost ~4 VALU ops per weight (byte extract, int->float, FMA, ->bf16).
// v2:
//  * tiled layout [N/16][K/256][chunk]: the 16 rows x 256 k one wave multiplies
//    are one contiguous chunk, lane-interleaved so every lane-specific 16-byte load
//    is one coalesced 1 KiB wave access; a K slice of a row group is contiguous;
//  * workgroup = 4 waves x 2 row groups = 128 weight rows sharing one x staging
//    (f16, LDS, double-buffered), split over K to fill the chip; 4-wave steps keep
//    occupancy granular (a 150-VGPR body still runs 12 waves per CU);
//  * nibbles become f16 by bit assembly: (w & 0x000F000F) | 0x6400_6400 is the
//    f16 pair (1024 + q_a, 1024 + q_b) for bytes 0 and 2 of a word (exact); one
//    v_pk_add_f16 removes the 1024 (exact), one v_pk_fma_f16 applies the block
//    scale and min with a single f16 rounding (11-bit mantissa: finer than the
//    bf16 weights of v1). Q6_K ORs its two high bits into bit 4-5 first, Q8_0
//    flips the sign bit (int8 + 128 in [0, 255]) before the OR;
//  * the MFMA k order inside each 8-element fragment is therefore the pair order
//    {0, 2, 1, 3, 4, 6, 5, 7}: x is converted to f16 ONCE per workgroup while
//    staging into LDS, already in that order, so A and B agree on every k;
//  * v_mfma_f32_16x16x32_f16 (same rate as bf16), fp32 accumulation; x rows beyond
//    the f16 range are caught on staging and rerun pre-scaled (qgemm2_body);
//  * all parts of a merged projection are one launch (part table: format, column
//    offset, rows; two formats per launch for the Q4_K/Q5_K + Q6_K mixes); split-K
//    writes fp32 partials [S, M, N_total] that the decode layer's fused epilogues
//    consume (RoPE + KV write, residual + RMSNorm, SiLU-GLU) — no reduce kernel.
// Measured (tools/bench_gguf.py, profiles/r2_gguf_v2.md): Llama-3-8B Q4_K_M at
// M = 1, gate|up 3.5-3.8 TB/s, lm_head (Q6_K) 4.5 TB/s, vs 1.5 / 2.9 for v1.
#include "hipserve/common.h"
#include "hipserve/kernels.h"
#include "hipserve/gguf_tiles.h"

namespace hipserve {

namespace {
using namespace gq;


// f16 range of the staged x: a value beyond +-65504 (bf16 activations reach ~3e38;
// Gemma-family hidden states are known to exceed the f16 range) converts to +-inf
// and is caught, not clamped: the inf makes every accumulator of its x row
// non-finite, so a workgroup vote on the accumulators after the K loop (no per-value
// test in the loop) triggers a second pass with each x row pre-scaled by a power of
// two 2^-k (k from the row's max over the workgroup's K range) that the epilogue
// undoes exactly (acc *= 2^k).

// One wave = RT row groups of 16 x the workgroup's K range; 8 waves share the
// x staging. Body per format; the kernel picks it per part (two formats per launch).
template <int QT, int MT, int RT, int NWAVES, bool kMoe = false, bool kX16 = false>
HS_DEVICE void qgemm2_body(_Float16 (&xs)[2][4 * x_plane<MT>()], float* xrow, unsigned short* __restrict__ out,
                           long out_stride,
                           float* __restrict__ ws, const unsigned short* __restrict__ x, long x_stride,
                           const Part& P, int M, int Ntot, int K, int sb_per_split, const MoeQ& moe = MoeQ{},
                           const unsigned short* __restrict__ x16 = nullptr) {
  constexpr int XR = 16 * MT;           // staged x rows (M padded)
  constexpr int NT = 64 * NWAVES;
  constexpr int CB = chunk_bytes<QT>();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int gi0 = (blockIdx.x - P.tile0) * (NWAVES * RT) + wave * RT;  // first row group of this wave
  const int ngroups = P.rows >> 4;
  // kMoe GLU (w13, RT 2): the wave's row group 0 is gate group gg, row group 1 the
  // matching up group gg + ngroups / 2 — equal MFMA layouts, so silu(gate) * up is
  // elementwise in registers and the bf16 gate|up never goes to HBM
  [[maybe_unused]] const bool glu = kMoe && RT == 2 && moe.glu != 0;
  [[maybe_unused]] const int gg = (int)blockIdx.x * NWAVES + wave;
  int gidx[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
    gidx[r] = glu ? min(gg, (ngroups >> 1) - 1) + r * (ngroups >> 1) : gi0 + r;
  const int nsb = K >> 8;
  const int sb0 = blockIdx.y * sb_per_split, sb1 = min(nsb, sb0 + sb_per_split);
  const unsigned char* base[RT];
  // bytes between consecutive super-chunks of a row group (k-major MoE experts: a whole
  // super-chunk column of the expert)
  const long sbs = kMoe && moe.kmajor ? (long)ngroups * CB : (long)CB;
  const long gstride = kMoe && moe.kmajor ? (long)CB : (long)nsb * CB;
#pragma unroll
  for (int r = 0; r < RT; ++r) base[r] = P.q + (long)min(gidx[r], ngroups - 1) * gstride;

  // x staging: 32 fragments (g, s) of 8 per row and super-chunk; thread -> (row, fragment)
  constexpr int XP = XR * 32 / NT;
  static_assert(XP * NT == XR * 32, "x staging must divide evenly (no guarded, sinkable loads)");
  u16x8 xv[XP];
  // kMoe: first slot of the expert tile; dense: first x row of this M tile (prefill
  // sweeps the prompt in XR-row tiles over blockIdx.z, K15)
  const int mrow0 = (int)blockIdx.z * XR;
  [[maybe_unused]] const unsigned short* xg[kMoe ? XP : 1];  // kMoe: gathered row of each staging item
  if constexpr (kMoe) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int slot = mrow0 + ((i * NT + tid) >> 5), pr = moe.slots[slot];
      xg[i] = x + (pr < 0 ? 0L : (long)(moe.gather_k > 0 ? pr / moe.gather_k : slot)) * x_stride;
    }
  }
  // dense: element offset of each staging item's row and k run (32-bit; the prefill
  // M tiles stay far below 2^31 elements), computed once instead of per super-chunk
  [[maybe_unused]] int xo[kMoe ? 1 : XP];
  if constexpr (!kMoe) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int idx = i * NT + tid, row = idx >> 5, fr = idx & 31;
      xo[i] = min(mrow0 + row, M - 1) * (int)x_stride + kbase<QT>(fr >> 3, fr & 7);
    }
  }
  // kX16: the producer of x (decode_fused.hip splitk_add_rmsnorm / splitk_glu) also
  // wrote it as f16 in the staging pair order (x16, same row stride): the first pass
  // stages those bits as they are — no per-workgroup bf16 -> f16 conversion (a
  // quarter of this body's VALU at M = 64). The pre-scaled second pass reads bf16 x.
  auto load_x = [&](int sb, auto scaled) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      // rows >= M are clamped, never stored (kMoe: padding slots read row 0, never stored)
      if constexpr (kMoe) {
        const int fr = (i * NT + tid) & 31;
        xv[i] = *reinterpret_cast<const u16x8*>(xg[i] + sb * 256 + kbase<QT>(fr >> 3, fr & 7));
      } else if constexpr (kX16 && !decltype(scaled)::value) {
        xv[i] = *reinterpret_cast<const u16x8*>(x16 + xo[i] + sb * 256);
      } else {
        xv[i] = *reinterpret_cast<const u16x8*>(x + xo[i] + sb * 256);
      }
    }
  };
  auto store_x = [&](int buf, auto scaled) {
    if constexpr (kX16 && !decltype(scaled)::value) {
#pragma unroll
      for (int i = 0; i < XP; ++i) {
        const int idx = i * NT + tid, row = idx >> 5, fr = idx & 31;
        *reinterpret_cast<u16x8*>(&xs[buf][(fr >> 3) * x_plane<MT>() + row * kXR + (fr & 7) * 8]) = xv[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int idx = i * NT + tid, row = idx >> 5, fr = idx & 31;
      const u32x4 w = __builtin_bit_cast(u32x4, xv[i]);  // bf16 pairs (0,1) (2,3) (4,5) (6,7)
      // pair order {0, 2, 1, 3, 4, 6, 5, 7}
      float f[8] = {bf_lo(w[0]), bf_lo(w[1]), bf_hi(w[0]), bf_hi(w[1]),
                    bf_lo(w[2]), bf_lo(w[3]), bf_hi(w[2]), bf_hi(w[3])};
      if constexpr (decltype(scaled)::value) {
        const float sc = xrow[row];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] *= sc;
      }
      f16x8 h;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = static_cast<_Float16>(f[e]);
      *reinterpret_cast<f16x8*>(&xs[buf][(fr >> 3) * x_plane<MT>() + row * kXR + (fr & 7) * 8]) = h;
    }
  };

  f32x4 acc[RT][MT];

  // Two register sets for the weights, used alternately (loop unrolled by 2): no
  // copies between iterations, so the only wait for a super-chunk's weights is at
  // their first use. Per iteration the x loads of the next super-chunk go out before
  // its weight loads: store_x's in-order vmcnt wait then leaves the weights in flight.
  Raw rawA[RT], rawB[RT];
  auto run = [&](auto scaled) {
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (sb0 < sb1) {
    load_x(sb0, scaled);
#pragma unroll
    for (int r = 0; r < RT; ++r) load_raw<QT>(base[r] + sb0 * sbs, g, c, lane, rawA[r]);
    store_x(0, scaled);
  }
  __syncthreads();
  auto iter = [&](int sb, Raw (&cur)[RT], Raw (&nxt)[RT]) {
    const int buf = (sb - sb0) & 1;
    // next super-chunk in flight while this one is decoded and multiplied; issued
    // unconditionally (the last iteration re-reads its own chunk) so no branch splits
    // the loads from their uses and the vmcnt waits stay counted, not drained
    const int sn = min(sb + 1, sb1 - 1);
    load_x(sn, scaled);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < RT; ++r) load_raw<QT>(base[r] + sn * sbs, g, c, lane, nxt[r]);
    __builtin_amdgcn_sched_barrier(0);  // the scheduler would sink them below the MFMAs
    const _Float16* xb = &xs[buf][g * x_plane<MT>() + c * kXR];  // fragment (g, s) of row 16t + c at + 8s
    Dec<QT> dec[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) dec[r].setup(cur[r], g);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      // the step's MT x fragments are read from LDS BEFORE the dequant VALU and held in
      // MT registers: left to itself the compiler reused one fragment register, so every
      // MFMA waited out a full LDS round trip (ds_read -> lgkmcnt(0) -> MFMA, x MT)
      f16x8 b[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t)  // one LDS read of x per (s, t), shared by the RT row groups
        b[t] = *reinterpret_cast<const f16x8*>(xb + 16 * t * kXR + 8 * s);
      __builtin_amdgcn_sched_barrier(0);
      f16x8 a[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) a[r] = dec[r].step(cur[r], g, s);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r], b[t], acc[r][t], 0, 0, 0);
    }
    store_x(buf ^ 1, scaled);
    __syncthreads();
  };
  int sb = sb0;
  for (; sb + 1 < sb1; sb += 2) {  // no exit inside the pair: the loop-carried vmcnt state stays exact
    iter(sb, rawA, rawB);
    iter(sb + 1, rawB, rawA);
  }
  if (sb < sb1) iter(sb, rawA, rawB);
  };
  run(std::false_type{});
  // some staged x beyond the f16 range (rare) became +-inf, which leaves a non-finite
  // accumulator in every output of its row: per-row power-of-two pre-scale, second pass
  bool bad = false;
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) bad |= !__builtin_isfinite(acc[r][t][e]);
  if (__syncthreads_or(bad)) {
    unsigned* xb = reinterpret_cast<unsigned*>(xrow);
    if (tid < XR) xb[tid] = 0u;
    __syncthreads();
    for (int sb2 = sb0; sb2 < sb1; ++sb2) {  // max |x| per staged row (ds_max_u32 on non-negative float bits)
      load_x(sb2, std::true_type{});
#pragma unroll
      for (int i = 0; i < XP; ++i) {
        const u32x4 w = __builtin_bit_cast(u32x4, xv[i]);
        unsigned mx = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = max(mx, max((w[e] << 16) & 0x7FFF0000u, w[e] & 0x7FFF0000u));
        atomicMax(&xb[(i * NT + tid) >> 5], mx);
      }
    }
    __syncthreads();
    if (tid < XR) {  // 2^-k with max |x| 2^-k < 2^15 (inf / NaN rows: k = 126, the result stays non-finite)
      const int ex = (int)(xb[tid] >> 23) - 127;
      xrow[tid] = __builtin_bit_cast(float, (unsigned)(127 - min(126, max(0, ex - 14))) << 23);
    }
    __syncthreads();
    run(std::true_type{});
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const float un = 1.f / xrow[16 * t + c];  // exact: a power of two
#pragma unroll
      for (int r = 0; r < RT; ++r) acc[r][t] *= un;
    }
  }
  if constexpr (kMoe && RT == 2) {
    if (glu) {
      if (gg >= (ngroups >> 1)) return;
      if constexpr (row_scaled<QT>()) {
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          const f32x4 rs = *reinterpret_cast<const f32x4*>(P.rs + 16 * gidx[r] + 4 * g);
#pragma unroll
          for (int t = 0; t < MT; ++t) acc[r][t] *= rs;
        }
      }
      const int col = 16 * gg + 4 * g;  // act column
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = mrow0 + 16 * t + c;
        if (moe.slots[m] < 0) continue;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned short gv = f32_to_bf16(acc[0][t][j]), uv = f32_to_bf16(acc[1][t][j]);
          o[j] = moe.glu == 2 ? gelu_mul1(gv, uv) : silu_mul1(gv, uv);
        }
        *reinterpret_cast<uint2*>(out + (long)m * out_stride + col) =
            uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
      }
      return;
    }
  }
  // C: col m = 16t + c, rows n = 16 gi + 4g + j
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    if (gi0 + r >= ngroups) continue;
    const int col = P.col + 16 * (gi0 + r) + 4 * g;
    if constexpr (row_scaled<QT>()) {
      const f32x4 rs = *reinterpret_cast<const f32x4*>(P.rs + 16 * (gi0 + r) + 4 * g);
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[r][t] *= rs;
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = mrow0 + 16 * t + c;  // output row (kMoe: slot)
      long wrow = (long)blockIdx.y * M + m;
      if constexpr (kMoe) {
        if (moe.slots[m] < 0) continue;
        wrow = (long)blockIdx.y * moe.nslots + m;
      } else if (m >= M) {
        continue;
      }
      if (ws != nullptr) {
        *reinterpret_cast<f32x4*>(ws + wrow * Ntot + col) = acc[r][t];
      } else {
        uint2 v;
        v.x = pack_bf16x2(acc[r][t][0], acc[r][t][1]);
        v.y = pack_bf16x2(acc[r][t][2], acc[r][t][3]);
        *reinterpret_cast<uint2*>(out + (long)m * out_stride + col) = v;
      }
    }
  }
}

template <int QA, int QB, int MT, int RT, int NWAVES, bool kX16 = false>
__global__ __launch_bounds__(64 * NWAVES) void qgemm2_kernel(unsigned short* __restrict__ out, long out_stride,
                                                            float* __restrict__ ws, const unsigned short* __restrict__ x,
                                                            long x_stride, Parts parts, int M, int Ntot, int K,
                                                            int sb_per_split, const unsigned short* __restrict__ x16) {
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][4 * x_plane<MT>()];
  __shared__ float xrow[16 * MT];  // per staged x row: power-of-two pre-scale (f16 range guard)
  const int tile = blockIdx.x;
  int pi = 0;
#pragma unroll
  for (int i = 1; i < kMaxParts; ++i)
    if (i < parts.n && tile >= parts.p[i].tile0) pi = i;
  const Part& P = parts.p[pi];
  if (QA == QB || P.qt == QA)
    qgemm2_body<QA, MT, RT, NWAVES, false, kX16>(xs, xrow, out, out_stride, ws, x, x_stride, P, M, Ntot, K,
                                                 sb_per_split, MoeQ{}, x16);
  else
    qgemm2_body<QB, MT, RT, NWAVES, false, kX16>(xs, xrow, out, out_stride, ws, x, x_stride, P, M, Ntot, K,
                                                 sb_per_split, MoeQ{}, x16);
}

// 33 <= M <= 64 body shape (HIPSERVE_QGEMM_M64, for A/B measurement): 0 = 8 waves x 1
// row group (default: measured 3-8 % faster at M = 64), 1 = 4 waves x 2 (both 128
// weight rows per workgroup), 2 = 8 waves x 2 (256 rows: half the x staging per weight byte)
int m64_variant() {
  static const int v = [] {
    const char* e = getenv("HIPSERVE_QGEMM_M64");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// the 256-row body for 33-64 rows: HIPSERVE_QGEMM_M64=2, and by default for LM-head
// widths (N >= 32K: 152 -> 136 us on the Q6_K 128K-vocab head, profiles/r4_gguf_m64_bodies.log;
// 8 waves x 1 row group stays faster on the layer projections)
bool m64_wide(int M, int Ntot) { return M > 32 && M <= 64 && (m64_variant() == 2 || (m64_variant() == 0 && Ntot >= 32768)); }

template <int QA, int QB>
void launch_t(void* out, long out_stride, float* ws, const void* x, long x_stride, const Parts& P, int tiles,
              int M, int Ntot, int K, int S, hipStream_t s, const void* x16) {
  constexpr int RT = 2, NW = kWaves;
  const int nsb = K / 256;
  const int per = (nsb + S - 1) / S;
  // M > 64 (K15, prefill): the 64-row body swept over the prompt, one M tile per blockIdx.z
  const dim3 grid(tiles, (nsb + per - 1) / per, M > 64 ? (M + 63) / 64 : 1), block(64 * NW);
  auto* o = static_cast<unsigned short*>(out);
  auto* xi = static_cast<const unsigned short*>(x);
  auto* xh = static_cast<const unsigned short*>(x16);
  if (M <= 16)
    qgemm2_kernel<QA, QB, 1, RT, NW><<<grid, block, 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per, nullptr);
  else if (M <= 32)
    qgemm2_kernel<QA, QB, 2, RT, NW><<<grid, block, 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per, nullptr);
  else if (m64_wide(M, Ntot) && xh != nullptr)  // 8 waves x 2 row groups: 256 rows share one x staging
    qgemm2_kernel<QA, QB, 4, 2, 8, true><<<grid, dim3(512), 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per,
                                                                    xh);
  else if (m64_wide(M, Ntot))
    qgemm2_kernel<QA, QB, 4, 2, 8><<<grid, dim3(512), 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per,
                                                              nullptr);
  else if (m64_variant() == 1)  // 4 waves x 2 row groups
    qgemm2_kernel<QA, QB, 4, RT, NW><<<grid, block, 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per, nullptr);
  else if (xh != nullptr && M <= 64)  // 8 waves x 1 row group, x staged from the producer's f16 copy
    qgemm2_kernel<QA, QB, 4, 1, 8, true><<<grid, dim3(512), 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per,
                                                                    xh);
  else  // 8 waves x 1 row group: half the accumulators and weight registers per wave
    qgemm2_kernel<QA, QB, 4, 1, 8><<<grid, dim3(512), 0, s>>>(o, out_stride, ws, xi, x_stride, P, M, Ntot, K, per,
                                                              nullptr);
}

// MoE experts: grid (row tiles of N, K splits, expert tiles); workgroups of tiles past
// the last one (tile_expert -1) exit before any barrier. The 16-slot body of the formats
// without a scale table (FP8, INT8C) fits 128 VGPRs without spills: 4 waves per SIMD
// instead of 3, a third more weight bytes in flight (the expert stream is bound by the
// loads in flight, not by its bytes: INT8's 12 % larger chunks ran as fast)
template <int QT, int MT, int RT, int NWAVES>
__global__ __launch_bounds__(64 * NWAVES) __attribute__((amdgpu_waves_per_eu(MT == 1 && QT != INT8 ? 4 : 1)))
void qmoe_kernel(unsigned short* __restrict__ out, long out_stride,
                                                          float* __restrict__ ws, const unsigned short* __restrict__ x,
                                                          long x_stride, const unsigned char* __restrict__ q,
                                                          const float* __restrict__ rs, MoeQ moe, int N, int K,
                                                          int sb_per_split) {
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][4 * x_plane<MT>()];
  __shared__ float xrow[16 * MT];
  const int e = moe.tile_expert[blockIdx.z];
  if (e < 0) return;
  const Part P{q + (long)e * moe.w_estride, rs != nullptr ? rs + (long)e * moe.rs_estride : nullptr, QT, N, 0, 0};
  qgemm2_body<QT, MT, RT, NWAVES, true>(xs, xrow, out, out_stride, ws, x, x_stride, P, 16 * MT, N, K, sb_per_split,
                                        moe);
}

template <int QT>
void moe_launch_t(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* q, const float* rs,
                  const MoeQ& moe, int tiles_cap, int tile, int N, int K, int S, hipStream_t s) {
  const int nsb = K / 256;
  const int per = (nsb + S - 1) / S;
  auto* o = static_cast<unsigned short*>(out);
  auto* xi = static_cast<const unsigned short*>(x);
  auto* qq = static_cast<const unsigned char*>(q);
  const int ysplit = (nsb + per - 1) / per;
  // GLU: 4 waves x one gate group (+ its up group) = 64 act columns per workgroup
  const int xt = moe.glu ? (N / 2 + 63) / 64 : (N + 127) / 128;
  if (tile == 16) {
    const dim3 grid(xt, ysplit, tiles_cap);
    qmoe_kernel<QT, 1, 2, kWaves><<<grid, 64 * kWaves, 0, s>>>(o, out_stride, ws, xi, x_stride, qq, rs, moe, N, K, per);
  } else if (tile == 32) {
    const dim3 grid(xt, ysplit, tiles_cap);
    qmoe_kernel<QT, 2, 2, kWaves><<<grid, 64 * kWaves, 0, s>>>(o, out_stride, ws, xi, x_stride, qq, rs, moe, N, K, per);
  } else {
    const dim3 grid((N + 127) / 128, ysplit, tiles_cap);
    qmoe_kernel<QT, 4, 1, 8><<<grid, 512, 0, s>>>(o, out_stride, ws, xi, x_stride, qq, rs, moe, N, K, per);
  }
}

// ---------------------------------------------------------------- tiled -> bf16
// Prefill: one wave per (row group, super-chunk) chunk, out[N, K] row-major bf16.
template <int QT>
// pack: 0 = row-major [N, K]; 1 / 2 = the packed prefill / decode GEMM layout of
// pack_decode_weight (2: gate/up-interleaved) for each stacked matrix of `nrows` rows
// (MoE experts: the row groups of expert e are [e nrows / 16, (e + 1) nrows / 16)) —
// every 8-value store of a lane is exactly one packed 16-byte piece.
__global__ __launch_bounds__(256) void dequant_tiled_kernel(unsigned short* __restrict__ out,
                                                            const unsigned char* __restrict__ q,
                                                            const float* __restrict__ rs, int ngroups, int K,
                                                            int pack, int nrows, int kmajor) {
  constexpr int CB = chunk_bytes<QT>();
  const int nsb = K >> 8;
  const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= (long)ngroups * nsb) return;
  const int gi = (int)(item / nsb), sb = (int)(item % nsb);
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  // kmajor: every stacked matrix of nrows rows is [K/256][nrows/16][chunk] (MoE w13)
  long src = item;
  if (kmajor) {
    const int kg = nrows >> 4, e = gi / kg;
    src = ((long)e * nsb + sb) * kg + (gi - e * kg);
  }
  Raw r;
  load_raw<QT>(q + src * CB, g, c, lane, r);
  Dec<QT> dec;
  dec.setup(r, g);
  unsigned short* row = out + (long)(16 * gi + c) * K + sb * 256;
  if (pack) {  // base of this lane's pieces in the packed copy of its matrix
    const int e = (16 * gi) / nrows, n = 16 * gi + c - e * nrows;
    int t, rgi;
    if (pack == 2) {  // tile t: gate rows [64 t, 64 t + 64), then the matching up rows
      const int half = nrows >> 1, up = n >= half, nn = up ? n - half : n;
      t = nn >> 6;
      rgi = (up ? 64 : 0) + (nn & 63);
    } else {
      t = n >> 7;
      rgi = n & 127;
    }
    // piece ((((t KS + sb) 8 + rg) 8 + s) 64 + lane), rg = rgi / 16, lane = g' 16 + (rgi % 16)
    row = out + (long)e * ((nrows + 127) / 128 * 128) * K +
          ((((long)t * (K >> 8) + sb) * 8 + (rgi >> 4)) * 8 * 64 + (rgi & 15)) * 8;
  }
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const f16x8 q = dec.ints(r, g, s);  // exact integers, pair order {0, 2, 1, 3, 4, 6, 5, 7}
    float d, m;
    dec.scale(r, g, s, d, m);           // fp32 scale: one rounding, to bf16, like the v1 dequant
    if constexpr (row_scaled<QT>()) d *= rs[16 * gi + c];
    constexpr int src[8] = {0, 2, 1, 3, 4, 6, 5, 7};
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16((float)q[src[j]] * d + m);
    const int kb = kbase<QT>(g, s);
    if (pack)  // k = 32 s' + 8 g' within the superblock -> slot s', lane g' 16 + row
      *reinterpret_cast<u16x8*>(row + ((kb >> 5) * 64 + ((kb >> 3) & 3) * 16) * 8) = o;
    else
      *reinterpret_cast<u16x8*>(row + kb) = o;
  }
}

// ---------------------------------------------------------------- tiled FP8 -> plain e4m3
// The per-channel FP8 tiled layout (ops/quant.py QuantPart.from_fp8: 16-byte piece (row n,
// k 16 c) of 128-k tile kt at [(n >> 4) nsb + kt / 2] 4096 + (c & 3) 1024 + (kt & 1) 512 +
// (c >> 2) 256 + (n & 15) 16) back to row-major [N, K] e4m3 bytes, for hipBLASLt's FP8
// prefill GEMM on a per-call scratch: the tiled decode copy stays the ONLY resident copy.
// One workgroup per 4 KiB chunk (16 rows x 256 k): a coalesced 16-byte read per thread,
// a transpose through LDS, and 16 threads per destination row writing its 256
// contiguous bytes (v1 gathered 16-byte pieces with the writes coalesced: ~2 TB/s).
__global__ __launch_bounds__(256) void fp8_untile_kernel(unsigned char* __restrict__ out,
                                                         const unsigned char* __restrict__ q, int K) {
  __shared__ __attribute__((aligned(16))) unsigned char t[16 * 272];  // 256-byte rows + 16 pad
  const int nsb = K >> 8, tid = threadIdx.x;
  const long ch = blockIdx.x;
  const int rg = (int)(ch / nsb), sb = (int)(ch - (long)rg * nsb);
  // source piece tid: row tid & 15, k 16 c + 128 (kt & 1) with c = 4 ((tid >> 4) & 1) + (tid >> 6),
  // kt & 1 = (tid >> 5) & 1
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q + ch * 4096 + tid * 16));
  const int c = 4 * ((tid >> 4) & 1) + (tid >> 6), kk = ((tid >> 5) & 1) * 128 + 16 * c;
  *reinterpret_cast<u32x4*>(&t[(tid & 15) * 272 + kk]) = v;
  __syncthreads();
  const int r = tid >> 4, j = tid & 15;
  *reinterpret_cast<u32x4*>(out + (long)(16 * rg + r) * K + sb * 256 + j * 16) =
      *reinterpret_cast<const u32x4*>(&t[r * 272 + j * 16]);
}

// ---------------------------------------------------------------- prefill GEMM
// qpg_kernel (GGUF prefill without the resident bf16 shadow):
// C[M, N] = X[M, K] . W^T straight from the tiled blocks, every weight dequantised ONCE
// per 256-token tile (the M-swept qgemm2 above does it once per 64 tokens and stages x
// for 128 weight rows; a dequantise-into-scratch + hipBLASLt pass writes and re-reads a
// bf16 copy of the whole matrix per call).
//   * X arrives as x16 (x_f16_pairs_kernel below): f16 in the weights' pair order, each
//     row pre-scaled by a power of two 2^-k that keeps it inside the f16 range, the
//     2^k in rsc[m] applied in the epilogue: converting bf16 x in every workgroup was
//     40 % of an earlier 8-wave body's VALU (tools/asm_stats.py; that body and a
//     4-wave / 128-token one: profiles/r4_qpf_bench_rt2.log, r4_qpf_bench_rt4.log);
//   * weight bytes per MFMA are 3.5x (Q4_K) fewer than a bf16 GEMM's, which is what
//     bounded the bf16 packed-layout kernel (profiles/r4_pw_diag_and_bench.log);
//   * epilogues: STORE (part columns), ADD (C is the residual: C = bf16(bf16(acc) + C)),
//     GLU (parts 0 / 1 = gate / up of the same format: a wave's first row groups are
//     gate rows, the others the matching up rows, act = silu(gate) * up in registers).
constexpr int QF_ROWS = 256;  // weight rows per STORE / ADD tile (GLU: 128 act columns)
struct QfArgs {
  Parts parts;
  const unsigned short* x16;  // [M, ldx] f16, pair order, row m scaled by 1 / rsc[m]
  const float* rsc;           // [M] power-of-two row scales
  long ldx;
  unsigned short* out;
  long ldo;
  int M, K, tiles_n, tiles_m;
};

// Shape: 4 waves x 4 row groups = 256 weight rows x 256 tokens (128 for Q5_K / Q6_K /
// Q8_0), one wave per SIMD, the 256 (128) accumulators in AGPRs. The earlier 8-wave body
// was bound by its dequant VALU per MFMA (a weight fragment fed only 8 MFMAs: 2.6 VALU per
// MFMA, MFMA pipe 45 % busy, profiles/r4_qpf_pmc_v1.log); here a fragment feeds 16, and x
// never passes through registers:
//   * x16 is staged by LDS-DMA (buffer_load ... lds, 1 KiB per wave instruction) in
//     half super-chunks (steps 0-3 / 4-7) into two LDS buffers; wave w loads plane
//     g = w, lane i of instruction j row 16 j + i / 4 and 16-byte slot i & 3, holding
//     fragment (i & 3) ^ ((i >> 4) & 3): the XOR swizzle makes every 16-lane group of
//     a B-fragment ds_read_b128 (rows 16 t .. 16 t + 15) hit 16 distinct bank quads;
//   * the next super-chunk's weight blocks load into the second register set while
//     this one is dequantised; each half buffer is refilled right after the barrier
//     that retires it, so a DMA has half a super-chunk (~4K MFMA cycles) to land;
//   * at 256 accumulators the MFMAs are inline asm on "+a" registers (no compiler AGPR
//     shuffles); the first one reading a freshly dequantised A operand carries the 2
//     wait states a VALU-written operand needs (s_nop 1).
template <int QT>
constexpr int qg_mt() { return QT == Q5_K || QT == Q6_K || QT == Q8_0 ? 8 : 16; }

// kAsm (256 accumulators, MT 16): the builtin had hipcc move accumulators between AGPRs
// and spill (tools/asm_stats.py); kNop: the first use of a freshly dequantised A operand
// (2 wait states after its VALU write; later uses of it are far from the write)
template <bool kAsm, bool kNop>
HS_DEVICE void qg_mfma(f32x4& acc, const f16x8& a, const f16x8& b) {
  if constexpr (!kAsm)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
  else if constexpr (kNop)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <int QT, int EPI>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void qpg_kernel(QfArgs A) {
  constexpr int RT = 4, NW = 4, MT = qg_mt<QT>(), XR = 16 * MT;
  constexpr int PLANE = XR * 64;  // bytes of one lane-group plane of a half buffer
  constexpr int NDMA = XR / 16;   // 1 KiB DMA instructions per wave and half
  constexpr int CB = chunk_bytes<QT>();
  constexpr bool kGlu = EPI == PW_EPI_GLU || EPI == PW_EPI_GEGLU;
  __shared__ __attribute__((aligned(1024))) unsigned char xs0[4 * PLANE];
  __shared__ __attribute__((aligned(1024))) unsigned char xs1[4 * PLANE];
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  constexpr int GM = 8;
  const int grp = L / (GM * A.tiles_n), first = grp * GM;
  const int gsz = min(GM, A.tiles_m - first);
  const int rrr = L - first * A.tiles_n;
  const int tm = first + rrr % gsz, tn = rrr / gsz;
  int pi = 0;
  if constexpr (!kGlu) {
#pragma unroll
    for (int i = 1; i < kMaxParts; ++i)
      if (i < A.parts.n && tn >= A.parts.p[i].tile0) pi = i;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int K = A.K, M = A.M, nsb = K >> 8;
  const Part& P = A.parts.p[pi];
  const int ngroups = P.rows >> 4;
  int gi[RT];
  const unsigned char* base[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    gi[r] = kGlu ? (tn * NW + wave) * (RT / 2) + r % (RT / 2) : (tn - P.tile0) * (QF_ROWS / 16) + wave * RT + r;
    const unsigned char* q = kGlu && r >= RT / 2 ? A.parts.p[1].q : P.q;
    base[r] = q + (long)min(gi[r], ngroups - 1) * nsb * CB;
  }
  // x16 rows of this tile; rows >= M lie outside the buffer range and read as zero
  const int mrow0 = tm * XR;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A.x16 + (long)mrow0 * A.ldx), 0, (int)((long)min(XR, M - mrow0) * A.ldx * 2), 0x00020000);
  const int sl = (lane & 3) ^ ((lane >> 4) & 3);  // fragment held by this lane's slot
  const int dvo0 = (((lane >> 2) * (int)A.ldx) + kbase<QT>(wave, sl)) * 2;
  const int dvo1 = (((lane >> 2) * (int)A.ldx) + kbase<QT>(wave, 4 + sl)) * 2;
  const int dstep = 16 * (int)A.ldx * 2;
  auto dma = [&](int sb, int h) {  // half h of super-chunk sb -> buffer h
    unsigned char* dst = (h ? xs1 : xs0) + wave * PLANE;
    const int vo = h ? dvo1 : dvo0;
#pragma unroll
    for (int j = 0; j < NDMA; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16,
                                               vo + j * dstep, sb * 512, 0, 0);  // rows in the range-checked offset
  };
  // B fragment (step s, token tile t): row 16 t + c, slot (s & 3) ^ ((c >> 2) & 3)
  const int rb = g * PLANE + c * 64;
  auto bfrag = [&](int s, int t) -> f16x8 {
    const unsigned char* src = (s < 4 ? xs0 : xs1) + rb + t * 1024 + (((s & 3) ^ ((c >> 2) & 3)) << 4);
    return *reinterpret_cast<const f16x8*>(src);
  };

  f32x4 acc[RT][MT];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[r][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  Raw rawA[RT], rawB[RT];
  dma(0, 0);
  dma(0, 1);
#pragma unroll
  for (int r = 0; r < RT; ++r) load_raw<QT>(base[r], g, c, lane, rawA[r]);
  __syncthreads();
  auto iter = [&](int sb, Raw (&cur)[RT], Raw (&nxt)[RT]) {
    const int sn = min(sb + 1, nsb - 1);  // the last super-chunk re-reads itself: no branch
#pragma unroll
    for (int r = 0; r < RT; ++r) load_raw<QT>(base[r] + (long)sn * CB, g, c, lane, nxt[r]);
    Dec<QT> dec[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) dec[r].setup(cur[r], g);
    // the A fragments of step s + 1 are dequantised between step s's MFMA groups (one
    // fragment per group of 4 x RT MFMAs): the MFMA pipe never waits for a dequant burst
    f16x8 a[RT], bq[4];
#pragma unroll
    for (int r = 0; r < RT; ++r) a[r] = dec[r].step(cur[r], g, 0);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (s == 4) {  // buffer 0 retired by every wave: refill it with the next half A
        __syncthreads();
        dma(sn, 0);
      }
      f16x8 an[RT];
      constexpr int NQ = MT / 4, PER = (RT + NQ - 1) / NQ;  // next-step fragments per group
      // x fragments one group ahead (from LDS, inside a half: the other half's buffer is
      // only complete after the barrier that opens it)
      if (s == 0 || s == 4) {
#pragma unroll
        for (int t = 0; t < 4; ++t) bq[t] = bfrag(s, t);
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        f16x8 b[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) b[t] = bq[t];
        const bool more = q + 1 < NQ || (s & 3) != 3;
        if (more) {
          const int sq = q + 1 < NQ ? s : s + 1, tq = q + 1 < NQ ? 4 * (q + 1) : 0;
#pragma unroll
          for (int t = 0; t < 4; ++t) bq[t] = bfrag(sq, tq + t);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < RT; ++r) {
            if (q == 0 && t == 0)
              qg_mfma<MT == 16, true>(acc[r][4 * q + t], a[r], b[t]);
            else
              qg_mfma<MT == 16, false>(acc[r][4 * q + t], a[r], b[t]);
          }
        if (s < 7) {
#pragma unroll
          for (int r = q * PER; r < min(RT, (q + 1) * PER); ++r) an[r] = dec[r].step(cur[r], g, s + 1);
        }
      }
      if (s < 7) {
#pragma unroll
        for (int r = 0; r < RT; ++r) a[r] = an[r];
      }
    }
    __syncthreads();  // buffer 1 retired
    dma(sn, 1);
  };
  int sb = 0;
  for (; sb + 1 < nsb; sb += 2) {
    iter(sb, rawA, rawB);
    iter(sb + 1, rawB, rawA);
  }
  if (sb < nsb) iter(sb, rawA, rawB);
  if constexpr (MT == 16)  // asm MFMAs: the hazard recognizer does not see them
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> accumulator reads
#pragma unroll
  for (int t = 0; t < MT; ++t) {  // undo the row pre-scale (exact: a power of two)
    const float sc = A.rsc[min(mrow0 + 16 * t + c, M - 1)];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r][t] *= sc;
  }
  if constexpr (kGlu) {
#pragma unroll
    for (int r = 0; r < RT / 2; ++r) {
      if (gi[r] >= ngroups) continue;
      const int col = 16 * gi[r] + 4 * g;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = mrow0 + 16 * t + c;
        if (m >= M) continue;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned short gv = f32_to_bf16(acc[r][t][j]), uv = f32_to_bf16(acc[r + RT / 2][t][j]);
          o[j] = EPI == PW_EPI_GEGLU ? gelu_mul1(gv, uv) : silu_mul1(gv, uv);
        }
        *reinterpret_cast<uint2*>(A.out + (long)m * A.ldo + col) =
            uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      if (gi[r] >= ngroups) continue;
      const int col = P.col + 16 * gi[r] + 4 * g;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = mrow0 + 16 * t + c;
        if (m >= M) continue;
        uint2* dst = reinterpret_cast<uint2*>(A.out + (long)m * A.ldo + col);
        float o[4];
        if constexpr (EPI == PW_EPI_ADD) {
          const uint2 rv = *dst;
          const unsigned short rr[4] = {(unsigned short)(rv.x & 0xffff), (unsigned short)(rv.x >> 16),
                                        (unsigned short)(rv.y & 0xffff), (unsigned short)(rv.y >> 16)};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = bf16_to_f32(f32_to_bf16(acc[r][t][j])) + bf16_to_f32(rr[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = acc[r][t][j];
        }
        *dst = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      }
    }
  }
}

template <int QT>
void qpg_launch(int epi, QfArgs A, hipStream_t s) {
  A.tiles_m = (A.M + 16 * qg_mt<QT>() - 1) / (16 * qg_mt<QT>());
  const dim3 grid(A.tiles_n * A.tiles_m), block(256);
  switch (epi) {
    case PW_EPI_STORE: qpg_kernel<QT, PW_EPI_STORE><<<grid, block, 0, s>>>(A); break;
    case PW_EPI_ADD: qpg_kernel<QT, PW_EPI_ADD><<<grid, block, 0, s>>>(A); break;
    case PW_EPI_GLU: qpg_kernel<QT, PW_EPI_GLU><<<grid, block, 0, s>>>(A); break;
    case PW_EPI_GEGLU: qpg_kernel<QT, PW_EPI_GEGLU><<<grid, block, 0, s>>>(A); break;
  }
}

// x [M, K] bf16 -> x16 [M, K] f16 in the pair order {0, 2, 1, 3, 4, 6, 5, 7} of every
// aligned 8-run, each row scaled by 2^-k (max |x| 2^-k in [2^14, 2^15)), rsc[m] = 2^k: the prefill GEMM's operand, converted once per activation instead
// of in every workgroup; bf16 -> f32 exact, -> f16 round to nearest (values below the f16
// normal range lose low bits, as in the decode kernel's staging)
__global__ __launch_bounds__(256) void x_f16_pairs_kernel(unsigned short* __restrict__ x16, float* __restrict__ rsc,
                                                          const unsigned short* __restrict__ x, long ldx, int K) {
  const int row = blockIdx.x, tid = threadIdx.x;
  const u16x8* src = reinterpret_cast<const u16x8*>(x + (long)row * ldx);
  u16x8* dst = reinterpret_cast<u16x8*>(x16 + (long)row * K);
  const int n8 = K >> 3;
  unsigned mx = 0;
  for (int j = tid; j < n8; j += 256) {
    const u32x4 w = __builtin_bit_cast(u32x4, src[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) mx = max(mx, max((w[e] << 16) & 0x7FFF0000u, w[e] & 0x7FFF0000u));
  }
  __shared__ unsigned red[4];
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = max(max(red[0], red[1]), max(red[2], red[3]));
  // 2^-k with max |x| 2^-k in [2^14, 2^15): rows of small activations are scaled UP as
  // well (their elements would otherwise sit in the f16 subnormal range and lose bits);
  // k >= -100 keeps both 2^k and 2^-k normal floats (all-zero rows); inf / NaN rows:
  // k = 126, the result stays non-finite
  const int ex = (int)(mx >> 23) - 127;
  const int k = min(126, max(-100, ex - 14));
  const float down = __builtin_bit_cast(float, (unsigned)(127 - k) << 23);
  if (tid == 0) rsc[row] = __builtin_bit_cast(float, (unsigned)(127 + k) << 23);
  constexpr int ord[8] = {0, 2, 1, 3, 4, 6, 5, 7};
  for (int j = tid; j < n8; j += 256) {
    const u16x8 v = src[j];
    u16x8 h;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      h[e] = __builtin_bit_cast(unsigned short, static_cast<_Float16>(bf16_to_f32(v[ord[e]]) * down));
    dst[j] = h;
  }
}

}  // namespace

int gguf_tiled_chunk_bytes(int qtype) {
  switch (qtype) {
    case Q4_0: return chunk_bytes<Q4_0>();
    case Q4_1: return chunk_bytes<Q4_1>();
    case Q8_0: return chunk_bytes<Q8_0>();
    case Q4_K: return chunk_bytes<Q4_K>();
    case Q5_K: return chunk_bytes<Q5_K>();
    case Q6_K: return chunk_bytes<Q6_K>();
    case FP8: return chunk_bytes<FP8>();
    case FP8B: return chunk_bytes<FP8B>();
    case INT8: return chunk_bytes<INT8>();
    case INT8C: return chunk_bytes<INT8C>();
  }
  return 0;
}

// Parts in the tiled layout. ws != nullptr: fp32 partials [S, M, Ntot]; else bf16
// out (S must be 1). Parts of one format, or of the pairs Q4_K+Q6_K / Q5_K+Q6_K
// (the K-quant mixes), share one launch; any other mix launches per format.
void launch_gguf_gemm_parts(void* out, long out_stride, float* ws, const void* x, long x_stride,
                            const GgufPart* parts, int nparts, int M, int Ntot, int K, int S, hipStream_t s,
                            const void* x16) {
  // weight rows per workgroup: 128, or 256 for the wide M = 33-64 body (m64_wide)
  const int ROWS = m64_wide(M, Ntot) ? 256 : 16 * 2 * kWaves;
  int fmts[kMaxParts], nf = 0;
  for (int i = 0; i < nparts; ++i) {
    bool seen = false;
    for (int j = 0; j < nf; ++j) seen |= fmts[j] == parts[i].qtype;
    if (!seen) fmts[nf++] = parts[i].qtype;
  }
  auto table = [&](int fa, int fb, int& tiles) {
    Parts P{};
    tiles = 0;
    for (int i = 0; i < nparts; ++i) {
      if (parts[i].qtype != fa && parts[i].qtype != fb) continue;
      P.p[P.n++] = Part{static_cast<const unsigned char*>(parts[i].q), parts[i].rs, parts[i].qtype, parts[i].rows,
                        parts[i].col, tiles};
      tiles += (parts[i].rows + ROWS - 1) / ROWS;
    }
    return P;
  };
  int tiles = 0;
  if (nf == 2) {
    const int a = fmts[0] < fmts[1] ? fmts[0] : fmts[1], b = fmts[0] < fmts[1] ? fmts[1] : fmts[0];
    if ((a == Q4_K || a == Q5_K) && b == Q6_K) {
      const Parts P = table(a, b, tiles);
      if (a == Q4_K) launch_t<Q4_K, Q6_K>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16);
      else launch_t<Q5_K, Q6_K>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16);
      return;
    }
  }
  for (int f = 0; f < nf; ++f) {
    const Parts P = table(fmts[f], fmts[f], tiles);
    switch (fmts[f]) {
      case Q4_0: launch_t<Q4_0, Q4_0>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case Q4_1: launch_t<Q4_1, Q4_1>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case Q8_0: launch_t<Q8_0, Q8_0>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case Q4_K: launch_t<Q4_K, Q4_K>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case Q5_K: launch_t<Q5_K, Q5_K>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case Q6_K: launch_t<Q6_K, Q6_K>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case FP8: launch_t<FP8, FP8>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case FP8B: launch_t<FP8B, FP8B>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case INT8: launch_t<INT8, INT8>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
      case INT8C: launch_t<INT8C, INT8C>(out, out_stride, ws, x, x_stride, P, tiles, M, Ntot, K, S, s, x16); break;
    }
  }
}

bool launch_qmoe_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* q,
                      const float* rs, int qtype, long w_estride, long rs_estride, const int* slots,
                      const int* tile_expert, int tiles_cap, int tile, int gather_k, int N, int K, int S,
                      hipStream_t s, bool kmajor, int glu) {
  if (tile != 16 && tile != 32 && tile != 64) return false;
  // GLU epilogue: the 16 / 32-slot bodies (two row groups per wave), whole K, N / 2 % 16
  if (glu && (tile == 64 || S != 1 || ws != nullptr || (N / 2) % 16)) return false;
  const MoeQ moe{slots, tile_expert, w_estride, rs_estride, gather_k, tiles_cap * tile, kmajor ? 1 : 0, glu};
  switch (qtype) {
    case FP8: moe_launch_t<FP8>(out, out_stride, ws, x, x_stride, q, rs, moe, tiles_cap, tile, N, K, S, s); return true;
    case INT8: moe_launch_t<INT8>(out, out_stride, ws, x, x_stride, q, rs, moe, tiles_cap, tile, N, K, S, s); return true;
    case INT8C: moe_launch_t<INT8C>(out, out_stride, ws, x, x_stride, q, rs, moe, tiles_cap, tile, N, K, S, s); return true;
  }
  return false;
}

// Prefill GEMM over tiled GGUF parts (qpg_kernel) on x16 / rsc from launch_x_f16_pairs
// (row stride K). STORE: out[:, col .. col + rows) per
// part; ADD: out is the residual (updated in place); GLU / GEGLU: parts 0 / 1 are gate / up
// (same format and rows), out[M, rows] = act(gate) * up. Formats: GGUF (Q4_0 .. Q6_K);
// a mix of formats launches once per format (one body per launch: a two-format kernel
// spills). Returns false for shapes / formats it does not take (the caller falls back).
void launch_x_f16_pairs(void* x16, float* rsc, const void* x, long ldx, int M, int K, hipStream_t s) {
  x_f16_pairs_kernel<<<M, 256, 0, s>>>(static_cast<unsigned short*>(x16), rsc, static_cast<const unsigned short*>(x),
                                       ldx, K);
}

bool launch_gguf_prefill(int epi, void* out, long ldo, const void* x16, const float* rsc, const GgufPart* parts,
                         int nparts, int M, int K, hipStream_t s) {
  const long ldx = K;
  const bool glu = epi == PW_EPI_GLU || epi == PW_EPI_GEGLU;
  if (M < 1 || K < 256 || K % 256 || nparts < 1 || nparts > kMaxParts || (glu && nparts != 2)) return false;
  if (epi != PW_EPI_STORE && epi != PW_EPI_ADD && !glu) return false;
  // 32-bit buffer offsets inside one x tile
  if ((long)256 * ldx * 2 >= (1L << 31)) return false;  // the largest tile's x rows (qpg: 256)
  for (int i = 0; i < nparts; ++i)
    if (parts[i].qtype < Q4_0 || parts[i].qtype > Q6_K || parts[i].rows % 16) return false;
  if (glu && (parts[0].qtype != parts[1].qtype || parts[0].rows != parts[1].rows)) return false;
  int fmts[kMaxParts], nf = 0;
  for (int i = 0; i < nparts; ++i) {
    bool seen = false;
    for (int j = 0; j < nf; ++j) seen |= fmts[j] == parts[i].qtype;
    if (!seen) fmts[nf++] = parts[i].qtype;
  }
  auto run = [&](int fa) {
    QfArgs A{};
    A.x16 = static_cast<const unsigned short*>(x16);
    A.rsc = rsc;
    A.ldx = ldx;
    A.out = static_cast<unsigned short*>(out);
    A.ldo = ldo;
    A.M = M;
    A.K = K;
    int tiles = 0;
    for (int i = 0; i < nparts; ++i) {
      if (parts[i].qtype != fa) continue;
      A.parts.p[A.parts.n++] = Part{static_cast<const unsigned char*>(parts[i].q), nullptr, parts[i].qtype,
                                    parts[i].rows, parts[i].col, tiles};
      tiles += (parts[i].rows + QF_ROWS - 1) / QF_ROWS;
    }
    A.tiles_n = glu ? (parts[0].rows + QF_ROWS / 2 - 1) / (QF_ROWS / 2) : tiles;
#define QF_CASE(QT_)          \
  if (fa == QT_) {              \
    qpg_launch<QT_>(epi, A, s); \
    return;                     \
  }
    QF_CASE(Q4_0) QF_CASE(Q4_1) QF_CASE(Q8_0) QF_CASE(Q4_K) QF_CASE(Q5_K) QF_CASE(Q6_K)
#undef QF_CASE
  };
  if (glu && nf != 1) return false;
  for (int f = 0; f < nf; ++f) run(fmts[f]);
  return true;
}

void launch_fp8_untile(void* out, const void* q, int N, int K, hipStream_t s) {
  const long chunks = (long)(N / 16) * (K / 256);
  if (chunks <= 0) return;
  fp8_untile_kernel<<<(unsigned)chunks, 256, 0, s>>>(static_cast<unsigned char*>(out),
                                                     static_cast<const unsigned char*>(q), K);
}

void launch_gguf_dequant_tiled(void* out, const void* q, const float* rs, int qtype, int N, int K, hipStream_t s,
                               int pack, int nrows, bool kmajor) {
  if (nrows <= 0) nrows = N;
  const long items = (long)(N / 16) * (K / 256);
  const dim3 grid((unsigned)((items + 3) / 4)), block(256);
  auto* o = static_cast<unsigned short*>(out);
  auto* qq = static_cast<const unsigned char*>(q);
  switch (qtype) {
    case Q4_0: dequant_tiled_kernel<Q4_0><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case Q4_1: dequant_tiled_kernel<Q4_1><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case Q8_0: dequant_tiled_kernel<Q8_0><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case Q4_K: dequant_tiled_kernel<Q4_K><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case Q5_K: dequant_tiled_kernel<Q5_K><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case Q6_K: dequant_tiled_kernel<Q6_K><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case FP8: dequant_tiled_kernel<FP8><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case FP8B: dequant_tiled_kernel<FP8B><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case INT8: dequant_tiled_kernel<INT8><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
    case INT8C: dequant_tiled_kernel<INT8C><<<grid, block, 0, s>>>(o, qq, rs, N / 16, K, pack, nrows, kmajor ? 1 : 0); break;
  }
}

}  // namespace hipserve
