// Prefill GEMM over the decode kernels' packed weight layout (VERDICT r3, next round item
// 1: one weight layout for prefill and decode, hand-written MFMA on the prefill hot path):
//
//   C[M, N] = X[M, K] . W[N, K]^T      bf16 in, fp32 accumulate, epilogue fused
//
// W is read from pack_decode_weight's copy (decode_gemm.hip),
// [ceil(N/128)][K/256][8 row groups][8 k-slots][64 lanes][8 bf16]: every 1 KiB
// (row group, k-slot) piece is exactly the first operand of one
// v_mfma_f32_16x16x32_bf16 for a wave (lane l: row 16 rg + (l & 15), k 32 s + 8 (l >> 4)).
// Weight fragments therefore go global -> VGPR with ONE coalesced buffer_load_dwordx4
// each and never touch LDS. Only X is staged through LDS. Per 32-deep K step a wave issues
// 8 LDS fragment reads + XP/2 staging writes, against 16 reads (+ 8 writes) when both
// operands are staged — LDS issue was what held the previous kernels at ~55 % MFMA
// busy (profiles/r3_pgemm_pmc.md).
//
// Geometry: 256 threads = 4 waves, one per SIMD (512 registers each), every wave a
// 128 (m) x 128 (n) output block = ONE packed weight tile: 64 accumulator tiles
// acc[rg][i] (rg: 16-row weight group, i: 16-row X group) = 256 fp32 per lane.
// WM x WN waves per workgroup: WM = 1 -> 128 x 512 (X staged once for four weight
// tiles), WM = 2 -> 256 x 256 (two waves stream the same weight tile, the second read
// is an L1 / L2 hit).
//
// Pipeline, per 64-deep K stage st (two 32-deep slots, 64 MFMAs per wave each):
//   slot 2st   : MFMA(wa, xa) row group by row group; after a group's 8 MFMAs its
//                weight register is reloaded with slot 2st + 2; the X fragments of slot
//                2st + 1 (xb) are read from LDS stage st; stage st + 1 (registers,
//                loaded two slots ago) is written to the other LDS buffer and stage
//                st + 2 is loaded from global; ONE barrier closes the slot.
//   slot 2st+1 : MFMA(wb, xb); wb reloaded with slot 2st + 3; xa <- LDS stage st + 1.
// Weight and X global loads are two slots (~2,000 MFMA cycles) ahead of their use. Loads
// past the end re-read the last slot / stage (clamped offsets: no branches in the loop,
// so the compiler's vmcnt waits stay exact). Rows past M read as zero (buffer range).
//
// Epilogues (lane holds C[m][n .. n+3], m = m0 + 128 wm + 16 i + (l & 15),
// n = 128 t + 16 rg + 4 (l >> 4)):
//   PW_EPI_STORE  C = bf16(acc) (+ bias[n])
//   PW_EPI_ADD    C (the residual, in place) = bf16(bf16(acc) + C)
//   PW_EPI_GLU    W packed with glu=true (each tile: 64 gate rows then their 64 up
//                 rows): gate rg and up rg + 4 sit in the same lane, so
//                 act[m, 64 t + 16 rg + 4 (l >> 4) + j] = silu(gate) * up in registers
//   PW_EPI_GEGLU  as GLU with tanh-GELU (Gemma)
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int PW_T = 256;

// Persistent tile walk: G workgroups (one per CU), workgroup b takes tiles
// L = it * G + r (r = b remapped so an XCD's workgroups hold consecutive r), and a
// logical tile L -> (tm, tn) walks groups of PW_GM m-tiles n-major: the ~32 workgroups an
// XCD runs at once cover 8 m-tiles x 4 n-tiles and share both operands in its L2.
constexpr int PW_GM = 8;
HS_DEVICE void pw_tile(int L, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int grp = L / (PW_GM * tiles_n), first = grp * PW_GM;
  const int gsz = min(PW_GM, tiles_m - first);
  const int r = L - first * tiles_n;
  tm = first + r % gsz;
  tn = r / gsz;
}

HS_DEVICE void pw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MFMA on an AGPR accumulator as inline asm: with the builtin, hipcc moved the 256
// accumulators between AGPRs inside the loop (tools/asm_stats.py: ~200 v_accvgpr moves
// per 128 MFMAs). asm MFMAs are invisible to the hazard recognizer: the epilogue covers the
// MFMA -> VALU read of the accumulators by hand.
HS_DEVICE void pw_mfma(f32x4& acc, const u32x4& w, const u32x4& x) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(x));
}

// per-tile operand streams of one wave: its weight tile and the workgroup's X rows
struct PwTile {
  __amdgpu_buffer_rsrc_t w, x;
  int m0, t;
  int xo[8];  // kGather: this thread's byte offsets of its X rows (row p * 32 + (tid >> 3))
};

template <int WM, bool kGroup, bool kGather = false>
HS_DEVICE PwTile pw_make(int L, int tiles_m, int tiles_n, int wn, const unsigned short* X, long ldx,
                         const unsigned short* Wp, int M, int ntiles, int KS, const PwGroup& grp) {
  constexpr int WN = 4 / WM, BM = 128 * WM;
  int tm, tn;
  pw_tile(L, tiles_m, tiles_n, tm, tn);
  PwTile T;
  T.m0 = tm * BM;
  T.t = tn * WN + wn;
  const int tl = min(T.t, ntiles - 1);  // waves past the last weight tile compute a copy, store nothing
  // this m-tile's expert. readfirstlane: a load through a generic pointer counts as
  // divergent, which put the weight descriptor in VGPRs and wrapped every weight load of
  // the main loop in a waterfall loop (tools/asm_stats.py: 197 VALU per loop body vs 0)
  if constexpr (kGroup) Wp += (long)__builtin_amdgcn_readfirstlane(grp.tile_expert[tm]) * grp.estride;
  T.w = __builtin_amdgcn_make_buffer_rsrc((void*)(Wp + (long)tl * KS * 32768), 0, KS * 65536, 0x00020000);
  if constexpr (kGather) {  // token rows through the slot table; padding slots read past the end = zero
    const int bytes = (int)((long)grp.x_rows * ldx * 2);
    T.x = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, bytes, 0x00020000);
    const int tid = threadIdx.x;
#pragma unroll
    for (int p = 0; p < BM / 32; ++p) {
      const int row = T.m0 + p * 32 + (tid >> 3);
      const int s = row < M ? grp.gather_slots[row] : -1;
      T.xo[p] = (s >= 0 ? (s / grp.gather_k) * (int)ldx * 2 : bytes) + (tid & 7) * 16;
    }
  } else {
    // rows >= M fall outside the buffer range and read as zero
    T.x = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (long)T.m0 * ldx), 0,
                                            (int)((long)min(BM, M - T.m0) * ldx * 2), 0x00020000);
  }
  return T;
}

// kGroup (MoE prefill experts): X rows are expert-sorted slots in BM-row tiles
// (moe_align with tile BM, moe_gather); m-tile tm multiplies expert grp.tile_expert[tm]'s
// packed weight (Wp + e * estride) and only the first *grp.num_tiles m-tiles (the
// device-side count: no host round trip, graph-capturable) are walked.
template <int WM, int EPI, bool kGroup, int RW, bool LDLY = false, bool kGather = false>
__global__ __launch_bounds__(PW_T) __attribute__((amdgpu_waves_per_eu(1, 1))) void pgw_kernel(
    const unsigned short* __restrict__ X, long ldx, const unsigned short* __restrict__ Wp,
    unsigned short* __restrict__ C, long ldc, int M, int N, int K, int tiles_m, int tiles_n,
    const unsigned short* __restrict__ bias, PwGroup grp) {
  constexpr int WN = 4 / WM, BM = 128 * WM, STAGE = BM * 128, XP = BM / 32;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  const int ntiles = (N + 127) >> 7;
  const int KS = K >> 8, nq = K >> 5, nst = K >> 6;
  if constexpr (kGroup) tiles_m = min(tiles_m, __builtin_amdgcn_readfirstlane(*grp.num_tiles));
  const int total = tiles_m * tiles_n, G = gridDim.x;
  const int r = xcd_remap(blockIdx.x, G);
  if (r >= total) return;

  // cur: the tile whose MFMAs run; nxt: the one the loads past cur's end stream in, so
  // the pipeline runs on across the tile boundary (only the epilogue sits between)
  PwTile cur = pw_make<WM, kGroup, kGather>(r, tiles_m, tiles_n, wn, X, ldx, Wp, M, ntiles, KS, grp);
  PwTile nxt = r + G < total ? pw_make<WM, kGroup, kGather>(r + G, tiles_m, tiles_n, wn, X, ldx, Wp, M, ntiles, KS, grp) : cur;

  const int wvo = lane * 16;
  auto wload = [&](int q, int rg) -> u32x4 {  // 32-deep slot q of cur (q >= nq: of nxt), row group rg
    const bool n = q >= nq;
    q = n ? q - nq : q;
    return __builtin_amdgcn_raw_buffer_load_b128(n ? nxt.w : cur.w, wvo, (q >> 3) * 65536 + rg * 8192 + (q & 7) * 1024,
                                                 0);
  };
  // X staging: thread -> rows 32 p + (tid >> 3), 16-byte chunk tid & 7 of the 128-byte
  // (64-deep) row
  int xvo[XP];
#pragma unroll
  for (int p = 0; p < XP; ++p) xvo[p] = (p * 32 + (tid >> 3)) * (int)ldx * 2 + (tid & 7) * 16;
  // LDS image [BM rows][128 B]: 16-byte chunk c of row r at chunk c ^ ((r >> 1) & 7), which
  // spreads each ds_read_b128 lane group (rows 0-3 / 12-15 of one chunk, 4-11 of the
  // next) over all 16 slots of a 256-byte bank row; (r >> 1) & 7 is the same for rows
  // r and r + 32 p
  const int xdo = (tid >> 3) * 128 + (((tid & 7) ^ ((tid >> 4) & 7)) * 16);
  // RW weight register sets (one per 32-deep slot in flight: a set's next slot is
  // loaded right after its MFMAs, RW slots ahead) and XS = RW / 2 X staging sets (stage
  // s + 1 + XS is loaded into the set stage s + 1 was just written to LDS from)
  constexpr int XS = RW / 2;
  u32x4 xst[XS][XP];
  auto xload = [&](int st, u32x4 (&xs)[XP]) {  // 64-deep stage st of cur (st >= nst: of nxt)
    const bool n = st >= nst;
    st = n ? st - nst : st;
#pragma unroll
    for (int p = 0; p < XP; ++p)
      xs[p] = __builtin_amdgcn_raw_buffer_load_b128(n ? nxt.x : cur.x, kGather ? (n ? nxt.xo[p] : cur.xo[p]) : xvo[p],
                                                    st * 128, 0);
  };
  auto xstore = [&](int buf, const u32x4 (&xs)[XP]) {
#pragma unroll
    for (int p = 0; p < XP; ++p) *reinterpret_cast<u32x4*>(lds + buf * STAGE + p * 4096 + xdo) = xs[p];
  };
  const int fr = lane & 15, fq = lane >> 4, sw = (fr >> 1) & 7;
  const int foff = (wm * 128 + fr) * 128;
  const int ch[2] = {(fq ^ sw) * 16, ((4 + fq) ^ sw) * 16};
  auto xfrag = [&](int buf, int h, int i) -> u32x4 {
    return *reinterpret_cast<const u32x4*>(lds + buf * STAGE + foff + i * 2048 + ch[h]);
  };

  f32x4 acc[8][8];
  u32x4 w[RW][8], xa[8], xb[8];
  int wvoj[RW];
#pragma unroll
  for (int j = 0; j < RW; ++j) wvoj[j] = wvo + j * 1024;

  // prologue (first tile only): stage 0 in LDS, stages 1 .. XS in registers, weight
  // slots 0 .. RW - 1 in flight; later tiles find theirs loaded by the previous tile's
  // last slots
  xload(0, xst[0]);
  xstore(0, xst[0]);
#pragma unroll
  for (int s = 1; s <= XS; ++s) xload(s, xst[s % XS]);
#pragma unroll
  for (int j = 0; j < RW; ++j)
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) w[j][rg] = wload(j, rg);
  pw_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) xa[i] = xfrag(0, 0, i);

  // one 32-deep slot: J (compile time) = slot index inside the RW-slot loop body. The
  // weight loads of one loop body all stream the same tile (nq % RW == 0): their buffer
  // resource and K offset are chosen once per body (wrs, wk), so a load costs one scalar
  // add — per-load selects cost ~6 SALU each and delayed the next MFMA group
  // (tools/asm_stats.py)
  auto slot = [&](auto jc, int s0, const __amdgpu_buffer_rsrc_t& wrs, int wk) {
    constexpr int J = decltype(jc)::value, H = J & 1;
    const int s = s0 + J / 2, buf = s & 1;
    constexpr int XI = (J / 2 + 1) % XS;  // staging set of stage s + 1 (s0 is a multiple of XS)
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
#pragma unroll
      for (int i = 0; i < 8; ++i) pw_mfma(acc[rg][i], w[J][rg], H ? xb[i] : xa[i]);
      // slot J's 1 KiB offset rides in a per-slot VGPR offset: 8 scalar adds per body, not 32.
      // LDLY: reload a group's weight register one group later, so the load is not issued
      // right behind the MFMAs still reading that register
      if constexpr (LDLY) {
        if (rg > 0) w[J][rg - 1] = __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoj[J], wk + (rg - 1) * 8192, 0);
        if (rg == 7) w[J][7] = __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoj[J], wk + 7 * 8192, 0);
      } else {
        w[J][rg] = __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoj[J], wk + rg * 8192, 0);
      }
      if constexpr (H == 0) {
        xb[rg] = xfrag(buf, 1, rg);
        if (rg == 2) xstore(buf ^ 1, xst[XI]);     // stage s + 1 (loaded XS stages ago)
        if (rg == 3) xload(s + 1 + XS, xst[XI]);
      } else {
        xa[rg] = xfrag(buf ^ 1, 0, rg);            // stage s + 1, visible since the barrier
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (H == 0) pw_barrier();  // stage s + 1 visible; every read of stage s - 1 done
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  for (int L = r;;) {
#pragma unroll
    for (int rg = 0; rg < 8; ++rg)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[rg][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int q0 = 0; q0 < nq; q0 += RW) {  // nq % 8 == 0; a tile starts in LDS buffer 0
      const int s0 = q0 >> 1;
      const bool wn = q0 + RW >= nq;  // this body's weight loads stream the next tile
      const int wq = wn ? q0 + RW - nq : q0 + RW;
      const __amdgpu_buffer_rsrc_t wrs = wn ? nxt.w : cur.w;
      const int wk = (wq >> 3) * 65536 + (wq & 7) * 1024;  // (wq & 7) + J <= 7
      slot(I0(), s0, wrs, wk);
      slot(I1(), s0, wrs, wk);
      if constexpr (RW == 4) {
        slot(I2(), s0, wrs, wk);
        slot(I3(), s0, wrs, wk);
      }
    }

    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA -> VALU reads
    const int t = cur.t, mb = cur.m0 + wm * 128 + fr;
    if (t < ntiles) {
      if constexpr (EPI == PW_EPI_GLU || EPI == PW_EPI_GEGLU) {
        const int I = N >> 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m = mb + 16 * i;
          if (m >= M) continue;
#pragma unroll
          for (int rg = 0; rg < 4; ++rg) {
            const int c = t * 64 + rg * 16 + 4 * fq;
            unsigned short o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const unsigned short g = f32_to_bf16(acc[rg][i][j]), u = f32_to_bf16(acc[rg + 4][i][j]);
              o[j] = EPI == PW_EPI_GEGLU ? gelu_mul1(g, u) : silu_mul1(g, u);
            }
            if (c < I)
              *reinterpret_cast<uint2*>(C + (long)m * ldc + c) =
                  uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
          }
        }
      } else {
#pragma unroll
        for (int rg = 0; rg < 8; ++rg) {
          const int n = t * 128 + rg * 16 + 4 * fq;
          if (n >= N) continue;
          float bv[4] = {0.f, 0.f, 0.f, 0.f};
          if (bias != nullptr)
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = n + j < N ? bf16_to_f32(bias[n + j]) : 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = mb + 16 * i;
            if (m >= M) continue;
            uint2* dst = reinterpret_cast<uint2*>(C + (long)m * ldc + n);
            float o[4];
            if constexpr (EPI == PW_EPI_ADD) {  // C is the residual: C = bf16(bf16(acc) + C)
              const uint2 rv = *dst;
              const unsigned short rr[4] = {(unsigned short)(rv.x & 0xffff), (unsigned short)(rv.x >> 16),
                                            (unsigned short)(rv.y & 0xffff), (unsigned short)(rv.y >> 16)};
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] = bf16_to_f32(f32_to_bf16(acc[rg][i][j])) + bf16_to_f32(rr[j]);
            } else {  // bias added to the fp32 accumulator, one rounding
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] = acc[rg][i][j] + bv[j];
            }
            *dst = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
          }
        }
      }
    }
    L += G;
    if (L >= total) break;
    cur = nxt;
    if (L + G < total) nxt = pw_make<WM, kGroup, kGather>(L + G, tiles_m, tiles_n, wn, X, ldx, Wp, M, ntiles, KS, grp);
  }
}

bool launch_prefill_gemm_packed(int epi, void* C, long ldc, const void* X, long ldx, const void* Wp, int M, int N,
                                int K, const void* bias, int wm, int grid_req, hipStream_t s, const PwGroup* group,
                                int rw) {
  const PwGroup grp = group != nullptr ? *group : PwGroup{nullptr, nullptr, 0};
  const bool grouped = group != nullptr;
  const bool gather = grouped && grp.gather_slots != nullptr;
  if (grouped && (bias != nullptr || epi == PW_EPI_ADD)) return false;
  // (the gather form always runs rw = 4, PW_LAUNCH1: any rw knob value is accepted)
  if (gather && (grp.gather_k < 1 || (long)grp.x_rows * ldx * 2 >= (1L << 31) - 4096)) return false;
  if (M < 1 || N < 1 || K < 256 || K % 256 || (wm != 1 && wm != 2) || (rw != 2 && rw != 4 && rw != 5)) return false;
  const bool glu = epi == PW_EPI_GLU || epi == PW_EPI_GEGLU;
  if (glu && (N % 128 || bias != nullptr)) return false;
  if (epi == PW_EPI_ADD && bias != nullptr) return false;
  // 32-bit buffer offsets: the weight stream of one tile and one workgroup's X rows
  if ((long)(K / 256) * 65536 >= (1L << 31) || (long)128 * wm * ldx * 2 >= (1L << 31)) return false;
  const int BM = 128 * wm, WN = 4 / wm;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = ((N + 127) / 128 + WN - 1) / WN;
  // persistent: one workgroup per CU (grid <= 0) unless the caller asks for a grid
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  }
  const int total = tiles_m * tiles_n;
  const dim3 grid(min(total, grid_req > 0 ? grid_req : ncu));
  auto* x = static_cast<const unsigned short*>(X);
  auto* w = static_cast<const unsigned short*>(Wp);
  auto* c = static_cast<unsigned short*>(C);
  auto* b = static_cast<const unsigned short*>(bias);
#define PW_LAUNCH1(WM_, E_, RW_)                                                                               \
  do {                                                                                                         \
    if (gather)                                                                                                \
      pgw_kernel<WM_, E_, true, 4, false, true><<<grid, PW_T, 0, s>>>(x, ldx, w, c, ldc, M, N, K, tiles_m, tiles_n, b, grp); \
    else if (grouped)                                                                                          \
      pgw_kernel<WM_, E_, true, RW_><<<grid, PW_T, 0, s>>>(x, ldx, w, c, ldc, M, N, K, tiles_m, tiles_n, b, grp);  \
    else                                                                                                       \
      pgw_kernel<WM_, E_, false, RW_><<<grid, PW_T, 0, s>>>(x, ldx, w, c, ldc, M, N, K, tiles_m, tiles_n, b, grp); \
  } while (0)
#define PW_LAUNCH(WM_, E_)                                                                                   \
  do {                                                                                                       \
    if (rw == 4)                                                                                             \
      PW_LAUNCH1(WM_, E_, 4);                                                                                \
    else if (rw == 2)                                                                                        \
      PW_LAUNCH1(WM_, E_, 2);                                                                                \
    else if (grouped)                                                                                        \
      pgw_kernel<WM_, E_, true, 4, true><<<grid, PW_T, 0, s>>>(x, ldx, w, c, ldc, M, N, K, tiles_m, tiles_n, b, grp);  \
    else                                                                                                     \
      pgw_kernel<WM_, E_, false, 4, true><<<grid, PW_T, 0, s>>>(x, ldx, w, c, ldc, M, N, K, tiles_m, tiles_n, b, grp); \
  } while (0)
#define PW_EPIS(WM_)                                          \
  switch (epi) {                                              \
    case PW_EPI_STORE: PW_LAUNCH(WM_, PW_EPI_STORE); return true; \
    case PW_EPI_ADD: PW_LAUNCH(WM_, PW_EPI_ADD); return true;     \
    case PW_EPI_GLU: PW_LAUNCH(WM_, PW_EPI_GLU); return true;     \
    case PW_EPI_GEGLU: PW_LAUNCH(WM_, PW_EPI_GEGLU); return true; \
    default: return false;                                    \
  }
  if (wm == 1) {
    PW_EPIS(1)
  }
  PW_EPIS(2)
#undef PW_EPIS
#undef PW_LAUNCH
#undef PW_LAUNCH1
}

}  // namespace hipserve
