// Prefill GEMM over the packed decode layout with BOTH operands staged by LDS-DMA
// (the global -> VGPR weight stream of prefill_gemm_packed.hip is what
// held it below hipBLASLt; with no weight loads that kernel reached 1.78 PFLOP/s):
//
//   C[M, N] = X[M, K] . W[N, K]^T      bf16 in, fp32 accumulate, epilogue fused
//
// W: pack_decode_weight's copy, [ceil(N/128)][K/256][8 rg][8 k-slot][64 lanes][8 bf16]:
// every (row group, 32-deep k-slot) piece is 1 KiB = the first operand of one
// v_mfma_f32_16x16x32_bf16 for a wave, lane-linear. An LDS-DMA wave instruction
// (buffer_load_dwordx4 ... lds, 16 B per lane, LDS address = base + 16 lane) copies a piece
// as is, and the wave's ds_read_b128 of it (lane l: bytes 16 l .. 16 l + 15) is
// conflict-free: no swizzle, no repack, ONE resident weight layout for decode and prefill.
//
// Workgroup: 512 threads = 8 waves (2 per SIMD), tile 256 (m) x 256 (n = two packed
// tiles). Wave w: X rows 128 (w >> 2) .. + 127 (8 m-tiles of 16), packed tile (w & 3) >> 1,
// row groups {2h, 2h + 1, 2h + 4, 2h + 5} (h = w & 1): 64 output columns, gate and up
// rows of a GLU-packed tile in the same lane. 32 accumulator tiles = 128 fp32 per lane.
//
// LDS: a ring of 4 slots of 32 KiB, one per 32-deep K step: [X 256 rows x 64 B][W 16
// pieces]. The X image is lane-linear too (16 rows x 64 B per DMA instruction); the
// per-lane SOURCE address carries the swizzle: 16-byte chunk c of row r sits at chunk
// c ^ sw(r), sw(r) = (-(r >> 2)) & 3, which puts the 16 lanes of every ds_read_b128 lane
// group of a B fragment (rows 16 t .. 16 t + 15, chunks (l >> 4)) on 16 distinct 16-byte
// bank slots.
//
// Pipeline, K step q (slot q & 3), two phases of 16 MFMAs per wave:
//   A: ds_read X(q) m-tiles 4-7            | MFMA W(q) x X(q) m-tiles 0-3
//   B: s_waitcnt vmcnt (own DMA of q + 1) -> s_barrier (every wave's DMA of q + 1 landed,
//      every read of slot q - 1 retired) -> DMA slot q + 3 into slot (q - 1)'s buffer ->
//      ds_read W(q + 1), X(q + 1) m-tiles 0-3 | MFMA W(q) x X(q) m-tiles 4-7
// One barrier per K step; a slot's DMA has two K steps (~2K MFMA cycles per SIMD) to land.
// The DMAs stay in flight across the barrier: raw s_barrier and counted vmcnt only (a
// __syncthreads() would drain them, cdna_hip_programming.md §5 "Pipelining across
// barriers"); all LDS is one __shared__ array.
//
// Epilogues (lane holds C[m][n .. n + 3], m = m0 + 128 (w >> 2) + 16 i + (l & 15),
// n = n0 + 128 u + 16 rg + 4 (l >> 4)): STORE (+ bias), ADD (C is the residual: C =
// bf16(bf16(acc) + C)), GLU / GEGLU (act[m, 64 t + 16 rg + 4 (l >> 4) + j] = act(gate) * up).
// Grouped (MoE experts): m-tile tm of X (expert-sorted slots, 256-row tiles) multiplies
// expert tile_expert[tm]'s packed weight; tiles past *num_tiles (device-side) exit at once.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

#include <cstdlib>

namespace hipserve {

namespace {

constexpr int PL_T = 512;
constexpr int PL_SLOT = 32768;  // bytes of one 32-deep K step: X 256 x 32 + W 256 x 32 bf16
constexpr int PL_WB = 16384;    // W pieces after the X image in a slot
constexpr int PL_GM = 8;        // m-tiles per tile group (L2 sharing of an XCD's workgroups)

typedef __attribute__((address_space(3))) void* lds_p;

template <int N>
HS_DEVICE void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct PlArgs {
  const unsigned short* X;
  long ldx;
  const unsigned short* Wp;
  unsigned short* C;
  long ldc;
  const unsigned short* bias;
  const int* tile_expert;
  const int* num_tiles;
  long estride;  // elements between experts' packed weights
  int M, N, K, tiles_m, tiles_n;
};

// NBUF: LDS ring slots (4: 128 KiB, DMA two K steps ahead; 5: all 160 KiB, three ahead);
// PRIO: s_setprio 1 around each MFMA cluster (cdna_hip_programming.md §5.5 T5)
template <int EPI, bool kGroup, int NBUF = 4, bool PRIO = false>
__global__ __launch_bounds__(PL_T) __attribute__((amdgpu_waves_per_eu(2, 2))) void pgl_kernel(PlArgs A) {
  constexpr int LEAD = NBUF - 1;  // K steps in flight ahead of the one being computed
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NBUF * PL_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  // tile: XCD-contiguous logical index, groups of PL_GM m-tiles walked n-major
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  {
    const int grp = L / (PL_GM * A.tiles_n), first = grp * PL_GM;
    const int gsz = min(PL_GM, A.tiles_m - first);
    const int r = L - first * A.tiles_n;
    tm = first + r % gsz;
    tn = r / gsz;
  }
  const unsigned short* Wp = A.Wp;
  if constexpr (kGroup) {
    if (tm >= __builtin_amdgcn_readfirstlane(*A.num_tiles)) return;
    Wp += (long)__builtin_amdgcn_readfirstlane(A.tile_expert[tm]) * A.estride;
  }
  const int K = A.K, M = A.M, N = A.N, nq = K >> 5, KS = K >> 8;
  const int ntiles = (N + 127) >> 7;
  const int m0 = tm * 256;

  // ---- DMA sources (per wave: X rows 32 w .. 32 w + 31, W pieces 2 w, 2 w + 1)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A.X + (long)m0 * A.ldx), 0, (int)((long)min(256, M - m0) * A.ldx * 2), 0x00020000);
  const int xrow = 32 * w + (lane >> 2);
  const int xch = ((lane & 3) ^ ((4 - ((lane >> 4) & 3)) & 3)) * 16;  // chunk c' holds c' ^ sw(row)
  const int xvo0 = xrow * (int)A.ldx * 2 + xch, xvo1 = xvo0 + 16 * (int)A.ldx * 2;
  const int wtile = min(2 * tn + (w >> 2), ntiles - 1);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Wp + (long)wtile * KS * 32768), 0, KS * 65536, 0x00020000);
  const int wvo0 = (2 * (w & 3)) * 8192 + 16 * lane, wvo1 = wvo0 + 8192;
  auto dma = [&](int q) {  // K step q (< nq) -> ring slot q % NBUF
    unsigned char* s = lds + (q % NBUF) * PL_SLOT + 2 * w * 1024;
    const int xk = q * 64, wk = (q >> 3) * 65536 + (q & 7) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_p)(s), 16, xvo0, xk, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_p)(s + 1024), 16, xvo1, xk, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(s + PL_WB), 16, wvo0, wk, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(s + PL_WB + 1024), 16, wvo1, wk, 0, 0);
  };

  // ---- fragment reads
  const int h = wn & 1, u = wn >> 1;
  const unsigned char* wrd = lds + PL_WB + (u * 8 + 2 * h) * 1024 + 16 * lane;  // + rg offset {0, 1, 4, 5} KiB
  const int xl = lane & 15;
  const unsigned char* xrd = lds + (128 * wm + xl) * 64 + 16 * ((lane >> 4) ^ ((4 - ((xl >> 2) & 3)) & 3));
  constexpr int RGO[4] = {0, 1, 4, 5};
  auto wfrag = [&](int q, int r) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(wrd + (q % NBUF) * PL_SLOT + RGO[r] * 1024);
  };
  auto xfrag = [&](int q, int i) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(xrd + (q % NBUF) * PL_SLOT + i * 1024);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[r][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K steps 0 .. LEAD - 1 in flight; wait for 0
#pragma unroll
  for (int q = 0; q < LEAD; ++q) dma(q);
  vm_wait<4 * (LEAD - 1)>();
  __builtin_amdgcn_s_barrier();
  bf16x8 wa[4], wb[4], xa[4], xb[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) wa[r] = wfrag(0, r);
#pragma unroll
  for (int i = 0; i < 4; ++i) xa[i] = xfrag(0, i);

  auto step = [&](int q, bf16x8(&wc)[4], bf16x8(&wnx)[4]) {
    // phase A
#pragma unroll
    for (int i = 0; i < 4; ++i) xb[i] = xfrag(q, 4 + i);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc[r], xa[i], acc[r][i], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    // phase B
    if (q + 1 < nq) {
      // own DMA of step q + 1 landed; the steps after it already issued (up to
      // q + LEAD - 1) stay in flight
      const int ahead = min(LEAD - 2, nq - 2 - q);
      if (ahead >= 2)
        vm_wait<8>();
      else if (ahead == 1)
        vm_wait<4>();
      else
        vm_wait<0>();
      // every LDS read this wave issued has returned before any wave may refill a slot
      // (hipcc may sink MFMAs, and with them their lgkmcnt waits, below the barrier)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (q + LEAD < nq) dma(q + LEAD);
    }
    // unconditional (after the last step: a stale, unused read): a branch around these
    // reads made hipcc's lgkmcnt waits for the phase-B fragments count only the short path
#pragma unroll
    for (int r = 0; r < 4; ++r) wnx[r] = wfrag(q + 1, r);
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = xfrag(q + 1, i);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[r][4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc[r], xb[i], acc[r][4 + i], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };
  for (int q = 0; q < nq; q += 2) {  // nq % 8 == 0
    step(q, wa, wb);
    step(q + 1, wb, wa);
  }

  // ---- epilogue
  const int t = 2 * tn + u;  // packed tile of this wave's columns
  if (t >= ntiles) return;
  const int mb = m0 + 128 * wm + xl, fq = lane >> 4;
  if constexpr (EPI == PW_EPI_GLU || EPI == PW_EPI_GEGLU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + 16 * i;
      if (m >= M) continue;
#pragma unroll
      for (int r = 0; r < 2; ++r) {  // gate rg 2h + r, up rg 2h + r + 4
        const int c = t * 64 + (2 * h + r) * 16 + 4 * fq;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned short g = f32_to_bf16(acc[r][i][j]), up = f32_to_bf16(acc[r + 2][i][j]);
          o[j] = EPI == PW_EPI_GEGLU ? gelu_mul1(g, up) : silu_mul1(g, up);
        }
        *reinterpret_cast<uint2*>(A.C + (long)m * A.ldc + c) =
            uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
      }
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = t * 128 + RGO[r] * 16 + 32 * h + 4 * fq;
      if (n >= N) continue;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (EPI == PW_EPI_STORE && A.bias != nullptr)
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = n + j < N ? bf16_to_f32(A.bias[n + j]) : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mb + 16 * i;
        if (m >= M) continue;
        uint2* dst = reinterpret_cast<uint2*>(A.C + (long)m * A.ldc + n);
        float o[4];
        if constexpr (EPI == PW_EPI_ADD) {
          const uint2 rv = *dst;
          const unsigned short rr[4] = {(unsigned short)(rv.x & 0xffff), (unsigned short)(rv.x >> 16),
                                        (unsigned short)(rv.y & 0xffff), (unsigned short)(rv.y >> 16)};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = bf16_to_f32(f32_to_bf16(acc[r][i][j])) + bf16_to_f32(rr[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = acc[r][i][j] + bv[j];
        }
        *dst = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      }
    }
  }
}


// ---------------------------------------------------------------- 4-wave form
// The same product at one wave per SIMD (256 threads), every wave a 128 (m) x 128 (n)
// block = one packed weight tile: 64 accumulator tiles (256 fp32) in AGPRs, MFMAs as
// inline asm on "+a" operands (the builtin made hipcc shuffle the accumulators between
// AGPRs and VGPRs, prefill_gemm_packed.hip). Per 32-deep K step a wave reads 8 W + 8 X
// fragments for 64 MFMAs (0.25 reads per MFMA; the 8-wave form: 0.375), and the step's
// other work is spread one item per MFMA group: after each row group's 8 MFMAs, one
// W and one X fragment of step q + 1 (ds_read_b128) and one of the wave's 8 DMA pieces
// of step q + 3 — the DMA issue cost overlaps the MFMAs instead of stalling the wave
// after the barrier.
HS_DEVICE void pl_mfma(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(x));
}

template <int EPI, bool kGroup>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void pgl4_kernel(PlArgs A) {
  constexpr int NBUF = 4;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NBUF * PL_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  {
    const int grp = L / (PL_GM * A.tiles_n), first = grp * PL_GM;
    const int gsz = min(PL_GM, A.tiles_m - first);
    const int r = L - first * A.tiles_n;
    tm = first + r % gsz;
    tn = r / gsz;
  }
  const unsigned short* Wp = A.Wp;
  if constexpr (kGroup) {
    if (tm >= __builtin_amdgcn_readfirstlane(*A.num_tiles)) return;
    Wp += (long)__builtin_amdgcn_readfirstlane(A.tile_expert[tm]) * A.estride;
  }
  const int K = A.K, M = A.M, N = A.N, nq = K >> 5, KS = K >> 8;
  const int ntiles = (N + 127) >> 7;
  const int m0 = tm * 256;

  // DMA: wave w copies X rows 64 w .. 64 w + 63 (4 pieces) and W pieces 4 w .. 4 w + 3
  // (packed tile 2 tn + (w >> 1), row groups 4 (w & 1) .. + 3) of every K step
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(A.X + (long)m0 * A.ldx), 0, (int)((long)min(256, M - m0) * A.ldx * 2), 0x00020000);
  const int xch = ((lane & 3) ^ ((4 - ((lane >> 4) & 3)) & 3)) * 16;
  const int xvo = (64 * w + (lane >> 2)) * (int)A.ldx * 2 + xch, xstep = 16 * (int)A.ldx * 2;
  const int wtile = min(2 * tn + (w >> 1), ntiles - 1);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(Wp + (long)wtile * KS * 32768), 0, KS * 65536, 0x00020000);
  const int wvo = (4 * (w & 1)) * 8192 + 16 * lane;
  auto dma1 = [&](int q, int j) {  // DMA piece j (0..7) of K step q: j < 4 X rows, else W
    unsigned char* s = lds + (q & 3) * PL_SLOT + 4 * w * 1024;
    if (j < 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_p)(s + j * 1024), 16, xvo + j * xstep, q * 64, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(s + PL_WB + (j - 4) * 1024), 16, wvo + (j - 4) * 8192,
                                               (q >> 3) * 65536 + (q & 7) * 1024, 0, 0);
  };

  // fragment reads: W piece (wn, rg) of the slot; X m-tile i of rows 128 wm ..
  const unsigned char* wrd = lds + PL_WB + wn * 8 * 1024 + 16 * lane;
  const int xl = lane & 15;
  const unsigned char* xrd = lds + (128 * wm + xl) * 64 + 16 * ((lane >> 4) ^ ((4 - ((xl >> 2) & 3)) & 3));

  f32x4 acc[8][8];
#pragma unroll
  for (int rg = 0; rg < 8; ++rg)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[rg][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K steps 0, 1, 2 in flight; wait for step 0
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) dma1(q, j);
  vm_wait<16>();
  __builtin_amdgcn_s_barrier();
  bf16x8 wa[8], xa[8], wb[8], xb[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    wa[r] = *reinterpret_cast<const bf16x8*>(wrd + r * 1024);
    xa[r] = *reinterpret_cast<const bf16x8*>(xrd + r * 1024);
  }

  // one K step; REFILL / VM (compile time): DMA step q + 3 (q + 3 < nq), and the vmcnt
  // that retires this wave's DMA of step q + 1 (8: step q + 2's pieces stay in flight; 0
  // near the end) — no per-DMA runtime branch in the MFMA stream
  auto step = [&](auto refill_c, auto vm_c, int q, bf16x8(&wc)[8], bf16x8(&xc)[8], bf16x8(&wnx)[8],
                  bf16x8(&xnx)[8]) {
    constexpr bool REFILL = decltype(refill_c)::value;
    constexpr int VM = decltype(vm_c)::value;
    // own DMA of step q + 1 landed; this wave's fragment reads of step q returned; then
    // every wave: step q + 1 visible, nobody reads step q - 1's slot any more (refilled
    // with step q + 3 below)
    vm_wait<VM>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int qn = q + 1 < nq ? q + 1 : q;  // the last step re-reads its own slot (unused)
    const unsigned char* wn_ = wrd + (qn & 3) * PL_SLOT;
    const unsigned char* xn_ = xrd + (qn & 3) * PL_SLOT;
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
#pragma unroll
      for (int i = 0; i < 8; ++i) pl_mfma(acc[rg][i], wc[rg], xc[i]);
      wnx[rg] = *reinterpret_cast<const bf16x8*>(wn_ + rg * 1024);
      xnx[rg] = *reinterpret_cast<const bf16x8*>(xn_ + rg * 1024);
      if constexpr (REFILL) dma1(q + 3, rg);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using V8 = std::integral_constant<int, 8>;
  using V0 = std::integral_constant<int, 0>;
  int q = 0;
  for (; q + 4 < nq; q += 2) {  // nq % 8 == 0: steps 0 .. nq - 5 refill and keep one step in flight
    step(T_{}, V8{}, q, wa, xa, wb, xb);
    step(T_{}, V8{}, q + 1, wb, xb, wa, xa);
  }
  step(T_{}, V8{}, q, wa, xa, wb, xb);      // nq - 4
  step(F_{}, V8{}, q + 1, wb, xb, wa, xa);  // nq - 3
  step(F_{}, V0{}, q + 2, wa, xa, wb, xb);  // nq - 2
  step(F_{}, V0{}, q + 3, wb, xb, wa, xa);  // nq - 1
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last asm MFMA -> VALU reads

  // ---- epilogue (lane: C[m][n .. n + 3], m = m0 + 128 wm + 16 i + (l & 15), n = 128 t + 16 rg + 4 (l >> 4))
  const int t = 2 * tn + wn;
  if (t >= ntiles) return;
  const int mb = m0 + 128 * wm + xl, fq = lane >> 4;
  if constexpr (EPI == PW_EPI_GLU || EPI == PW_EPI_GEGLU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + 16 * i;
      if (m >= M) continue;
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {  // gate rg, up rg + 4
        const int c = t * 64 + rg * 16 + 4 * fq;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned short g = f32_to_bf16(acc[rg][i][j]), up = f32_to_bf16(acc[rg + 4][i][j]);
          o[j] = EPI == PW_EPI_GEGLU ? gelu_mul1(g, up) : silu_mul1(g, up);
        }
        *reinterpret_cast<uint2*>(A.C + (long)m * A.ldc + c) =
            uint2{(unsigned)o[0] | ((unsigned)o[1] << 16), (unsigned)o[2] | ((unsigned)o[3] << 16)};
      }
    }
  } else {
#pragma unroll
    for (int rg = 0; rg < 8; ++rg) {
      const int n = t * 128 + rg * 16 + 4 * fq;
      if (n >= N) continue;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (EPI == PW_EPI_STORE && A.bias != nullptr)
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = n + j < N ? bf16_to_f32(A.bias[n + j]) : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mb + 16 * i;
        if (m >= M) continue;
        uint2* dst = reinterpret_cast<uint2*>(A.C + (long)m * A.ldc + n);
        float o[4];
        if constexpr (EPI == PW_EPI_ADD) {
          const uint2 rv = *dst;
          const unsigned short rr[4] = {(unsigned short)(rv.x & 0xffff), (unsigned short)(rv.x >> 16),
                                        (unsigned short)(rv.y & 0xffff), (unsigned short)(rv.y >> 16)};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = bf16_to_f32(f32_to_bf16(acc[rg][i][j])) + bf16_to_f32(rr[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = acc[rg][i][j] + bv[j];
        }
        *dst = uint2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      }
    }
  }
}

}  // namespace

// variant (A/B measurement; < 0: HIPSERVE_PGL_VAR, default 0): bit 0 = 5-slot ring, bit 1 = setprio
static int pgl_variant(int v) {
  if (v >= 0) return v;
  static const int e = [] {
    const char* s = getenv("HIPSERVE_PGL_VAR");
    return s ? atoi(s) : 0;
  }();
  return e;
}

bool launch_prefill_gemm_lds(int epi, void* C, long ldc, const void* X, long ldx, const void* Wp, int M, int N, int K,
                             const void* bias, hipStream_t s, const PwGroup* group, int variant) {
  variant = pgl_variant(variant) & 7;
  const bool grouped = group != nullptr;
  if (M < 1 || N < 1 || K < 256 || K % 256) return false;
  const bool glu = epi == PW_EPI_GLU || epi == PW_EPI_GEGLU;
  if (glu && (N % 128 || bias != nullptr)) return false;
  if (epi == PW_EPI_ADD && bias != nullptr) return false;
  if (grouped && (bias != nullptr || epi == PW_EPI_ADD)) return false;
  if (ldx % 8 || ldc % 4) return false;
  // 32-bit buffer offsets: one packed tile's weight stream, one workgroup's X rows
  if ((long)(K / 256) * 65536 >= (1L << 31) || (long)256 * ldx * 2 >= (1L << 31)) return false;
  PlArgs a;
  a.X = static_cast<const unsigned short*>(X);
  a.ldx = ldx;
  a.Wp = static_cast<const unsigned short*>(Wp);
  a.C = static_cast<unsigned short*>(C);
  a.ldc = ldc;
  a.bias = static_cast<const unsigned short*>(bias);
  a.tile_expert = grouped ? group->tile_expert : nullptr;
  a.num_tiles = grouped ? group->num_tiles : nullptr;
  a.estride = grouped ? group->estride : 0;
  a.M = M;
  a.N = N;
  a.K = K;
  a.tiles_m = (M + 255) / 256;
  a.tiles_n = ((N + 127) / 128 + 1) / 2;
  const dim3 grid(a.tiles_m * a.tiles_n), block(PL_T);
  if (variant >= 4) {  // the 4-wave form
#define PL4(E_)                                                          \
  do {                                                                   \
    if (grouped)                                                         \
      pgl4_kernel<E_, true><<<grid, 256, 0, s>>>(a);                     \
    else                                                                 \
      pgl4_kernel<E_, false><<<grid, 256, 0, s>>>(a);                    \
  } while (0)
    switch (epi) {
      case PW_EPI_STORE: PL4(PW_EPI_STORE); return true;
      case PW_EPI_ADD: PL4(PW_EPI_ADD); return true;
      case PW_EPI_GLU: PL4(PW_EPI_GLU); return true;
      case PW_EPI_GEGLU: PL4(PW_EPI_GEGLU); return true;
    }
#undef PL4
    return false;
  }
#define PL_LAUNCH2(E_, G_)                                                  \
  do {                                                                      \
    switch (variant) {                                                      \
      case 0: pgl_kernel<E_, G_, 4, false><<<grid, block, 0, s>>>(a); break; \
      case 1: pgl_kernel<E_, G_, 5, false><<<grid, block, 0, s>>>(a); break; \
      case 2: pgl_kernel<E_, G_, 4, true><<<grid, block, 0, s>>>(a); break;  \
      default: pgl_kernel<E_, G_, 5, true><<<grid, block, 0, s>>>(a); break; \
    }                                                                       \
  } while (0)
#define PL_LAUNCH(E_)          \
  do {                         \
    if (grouped)               \
      PL_LAUNCH2(E_, true);    \
    else                       \
      PL_LAUNCH2(E_, false);   \
  } while (0)
  switch (epi) {
    case PW_EPI_STORE: PL_LAUNCH(PW_EPI_STORE); return true;
    case PW_EPI_ADD: PL_LAUNCH(PW_EPI_ADD); return true;
    case PW_EPI_GLU: PL_LAUNCH(PW_EPI_GLU); return true;
    case PW_EPI_GEGLU: PL_LAUNCH(PW_EPI_GEGLU); return true;
  }
#undef PL_LAUNCH
#undef PL_LAUNCH2
  return false;
}

}  // namespace hipserve
