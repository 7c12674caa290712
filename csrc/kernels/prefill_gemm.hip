// Prefill GEMM for gfx950 (SURVEY K6-K9 at prefill sizes; VERDICT r2 next-round
// item 3): C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32 accumulate, with the
// layer's elementwise epilogue fused into the tile store.
//
// Tile 256 x 256 x 64, 512 threads = 8 waves as 2 (m) x 4 (n), each wave a 128 x 64
// output block on v_mfma_f32_16x16x32_bf16 (32 accumulators = 128 VGPRs). The
// weight fragment is the MFMA's FIRST operand, so a lane's 4 results are 4
// consecutive output columns of one row (8-byte stores, row-wise epilogues).
//
// Staging: global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave instruction, no VGPR
// round trip) into two 64 KiB stages (A 32 KiB + B 32 KiB each, 128 KiB, one
// workgroup per CU). The LDS image is lane-linear ([row][64 k] with 128-B rows);
// bank conflicts of the ds_read_b128 fragment reads are removed on the SOURCE side:
// 16-B chunk c of row r is stored at chunk c ^ ((r >> 1) & 7), which spreads every
// ds_read_b128 lane group (16 rows, two chunks) over all 16 slots of a bank row.
// The next K tile is issued into the other stage before the current tile's
// fragment reads, so its HBM/L2 latency hides under 64 MFMAs per wave.
//
// Blocks are remapped XCD-aware (xcd_remap): consecutive remapped blocks share a
// B (weight) column panel and run on one XCD, so the panel is served from that
// XCD's L2.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int PG_BM = 256, PG_BN = 256, PG_BK = 64, PG_T = 512;
constexpr int PG_TILE = PG_BM * PG_BK * 2;  // bytes of one operand tile per stage

// Global weight row of row r of the tile's B panel. GLU: the merged [gate; up] weight
// (2I rows) is read in its own layout, tile tn taking gate rows 128 tn .. + 127 then
// the matching up rows I + 128 tn .. + 127 — no repacked copy of the weight.
template <int EPI>
HS_DEVICE int pg_brow(int n0, int tn, int r, int N) {
  if constexpr (EPI == PG_EPI_GLU) return r < 128 ? tn * 128 + r : (N >> 1) + tn * 128 + (r - 128);
  return min(n0 + r, N - 1);
}

// Epilogue of a 256 x 256 tile: lane holds C[m][n .. n+3] for m = m0 + 128 wr + 16 i + fr,
// n = n0 + 64 wc + 16 j + 4 fq (acc[j][i]). Uses the whole LDS array (GLU exchange).
template <int EPI>
HS_DEVICE void pg_epilogue(f32x4 (&acc)[4][8], unsigned char* lds, unsigned short* __restrict__ C, long ldc, int M,
                           int m0, int n0, int tn, int wr, int wc, int fr, int fq, int lane) {
  if constexpr (EPI == PG_EPI_STORE || EPI == PG_EPI_ADD) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + fr;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + j * 16 + 4 * fq;
        uint2* dst = reinterpret_cast<uint2*>(C + (long)m * ldc + n);
        uint2 v;
        if constexpr (EPI == PG_EPI_ADD) {  // C is the residual: C = bf16(bf16(acc) + C)
          const uint2 r = *dst;
          const unsigned short rr[4] = {(unsigned short)(r.x & 0xffff), (unsigned short)(r.x >> 16),
                                        (unsigned short)(r.y & 0xffff), (unsigned short)(r.y >> 16)};
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = bf16_to_f32(f32_to_bf16(acc[j][i][e])) + bf16_to_f32(rr[e]);
          v.x = pack_bf16x2(o[0], o[1]);
          v.y = pack_bf16x2(o[2], o[3]);
        } else {
          v.x = pack_bf16x2(acc[j][i][0], acc[j][i][1]);
          v.y = pack_bf16x2(acc[j][i][2], acc[j][i][3]);
        }
        *dst = v;
      }
    }
  } else if constexpr (EPI == PG_EPI_GLU) {
    // tile columns 0..127 = gate rows, 128..255 = the matching up rows (pg_brow).
    // Waves wc = 2, 3 hand their bf16-rounded up values to the
    // gate waves wc = 0, 1 through LDS; act[m, 128 tn + c] = silu(gate) * up.
    float* ex = reinterpret_cast<float*>(lds);  // [2 wr][2 wc-1][8 i][4 j][64 lanes][4] fp32 = 128 KiB
    if (wc >= 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = bf16_to_f32(f32_to_bf16(acc[j][i][e]));
          *reinterpret_cast<f32x4*>(ex + ((((wr * 2 + (wc - 2)) * 8 + i) * 4 + j) * 64 + lane) * 4) = v;
        }
    }
    __syncthreads();
    if (wc < 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + wr * 128 + i * 16 + fr;
        if (m >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(ex + ((((wr * 2 + wc) * 8 + i) * 4 + j) * 64 + lane) * 4);
          unsigned short o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = silu_mul1(f32_to_bf16(acc[j][i][e]), f32_to_bf16(u[e]));
          uint2 v;
          v.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
          v.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
          const int c = tn * 128 + wc * 64 + j * 16 + 4 * fq;
          *reinterpret_cast<uint2*>(C + (long)m * ldc + c) = v;
        }
      }
    }
  }
}

template <int EPI>
__global__ __launch_bounds__(PG_T) void pgemm_kernel(const unsigned short* __restrict__ A, long lda,
                                                     const unsigned short* __restrict__ B, long ldb,
                                                     unsigned short* __restrict__ C, long ldc, int M, int N, int K,
                                                     int tiles_m, int tiles_n, PgEpi E) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * 2 * PG_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid / tiles_m, tm = bid - tn * tiles_m;
  const int m0 = tm * PG_BM, n0 = tn * PG_BN;
  const int nk = K / PG_BK;

  // staging sources: wave w fills rows [32w, 32w + 32) of both tiles, 8 rows per instruction
  const unsigned short* asrc[4];
  const unsigned short* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wave * 32 + i * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((r >> 1) & 7);  // logical chunk stored at physical chunk lane & 7
    asrc[i] = A + (long)min(m0 + r, M - 1) * lda + lc * 8;
    bsrc[i] = B + (long)pg_brow<EPI>(n0, tn, r, N) * ldb + lc * 8;
  }
  auto stage = [&](int buf, int kt) {
    unsigned char* base = lds + buf * 2 * PG_TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + kt * PG_BK),
                                       (lds_ptr_t)(base + (wave * 32 + i * 8) * 128), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + kt * PG_BK),
                                       (lds_ptr_t)(base + PG_TILE + (wave * 32 + i * 8) * 128), 16, 0, 0);
  };
  // fragment read offsets: rows (lane & 15) + 16 i, chunk 4 s + (lane >> 4), swizzled
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fr >> 1) & 7;
  const int a_off = (wr * 128 + fr) * 128, b_off = PG_TILE + (wc * 64 + fr) * 128;
  const int ch0 = ((0 + fq) ^ sw) * 16, ch1 = ((4 + fq) ^ sw) * 16;

  f32x4 acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(buf ^ 1, kt + 1);
    const unsigned char* sb = lds + buf * 2 * PG_TILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ch = s ? ch1 : ch0;
      u16x8 bf[4], af[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const u16x8*>(sb + b_off + j * 2048 + ch);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = *reinterpret_cast<const u16x8*>(sb + a_off + i * 2048 + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, bf[j]),
                                                              __builtin_bit_cast(bf16x8, af[i]), acc[j][i], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  pg_epilogue<EPI>(acc, lds, C, ldc, M, m0, n0, tn, wr, wc, fr, fq, lane);
}

// ---- v2: half-tile pipeline. Each K tile runs as 4 phases (one 64 x 32 output
// quadrant of the wave's 128 x 64 block per phase: 16 MFMAs) with raw s_barriers
// and counted vmcnt waits, so LDS-DMA traffic of the next two tiles stays in flight
// across every barrier (cdna_hip_programming.md §5 T3/T4) and no fragment read is
// waited on by the MFMAs that follow it (schedule in the loop below).
// kGroup (MoE prefill experts): A rows are expert-sorted and padded to 256-row tiles
// (moe_align with tile 256); tile_expert[tm] names the expert whose weight
// (B + e * b_estride) the m-tile multiplies, -1 = unused tile. Device-side offsets:
// no host round trip, graph-capturable.
template <int EPI, bool kGroup>
__global__ __launch_bounds__(PG_T) void pgemm2_kernel(const unsigned short* __restrict__ A, long lda,
                                                      const unsigned short* __restrict__ B, long ldb,
                                                      unsigned short* __restrict__ C, long ldc, int M, int N, int K,
                                                      int tiles_m, int tiles_n, PgEpi E) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * 2 * PG_TILE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = bid / tiles_m, tm = bid - tn * tiles_m;
  const int m0 = tm * PG_BM, n0 = tn * PG_BN;
  if constexpr (kGroup) {
    const int e = E.tile_expert[tm];
    if (e < 0) return;
    B += (long)e * E.b_estride;
  }
  const int nk = K / PG_BK;

  // half-tile staging: wave w moves half rows [16w, 16w + 16) in 2 instructions of 8
  // rows, as buffer_load ... lds with a per-lane 32-bit offset (8 VGPRs for all the
  // staging addresses; 64-bit pointers would push the loop past 256 VGPRs into
  // scratch, whose reload waits drain the LDS-DMA queue) and the K step in soffset
  unsigned int voff[2][2][2];  // [operand A/B][half][instr]
  int dst[2][2][2];            // LDS byte offset inside a stage (wave-uniform)
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j0 = wave * 16 + i * 8, j = j0 + (lane >> 3);
      const int ra0 = (j0 >> 6) * 128 + h * 64 + (j0 & 63), ra = (j >> 6) * 128 + h * 64 + (j & 63);
      const int rb0 = (j0 >> 5) * 64 + h * 32 + (j0 & 31), rb = (j >> 5) * 64 + h * 32 + (j & 31);
      voff[0][h][i] = (unsigned)((long)min(m0 + ra, M - 1) * lda * 2 + ((lane & 7) ^ ((ra >> 1) & 7)) * 16);
      voff[1][h][i] = (unsigned)((long)pg_brow<EPI>(n0, tn, rb, N) * ldb * 2 + ((lane & 7) ^ ((rb >> 1) & 7)) * 16);
      dst[0][h][i] = ra0 * 128;
      dst[1][h][i] = PG_TILE + rb0 * 128;
    }
  const __amdgpu_buffer_rsrc_t rsrc[2] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)min((long)M * lda * 2, 0x7fffffffL), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, (int)min((long)N * ldb * 2, 0x7fffffffL), 0x00020000)};
  auto stage_half = [&](int op, int h, int buf, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc[op], (lds_ptr_t)(lds + buf * 2 * PG_TILE + dst[op][h][i]), 16,
                                               voff[op][h][i], kt * PG_BK * 2, 0, 0);
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fr >> 1) & 7;
  const int a_off = (wr * 128 + fr) * 128, b_off = PG_TILE + (wc * 64 + fr) * 128;
  const int chs[2] = {((0 + fq) ^ sw) * 16, ((4 + fq) ^ sw) * 16};

  f32x4 acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments in registers: A rows of both quadrant rows, B columns of both quadrant
  // columns. Every read is issued one phase (or more) before its MFMAs:
  //   phase 0  MFMA (A0, B0)  | read B1 of this tile
  //   phase 1  MFMA (A0, B1)  | read A1 of this tile
  //   phase 2  MFMA (A1, B0)  |
  //   phase 3  MFMA (A1, B1)  | read A0, B0 of the NEXT tile (other stage)
  // LDS-DMA: tile kt+2's A0/B0 halves into this stage in phase 0 (this tile's A0/B0
  // were read during the previous tile's phase 3), its A1/B1 halves in phase 2 (read
  // in phases 0 / 1). Waits: end of phase 2 -> the next tile's A0/B0 landed (vmcnt 12),
  // end of phase 3 -> its A1/B1 landed (vmcnt 8). Barriers after phases 1, 2, 3.
  u16x8 bfr[4][2], afr[2][4][2];
  auto read_b = [&](const unsigned char* sb, int qn) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        bfr[2 * qn + jj][s2] = *reinterpret_cast<const u16x8*>(sb + b_off + (2 * qn + jj) * 2048 + chs[s2]);
  };
  auto read_a = [&](const unsigned char* sb, int qm) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        afr[qm][ii][s2] = *reinterpret_cast<const u16x8*>(sb + a_off + (4 * qm + ii) * 2048 + chs[s2]);
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // prologue: tiles 0 and 1 in flight; tile 0 and tile 1's A0/B0 landed; tile 0's A0/B0 read
  stage_half(0, 0, 0, 0);
  stage_half(1, 0, 0, 0);
  stage_half(0, 1, 0, 0);
  stage_half(1, 1, 0, 0);
  if (nk > 1) {
    stage_half(0, 0, 1, 1);
    stage_half(1, 0, 1, 1);
    stage_half(0, 1, 1, 1);
    stage_half(1, 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  barrier();
  read_a(lds, 0);
  read_b(lds, 0);

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const unsigned char* sb = lds + buf * 2 * PG_TILE;
    const bool more2 = kt + 2 < nk, more1 = kt + 1 < nk;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int qm = p >> 1, qn = p & 1;
      if (p == 0 && more2) {
        stage_half(0, 0, buf, kt + 2);
        stage_half(1, 0, buf, kt + 2);
      }
      if (p == 2 && more2) {
        stage_half(0, 1, buf, kt + 2);
        stage_half(1, 1, buf, kt + 2);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        if (s2 == 1) {  // the next phase's fragments, behind the first half of this phase's MFMAs
          __builtin_amdgcn_sched_barrier(0);
          if (p == 0) read_b(sb, 1);
          if (p == 1) read_a(sb, 1);
          if (p == 3 && more1) {
            read_a(lds + (buf ^ 1) * 2 * PG_TILE, 0);
            read_b(lds + (buf ^ 1) * 2 * PG_TILE, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int ii = 0; ii < 4; ++ii)
            acc[2 * qn + jj][4 * qm + ii] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, bfr[2 * qn + jj][s2]), __builtin_bit_cast(bf16x8, afr[qm][ii][s2]),
                acc[2 * qn + jj][4 * qm + ii], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
      if (p == 2) {  // the next tile's A0 / B0 halves landed (read in phase 3)
        if (more2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if (more1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (p == 3) {  // the next tile's A1 / B1 halves landed (read in its phases 0 / 1)
        if (more2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (p != 0) barrier();
    }
  }
  pg_epilogue<EPI>(acc, lds, C, ldc, M, m0, n0, tn, wr, wc, fr, fq, lane);
}

static bool pg_shape_ok(int M, int N, int K) { return M >= 1 && N % PG_BN == 0 && K % PG_BK == 0 && K >= PG_BK; }

bool launch_prefill_gemm(int epi, void* C, long ldc, const void* A, long lda, const void* B, long ldb, int M, int N,
                         int K, const PgEpi& E, hipStream_t s) {
  if (!pg_shape_ok(M, N, K)) return false;
  const int tiles_m = (M + PG_BM - 1) / PG_BM, tiles_n = N / PG_BN;
  const dim3 grid(tiles_m * tiles_n);
  auto* a = static_cast<const unsigned short*>(A);
  auto* b = static_cast<const unsigned short*>(B);
  auto* c = static_cast<unsigned short*>(C);
  if (E.tile_expert != nullptr) {  // grouped (MoE experts): M = tiles_cap * 256 slot rows
    switch (epi) {
      case PG_EPI_STORE: pgemm2_kernel<PG_EPI_STORE, true><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
      case PG_EPI_GLU: pgemm2_kernel<PG_EPI_GLU, true><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
      default: return false;
    }
  }
  if (E.variant == 2) {
    switch (epi) {
      case PG_EPI_STORE: pgemm2_kernel<PG_EPI_STORE, false><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
      case PG_EPI_ADD: pgemm2_kernel<PG_EPI_ADD, false><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
      case PG_EPI_GLU: pgemm2_kernel<PG_EPI_GLU, false><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
      default: return false;
    }
  }
  switch (epi) {
    case PG_EPI_STORE: pgemm_kernel<PG_EPI_STORE><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
    case PG_EPI_ADD: pgemm_kernel<PG_EPI_ADD><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
    case PG_EPI_GLU: pgemm_kernel<PG_EPI_GLU><<<grid, PG_T, 0, s>>>(a, lda, b, ldb, c, ldc, M, N, K, tiles_m, tiles_n, E); return true;
    default: return false;
  }
}

// [gate; up] rows (2I x K) -> per 256-row tile t: gate rows [128t, 128t + 128) then
// up rows I + [128t, 128t + 128). One thread per 16-byte piece.
__global__ __launch_bounds__(256) void pack_glu_rows_kernel(unsigned short* __restrict__ out,
                                                            const unsigned short* __restrict__ w, int I, int K) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int kv = K / 8;
  if (i >= 2L * I * kv) return;
  const long row = i / kv;
  const int c = (int)(i - row * kv);
  const long t = row / 256, q = row % 256;
  const long src = q < 128 ? t * 128 + q : I + t * 128 + (q - 128);
  reinterpret_cast<u16x8*>(out)[i] = reinterpret_cast<const u16x8*>(w + src * K)[c];
}

void launch_pack_glu_rows(void* out, const void* w, int I, int K, hipStream_t s) {
  const long n = 2L * I * (K / 8);
  pack_glu_rows_kernel<<<(n + 255) / 256, 256, 0, s>>>(static_cast<unsigned short*>(out),
                                                        static_cast<const unsigned short*>(w), I, K);
}

}  // namespace hipserve
