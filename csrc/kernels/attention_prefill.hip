// Varlen causal prefill attention over the paged KV cache.
//
// Handles plain prefill, chunked prefill and prefix-cached prompts uniformly:
// K/V for every key (old context + the new chunk) are read from the paged cache,
// which rope_cache.hip has already filled for the new tokens.
//
// Structure (gfx950):
//  * workgroup = 128 query rows of one sequence x one query head; 4 waves x 32
//    rows; waves are independent (no LDS, no barriers), each stops at its own
//    causal limit.
//  * S^T = K . Q^T on v_mfma_f32_32x32x16_bf16: the query row sits on the MFMA
//    column = the lane, so every lane owns 16 scores of ONE query row and the
//    row max/sum need one cross-lane op (lane ^ 32).
//  * O^T = V^T . P^T: the S^T accumulator is reused as the B operand without any
//    lane movement (accumulator-as-operand, guide §3); the matching A operand is
//    V^T, which the transposed-per-block V cache serves as two 8-byte loads.
//  * online softmax in the log2 domain.
#include <cstdlib>

#include <type_traits>

#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

// max / sum of v over lanes l and l ^ 32 with one v_permlane32_swap (gfx950: the two
// results hold, per lane, v of lane l and of lane l ^ 32 in some order) instead of an
// LDS round trip (ds_bpermute) that the next instruction waits on
HS_DEVICE float xor32_max(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
HS_DEVICE float xor32_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

typedef unsigned short u16x4v __attribute__((ext_vector_type(4)));

template <int D, typename KV>
__global__ __launch_bounds__(256) void prefill_attn_kernel(
    unsigned short* __restrict__ out, long out_stride,
    const unsigned short* __restrict__ q, long q_stride,
    const KV* __restrict__ k_cache,
    const KV* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ tiles, int nq, int nkv, int block_size,
    float scale, int window) {
  constexpr int KS = D / 16;   // k-steps of QK (K = 16 per MFMA)
  constexpr int NB = D / 32;   // 32-row d blocks of O^T
  const int seq = tiles[2 * blockIdx.x], r0 = tiles[2 * blockIdx.x + 1];
  const int h = blockIdx.y;
  const int kh = h / (nq / nkv);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = lane & 31, half = lane >> 5;
  const int q0 = cu_q[seq];
  const int qlen = cu_q[seq + 1] - q0;
  const int ctx = ctx_lens[seq];
  const int wrow0 = r0 + wave * 32;
  if (wrow0 >= qlen) return;
  const int row = min(wrow0 + qi, qlen - 1);
  const int pos = ctx - qlen + row;        // absolute position of this query row
  const int max_key = ctx - qlen + min(wrow0 + 31, qlen - 1);
  const int* btab = block_tables + (long)seq * bt_stride;
  const long head_stride = (long)block_size * D;

  bf16x8 qf[KS];
  {
    const unsigned short* qp = q + (long)(q0 + row) * q_stride + (long)h * D + 8 * half;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks));
  }
  const float sl2 = scale * 1.4426950408889634f;
  f32x16 o[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[nb][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  const int nkt = max_key / 32 + 1;
  // sliding window: the wave's first row sees keys >= its pos - window + 1
  const int kt0 = window > 0 ? max(0, ctx - qlen + wrow0 - window + 1) / 32 : 0;
  for (int kt = kt0; kt < nkt; ++kt) {
    const int kbase = kt * 32;
    // K fragment rows: key kbase + qi (clamped into the valid context)
    const int key = min(kbase + qi, ctx - 1);
    const KV* kp = k_cache +
        ((long)btab[key / block_size] * nkv + kh) * head_stride +
        (long)(key % block_size) * D + 8 * half;
    u16x8 kf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = kv_widen8(kv_load8(kp + 16 * ks));
    // V^T fragments: row d = 32*nb + qi; k-slot j of half h, step s ->
    // key kbase + 16s + 8(j>>2) + 4h + (j&3): two runs of 4 contiguous tokens.
    u16x4v vf[NB][2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int run = 0; run < 2; ++run) {
        int k4 = kbase + 16 * s + 8 * run + 4 * half;
        if (k4 > ctx - 1) k4 = (ctx - 1) & ~3;
        const KV* vp = v_cache +
            ((long)btab[k4 / block_size] * nkv + kh) * head_stride + (k4 % block_size) +
            (long)qi * block_size;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          vf[nb][s][run] = kv_widen4(*reinterpret_cast<const std::conditional_t<sizeof(KV) == 2, u16x4v, unsigned>*>(
              vp + (long)32 * nb * block_size));
      }

    f32x16 st;
#pragma unroll
    for (int r = 0; r < 16; ++r) st[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      st = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks]), qf[ks], st, 0, 0, 0);

    float mx = -1e30f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kk = kbase + (r & 3) + 8 * (r >> 2) + 4 * half;
      const float v = (kk <= pos && (window <= 0 || kk > pos - window)) ? st[r] * sl2 : -INFINITY;
      st[r] = v;
      mx = fmaxf(mx, v);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float psum = 0.f;
    bf16x8 pb[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = exp2f(st[r] - m_new);
      psum += p;
      pb[r >> 3][r & 7] = static_cast<__bf16>(p);
    }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[nb][r] *= alpha;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = vf[nb][s][0][j]; a[j + 4] = vf[nb][s][1][j]; }
        o[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), pb[s], o[nb], 0, 0, 0);
      }
  }
  l_run = xor32_sum(l_run);
  const float inv = 1.f / l_run;
  if (wrow0 + qi < qlen) {
    unsigned short* op = out + (long)(q0 + wrow0 + qi) * out_stride + (long)h * D;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4v w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f32_to_bf16(o[nb][4 * g + j] * inv);
        *reinterpret_cast<u16x4v*>(op + 32 * nb + 8 * g + 4 * half) = w;
      }
  }
}

// ---- v2: LDS-shared K/V tiles, GQA heads per workgroup (D = 128, G = nq/nkv >= 2) ----
//
//  * workgroup = NWV (4 or 8) waves = HG query heads of ONE kv head x NWV/HG blocks
//    of 32 query rows (G = 4, NWV = 4: 4 heads x 32 rows); every K/V tile is loaded
//    once into LDS and read by all waves (v1: every wave re-read it from L2 per
//    query head). 8 waves (default); 4 (HIPSERVE_PREFILL_ATTN_WAVES=4) measured
//    2.5-2.8x slower (one 4-wave workgroup per CU resident).
//  * 64-key tiles, double-buffered in LDS; global loads run two tiles ahead in two
//    register sets (tile t+2 is issued before tile t's MFMAs, tile t+1 is written
//    to LDS after them: issue-early / write-late), one barrier per tile.
//  * S^T = K . Q^T (swapped, so a lane owns 16 keys of one query row) with the K
//    rows of each 16-key group stored in LDS with key bits 2 and 3 swapped: the S^T
//    accumulator of a lane then holds 8 CONTIGUOUS keys per MFMA k-slot, so it is
//    the P^T B operand of O^T = V^T . P^T as is, and the matching V^T A operand is a
//    single ds_read_b128 from the transposed V tile.
//  * one online-softmax update per 64 keys; O is rescaled only when some row's
//    max moved (exact: alpha == 1 otherwise); masks only on diagonal tiles.
//  * LDS rows padded (K 272 B, V^T 144 B): the 16 lanes of each b128 read phase
//    hit 16 distinct 16-byte bank groups.
//  * heaviest query tiles are dispatched first against the causal tail.
static bool getenv_flag(const char* name) {
  const char* e = getenv(name);
  return e != nullptr && *e != 0 && *e != '0';
}

constexpr int PA2_KT = 64, PA2_KLD = 128 + 8, PA2_VLD = 64 + 8;

// (A stagger — waves 4-7 issuing each tile's P.V one tile late, a third LDS buffer holding
// its V^T, MI355X_MICROARCH.md "Two waves per SIMD" item 9 — needed 16 more VGPRs than the
// 256 of two waves per SIMD and spilled: 1.4-1.5x slower, profiles/r5_prefill_attn_bench.log.)
// KV: cache element, bf16 or e4m3; e4m3 pieces (8 bytes) are widened to bf16 on their way
// into the LDS ring, so the MFMA / softmax body is the same for both
template <int HG, int NWV, typename KV>
__global__ __launch_bounds__(64 * NWV) void prefill_attn_v2_kernel(
    unsigned short* __restrict__ out, long out_stride, const unsigned short* __restrict__ q, long q_stride,
    const KV* __restrict__ k_cache, const KV* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ cu_q,
    const int* __restrict__ ctx_lens, const int* __restrict__ tiles, int nq, int nkv, int block_size,
    float scale, int window, int prio) {
  constexpr int D = 128, KS = 8, NB = 4;
  constexpr int RB = NWV / HG, QR = 32 * RB, SUB = 128 / QR;
  constexpr int NT = 64 * NWV, NP = 1024 / NT;  // threads; K (and V^T) 16-byte pieces per thread
  constexpr int NBUF = 2;
  __shared__ __attribute__((aligned(16))) unsigned short kl[NBUF][PA2_KT * PA2_KLD];
  __shared__ __attribute__((aligned(16))) unsigned short vl[NBUF][D * PA2_VLD];

  // dispatch order (x fastest) -> (kv-head group fastest, host tile, heavier sub-tile first):
  // with the host tiles sorted by descending causal work (model_runner) the largest
  // workgroups go out first (longest-processing-time order against the causal tail)
  const int L = blockIdx.x + gridDim.x * blockIdx.y, gy = gridDim.y;
  const int gyi = L % gy, rest = L / gy;
  const int t = rest / SUB, sub = SUB - 1 - (rest - t * SUB);
  const int seq = tiles[2 * t], r0 = tiles[2 * t + 1] + sub * QR;
  const int q0 = cu_q[seq], qlen = cu_q[seq + 1] - q0;
  if (r0 >= qlen) return;  // whole workgroup: before any barrier
  const int ctx = ctx_lens[seq];
  const int G = nq / nkv;
  const int kh = gyi / (G / HG);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hs = wave % HG, rb = wave / HG;
  const int h = gyi * HG + hs;
  const int qi = lane & 31, half = lane >> 5;
  const int wrow0 = r0 + rb * 32;
  const bool wactive = wrow0 < qlen;
  const int row = min(wrow0 + qi, qlen - 1);
  const int pos = ctx - qlen + row;
  const int wmax_key = ctx - qlen + min(wrow0 + 31, qlen - 1);
  const int wmin_pos = ctx - qlen + wrow0;
  const int nkt = (ctx - qlen + min(r0 + QR - 1, qlen - 1)) / PA2_KT + 1;
  // sliding window: rows see keys [pos - window + 1, pos]; the workgroup starts at
  // the tile holding its first row's lowest key
  const int kt0 = window > 0 ? max(0, ctx - qlen + r0 - window + 1) / PA2_KT : 0;
  const int* btab = block_tables + (long)seq * bt_stride;
  const long hstride = (long)block_size * D;
  // block sizes are powers of two (launcher check): shifts, not integer divisions,
  // in the per-tile paging math (the divisions were ~1/3 of the tile's VALU)
  const int bsh = __builtin_ctz(block_size), bmask = block_size - 1;
  // the block ids of this workgroup's key range, staged in LDS once: a per-piece global
  // load of the id right before each K / V load made hipcc wait vmcnt(0) four times per
  // tile, draining the two tiles of K / V loads kept in flight ahead of the MFMAs
  extern __shared__ int bts[];
  const int blk_lo = (kt0 * PA2_KT) >> bsh, blk_hi = (min(nkt * PA2_KT, ctx) - 1) >> bsh;
  for (int i = threadIdx.x; i <= blk_hi - blk_lo; i += 64 * NWV) bts[i] = btab[blk_lo + i];
  __syncthreads();

  // staging: NP K pieces + NP V^T pieces of 16 B per thread per tile
  // two register sets: tile kt+2 loads while tile kt+1's registers wait for their LDS write
  using KV8 = typename KvVec<KV>::T;
  KV8 ska[NP], sva[NP], skb[NP], svb[NP];
  // staging addresses: block id x the elements of one block of all kv heads (< 2^32: one
  // 32 x 32 -> 64-bit multiply-add per piece) + a 32-bit in-block offset; the kv head's
  // base is folded into the workgroup's K / V pointers
  const unsigned blk_elems = (unsigned)(nkv * hstride);
  const KV* kc_h = k_cache + (long)kh * hstride;
  const KV* vc_h = v_cache + (long)kh * hstride;
  auto stage_load = [&](KV8(&sk)[NP], KV8(&sv)[NP], int kt) {
    const int kbase = kt * PA2_KT;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int p = tid + NT * i;
      const int key = min(kbase + (p >> 4), ctx - 1);
      const unsigned kid = (unsigned)bts[(key >> bsh) - blk_lo];
      sk[i] = kv_load8(kc_h + ((unsigned long)kid * blk_elems + (unsigned)((key & bmask) * D + (p & 15) * 8)));
      // V^T: 16-key group sc, row d, 8-key half: one block's [D][16] chunk per 256 threads
      const int sc = p >> 8, d = (p >> 1) & 127, k8 = p & 1;
      int vkey = kbase + 16 * sc + 8 * k8;
      if (vkey > ctx - 1) vkey = (ctx - 1) & ~7;
      const unsigned vid = (unsigned)bts[(vkey >> bsh) - blk_lo];
      sv[i] = kv_load8(vc_h + ((unsigned long)vid * blk_elems + (unsigned)(d * block_size + (vkey & bmask))));
    }
  };
  auto stage_store = [&](const KV8(&sk)[NP], const KV8(&sv)[NP], int buf) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int p = tid + NT * i;
      const int kk = p >> 4;
      const int krow = (kk & ~12) | ((kk & 4) << 1) | ((kk & 8) >> 1);  // swap key bits 2 and 3
      *reinterpret_cast<u16x8*>(&kl[buf][krow * PA2_KLD + (p & 15) * 8]) = kv_widen8(sk[i]);
      const int sc = p >> 8, d = (p >> 1) & 127, k8 = p & 1;
      *reinterpret_cast<u16x8*>(&vl[buf][d * PA2_VLD + 16 * sc + 8 * k8]) = kv_widen8(sv[i]);
    }
  };

  bf16x8 qf[KS];
  {
    const unsigned short* qp = q + (long)(q0 + row) * q_stride + (long)h * D + 8 * half;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks));
  }
  const float sl2 = scale * 1.4426950408889634f;
  f32x16 o[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[nb][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  auto compute = [&](int kt, int buf) __attribute__((always_inline)) {
    const int kbase = kt * PA2_KT;
    if (wactive && kbase <= wmax_key && (window <= 0 || kbase + PA2_KT - 1 > wmin_pos - window)) {
      const unsigned short* kb = &kl[buf][qi * PA2_KLD + 8 * half];
      f32x16 st[2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
        for (int r = 0; r < 16; ++r) st[h2][r] = 0.f;
      if (prio) __builtin_amdgcn_s_setprio(1);  // MFMA cluster: the partner wave's softmax VALU waits
      // K fragments read one k-step ahead of their MFMAs (two register sets): hipcc left to
      // itself waited out each fragment's LDS latency right before its MFMA
      u16x8 kf[2][2];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) kf[0][h2] = *reinterpret_cast<const u16x8*>(kb + (32 * h2) * PA2_KLD);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
            kf[(ks + 1) & 1][h2] = *reinterpret_cast<const u16x8*>(kb + (32 * h2) * PA2_KLD + 16 * (ks + 1));
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the reads of k-step ks + 1 ahead of k-step ks's MFMAs
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)  // two independent accumulation chains interleaved
          st[h2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, kf[ks & 1][h2]), qf[ks], st[h2],
                                                           0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (prio) __builtin_amdgcn_s_setprio(0);
      // diagonal tile (causal mask) or a tile crossing some row's window start
      // (key offsets inside the tile are compile-time per accumulator slot: one compare +
      // select per score against the lane's limit, the window test only when one is set)
      if (kbase + PA2_KT - 1 > wmin_pos || (window > 0 && kbase <= wmax_key - window)) {
        const int lim = pos - kbase - 8 * half;  // slot offset > lim: a future key
        if (window <= 0) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (32 * h2 + 16 * (r >> 3) + 4 * ((r >> 2) & 1) + (r & 3) > lim) st[h2][r] = -INFINITY;
        } else {
          const int wlo = lim - window;  // slot offset <= wlo: before the window
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int off = 32 * h2 + 16 * (r >> 3) + 4 * ((r >> 2) & 1) + (r & 3);
              if (off > lim || off <= wlo) st[h2][r] = -INFINITY;
            }
        }
      }
      float mx = -1e30f;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[h2][r]);
      mx = xor32_max(mx);
      const float m_new = fmaxf(m_run, mx * sl2);
      // deferred rescale: the running max is kept while no row's max grew by more than
      // 8 (log2 units), so P = exp2(s - m_run) stays <= 256 (exact enough in bf16 / fp32;
      // O and l always share m_run) and the 64-accumulator rescale runs on few tiles
      if (!__all(m_new - m_run <= 8.f)) {
        const float alpha = exp2f(m_run - m_new);
        l_run *= alpha;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[nb][r] *= alpha;
        m_run = m_new;
      }
      float ps[4] = {0.f, 0.f, 0.f, 0.f};  // four independent chains, not one 32-add dependency chain
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        bf16x8 pb[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[h2][r], sl2, -m_run));
          ps[r & 3] += p;
          pb[r >> 3][r & 7] = static_cast<__bf16>(p);
        }
        if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const unsigned short* vb = &vl[buf][qi * PA2_VLD + 32 * h2 + 16 * s2 + 8 * half];
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            const u16x8 a = *reinterpret_cast<const u16x8*>(vb + 32 * nb * PA2_VLD);
            o[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), pb[s2], o[nb], 0, 0, 0);
          }
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
      }
      l_run += (ps[0] + ps[1]) + (ps[2] + ps[3]);
    }
  };

  auto run = [&](int kt, int buf) __attribute__((always_inline)) { compute(kt, buf); };
  auto nxt = [](int b) __attribute__((always_inline)) { return b + 1 == NBUF ? 0 : b + 1; };

  stage_load(ska, sva, kt0);
  if (kt0 + 1 < nkt) stage_load(skb, svb, kt0 + 1);
  stage_store(ska, sva, 0);
  __syncthreads();
  int bc = 0;  // LDS buffer of tile kt
  for (int kt = kt0; kt < nkt; kt += 2) {
    const int b1 = nxt(bc), b2 = nxt(b1);
    // tile kt in buffer bc; set b holds tile kt+1
    if (kt + 2 < nkt) stage_load(ska, sva, kt + 2);
    run(kt, bc);
    if (kt + 1 < nkt) stage_store(skb, svb, b1);
    __syncthreads();
    if (kt + 1 >= nkt) break;
    // tile kt+1 in buffer b1; set a holds tile kt+2
    if (kt + 3 < nkt) stage_load(skb, svb, kt + 3);
    run(kt + 1, b1);
    if (kt + 2 < nkt) stage_store(ska, sva, b2);
    __syncthreads();
    bc = b2;
  }
  if (!wactive) return;
  l_run = xor32_sum(l_run);
  const float inv = 1.f / l_run;
  if (wrow0 + qi < qlen) {
    unsigned short* op = out + (long)(q0 + wrow0 + qi) * out_stride + (long)h * D;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4v w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f32_to_bf16(o[nb][4 * g + j] * inv);
        *reinterpret_cast<u16x4v*>(op + 32 * nb + 8 * g + 4 * half) = w;
      }
  }
}

void launch_prefill_attention(void* out, long out_stride, const void* q,
                              long q_stride, const void* k_cache,
                              const void* v_cache, const int* block_tables,
                              int bt_stride, const int* cu_q, const int* ctx_lens,
                              const int* tiles, int ntiles, int nq, int nkv, int D,
                              int block_size, float scale, int window, hipStream_t s, bool kv_f8) {
  if (ntiles <= 0) return;
  const int G = nq / nkv;
  // v2 keeps the sequence's block ids in LDS next to its 70 KiB K / V ring (160 KiB per CU)
  if (D == 128 && block_size % 16 == 0 && (block_size & (block_size - 1)) == 0 && G >= 2 && (G & (G - 1)) == 0 &&
      (size_t)bt_stride * sizeof(int) <= 64 * 1024 &&
      !getenv_flag("HIPSERVE_PREFILL_ATTN_V1")) {
    const char* ew = getenv("HIPSERVE_PREFILL_ATTN_WAVES");  // 8 (default) or 4 waves per workgroup
    const int nwv = (ew != nullptr && atoi(ew) == 4) ? 4 : 8;
    const int HG = G >= nwv ? nwv : G;
    // s_setprio 1 around each MFMA cluster (the partner wave's softmax VALU yields to it):
    // 3 % faster at 1K-32K tokens (profiles/r4_prefill_attn_setprio.log; a static
    // priority for the younger wave of each SIMD gained 1 %); HIPSERVE_PREFILL_ATTN_PRIO=0
    // turns it off
    const char* ep = getenv("HIPSERVE_PREFILL_ATTN_PRIO");
    const int prio = ep != nullptr && atoi(ep) == 0 ? 0 : 1;
    const int sub = 128 / (32 * (nwv / HG));
    dim3 g2(ntiles * sub, nkv * (G / HG));
    auto* o2 = static_cast<unsigned short*>(out);
    auto* q2 = static_cast<const unsigned short*>(q);
    auto* k2 = static_cast<const unsigned short*>(k_cache);
    auto* v2 = static_cast<const unsigned short*>(v_cache);
    auto* k28 = static_cast<const unsigned char*>(k_cache);
    auto* v28 = static_cast<const unsigned char*>(v_cache);
    // block ids of one sequence (the per-workgroup key range is at most this) in dynamic LDS
    const size_t bt_lds = (size_t)bt_stride * sizeof(int);
#define PA2_LAUNCH_KV(hg, nw, KVT, KP, VP)                                                                   \
  do {                                                                                                      \
    static bool attr = [] { /* static 70 KiB + the block ids: above the 64 KiB default (160 KiB per CU) */ \
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&prefill_attn_v2_kernel<hg, nw, KVT>),       \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess;      \
    }();                                                                                                    \
    (void)attr;                                                                                             \
    prefill_attn_v2_kernel<hg, nw, KVT><<<g2, 64 * nw, bt_lds, s>>>(o2, out_stride, q2, q_stride, KP, VP,    \
                                                                    block_tables, bt_stride, cu_q, ctx_lens, \
                                                                    tiles, nq, nkv, block_size, scale, window, \
                                                                    prio);                                  \
  } while (0)
#define PA2_LAUNCH(hg, nw)                                                                                  \
  do {                                                                                                      \
    if (kv_f8) PA2_LAUNCH_KV(hg, nw, unsigned char, k28, v28);                                             \
    else PA2_LAUNCH_KV(hg, nw, unsigned short, k2, v2);                                                     \
  } while (0)
    if (nwv == 8) {
      if (HG == 8) PA2_LAUNCH(8, 8);
      else if (HG == 4) PA2_LAUNCH(4, 8);
      else PA2_LAUNCH(2, 8);
    } else {
      if (HG == 4) PA2_LAUNCH(4, 4);
      else PA2_LAUNCH(2, 4);
    }
#undef PA2_LAUNCH
#undef PA2_LAUNCH_KV
    return;
  }
  dim3 grid(ntiles, nq), block(256);
  auto* o = static_cast<unsigned short*>(out);
  auto* qq = static_cast<const unsigned short*>(q);
  auto* kc = static_cast<const unsigned short*>(k_cache);
  auto* vc = static_cast<const unsigned short*>(v_cache);
#define PA1_LAUNCH(dd)                                                                                          \
  do {                                                                                                          \
    if (kv_f8)                                                                                                  \
      prefill_attn_kernel<dd, unsigned char><<<grid, block, 0, s>>>(                                            \
          o, out_stride, qq, q_stride, static_cast<const unsigned char*>(k_cache),                              \
          static_cast<const unsigned char*>(v_cache), block_tables, bt_stride, cu_q, ctx_lens, tiles, nq, nkv,  \
          block_size, scale, window);                                                                           \
    else                                                                                                        \
      prefill_attn_kernel<dd, unsigned short><<<grid, block, 0, s>>>(o, out_stride, qq, q_stride, kc, vc,        \
                                                                     block_tables, bt_stride, cu_q, ctx_lens,   \
                                                                     tiles, nq, nkv, block_size, scale, window); \
  } while (0)
  if (D == 128) PA1_LAUNCH(128);
  else if (D == 96) PA1_LAUNCH(96);
  else PA1_LAUNCH(64);
#undef PA1_LAUNCH
}

}  // namespace hipserve
