// Paged decode attention for gfx950: one query token per sequence,
// GQA-packed, split over the context ("partitions") with a separate reduce.
//
// Design (MI355X-first, not a CUDA warp-tiling port):
//  * workgroup = (partition of PS tokens, kv head, sequence); 4 waves; each wave
//    streams 32-token chunks (chunk c = wave, wave+4, ...) of its partition.
//  * QK^T runs on MFMA v_mfma_f32_16x16x32_bf16 in the *swapped* form
//    S^T = K . Q^T: A = 16 K rows (tokens), B = Q^T with the G query heads of the
//    kv group on the 16 MFMA columns (G <= 16; padding columns are zero).
//    The 16 A rows of the two 16-row tiles of a chunk are chosen so that lane
//    group g (= lane>>4) ends up holding tokens 8g..8g+7 of the chunk — exactly
//    the k-slots the PV MFMA wants in its A operand: P needs no lane movement.
//  * PV runs on the same MFMA with A = P (rows = heads), B = V. The V cache is
//    stored transposed per block ([D][block_size]) so each B fragment (8
//    consecutive tokens of one d column) is ONE 16-byte global load to VGPRs:
//    no LDS round trip on the memory-bound path (guide: GEMV / M<=16 row).
//  * online softmax in the log2 domain; the 4 waves are merged through LDS.
//  * num_partitions == 1 writes the bf16 output directly; otherwise partials
//    (normalised O + (max, sum)) go to a workspace reduced by a second kernel.
// Grid dims are fixed by (B, nkv, max_partitions) so the launch is hipGraph
// capturable for a batch-size bucket; partitions past a sequence's end exit.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

#include <cstdlib>

namespace hipserve {

constexpr int kDecWavesMax = 8;
constexpr int kChunk = 32;
constexpr float kLog2e = 1.4426950408889634f;

// out16 (optional): an f16 copy of the bf16 output in the quantised decode GEMMs' staging
// pair order {0, 2, 1, 3, 4, 6, 5, 7} per aligned 8-run — the o-projection's x16 operand
// (gguf_mfma.hip), written here instead of by a conversion kernel
HS_DEVICE void store_o16(unsigned short* __restrict__ out16, long row_off, int e, unsigned short bf) {
  const int p = (e & ~7) | (e & 4) | ((e & 1) << 1) | ((e >> 1) & 1);
  out16[row_off + p] = __builtin_bit_cast(unsigned short, static_cast<_Float16>(bf16_to_f32(bf)));
}

// Fused decode input (kQKV): the qkv projection's fp32 split-K partials instead of a
// bf16 q row. The kernel sums them, applies RoPE to q (and to the new token's k),
// writes the new token's k / v into the paged cache and attends — replacing the
// separate splitk_rope_cache launch of the fused decode layer. Rounding matches that
// kernel exactly (bf16 after the sum, bf16 after RoPE).
struct QkvIn {
  const float* ws;        // partials [S, B, N], N = (nq + 2 nkv) * D
  long slice;             // B * N
  int S, N;
  const long* positions;  // [B]
  const long* slots;      // [B], -1 = padding row (no cache write)
  const float* cos_sin;   // [max_pos, D]: cos in [0, D/2), sin in [D/2, D)
  unsigned short* k_cache;
  unsigned short* v_cache;
  int mode;               // 0 = rotate-half (HF), 1 = interleaved pairs (GGUF llama)
  const float* qw;        // per-head q / k RMSNorm weights [D] before RoPE (Qwen3), or null;
  const float* kw;        // rotate-half only; rounding as splitk_rope_cache (bf16 after the norm)
  float eps;
};

// per-head RMSNorm of 8 + 8 values (d and d + D/2 of one rotate-half chunk) whose
// head spans lanes: the same sum order as splitk_rope_cache's kNorm branch (own x
// terms, own y terms, then the chunk-xor partners), applied and rounded to bf16
template <int D>
HS_DEVICE void qk_norm_apply(float (&x)[8], float (&y)[8], float ss, const float* nw, int d0, float eps) {
  const float inv = rsqrtf(ss / D + eps);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    x[j] = bf16_to_f32(f32_to_bf16(x[j] * inv * nw[d0 + j]));
    y[j] = bf16_to_f32(f32_to_bf16(y[j] * inv * nw[D / 2 + d0 + j]));
  }
}
HS_DEVICE float sumsq16(const float (&x)[8], const float (&y)[8]) {
  float ss = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) ss += x[j] * x[j];
#pragma unroll
  for (int j = 0; j < 8; ++j) s2 += y[j] * y[j];
  return ss + s2;
}

// 8 consecutive partial sums over the S slices, rounded to bf16 (as splitk_rope_cache)
HS_DEVICE void qkv_sum8(float (&o)[8], const float* p, long slice, int S) {
  f32x4 lo, hi;
  sum_slices8(lo, hi, p, slice, S);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = bf16_to_f32(f32_to_bf16(lo[j]));
    o[j + 4] = bf16_to_f32(f32_to_bf16(hi[j]));
  }
}

// two register sets for the chunk pipeline: keep VGPR + AGPR <= 256 so two waves fit
// per SIMD (two 4-wave workgroups per CU — B = 64 x 8 kv heads is 2 per CU)
// KV: the cache element, bf16 (unsigned short) or e4m3 (unsigned char, widened to bf16
// in registers right before its MFMA: half the HBM bytes of the memory-bound stream)
template <int D, int kDecWaves, bool kQKV = false, bool kNT = true, typename KV = unsigned short>
__global__ __launch_bounds__(64 * kDecWaves) __attribute__((amdgpu_waves_per_eu(2, 8))) void paged_decode_kernel(
    unsigned short* __restrict__ out, long out_stride,
    const unsigned short* __restrict__ q, long q_stride,
    const KV* __restrict__ k_cache,
    const KV* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ context_lens, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, int nq, int nkv, int block_size, int part_size,
    int max_parts, float scale, int window, QkvIn qi = QkvIn{}, unsigned short* __restrict__ out16 = nullptr) {
  static_assert(D == 128 || D == 96 || D == 64, "head_dim 64, 96 or 128");
  static_assert(!kQKV || sizeof(KV) == 2, "the fused qkv decode writes a bf16 cache");
  constexpr int KS = D / 32;  // k-steps of the QK MFMA
  constexpr int NB = D / 16;  // 16-column blocks of the PV output
  // e4m3 cache (head_dim 64 / 128): 64-token chunks so every K / V load is 16 bytes (16 d
  // of one key, 16 keys of one V^T row) — with 32-token chunks the e4m3 stream ran as
  // 8-byte loads at ~3.7 TB/s, issue- rather than HBM-bound. The QK MFMA's k index is
  // permuted to match: k-step ks, lane group g, slot j <-> d = 16 g + 64 (ks >> 1) + 8 (ks & 1) + j
  // (Q is loaded in the same order); S tile t, row m <-> key 16 (m >> 2) + 4 t + (m & 3), so
  // lane group g holds keys 16 g .. 16 g + 15 of the chunk: keys 16 g + j feed the first
  // P.V MFMA's k-slots 8 g + j and keys 16 g + 8 + j the second, as the V^T load splits
  constexpr bool kWide = sizeof(KV) == 1 && KS % 2 == 0;
  constexpr int CH = kWide ? 2 * kChunk : kChunk;
  const int part = blockIdx.x, kh = blockIdx.y, b = blockIdx.z;
  const int ctx = context_lens[b];
  // sliding window: keys [lo, ctx); partitions start at lo rounded down to a
  // 32-token chunk (aligned V loads), the keys below lo are masked
  const int lo = window > 0 ? max(0, ctx - window) : 0;
  const int lo_al = lo & ~(CH - 1);
  const int start = lo_al + part * part_size;
  if (start >= ctx) return;
  const int end = min(start + part_size, ctx);
  const int G = nq / nkv;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = lane & 15, grp = lane >> 4;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* bt = reinterpret_cast<int*>(smem);                       // <= 256 block ids
  float* red = reinterpret_cast<float*>(smem + 1024);          // m,l per wave/head
  float* olds = red + 2 * kDecWaves * 16;                      // [waves][16][D]

  // power-of-two block sizes (EngineConfig): shifts / masks in the per-chunk paging math
  const int bsh = __builtin_ctz(block_size), bmask = block_size - 1;
  const int first_blk = start >> bsh;
  const int nbt = ((end - 1) >> bsh) - first_blk + 1;
  const int* btab = block_tables + (long)b * bt_stride + first_blk;
  for (int i = threadIdx.x; i < nbt; i += blockDim.x) bt[i] = btab[i];
  __syncthreads();

  const long kv_head_stride = (long)block_size * D;  // elements per (block, head)
  const int nchunks = (end - start + CH - 1) / CH;
  const int last_tok = ctx - 1;
  const int bt_base_tok = first_blk * block_size;

  // Software pipeline over this wave's chunks (wave, wave + W, ...): the K / V
  // loads of the next chunk are issued before the current chunk's MFMAs, from two
  // register sets used alternately (loop unrolled by 2, no exit inside a pair, loads
  // unconditional with the chunk index clamped), so each chunk's HBM latency hides
  // behind the previous chunk's math instead of being exposed once per chunk.
  using KV8 = typename KvVec<KV>::T;
  struct Chunk {
    KV8 ka[KS], kb[KS], vv[NB];
  };
  struct ChunkW {  // kWide: 16 e4m3 per register quad
    u32x4 k[4][KS / 2 > 0 ? KS / 2 : 1], v[NB];
  };
  // K / V are read exactly once per step by one wave: non-temporal loads (aux nt) keep
  // them from evicting the weights' and partials' lines and shorten issue -> landed
  auto ld = [](const KV* p) -> KV8 {
    if constexpr (kNT) return kv_load8_nt(p);
    else return kv_load8(p);
  };
  auto ld16 = [](const KV* p) -> u32x4 {
    if constexpr (kNT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
  };
  [[maybe_unused]] auto load_chunk_w = [&](int c, ChunkW& ch) {
    const int cs = start + min(c, nchunks - 1) * CH;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tk = min(cs + 16 * (col >> 2) + 4 * t + (col & 3), last_tok);
      const KV* kp = k_cache + ((long)bt[(tk - bt_base_tok) >> bsh] * nkv + kh) * kv_head_stride +
                     (long)(tk & bmask) * D + 16 * grp;
#pragma unroll
      for (int hh = 0; hh < KS / 2; ++hh) ch.k[t][hh] = ld16(kp + 64 * hh);
    }
    int tv = cs + 16 * grp;
    if (tv > last_tok) tv = last_tok & ~15;
    const KV* vb = v_cache + ((long)bt[(tv - bt_base_tok) >> bsh] * nkv + kh) * kv_head_stride + (tv & bmask) +
                   (long)col * block_size;
#pragma unroll
    for (int n = 0; n < NB; ++n) ch.v[n] = ld16(vb + (long)16 * n * block_size);
  };
  auto load_chunk = [&](int c, Chunk& ch) {
    const int cs = start + min(c, nchunks - 1) * kChunk;
    // K: tile a row m -> token 8*(m>>2) + (m&3); tile b -> +4
    const int m = col;
    int ta = cs + 8 * (m >> 2) + (m & 3);
    int tb = ta + 4;
    ta = min(ta, last_tok);
    tb = min(tb, last_tok);
    const KV* ka = k_cache +
        ((long)bt[(ta - bt_base_tok) >> bsh] * nkv + kh) * kv_head_stride +
        (long)(ta & bmask) * D + 8 * grp;
    const KV* kb = k_cache +
        ((long)bt[(tb - bt_base_tok) >> bsh] * nkv + kh) * kv_head_stride +
        (long)(tb & bmask) * D + 8 * grp;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ch.ka[ks] = ld(ka + 32 * ks);
      ch.kb[ks] = ld(kb + 32 * ks);
    }
    // V: lane holds V^T[d = 16n + col][tokens 8*grp .. +7]
    int tv = cs + 8 * grp;
    if (tv > last_tok) tv = last_tok & ~7;
    const KV* vb = v_cache +
        ((long)bt[(tv - bt_base_tok) >> bsh] * nkv + kh) * kv_head_stride +
        (tv & bmask) + (long)col * block_size;
#pragma unroll
    for (int n = 0; n < NB; ++n) ch.vv[n] = ld(vb + (long)16 * n * block_size);
  };
  Chunk A, B;
  bool pre = false;  // kQKV: this wave's first chunk already in flight (A)

  // Q fragment: B[k = d][n = head]; lane holds head `col`, d = 8*grp + 32*ks + j
  bf16x8 qf[KS];
  if constexpr (!kQKV) {
    const int h = kh * G + col;
    const unsigned short* qrow = q + (long)b * q_stride + (long)h * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = kWide ? 16 * grp + 64 * (ks >> 1) + 8 * (ks & 1) : 8 * grp + 32 * ks;
      u16x8 v = (col < G) ? *reinterpret_cast<const u16x8*>(qrow + d0) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      qf[ks] = __builtin_bit_cast(bf16x8, v);
    }
  } else {
    static_assert(!kQKV || KS % 2 == 0, "fused qkv decode: head_dim 64 or 128");
    // this wave's first K / V chunk goes out before the partial sums below, so their
    // latency overlaps the stream instead of preceding it — unless that chunk is the
    // last one, which holds the new token written below
    if (wave < nchunks && !(end == ctx && wave == nchunks - 1)) {
      load_chunk(wave, A);
      pre = true;
    }
    constexpr int half = D / 2;
    const long pos = qi.positions[b];
    const float* cs = qi.cos_sin + pos * D;
    const float* wrow = qi.ws + (long)b * qi.N;
    // --- the new token's k (RoPE) and v into the paged cache, by the ONE wave of the
    //     workgroup whose partition holds the last position that will stream the last
    //     chunk (chunk c belongs to wave c % W): no workgroup barrier, the other waves
    //     start streaming at once and never read the new token
    const long slot = qi.slots[b];
    const int nch = (end - start + CH - 1) / CH;
    if (end == ctx && slot >= 0 && wave == (nch - 1) % kDecWaves) {
      const long blk = slot / block_size;
      const int off = (int)(slot % block_size);
      const int nk_items = qi.mode == 0 ? half / 8 : D / 8;
      const int it = lane;
      if (it < nk_items + D / 8) {
        if (it >= nk_items) {  // v: transposed cache block (tokens contiguous per d)
          const int c8 = it - nk_items;
          float x[8];
          qkv_sum8(x, wrow + (long)(nq + nkv) * D + (long)kh * D + c8 * 8, qi.slice, qi.S);
          unsigned short* vc = qi.v_cache + (blk * nkv + kh) * (long)D * block_size + off;
#pragma unroll
          for (int j = 0; j < 8; ++j) vc[(c8 * 8 + j) * block_size] = f32_to_bf16(x[j]);
        } else {
          const float* kr = wrow + (long)nq * D + (long)kh * D;
          unsigned short* kc = qi.k_cache + ((blk * nkv + kh) * block_size + off) * (long)D;
          if (qi.mode == 0) {
            float x[8], y[8];
            qkv_sum8(x, kr + it * 8, qi.slice, qi.S);
            qkv_sum8(y, kr + half + it * 8, qi.slice, qi.S);
            if (qi.kw != nullptr) {  // lanes 0 .. D/16-1 hold the head's chunks: xor within them
              float ss = sumsq16(x, y);
              for (int o = nk_items / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
              qk_norm_apply<D>(x, y, ss, qi.kw, it * 8, qi.eps);
            }
            u16x8 va, vb;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float co = cs[it * 8 + j], si = cs[half + it * 8 + j];
              float ra, rb;
              rope_rot(x[j], y[j], co, si, ra, rb);
              va[j] = f32_to_bf16(ra);
              vb[j] = f32_to_bf16(rb);
            }
            *reinterpret_cast<u16x8*>(kc + it * 8) = va;
            *reinterpret_cast<u16x8*>(kc + half + it * 8) = vb;
          } else {
            float x[8];
            qkv_sum8(x, kr + it * 8, qi.slice, qi.S);
            u16x8 v;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
              const int i = it * 4 + p;
              const float co = cs[i], si = cs[half + i];
              float ra, rb;
              rope_rot(x[2 * p], x[2 * p + 1], co, si, ra, rb);
              v[2 * p] = f32_to_bf16(ra);
              v[2 * p + 1] = f32_to_bf16(rb);
            }
            *reinterpret_cast<u16x8*>(kc + it * 8) = v;
          }
        }
      }
    }
    // --- q: sum, round, RoPE in-lane (partner d +- D/2 is fragment ks +- KS/2;
    //     interleaved pairs sit inside each 8-run), round. Computed ONCE per workgroup:
    //     wave w owns fragment pair (w, w + KS/2) (rotate-half) or fragment w
    //     (interleaved), publishes it in LDS, and every wave reads all KS fragments
    //     after the barrier (which also orders the new token's K / V stores before any
    //     wave's loads of the last chunk)
    u16x8* qsh = reinterpret_cast<u16x8*>(olds + kDecWaves * 16 * D);  // [KS][64 lanes]
    const int h = kh * G + col;
    auto q_frag = [&](int ks, float (&v)[8]) {
      if (col < G) {
        qkv_sum8(v, wrow + (long)h * D + 8 * grp + 32 * ks, qi.slice, qi.S);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
    };
    auto q_store = [&](int ks, const float (&v)[8]) {
      u16x8 u;
#pragma unroll
      for (int j = 0; j < 8; ++j) u[j] = col < G ? f32_to_bf16(v[j]) : 0;
      qsh[ks * 64 + lane] = u;
    };
    if (qi.mode == 0 && qi.qw != nullptr) {
      // per-head q norm: the head's rotate-half chunk c = 4 ks + grp (D = 128) sits in
      // fragments ks < KS/2 of lane group grp, so wave 0 computes every fragment: the
      // chunk-xor tree of splitk_rope_cache is in-lane (xor 4 at D = 128) then lane xor
      // 32 (chunk xor 2) and 16 (chunk xor 1); bit-identical sums
      if (wave == 0) {
        float x[KS / 2][8], y[KS / 2][8];
        float ssk[KS / 2];
#pragma unroll
        for (int ks = 0; ks < KS / 2; ++ks) {
          q_frag(ks, x[ks]);
          q_frag(ks + KS / 2, y[ks]);
          ssk[ks] = sumsq16(x[ks], y[ks]);
        }
        float ss = ssk[0];
        if constexpr (KS / 2 == 2) ss += ssk[1];
        ss += __shfl_xor(ss, 32, 64);
        ss += __shfl_xor(ss, 16, 64);
#pragma unroll
        for (int ks = 0; ks < KS / 2; ++ks) {
          qk_norm_apply<D>(x[ks], y[ks], ss, qi.qw, 8 * grp + 32 * ks, qi.eps);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = 8 * grp + 32 * ks + j;
            const float co = cs[i], si = cs[half + i];
            const float a = x[ks][j], bb = y[ks][j];
            rope_rot(a, bb, co, si, x[ks][j], y[ks][j]);
          }
          q_store(ks, x[ks]);
          q_store(ks + KS / 2, y[ks]);
        }
      }
    } else if (qi.mode == 0) {
      for (int ks = wave; ks < KS / 2; ks += kDecWaves) {
        float x[8], y[8];
        q_frag(ks, x);
        q_frag(ks + KS / 2, y);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * grp + 32 * ks + j;
          const float co = cs[i], si = cs[half + i];
          const float a = x[j], bb = y[j];
          rope_rot(a, bb, co, si, x[j], y[j]);
        }
        q_store(ks, x);
        q_store(ks + KS / 2, y);
      }
    } else {
      for (int ks = wave; ks < KS; ks += kDecWaves) {
        float x[8];
        q_frag(ks, x);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int i = (8 * grp + 32 * ks) / 2 + p;
          const float co = cs[i], si = cs[half + i];
          const float a = x[2 * p], bb = x[2 * p + 1];
          rope_rot(a, bb, co, si, x[2 * p], x[2 * p + 1]);
        }
        q_store(ks, x);
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, qsh[ks * 64 + lane]);
  }
  const float sl2 = scale * kLog2e;
  f32x4 o[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -1e30f, l_run = 0.f;

  auto compute_chunk = [&](int c, const Chunk& ch) {
    const int cs = start + c * kChunk;
    // ---- S^T = K . Q^T
    f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      sa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv_widen8(ch.ka[ks])), qf[ks], sa, 0, 0, 0);
      sb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv_widen8(ch.kb[ks])), qf[ks], sb, 0, 0, 0);
    }
    // lane holds scores of tokens cs + 8*grp + r (sa) and + 4 + r (sb) for head col
    float sc[8];
    float mx = -1e30f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t0 = cs + 8 * grp + r;
      sc[r] = (t0 >= lo && t0 <= last_tok) ? sa[r] * sl2 : -1e30f;
      sc[r + 4] = (t0 + 4 >= lo && t0 + 4 <= last_tok) ? sb[r] * sl2 : -1e30f;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) mx = fmaxf(mx, sc[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float psum = 0.f;
    bf16x8 pf;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float pr = exp2f(sc[r] - m_new);
      psum += pr;
      pf[r] = static_cast<__bf16>(pr);
    }
    l_run = l_run * alpha + psum;
    // rescale O: rows of the PV output are heads 4*grp + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a_r = __shfl(alpha, 4 * grp + r, 64);
#pragma unroll
      for (int n = 0; n < NB; ++n) o[n][r] *= a_r;
    }
    // ---- O += P . V
#pragma unroll
    for (int n = 0; n < NB; ++n)
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, kv_widen8(ch.vv[n])), o[n], 0, 0, 0);
  };
  [[maybe_unused]] auto compute_chunk_w = [&](int c, const ChunkW& ch) {
    const int cs = start + c * CH;
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int hh = 0; hh < KS / 2; ++hh) {
        const u32x4 w = ch.k[t][hh];
        st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv_widen8(u32x2{w[0], w[1]})),
                                                        qf[2 * hh], st[t], 0, 0, 0);
        st[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv_widen8(u32x2{w[2], w[3]})),
                                                        qf[2 * hh + 1], st[t], 0, 0, 0);
      }
    }
    // lane holds the scores of keys cs + 16 grp + 4 t + r for head col
    float sc[16];
    float mx = -1e30f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int tk = cs + 16 * grp + 4 * t + r;
        sc[4 * t + r] = (tk >= lo && tk <= last_tok) ? st[t][r] * sl2 : -1e30f;
        mx = fmaxf(mx, sc[4 * t + r]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    m_run = m_new;
    float psum = 0.f;
    bf16x8 p0, p1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a0 = exp2f(sc[j] - m_new), a1 = exp2f(sc[8 + j] - m_new);
      psum += a0 + a1;
      p0[j] = static_cast<__bf16>(a0);
      p1[j] = static_cast<__bf16>(a1);
    }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a_r = __shfl(alpha, 4 * grp + r, 64);
#pragma unroll
      for (int n = 0; n < NB; ++n) o[n][r] *= a_r;
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const u32x4 w = ch.v[n];
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(p0, __builtin_bit_cast(bf16x8, kv_widen8(u32x2{w[0], w[1]})),
                                                     o[n], 0, 0, 0);
      o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(p1, __builtin_bit_cast(bf16x8, kv_widen8(u32x2{w[2], w[3]})),
                                                     o[n], 0, 0, 0);
    }
  };
  constexpr int W = kDecWaves;
  int c = wave;
  if constexpr (kWide) {
    ChunkW AW, BW;
    if (c < nchunks) {
      load_chunk_w(c, AW);
      for (; c + W < nchunks; c += 2 * W) {
        load_chunk_w(c + W, BW);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk_w(c, AW);
        load_chunk_w(c + 2 * W, AW);
        __builtin_amdgcn_sched_barrier(0);
        compute_chunk_w(c + W, BW);
      }
      if (c < nchunks) compute_chunk_w(c, AW);
    }
  } else if (c < nchunks) {
    if (!pre) load_chunk(c, A);
    for (; c + W < nchunks; c += 2 * W) {
      load_chunk(c + W, B);
      __builtin_amdgcn_sched_barrier(0);
      compute_chunk(c, A);
      load_chunk(c + 2 * W, A);
      __builtin_amdgcn_sched_barrier(0);
      compute_chunk(c + W, B);
    }
    if (c < nchunks) compute_chunk(c, A);
  }

  // ---- per-wave row sums, then merge the 4 waves through LDS
  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  if (lane < 16) {
    red[(wave * 16 + lane) * 2 + 0] = m_run;
    red[(wave * 16 + lane) * 2 + 1] = l_run;
  }
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 4 * grp + r;
      olds[(wave * 16 + h) * D + 16 * n + col] = o[n][r];
    }
  __syncthreads();

  const int nparts_seq = (ctx - lo_al + part_size - 1) / part_size;
  for (int it = threadIdx.x; it < G * D; it += blockDim.x) {
    const int h = it / D, d = it % D;
    float M = -1e30f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) M = fmaxf(M, red[(w * 16 + h) * 2]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) {
      const float f = exp2f(red[(w * 16 + h) * 2] - M);
      L += red[(w * 16 + h) * 2 + 1] * f;
      acc += olds[(w * 16 + h) * D + d] * f;
    }
    const int hq = kh * G + h;
    if (nparts_seq == 1) {
      const unsigned short ob = f32_to_bf16(acc / L);
      out[(long)b * out_stride + (long)hq * D + d] = ob;
      if (out16 != nullptr) store_o16(out16, (long)b * out_stride, hq * D + d, ob);
    } else {
      const long base = ((long)b * nq + hq) * max_parts + part;
      tmp_out[base * D + d] = acc / L;
      if (d == 0) {
        tmp_ml[base * 2 + 0] = M;
        tmp_ml[base * 2 + 1] = L;
      }
    }
  }
}

// Merge partitions: one workgroup per (head, sequence) of G lane groups (reduce_groups), one
// lane per d. The partitions are split over the groups (p = grp, grp + G, ...) and each
// lane keeps 4 independent partial sums, so a long context's 100+ partitions are 4 x G
// loads in flight per lane instead of one serial L2 round trip per partition (32K-token
// contexts, 128 partitions: 22 us per layer serially, profiles/r4_prof32k_summary.md).
// lane groups: G * D <= 512 lanes in whole waves (D = 96: 4 groups, 384 lanes)
template <int D>
constexpr int reduce_groups() { return D == 96 ? 4 : 512 / D; }

template <int D>
__global__ __launch_bounds__(512) void paged_decode_reduce_kernel(
    unsigned short* __restrict__ out, long out_stride,
    const float* __restrict__ tmp_out, const float* __restrict__ tmp_ml,
    const int* __restrict__ context_lens, int nq, int part_size, int max_parts, int window, int align,
    unsigned short* __restrict__ out16 = nullptr) {
  constexpr int G = reduce_groups<D>();
  static_assert(G * D % 64 == 0, "whole waves");
  const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int d = tid % D, grp = tid / D;
  const int ctx = context_lens[b];
  // the attention kernel's partition origin: the window start rounded down to its chunk
  const int lo_al = (window > 0 ? max(0, ctx - window) : 0) & ~(align - 1);
  const int np = (ctx - lo_al + part_size - 1) / part_size;
  if (np <= 1) return;
  const long base = ((long)b * nq + h) * max_parts;
  __shared__ float red[G * D + G + 16];
  // M = max over the partitions' running maxima (block reduction)
  float M = -1e30f;
  for (int p = tid; p < np; p += G * D) M = fmaxf(M, tmp_ml[(base + p) * 2]);
  for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o));
  if ((tid & 63) == 0) red[G * D + G + (tid >> 6)] = M;
  __syncthreads();
  M = -1e30f;
#pragma unroll
  for (int w = 0; w < G * D / 64; ++w) M = fmaxf(M, red[G * D + G + w]);
  float L[4] = {0.f, 0.f, 0.f, 0.f}, acc[4] = {0.f, 0.f, 0.f, 0.f};
  int p = grp;
  for (; p + 3 * G < np; p += 4 * G) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long q = base + p + u * G;
      const float w = exp2f(tmp_ml[q * 2] - M) * tmp_ml[q * 2 + 1];
      L[u] += w;
      acc[u] += w * tmp_out[q * D + d];
    }
  }
  for (; p < np; p += G) {
    const float w = exp2f(tmp_ml[(base + p) * 2] - M) * tmp_ml[(base + p) * 2 + 1];
    L[0] += w;
    acc[0] += w * tmp_out[(base + p) * D + d];
  }
  red[grp * D + d] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (d == 0) red[G * D + grp] = (L[0] + L[1]) + (L[2] + L[3]);
  __syncthreads();
  if (grp == 0) {
    float a = 0.f, l = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      a += red[g * D + d];
      l += red[G * D + g];
    }
    const unsigned short ob = f32_to_bf16(a / l);
    out[(long)b * out_stride + (long)h * D + d] = ob;
    if (out16 != nullptr) store_o16(out16, (long)b * out_stride, h * D + d, ob);
  }
}

static size_t smem_bytes(int D, int waves) {
  // block ids, per-wave (m, l), per-wave O, then the fused path's q fragments [D/32][64] x 16 B
  return 1024 + (size_t)2 * waves * 16 * sizeof(float) + (size_t)waves * 16 * D * sizeof(float) +
         (size_t)(D / 32) * 64 * 16;
}

size_t paged_decode_smem_bytes(int D) { return smem_bytes(D, kDecWavesMax); }

// waves per workgroup (HIPSERVE_DECODE_WAVES = 4 | 8). 8 waves = more concurrent
// 32-token chunk streams per (sequence, kv head) but measured no faster on
// MI355X (B=64 ctx 1152: 48.2 vs 47.3 us; profiles/decode_partition_sweep.md).
static int decode_waves() {
  static const int env = [] {
    const char* e = getenv("HIPSERVE_DECODE_WAVES");
    return e ? atoi(e) : 4;
  }();
  return env == 8 ? 8 : 4;
}

// K / V load policy. Non-temporal when the grid streams the KV at full chip
// bandwidth (>= 256 workgroups): Llama-3-8B, B = 64, ctx 1152, cold KV 56.8 -> 51.6 us,
// decode step 5.51 -> 5.36 ms. Small grids (B = 1, 16 workgroups) are latency-bound and
// lose with nt (26.7 -> 37.2 us): default policy there. HIPSERVE_DECODE_NT = 0 disables.
static bool decode_nt(long workgroups) {
  static const bool env = [] {
    const char* e = getenv("HIPSERVE_DECODE_NT");
    return !(e && atoi(e) == 0);
  }();
  return env && workgroups >= 256;
}

// the decode kernel's chunk (= window-origin alignment): 64 keys for an e4m3 cache at head_dim
// 64 / 128 (paged_decode_kernel kWide), else 32
static int dec_align(int D, bool kv_f8) { return kv_f8 && D != 96 ? 2 * kChunk : kChunk; }

void launch_paged_decode(void* out, long out_stride, const void* q, long q_stride,
                         const void* k_cache, const void* v_cache,
                         const int* block_tables, int bt_stride,
                         const int* context_lens, float* tmp_out, float* tmp_ml,
                         int B, int nq, int nkv, int D, int block_size,
                         int part_size, int max_parts, float scale, int window,
                         hipStream_t s, void* out16, bool kv_f8) {
  if (B <= 0) return;
  auto* o16 = static_cast<unsigned short*>(out16);
  const int waves = decode_waves();
  dim3 grid(max_parts, nkv, B), block(64 * waves);
  const size_t smem = smem_bytes(D, waves);
  auto* o = static_cast<unsigned short*>(out);
  auto* qq = static_cast<const unsigned short*>(q);
  auto* kc = static_cast<const unsigned short*>(k_cache);
  auto* vc = static_cast<const unsigned short*>(v_cache);
  auto* kc8 = static_cast<const unsigned char*>(k_cache);
  auto* vc8 = static_cast<const unsigned char*>(v_cache);
#define HS_DECODE_KV(DD, WW, NT)                                                                              \
  do {                                                                                                      \
    if (kv_f8)                                                                                              \
      paged_decode_kernel<DD, WW, false, NT, unsigned char><<<grid, block, smem, s>>>(                      \
          o, out_stride, qq, q_stride, kc8, vc8, block_tables, bt_stride, context_lens, tmp_out, tmp_ml, nq, \
          nkv, block_size, part_size, max_parts, scale, window, QkvIn{}, o16);                              \
    else                                                                                                    \
      paged_decode_kernel<DD, WW, false, NT><<<grid, block, smem, s>>>(                                     \
          o, out_stride, qq, q_stride, kc, vc, block_tables, bt_stride, context_lens, tmp_out, tmp_ml, nq,  \
          nkv, block_size, part_size, max_parts, scale, window, QkvIn{}, o16);                              \
  } while (0)
#define HS_DECODE(DD, WW)                                                                                   \
  do {                                                                                                      \
    if (decode_nt((long)max_parts * nkv * B)) HS_DECODE_KV(DD, WW, true);                                   \
    else HS_DECODE_KV(DD, WW, false);                                                                       \
  } while (0)
#define HS_DECODE_D(DD)                                                                                      \
  do {                                                                                                      \
    if (waves == 8) HS_DECODE(DD, 8);                                                                       \
    else HS_DECODE(DD, 4);                                                                                  \
    if (max_parts > 1)                                                                                      \
      paged_decode_reduce_kernel<DD><<<dim3(nq, B), dim3(reduce_groups<DD>() * DD), 0, s>>>(o, out_stride, tmp_out, tmp_ml, \
                                                                       context_lens, nq, part_size, max_parts, \
                                                                       window, dec_align(DD, kv_f8), o16);  \
  } while (0)
  if (D == 128) HS_DECODE_D(128);
  else if (D == 96) HS_DECODE_D(96);
  else HS_DECODE_D(64);
#undef HS_DECODE_D
#undef HS_DECODE
#undef HS_DECODE_KV
}

// Fused decode: qkv partials -> RoPE + KV write + attention (see QkvIn). D in {64, 128}.
void launch_paged_decode_qkv(void* out, long out_stride, const float* ws, int S, int N, const long* positions,
                             const long* slots, const float* cos_sin, int mode, void* k_cache, void* v_cache,
                             const int* block_tables, int bt_stride, const int* context_lens, float* tmp_out,
                             float* tmp_ml, int B, int nq, int nkv, int D, int block_size, int part_size,
                             int max_parts, float scale, int window, hipStream_t s, void* out16,
                             const float* qw, const float* kw, float eps) {
  if (B <= 0) return;
  auto* o16 = static_cast<unsigned short*>(out16);
  const int waves = decode_waves();
  dim3 grid(max_parts, nkv, B), block(64 * waves);
  const size_t smem = smem_bytes(D, waves);
  auto* o = static_cast<unsigned short*>(out);
  auto* kc = static_cast<unsigned short*>(k_cache);
  auto* vc = static_cast<unsigned short*>(v_cache);
  const QkvIn qi{ws, (long)B * N, S, N, positions, slots, cos_sin, kc, vc, mode, qw, kw, eps};
#define HS_DECODE_QKV(DD, WW)                                                                                  \
  do {                                                                                                        \
    if (decode_nt((long)max_parts * nkv * B))                                                                 \
      paged_decode_kernel<DD, WW, true, true><<<grid, block, smem, s>>>(                                      \
          o, out_stride, nullptr, 0, kc, vc, block_tables, bt_stride, context_lens, tmp_out, tmp_ml, nq, nkv, \
          block_size, part_size, max_parts, scale, window, qi, o16);                                          \
    else                                                                                                      \
      paged_decode_kernel<DD, WW, true, false><<<grid, block, smem, s>>>(                                     \
          o, out_stride, nullptr, 0, kc, vc, block_tables, bt_stride, context_lens, tmp_out, tmp_ml, nq, nkv, \
          block_size, part_size, max_parts, scale, window, qi, o16);                                          \
  } while (0)
#define HS_DECODE_QKV_D(DD)                                                                                   \
  do {                                                                                                        \
    if (waves == 8) HS_DECODE_QKV(DD, 8);                                                                     \
    else HS_DECODE_QKV(DD, 4);                                                                                \
    if (max_parts > 1)                                                                                        \
      paged_decode_reduce_kernel<DD><<<dim3(nq, B), dim3(reduce_groups<DD>() * DD), 0, s>>>(o, out_stride, tmp_out, tmp_ml,   \
                                                                       context_lens, nq, part_size, max_parts,   \
                                                                       window, kChunk, o16);                  \
  } while (0)
  if (D == 128) HS_DECODE_QKV_D(128);
  else HS_DECODE_QKV_D(64);
#undef HS_DECODE_QKV_D
#undef HS_DECODE_QKV
}

}  // namespace hipserve
