// Mixture-of-experts kernels for Mixtral-style sparse MLPs on
// gfx950. Graph-capturable: every grid is sized from static upper bounds and the
// data-dependent parts (tile count, expert of a tile) are read on the device.
//
//   moe_topk_softmax  router logits -> top-k experts + renormalised weights
//                     (one wave per token, experts on lanes, wave64 reductions)
//   moe_align         token/expert pairs sorted by expert into 16-row tiles,
//                     padding slots = -1 (one 1024-thread workgroup, LDS counts)
//   moe_gemm          per tile: out[slot] = x[row(slot)] . W_e^T on MFMA, rows
//                     gathered through the slot list (token rows for w13, slot rows
//                     for w2); each expert's weights stream once per 16-row tile
//   moe_combine       y rows of a token's k pairs, weighted sum -> hidden state
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

template <typename T>
HS_DEVICE float ld_f(const T* p, long i);
template <>
HS_DEVICE float ld_f<unsigned short>(const unsigned short* p, long i) { return bf16_to_f32(p[i]); }
template <>
HS_DEVICE float ld_f<float>(const float* p, long i) { return p[i]; }

// One wave per token, expert e on lane e % 64, slot e / 64 (E <= 128). renorm:
// weights / sum over the selected k (Mixtral, Qwen3-MoE norm_topk_prob); else the
// plain softmax probabilities of the selected experts.
// S > 0: ``logits`` are the router decode GEMM's fp32 split-K partials [S, T, E]; each
// logit is their in-order sum rounded to bf16, as splitk_reduce would have written it
// (bit-identical to reduce + this kernel, one launch fewer per MoE layer).
template <typename T>
__global__ __launch_bounds__(256) void moe_topk_softmax_kernel(const T* __restrict__ logits, float* __restrict__ w,
                                                               int* __restrict__ ids, int Tn, int E, int k,
                                                               int renorm, int S = 0) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= Tn) return;
  float v[2], p[2];
  int rank[2] = {-1, -1};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int e = lane + 64 * s;
    if constexpr (sizeof(T) == 4) {
      if (S > 0) {  // 8 slices' loads in flight at a time, summed in slice order
        float acc = 0.f;
        const int ec = e < E ? e : 0;
        for (int j0 = 0; j0 < S; j0 += 8) {
          float pv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) pv[i] = j0 + i < S ? ld_f<T>(logits, ((long)(j0 + i) * Tn + t) * E + ec) : 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (j0 + i < S) acc += pv[i];
        }
        v[s] = e < E ? bf16_to_f32(f32_to_bf16(acc)) : -INFINITY;
        continue;
      }
    }
    v[s] = e < E ? ld_f<T>(logits, (long)t * E + e) : -INFINITY;
  }
  const float mx = wave_max(fmaxf(v[0], v[1]));
  float ex[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) ex[s] = (lane + 64 * s) < E ? __expf(v[s] - mx) : 0.f;
  const float sum = wave_sum(ex[0] + ex[1]);
#pragma unroll
  for (int s = 0; s < 2; ++s) p[s] = ex[s] / sum;
  float sel_sum = 0.f;
  for (int j = 0; j < k; ++j) {
    // argmax over (lane, slot), ties -> lower expert id: the wave max of the unselected
    // probabilities, then the lowest lane holding it (slot 0 = experts 0-63 first)
    const float c0 = rank[0] < 0 && lane < E ? p[0] : -1.f;
    const float c1 = rank[1] < 0 && lane + 64 < E ? p[1] : -1.f;
    const float bv = wave_max(fmaxf(c0, c1));  // DPP reduction (common.h), wave-uniform
    const unsigned long long b0 = __ballot(c0 == bv), b1 = __ballot(c1 == bv);
    const int bi = b0 ? __builtin_ctzll(b0) : 64 + __builtin_ctzll(b1);
    if (bi == lane) rank[0] = j;
    if (bi == lane + 64) rank[1] = j;
    sel_sum += bv;
  }
  const float norm = renorm ? 1.f / sel_sum : 1.f;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (rank[s] >= 0) {
      w[(long)t * k + rank[s]] = p[s] * norm;
      ids[(long)t * k + rank[s]] = lane + 64 * s;
    }
  }
}

__global__ __launch_bounds__(1024) void moe_align_kernel(const int* __restrict__ ids, int npairs, int E, int tile,
                                                         int* __restrict__ slots, int slots_cap,
                                                         int* __restrict__ tile_expert, int tiles_cap,
                                                         int* __restrict__ num_tiles, int* __restrict__ pair_slot,
                                                         int* __restrict__ group_end) {
  __shared__ int cnt[128], off[129], cur[128];
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < 128) { cnt[tid] = 0; cur[tid] = 0; }
  __syncthreads();
  for (int p = tid; p < npairs; p += 1024) atomicAdd(&cnt[ids[p]], 1);
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the tile-padded counts, 2 experts per lane (E <= 128)
    const int e0 = 2 * lane, e1 = 2 * lane + 1;
    const int a = e0 < E ? (cnt[e0] + tile - 1) / tile * tile : 0;
    const int b = e1 < E ? (cnt[e1] + tile - 1) / tile * tile : 0;
    int incl = a + b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int excl = incl - a - b;
    off[e0] = excl;
    off[e1] = excl + a;
    if (group_end != nullptr) {  // per-expert end row of the padded expert-sorted slots (grouped GEMM offsets)
      if (e0 < E) group_end[e0] = excl + a;
      if (e1 < E) group_end[e1] = incl;
    }
    if (lane == 63) {
      off[128] = incl;
      *num_tiles = incl / tile;
    }
  }
  __syncthreads();
  const int total = off[128];
  for (int s = tid; s < slots_cap; s += 1024) slots[s] = -1;
  // each expert labels its own tiles; tiles past the used range are -1
  if (tid < E)
    for (int t = off[tid] / tile; t < (off[tid] + (cnt[tid] + tile - 1) / tile * tile) / tile; ++t) tile_expert[t] = tid;
  for (int t = total / tile + tid; t < tiles_cap; t += 1024) tile_expert[t] = -1;
  __syncthreads();
  for (int p = tid; p < npairs; p += 1024) {
    const int e = ids[p];
    const int pos = off[e] + atomicAdd(&cur[e], 1);
    slots[pos] = p;
    pair_slot[p] = pos;
  }
}

// Multi-workgroup moe_align for prefill-sized pair counts (one workgroup scatters ~0.6 ns
// per pair: 157 us per layer at 262K pairs). Pass 1: per-block expert histograms
// hist[b][E]. Pass 2: every block sums the table (nb x E ints) into the padded expert
// offsets and its own prefix, then scatters its chunk; block 0 also writes the tile table,
// the tile count and the padding slots (disjoint from every real slot, so no ordering
// between blocks is needed).
constexpr int kAlignChunk = 4096;
__global__ __launch_bounds__(1024) void moe_count_kernel(const int* __restrict__ ids, int npairs,
                                                         int* __restrict__ hist) {
  __shared__ int cnt[128];
  const int tid = threadIdx.x, b = blockIdx.x;
  if (tid < 128) cnt[tid] = 0;
  __syncthreads();
  const int end = min(npairs, (b + 1) * kAlignChunk);
  for (int p = b * kAlignChunk + tid; p < end; p += 1024) atomicAdd(&cnt[ids[p]], 1);
  __syncthreads();
  if (tid < 128) hist[b * 128 + tid] = cnt[tid];
}

__global__ __launch_bounds__(1024) void moe_place_kernel(const int* __restrict__ ids, int npairs, int E, int tile,
                                                         const int* __restrict__ hist, int nb,
                                                         int* __restrict__ slots, int slots_cap,
                                                         int* __restrict__ tile_expert, int tiles_cap,
                                                         int* __restrict__ num_tiles, int* __restrict__ pair_slot,
                                                         int* __restrict__ group_end) {
  __shared__ int cnt[128], pre[128], off[129], cur[128];
  const int tid = threadIdx.x, lane = tid & 63, b = blockIdx.x;
  if (tid < 128) {  // expert totals and this block's prefix over the blocks before it
    int c = 0, q = 0;
    for (int j = 0; j < nb; ++j) {
      const int h = hist[j * 128 + tid];
      c += h;
      q += j < b ? h : 0;
    }
    cnt[tid] = c;
    pre[tid] = q;
    cur[tid] = 0;
  }
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the tile-padded counts, 2 experts per lane (E <= 128)
    const int e0 = 2 * lane, e1 = 2 * lane + 1;
    const int a = e0 < E ? (cnt[e0] + tile - 1) / tile * tile : 0;
    const int c = e1 < E ? (cnt[e1] + tile - 1) / tile * tile : 0;
    int incl = a + c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    const int excl = incl - a - c;
    off[e0] = excl;
    off[e1] = excl + a;
    if (b == 0 && group_end != nullptr) {
      if (e0 < E) group_end[e0] = excl + a;
      if (e1 < E) group_end[e1] = incl;
    }
    if (lane == 63) {
      off[128] = incl;
      if (b == 0) *num_tiles = incl / tile;
    }
  }
  __syncthreads();
  if (b == 0) {
    const int total = off[128];
    for (int e = 0; e < E; ++e) {  // padding slots of each expert, then the unused tail
      const int lo = off[e] + cnt[e], hi = off[e] + (cnt[e] + tile - 1) / tile * tile;
      for (int s = lo + tid; s < hi; s += 1024) slots[s] = -1;
      for (int t = off[e] / tile + tid; t < hi / tile; t += 1024) tile_expert[t] = e;
    }
    for (int s = total + tid; s < slots_cap; s += 1024) slots[s] = -1;
    for (int t = total / tile + tid; t < tiles_cap; t += 1024) tile_expert[t] = -1;
  }
  const int end = min(npairs, (b + 1) * kAlignChunk);
  for (int p = b * kAlignChunk + tid; p < end; p += 1024) {
    const int e = ids[p];
    const int pos = off[e] + pre[e] + atomicAdd(&cur[e], 1);
    slots[pos] = p;
    pair_slot[p] = pos;
  }
}

int moe_align_blocks(int npairs) { return npairs > 4 * kAlignChunk ? (npairs + kAlignChunk - 1) / kAlignChunk : 1; }

// out[slot, N] = x[row(slot), K] . W[e, N, K]^T; row(slot) = pair / k (gather) or slot.
// A tile = 16*MT consecutive slots of one expert; each W fragment feeds MT MFMAs.
template <int MT, int KW>
__global__ __launch_bounds__(64 * KW) void moe_gemm_kernel(
    unsigned short* __restrict__ out, long out_stride, const unsigned short* __restrict__ x, long x_stride,
    const unsigned short* __restrict__ w, const int* __restrict__ slots, const int* __restrict__ tile_expert,
    int gather_k, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [KW][MT][64][4]
  const int tile = blockIdx.y;
  const int e = tile_expert[tile];
  if (e < 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int n0 = blockIdx.x * 16;
  int pr[MT];
  const unsigned short* xr[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int slot = tile * 16 * MT + 16 * t + c;
    pr[t] = slots[slot];
    const long xrow = pr[t] < 0 ? 0 : (gather_k > 0 ? pr[t] / gather_k : slot);
    xr[t] = x + xrow * x_stride + 64 * g;
  }
  const unsigned short* wr = w + ((long)e * N + min(n0 + c, N - 1)) * K + 64 * g;
  const int kw = K / KW, k0 = wave * kw, k1 = k0 + kw;
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kk = k0; kk < k1; kk += 256) {
    u16x8 a[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) a[s] = *reinterpret_cast<const u16x8*>(wr + kk + 8 * s);
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xr[t] + kk + 8 * s);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[s]),
                                                         __builtin_bit_cast(bf16x8, b), acc[t], 0, 0, 0);
      }
  }
  if constexpr (KW > 1) {
#pragma unroll
    for (int t = 0; t < MT; ++t) *reinterpret_cast<f32x4*>(red + ((wave * MT + t) * 64 + lane) * 4) = acc[t];
    __syncthreads();
    if (wave != 0) return;
#pragma unroll
    for (int t = 0; t < MT; ++t)
      for (int q = 1; q < KW; ++q) acc[t] += *reinterpret_cast<const f32x4*>(red + ((q * MT + t) * 64 + lane) * 4);
  }
  // C: col = slot-in-tile (lane & 15), rows n = n0 + 4g + j
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    if (pr[t] < 0) continue;
    const long slot = tile * 16 * MT + 16 * t + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 4 * g + j;
      if (n < N) out[slot * out_stride + n] = f32_to_bf16(acc[t][j]);
    }
  }
}

__global__ __launch_bounds__(256) void moe_combine_kernel(unsigned short* __restrict__ out, const unsigned short* __restrict__ y,
                                                          const float* __restrict__ w, const int* __restrict__ pair_slot,
                                                          int k, int H) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const float wt = w[(long)t * k + j];
      const u16x8 v = *reinterpret_cast<const u16x8*>(y + (long)pair_slot[t * k + j] * H + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += wt * bf16_to_f32(v[e]);
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(acc[e]);
    *reinterpret_cast<u16x8*>(out + (long)t * H + 8 * c) = o;
  }
}

// Split-K w2 partials ws[s][slot][H] (fp32): each pair's y row is bf16(sum over s),
// exactly what the bf16 expert GEMM output would be, then the weighted sum.
__global__ __launch_bounds__(256) void moe_combine_partial_kernel(unsigned short* __restrict__ out,
                                                                  const float* __restrict__ ws, long slab, int S,
                                                                  const float* __restrict__ w,
                                                                  const int* __restrict__ pair_slot, int k, int H) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x; c < H / 8; c += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const float wt = w[(long)t * k + j];
      const float* p = ws + (long)pair_slot[t * k + j] * H + 8 * c;
      f32x4 lo, hi;
      sum_slices8(lo, hi, p, slab, S);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[e] += wt * bf16_to_f32(f32_to_bf16(lo[e]));
        acc[e + 4] += wt * bf16_to_f32(f32_to_bf16(hi[e]));
      }
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(acc[e]);
    *reinterpret_cast<u16x8*>(out + (long)t * H + 8 * c) = o;
  }
}

// Decode MoE tail in one kernel: the weighted combine of a token's k expert rows (bf16
// y [slots, H], or fp32 w2 partials [S, slots, H] summed per pair in slice order) rounded
// to bf16 as moe_combine(_partial) writes it, then the residual add and the NEXT layer's
// RMSNorm exactly as fused_add_rmsnorm (norm.hip: same thread -> element map, same block
// reduction): bit-identical to the two-kernel chain, one launch fewer per MoE layer.
template <int NT, int VPT, bool kWF32, bool kPartial>
__global__ __launch_bounds__(NT) void moe_combine_add_rmsnorm_kernel(
    unsigned short* __restrict__ out, unsigned short* __restrict__ residual, const void* __restrict__ y, long slab,
    int S, const float* __restrict__ w, const int* __restrict__ pair_slot, int k, int H,
    const void* __restrict__ weight, float eps) {
  __shared__ float scratch[16];
  const int t = blockIdx.x;
  const int nvec = H >> 3;
  u16x8* rr = reinterpret_cast<u16x8*>(residual + (long)t * H);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < k; ++j) {
        const float wt = w[(long)t * k + j];
        const long row = (long)pair_slot[t * k + j] * H + 8 * idx;
        if constexpr (kPartial) {
          f32x4 lo, hi;
          sum_slices8(lo, hi, static_cast<const float*>(y) + row, slab, S);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[e] += wt * bf16_to_f32(f32_to_bf16(lo[e]));
            acc[e + 4] += wt * bf16_to_f32(f32_to_bf16(hi[e]));
          }
        } else {
          const u16x8 yv = *reinterpret_cast<const u16x8*>(static_cast<const unsigned short*>(y) + row);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += wt * bf16_to_f32(yv[e]);
        }
      }
      const u16x8 b = rr[idx];
      u16x8 sres;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = bf16_to_f32(f32_to_bf16(acc[e])) + bf16_to_f32(b[e]);
        sres[e] = f32_to_bf16(f);
        v[i][e] = bf16_to_f32(sres[e]);
      }
      rr[idx] = sres;
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += v[i][e] * v[i][e];
    }
  }
  ss = block_sum(ss, scratch);
  const float inv = rsqrtf(ss / H + eps);
  u16x8* orow = reinterpret_cast<u16x8*>(out + (long)t * H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * NT;
    if (idx < nvec) {
      float wv[8];
      if constexpr (kWF32) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(weight) + idx * 2;
        const f32x4 w0 = wp[0], w1 = wp[1];
#pragma unroll
        for (int e = 0; e < 4; ++e) { wv[e] = w0[e]; wv[e + 4] = w1[e]; }
      } else {
        const u16x8 wb = reinterpret_cast<const u16x8*>(weight)[idx];
#pragma unroll
        for (int e = 0; e < 8; ++e) wv[e] = bf16_to_f32(wb[e]);
      }
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(v[i][e] * inv * wv[e]);
      orow[idx] = o;
    }
  }
}

template <bool kWF32, bool kPartial>
static void mcn_launch(void* out, void* residual, const void* y, long slab, int S, const float* w, const int* ps,
                       int T, int k, int H, const void* nw, float eps, hipStream_t s) {
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  const int nvec = H / 8;
  if (norm_threads(H) == 256) {
    if (nvec <= 256) moe_combine_add_rmsnorm_kernel<256, 1, kWF32, kPartial><<<T, 256, 0, s>>>(o, r, y, slab, S, w, ps, k, H, nw, eps);
    else moe_combine_add_rmsnorm_kernel<256, 2, kWF32, kPartial><<<T, 256, 0, s>>>(o, r, y, slab, S, w, ps, k, H, nw, eps);
  } else {
    if (nvec <= 512) moe_combine_add_rmsnorm_kernel<512, 1, kWF32, kPartial><<<T, 512, 0, s>>>(o, r, y, slab, S, w, ps, k, H, nw, eps);
    else if (nvec <= 1024) moe_combine_add_rmsnorm_kernel<512, 2, kWF32, kPartial><<<T, 512, 0, s>>>(o, r, y, slab, S, w, ps, k, H, nw, eps);
    else moe_combine_add_rmsnorm_kernel<512, 4, kWF32, kPartial><<<T, 512, 0, s>>>(o, r, y, slab, S, w, ps, k, H, nw, eps);
  }
}

void launch_moe_combine_add_rmsnorm(void* out, void* residual, const void* y, long slab, int S, const float* w,
                                    const int* pair_slot, int T, int k, int H, const void* norm_w, bool norm_f32,
                                    float eps, hipStream_t s) {
  if (T <= 0) return;
  if (S > 0) {
    if (norm_f32) mcn_launch<true, true>(out, residual, y, slab, S, w, pair_slot, T, k, H, norm_w, eps, s);
    else mcn_launch<false, true>(out, residual, y, slab, S, w, pair_slot, T, k, H, norm_w, eps, s);
  } else {
    if (norm_f32) mcn_launch<true, false>(out, residual, y, slab, 0, w, pair_slot, T, k, H, norm_w, eps, s);
    else mcn_launch<false, false>(out, residual, y, slab, 0, w, pair_slot, T, k, H, norm_w, eps, s);
  }
}

void launch_moe_topk_softmax(const void* logits, bool logits_f32, float* w, int* ids, int T, int E, int k,
                             bool renorm, hipStream_t s, int splits) {
  if (T <= 0) return;
  dim3 grid((T + 3) / 4), block(256);
  if (logits_f32)
    moe_topk_softmax_kernel<float><<<grid, block, 0, s>>>(static_cast<const float*>(logits), w, ids, T, E, k,
                                                          renorm ? 1 : 0, splits);
  else
    moe_topk_softmax_kernel<unsigned short><<<grid, block, 0, s>>>(static_cast<const unsigned short*>(logits), w, ids,
                                                                   T, E, k, renorm ? 1 : 0);
}

void launch_moe_align(const int* ids, int npairs, int E, int tile, int* slots, int slots_cap, int* tile_expert,
                      int tiles_cap, int* num_tiles, int* pair_slot, int* group_end, hipStream_t s, int* hist) {
  const int nb = moe_align_blocks(npairs);
  if (nb > 1 && hist != nullptr) {
    moe_count_kernel<<<nb, 1024, 0, s>>>(ids, npairs, hist);
    moe_place_kernel<<<nb, 1024, 0, s>>>(ids, npairs, E, tile, hist, nb, slots, slots_cap, tile_expert, tiles_cap,
                                         num_tiles, pair_slot, group_end);
    return;
  }
  moe_align_kernel<<<1, 1024, 0, s>>>(ids, npairs, E, tile, slots, slots_cap, tile_expert, tiles_cap, num_tiles,
                                      pair_slot, group_end);
}

// Prefill MoE input: xs[slot] = x[slots[slot] / k] (the token of the pair in that
// slot), zero rows for padding slots — the A operand of the grouped expert GEMM.
// One workgroup per 8 slots, 16-byte vectors.
__global__ __launch_bounds__(256) void moe_gather_kernel(unsigned short* __restrict__ out,
                                                         const unsigned short* __restrict__ x, long x_stride,
                                                         const int* __restrict__ slots, int nslots, int k, int H) {
  const int vpr = H >> 3;  // 16-byte vectors per row
  const int slot = blockIdx.x * 8 + threadIdx.x / 32;
  if (slot >= nslots) return;
  const int p = slots[slot];
  u16x8* dst = reinterpret_cast<u16x8*>(out + (long)slot * H);
  if (p < 0) {
    for (int v = threadIdx.x & 31; v < vpr; v += 32) dst[v] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    return;
  }
  const u16x8* src = reinterpret_cast<const u16x8*>(x + (long)(p / k) * x_stride);
  for (int v = threadIdx.x & 31; v < vpr; v += 32) dst[v] = src[v];
}

void launch_moe_gather(void* out, const void* x, long x_stride, const int* slots, int nslots, int k, int H,
                       hipStream_t s) {
  if (nslots <= 0) return;
  moe_gather_kernel<<<(nslots + 7) / 8, 256, 0, s>>>(static_cast<unsigned short*>(out),
                                                     static_cast<const unsigned short*>(x), x_stride, slots, nslots,
                                                     k, H);
}

template <int MT>
static void moe_gemm_mt(void* out, long out_stride, const void* x, long x_stride, const void* w, const int* slots,
                        const int* tile_expert, int tiles_cap, int gather_k, int N, int K, hipStream_t s) {
  const int kw = (K % 1024 == 0) ? 4 : ((K % 512 == 0) ? 2 : 1);
  dim3 grid((N + 15) / 16, tiles_cap), block(64 * kw);
  const size_t smem = kw > 1 ? (size_t)kw * MT * 64 * 4 * sizeof(float) : 0;
  auto* o = static_cast<unsigned short*>(out);
  auto* xi = static_cast<const unsigned short*>(x);
  auto* wi = static_cast<const unsigned short*>(w);
  if (kw == 4)
    moe_gemm_kernel<MT, 4><<<grid, block, smem, s>>>(o, out_stride, xi, x_stride, wi, slots, tile_expert, gather_k, N, K);
  else if (kw == 2)
    moe_gemm_kernel<MT, 2><<<grid, block, smem, s>>>(o, out_stride, xi, x_stride, wi, slots, tile_expert, gather_k, N, K);
  else
    moe_gemm_kernel<MT, 1><<<grid, block, smem, s>>>(o, out_stride, xi, x_stride, wi, slots, tile_expert, gather_k, N, K);
}

void launch_moe_gemm(void* out, long out_stride, const void* x, long x_stride, const void* w, const int* slots,
                     const int* tile_expert, int tiles_cap, int tile, int gather_k, int N, int K, hipStream_t s) {
  if (tile == 16) moe_gemm_mt<1>(out, out_stride, x, x_stride, w, slots, tile_expert, tiles_cap, gather_k, N, K, s);
  else if (tile == 32) moe_gemm_mt<2>(out, out_stride, x, x_stride, w, slots, tile_expert, tiles_cap, gather_k, N, K, s);
  else moe_gemm_mt<4>(out, out_stride, x, x_stride, w, slots, tile_expert, tiles_cap, gather_k, N, K, s);
}

void launch_moe_combine(void* out, const void* y, const float* w, const int* pair_slot, int T, int k, int H,
                        hipStream_t s) {
  if (T <= 0) return;
  moe_combine_kernel<<<T, 256, 0, s>>>(static_cast<unsigned short*>(out), static_cast<const unsigned short*>(y), w,
                                       pair_slot, k, H);
}

void launch_moe_combine_partial(void* out, const float* ws, long slab, int S, const float* w, const int* pair_slot,
                                int T, int k, int H, hipStream_t s) {
  if (T <= 0) return;
  moe_combine_partial_kernel<<<T, 256, 0, s>>>(static_cast<unsigned short*>(out), ws, slab, S, w, pair_slot, k, H);
}

}  // namespace hipserve
