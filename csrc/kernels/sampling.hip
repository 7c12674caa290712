// Fused token sampler: greedy / temperature / top-k / top-p with a
// counter-based RNG, one 1024-thread workgroup per logits row, no sort.
//
// gfx950 design: the whole row is loaded ONCE (16-byte vector loads) into
// registers as packed bf16 (V = 128256 -> 63 VGPRs per lane at 1024 lanes), so
// every later pass is register + LDS work, never another HBM/L2 sweep:
//   pass 1  online (max, sum exp, argmax)                  -> greedy + logprob
//   top-k   4-ary bisection over the order-preserving 16-bit key space (count)
//   top-p   the same bisection over the exp-mass of the top-k survivors
//           (block reductions only: no LDS atomics, clustered logits would
//           serialise a histogram)
//   sample  Gumbel-max race among survivors: argmax (x-m)/T - log(-log u_i),
//           u_i = hash(row_key(seed, step), i) — an exact draw from the filtered
//           softmax; elements that provably cannot win skip the hash
#include "hipserve/common.h"
#include "hipserve/kernels.h"

#include <cstdio>
#include <cstdlib>

namespace hipserve {

constexpr int kSampThreads = 1024;
constexpr int kMcMinVocab = 8192;  // multi-CU path from this vocabulary size up
constexpr int kSampWaves = kSampThreads / 64;

HS_DEVICE unsigned int key16(unsigned short b) {  // order-preserving bf16 key
  return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}

// Counter-based RNG: the (seed, step) pair is folded into a 32-bit row key once;
// per element one 32-bit murmur3-style finaliser (2 multiplies) gives u in (0,1).
HS_DEVICE unsigned int row_key(unsigned long long seed, unsigned long long step) {
  unsigned long long x = seed * 0x9E3779B97F4A7C15ull ^ (step + 0xD1B54A32D192ED03ull) * 0xBF58476D1CE4E5B9ull;
  x ^= x >> 31; x *= 0x7FB5D329728EA185ull;
  x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull;
  x ^= x >> 33;
  return (unsigned int)x ^ (unsigned int)(x >> 32);
}

HS_DEVICE float uniform01(unsigned int key, unsigned int i) {
  unsigned int h = key ^ (i * 0x9E3779B9u + 0x7F4A7C15u);
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return ((float)(h >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// Make the register-resident row opaque between passes so the compiler does not
// CSE per-element conversions across passes (which would keep 128 extra floats
// live and spill).
template <int NV>
HS_DEVICE void opaque(u16x8 (&d)[NV]) {
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    u32x4 t = __builtin_bit_cast(u32x4, d[j]);
    asm volatile("" : "+v"(t));
    d[j] = __builtin_bit_cast(u16x8, t);
  }
}

template <typename T>
struct RowLoader;
template <>
struct RowLoader<unsigned short> {
  HS_DEVICE static void load8(const unsigned short* p, int idx, int V, u16x8& o) {
    if (idx + 8 <= V) {
      o = *reinterpret_cast<const u16x8*>(p + idx);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (idx + e < V) ? p[idx + e] : (unsigned short)0xFF80u;
    }
  }
};
template <>
struct RowLoader<float> {
  HS_DEVICE static void load8(const float* p, int idx, int V, u16x8& o) {
    if (idx + 8 <= V) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(p + idx);
      const f32x4 b = *reinterpret_cast<const f32x4*>(p + idx + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { o[e] = f32_to_bf16(a[e]); o[e + 4] = f32_to_bf16(b[e]); }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (idx + e < V) ? f32_to_bf16(p[idx + e]) : (unsigned short)0xFF80u;
    }
  }
};

template <int NV, typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    long* __restrict__ out_tok, float* __restrict__ out_lp,
    const T* __restrict__ logits, long stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const long* __restrict__ seeds,
    const long* __restrict__ steps) {
  // Elements [0, R) live in registers (NV 16-byte chunks per lane), the rest of
  // the row [R, V) in LDS (dynamic shared memory, 16-byte chunks).
  constexpr int R = kSampThreads * NV * 8;
  __shared__ float hist[3][kSampWaves];
  __shared__ float red_a[kSampWaves], red_b[kSampWaves];
  __shared__ int red_i[kSampWaves];
  extern __shared__ __attribute__((aligned(16))) u16x8 lrow[];
  const int row = blockIdx.x;
  const T* x = logits + row * stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nl = V > R ? (V - R + 7) / 8 : 0;  // LDS chunks

  u16x8 d[NV];  // packed bf16: 4 VGPRs per 16-byte chunk
#pragma unroll
  for (int j = 0; j < NV; ++j) RowLoader<T>::load8(x, 8 * (tid + kSampThreads * j), V, d[j]);
  for (int c = tid; c < nl; c += kSampThreads) {
    u16x8 t;
    RowLoader<T>::load8(x, R + 8 * c, V, t);
    lrow[c] = t;
  }
  __syncthreads();

  // visit(f): f(index, bf16 bits) for every element of this lane
  auto visit = [&](auto&& f) {
    opaque(d);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      const int base = 8 * (tid + kSampThreads * j);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f(base + e, (unsigned short)d[j][e]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    for (int c = tid; c < nl; c += kSampThreads) {
      const u16x8 t = lrow[c];
      const int base = R + 8 * c;
#pragma unroll
      for (int e = 0; e < 8; ++e) f(base + e, (unsigned short)t[e]);
    }
  };

  // ---- pass 1: max, argmax, then sum exp(x - max)
  float m = -INFINITY;
  int am = 0x7fffffff;
  visit([&](int idx, unsigned short b) {
    const float v = bf16_to_f32(b);
    if (v > m || (v == m && idx < am)) { m = v; am = idx; }
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
  }
  if (lane == 0) { red_a[wid] = m; red_i[wid] = am; }
  __syncthreads();
  m = red_a[0]; am = red_i[0];
#pragma unroll
  for (int w = 1; w < kSampWaves; ++w)
    if (red_a[w] > m || (red_a[w] == m && red_i[w] < am)) { m = red_a[w]; am = red_i[w]; }
  const float rmax = m;
  float s = 0.f;
  visit([&](int, unsigned short b) { s += __expf(bf16_to_f32(b) - rmax); });
  s = wave_sum(s);
  __syncthreads();
  if (lane == 0) red_b[wid] = s;
  __syncthreads();
  float rsum = 0.f;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) rsum += red_b[w];
  // an all-NaN row never updates (m, am): emit token 0, never an id past the
  // vocabulary (the next step would gather an embedding row out of bounds)
  const int ramax = am < V ? am : 0;

  const float temp = temperature[row];
  if (!(temp > 1e-5f)) {
    if (tid == 0) {
      out_tok[row] = ramax;
      if (out_lp) out_lp[row] = -__logf(rsum);
    }
    return;
  }
  const float inv_t = 1.f / temp;
  const int k = top_k[row];
  const float p = top_p[row];
  unsigned int floor_key = 0;  // survivors: key16 >= floor_key

  // Threshold search on the 16-bit key space: largest key T with
  // f(T) = sum_{key >= T} w >= target, w = 1 (top-k) or exp((x-m)/T) (top-p).
  // 4-ary bisection: 3 probes per register sweep, 8 sweeps, block sums only
  // (no LDS atomics: clustered logits would serialise a histogram).
  for (int mode = 0; mode < 2; ++mode) {
    if (mode == 0 && !(k > 0 && k < V)) continue;
    if (mode == 1 && !(p < 1.f)) continue;
    float target = (float)k;
    if (mode == 1) {  // nucleus mass among the (top-k) survivors
      float t = 0.f;
      visit([&](int idx, unsigned short b) {
        if (idx < V && key16(b) >= floor_key) t += __expf((bf16_to_f32(b) - rmax) * inv_t);
      });
      t = wave_sum(t);
      __syncthreads();
      if (lane == 0) red_b[wid] = t;
      __syncthreads();
      float tt = 0.f;
#pragma unroll
      for (int w = 0; w < kSampWaves; ++w) tt += red_b[w];
      target = p * tt;
    }
    unsigned int lo = floor_key, hi = 65536u;  // invariant: f(lo) >= target > f(hi)
#pragma unroll 1
    while (hi - lo > 1) {
      const unsigned int step = (hi - lo + 3) / 4;
      const unsigned int t1 = min(lo + step, hi - 1), t2 = min(lo + 2 * step, hi - 1),
                         t3 = min(lo + 3 * step, hi - 1);
      float a1 = 0.f, a2 = 0.f, a3 = 0.f;
      visit([&](int idx, unsigned short b) {
        const unsigned int key = key16(b);
        if (idx >= V || key < t1) return;
        const float w = (mode == 0) ? 1.f : __expf((bf16_to_f32(b) - rmax) * inv_t);
        a1 += w;
        a2 += key >= t2 ? w : 0.f;
        a3 += key >= t3 ? w : 0.f;
      });
      a1 = wave_sum(a1); a2 = wave_sum(a2); a3 = wave_sum(a3);
      __syncthreads();
      if (lane == 0) { hist[0][wid] = a1; hist[1][wid] = a2; hist[2][wid] = a3; }
      __syncthreads();
      float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int w = 0; w < kSampWaves; ++w) { s1 += hist[0][w]; s2 += hist[1][w]; s3 += hist[2][w]; }
      if (s3 >= target) lo = t3;
      else if (s2 >= target) { lo = t2; hi = t3; }
      else if (s1 >= target) { lo = t1; hi = t2; }
      else hi = t1;
    }
    floor_key = lo;
  }

  // ---- Gumbel-max among survivors
  const unsigned int rkey = row_key((unsigned long long)seeds[row], (unsigned long long)steps[row]);
  // max Gumbel noise for 24-bit u is 17.33 and the argmax token scores >= -2.85:
  // an element whose scaled logit is below -20.3 can never win -> no hash needed.
  constexpr float kNoWin = -20.3f;
  float best = -INFINITY;
  int bi = ramax;
  visit([&](int idx, unsigned short b) {
    if (idx >= V || key16(b) < floor_key) return;
    const float z = (bf16_to_f32(b) - rmax) * inv_t;
    if (z < kNoWin) return;
    const float u = uniform01(rkey, (unsigned int)idx);
    const float g = z - __logf(-__logf(u));
    if (g > best) { best = g; bi = idx; }
  });
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
  }
  if (lane == 0) { red_a[wid] = best; red_i[wid] = bi; }
  __syncthreads();
  if (tid == 0) {
    float bb = red_a[0];
    int ii = red_i[0];
    for (int w = 1; w < kSampWaves; ++w)
      if (red_a[w] > bb || (red_a[w] == bb && red_i[w] < ii)) { bb = red_a[w]; ii = red_i[w]; }
    out_tok[row] = ii;
    if (out_lp) {
      float xv;
      if constexpr (sizeof(T) == 2) xv = bf16_to_f32(reinterpret_cast<const unsigned short*>(x)[ii]);
      else xv = bf16_to_f32(f32_to_bf16(reinterpret_cast<const float*>(x)[ii]));
      out_lp[row] = (xv - rmax) - __logf(rsum);
    }
  }
}

constexpr size_t kSampLdsBudget = 142 * 1024;  // dynamic LDS for the row tail

template <typename T>
static void launch_sample_t(long* out_tok, float* out_lp, const T* logits, long stride, int rows,
                            int V, const float* temperature, const int* top_k, const float* top_p,
                            const long* seeds, const long* steps, hipStream_t s) {
  if (V <= kSampThreads * 32) {
    sample_kernel<4, T><<<rows, kSampThreads, 0, s>>>(out_tok, out_lp, logits, stride, V, temperature, top_k, top_p, seeds, steps);
    return;
  }
  constexpr int R = kSampThreads * 7 * 8;
  const size_t lds = V > R ? (size_t)((V - R + 7) / 8) * 16 : 0;
  if (lds > kSampLdsBudget) {
    fprintf(stderr, "hipserve sample: vocab %d exceeds the register+LDS row budget\n", V);
    abort();
  }
  sample_kernel<8, T><<<rows, kSampThreads, lds, s>>>(out_tok, out_lp, logits, stride, V, temperature, top_k, top_p, seeds, steps);
}

// ============================================================================
// Multi-CU sampler (large vocabularies). The single-workgroup kernel above is
// latency-bound per row (~170 us for a 128K-vocab top-p row whether B is 1 or
// 256: one CU walks the row ~12 times), so a row is split into 16K-element
// chunks, one 256-thread workgroup each, and the threshold searches become a
// two-level histogram of the same order-preserving 16-bit key:
//   coarse: key >> 11 (32 bins), accumulated in per-thread private LDS columns
//           ([bin][thread]: conflict-free, no atomics — clustered logits made
//           LDS atomics on 256 exponent bins serialise: 65 us per chunk);
//   fine:   key & 2047 (2048 bins) of the ONE selected coarse bin, LDS atomics
//           (lanes spread over 2048 addresses).
//   mc_stats   (chunk)  max / argmax / sum exp, coarse count + exp-mass
//   mc_coarse  (row)    combine -> greedy result; coarse bins of the thresholds
//   mc_fine    (chunk)  fine histograms inside the selected bin(s)
//   mc_thresh  (row)    exact 16-bit thresholds (a second fine round only when
//                       top-k and top-p are both active and the nucleus bin moved)
//   mc_gumbel  (chunk)  Gumbel-max among survivors, same hash as above
//   mc_final   (row)    argmax over chunks -> token, logprob
// Same semantics as sample_kernel (bit-identical draws given the thresholds;
// the threshold masses are summed in a different order).
constexpr int kMcThreads = 256;
constexpr int kMcVec = 4;                            // 16-byte pieces per thread
constexpr int kMcChunk = kMcThreads * kMcVec * 8;    // 8192 elements per workgroup
constexpr int kMcWaves = kMcThreads / 64;
constexpr int kCoarseBits = 5, kFineBits = 11;
constexpr int kCoarse = 1 << kCoarseBits, kFine = 1 << kFineBits;

struct McLayout {  // per-row workspace, in floats
  int C;
  HS_HOST_DEVICE long stats() const { return 0; }                          // [C][4] m, s1, massT, argmax
  HS_HOST_DEVICE long hcnt() const { return 4L * C; }                      // [C][32] uint
  HS_HOST_DEVICE long hmass() const { return hcnt() + (long)kCoarse * C; } // [C][32]
  HS_HOST_DEVICE long fcnt() const { return hmass() + (long)kCoarse * C; } // [C][2048] uint
  HS_HOST_DEVICE long fmassA() const { return fcnt() + (long)kFine * C; }  // [C][2048]
  HS_HOST_DEVICE long fmassB() const { return fmassA() + (long)kFine * C; }// [C][2048]
  HS_HOST_DEVICE long best() const { return fmassB() + (long)kFine * C; }  // [C][2] g, idx
  HS_HOST_DEVICE long state() const { return best() + 2L * C; }            // [32]
  HS_HOST_DEVICE long cmass() const { return state() + 32; }               // [32] combined coarse mass
  HS_HOST_DEVICE long size() const { return (cmass() + kCoarse + 3) & ~3L; }  // 16-byte aligned rows
};
enum { ST_DONE = 0, ST_M, ST_RSUM, ST_INVT, ST_HK, ST_KREM, ST_HP0, ST_FLOOR, ST_BINA, ST_BINB, ST_NEED2,
       ST_TARGET };

template <typename T>
HS_DEVICE void mc_load(const T* __restrict__ row, int chunk, int V, u16x8 (&d)[kMcVec]) {
#pragma unroll
  for (int j = 0; j < kMcVec; ++j)
    RowLoader<T>::load8(row, chunk * kMcChunk + 8 * (threadIdx.x + kMcThreads * j), V, d[j]);
}

HS_DEVICE int mc_idx(int chunk, int j, int e) { return chunk * kMcChunk + 8 * (threadIdx.x + kMcThreads * j) + e; }

template <typename T>
__global__ __launch_bounds__(kMcThreads) void mc_stats_kernel(const T* __restrict__ logits, long stride, int V,
                                                             const float* __restrict__ temperature,
                                                             const int* __restrict__ top_k,
                                                             const float* __restrict__ top_p,
                                                             float* __restrict__ ws, int C) {
  const int chunk = blockIdx.x, row = blockIdx.y;
  const McLayout L{C};
  float* w = ws + (long)row * L.size();
  __shared__ unsigned int cntp[kCoarse][kMcThreads];  // [bin][thread]: bank = thread
  __shared__ float massp[kCoarse][kMcThreads];
  __shared__ float red_a[kMcWaves];
  __shared__ int red_i[kMcWaves];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  u16x8 d[kMcVec];
  mc_load(logits + (long)row * stride, chunk, V, d);
  float m = -INFINITY;
  int am = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < kMcVec; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = mc_idx(chunk, j, e);
      const float v = bf16_to_f32(d[j][e]);
      if (idx < V && (v > m || (v == m && idx < am))) { m = v; am = idx; }
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    if (m2 > m || (m2 == m && a2 < am)) { m = m2; am = a2; }
  }
  if (lane == 0) { red_a[wid] = m; red_i[wid] = am; }
  __syncthreads();
  m = red_a[0]; am = red_i[0];
#pragma unroll
  for (int k = 1; k < kMcWaves; ++k)
    if (red_a[k] > m || (red_a[k] == m && red_i[k] < am)) { m = red_a[k]; am = red_i[k]; }
  const float temp = temperature[row];
  const bool sampling = temp > 1e-5f;
  const int k = top_k[row];
  const bool hist_k = sampling && k > 0 && k < V, hist_p = sampling && top_p[row] < 1.f;
  const float inv_t = sampling ? 1.f / temp : 0.f;
  if (hist_k || hist_p) {
#pragma unroll
    for (int b = 0; b < kCoarse; ++b) { cntp[b][tid] = 0u; massp[b][tid] = 0.f; }
  }
  float s1 = 0.f, sT = 0.f;
#pragma unroll
  for (int j = 0; j < kMcVec; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (mc_idx(chunk, j, e) >= V) continue;
      const float v = bf16_to_f32(d[j][e]);
      s1 += __expf(v - m);
      if (sampling) {
        const float wt = __expf((v - m) * inv_t);
        sT += wt;
        const int b = key16(d[j][e]) >> kFineBits;
        if (hist_k) cntp[b][tid] += 1u;
        if (hist_p) massp[b][tid] += wt;
      }
    }
  s1 = wave_sum(s1);
  sT = wave_sum(sT);
  __syncthreads();
  if (lane == 0) red_a[wid] = s1;
  __syncthreads();
  float S1 = 0.f;
#pragma unroll
  for (int q = 0; q < kMcWaves; ++q) S1 += red_a[q];
  __syncthreads();
  if (lane == 0) red_a[wid] = sT;
  __syncthreads();
  float ST = 0.f;
#pragma unroll
  for (int q = 0; q < kMcWaves; ++q) ST += red_a[q];
  if (tid == 0) {
    float* st = w + L.stats() + 4 * chunk;
    st[0] = m;
    st[1] = S1;
    st[2] = ST;
    st[3] = __int_as_float(am);
  }
  if (hist_k || hist_p) {
    // bin b = tid >> 3 summed by 8 threads over 32 thread columns each
    const int b = tid >> 3, part = tid & 7;
    unsigned int c = 0;
    float ms = 0.f;
#pragma unroll
    for (int i = 0; i < kMcThreads / 8; ++i) {
      const int col = part * (kMcThreads / 8) + i;
      c += cntp[b][col];
      ms += massp[b][col];
    }
#pragma unroll
    for (int o = 4; o > 0; o >>= 1) {
      c += __shfl_xor(c, o, 64);
      ms += __shfl_xor(ms, o, 64);
    }
    if (part == 0) {
      reinterpret_cast<unsigned int*>(w + L.hcnt())[kCoarse * chunk + b] = c;
      w[L.hmass() + kCoarse * chunk + b] = ms;
    }
  }
}

// One workgroup per row: combine the chunk statistics; greedy rows finish here.
__global__ __launch_bounds__(64) void mc_coarse_kernel(long* __restrict__ out_tok, float* __restrict__ out_lp,
                                                       const float* __restrict__ temperature,
                                                       const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                       int V, float* __restrict__ ws, int C) {
  const int row = blockIdx.x;
  const McLayout L{C};
  float* w = ws + (long)row * L.size();
  float* st = w + L.state();
  __shared__ unsigned int cnt[kCoarse];
  __shared__ float mass[kCoarse];
  // lanes 0..C-1 hold the chunk stats; wave reductions for max / argmax / rsum
  const int lane = threadIdx.x;
  float m = -INFINITY, s1 = 0.f;
  int a = 0x7fffffff;
  if (lane < C) {
    m = w[L.stats() + 4 * lane];
    s1 = w[L.stats() + 4 * lane + 1];
    a = __float_as_int(w[L.stats() + 4 * lane + 3]);
  }
  float M = m;
  int A = a;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(M, o, 64);
    const int a2 = __shfl_xor(A, o, 64);
    if (m2 > M || (m2 == M && a2 < A)) { M = m2; A = a2; }
  }
  const float R = wave_sum(lane < C ? s1 * __expf(m - M) : 0.f);
  const float temp = temperature[row];
  if (!(temp > 1e-5f)) {
    if (lane == 0) {
      out_tok[row] = A < V ? A : 0;  // all-NaN row: token 0, never an id past V
      if (out_lp) out_lp[row] = -__logf(R);
      st[ST_DONE] = 1.f;
    }
    return;
  }
  const float inv_t = 1.f / temp;
  const int k = top_k[row];
  const float p = top_p[row];
  const bool use_k = k > 0 && k < V, use_p = p < 1.f;
  if (lane < kCoarse) {
    unsigned int c = 0;
    float ms = 0.f;
    for (int q = 0; q < C; ++q) {
      if (use_k) c += reinterpret_cast<const unsigned int*>(w + L.hcnt())[kCoarse * q + lane];
      if (use_p) ms += w[L.hmass() + kCoarse * q + lane] * __expf((w[L.stats() + 4 * q] - M) * inv_t);
    }
    cnt[lane] = c;
    mass[lane] = ms;
    w[L.cmass() + lane] = ms;
  }
  __syncthreads();
  if (lane != 0) return;
  int hk = -1, krem = 0;
  if (use_k) {
    unsigned int acc = 0;
    for (int b = kCoarse - 1; b >= 0; --b) {
      if (acc + cnt[b] >= (unsigned int)k) { hk = b; krem = k - (int)acc; break; }
      acc += cnt[b];
    }
  }
  int hp0 = -1;
  if (use_p) {
    float tot = 0.f;
    for (int b = kCoarse - 1; b >= max(hk, 0); --b) tot += mass[b];
    const float target = p * tot;  // exact without top-k, an upper bound with it
    float acc = 0.f;
    for (int b = kCoarse - 1; b >= max(hk, 0); --b) {
      acc += mass[b];
      if (acc >= target) { hp0 = b; break; }
    }
    if (hp0 < 0) hp0 = max(hk, 0);
  }
  st[ST_DONE] = 0.f;
  st[ST_M] = M;
  st[ST_RSUM] = R;
  st[ST_INVT] = inv_t;
  st[ST_HK] = (float)hk;
  st[ST_KREM] = (float)krem;
  st[ST_HP0] = (float)hp0;
  st[ST_BINA] = (float)(use_k ? hk : hp0);
  st[ST_BINB] = (float)(use_k && use_p && hp0 != hk ? hp0 : -1);
  st[ST_NEED2] = 0.f;
  st[ST_FLOOR] = 0.f;
}

// Fine histograms (key & 2047) of the bins named in the row state: round 0 ->
// bin A (count + mass) and bin B (mass); round 1 -> bin ST_BINB (mass) for rows
// that flagged ST_NEED2.
template <typename T>
__global__ __launch_bounds__(kMcThreads) void mc_fine_kernel(const T* __restrict__ logits, long stride, int V,
                                                            float* __restrict__ ws, int C, int round) {
  const int chunk = blockIdx.x, row = blockIdx.y;
  const McLayout L{C};
  float* w = ws + (long)row * L.size();
  const float* st = w + L.state();
  if (st[ST_DONE] != 0.f) return;
  if (round == 1 && st[ST_NEED2] == 0.f) return;
  const int binA = round == 0 ? (int)st[ST_BINA] : -1;
  const int binB = (int)st[ST_BINB];
  if (binA < 0 && binB < 0) return;
  __shared__ unsigned int fc[kFine];
  __shared__ float fa[kFine], fb[kFine];
  for (int i = threadIdx.x; i < kFine; i += kMcThreads) { fc[i] = 0u; fa[i] = 0.f; fb[i] = 0.f; }
  u16x8 d[kMcVec];
  mc_load(logits + (long)row * stride, chunk, V, d);
  const float m = w[L.stats() + 4 * chunk];
  const float inv_t = st[ST_INVT];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kMcVec; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (mc_idx(chunk, j, e) >= V) continue;
      const unsigned int key = key16(d[j][e]);
      const int hi = key >> kFineBits, lo = key & (kFine - 1);
      if (hi != binA && hi != binB) continue;
      const float wt = __expf((bf16_to_f32(d[j][e]) - m) * inv_t);
      if (hi == binA) {
        atomicAdd(&fc[lo], 1u);
        atomicAdd(&fa[lo], wt);
      }
      if (hi == binB) atomicAdd(&fb[lo], wt);
    }
  __syncthreads();
  for (int b = threadIdx.x; b < kFine; b += kMcThreads) {
    if (round == 0) {
      reinterpret_cast<unsigned int*>(w + L.fcnt())[kFine * chunk + b] = fc[b];
      w[L.fmassA() + kFine * chunk + b] = fa[b];
    }
    w[L.fmassB() + kFine * chunk + b] = fb[b];
  }
}

// Largest l >= lmin with base + sum_{l' >= l, l' >= lmin} v[l'] >= target over the
// 2048 fine bins (LDS), block-parallel: 8 bins per thread, suffix scan of the
// per-thread sums. Returns lmin when the target is never reached (rounding).
template <typename V>
HS_DEVICE int suffix_find(const V* v, V base, V target, int lmin, V* scan, int* res) {
  const int t = threadIdx.x;  // 256 threads, bins [8t, 8t + 8)
  V seg = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int l = 8 * t + i;
    if (l >= lmin) seg += v[l];
  }
  scan[t] = seg;
  if (t == 0) *res = lmin;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive suffix scan
    const V add = t + o < 256 ? scan[t + o] : (V)0;
    __syncthreads();
    scan[t] += add;
    __syncthreads();
  }
  const V above = base + (t + 1 < 256 ? scan[t + 1] : (V)0);
  if (above < target && above + seg >= target) {
    V acc = above;
    for (int i = 7; i >= 0; --i) {
      const int l = 8 * t + i;
      if (l < lmin) break;
      acc += v[l];
      if (acc >= target) { *res = l; break; }
    }
  }
  __syncthreads();
  const int r = *res;
  __syncthreads();
  return r;
}

// Exact 16-bit thresholds. round 0: top-k, then top-p (flags ST_NEED2 when the
// nucleus crosses into a coarse bin whose fine histogram was not collected);
// round 1: finish the flagged rows.
__global__ __launch_bounds__(256) void mc_thresh_kernel(const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                        int V, float* __restrict__ ws, int C, int round) {
  const int row = blockIdx.x;
  const McLayout L{C};
  float* w = ws + (long)row * L.size();
  float* st = w + L.state();
  if (st[ST_DONE] != 0.f) return;
  if (round == 1 && st[ST_NEED2] == 0.f) return;
  const int k = top_k[row];
  const float p = top_p[row];
  const bool use_k = k > 0 && k < V, use_p = p < 1.f;
  if (!use_k && !use_p) {  // plain temperature sampling: no threshold
    if (threadIdx.x == 0) st[ST_FLOOR] = 0.f;
    return;
  }
  __shared__ unsigned int fc[kFine];
  __shared__ float fa[kFine], fb[kFine];
  __shared__ float fscan[256];
  __shared__ unsigned int uscan[256];
  __shared__ float scale[64];
  __shared__ int res;
  const float M = st[ST_M], inv_t = st[ST_INVT];
  if (threadIdx.x < C) scale[threadIdx.x] = __expf((w[L.stats() + 4 * threadIdx.x] - M) * inv_t);
  __syncthreads();
  const bool needA = round == 0, needB = (int)st[ST_BINB] >= 0;
  {
    // thread t combines bins [8t, 8t + 8) over the chunks with 16-byte loads
    const int b0 = 8 * threadIdx.x;
    u32x4 c0 = {0u, 0u, 0u, 0u}, c1 = {0u, 0u, 0u, 0u};
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, e0 = a0, e1 = a0;
#pragma unroll 4
    for (int q = 0; q < C; ++q) {
      const float sc = scale[q];
      if (needA) {
        if (use_k) {
          const u32x4* cp = reinterpret_cast<const u32x4*>(w + L.fcnt() + (long)kFine * q + b0);
          c0 += cp[0];
          c1 += cp[1];
        }
        const f32x4* ap = reinterpret_cast<const f32x4*>(w + L.fmassA() + (long)kFine * q + b0);
        a0 += ap[0] * sc;
        a1 += ap[1] * sc;
      }
      if (needB) {
        const f32x4* bp = reinterpret_cast<const f32x4*>(w + L.fmassB() + (long)kFine * q + b0);
        e0 += bp[0] * sc;
        e1 += bp[1] * sc;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fc[b0 + i] = c0[i]; fc[b0 + 4 + i] = c1[i];
      fa[b0 + i] = a0[i]; fa[b0 + 4 + i] = a1[i];
      fb[b0 + i] = e0[i]; fb[b0 + 4 + i] = e1[i];
    }
  }
  __syncthreads();
  const float* cm = w + L.cmass();
  const int hk = (int)st[ST_HK];
  if (round == 1) {  // the nucleus bin ST_BINB, target stored by round 0
    const int hp = (int)st[ST_BINB];
    float acc = 0.f;
    for (int b = kCoarse - 1; b > hp; --b) acc += cm[b];
    const int lo = suffix_find<float>(fb, acc, st[ST_TARGET], 0, fscan, &res);
    if (threadIdx.x == 0) st[ST_FLOOR] = (float)((hp << kFineBits) | lo);
    return;
  }
  int floor_k = 0, lo_k = 0;
  if (use_k) {
    lo_k = suffix_find<unsigned int>(fc, 0u, (unsigned int)st[ST_KREM], 0, uscan, &res);
    floor_k = (hk << kFineBits) | lo_k;
  }
  int floor = floor_k;
  if (use_p) {
    // survivor mass: coarse bins above hb whole, bin hk only from lo_k (top-k)
    const int hb = use_k ? hk : 0;
    float in_hk = 0.f;
    if (use_k) {
      // survivor mass inside bin hk: sum of fa[l] for l >= lo_k (block reduction)
      float part = 0.f;
      for (int l = threadIdx.x; l < kFine; l += 256)
        if (l >= lo_k) part += fa[l];
      part = block_sum(part, fscan);
      in_hk = part;
    }
    float tot = in_hk;
    for (int b = kCoarse - 1; b >= (use_k ? hb + 1 : 0); --b) tot += cm[b];
    const float target = p * tot;
    // coarse bin hp of the nucleus threshold; acc = survivor mass above it
    float acc = 0.f;
    int hp = hb;
    for (int b = kCoarse - 1; b > hb; --b) {
      if (acc + cm[b] >= target) { hp = b; break; }
      acc += cm[b];
    }
    const float* fine = nullptr;
    int lmin = 0;
    if (use_k && hp == hk) { fine = fa; lmin = lo_k; }
    else if (!use_k && hp == (int)st[ST_BINA]) fine = fa;
    else if (use_k && hp == (int)st[ST_BINB]) fine = fb;
    if (fine != nullptr) {
      const int lo = suffix_find<float>(fine, acc, target, lmin, fscan, &res);
      floor = (hp << kFineBits) | lo;
    } else if (threadIdx.x == 0) {  // the nucleus bin has no fine histogram yet: second round
      st[ST_NEED2] = 1.f;
      st[ST_BINB] = (float)hp;
      st[ST_TARGET] = target;
      floor = hp << kFineBits;
    }
  }
  if (threadIdx.x == 0) st[ST_FLOOR] = (float)floor;
}

template <typename T>
__global__ __launch_bounds__(kMcThreads) void mc_gumbel_kernel(const T* __restrict__ logits, long stride, int V,
                                                              const long* __restrict__ seeds,
                                                              const long* __restrict__ steps, float* __restrict__ ws,
                                                              int C) {
  const int chunk = blockIdx.x, row = blockIdx.y;
  const McLayout L{C};
  float* w = ws + (long)row * L.size();
  const float* st = w + L.state();
  if (st[ST_DONE] != 0.f) return;
  __shared__ float red_a[kMcWaves];
  __shared__ int red_i[kMcWaves];
  u16x8 d[kMcVec];
  mc_load(logits + (long)row * stride, chunk, V, d);
  const float M = st[ST_M], inv_t = st[ST_INVT];
  const unsigned int floor_key = (unsigned int)st[ST_FLOOR];
  const unsigned int rkey = row_key((unsigned long long)seeds[row], (unsigned long long)steps[row]);
  constexpr float kNoWin = -20.3f;
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < kMcVec; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = mc_idx(chunk, j, e);
      if (idx >= V || key16(d[j][e]) < floor_key) continue;
      const float z = (bf16_to_f32(d[j][e]) - M) * inv_t;
      if (z < kNoWin) continue;
      const float u = uniform01(rkey, (unsigned int)idx);
      const float g = z - __logf(-__logf(u));
      if (g > best || (g == best && idx < bi)) { best = g; bi = idx; }
    }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
  }
  if (lane == 0) { red_a[wid] = best; red_i[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < kMcWaves; ++q)
      if (red_a[q] > best || (red_a[q] == best && red_i[q] < bi)) { best = red_a[q]; bi = red_i[q]; }
    w[L.best() + 2 * chunk] = best;
    w[L.best() + 2 * chunk + 1] = __int_as_float(bi);
  }
}

template <typename T>
__global__ __launch_bounds__(64) void mc_final_kernel(long* __restrict__ out_tok, float* __restrict__ out_lp,
                                                      const T* __restrict__ logits, long stride, int V,
                                                      const float* __restrict__ ws, int C) {
  const int row = blockIdx.x;
  const McLayout L{C};
  const float* w = ws + (long)row * L.size();
  const float* st = w + L.state();
  if (st[ST_DONE] != 0.f || threadIdx.x != 0) return;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int c = 0; c < C; ++c) {
    const float g = w[L.best() + 2 * c];
    const int i = __float_as_int(w[L.best() + 2 * c + 1]);
    if (g > best || (g == best && i < bi)) { best = g; bi = i; }
  }
  if (!(bi >= 0 && bi < V)) bi = 0;  // no survivor (NaN row): token 0
  out_tok[row] = bi;
  if (out_lp) {
    float xv;
    if constexpr (sizeof(T) == 2) xv = bf16_to_f32(reinterpret_cast<const unsigned short*>(logits + (long)row * stride)[bi]);
    else xv = bf16_to_f32(f32_to_bf16(reinterpret_cast<const float*>(logits + (long)row * stride)[bi]));
    out_lp[row] = (xv - st[ST_M]) - __logf(st[ST_RSUM]);
  }
}

size_t sample_workspace_floats(int rows, int V) {
  if (V < kMcMinVocab) return 0;
  const McLayout L{(V + kMcChunk - 1) / kMcChunk};
  return (size_t)rows * L.size();
}

template <typename T>
static void launch_sample_mc(long* out_tok, float* out_lp, const T* logits, long stride, int rows, int V,
                             const float* temperature, const int* top_k, const float* top_p, const long* seeds,
                             const long* steps, float* ws, bool two_rounds, hipStream_t s) {
  const int C = (V + kMcChunk - 1) / kMcChunk;
  const dim3 cg(C, rows);
  mc_stats_kernel<T><<<cg, kMcThreads, 0, s>>>(logits, stride, V, temperature, top_k, top_p, ws, C);
  mc_coarse_kernel<<<rows, 64, 0, s>>>(out_tok, out_lp, temperature, top_k, top_p, V, ws, C);
  mc_fine_kernel<T><<<cg, kMcThreads, 0, s>>>(logits, stride, V, ws, C, 0);
  mc_thresh_kernel<<<rows, 256, 0, s>>>(top_k, top_p, V, ws, C, 0);
  if (two_rounds) {  // rows with top-k AND top-p may need a second fine round; else it is a no-op
    mc_fine_kernel<T><<<cg, kMcThreads, 0, s>>>(logits, stride, V, ws, C, 1);
    mc_thresh_kernel<<<rows, 256, 0, s>>>(top_k, top_p, V, ws, C, 1);
  }
  mc_gumbel_kernel<T><<<cg, kMcThreads, 0, s>>>(logits, stride, V, seeds, steps, ws, C);
  mc_final_kernel<T><<<rows, 64, 0, s>>>(out_tok, out_lp, logits, stride, V, ws, C);
}

void launch_sample(long* out_tok, float* out_lp, const void* logits, bool is_bf16,
                   long stride, int rows, int V, const float* temperature,
                   const int* top_k, const float* top_p, const long* seeds,
                   const long* steps, float* ws, hipStream_t s, bool two_rounds) {
  if (rows <= 0) return;
  if (ws != nullptr && V >= kMcMinVocab) {
    if (is_bf16)
      launch_sample_mc(out_tok, out_lp, static_cast<const unsigned short*>(logits), stride, rows, V, temperature,
                       top_k, top_p, seeds, steps, ws, two_rounds, s);
    else
      launch_sample_mc(out_tok, out_lp, static_cast<const float*>(logits), stride, rows, V, temperature, top_k,
                       top_p, seeds, steps, ws, two_rounds, s);
    return;
  }
  if (is_bf16)
    launch_sample_t(out_tok, out_lp, static_cast<const unsigned short*>(logits), stride, rows, V, temperature, top_k, top_p, seeds, steps, s);
  else
    launch_sample_t(out_tok, out_lp, static_cast<const float*>(logits), stride, rows, V, temperature, top_k, top_p, seeds, steps, s);
}

}  // namespace hipserve
