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

void launch_sample(long* out_tok, float* out_lp, const void* logits, bool is_bf16,
                   long stride, int rows, int V, const float* temperature,
                   const int* top_k, const float* top_p, const long* seeds,
                   const long* steps, hipStream_t s) {
  if (rows <= 0) return;
  if (is_bf16)
    launch_sample_t(out_tok, out_lp, static_cast<const unsigned short*>(logits), stride, rows, V, temperature, top_k, top_p, seeds, steps, s);
  else
    launch_sample_t(out_tok, out_lp, static_cast<const float*>(logits), stride, rows, V, temperature, top_k, top_p, seeds, steps, s);
}

}  // namespace hipserve
