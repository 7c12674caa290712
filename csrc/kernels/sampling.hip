// Fused token sampler: greedy / temperature / top-k / top-p with a
// counter-based RNG, one 1024-thread workgroup per logits row, no sort.
//
//   pass 1  online (max, sum exp, argmax) over the raw row  -> greedy + logprob
//   top-k   3-pass radix select (11/11/10 bits) on order-preserving float keys
//   top-p   the same radix passes over exp-mass histograms of the top-k survivors
//   sample  Gumbel-max race among survivors: argmax (x-m)/T - log(-log u_i),
//           u_i = hash(seed, step, i) — exact sampling from the filtered softmax
// Histograms live in LDS (2048 f32 bins, ds_add_f32); the row itself is re-read
// from L2/MALL each pass (it was just written by the LM-head GEMM).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int kSampThreads = 1024;
constexpr int kBins = 2048;

template <typename T>
HS_DEVICE float load_logit(const T* p, int i);
template <>
HS_DEVICE float load_logit<unsigned short>(const unsigned short* p, int i) { return bf16_to_f32(p[i]); }
template <>
HS_DEVICE float load_logit<float>(const float* p, int i) { return p[i]; }

HS_DEVICE unsigned int fkey(float f) {
  const unsigned int u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

HS_DEVICE float uniform01(unsigned long long seed, unsigned long long step, unsigned int i) {
  unsigned long long x = seed * 0x9E3779B97F4A7C15ull ^ (step + 0xD1B54A32D192ED03ull) * 0xBF58476D1CE4E5B9ull ^
                         ((unsigned long long)i + 1) * 0x94D049BB133111EBull;
  x ^= x >> 31; x *= 0x7FB5D329728EA185ull;
  x ^= x >> 27; x *= 0x81DADEF4BC2DD44Dull;
  x ^= x >> 33;
  return ((float)(unsigned int)(x >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

// Exclusive prefix over threads (block of 1024) of v; returns exclusive prefix,
// writes the block total into *total. scratch >= 17 floats.
HS_DEVICE float block_excl_scan(float v, float* scratch, float* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) scratch[wid] = inc;
  __syncthreads();
  if (wid == 0) {
    float w = lane < 16 ? scratch[lane] : 0.f;
    float wi = w;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float t = __shfl_up(wi, o, 64);
      if (lane >= o) wi += t;
    }
    if (lane < 16) scratch[lane] = wi - w;  // exclusive wave offsets
    if (lane == 15) scratch[16] = wi;
  }
  __syncthreads();
  const float ex = scratch[wid] + inc - v;
  *total = scratch[16];
  __syncthreads();
  return ex;
}

template <typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    long* __restrict__ out_tok, float* __restrict__ out_lp,
    const T* __restrict__ logits, long stride, int V,
    const float* __restrict__ temperature, const int* __restrict__ top_k,
    const float* __restrict__ top_p, const long* __restrict__ seeds,
    const long* __restrict__ steps) {
  __shared__ float hist[kBins];
  __shared__ float scratch[32];
  __shared__ float red_m[16], red_s[16];
  __shared__ int red_i[16];
  __shared__ unsigned int sh_prefix;
  __shared__ float sh_target;
  const int row = blockIdx.x;
  const T* x = logits + row * stride;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // ---- pass 1: online max / sumexp / argmax
  float m = -INFINITY, s = 0.f;
  int am = 0x7fffffff;
  for (int i = tid; i < V; i += kSampThreads) {
    const float v = load_logit<T>(x, i);
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; am = i; }
    else s += __expf(v - m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    if (m2 > m || (m2 == m && a2 < am)) am = a2;
    m = mn;
  }
  if (lane == 0) { red_m[wid] = m; red_s[wid] = s; red_i[wid] = am; }
  __syncthreads();
  if (wid == 0) {
    m = lane < 16 ? red_m[lane] : -INFINITY;
    s = lane < 16 ? red_s[lane] : 0.f;
    am = lane < 16 ? red_i[lane] : 0x7fffffff;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
      const int a2 = __shfl_xor(am, o, 64);
      const float mn = fmaxf(m, m2);
      s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
      if (m2 > m || (m2 == m && a2 < am)) am = a2;
      m = mn;
    }
    if (lane == 0) { red_m[0] = m; red_s[0] = s; red_i[0] = am; }
  }
  __syncthreads();
  const float rmax = red_m[0], rsum = red_s[0];
  const int ramax = red_i[0];
  __syncthreads();
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
  unsigned int floor_key = 0;  // survivors: fkey(x) >= floor_key

  // ---- radix threshold search; mode 0 = count (top-k), 1 = mass (top-p)
  for (int mode = 0; mode < 2; ++mode) {
    if (mode == 0 && !(k > 0 && k < V)) continue;
    if (mode == 1 && !(p < 1.f)) continue;
    unsigned int prefix = 0;
    float target = (mode == 0) ? (float)k : 0.f;
#pragma unroll 1
    for (int pass = 0; pass < 3; ++pass) {
      const int shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
      const int nbits = pass == 2 ? 10 : 11;
      const unsigned int bmask = (1u << nbits) - 1u;
      const int hi_shift = shift + nbits;  // bits above this pass are fixed by prefix
      for (int b = tid; b < kBins; b += kSampThreads) hist[b] = 0.f;
      __syncthreads();
      for (int i = tid; i < V; i += kSampThreads) {
        const float v = load_logit<T>(x, i);
        const unsigned int key = fkey(v);
        if (key < floor_key) continue;
        if (hi_shift < 32 && (key >> hi_shift) != (prefix >> hi_shift)) continue;
        const float w = (mode == 0) ? 1.f : __expf((v - rmax) * inv_t);
        atomicAdd(&hist[(key >> shift) & bmask], w);
      }
      __syncthreads();
      // positions run from the top bin downwards; thread t owns positions 2t, 2t+1
      const int nb = 1 << nbits;
      const int b0 = nb - 1 - 2 * tid, b1 = b0 - 1;
      const float h0 = (b0 >= 0) ? hist[b0] : 0.f;
      const float h1 = (b1 >= 0) ? hist[b1] : 0.f;
      float total;
      const float ex = block_excl_scan(h0 + h1, scratch, &total);
      if (mode == 1 && pass == 0) target = p * total;
      const float tgt = fminf(target, total);
      if (tid == 0) sh_prefix = 0xffffffffu;
      __syncthreads();
      if (h0 > 0.f && ex < tgt && tgt <= ex + h0) {
        sh_prefix = prefix | ((unsigned int)b0 << shift);
        sh_target = tgt - ex;
      } else if (h1 > 0.f && ex + h0 < tgt && tgt <= ex + h0 + h1) {
        sh_prefix = prefix | ((unsigned int)b1 << shift);
        sh_target = tgt - ex - h0;
      }
      __syncthreads();
      if (sh_prefix == 0xffffffffu) {  // numerically empty: this filter keeps all
        prefix = 0;
        break;
      }
      prefix = sh_prefix;
      target = sh_target;
      __syncthreads();
    }
    floor_key = prefix > floor_key ? prefix : floor_key;
  }

  // ---- Gumbel-max among survivors
  const unsigned long long seed = (unsigned long long)seeds[row];
  const unsigned long long step = (unsigned long long)steps[row];
  float best = -INFINITY;
  int bi = ramax;
  for (int i = tid; i < V; i += kSampThreads) {
    const float v = load_logit<T>(x, i);
    if (fkey(v) < floor_key) continue;
    const float u = uniform01(seed, step, (unsigned int)i);
    const float g = (v - rmax) * inv_t - __logf(-__logf(u));
    if (g > best) { best = g; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float b2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
  }
  if (lane == 0) { red_m[wid] = best; red_i[wid] = bi; }
  __syncthreads();
  if (tid == 0) {
    float bb = red_m[0];
    int ii = red_i[0];
    for (int w = 1; w < 16; ++w)
      if (red_m[w] > bb || (red_m[w] == bb && red_i[w] < ii)) { bb = red_m[w]; ii = red_i[w]; }
    out_tok[row] = ii;
    if (out_lp) out_lp[row] = (load_logit<T>(x, ii) - rmax) - __logf(rsum);
  }
}

void launch_sample(long* out_tok, float* out_lp, const void* logits, bool is_bf16,
                   long stride, int rows, int V, const float* temperature,
                   const int* top_k, const float* top_p, const long* seeds,
                   const long* steps, hipStream_t s) {
  if (rows <= 0) return;
  if (is_bf16)
    sample_kernel<unsigned short><<<rows, kSampThreads, 0, s>>>(out_tok, out_lp, static_cast<const unsigned short*>(logits), stride, V, temperature, top_k, top_p, seeds, steps);
  else
    sample_kernel<float><<<rows, kSampThreads, 0, s>>>(out_tok, out_lp, static_cast<const float*>(logits), stride, V, temperature, top_k, top_p, seeds, steps);
}

}  // namespace hipserve
