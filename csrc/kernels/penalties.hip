// OpenAI sampling extras on the device: presence / frequency /
// repetition penalties and top-n log-probabilities, graph-capturable so a batch
// with one penalised or logprobs request stays on the decode hipGraph + one-step
// lookahead path (the sampled tokens never visit the host between steps).
//
// State per penalised sequence (a "slot", assigned by the runner):
//   counts[slot][V]  int32  occurrences of each token in the GENERATED tokens
//   seen[slot][V/32] bits   token occurred in the prompt or the generated tokens
// Semantics (vLLM / OpenAI): repetition penalty on prompt+output tokens first
// (l > 0 ? l / r : l * r), then l -= frequency * count + presence * (count > 0).
//   penalty_init    (re)build a slot from prompt + already generated ids (the
//                   step that samples a sequence's first token, or a recompute)
//   penalty_apply   logits rows in place, rows with slot < 0 untouched
//   penalty_update  count the tokens sampled this step (after the sampler)
//   top_logprobs    per row with n > 0: n largest log-softmax entries (radix
//                   select on the order-preserving 16-bit key of the bf16-rounded
//                   value, then every candidate in the selected bin up to 64 is
//                   ordered by its exact value, ties -> lowest id). The runner calls it
//                   BEFORE penalty_apply: top-n log-probs are of the raw model
//                   distribution (vLLM's default raw-logprobs mode).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

HS_DEVICE float ld_logit(const unsigned short* p, long i) { return bf16_to_f32(p[i]); }
HS_DEVICE float ld_logit(const float* p, long i) { return p[i]; }
HS_DEVICE void st_logit(unsigned short* p, long i, float v) { p[i] = f32_to_bf16(v); }
HS_DEVICE void st_logit(float* p, long i, float v) { p[i] = v; }

HS_DEVICE bool pen_active(float pres, float freq, float rep) {
  return pres != 0.f || freq != 0.f || rep != 1.f;
}

// grid (ceil(V / (256*8)), rows): 8 consecutive vocab entries per thread
template <typename T>
__global__ __launch_bounds__(256) void penalty_apply_kernel(T* __restrict__ logits, long stride, int V,
                                                            const int* __restrict__ slot,
                                                            const float* __restrict__ pres,
                                                            const float* __restrict__ freq,
                                                            const float* __restrict__ rep,
                                                            const int* __restrict__ counts,
                                                            const unsigned int* __restrict__ seen, int words) {
  const int r = blockIdx.y;
  const int s = slot[r];
  if (s < 0) return;
  const float pp = pres[r], fp = freq[r], rp = rep[r];
  if (!pen_active(pp, fp, rp)) return;
  const int v0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (v0 >= V) return;
  T* row = logits + (long)r * stride;
  const int* cnt = counts + (long)s * V;
  const unsigned int w = seen[(long)s * words + (v0 >> 5)];  // 8 | 32: one word covers the 8
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int v = v0 + e;
    if (v >= V) break;
    float l = ld_logit(row, v);
    if ((w >> (v & 31)) & 1u) l = l > 0.f ? l / rp : l * rp;
    const int c = cnt[v];
    l -= fp * (float)c + (c > 0 ? pp : 0.f);
    st_logit(row, v, l);
  }
}

// one thread per sampled row (rows never share a slot)
__global__ __launch_bounds__(256) void penalty_update_kernel(const long* __restrict__ tok,
                                                             const int* __restrict__ slot, int n,
                                                             int* __restrict__ counts,
                                                             unsigned int* __restrict__ seen, int V, int words) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const int s = slot[r];
  const long t = tok[r];
  if (s < 0 || t < 0 || t >= V) return;
  counts[(long)s * V + t] += 1;
  seen[(long)s * words + (t >> 5)] |= 1u << (t & 31);
}

// one block per initialised slot: zero it, then add the prompt (seen only) and
// the already generated tokens (count + seen). ids of slot j: toks[off[j] .. off[j+1]),
// the first n_prompt[j] of them are prompt ids.
__global__ __launch_bounds__(256) void penalty_init_kernel(int* __restrict__ counts, unsigned int* __restrict__ seen,
                                                           int V, int words, const int* __restrict__ slots,
                                                           const int* __restrict__ off,
                                                           const int* __restrict__ n_prompt,
                                                           const int* __restrict__ toks) {
  const int j = blockIdx.x;
  const int s = slots[j];
  int* cnt = counts + (long)s * V;
  unsigned int* sn = seen + (long)s * words;
  for (int v = threadIdx.x; v < V; v += 256) cnt[v] = 0;
  for (int w = threadIdx.x; w < words; w += 256) sn[w] = 0u;
  __syncthreads();
  const int a = off[j], b = off[j + 1], np = n_prompt[j];
  for (int i = a + threadIdx.x; i < b; i += 256) {
    const int t = toks[i];
    if (t < 0 || t >= V) continue;
    atomicOr(&sn[t >> 5], 1u << (t & 31));
    if (i - a >= np) atomicAdd(&cnt[t], 1);
  }
}

// ------------------------------------------------------------------ top-n logprobs
constexpr int kTopT = 1024;

HS_DEVICE unsigned int key16f(float f) {  // order-preserving key of the bf16-rounded value
  const unsigned short b = f32_to_bf16(f);
  return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}

template <typename T>
__global__ __launch_bounds__(kTopT) void top_logprobs_kernel(const T* __restrict__ logits, long stride, int V,
                                                             const int* __restrict__ nreq, int* __restrict__ out_ids,
                                                             float* __restrict__ out_lp, int K) {
  __shared__ float red[16];
  __shared__ unsigned int hist[256];
  __shared__ unsigned int s_sel[3];  // threshold key, count strictly above, remaining ties to take
  __shared__ int s_tie_scan[kTopT];
  __shared__ float c_val[64];
  __shared__ int c_idx[64];
  __shared__ unsigned int c_n;
  const int r = blockIdx.x, t = threadIdx.x;
  const int n = min(nreq[r], K);
  if (n <= 0) {
    if (t < K) {
      out_ids[(long)r * K + t] = -1;
      out_lp[(long)r * K + t] = -INFINITY;
    }
    return;
  }
  const T* row = logits + (long)r * stride;
  // 1. log-sum-exp
  float m = -INFINITY;
  for (int v = t; v < V; v += kTopT) m = fmaxf(m, ld_logit(row, v));
  m = block_max(m, red);
  float se = 0.f;
  for (int v = t; v < V; v += kTopT) se += __expf(ld_logit(row, v) - m);
  se = block_sum(se, red);
  const float lse = m + __logf(se);
  // 2. radix select of the n-th largest 16-bit key: high byte, then low byte
  unsigned int prefix = 0, above = 0;  // keys with the selected high byte; count of keys above the bin
  for (int round = 0; round < 2; ++round) {
    for (int i = t; i < 256; i += kTopT) hist[i] = 0;
    __syncthreads();
    for (int v = t; v < V; v += kTopT) {
      const unsigned int k = key16f(ld_logit(row, v));
      if (round == 0) atomicAdd(&hist[k >> 8], 1u);
      else if ((k >> 8) == prefix) atomicAdd(&hist[k & 255], 1u);
    }
    __syncthreads();
    if (t == 0) {
      unsigned int acc = above;
      int b = 255;
      for (; b > 0; --b) {
        if (acc + hist[b] >= (unsigned)n) break;
        acc += hist[b];
      }
      s_sel[0] = round == 0 ? (unsigned)b : (prefix << 8) | (unsigned)b;
      s_sel[1] = acc;  // strictly above the selected bin
    }
    __syncthreads();
    if (round == 0) {
      prefix = s_sel[0];
      above = s_sel[1];
    }
    __syncthreads();
  }
  const unsigned int kth = s_sel[0];
  const unsigned int n_above = s_sel[1];
  // every key in the selected bin is a candidate (the bin rounds fp32 logits to bf16,
  // so the true n-th largest may sit anywhere in it) while they fit the 64 slots;
  // past that the lowest-index ones — the one documented bound on exactness (more than
  // 64 logits within one bf16 ulp of the n-th largest; hipserve/ops/reference.py)
  const int take_ties = 64 - (int)n_above;
  // 3. collect: every key > kth, then the lowest-index ties (contiguous chunks per
  //    thread + a block scan give each tie its global index rank)
  if (t == 0) c_n = 0;
  const int chunk = (V + kTopT - 1) / kTopT;
  const int lo = t * chunk, hi = min(V, lo + chunk);
  int nt = 0;
  for (int v = lo; v < hi; ++v) nt += key16f(ld_logit(row, v)) == kth;
  s_tie_scan[t] = nt;
  __syncthreads();
  for (int d = 1; d < kTopT; d <<= 1) {  // inclusive scan
    const int x = t >= d ? s_tie_scan[t - d] : 0;
    __syncthreads();
    s_tie_scan[t] += x;
    __syncthreads();
  }
  int rank = s_tie_scan[t] - nt;
  for (int v = lo; v < hi; ++v) {
    const float l = ld_logit(row, v);
    const unsigned int k = key16f(l);
    bool take = k > kth;
    if (k == kth) take = rank++ < take_ties;
    if (take) {
      const unsigned int p = atomicAdd(&c_n, 1u);
      if (p < 64) {
        c_val[p] = l;
        c_idx[p] = v;
      }
    }
  }
  __syncthreads();
  // 4. order (exact value desc, id asc) and write the first n
  if (t == 0) {
    const int cn = min((int)c_n, 64);
    for (int i = 1; i < cn; ++i) {
      const float k = c_val[i];
      const int x = c_idx[i];
      int j = i - 1;
      while (j >= 0 && (c_val[j] < k || (c_val[j] == k && c_idx[j] > x))) {
        c_val[j + 1] = c_val[j];
        c_idx[j + 1] = c_idx[j];
        --j;
      }
      c_val[j + 1] = k;
      c_idx[j + 1] = x;
    }
    for (int i = 0; i < K; ++i) {
      const bool ok = i < n && i < cn;
      out_ids[(long)r * K + i] = ok ? c_idx[i] : -1;
      out_lp[(long)r * K + i] = ok ? c_val[i] - lse : -INFINITY;
    }
  }
}

// ------------------------------------------------------------------ host side
void launch_penalty_apply(void* logits, bool is_bf16, long stride, int rows, int V, const int* slot,
                          const float* pres, const float* freq, const float* rep, const int* counts,
                          const unsigned int* seen, hipStream_t s) {
  if (rows <= 0) return;
  const int words = (V + 31) / 32;
  const dim3 grid((V + 256 * 8 - 1) / (256 * 8), rows);
  if (is_bf16)
    penalty_apply_kernel<unsigned short><<<grid, 256, 0, s>>>(static_cast<unsigned short*>(logits), stride, V,
                                                              slot, pres, freq, rep, counts, seen, words);
  else
    penalty_apply_kernel<float><<<grid, 256, 0, s>>>(static_cast<float*>(logits), stride, V, slot, pres, freq, rep,
                                                     counts, seen, words);
}

void launch_penalty_update(const long* tok, const int* slot, int n, int* counts, unsigned int* seen, int V,
                           hipStream_t s) {
  if (n <= 0) return;
  penalty_update_kernel<<<(n + 255) / 256, 256, 0, s>>>(tok, slot, n, counts, seen, V, (V + 31) / 32);
}

void launch_penalty_init(int* counts, unsigned int* seen, int V, const int* slots, const int* off,
                         const int* n_prompt, const int* toks, int ninit, hipStream_t s) {
  if (ninit <= 0) return;
  penalty_init_kernel<<<ninit, 256, 0, s>>>(counts, seen, V, (V + 31) / 32, slots, off, n_prompt, toks);
}

void launch_top_logprobs(const void* logits, bool is_bf16, long stride, int rows, int V, const int* nreq,
                         int* out_ids, float* out_lp, int K, hipStream_t s) {
  if (rows <= 0) return;
  if (is_bf16)
    top_logprobs_kernel<unsigned short><<<rows, kTopT, 0, s>>>(static_cast<const unsigned short*>(logits), stride,
                                                               V, nreq, out_ids, out_lp, K);
  else
    top_logprobs_kernel<float><<<rows, kTopT, 0, s>>>(static_cast<const float*>(logits), stride, V, nreq, out_ids,
                                                      out_lp, K);
}

}  // namespace hipserve
