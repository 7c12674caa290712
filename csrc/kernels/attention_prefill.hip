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
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

typedef unsigned short u16x4v __attribute__((ext_vector_type(4)));

template <int D>
__global__ __launch_bounds__(256) void prefill_attn_kernel(
    unsigned short* __restrict__ out, long out_stride,
    const unsigned short* __restrict__ q, long q_stride,
    const unsigned short* __restrict__ k_cache,
    const unsigned short* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride,
    const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    const int* __restrict__ tiles, int nq, int nkv, int block_size,
    float scale) {
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
  for (int kt = 0; kt < nkt; ++kt) {
    const int kbase = kt * 32;
    // K fragment rows: key kbase + qi (clamped into the valid context)
    const int key = min(kbase + qi, ctx - 1);
    const unsigned short* kp = k_cache +
        ((long)btab[key / block_size] * nkv + kh) * head_stride +
        (long)(key % block_size) * D + 8 * half;
    u16x8 kf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = *reinterpret_cast<const u16x8*>(kp + 16 * ks);
    // V^T fragments: row d = 32*nb + qi; k-slot j of half h, step s ->
    // key kbase + 16s + 8(j>>2) + 4h + (j&3): two runs of 4 contiguous tokens.
    u16x4v vf[NB][2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int run = 0; run < 2; ++run) {
        int k4 = kbase + 16 * s + 8 * run + 4 * half;
        if (k4 > ctx - 1) k4 = (ctx - 1) & ~3;
        const unsigned short* vp = v_cache +
            ((long)btab[k4 / block_size] * nkv + kh) * head_stride + (k4 % block_size) +
            (long)qi * block_size;
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          vf[nb][s][run] = *reinterpret_cast<const u16x4v*>(vp + (long)32 * nb * block_size);
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
      const float v = (kk <= pos) ? st[r] * sl2 : -1e30f;
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
  l_run += __shfl_xor(l_run, 32, 64);
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
                              int block_size, float scale, hipStream_t s) {
  if (ntiles <= 0) return;
  dim3 grid(ntiles, nq), block(256);
  auto* o = static_cast<unsigned short*>(out);
  auto* qq = static_cast<const unsigned short*>(q);
  auto* kc = static_cast<const unsigned short*>(k_cache);
  auto* vc = static_cast<const unsigned short*>(v_cache);
  if (D == 128)
    prefill_attn_kernel<128><<<grid, block, 0, s>>>(o, out_stride, qq, q_stride, kc, vc, block_tables, bt_stride, cu_q, ctx_lens, tiles, nq, nkv, block_size, scale);
  else
    prefill_attn_kernel<64><<<grid, block, 0, s>>>(o, out_stride, qq, q_stride, kc, vc, block_tables, bt_stride, cu_q, ctx_lens, tiles, nq, nkv, block_size, scale);
}

}  // namespace hipserve
