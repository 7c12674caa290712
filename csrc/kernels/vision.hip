// Qwen3-VL vision tower kernels (gfx950): LayerNorm (+ fused residual add), GELU,
// 2D RoPE of the ViT q/k heads and bidirectional per-frame attention.
//
// The reference never contains model code: it serves its Qwen3-VL default
// (vllm-models/helm-chart/values.yaml:8-12) through vLLM; these are the in-house
// kernels of hipserve/models/vision.py.
//
// vision_attn_kernel — varlen, non-causal, head_dim D <= 128 (multiple of 8; Qwen3-VL:
// 72 for the 30B/235B towers, 64 for the small ones), one query head per workgroup,
// 4 waves x 32 query rows, K/V tiles of 64 keys double-buffered in LDS and shared by
// the 4 waves:
//  * S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 (the query row is the MFMA column =
//    the lane: a lane owns 16 scores of one row, row max / sum need one lane ^ 32
//    exchange). K rows of each 16-key group sit in LDS with key bits 2 and 3 swapped,
//    so the S^T accumulator holds 8 consecutive keys per MFMA k-slot and feeds
//    O^T = V^T . P^T as the B operand without lane movement; V^T is transposed into
//    LDS by the staging stores (each thread packs one d of two keys into a dword: a
//    wave's stores cover all 64 banks), read back as one ds_read_b128 per slot.
//  * at most 256 VGPRs (amdgpu_waves_per_eu 2): two waves per SIMD hide the
//    dependent-MFMA and softmax latency (278 registers gave one wave per SIMD and
//    4.4x less throughput).
//  * d is zero-padded to a multiple of 16 for QK (KS k-steps) and of 32 for PV (NB
//    row blocks); the padding rows of V^T are zeroed once, Q/K padding is loaded as 0.
//  * online softmax in the log2 domain; only the segment's last tile is masked.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

// ---------------------------------------------------------------- LayerNorm
// one wave per row; VPT 8-element vectors per lane (C <= 512 * VPT)
template <int VPT, bool kAdd>
__global__ __launch_bounds__(256) void layernorm_kernel(unsigned short* __restrict__ out,
                                                        unsigned short* __restrict__ residual,
                                                        const unsigned short* __restrict__ x,
                                                        const unsigned short* __restrict__ w,
                                                        const unsigned short* __restrict__ b, int rows, int C,
                                                        float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = threadIdx.x & 63;
  const int nvec = C >> 3;
  const u16x8* xr = reinterpret_cast<const u16x8*>(x + (long)row * C);
  u16x8* rr = kAdd ? reinterpret_cast<u16x8*>(residual + (long)row * C) : nullptr;
  float v[VPT][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = lane + 64 * i;
    if (idx < nvec) {
      const u16x8 a = xr[idx];
      if constexpr (kAdd) {
        const u16x8 r = rr[idx];
        u16x8 t;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          t[j] = f32_to_bf16(bf16_to_f32(a[j]) + bf16_to_f32(r[j]));
          v[i][j] = bf16_to_f32(t[j]);
        }
        rr[idx] = t;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf16_to_f32(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i)
    if (lane + 64 * i < nvec)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
  const float inv = rsqrtf(wave_sum(q) / C + eps);
  u16x8* orow = reinterpret_cast<u16x8*>(out + (long)row * C);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = lane + 64 * i;
    if (idx < nvec) {
      const u16x8 wv = reinterpret_cast<const u16x8*>(w)[idx];
      const u16x8 bv = reinterpret_cast<const u16x8*>(b)[idx];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = f32_to_bf16(fmaf((v[i][j] - mean) * inv, bf16_to_f32(wv[j]), bf16_to_f32(bv[j])));
      orow[idx] = o;
    }
  }
}

void launch_layernorm(void* out, void* residual, const void* x, const void* w, const void* b, int rows, int C,
                      float eps, hipStream_t s) {
  if (rows <= 0) return;
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  auto* xx = static_cast<const unsigned short*>(x);
  auto* ww = static_cast<const unsigned short*>(w);
  auto* bb = static_cast<const unsigned short*>(b);
  const int nvec = C / 8;
  dim3 grid(cdiv(rows, 4));
#define LN_LAUNCH(vpt)                                                                                          \
  do {                                                                                                          \
    if (r) layernorm_kernel<vpt, true><<<grid, 256, 0, s>>>(o, r, xx, ww, bb, rows, C, eps);                    \
    else layernorm_kernel<vpt, false><<<grid, 256, 0, s>>>(o, r, xx, ww, bb, rows, C, eps);                     \
  } while (0)
  if (nvec <= 64) LN_LAUNCH(1);
  else if (nvec <= 128) LN_LAUNCH(2);
  else if (nvec <= 192) LN_LAUNCH(3);
  else if (nvec <= 256) LN_LAUNCH(4);
  else if (nvec <= 384) LN_LAUNCH(6);
  else if (nvec <= 576) LN_LAUNCH(9);
  else LN_LAUNCH(16);
#undef LN_LAUNCH
}

// ---------------------------------------------------------------- GELU (in place)
template <bool kTanh>
__global__ __launch_bounds__(256) void gelu_kernel(unsigned short* __restrict__ x, long nvec) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nvec) return;
  u16x8 a = reinterpret_cast<u16x8*>(x)[i];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float f = bf16_to_f32(a[j]);
    float g;
    if constexpr (kTanh) {
      const float u = 0.7978845608028654f * fmaf(0.044715f * f, f * f, f);
      g = 0.5f * f * (1.f + tanhf(u));
    } else {
      g = 0.5f * f * (1.f + erff(f * 0.7071067811865476f));
    }
    a[j] = f32_to_bf16(g);
  }
  reinterpret_cast<u16x8*>(x)[i] = a;
}

void launch_gelu(void* x, long n, bool tanh_approx, hipStream_t s) {
  const long nvec = n / 8;
  if (nvec <= 0) return;
  dim3 grid((unsigned)((nvec + 255) / 256));
  if (tanh_approx) gelu_kernel<true><<<grid, 256, 0, s>>>(static_cast<unsigned short*>(x), nvec);
  else gelu_kernel<false><<<grid, 256, 0, s>>>(static_cast<unsigned short*>(x), nvec);
}

// ---------------------------------------------------------------- 2D RoPE (q, k in place)
// one thread per (token, q|k head): the head's D values in registers (16-byte loads),
// rotate-half pairs (j, j + D/2) against the token's table row [cos(D/2) | sin(D/2)]
template <int D>
__global__ __launch_bounds__(256) void vision_rope_kernel(unsigned short* __restrict__ qkv,
                                                          const float* __restrict__ cos_sin, int T, int nh) {
  constexpr int NV = D / 8, H = D / 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= 2L * T * nh) return;
  const int t = (int)(i / (2 * nh)), head = (int)(i - (long)t * 2 * nh);  // q heads then k heads
  u16x8* p = reinterpret_cast<u16x8*>(qkv + (long)t * 3 * nh * D + (long)head * D);
  const float* cs = cos_sin + (long)t * D;
  float x[D];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const u16x8 a = p[v];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[8 * v + j] = bf16_to_f32(a[j]);
  }
  float y[D];
#pragma unroll
  for (int j = 0; j < H; ++j) rope_rot(x[j], x[j + H], cs[j], cs[H + j], y[j], y[j + H]);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(y[8 * v + j]);
    p[v] = o;
  }
}

// ---------------------------------------------------------------- attention
typedef unsigned short u16x4v __attribute__((ext_vector_type(4)));
constexpr int VA_KT = 64, VA_NWV = 4, VA_NT = 64 * VA_NWV;

template <int KS, int NB>
__global__ __launch_bounds__(VA_NT) __attribute__((amdgpu_waves_per_eu(2, 8))) void vision_attn_kernel(unsigned short* __restrict__ out,
                                                            const unsigned short* __restrict__ qkv,
                                                            const int* __restrict__ cu,
                                                            const int* __restrict__ tiles, int nh, int D,
                                                            float scale) {
  constexpr int DK = 16 * KS, DV = 32 * NB;  // padded d for QK and for PV
  constexpr int KLD = DK + 8, VLD = VA_KT + 8;
  constexpr int KPR = DK / 8;                          // 16-byte K pieces per key row
  constexpr int NPK = (VA_KT * KPR + VA_NT - 1) / VA_NT;
  // V staging items: (key pair, 8-d piece); a thread loads the piece of both keys and
  // writes 8 dwords of V^T (d, key pair) — a wave's 32 key pairs x 2 pieces hit 64 banks
  constexpr int NPV = (VA_KT / 2 * (DV / 8) + VA_NT - 1) / VA_NT;
  __shared__ __attribute__((aligned(16))) unsigned short kl[2][VA_KT * KLD];
  __shared__ __attribute__((aligned(16))) unsigned short vl[2][DV * VLD];

  const int seg = tiles[2 * blockIdx.x], r0 = tiles[2 * blockIdx.x + 1];
  const int h = blockIdx.y;
  const int s0 = cu[seg], len = cu[seg + 1] - s0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int qi = lane & 31, half = lane >> 5;
  const int wrow0 = r0 + 32 * wave;
  const bool wactive = wrow0 < len;
  const int row = min(wrow0 + qi, len - 1);
  const long rs = 3L * nh * D;  // qkv row stride
  const unsigned short* kbase_p = qkv + (long)s0 * rs + (long)(nh + h) * D;
  const unsigned short* vbase_p = qkv + (long)s0 * rs + (long)(2 * nh + h) * D;
  const int nkt = (len + VA_KT - 1) / VA_KT;
  const int nvp = D / 8;  // valid 16-byte pieces of a V row

  // V^T padding rows (d >= D) are never written by the staging: zero them once
  for (int i = tid; i < 2 * (DV - D) * VLD; i += VA_NT) {
    const int bsel = i / ((DV - D) * VLD), rem = i - bsel * (DV - D) * VLD;
    vl[bsel][D * VLD + rem] = 0;
  }

  u16x8 ska[NPK], sva[NPV][2], skb[NPK], svb[NPV][2];
  auto stage_load = [&](u16x8(&sk)[NPK], u16x8(&sv)[NPV][2], int kt) {
    const int kb = kt * VA_KT;
#pragma unroll
    for (int i = 0; i < NPK; ++i) {
      const int p = tid + VA_NT * i;
      const int key = p / KPR, pc = p - key * KPR;
      const int kk = min(kb + key, len - 1);
      u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      if (p < VA_KT * KPR && 8 * pc < D) z = *reinterpret_cast<const u16x8*>(kbase_p + (long)kk * rs + 8 * pc);
      sk[i] = z;
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int p = tid + VA_NT * i;
      const int kp = p & 31, pc = p >> 5;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int kk = min(kb + 2 * kp + e, len - 1);
        u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
        if (pc < nvp) z = *reinterpret_cast<const u16x8*>(vbase_p + (long)kk * rs + 8 * pc);
        sv[i][e] = z;
      }
    }
  };
  auto stage_store = [&](const u16x8(&sk)[NPK], const u16x8(&sv)[NPV][2], int buf) {
#pragma unroll
    for (int i = 0; i < NPK; ++i) {
      const int p = tid + VA_NT * i;
      if (p < VA_KT * KPR) {
        const int key = p / KPR, pc = p - key * KPR;
        const int krow = (key & ~12) | ((key & 4) << 1) | ((key & 8) >> 1);  // swap key bits 2 and 3
        *reinterpret_cast<u16x8*>(&kl[buf][krow * KLD + 8 * pc]) = sk[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NPV; ++i) {
      const int p = tid + VA_NT * i;
      const int kp = p & 31, pc = p >> 5;
      if (pc < nvp) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          *reinterpret_cast<unsigned int*>(&vl[buf][(8 * pc + j) * VLD + 2 * kp]) =
              (unsigned int)sv[i][0][j] | ((unsigned int)sv[i][1][j] << 16);
      }
    }
  };

  bf16x8 qf[KS];
  {
    const unsigned short* qp = qkv + (long)(s0 + row) * rs + (long)h * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int d0 = 16 * ks + 8 * half;
      u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      if (d0 < D) z = *reinterpret_cast<const u16x8*>(qp + d0);
      qf[ks] = __builtin_bit_cast(bf16x8, z);
    }
  }
  const float sl2 = scale * 1.4426950408889634f;
  f32x16 o[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[nb][r] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  auto compute = [&](int kt, int buf) {
    if (!wactive) return;
    const int kb = kt * VA_KT;
    const unsigned short* kr = &kl[buf][qi * KLD + 8 * half];
    f32x16 st[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int r = 0; r < 16; ++r) st[h2][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(kr + (32 * h2) * KLD + 16 * ks);
        st[h2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), qf[ks], st[h2], 0, 0, 0);
      }
    if (kb + VA_KT > len) {  // the segment's last tile: keys past its end
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kb + 32 * h2 + 16 * (r >> 3) + 8 * half + 4 * ((r >> 2) & 1) + (r & 3);
          if (key >= len) st[h2][r] = -INFINITY;
        }
    }
    float mx = -1e30f;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[h2][r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx * sl2);
    if (!__all(m_new == m_run)) {
      const float alpha = exp2f(m_run - m_new);
      l_run *= alpha;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[nb][r] *= alpha;
      m_run = m_new;
    }
    float psum = 0.f;
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      bf16x8 pb[2];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[h2][r], sl2, -m_run));
        psum += p;
        pb[r >> 3][r & 7] = static_cast<__bf16>(p);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const unsigned short* vb = &vl[buf][qi * VLD + 32 * h2 + 16 * s2 + 8 * half];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          const u16x8 a = *reinterpret_cast<const u16x8*>(vb + 32 * nb * VLD);
          o[nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), pb[s2], o[nb], 0, 0, 0);
        }
      }
    }
    l_run += psum;
  };

  stage_load(ska, sva, 0);
  if (nkt > 1) stage_load(skb, svb, 1);
  stage_store(ska, sva, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; kt += 2) {
    if (kt + 2 < nkt) stage_load(ska, sva, kt + 2);
    compute(kt, 0);
    if (kt + 1 < nkt) stage_store(skb, svb, 1);
    __syncthreads();
    if (kt + 1 >= nkt) break;
    if (kt + 3 < nkt) stage_load(skb, svb, kt + 3);
    compute(kt + 1, 1);
    if (kt + 2 < nkt) stage_store(ska, sva, 0);
    __syncthreads();
  }
  if (!wactive) return;
  l_run += __shfl_xor(l_run, 32, 64);
  const float inv = 1.f / l_run;
  if (wrow0 + qi < len) {
    unsigned short* op = out + (long)(s0 + wrow0 + qi) * nh * D + (long)h * D;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * nb + 8 * g + 4 * half;
        if (d0 < D) {
          u16x4v w;
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = f32_to_bf16(o[nb][4 * g + j] * inv);
          *reinterpret_cast<u16x4v*>(op + d0) = w;
        }
      }
  }
}

void launch_vision_attention(void* out, void* qkv, const float* cos_sin, const int* cu, const int* tiles,
                             int ntiles, int T, int nh, int D, float scale, hipStream_t s) {
  if (T <= 0 || ntiles <= 0) return;
  auto* q = static_cast<unsigned short*>(qkv);
  const unsigned rg = (unsigned)((2L * T * nh + 255) / 256);
  switch (D) {
    case 64: vision_rope_kernel<64><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
    case 72: vision_rope_kernel<72><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
    case 80: vision_rope_kernel<80><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
    case 96: vision_rope_kernel<96><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
    case 128: vision_rope_kernel<128><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
    default: vision_rope_kernel<16><<<rg, 256, 0, s>>>(q, cos_sin, T, nh); break;
  }
  dim3 grid(ntiles, nh);
  auto* o = static_cast<unsigned short*>(out);
#define VA_LAUNCH(ks, nb) vision_attn_kernel<ks, nb><<<grid, VA_NT, 0, s>>>(o, q, cu, tiles, nh, D, scale)
  if (D <= 64) VA_LAUNCH(4, 2);
  else if (D <= 80) VA_LAUNCH(5, 3);
  else if (D <= 96) VA_LAUNCH(6, 3);
  else VA_LAUNCH(8, 4);
#undef VA_LAUNCH
}

}  // namespace hipserve
