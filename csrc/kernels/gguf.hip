// GGUF block-quantized matmul for the GGUF tier on gfx950.
//
// Weight formats as laid out in HBM (repacked once at load by hipserve/ops/quant.py):
//   Q4_K  native 144-byte super-blocks (d, dmin, 12 B packed 6-bit scales/mins, 128 B nibbles)
//   Q5_K  native 176-byte super-blocks (+32 B high bits)
//   Q6_K  210-byte super-blocks padded to 224 B (16-byte aligned loads)
//   Q8_0  SoA: int8 qs [N][K] then fp16 d [N][K/32]
//   Q4_0  SoA: nibble qs [N][K/2] then fp16 d [N][K/32]      (Q4_1: + fp16 m [N][K/32])
//
// qgemm (decode, M <= 64): out[M,N] = x[M,K] . dequant(W)[N,K]^T on MFMA
// v_mfma_f32_16x16x32_bf16 in the form out^T = W . x^T. Weights are dequantised
// in registers straight into A fragments — never written back — so HBM traffic is
// the quantised bytes (4.5 b/w for Q4_K) + x. The MFMA k order is permuted per
// format so that each lane decodes whole contiguous byte runs of ONE block
// (64 k per lane per 256-k super-block); x fragments follow the same permutation
// from an LDS-staged x chunk shared by the workgroup's 4 waves (64 rows).
// Split-K over workgroups fills the 256 CUs when N is small: each K slice writes
// its own fp32 slab ws[split, M, N] (plain stores, no pre-zeroing, no atomics:
// deterministic and hipGraph-safe) and a reduce kernel sums the slabs in order.
//
// qdequant (prefill, large M): the same decoders write a bf16 copy that feeds a
// hipBLASLt GEMM (compute-bound regime, dequant traffic is noise there).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

enum QT { QT_Q4_0 = 0, QT_Q4_1 = 1, QT_Q8_0 = 2, QT_Q4_K = 3, QT_Q5_K = 4, QT_Q6_K = 5, QT_BF16 = 6 };

struct QParams {
  const unsigned char* q;   // quant bytes / super-blocks
  const unsigned short* d;  // SoA scales (fp16), Q8_0/Q4_0/Q4_1
  const unsigned short* m;  // SoA mins (fp16), Q4_1
  int K;
  long row_bytes;           // bytes per row of q
};

HS_DEVICE float h2f(unsigned short h) { return static_cast<float>(__builtin_bit_cast(_Float16, h)); }

HS_DEVICE u32x4 ld16(const unsigned char* p) { return *reinterpret_cast<const u32x4*>(p); }

HS_DEVICE unsigned int byte_of(const u32x4 (&v)[2], int i) {  // i in [0, 32)
  return (v[i >> 4][(i >> 2) & 3] >> (8 * (i & 3))) & 0xFFu;
}

HS_DEVICE void scale_min_k4(int j, const unsigned char* s, float& sc, float& mn) {
  if (j < 4) {
    sc = s[j] & 63;
    mn = s[j + 4] & 63;
  } else {
    sc = (s[j + 4] & 0xF) | ((s[j - 4] >> 6) << 4);
    mn = (s[j + 4] >> 4) | ((s[j] >> 6) << 4);
  }
}

// k index (within a 256-k super-chunk) of fragment element j, step s, lane group g
template <int QT>
HS_DEVICE int kbase(int g, int s) {
  if constexpr (QT == QT_Q6_K) {
    const int q = (g & 1) + 2 * (s >> 2);
    return 128 * (g >> 1) + 32 * q + 8 * (s & 3);
  } else {
    return 64 * g + 32 * (s >> 2) + 8 * (s & 3);
  }
}

// Per-lane raw bytes of one super-chunk (256 k) of one weight row: loaded one
// super-chunk ahead by the decode GEMM (load_raw), decoded into MFMA A
// fragments when its turn comes (decode_raw) — the loads stay in flight while
// the previous super-chunk is decoded and multiplied.
struct RawQ {
  u32x4 v[8];            // quant bytes (per format: see load_raw)
  unsigned short h[4];   // SoA fp16 scales / mins (Q8_0, Q4_0, Q4_1)
};

template <int QT>
HS_DEVICE void load_raw(const QParams& p, long row, int sb, int g, RawQ& r) {
  if constexpr (QT == QT_BF16) {  // plain bf16 rows: 128 contiguous bytes per lane
    const unsigned char* rp = p.q + row * p.row_bytes + (long)sb * 512 + 128 * g;
#pragma unroll
    for (int s = 0; s < 8; ++s) r.v[s] = ld16(rp + 16 * s);
  } else if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) {
    constexpr int BB = QT == QT_Q4_K ? 144 : 176;
    const unsigned char* bp = p.q + row * p.row_bytes + (long)sb * BB;
    const int qoff = QT == QT_Q4_K ? 16 : 48;
    r.v[0] = ld16(bp);                     // d, dmin, 12 B packed scales/mins
    r.v[1] = ld16(bp + qoff + 32 * g);
    r.v[2] = ld16(bp + qoff + 32 * g + 16);
    if constexpr (QT == QT_Q5_K) { r.v[3] = ld16(bp + 16); r.v[4] = ld16(bp + 32); }
  } else if constexpr (QT == QT_Q6_K) {
    const unsigned char* bp = p.q + row * p.row_bytes + (long)sb * 224;
    const int h = g >> 1, odd = g & 1;
    r.v[0] = ld16(bp + 64 * h + 32 * odd);
    r.v[1] = ld16(bp + 64 * h + 32 * odd + 16);
    r.v[2] = ld16(bp + 128 + 32 * h);
    r.v[3] = ld16(bp + 128 + 32 * h + 16);
    r.v[4] = ld16(bp + 192);               // 16 int8 sub-block scales
    r.v[5] = ld16(bp + 208);               // d (+ padding)
  } else if constexpr (QT == QT_Q8_0) {
    const unsigned char* qp = p.q + row * (long)p.K + (long)sb * 256 + 64 * g;
    const unsigned short* dp = p.d + row * (long)(p.K / 32) + sb * 8 + 2 * g;
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = ld16(qp + 16 * i);
    r.h[0] = dp[0];
    r.h[1] = dp[1];
  } else {  // Q4_0 / Q4_1 SoA
    const unsigned char* qp = p.q + row * (long)(p.K / 2) + (long)sb * 128 + 32 * g;
    const long di = row * (long)(p.K / 32) + sb * 8 + 2 * g;
    r.v[0] = ld16(qp);
    r.v[1] = ld16(qp + 16);
    r.h[0] = p.d[di];
    r.h[1] = p.d[di + 1];
    if constexpr (QT == QT_Q4_1) { r.h[2] = p.m[di]; r.h[3] = p.m[di + 1]; }
  }
}

// Decode the 64 weights lane group g owns in the loaded super-chunk into the 8
// bf16x8 A fragments of the 8 MFMA k-steps.
template <int QT>
HS_DEVICE void decode_raw(const RawQ& r, int g, bf16x8 (&a)[8]) {
  if constexpr (QT == QT_BF16) {
#pragma unroll
    for (int s = 0; s < 8; ++s) a[s] = __builtin_bit_cast(bf16x8, r.v[s]);
  } else if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) {
    const u32x4 hdr = r.v[0];
    unsigned char sc12[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) sc12[i] = (hdr[1 + i / 4] >> (8 * (i & 3))) & 0xFF;
    const float d = h2f(hdr[0] & 0xFFFF), dmin = h2f(hdr[0] >> 16);
    float s1, m1, s2, m2;
    scale_min_k4(2 * g, sc12, s1, m1);
    scale_min_k4(2 * g + 1, sc12, s2, m2);
    const float d1 = d * s1, mm1 = dmin * m1, d2 = d * s2, mm2 = dmin * m2;
    const u32x4 qs[2] = {r.v[1], r.v[2]};
    u32x4 qh[2];
    if constexpr (QT == QT_Q5_K) { qh[0] = r.v[3]; qh[1] = r.v[4]; }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = 8 * (s & 3) + j;
        const unsigned int b = byte_of(qs, l);
        float q = (s < 4) ? (float)(b & 0xF) : (float)(b >> 4);
        if constexpr (QT == QT_Q5_K) {
          const unsigned int hb = byte_of(qh, l);
          q += ((hb >> (2 * g + (s >> 2))) & 1) ? 16.f : 0.f;
        }
        a[s][j] = static_cast<__bf16>((s < 4) ? d1 * q - mm1 : d2 * q - mm2);
      }
  } else if constexpr (QT == QT_Q6_K) {
    const u32x4 ql[2] = {r.v[0], r.v[1]};
    const u32x4 qh[2] = {r.v[2], r.v[3]};
    const u32x4 scv = r.v[4];
    const float d = h2f(r.v[5][0] & 0xFFFF);
    const int h = g >> 1, odd = g & 1;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int q = odd + 2 * (s >> 2);
      const int si = 8 * h + 2 * q + ((s & 3) >= 2 ? 1 : 0);
      const float sc = (float)(signed char)((scv[si >> 2] >> (8 * (si & 3))) & 0xFF);
      const float ds = d * sc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int l = 8 * (s & 3) + j;
        const unsigned int b = byte_of(ql, l);
        const unsigned int lo = (s < 4) ? (b & 0xF) : (b >> 4);
        const unsigned int hi = (byte_of(qh, l) >> (2 * q)) & 3;
        a[s][j] = static_cast<__bf16>(ds * (float)((int)(lo | (hi << 4)) - 32));
      }
    }
  } else if constexpr (QT == QT_Q8_0) {
    const float dA = h2f(r.h[0]), dB = h2f(r.h[1]);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float dd = (s < 4) ? dA : dB;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * s + j;  // byte within the lane's 64
        const signed char c = (signed char)((r.v[i >> 4][(i >> 2) & 3] >> (8 * (i & 3))) & 0xFF);
        a[s][j] = static_cast<__bf16>(dd * (float)c);
      }
    }
  } else {  // Q4_0 / Q4_1
    const float dA = h2f(r.h[0]), dB = h2f(r.h[1]);
    float mA = 0.f, mB = 0.f;
    if constexpr (QT == QT_Q4_1) { mA = h2f(r.h[2]); mB = h2f(r.h[3]); }
    const u32x4 v[2] = {r.v[0], r.v[1]};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int blk = s >> 2;
      const float dd = blk ? dB : dA, mm = blk ? mB : mA;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = 8 * (s & 3) + j;       // element in the 32-block
        const unsigned int b = byte_of(v, 16 * blk + (e & 15));
        const float q = (e < 16) ? (float)(b & 0xF) : (float)(b >> 4);
        a[s][j] = static_cast<__bf16>(QT == QT_Q4_0 ? dd * (q - 8.f) : dd * q + mm);
      }
    }
  }
}

template <int QT>
HS_DEVICE void decode_lane(const QParams& p, long row, int sb, int g, bf16x8 (&a)[8]) {
  RawQ r;
  load_raw<QT>(p, row, sb, g, r);
  decode_raw<QT>(r, g, a);
}

constexpr int kXPad = 8;  // LDS row padding (bf16) for conflict-free b128 reads

template <int QT, int MT, int NWAVES>
__global__ __launch_bounds__(64 * NWAVES) void qgemm_kernel(
    unsigned short* __restrict__ out, float* __restrict__ ws, const unsigned short* __restrict__ x,
    long x_stride, long out_stride, QParams p, int M, int N, int K, int sb_per_split) {
  constexpr int XR = 16 * MT;            // staged x rows
  constexpr int XS = 256 + kXPad;        // LDS row stride (elements)
  __shared__ __attribute__((aligned(16))) unsigned short xs[XR * XS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  constexpr int NT = 64 * NWAVES;     // threads; the workgroup owns 16 * NWAVES weight rows
  const int n0 = blockIdx.x * (16 * NWAVES) + wave * 16;
  const int nsb = K / 256;
  const int sb0 = blockIdx.y * sb_per_split;
  const int sb1 = min(nsb, sb0 + sb_per_split);
  const long row = min(n0 + c, N - 1);
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline over super-chunks: the quant bytes AND the x slice of
  // super-chunk sb+1 are loaded (into registers) before super-chunk sb is
  // decoded and multiplied, so HBM / L2 latency overlaps the dequant VALU work
  // and the MFMAs instead of being exposed once per 256 k.
  constexpr int XP = (XR * 32 + NT - 1) / NT;  // 16-byte x pieces per thread per super-chunk
  u16x8 xv[XP];
  auto load_x = [&](int sb) {
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int idx = min(i * NT + (int)threadIdx.x, XR * 32 - 1), r = idx >> 5, cc = idx & 31;
      // rows >= M are clamped, not zeroed: they only feed outputs m >= M (never stored)
      xv[i] = *reinterpret_cast<const u16x8*>(x + min(r, M - 1) * x_stride + sb * 256 + cc * 8);
    }
  };
  RawQ raw;
  if (sb0 < sb1) {
    load_x(sb0);
    load_raw<QT>(p, row, sb0, g, raw);
  }
  for (int sb = sb0; sb < sb1; ++sb) {
    __syncthreads();  // previous super-chunk's LDS reads are done
#pragma unroll
    for (int i = 0; i < XP; ++i) {
      const int idx = i * NT + threadIdx.x, r = idx >> 5, cc = idx & 31;
      if (idx < XR * 32) *reinterpret_cast<u16x8*>(xs + r * XS + cc * 8) = xv[i];
    }
    const RawQ cur = raw;
    if (sb + 1 < sb1) {  // prefetch the next super-chunk
      load_x(sb + 1);
      load_raw<QT>(p, row, sb + 1, g, raw);
    }
    __syncthreads();
    bf16x8 a[8];
    decode_raw<QT>(cur, g, a);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int kb = kbase<QT>(g, s);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 bv = *reinterpret_cast<const u16x8*>(xs + (16 * t + c) * XS + kb);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], __builtin_bit_cast(bf16x8, bv), acc[t], 0, 0, 0);
      }
    }
  }
  // C layout: col = m (lane & 15), rows n = 4*g + r
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + c;
    if (m >= M) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 4 * g + r;
      if (n >= N) continue;
      if (ws) ws[((long)blockIdx.y * M + m) * N + n] = acc[t][r];
      else out[m * out_stride + n] = f32_to_bf16(acc[t][r]);
    }
  }
}

// out[m, n] = bf16(sum over the S slabs, in slab order)
__global__ void splitk_sum_bf16_kernel(unsigned short* __restrict__ out, const float* __restrict__ ws, int M, int N,
                                       int S, long out_stride) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  const long MN = (long)M * N;
  if (i >= MN) return;
  const int m = i / N, n = i % N;
  float v = ws[i];
  for (int s = 1; s < S; ++s) v += ws[s * MN + i];
  out[m * out_stride + n] = f32_to_bf16(v);
}

template <int QT>
__global__ __launch_bounds__(256) void qdequant_kernel(unsigned short* __restrict__ out, QParams p, int N,
                                                       int K) {
  const long t = blockIdx.x * 256L + threadIdx.x;  // (row, sb, g)
  const int nsb = K / 256;
  if (t >= (long)N * nsb * 4) return;
  const int g = t & 3;
  const long rs = t >> 2;
  const long row = rs / nsb;
  const int sb = rs % nsb;
  bf16x8 a[8];
  decode_lane<QT>(p, row, sb, g, a);
#pragma unroll
  for (int s = 0; s < 8; ++s)
    *reinterpret_cast<bf16x8*>(out + row * K + sb * 256 + kbase<QT>(g, s)) = a[s];
}

template <int QT>
static void launch_qgemm_t(void* out, float* ws, const void* x, long x_stride, long out_stride,
                           const QParams& p, int M, int N, int K, int splits, hipStream_t s) {
  // 4 waves = 64 weight rows per workgroup (8-wave 128-row tiles halve the x
  // staging traffic but measured slower at M = 64: 21.6 vs 18.6 us per Q4_K call)
  constexpr int NW = 4;
  const int nsb = K / 256;
  const int per = (nsb + splits - 1) / splits;
  dim3 grid((N + 16 * NW - 1) / (16 * NW), (nsb + per - 1) / per), block(64 * NW);
  auto* o = static_cast<unsigned short*>(out);
  auto* xi = static_cast<const unsigned short*>(x);
  if (M <= 16) qgemm_kernel<QT, 1, NW><<<grid, block, 0, s>>>(o, ws, xi, x_stride, out_stride, p, M, N, K, per);
  else if (M <= 32) qgemm_kernel<QT, 2, NW><<<grid, block, 0, s>>>(o, ws, xi, x_stride, out_stride, p, M, N, K, per);
  else qgemm_kernel<QT, 4, NW><<<grid, block, 0, s>>>(o, ws, xi, x_stride, out_stride, p, M, N, K, per);
}

void launch_gguf_gemm(void* out, float* ws, const void* x, long x_stride, long out_stride,
                      const void* q, const void* d, const void* m, int qtype, long row_bytes,
                      int M, int N, int K, int splits, hipStream_t s) {
  QParams p{static_cast<const unsigned char*>(q), static_cast<const unsigned short*>(d),
            static_cast<const unsigned short*>(m), K, row_bytes};
  const int nsb = K / 256;
  const int slabs = (nsb + (nsb + splits - 1) / splits - 1) / ((nsb + splits - 1) / splits);  // grid.y
  switch (qtype) {
    case QT_Q4_0: launch_qgemm_t<QT_Q4_0>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_Q4_1: launch_qgemm_t<QT_Q4_1>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_Q8_0: launch_qgemm_t<QT_Q8_0>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_Q4_K: launch_qgemm_t<QT_Q4_K>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_Q5_K: launch_qgemm_t<QT_Q5_K>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_Q6_K: launch_qgemm_t<QT_Q6_K>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
    case QT_BF16: launch_qgemm_t<QT_BF16>(out, ws, x, x_stride, out_stride, p, M, N, K, splits, s); break;
  }
  if (ws) {
    const long n = (long)M * N;
    splitk_sum_bf16_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(static_cast<unsigned short*>(out), ws, M, N,
                                                                       slabs, out_stride);
  }
}

void launch_gguf_dequant(void* out, const void* q, const void* d, const void* m, int qtype,
                         long row_bytes, int N, int K, hipStream_t s) {
  QParams p{static_cast<const unsigned char*>(q), static_cast<const unsigned short*>(d),
            static_cast<const unsigned short*>(m), K, row_bytes};
  const long threads = (long)N * (K / 256) * 4;
  dim3 grid((unsigned)((threads + 255) / 256)), block(256);
  auto* o = static_cast<unsigned short*>(out);
  switch (qtype) {
    case QT_Q4_0: qdequant_kernel<QT_Q4_0><<<grid, block, 0, s>>>(o, p, N, K); break;
    case QT_Q4_1: qdequant_kernel<QT_Q4_1><<<grid, block, 0, s>>>(o, p, N, K); break;
    case QT_Q8_0: qdequant_kernel<QT_Q8_0><<<grid, block, 0, s>>>(o, p, N, K); break;
    case QT_Q4_K: qdequant_kernel<QT_Q4_K><<<grid, block, 0, s>>>(o, p, N, K); break;
    case QT_Q5_K: qdequant_kernel<QT_Q5_K><<<grid, block, 0, s>>>(o, p, N, K); break;
    case QT_Q6_K: qdequant_kernel<QT_Q6_K><<<grid, block, 0, s>>>(o, p, N, K); break;
  }
}

}  // namespace hipserve
