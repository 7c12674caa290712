// Quantised decode GEMM v3: y[M, N] = x[M, K] . W^T for M <= 64 with
// W in the tiled quantised layout (gguf_tiles.h: GGUF Q4_0 .. Q6_K, FP8, INT8).
//
// Why v2 (gguf_mfma.hip qgemm2_kernel) streamed only 1.1-2.2 TB/s of quantised bytes at
// M = 64 (profiles/r4_gguf_m64_bodies.log, r2_qgemm_m64_pmc.md: 42 % of wave cycles in
// s_waitcnt): every workgroup staged x (64 rows x 256 f16 = 32 KiB per super-chunk, more
// bytes than its 128 weight rows' blocks) through registers and LDS once per super-chunk,
// with one super-chunk of weights in flight. A first v3 moved both operands to LDS-DMA
// rings: the x re-staging then dominated the per-CU DMA path (lm_head 234 vs 138 us).
// The fix is to stage x ONCE per workgroup:
//  * split K into S slices of at most XSC super-chunks (x slice <= 128 KiB of LDS); a
//    persistent grid of one workgroup per CU, S | grid, workgroup b takes slice b % S;
//  * the workgroup DMAs its x slice (f16, the producer's pair-order copy x16) into LDS
//    once, one barrier, and from then on its waves never synchronise again: each wave
//    walks its row groups (16 weight rows, round-robin over the slice's waves) x the
//    slice's super-chunks as one flat item stream, the raw weight chunk of item i + 3
//    loading into registers while item i is dequantised (gq::Dec, subnormal-integer
//    f16) and multiplied (v_mfma_f32_16x16x32_f16) against x fragments read from LDS;
//  * x fragments are conflict-free ds_read_b128s: 16-byte chunk j of row m sits at
//    chunk j ^ f(m & 15), f(c) = c ^ (((c >> 2) ^ (c >> 3)) & 1) * D, D = the chunk
//    distance between lane groups 0 and 1 (8; Q6_K: 4), so every 16-lane group of a
//    B-fragment read hits 16 distinct 16-byte bank slots.
// x16 holds f16 copies of bf16 activations; a value beyond the f16 range becomes inf
// there, so a wave whose accumulators come out non-finite (rare: Gemma-family hidden
// states) recomputes that row group from the bf16 x with power-of-two row pre-scales
// (q3_slow, plain loads) — the same result as v2's rerun, bit for bit.
// Outputs as v2: fp32 split-K partials ws[S, M, Ntot] for the fused decode epilogues, or
// bf16 out when S == 1; bit-identical to v2 (same dequant, same MFMA order per
// accumulator: super-chunks in order, steps in order).
#include "hipserve/common.h"
#include "hipserve/gguf_tiles.h"
#include "hipserve/kernels.h"

#include <cstdlib>

namespace hipserve {

namespace {
using namespace gq;

typedef __attribute__((address_space(3))) void* lds_p;

constexpr int Q3_XLDS = 131072;  // x slice bytes of LDS
constexpr int Q3_NW = 8;         // waves per workgroup (2 per SIMD)

template <int MT>
constexpr int q3_xsc() { return Q3_XLDS / (MT * 16 * 512); }  // super-chunks of x per slice

template <int QT>
constexpr int q3_d() { return QT == Q6_K ? 4 : 8; }  // chunk distance of lane groups 0 / 1

HS_DEVICE int q3_swz(int c, int d) { return c ^ ((((c >> 2) ^ (c >> 3)) & 1) * d); }

// rows of this wave recomputed from bf16 x with per-row power-of-two pre-scales (the
// accumulators of the fast pass were non-finite: an x value beyond the f16 range)
template <int QT, int MT>
HS_DEVICE void q3_slow(f32x4 (&acc)[MT], const unsigned short* __restrict__ x, long ldx, int M,
                       const unsigned char* __restrict__ wq, int sb0, int sb1) {
  constexpr int CB = chunk_bytes<QT>();
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  // max |x| of row `lane` over [sb0, sb1) -> scale 2^-k with max 2^-k < 2^15
  float sc_me = 1.f;
  if (lane < 16 * MT && lane < M) {
    const unsigned short* xr = x + (long)lane * ldx;
    unsigned mx = 0;
    for (int k = sb0 * 256; k < sb1 * 256; k += 8) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(xr + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) mx = max(mx, max((w[e] << 16) & 0x7FFF0000u, w[e] & 0x7FFF0000u));
    }
    const int ex = (int)(mx >> 23) - 127;
    sc_me = __builtin_bit_cast(float, (unsigned)(127 - min(126, max(0, ex - 14))) << 23);
  }
  float sc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) sc[t] = __shfl(sc_me, 16 * t + c, 64);
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sb = sb0; sb < sb1; ++sb) {
    Raw r;
    load_raw<QT>(wq + (long)sb * CB, g, c, lane, r);
    Dec<QT> dec;
    dec.setup(r, g);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const f16x8 a = dec.step(r, g, s);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = min(16 * t + c, M - 1);
        const u16x8 v = *reinterpret_cast<const u16x8*>(x + (long)m * ldx + sb * 256 + kbase<QT>(g, s));
        constexpr int ord[8] = {0, 2, 1, 3, 4, 6, 5, 7};
        f16x8 b;
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = static_cast<_Float16>(bf16_to_f32(v[ord[e]]) * sc[t]);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[t], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] *= 1.f / sc[t];  // exact: a power of two
}

struct Q3Args {
  unsigned short* out;  // bf16 [M, >= Ntot] (S == 1, ws == nullptr)
  long out_stride;
  float* ws;            // fp32 partials [S, M, Ntot]
  const unsigned short* x;    // bf16 [M, >= K] (the slow path)
  const unsigned short* x16;  // f16 pair order, same row stride
  long ldx;
  Parts parts;          // tile0 = first global row group of the part
  int ngroups;          // row groups of all parts
  int M, Ntot, K, per, S;  // per: super-chunks per K slice
};

template <int QT, int MT>
__global__ __launch_bounds__(64 * Q3_NW) void qgemm3_kernel(Q3Args A) {
  constexpr int CB = chunk_bytes<QT>(), XSC = MT * 16 * 512;  // x bytes per super-chunk
  __shared__ __attribute__((aligned(1024))) unsigned char lds[q3_xsc<MT>() * XSC];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int M = A.M, nsb = A.K >> 8;
  const int split = blockIdx.x % A.S, wg = blockIdx.x / A.S, nwg = gridDim.x / A.S;
  const int sb0 = split * A.per, sb1 = min(nsb, sb0 + A.per), nsc = sb1 - sb0;

  // ---- x slice -> LDS, once: piece j (1 KiB) = rows 2 jr, 2 jr + 1 of super-chunk j / (8 MT)
  {
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void*)A.x16, 0, (int)((long)M * A.ldx * 2), 0x00020000);
    const int ldx2 = (int)A.ldx * 2, pieces = nsc * MT * 8;
    for (int j = w; j < pieces; j += Q3_NW) {
      const int sc = j / (MT * 8), jr = j - sc * MT * 8;
      const int m = 2 * jr + (lane >> 5), jl = (lane & 31) ^ q3_swz(m & 15, q3_d<QT>());
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_p)(lds + j * 1024), 16, m * ldx2 + jl * 16,
                                               (sb0 + sc) * 512, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // x fragment addresses: row 16 t + c, chunk (kbase(g, s) / 8) ^ f(c) of the super-chunk
  const int fc = q3_swz(c, q3_d<QT>());
  int xa[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) xa[s] = c * 512 + (((kbase<QT>(g, s) >> 3) ^ fc) << 4);

  // ---- this wave's items: row groups r = gw, gw + TW, ... x super-chunks of the slice
  const int TW = nwg * Q3_NW, gw = wg * Q3_NW + w;
  const int nrg = gw < A.ngroups ? (A.ngroups - 1 - gw) / TW + 1 : 0;
  const int nitems = nrg * nsc;
  auto chunk = [&](int i) -> const unsigned char* {  // raw chunk of item i (clamped: no branch)
    i = min(i, nitems - 1);
    const int rr = i / nsc, sc = i - rr * nsc;
    const int r = gw + rr * TW;
    int pi = 0;
#pragma unroll
    for (int k = 1; k < kMaxParts; ++k)
      if (k < A.parts.n && r >= A.parts.p[k].tile0) pi = k;
    const Part& P = A.parts.p[pi];
    return P.q + ((long)(r - P.tile0) * nsb + sb0 + sc) * CB;
  };

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const Raw& raw, int sc) {
    const unsigned char* sp = lds + sc * XSC;
    Dec<QT> dec;
    dec.setup(raw, g);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      f16x8 b[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) b[t] = *reinterpret_cast<const f16x8*>(sp + xa[s] + t * 8192);
      const f16x8 a = dec.step(raw, g, s);
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[t], acc[t], 0, 0, 0);
    }
  };
  auto finish = [&](int i) {  // item i ended its row group: epilogue, then zero the accumulators
    const int r = gw + (i / nsc) * TW;
    int pi = 0;
#pragma unroll
    for (int k = 1; k < kMaxParts; ++k)
      if (k < A.parts.n && r >= A.parts.p[k].tile0) pi = k;
    const Part& P = A.parts.p[pi];
    const int gi = r - P.tile0;
    bool bad = false;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) bad |= !__builtin_isfinite(acc[t][e]);
    if (__any(bad)) q3_slow<QT, MT>(acc, A.x, A.ldx, M, P.q + (long)gi * nsb * CB, sb0, sb1);
    const int col = P.col + 16 * gi + 4 * g;
    if constexpr (QT == FP8 || QT == FP8B) {
      const f32x4 rs = *reinterpret_cast<const f32x4*>(P.rs + 16 * gi + 4 * g);
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[t] *= rs;
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + c;
      if (m < M) {
        if (A.ws != nullptr) {
          *reinterpret_cast<f32x4*>(A.ws + ((long)split * M + m) * A.Ntot + col) = acc[t];
        } else {
          uint2 v;
          v.x = pack_bf16x2(acc[t][0], acc[t][1]);
          v.y = pack_bf16x2(acc[t][2], acc[t][3]);
          *reinterpret_cast<uint2*>(A.out + (long)m * A.out_stride + col) = v;
        }
      }
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  // three raw register sets, used in rotation (loop unrolled by three: static indices),
  // each refilled with item i + 3 right after item i's dequant has read it
  Raw r0, r1, r2;
  if (nitems > 0) {
    load_raw<QT>(chunk(0), g, c, lane, r0);
    load_raw<QT>(chunk(1), g, c, lane, r1);
    load_raw<QT>(chunk(2), g, c, lane, r2);
  }
  auto item = [&](int i, Raw& cur) {
    const int sc = i % nsc;
    compute(cur, sc);
    load_raw<QT>(chunk(i + 3), g, c, lane, cur);  // the last items re-load the last chunk (unused)
    if (sc == nsc - 1) finish(i);
  };
  int i = 0;
  for (; i + 2 < nitems; i += 3) {
    item(i, r0);
    item(i + 1, r1);
    item(i + 2, r2);
  }
  if (i < nitems) item(i, r0);
  if (i + 1 < nitems) item(i + 1, r1);
}

template <int QT, int MT>
void q3_launch(const Q3Args& a, int grid, hipStream_t s) {
  qgemm3_kernel<QT, MT><<<grid, 64 * Q3_NW, 0, s>>>(a);
}

template <int QT>
void q3_launch_m(const Q3Args& a, int grid, hipStream_t s) {
  if (a.M <= 16)
    q3_launch<QT, 1>(a, grid, s);
  else if (a.M <= 32)
    q3_launch<QT, 2>(a, grid, s);
  else
    q3_launch<QT, 4>(a, grid, s);
}

int q3_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1) ncu = 256;
  }
  return ncu;
}

}  // namespace

bool qgemm3_enabled() {
  static const int e = [] {
    const char* s = getenv("HIPSERVE_QGEMM3");
    return s ? atoi(s) : 1;
  }();
  return e != 0;
}

// every part in one launch (one instantiation per format: formats launch separately)
bool launch_qgemm3(void* out, long out_stride, float* ws, const void* x, const void* x16, long ldx,
                   const GgufPart* parts, int nparts, int M, int Ntot, int K, int S, hipStream_t s) {
  if (M < 1 || M > 64 || x16 == nullptr || K % 256 || ldx % 8) return false;
  if ((long)M * ldx * 2 >= (1L << 31)) return false;
  const int nsb = K / 256, per = (nsb + S - 1) / S, Sx = (nsb + per - 1) / per;
  const int xsc = M <= 16 ? q3_xsc<1>() : M <= 32 ? q3_xsc<2>() : q3_xsc<4>();
  if (per > xsc) return false;  // the x slice would not fit the LDS: the caller runs v2
  if (ws == nullptr && Sx != 1) return false;
  int fmts[kMaxParts], nf = 0;
  for (int i = 0; i < nparts; ++i) {
    if (parts[i].qtype < Q4_0 || parts[i].qtype > INT8 || parts[i].rows % 16) return false;
    bool seen = false;
    for (int j = 0; j < nf; ++j) seen |= fmts[j] == parts[i].qtype;
    if (!seen) fmts[nf++] = parts[i].qtype;
  }
  // persistent grid: one workgroup per CU, a multiple of the slice count
  const int grid = max(1, q3_cus() / Sx) * Sx;
  for (int f = 0; f < nf; ++f) {
    Q3Args a{};
    a.out = static_cast<unsigned short*>(out);
    a.out_stride = out_stride;
    a.ws = ws;
    a.x = static_cast<const unsigned short*>(x);
    a.x16 = static_cast<const unsigned short*>(x16);
    a.ldx = ldx;
    a.M = M;
    a.Ntot = Ntot;
    a.K = K;
    a.per = per;
    a.S = Sx;
    int groups = 0;
    for (int i = 0; i < nparts; ++i) {
      if (parts[i].qtype != fmts[f]) continue;
      a.parts.p[a.parts.n++] = Part{static_cast<const unsigned char*>(parts[i].q), parts[i].rs, parts[i].qtype,
                                    parts[i].rows, parts[i].col, groups};
      groups += parts[i].rows / 16;
    }
    a.ngroups = groups;
    switch (fmts[f]) {
      case Q4_0: q3_launch_m<Q4_0>(a, grid, s); break;
      case Q4_1: q3_launch_m<Q4_1>(a, grid, s); break;
      case Q8_0: q3_launch_m<Q8_0>(a, grid, s); break;
      case Q4_K: q3_launch_m<Q4_K>(a, grid, s); break;
      case Q5_K: q3_launch_m<Q5_K>(a, grid, s); break;
      case Q6_K: q3_launch_m<Q6_K>(a, grid, s); break;
      case FP8: q3_launch_m<FP8>(a, grid, s); break;
      case FP8B: q3_launch_m<FP8B>(a, grid, s); break;
      case INT8: q3_launch_m<INT8>(a, grid, s); break;
    }
  }
  return true;
}

}  // namespace hipserve
