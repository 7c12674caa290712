// Quantised decode GEMM v3: y[M, N] = x[M, K] . W^T for M <= 64 with
// W in the tiled quantised layout (gguf_tiles.h: GGUF Q4_0 .. Q6_K, FP8, INT8), both
// operands staged by LDS-DMA.
//
// Why v2 (gguf_mfma.hip qgemm2_kernel) streamed only 1.1-2.2 TB/s of quantised bytes at
// M = 64 (profiles/r4_gguf_m64_bodies.log, r2_qgemm_m64_pmc.md: 42 % of wave cycles in
// s_waitcnt, 11 VALU per MFMA): its weights went global -> VGPR one super-chunk ahead
// (deeper register rings cost occupancy: r2_qgemm_deep_ring_negative.md) and x was staged
// through registers. Here:
//  * a workgroup of NW waves = NW row groups of 16 rows; per 256-deep super-chunk (SC) its
//    LDS slot holds x (MT * 16 rows x 256 f16, from the producer's f16 pair-order copy
//    x16) and each wave's raw weight chunk (CB bytes, the tiled chunk exactly as stored);
//  * a ring of 3 slots: the DMA of SC sb + 2 is issued when SC sb starts, so every
//    byte has two SCs (~1.3 us) to land without holding a register; in-flight bytes
//    per CU = two slots (100+ KB);
//  * a wave reads its chunk with ds_reads at the global layout's offsets (gq::load_raw on
//    the LDS copy) and dequantises in registers as v2 does (subnormal-integer f16, one
//    v_pk_fma per pair); x fragments are conflict-free ds_read_b128s: chunk j of row m
//    sits at chunk j ^ f(m & 15), f(c) = c ^ (((c >> 2) ^ (c >> 3)) & 1) * D with D = the
//    chunk distance between lane groups 0 and 1 (8; Q6_K: 4), which puts every 16-lane
//    group of a B-fragment read on 16 distinct 16-byte bank slots;
//  * one s_barrier per SC (x is shared); the weight half of a slot is private to its wave
//    (its own vmcnt orders it). Raw s_barrier + counted vmcnt: the DMAs stay in flight.
// x16 holds f16 copies of bf16 activations; a value beyond the f16 range becomes inf
// there, so a workgroup whose accumulators come out non-finite (rare: Gemma-family
// hidden states) recomputes its rows from the bf16 x with power-of-two row pre-scales
// (q3_slow, plain loads) — the same contract as v2.
// Outputs as v2: fp32 split-K partials ws[S, M, Ntot] for the fused decode epilogues, or
// bf16 out when S == 1.
#include "hipserve/common.h"
#include "hipserve/gguf_tiles.h"
#include "hipserve/kernels.h"

#include <cstdlib>

namespace hipserve {

namespace {
using namespace gq;

typedef __attribute__((address_space(3))) void* lds_p;

constexpr int Q3_LDS = 163840;  // the whole CU
constexpr int Q3_NSLOT = 3;

template <int QT, int MT>
constexpr int q3_nw() {  // waves (16-row groups) per workgroup: 3 slots fit the LDS
  constexpr int xb = MT * 16 * 512, cb = chunk_bytes<QT>();
  int nw = MT == 4 ? 8 : 16;
  while (nw > 4 && Q3_NSLOT * (xb + nw * cb) > Q3_LDS) --nw;
  return nw;
}
template <int QT, int MT>
constexpr int q3_slot() { return MT * 16 * 512 + q3_nw<QT, MT>() * chunk_bytes<QT>(); }

template <int QT>
constexpr int q3_d() { return QT == Q6_K ? 4 : 8; }  // chunk distance of lane groups 0 / 1

// 16-byte chunk (0..31) of the 256 f16 of an x row that lane group g reads at step s
template <int QT>
HS_DEVICE int q3_chunk(int g, int s) { return kbase<QT>(g, s) >> 3; }

HS_DEVICE int q3_swz(int c, int d) { return c ^ ((((c >> 2) ^ (c >> 3)) & 1) * d); }

template <int N>
HS_DEVICE void q3_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// rows of this wave recomputed from bf16 x with per-row power-of-two pre-scales (the
// accumulators of the fast pass were non-finite: an x value beyond the f16 range)
template <int QT, int MT>
HS_DEVICE void q3_slow(f32x4 (&acc)[MT], const unsigned short* __restrict__ x, long ldx, int M,
                       const unsigned char* __restrict__ wq, int nsb, int sb0, int sb1) {
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
  Parts parts;
  int M, Ntot, K, per;  // per: super-chunks per K split
};

// compile-time geometry of one (format, row tile) instantiation. (The DMA lambda computes
// its per-lane x offsets inline: with them precomputed into local int arrays read inside
// the lambda, hipcc (ROCm 7.2) silently emitted no host stub for the kernel.)
template <int QT, int MT>
struct Q3G {
  static constexpr int NW = q3_nw<QT, MT>(), CB = chunk_bytes<QT>(), SLOT = q3_slot<QT, MT>();
  static constexpr int XB = MT * 16 * 512;           // x image bytes of a slot
  static constexpr int XI = XB / 1024;               // x DMA instructions per slot
  static constexpr int NXW = (XI + NW - 1) / NW;     // ... per wave (the last ones may repeat a piece)
  static constexpr int N4 = CB / 1024, N1 = (CB % 1024) / 256, TAIL = CB % 256;
  static constexpr int NDMA = NXW + N4 + N1 + (TAIL ? 1 : 0);  // DMA instructions per wave and slot
};

template <int QT, int MT, int NT>
__global__ __launch_bounds__(NT) void qgemm3_kernel(Q3Args A) {
  using C_ = Q3G<QT, MT>;
  constexpr int NW = C_::NW, CB = C_::CB, SLOT = C_::SLOT, XB = C_::XB, XI = C_::XI, NXW = C_::NXW;
  constexpr int NDMA = C_::NDMA;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[Q3_NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  const int tile = blockIdx.x;
  int pi = 0;
#pragma unroll
  for (int i = 1; i < kMaxParts; ++i)
    if (i < A.parts.n && tile >= A.parts.p[i].tile0) pi = i;
  const Part& P = A.parts.p[pi];
  const int ngroups = P.rows >> 4, nsb = A.K >> 8, M = A.M;
  const int gi = (tile - P.tile0) * NW + w;  // this wave's row group (>= ngroups: computes a copy, stores nothing)
  const int gl = min(gi, ngroups - 1);
  const int sb0 = blockIdx.y * A.per, sb1 = min(nsb, sb0 + A.per);

  // ---- DMA sources
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.x16, 0, (int)((long)M * A.ldx * 2), 0x00020000);
  const int ldx2 = (int)A.ldx * 2;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)P.q, 0, ngroups * nsb * CB, 0x00020000);
  const int wbase = gl * nsb * CB;  // byte offset of this wave's row group
  auto dma = [&](int sb, int slot) {
    unsigned char* s = lds + slot * C_::SLOT;
#pragma unroll
    for (int i = 0; i < C_::NXW; ++i) {
      // 1 KiB piece j = x rows 2 j, 2 j + 1 (the last waves may repeat piece XI - 1);
      // lane -> row m, LDS chunk lane & 31 holding x chunk (lane & 31) ^ f(m & 15)
      const int j = min(w + C_::NW * i, C_::XI - 1);
      const int m = 2 * j + (lane >> 5), jl = (lane & 31) ^ q3_swz(m & 15, q3_d<QT>());
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_p)(s + j * 1024), 16, m * ldx2 + jl * 16, sb * 512, 0, 0);
    }
    unsigned char* d = s + C_::XB + w * C_::CB;
    const int so = wbase + sb * C_::CB;
#pragma unroll
    for (int n = 0; n < C_::N4; ++n)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(d + 1024 * n), 16, lane * 16 + 1024 * n, so, 0, 0);
#pragma unroll
    for (int n = 0; n < C_::N1; ++n)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(d + 1024 * C_::N4 + 256 * n), 4,
                                               lane * 4 + 1024 * C_::N4 + 256 * n, so, 0, 0);
    if constexpr (C_::TAIL > 0) {
      if (lane < C_::TAIL / 4)  // lanes 0 .. TAIL/4 - 1 are active in every wave: always issued
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (lds_p)(d + 1024 * C_::N4 + 256 * C_::N1), 4,
                                                 lane * 4 + 1024 * C_::N4 + 256 * C_::N1, so, 0, 0);
    }
  };

  // x fragment addresses (slot-relative): row 16 t + c, chunk q3_chunk(g, s) ^ f(c)
  const int fc = q3_swz(c, q3_d<QT>());
  int xa[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) xa[s] = c * 512 + ((q3_chunk<QT>(g, s) ^ fc) << 4);

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (sb0 < sb1) {
    dma(sb0, 0);
    if (sb0 + 1 < sb1) dma(sb0 + 1, 1);
  }
  int slot = 0;
  for (int sb = sb0; sb < sb1; ++sb) {
    if (sb + 1 < sb1)
      q3_vmwait<NDMA>();  // own DMA of sb landed; sb + 1's in flight
    else
      q3_vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot sb - 1 returned
    __builtin_amdgcn_s_barrier();                        // every wave's x DMA of sb landed
    if (sb + 2 < sb1) dma(sb + 2, slot == 0 ? 2 : slot - 1);
    const unsigned char* sp = lds + slot * SLOT;
    Raw raw;
    load_raw<QT>(sp + XB + w * CB, g, c, lane, raw);
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
    slot = slot == Q3_NSLOT - 1 ? 0 : slot + 1;
  }

  bool bad = false;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) bad |= !__builtin_isfinite(acc[t][e]);
  if (__any(bad))  // per wave: this wave's rows
    q3_slow<QT, MT>(acc, A.x, A.ldx, M, P.q + (long)gl * nsb * CB, nsb, sb0, sb1);

  if (gi >= ngroups) return;
  const int col = P.col + 16 * gi + 4 * g;
  if constexpr (QT == FP8 || QT == FP8B) {
    const f32x4 rs = *reinterpret_cast<const f32x4*>(P.rs + 16 * gi + 4 * g);
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] *= rs;
  }
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    const int m = 16 * t + c;
    if (m >= M) continue;
    if (A.ws != nullptr) {
      *reinterpret_cast<f32x4*>(A.ws + ((long)blockIdx.y * M + m) * A.Ntot + col) = acc[t];
    } else {
      uint2 v;
      v.x = pack_bf16x2(acc[t][0], acc[t][1]);
      v.y = pack_bf16x2(acc[t][2], acc[t][3]);
      *reinterpret_cast<uint2*>(A.out + (long)m * A.out_stride + col) = v;
    }
  }
}

template <int QT, int MT>
void q3_launch(const Q3Args& a, int tiles, int S, hipStream_t s) {
  constexpr int NT = 64 * q3_nw<QT, MT>();
  qgemm3_kernel<QT, MT, NT><<<dim3(tiles, S), NT, 0, s>>>(a);
}

template <int QT>
void q3_launch_m(const Q3Args& a, int tiles, int S, hipStream_t s) {
  if (a.M <= 16)
    q3_launch<QT, 1>(a, tiles, S, s);
  else if (a.M <= 32)
    q3_launch<QT, 2>(a, tiles, S, s);
  else
    q3_launch<QT, 4>(a, tiles, S, s);
}

template <int QT>
int q3_rows(int M) {
  return 16 * (M <= 16 ? q3_nw<QT, 1>() : M <= 32 ? q3_nw<QT, 2>() : q3_nw<QT, 4>());
}

}  // namespace

bool qgemm3_enabled() {
  static const int e = [] {
    const char* s = getenv("HIPSERVE_QGEMM3");
    return s ? atoi(s) : 1;
  }();
  return e != 0;
}

// parts of one launch: every part of format qt (one kernel instantiation per format)
bool launch_qgemm3(void* out, long out_stride, float* ws, const void* x, const void* x16, long ldx,
                   const GgufPart* parts, int nparts, int M, int Ntot, int K, int S, hipStream_t s) {
  if (M < 1 || M > 64 || x16 == nullptr || K % 256 || ldx % 8) return false;
  if ((long)M * ldx * 2 >= (1L << 31)) return false;
  const int nsb = K / 256, per = (nsb + S - 1) / S, Sx = (nsb + per - 1) / per;
  int fmts[kMaxParts], nf = 0;
  for (int i = 0; i < nparts; ++i) {
    if (parts[i].qtype < Q4_0 || parts[i].qtype > INT8) return false;
    if ((long)(parts[i].rows / 16) * nsb * gguf_tiled_chunk_bytes(parts[i].qtype) >= (1L << 31)) return false;
    bool seen = false;
    for (int j = 0; j < nf; ++j) seen |= fmts[j] == parts[i].qtype;
    if (!seen) fmts[nf++] = parts[i].qtype;
  }
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
    int rows = 0;
    switch (fmts[f]) {
      case Q4_0: rows = q3_rows<Q4_0>(M); break;
      case Q4_1: rows = q3_rows<Q4_1>(M); break;
      case Q8_0: rows = q3_rows<Q8_0>(M); break;
      case Q4_K: rows = q3_rows<Q4_K>(M); break;
      case Q5_K: rows = q3_rows<Q5_K>(M); break;
      case Q6_K: rows = q3_rows<Q6_K>(M); break;
      case FP8: rows = q3_rows<FP8>(M); break;
      case FP8B: rows = q3_rows<FP8B>(M); break;
      case INT8: rows = q3_rows<INT8>(M); break;
    }
    int tiles = 0;
    for (int i = 0; i < nparts; ++i) {
      if (parts[i].qtype != fmts[f]) continue;
      a.parts.p[a.parts.n++] = Part{static_cast<const unsigned char*>(parts[i].q), parts[i].rs, parts[i].qtype,
                                    parts[i].rows, parts[i].col, tiles};
      tiles += (parts[i].rows + rows - 1) / rows;
    }
    switch (fmts[f]) {
      case Q4_0: q3_launch_m<Q4_0>(a, tiles, Sx, s); break;
      case Q4_1: q3_launch_m<Q4_1>(a, tiles, Sx, s); break;
      case Q8_0: q3_launch_m<Q8_0>(a, tiles, Sx, s); break;
      case Q4_K: q3_launch_m<Q4_K>(a, tiles, Sx, s); break;
      case Q5_K: q3_launch_m<Q5_K>(a, tiles, Sx, s); break;
      case Q6_K: q3_launch_m<Q6_K>(a, tiles, Sx, s); break;
      case FP8: q3_launch_m<FP8>(a, tiles, Sx, s); break;
      case FP8B: q3_launch_m<FP8B>(a, tiles, Sx, s); break;
      case INT8: q3_launch_m<INT8>(a, tiles, Sx, s); break;
    }
  }
  return true;
}

}  // namespace hipserve
