// Shared device helpers of the tiled quantised-weight kernels (gguf_mfma.hip: the v2
// decode GEMM, K15 / qpg prefill, dequant; fp8_decode.hip):
// the per-format tiled chunk layouts, raw loads, and the subnormal-integer dequant.
#pragma once

#include "hipserve/common.h"

namespace hipserve {
namespace gq {


// GGUF block formats + FP8 e4m3 weights (per-row scale; FP8B adds 128 x 128 block
// scales, the block-FP8 checkpoints)
// INT8: unsigned 8-bit weights (compressed-tensors pack-quantized / AWQ 8-bit) with
// a group scale and zero point per half lane-quarter (32 k): w = (u - 128 - zp) * s.
// INT8C: the per-channel symmetric case (one scale per row, no zero point — the
// reference's AWQ-8bit / W8A16 exports): the bytes alone, the row scale applied to the
// fp32 accumulators in the epilogue as for FP8 (11 % fewer bytes than INT8's per-32-k
// scale / offset table, and the integers enter the MFMA exactly)
enum { Q4_0 = 0, Q4_1 = 1, Q8_0 = 2, Q4_K = 3, Q5_K = 4, Q6_K = 5, FP8 = 6, FP8B = 7, INT8 = 8, INT8C = 9 };

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr unsigned kMagic = 0x64006400u;  // f16 pair (1024, 1024)
// x in LDS: 4 planes (lane group g) of [row][8 fragments of 8 f16 + 8 pad]: a row is
// 36 words (36 / 4 = 9, odd) and a plane a multiple of 64 words, so the 16 lanes of
// each ds_read_b128 lane group (rows c, planes g) land on 16 distinct 4-bank slots
// (slot = 9 c + s mod 16): conflict-free (the plain [row][256 + 8] image was 2-way)
constexpr int kXR = 72;  // row stride in f16 (8 fragments x 8 + 8 pad)
template <int MT>
constexpr int x_plane() { return 16 * MT * kXR; }

HS_DEVICE h2 as_h2(unsigned u) { return __builtin_bit_cast(h2, u); }
HS_DEVICE unsigned as_u(h2 h) { return __builtin_bit_cast(unsigned, h); }
HS_DEVICE float h2f(unsigned short h) { return static_cast<float>(__builtin_bit_cast(_Float16, h)); }
HS_DEVICE h2 splat(float f) {
  const _Float16 v = static_cast<_Float16>(f);
  return h2{v, v};
}
HS_DEVICE u32x4 ld16(const unsigned char* p) { return *reinterpret_cast<const u32x4*>(p); }

// the 16-byte fragment of 8 f16 values from 4 packed pairs
HS_DEVICE f16x8 frag(h2 a, h2 b, h2 c, h2 d) {
  return __builtin_bit_cast(f16x8, u32x4{as_u(a), as_u(b), as_u(c), as_u(d)});
}

// nibbles at bit offset sh of bytes (0, 2) and (1, 3) of w -> 1024 + q pairs
HS_DEVICE void nib_pairs(unsigned w, int sh, unsigned& p02, unsigned& p13) {
  p02 = ((w >> sh) & 0x000F000Fu) | kMagic;
  p13 = ((w >> (sh + 8)) & 0x000F000Fu) | kMagic;
}

struct Raw {
  u32x4 v[5];
  unsigned s2[2];  // Q6_K: the lane's 4 int8 sub-block scales (2 words, 2 bytes used each)
  unsigned short h[4];
};

// Tiled weight layout (hipserve/ops/quant.py repack_tiled): a part is
// [N/16 row groups][K/256 super-chunks][CB bytes]; one chunk = the 16 rows x 256 k a
// wave multiplies, arranged so every lane-specific 16-byte load of the wave is one
// fully coalesced 1 KiB access (lane = 16 g + c: row c, k quarter g):
//   Q4_K  [16 hdr x 16][2 x 64 lanes x 16 qs]                       2304 B
//   Q5_K  Q4_K + [16 rows x 32 qh]                                  2816 B
//   Q6_K  [2 x 64 lanes x 16 ql][16 rows x 64 qh][16 x 16 scales][16 x 2 d]  3360 B
//   Q8_0  [4 x 64 lanes x 16 q][16 rows x 8 d]                      4352 B
//   Q4_0  [2 x 64 lanes x 16 q][16 rows x 8 d]                      2304 B
//   Q4_1  Q4_0 + [16 rows x 8 m]                                    2560 B
//   FP8   [4 x 64 lanes x 16 q]                                     4096 B
//   FP8B  FP8 + [16 rows x 2 f32 block scales]                      4224 B
//   INT8  [4 x 64 lanes x 16 u8][16 rows x 4 g x 2 halves x (f16 scale, f16 offset)]  4608 B
//   INT8C [4 x 64 lanes x 16 u8]                                    4096 B
template <int QT>
constexpr int chunk_bytes() {
  return QT == Q4_K ? 2304 : QT == Q5_K ? 2816 : QT == Q6_K ? 3360 : QT == Q8_0 ? 4352 : QT == Q4_0 ? 2304
       : QT == Q4_1 ? 2560 : QT == FP8 || QT == INT8C ? 4096 : QT == FP8B ? 4224 : 4608;
}
// formats whose per-row scale (Part::rs) multiplies the accumulators in the epilogue
template <int QT>
constexpr bool row_scaled() { return QT == FP8 || QT == FP8B || QT == INT8C; }

struct Part {
  const unsigned char* q;
  const float* rs;  // per-row output scale (FP8, INT8C), nullptr for GGUF formats
  int qt;       // format of the part
  int rows;     // N of the part (multiple of 16)
  int col;      // first output column
  int tile0;    // first tile index of the part in the launch
};
constexpr int kMaxParts = 4;
// 4-wave workgroups of 2 row groups per wave (128 rows): occupancy then comes in
// 4-wave steps, so a 150-VGPR body still runs 3 workgroups (12 waves) per CU
constexpr int kWaves = 4;
struct Parts {
  Part p[kMaxParts];
  int n;
};
// MoE expert tiles (moe_align, moe.hip): the workgroup's blockIdx.z is one tile of
// 16 * MT expert-sorted pair slots; its x rows are gathered (token = pair / gather_k,
// or the slot itself for w2 over the activations) and its outputs land on slot rows
struct MoeQ {
  const int* slots;        // [nslots] pair index (token * k + j) or -1 (padding)
  const int* tile_expert;  // [tiles_cap] expert of each tile, -1 past the last tile
  long w_estride;          // bytes of one expert's tiled weight
  long rs_estride;         // floats of one expert's row scales (FP8, INT8C), 0 otherwise
  int gather_k;            // > 0: x row = pair / gather_k; 0: x row = slot
  int nslots;              // slot rows of out / of each ws split
  int kmajor = 0;          // expert weights [K/256][N/16][chunk] (super-chunk major), else [N/16][K/256][chunk]
  int glu = 0;             // 1 / 2: SiLU / GELU-tanh GLU epilogue (w13 rows = gate | up; out [slots, N / 2])
};

template <int QT>
HS_DEVICE void load_raw(const unsigned char* ch, int g, int c, int lane, Raw& r) {
  if constexpr (QT == Q4_K || QT == Q5_K) {
    r.v[0] = ld16(ch + 16 * c);  // d, dmin, 12 B of 6-bit scales / mins
    r.v[1] = ld16(ch + 256 + 16 * lane);
    r.v[2] = ld16(ch + 1280 + 16 * lane);
    if constexpr (QT == Q5_K) {
      r.v[3] = ld16(ch + 2304 + 32 * c);
      r.v[4] = ld16(ch + 2320 + 32 * c);
    }
  } else if constexpr (QT == Q6_K) {
    r.v[0] = ld16(ch + 16 * lane);
    r.v[1] = ld16(ch + 1024 + 16 * lane);
    r.v[2] = ld16(ch + 2048 + 64 * c + 32 * (g >> 1));
    r.v[3] = ld16(ch + 2064 + 64 * c + 32 * (g >> 1));
    const uint2 sc = *reinterpret_cast<const uint2*>(ch + 3072 + 16 * c + 8 * (g >> 1));  // scales 8h..8h+7
    r.s2[0] = sc.x;
    r.s2[1] = sc.y;
    r.h[0] = *reinterpret_cast<const unsigned short*>(ch + 3328 + 2 * c);
  } else if constexpr (QT == INT8) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = ld16(ch + 1024 * i + 16 * lane);
    const uint2 so = *reinterpret_cast<const uint2*>(ch + 4096 + 32 * c + 8 * g);  // (sA, oA), (sB, oB)
    r.s2[0] = so.x;
    r.s2[1] = so.y;
  } else if constexpr (QT == FP8 || QT == FP8B || QT == INT8C) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = ld16(ch + 1024 * i + 16 * lane);
    if constexpr (QT == FP8B)  // the lane's 64 k sit in 128-block (g >> 1) of this super-chunk
      r.s2[0] = *reinterpret_cast<const unsigned*>(ch + 4096 + 8 * c + 4 * (g >> 1));
  } else if constexpr (QT == Q8_0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) r.v[i] = ld16(ch + 1024 * i + 16 * lane);
    const unsigned dd = *reinterpret_cast<const unsigned*>(ch + 4096 + 16 * c + 4 * g);
    r.h[0] = dd & 0xFFFF;
    r.h[1] = dd >> 16;
  } else {  // Q4_0 / Q4_1
    r.v[0] = ld16(ch + 16 * lane);
    r.v[1] = ld16(ch + 1024 + 16 * lane);
    const unsigned dd = *reinterpret_cast<const unsigned*>(ch + 2048 + 16 * c + 4 * g);
    r.h[0] = dd & 0xFFFF;
    r.h[1] = dd >> 16;
    if constexpr (QT == Q4_1) {
      const unsigned mm = *reinterpret_cast<const unsigned*>(ch + 2304 + 16 * c + 4 * g);
      r.h[2] = mm & 0xFFFF;
      r.h[3] = mm >> 16;
    }
  }
}

HS_DEVICE unsigned word(const u32x4 (&v)[2], int i) { return v[i >> 2][i & 3]; }  // i in [0, 8)

// 6-bit scale / min j of a K-quant super-block from its 12 packed bytes (words
// w1 w2 w3 = bytes 0-3, 4-7, 8-11). j is lane-dependent: bytes are picked with
// shifts by 8 (j & 3) (every byte used sits at j, j +- 4), never by indexing a
// register array (that becomes compare/select chains).
HS_DEVICE void scale_min_k4(int j, unsigned w1, unsigned w2, unsigned w3, float& sc, float& mn) {
  const int sh = 8 * (j & 3);
  const unsigned lo = (w1 >> sh) & 0xFF, mid = (w2 >> sh) & 0xFF, hi = (w3 >> sh) & 0xFF;
  const unsigned s_hi = (hi & 0xF) | ((lo >> 6) << 4), m_hi = (hi >> 4) | ((mid >> 6) << 4);
  sc = (float)(j < 4 ? (lo & 63) : s_hi);
  mn = (float)(j < 4 ? (mid & 63) : m_hi);
}

// k of element j (fragment order) of step s, lane group g: contiguous 8-runs whose
// base matches v1's kbase; inside a run the pair order {0, 2, 1, 3, 4, 6, 5, 7}
template <int QT>
HS_DEVICE int kbase(int g, int s) {
  if constexpr (QT == Q6_K) {
    const int q = (g & 1) + 2 * (s >> 2);
    return 128 * (g >> 1) + 32 * q + 8 * (s & 3);
  } else {
    return 64 * g + 32 * (s >> 2) + 8 * (s & 3);
  }
}

// Subnormal-integer dequant (Dec::sub_ints / step): the integer q of a weight is
// placed at bit kSub of an f16 (q << kSub < 1024: a subnormal, exactly q 2^(kSub-24)),
// and ONE v_pk_fma per pair computes q * (d 2^(24-kSub)) + c, where c holds the
// format's zero point (-8 d, -32 d, -128 d) or the K-quant min. Every factor is a
// power-of-two multiple of the f16-rounded scale, so for scales in the f16 normal range
// the weights are bit-identical to the magic-number path (1024 + q, v_pk_add -1024,
// v_pk_fma) at 2 instead of 3 ops per pair word and no v_pk_add. NOT bit-identical when
// a block's d sc is itself f16-subnormal (< 2^-14 ~ 6.1e-5): there d sc 2^(24-kSub) is a
// normal f16 that keeps more mantissa bits than the magic path's subnormal scale, so v2
// is the closer of the two to the fp32 block decoder (tests/test_gguf_gpu.py
// test_mfma_v2_tiny_scales). Range: d 2^(24-kSub) must stay below 65504 —
// ops/quant.py sub_scale_ok() checks every block's scale at load (Q4_K / Q4_0 / Q4_1
// d sc < 0.25, Q5_K < 0.125, Q6_K < 0.0625, Q8_0 < 0.0156) and sends weights beyond
// it to the v1 kernel.
template <int QT>
constexpr int sub_shift() { return QT == Q5_K ? 5 : QT == Q6_K ? 4 : QT == Q8_0 ? 2 : 6; }
template <int QT>
constexpr float sub_up() {
  return QT == Q4_K || QT == Q5_K || QT == Q6_K || QT == Q8_0 || QT == Q4_0 || QT == Q4_1
             ? (float)(1 << (24 - sub_shift<QT>())) : 1.f;
}
template <int QT>
constexpr float sub_zero() { return QT == Q4_0 ? -8.f : QT == Q6_K ? -32.f : QT == Q8_0 ? -128.f : 0.f; }

// Decode step s (8 weights) of the lane's super-chunk. ints(): the 8 quantised
// integers (minus the format's zero point) as exact f16, pair order; step(): the
// weights in f16 (one v_pk_fma per pair with the block scale / min); scale():
// the same scale / min in fp32 for the exact bf16 dequant of the prefill path.
template <int QT>
struct Dec {
  h2 dA, cA, dB, cB;        // per-step-group scale / offset pairs (K-quants: sub-blocks; SoA: blocks)
  float fdA, fcA, fdB, fcB;  // the same in fp32
  float d6;                  // Q6_K super-block scale

  HS_DEVICE void setup(const Raw& r, int g) {
    fcA = fcB = 0.f;
    if constexpr (QT == Q4_K || QT == Q5_K) {
      const u32x4 hdr = r.v[0];
      const float d = h2f(hdr[0] & 0xFFFF), dmin = h2f(hdr[0] >> 16);
      float s1, m1, s2, m2;
      scale_min_k4(2 * g, hdr[1], hdr[2], hdr[3], s1, m1);
      scale_min_k4(2 * g + 1, hdr[1], hdr[2], hdr[3], s2, m2);
      fdA = d * s1;
      fcA = -dmin * m1;
      fdB = d * s2;
      fcB = -dmin * m2;
    } else if constexpr (QT == Q6_K) {
      d6 = h2f(r.h[0]);
    } else if constexpr (QT == FP8 || QT == FP8B || QT == INT8C) {
      fdA = fdB = QT == FP8B ? __builtin_bit_cast(float, r.s2[0]) : 1.f;
    } else if constexpr (QT == INT8) {  // c = offset (-1024 - 128 - zp), applied before the scale
      fdA = h2f(r.s2[0] & 0xFFFF);
      fcA = h2f(r.s2[0] >> 16);
      fdB = h2f(r.s2[1] & 0xFFFF);
      fcB = h2f(r.s2[1] >> 16);
    } else {
      fdA = h2f(r.h[0]);
      fdB = h2f(r.h[1]);
      if constexpr (QT == Q4_1) {
        fcA = h2f(r.h[2]);
        fcB = h2f(r.h[3]);
      }
    }
    // step(): integers enter as subnormal f16 q 2^(kSub - 24) (sub_ints), so the
    // scale pairs carry 2^(24 - kSub) and the zero point moves into the FMA addend
    // (exact: power-of-two multiples of the f16-rounded scale)
    constexpr float up = sub_up<QT>(), zp = sub_zero<QT>();
    dA = splat(fdA * up);
    dB = splat(fdB * up);
    if constexpr (QT == Q4_0 || QT == Q8_0) {
      cA = splat(zp * (float)(_Float16)fdA);
      cB = splat(zp * (float)(_Float16)fdB);
    } else {
      cA = splat(fcA);
      cB = splat(fcB);
    }
  }

  HS_DEVICE void scale(const Raw& r, int g, int s, float& d, float& c) const {
    if constexpr (QT == Q6_K) {
      // sub-block 8h + 2q + ((s & 3) >> 1), q = (g & 1) + 2 (s >> 2): byte 2 (g & 1) + ((s & 3) >> 1)
      // of the lane's scale word (s >> 2)
      d = d6 * (float)(signed char)((r.s2[s >> 2] >> (8 * (2 * (g & 1) + ((s & 3) >> 1)))) & 0xFF);
      c = 0.f;
    } else if constexpr (QT == INT8) {
      d = s < 4 ? fdA : fdB;
      c = 0.f;
    } else if constexpr (QT == Q4_K || QT == Q5_K || QT == Q8_0) {
      d = s < 4 ? fdA : fdB;
      c = s < 4 ? fcA : fcB;
    } else {
      d = (s >> 2) ? fdB : fdA;
      c = (s >> 2) ? fcB : fcA;
    }
  }

  HS_DEVICE f16x8 ints(const Raw& r, int g, int s) const {
    if constexpr (QT == INT8C) {  // u - 128 exact: (1024 + u) - 1152
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)], wb = qv[s >> 1][2 * (s & 1) + 1];
      const h2 cc = splat(-1152.f);
      const unsigned p0 = (wa & 0x00FF00FFu) | kMagic, p1 = ((wa >> 8) & 0x00FF00FFu) | kMagic;
      const unsigned p2 = (wb & 0x00FF00FFu) | kMagic, p3 = ((wb >> 8) & 0x00FF00FFu) | kMagic;
      return frag(as_h2(p0) + cc, as_h2(p1) + cc, as_h2(p2) + cc, as_h2(p3) + cc);
    }
    if constexpr (QT == INT8) {  // u - 128 - zp, exact
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)], wb = qv[s >> 1][2 * (s & 1) + 1];
      const h2 cc = s < 4 ? cA : cB;
      const unsigned p0 = (wa & 0x00FF00FFu) | kMagic, p1 = ((wa >> 8) & 0x00FF00FFu) | kMagic;
      const unsigned p2 = (wb & 0x00FF00FFu) | kMagic, p3 = ((wb >> 8) & 0x00FF00FFu) | kMagic;
      return frag(as_h2(p0) + cc, as_h2(p1) + cc, as_h2(p2) + cc, as_h2(p3) + cc);
    }
    if constexpr (QT == FP8 || QT == FP8B) {
      // e4m3 -> f16 by moving bits: sign to bit 15, exponent + mantissa to bits 7-13
      // gives the value / 256 exactly (normals and subnormals; the 256 is folded into
      // the row scale). Bytes (0, 2) and (1, 3) of a word pair up as in the GGUF paths.
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)], wb = qv[s >> 1][2 * (s & 1) + 1];
      const unsigned p0 = ((wa << 7) & 0x3F803F80u) | ((wa << 8) & 0x80008000u);
      const unsigned p1 = ((wa >> 1) & 0x3F803F80u) | (wa & 0x80008000u);
      const unsigned p2 = ((wb << 7) & 0x3F803F80u) | ((wb << 8) & 0x80008000u);
      const unsigned p3 = ((wb >> 1) & 0x3F803F80u) | (wb & 0x80008000u);
      return frag(as_h2(p0), as_h2(p1), as_h2(p2), as_h2(p3));
    }
    unsigned p[4];
    _Float16 z;  // 1024 + zero point
    if constexpr (QT == Q4_K || QT == Q5_K) {
      const u32x4 qs[2] = {r.v[1], r.v[2]};
      const int sh = s < 4 ? 0 : 4;
      const unsigned wa = word(qs, 2 * (s & 3)), wb = word(qs, 2 * (s & 3) + 1);
      nib_pairs(wa, sh, p[0], p[1]);
      nib_pairs(wb, sh, p[2], p[3]);
      if constexpr (QT == Q5_K) {  // + 16 where the high bit of the element is set
        const u32x4 qh[2] = {r.v[3], r.v[4]};
        const int bit = 2 * g + (s >> 2);
        const unsigned ha = word(qh, 2 * (s & 3)), hb = word(qh, 2 * (s & 3) + 1);
        p[0] |= ((ha >> bit) & 0x00010001u) << 4;
        p[1] |= ((ha >> (bit + 8)) & 0x00010001u) << 4;
        p[2] |= ((hb >> bit) & 0x00010001u) << 4;
        p[3] |= ((hb >> (bit + 8)) & 0x00010001u) << 4;
      }
      z = (_Float16)1024.f;
    } else if constexpr (QT == Q6_K) {
      const u32x4 ql[2] = {r.v[0], r.v[1]};
      const u32x4 qh[2] = {r.v[2], r.v[3]};
      const int q = (g & 1) + 2 * (s >> 2);
      const int sh = s < 4 ? 0 : 4;
      const unsigned la = word(ql, 2 * (s & 3)), lb = word(ql, 2 * (s & 3) + 1);
      const unsigned ha = word(qh, 2 * (s & 3)) >> (2 * q), hb = word(qh, 2 * (s & 3) + 1) >> (2 * q);
      nib_pairs(la, sh, p[0], p[1]);
      nib_pairs(lb, sh, p[2], p[3]);
      p[0] |= (ha & 0x00030003u) << 4;
      p[1] |= ((ha >> 8) & 0x00030003u) << 4;
      p[2] |= (hb & 0x00030003u) << 4;
      p[3] |= ((hb >> 8) & 0x00030003u) << 4;
      z = (_Float16)1056.f;  // q6 - 32
    } else if constexpr (QT == Q8_0) {
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)] ^ 0x80808080u, wb = qv[s >> 1][2 * (s & 1) + 1] ^ 0x80808080u;
      p[0] = (wa & 0x00FF00FFu) | kMagic;
      p[1] = ((wa >> 8) & 0x00FF00FFu) | kMagic;
      p[2] = (wb & 0x00FF00FFu) | kMagic;
      p[3] = ((wb >> 8) & 0x00FF00FFu) | kMagic;
      z = (_Float16)1152.f;  // int8 value
    } else {  // Q4_0 / Q4_1: block (s >> 2); elements 0-15 low nibbles, 16-31 high
      const u32x4 v[2] = {r.v[0], r.v[1]};
      const int blk = s >> 2, e = s & 3;
      const int sh = e < 2 ? 0 : 4;
      const unsigned wa = word(v, 4 * blk + 2 * (e & 1)), wb = word(v, 4 * blk + 2 * (e & 1) + 1);
      nib_pairs(wa, sh, p[0], p[1]);
      nib_pairs(wb, sh, p[2], p[3]);
      z = (_Float16)(QT == Q4_0 ? 1032.f : 1024.f);  // q - 8 / q
    }
    const h2 off = h2{-z, -z};
    return frag(as_h2(p[0]) + off, as_h2(p[1]) + off, as_h2(p[2]) + off, as_h2(p[3]) + off);
  }

  // the 8 quantised integers of step s as SUBNORMAL f16 q * 2^(kSub - 24) (exact:
  // q << kSub < 1024 stays in the mantissa), pair order; no magic-number OR and no
  // zero-point subtraction: the step's one v_pk_fma applies scale, zero point and min
  HS_DEVICE f16x8 sub_ints(const Raw& r, int g, int s) const {
    constexpr int S = sub_shift<QT>();
    unsigned p[4];
    if constexpr (QT == Q4_K || QT == Q5_K || QT == Q4_0 || QT == Q4_1) {
      unsigned wa, wb;
      int sh;
      if constexpr (QT == Q4_K || QT == Q5_K) {
        const u32x4 qs[2] = {r.v[1], r.v[2]};
        sh = s < 4 ? 0 : 4;
        wa = word(qs, 2 * (s & 3));
        wb = word(qs, 2 * (s & 3) + 1);
      } else {
        const u32x4 v[2] = {r.v[0], r.v[1]};
        const int blk = s >> 2, e = s & 3;
        sh = e < 2 ? 0 : 4;
        wa = word(v, 4 * blk + 2 * (e & 1));
        wb = word(v, 4 * blk + 2 * (e & 1) + 1);
      }
      constexpr unsigned m = 0x000F000Fu << S;
      // nibble at bit sh of bytes (0, 2) / (1, 3) moved to bit S: one shift + one and
      p[0] = (sh <= S ? wa << (S - sh) : wa >> (sh - S)) & m;
      p[1] = (wa >> (sh + 8 - S)) & m;
      p[2] = (sh <= S ? wb << (S - sh) : wb >> (sh - S)) & m;
      p[3] = (wb >> (sh + 8 - S)) & m;
      if constexpr (QT == Q5_K) {  // + 16 where the high bit of the element is set
        const u32x4 qh[2] = {r.v[3], r.v[4]};
        const int bit = 2 * g + (s >> 2);
        const unsigned ha = word(qh, 2 * (s & 3)), hb = word(qh, 2 * (s & 3) + 1);
        p[0] |= ((ha >> bit) & 0x00010001u) << (4 + S);
        p[1] |= ((ha >> (bit + 8)) & 0x00010001u) << (4 + S);
        p[2] |= ((hb >> bit) & 0x00010001u) << (4 + S);
        p[3] |= ((hb >> (bit + 8)) & 0x00010001u) << (4 + S);
      }
    } else if constexpr (QT == Q6_K) {
      const u32x4 ql[2] = {r.v[0], r.v[1]};
      const u32x4 qh[2] = {r.v[2], r.v[3]};
      const int q = (g & 1) + 2 * (s >> 2);
      const int sh = s < 4 ? 0 : 4;
      const unsigned la = word(ql, 2 * (s & 3)), lb = word(ql, 2 * (s & 3) + 1);
      const unsigned ha = word(qh, 2 * (s & 3)) >> (2 * q), hb = word(qh, 2 * (s & 3) + 1) >> (2 * q);
      constexpr unsigned m = 0x000F000Fu << S;
      p[0] = ((sh <= S ? la << (S - sh) : la >> (sh - S)) & m) | ((ha & 0x00030003u) << (4 + S));
      p[1] = ((la >> (sh + 8 - S)) & m) | (((ha >> 8) & 0x00030003u) << (4 + S));
      p[2] = ((sh <= S ? lb << (S - sh) : lb >> (sh - S)) & m) | ((hb & 0x00030003u) << (4 + S));
      p[3] = ((lb >> (sh + 8 - S)) & m) | (((hb >> 8) & 0x00030003u) << (4 + S));
    } else {  // Q8_0: int8 + 128 in [0, 255]
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)] ^ 0x80808080u, wb = qv[s >> 1][2 * (s & 1) + 1] ^ 0x80808080u;
      constexpr unsigned m = 0x00FF00FFu << S;
      p[0] = (wa << S) & m;
      p[1] = (wa >> (8 - S)) & m;
      p[2] = (wb << S) & m;
      p[3] = (wb >> (8 - S)) & m;
    }
    return frag(as_h2(p[0]), as_h2(p[1]), as_h2(p[2]), as_h2(p[3]));
  }

  HS_DEVICE f16x8 step(const Raw& r, int g, int s) const {
    if constexpr (QT == Q4_K || QT == Q5_K || QT == Q6_K || QT == Q8_0 || QT == Q4_0 || QT == Q4_1) {
      const u32x4 qu = __builtin_bit_cast(u32x4, sub_ints(r, g, s));
      h2 dd, cc;
      if constexpr (QT == Q6_K) {
        float d, c;
        scale(r, g, s, d, c);
        dd = splat(d * sub_up<QT>());
        cc = splat(sub_zero<QT>() * (float)(_Float16)d);
      } else if constexpr (QT == Q4_0 || QT == Q4_1) {
        dd = (s >> 2) ? dB : dA;
        cc = (s >> 2) ? cB : cA;
      } else {
        dd = s < 4 ? dA : dB;
        cc = s < 4 ? cA : cB;
      }
      return frag(as_h2(qu[0]) * dd + cc, as_h2(qu[1]) * dd + cc, as_h2(qu[2]) * dd + cc, as_h2(qu[3]) * dd + cc);
    }
    if constexpr (QT == INT8) {  // (1024 + u + off) * s: exact integer, one rounding
      const u32x4 qv[4] = {r.v[0], r.v[1], r.v[2], r.v[3]};
      const unsigned wa = qv[s >> 1][2 * (s & 1)], wb = qv[s >> 1][2 * (s & 1) + 1];
      const h2 dd = s < 4 ? dA : dB, cc = s < 4 ? cA : cB;
      const unsigned p0 = (wa & 0x00FF00FFu) | kMagic, p1 = ((wa >> 8) & 0x00FF00FFu) | kMagic;
      const unsigned p2 = (wb & 0x00FF00FFu) | kMagic, p3 = ((wb >> 8) & 0x00FF00FFu) | kMagic;
      return frag((as_h2(p0) + cc) * dd, (as_h2(p1) + cc) * dd, (as_h2(p2) + cc) * dd, (as_h2(p3) + cc) * dd);
    }
    const f16x8 q = ints(r, g, s);
    if constexpr (QT == FP8 || QT == INT8C) return q;  // row scale in the epilogue
    if constexpr (QT == FP8B) {
      const u32x4 qu = __builtin_bit_cast(u32x4, q);
      return frag(as_h2(qu[0]) * dA, as_h2(qu[1]) * dA, as_h2(qu[2]) * dA, as_h2(qu[3]) * dA);
    }
    h2 dd, cc;
    if constexpr (QT == Q6_K) {
      float d, c;
      scale(r, g, s, d, c);
      dd = splat(d);
      cc = h2{(_Float16)0.f, (_Float16)0.f};
    } else if constexpr (QT == Q4_0 || QT == Q4_1) {
      dd = (s >> 2) ? dB : dA;
      cc = (s >> 2) ? cB : cA;
    } else {
      dd = s < 4 ? dA : dB;
      cc = s < 4 ? cA : cB;
    }
    const u32x4 qu = __builtin_bit_cast(u32x4, q);
    if constexpr (QT == Q6_K || QT == Q8_0 || QT == Q4_0)  // no min term
      return frag(as_h2(qu[0]) * dd, as_h2(qu[1]) * dd, as_h2(qu[2]) * dd, as_h2(qu[3]) * dd);
    else
      return frag(as_h2(qu[0]) * dd + cc, as_h2(qu[1]) * dd + cc, as_h2(qu[2]) * dd + cc, as_h2(qu[3]) * dd + cc);
  }
};

// bf16 word halves -> fp32 (exact: one shift or mask)
HS_DEVICE float bf_lo(unsigned w) { return __builtin_bit_cast(float, w << 16); }
HS_DEVICE float bf_hi(unsigned w) { return __builtin_bit_cast(float, w & 0xFFFF0000u); }

}  // namespace gq
}  // namespace hipserve
