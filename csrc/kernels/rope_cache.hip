// Fused rotary embedding + paged KV-cache write.
//
// qkv:  [T, (nq + 2*nkv) * D] bf16 — the merged QKV projection output (row stride
//       given). Q is rotated in place; rotated K and raw V are scattered into the
//       paged cache at slot_mapping[t] (slot < 0 => padding token, skipped).
// Cache layouts (chosen for the MFMA attention kernels, see attention_decode.hip):
//   k_cache [num_blocks, nkv, block_size, D]   (token rows, d contiguous)
//   v_cache [num_blocks, nkv, D, block_size]   (transposed per block: tokens
//                                              contiguous, so PV B-fragments are
//                                              16-byte loads straight to VGPRs)
// cos_sin: [max_pos, D] fp32 = [cos(D/2) | sin(D/2)].
// mode: 0 = NeoX rotate-half (HF Llama), 1 = interleaved pairs (GGUF llama).
// KV: cache element, bf16 (unsigned short) or e4m3 (unsigned char, common.h kv_store*).
#include <cstdlib>

#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

template <int kMode>
HS_DEVICE void rotate8(float (&x)[8], float (&y)[8], const float* cs, int i0,
                       int half) {
  // NeoX: x = elems [i0, i0+8) of the first half, y = same of the second half.
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float c = cs[i0 + j], s = cs[half + i0 + j];
    const float a = x[j], b = y[j];
    rope_rot(a, b, c, s, x[j], y[j]);
  }
}

// One workgroup per token; threads stride over (head, 8-wide chunk) work items.
template <int kMode, typename KV>
__global__ __launch_bounds__(256) void rope_cache_kernel(
    unsigned short* __restrict__ qkv, long qkv_stride,
    const long* __restrict__ positions, const long* __restrict__ slots,
    const float* __restrict__ cos_sin, KV* __restrict__ k_cache,
    KV* __restrict__ v_cache, int nq, int nkv, int D,
    int block_size) {
  const int t = blockIdx.x;
  const long pos = positions[t];
  const long slot = slots[t];
  const int half = D / 2;
  const float* cs = cos_sin + pos * D;
  unsigned short* row = qkv + t * qkv_stride;
  const long blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? (int)(slot % block_size) : 0;

  if constexpr (kMode == 0) {
    // rotate-half: a work item = (head, chunk of 8 in the first half)
    const int chunks = half / 8;
    const int items = (nq + nkv) * chunks;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
      const int h = it / chunks, c = it % chunks;
      unsigned short* base = row + h * D;
      u16x8 va = *reinterpret_cast<u16x8*>(base + c * 8);
      u16x8 vb = *reinterpret_cast<u16x8*>(base + half + c * 8);
      float x[8], y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { x[j] = bf16_to_f32(va[j]); y[j] = bf16_to_f32(vb[j]); }
      rotate8<0>(x, y, cs, c * 8, half);
#pragma unroll
      for (int j = 0; j < 8; ++j) { va[j] = f32_to_bf16(x[j]); vb[j] = f32_to_bf16(y[j]); }
      if (h < nq) {
        *reinterpret_cast<u16x8*>(base + c * 8) = va;
        *reinterpret_cast<u16x8*>(base + half + c * 8) = vb;
      } else if (slot >= 0) {
        const int kh = h - nq;
        KV* kc = k_cache + ((blk * nkv + kh) * block_size + off) * (long)D;
        kv_store8(kc + c * 8, va);
        kv_store8(kc + half + c * 8, vb);
      }
    }
  } else {
    // interleaved pairs (2i, 2i+1): a work item = (head, chunk of 8 = 4 pairs)
    const int chunks = D / 8;
    const int items = (nq + nkv) * chunks;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
      const int h = it / chunks, c = it % chunks;
      unsigned short* base = row + h * D;
      u16x8 v = *reinterpret_cast<u16x8*>(base + c * 8);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int i = c * 4 + p;  // pair index
        const float co = cs[i], si = cs[half + i];
        const float a = bf16_to_f32(v[2 * p]), b = bf16_to_f32(v[2 * p + 1]);
        float ra, rb;
        rope_rot(a, b, co, si, ra, rb);
        v[2 * p] = f32_to_bf16(ra);
        v[2 * p + 1] = f32_to_bf16(rb);
      }
      if (h < nq) {
        *reinterpret_cast<u16x8*>(base + c * 8) = v;
      } else if (slot >= 0) {
        const int kh = h - nq;
        KV* kc = k_cache + ((blk * nkv + kh) * block_size + off) * (long)D;
        kv_store8(kc + c * 8, v);
      }
    }
  }
  // V: copy to the transposed cache block (tokens contiguous per d).
  if (slot >= 0) {
    const unsigned short* vrow = row + (nq + nkv) * D;
    const int chunks = D / 8;
    for (int it = threadIdx.x; it < nkv * chunks; it += blockDim.x) {
      const int kh = it / chunks, c = it % chunks;
      const u16x8 v = *reinterpret_cast<const u16x8*>(vrow + kh * D + c * 8);
      KV* vc = v_cache + (blk * nkv + kh) * (long)D * block_size + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) kv_store1(vc + (c * 8 + j) * block_size, v[j]);
    }
  }
}

// Prefill form: one workgroup per 16 consecutive tokens. q / k exactly as above
// (flattened (token, item) loop); V goes through LDS so that the 16 lanes of a group
// write 16 consecutive tokens of one V^T row of a block (32 contiguous bytes when the
// tokens share a block) instead of 64 lanes storing 2 bytes 32 bytes apart — the
// per-token kernel's scattered V stores cost about half of its time at 8K-token chunks.
constexpr int kRopeTile = 16;

template <int kMode, typename KV>
__global__ __launch_bounds__(256) void rope_cache_tile_kernel(
    unsigned short* __restrict__ qkv, long qkv_stride, const long* __restrict__ positions,
    const long* __restrict__ slots, const float* __restrict__ cos_sin, KV* __restrict__ k_cache,
    KV* __restrict__ v_cache, int T, int nq, int nkv, int D, int block_size, int vfast) {
  extern __shared__ __attribute__((aligned(16))) unsigned short vs[];  // [16][nkv * D + 8]
  const int t0 = blockIdx.x * kRopeTile;
  const int nt = min(kRopeTile, T - t0);
  const int half = D / 2;
  const int chunks = kMode == 0 ? half / 8 : D / 8;
  // thread -> (token, 8-wide chunk c, head parity): the chunk's cos / sin sit in
  // registers and are reused over every second q / k head of the token (the per-token
  // kernel re-read them from cache for each head: 4x the qkv bytes)
  const int nh = nq + nkv;
  const int per_tok = chunks * 2;
  for (int it = threadIdx.x; it < nt * per_tok; it += blockDim.x) {
    const int tt = it / per_tok, c = (it % per_tok) >> 1, hpar = it & 1;
    const int t = t0 + tt;
    const long pos = positions[t];
    const long slot = slots[t];
    const float* cs = cos_sin + pos * D;
    unsigned short* row = qkv + t * qkv_stride;
    const long blk = slot >= 0 ? slot / block_size : 0;
    const int off = slot >= 0 ? (int)(slot % block_size) : 0;
    if constexpr (kMode == 0) {
      float co[8], si[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { co[j] = cs[c * 8 + j]; si[j] = cs[half + c * 8 + j]; }
      // 4 heads per batch with all their loads issued first: the per-thread head
      // loop is otherwise one dependent memory round trip per head
      for (int h0 = hpar; h0 < nh; h0 += 8) {
        u16x8 va[4], vb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int h = min(h0 + 2 * q, nh - 1);
          va[q] = *reinterpret_cast<const u16x8*>(row + h * D + c * 8);
          vb[q] = *reinterpret_cast<const u16x8*>(row + h * D + half + c * 8);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int h = h0 + 2 * q;
          if (h >= nh || (h >= nq && slot < 0)) continue;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float ra, rb;
            rope_rot(bf16_to_f32(va[q][j]), bf16_to_f32(vb[q][j]), co[j], si[j], ra, rb);
            va[q][j] = f32_to_bf16(ra);
            vb[q][j] = f32_to_bf16(rb);
          }
          if (h < nq) {
            *reinterpret_cast<u16x8*>(row + h * D + c * 8) = va[q];
            *reinterpret_cast<u16x8*>(row + h * D + half + c * 8) = vb[q];
          } else {
            KV* dst = k_cache + ((blk * nkv + (h - nq)) * block_size + off) * (long)D;
            kv_store8(dst + c * 8, va[q]);
            kv_store8(dst + half + c * 8, vb[q]);
          }
        }
      }
    } else {
      float co[4], si[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) { co[p] = cs[c * 4 + p]; si[p] = cs[half + c * 4 + p]; }
      for (int h0 = hpar; h0 < nh; h0 += 8) {
        u16x8 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = *reinterpret_cast<const u16x8*>(row + min(h0 + 2 * q, nh - 1) * D + c * 8);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int h = h0 + 2 * q;
          if (h >= nh || (h >= nq && slot < 0)) continue;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            float ra, rb;
            rope_rot(bf16_to_f32(v[q][2 * p]), bf16_to_f32(v[q][2 * p + 1]), co[p], si[p], ra, rb);
            v[q][2 * p] = f32_to_bf16(ra);
            v[q][2 * p + 1] = f32_to_bf16(rb);
          }
          if (h < nq) *reinterpret_cast<u16x8*>(row + h * D + c * 8) = v[q];
          else kv_store8(k_cache + ((blk * nkv + (h - nq)) * block_size + off) * (long)D + c * 8, v[q]);
        }
      }
    }
  }
  // V rows of the tile -> LDS (16-byte loads), then token-fastest 2-byte stores
  const int VW = nkv * D, VR = VW + 8;  // LDS row stride: +16 B keeps the 16 token rows on distinct banks
  const int vchunks = VW / 8;
  for (int it = threadIdx.x; it < nt * vchunks; it += blockDim.x) {
    const int tt = it / vchunks, c = it % vchunks;
    *reinterpret_cast<u16x8*>(vs + tt * VR + c * 8) =
        *reinterpret_cast<const u16x8*>(qkv + (t0 + tt) * qkv_stride + (nq + nkv) * D + c * 8);
  }
  __syncthreads();
  // The 16 tokens usually fill 16 consecutive slots of one block (prefill of a
  // block-aligned sequence): each V^T row segment is then 32 contiguous bytes, written
  // as two 16-byte stores gathered from 8 LDS rows each (8 stores per thread instead
  // of 64 2-byte stores, each with its own slot load and 64-bit divide).
  const long s0 = slots[t0];
  const int off0 = s0 >= 0 ? (int)(s0 % block_size) : 1;
  bool contig = vfast && nt == kRopeTile && (block_size & 7) == 0 && (off0 & 7) == 0 && off0 + kRopeTile <= block_size;
  for (int i = 1; contig && i < kRopeTile; ++i) contig = slots[t0 + i] == s0 + i;  // block-uniform
  if (contig) {
    const long blk = s0 / block_size;
    for (int it = threadIdx.x; it < 2 * VW; it += blockDim.x) {
      const int r = it >> 1, hl = it & 1;
      const int kh = r / D, d = r % D;
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = vs[(hl * 8 + j) * VR + r];
      kv_store8(v_cache + (blk * nkv + kh) * (long)D * block_size + (long)d * block_size + off0 + hl * 8, v);
    }
    return;
  }
  // general case: lane -> one token (blockDim.x % 16 == 0), its slot decoded once
  const int tt = threadIdx.x & (kRopeTile - 1);
  const long slot = tt < nt ? slots[t0 + tt] : -1;
  if (slot < 0) return;  // after the only barrier
  const long blk = slot / block_size;
  const int off = (int)(slot % block_size);
  for (int r = threadIdx.x / kRopeTile; r < VW; r += blockDim.x / kRopeTile) {
    const int kh = r / D, d = r % D;
    kv_store1(v_cache + (blk * nkv + kh) * (long)D * block_size + (long)d * block_size + off, vs[tt * VR + r]);
  }
}

static bool rope_tile_enabled() {
  static const bool on = [] {
    const char* e = getenv("HIPSERVE_ROPE_TILE");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static int rope_vfast() {  // HIPSERVE_ROPE_VFAST=0: 2-byte V^T stores for every tile (A/B)
  static const int on = [] {
    const char* e = getenv("HIPSERVE_ROPE_VFAST");
    return !(e && atoi(e) == 0) ? 1 : 0;
  }();
  return on;
}

template <typename KV>
static void rope_cache_t(unsigned short* q, long qkv_stride, const long* positions, const long* slots,
                         const float* cos_sin, KV* kc, KV* vc, int T, int nq, int nkv, int D, int block_size,
                         int mode, hipStream_t s) {
  // prefill chunks: the tile kernel (one workgroup per 16 tokens) only once there are
  // >= 128 of them; below that the per-token kernel's wider grid wins (tools/bench_rope.py:
  // 256 tokens 6-7 vs 13-17 us, 1,024 tokens within +-2 us, 4,096 tokens 23-33 vs 32-51 us)
  if (T >= 2048 && nkv * D <= 2048 && rope_tile_enabled()) {
    const dim3 tg((T + kRopeTile - 1) / kRopeTile);
    const size_t smem = (size_t)kRopeTile * (nkv * D + 8) * sizeof(unsigned short);
    if (mode == 0)
      rope_cache_tile_kernel<0, KV><<<tg, 256, smem, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, T, nq,
                                                          nkv, D, block_size, rope_vfast());
    else
      rope_cache_tile_kernel<1, KV><<<tg, 256, smem, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, T, nq,
                                                          nkv, D, block_size, rope_vfast());
    return;
  }
  if (mode == 0)
    rope_cache_kernel<0, KV><<<T, 256, 0, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, nq, nkv, D,
                                               block_size);
  else
    rope_cache_kernel<1, KV><<<T, 256, 0, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, nq, nkv, D,
                                               block_size);
}

void launch_rope_cache(void* qkv, long qkv_stride, const long* positions,
                       const long* slots, const float* cos_sin, void* k_cache,
                       void* v_cache, int T, int nq, int nkv, int D,
                       int block_size, int mode, hipStream_t s, bool kv_f8) {
  if (T <= 0) return;
  auto* q = static_cast<unsigned short*>(qkv);
  if (kv_f8)
    rope_cache_t(q, qkv_stride, positions, slots, cos_sin, static_cast<unsigned char*>(k_cache),
                 static_cast<unsigned char*>(v_cache), T, nq, nkv, D, block_size, mode, s);
  else
    rope_cache_t(q, qkv_stride, positions, slots, cos_sin, static_cast<unsigned short*>(k_cache),
                 static_cast<unsigned short*>(v_cache), T, nq, nkv, D, block_size, mode, s);
}

}  // namespace hipserve
