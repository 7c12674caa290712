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
template <int kMode>
__global__ __launch_bounds__(256) void rope_cache_kernel(
    unsigned short* __restrict__ qkv, long qkv_stride,
    const long* __restrict__ positions, const long* __restrict__ slots,
    const float* __restrict__ cos_sin, unsigned short* __restrict__ k_cache,
    unsigned short* __restrict__ v_cache, int nq, int nkv, int D,
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
        unsigned short* kc = k_cache + ((blk * nkv + kh) * block_size + off) * (long)D;
        *reinterpret_cast<u16x8*>(kc + c * 8) = va;
        *reinterpret_cast<u16x8*>(kc + half + c * 8) = vb;
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
        unsigned short* kc = k_cache + ((blk * nkv + kh) * block_size + off) * (long)D;
        *reinterpret_cast<u16x8*>(kc + c * 8) = v;
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
      unsigned short* vc = v_cache + (blk * nkv + kh) * (long)D * block_size + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) vc[(c * 8 + j) * block_size] = v[j];
    }
  }
}

void launch_rope_cache(void* qkv, long qkv_stride, const long* positions,
                       const long* slots, const float* cos_sin, void* k_cache,
                       void* v_cache, int T, int nq, int nkv, int D,
                       int block_size, int mode, hipStream_t s) {
  if (T <= 0) return;
  dim3 grid(T), block(256);
  auto* q = static_cast<unsigned short*>(qkv);
  auto* kc = static_cast<unsigned short*>(k_cache);
  auto* vc = static_cast<unsigned short*>(v_cache);
  if (mode == 0)
    rope_cache_kernel<0><<<grid, block, 0, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, nq, nkv, D, block_size);
  else
    rope_cache_kernel<1><<<grid, block, 0, s>>>(q, qkv_stride, positions, slots, cos_sin, kc, vc, nq, nkv, D, block_size);
}

}  // namespace hipserve
