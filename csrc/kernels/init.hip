// On-device synthetic weight init: a 70B model is 140 GB of
// bf16 and must never be generated on the host.
//
// value(r, c) = bf16(((h >> 8) * 2^-24 - 0.5) * 2 * scale),
//   h = mix32(mix32(gr * gcols + gc) ^ key),  gr = row0 + r, gc = col0 + c
//
// Keyed by the element's GLOBAL (unsharded) coordinates, so every TP rank fills
// exactly its shard of the same full matrix: dummy weights are identical for any
// TP degree (and bit-identical to ops/reference.py's torch version — only exact
// fp32 multiplies/subtractions and a round-to-nearest-even bf16 conversion).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

HS_DEVICE unsigned int mix32(unsigned int x) {  // "lowbias32" finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void fill_uniform_kernel(unsigned short* __restrict__ out, long ld, int rows,
                                                           int cols, long row0, long col0, long gcols,
                                                           unsigned int key, float scale) {
  const long n = (long)rows * cols;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / cols), c = (int)(i - (long)r * cols);
    const unsigned int idx = (unsigned int)((row0 + r) * gcols + (col0 + c));
    const unsigned int h = mix32(mix32(idx) ^ key);
    const float u = (float)(h >> 8) * 5.9604644775390625e-08f;  // 2^-24, exact
    out[r * ld + c] = f32_to_bf16((u - 0.5f) * (2.0f * scale));
  }
}

void launch_fill_uniform(void* out, long ld, int rows, int cols, long row0, long col0, long gcols,
                         unsigned int key, float scale, hipStream_t s) {
  const long n = (long)rows * cols;
  if (n <= 0) return;
  const long blocks = std::min<long>((n + 255) / 256, 256L * 64);
  fill_uniform_kernel<<<blocks, 256, 0, s>>>(static_cast<unsigned short*>(out), ld, rows, cols, row0, col0, gcols,
                                             key, scale);
}

}  // namespace hipserve
