// GLU activations of the merged gate_up projection output:
// SiLU(gate) * up (Llama / Qwen / Mixtral) and tanh-GELU(gate) * up (Gemma GeGLU).
// in: [T, 2*I] (gate | up), out: [T, I]. 16-byte vectors, grid-stride loop
// capped at 8 workgroups per CU (memory-bound op, HBM roofline target).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

template <bool kGelu>
__global__ __launch_bounds__(256) void glu_and_mul_kernel(
    unsigned short* __restrict__ out, const unsigned short* __restrict__ in,
    long rows, int inter, long in_stride, long out_stride) {
  const int vpr = inter >> 3;  // vectors per row
  const long total = rows * vpr;
  for (long v = blockIdx.x * 256L + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const long r = v / vpr;
    const int c = (int)(v - r * vpr);
    const u16x8 g = *reinterpret_cast<const u16x8*>(in + r * in_stride + c * 8);
    const u16x8 u = *reinterpret_cast<const u16x8*>(in + r * in_stride + inter + c * 8);
    *reinterpret_cast<u16x8*>(out + r * out_stride + c * 8) = kGelu ? gelu_mul8(g, u) : silu_mul8(g, u);
  }
}

static void launch_glu(bool gelu, void* out, const void* in, long rows, int inter, long in_stride, long out_stride,
                       hipStream_t s) {
  const long total = rows * (inter / 8);
  long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  auto* o = static_cast<unsigned short*>(out);
  auto* i = static_cast<const unsigned short*>(in);
  if (gelu)
    glu_and_mul_kernel<true><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(o, i, rows, inter, in_stride, out_stride);
  else
    glu_and_mul_kernel<false><<<dim3((unsigned)blocks), dim3(256), 0, s>>>(o, i, rows, inter, in_stride, out_stride);
}

void launch_silu_and_mul(void* out, const void* in, long rows, int inter,
                         long in_stride, long out_stride, hipStream_t s) {
  launch_glu(false, out, in, rows, inter, in_stride, out_stride, s);
}

void launch_gelu_and_mul(void* out, const void* in, long rows, int inter,
                         long in_stride, long out_stride, hipStream_t s) {
  launch_glu(true, out, in, rows, inter, in_stride, out_stride, s);
}

}  // namespace hipserve
