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

// GLU with the per-token e4m3 output the FP8 down projection takes (prefill, FP8
// models): one 1024-thread block per row holds the row's act in registers, reduces its
// amax and writes e4m3 + row scale — act bf16 values as glu_and_mul rounds them,
// quantised as act_quant_fp8 does (bit-identical to glu_and_mul -> act_quant_fp8), with
// no bf16 act round trip through HBM. out (bf16 act) is optional.
template <bool kGelu, int VPT>
__global__ __launch_bounds__(1024) void glu_quant_kernel(unsigned short* __restrict__ out,
                                                         unsigned char* __restrict__ q8, float* __restrict__ xs,
                                                         const unsigned short* __restrict__ in, int inter,
                                                         long in_stride) {
  __shared__ float red[16];
  const long r = blockIdx.x;
  const int vpr = inter >> 3;
  u16x8 a[VPT];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < vpr) {
      const u16x8 g = *reinterpret_cast<const u16x8*>(in + r * in_stride + c * 8);
      const u16x8 u = *reinterpret_cast<const u16x8*>(in + r * in_stride + inter + c * 8);
      a[i] = kGelu ? gelu_mul8(g, u) : silu_mul8(g, u);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(bf16_to_f32(a[i][e])));
      if (out != nullptr) *reinterpret_cast<u16x8*>(out + r * inter + c * 8) = a[i];
    }
  }
  amax = block_max(amax, red);
  const float inv = amax > 0.f ? 448.f / amax : 1.f;
  if (threadIdx.x == 0) xs[r] = amax > 0.f ? amax / 448.f : 1.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 1024;
    if (c < vpr) *reinterpret_cast<uint2*>(q8 + r * inter + c * 8) = e4m3_8(a[i], inv);
  }
}

bool launch_glu_quant(bool gelu, void* out, void* q8, float* xs, const void* in, long rows, int inter,
                      long in_stride, hipStream_t s) {
  const int vpr = inter / 8;
  if (rows < 1 || inter % 8 || vpr > 4 * 1024) return false;
  auto* o = static_cast<unsigned short*>(out);
  auto* q = static_cast<unsigned char*>(q8);
  auto* i = static_cast<const unsigned short*>(in);
  const dim3 grid((unsigned)rows);
#define GQ(V)                                                                                         \
  if (gelu) glu_quant_kernel<true, V><<<grid, 1024, 0, s>>>(o, q, xs, i, inter, in_stride);           \
  else glu_quant_kernel<false, V><<<grid, 1024, 0, s>>>(o, q, xs, i, inter, in_stride);               \
  return true;
  if (vpr <= 1024) { GQ(1) }
  if (vpr <= 2048) { GQ(2) }
  GQ(4)
#undef GQ
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
