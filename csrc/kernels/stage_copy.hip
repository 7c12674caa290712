// Batched host<->device staging copy for the pipelined decode step.
//
// The decode loop moves ~6 small buffers per step (ids/positions/slots/seeds,
// block tables + context lengths, temperatures/top-p in; sampled ids + logprobs
// out). As hipMemcpyAsync calls each one is a separate blit dispatch, and the
// v6 decode-step trace (profiles/r1_bench_llama3_8b_v6_trace.md) shows ~0.25 ms
// of idle GPU per step in front of them. Here ONE dispatch moves all of a
// direction's buffers: pinned host memory is read / written in place through
// its device mapping (zero-copy). Accesses are system-scope atomics (vector
// memory ops with the cache-bypass bits), so the host's staging writes of the
// previous launch and the GPU's writes for the host never sit stale in L2.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

HS_DEVICE void copy_words(unsigned int* __restrict__ dst, const unsigned int* __restrict__ src, long n,
                          bool sys_src, bool sys_dst) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned int v = sys_src ? __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : src[i];
    if (sys_dst)
      __hip_atomic_store(dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      dst[i] = v;
  }
}

__global__ __launch_bounds__(256) void stage_copy_kernel(StageCopyArgs a) {
  const int c = blockIdx.y;  // one grid row per buffer
  copy_words(static_cast<unsigned int*>(a.dst[c]), static_cast<const unsigned int*>(a.src[c]), a.words[c],
             (a.host_mask >> (2 * c)) & 1, (a.host_mask >> (2 * c + 1)) & 1);
  if ((a.host_mask >> (2 * c + 1)) & 1) __threadfence_system();
}

void launch_stage_copy(const StageCopyArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  long mx = 0;
  for (int i = 0; i < a.n; ++i) mx = std::max(mx, a.words[i]);
  if (mx == 0) return;
  const int bx = (int)std::min<long>((mx + 255) / 256, 64);
  stage_copy_kernel<<<dim3(bx, a.n), 256, 0, s>>>(a);
}

}  // namespace hipserve

