// In-house all-reduce over xGMI peer memory (SURVEY §2.E C1, §5 "Distributed
// communication backend"): decode-sized TP all-reduces (16 KiB .. a few MiB) are
// latency-bound through RCCL's ring, which crosses one xGMI link per hop. On a
// fully connected 8xMI355X node every GPU can load from all 7 peers at once:
//
//   one-shot  (<= ~256 KiB): every rank reads ALL peers' buffers and reduces the
//             whole tensor locally — one barrier, 7 links busy in parallel;
//   two-shot  (larger):      reduce-scatter (rank r sums chunk r from every peer)
//             -> barrier -> all-gather (chunk p read from peer p) — each link carries
//             2/N of the message instead of the ring's 2(N-1)/N per hop chain.
//
// Buffers: each rank owns one uncached (fine-grained, hipDeviceMallocUncached)
// block = 2 data regions (alternating by call parity, so call k+1 can be written
// while slow peers still read call k) + flag words; peers map it with HIP IPC.
// The input is first copied into the rank's own region (so any tensor can be
// reduced and the call is hipGraph-capturable: all pointers are fixed, the call
// counter lives on the device). Barriers are grid-wide across ranks (every block
// of every rank), flags with system-scope release/acquire; every wait has an
// iteration cap that raises an error flag and exits instead of hanging the GPU.
//
// Reference: vLLM's NCCL + custom all-reduce under `--tensor-parallel-size`
// (vllm-models/helm-chart/templates/model-deployments.yaml:37-38).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_BLOCKS = 64;
constexpr int CAR_THREADS = 512;
constexpr int CAR_BLOCKS = 32;

// flag area layout (uint32): [phase 0..1][src rank][block]   + per-block call counter
struct CarFlags {
  unsigned int flag[2][CAR_MAX_RANKS][CAR_MAX_BLOCKS];
  unsigned int counter[CAR_MAX_BLOCKS];
  unsigned int error;
};

struct CarPeers {
  unsigned char* data[CAR_MAX_RANKS];  // base of each rank's 2 data regions
  CarFlags* flags[CAR_MAX_RANKS];
};

struct CarState {
  int rank = 0, world = 1;
  size_t max_bytes = 0;
  unsigned char* own = nullptr;  // own allocation: 2*max_bytes data + CarFlags
  CarPeers peers{};
  bool opened[CAR_MAX_RANKS] = {};
};

HS_DEVICE void car_signal(CarFlags* peer_flags, int phase, int src_rank, int blk, unsigned int epoch) {
  __hip_atomic_store(&peer_flags->flag[phase][src_rank][blk], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

HS_DEVICE bool car_wait(CarFlags* own_flags, int phase, int src_rank, int blk, unsigned int epoch) {
  unsigned int spins = 0;
  while (__hip_atomic_load(&own_flags->flag[phase][src_rank][blk], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) <
         epoch) {
    if (++spins > (1u << 26)) {  // ~seconds: a peer never arrived -> fail loudly, never hang
      __hip_atomic_store(&own_flags->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Cross-rank grid barrier for `phase`: every block releases its prior stores and
// sets its flag on every peer, then waits until ALL blocks of ALL ranks have set
// theirs (local polling of the own uncached flag area, one flag per thread).
// Being global, it also proves every peer finished reading the previous call,
// whatever element partition that call used.
HS_DEVICE bool car_barrier(const CarPeers& P, int rank, int world, int phase, int blk, int nblk,
                           unsigned int epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = 1;
  if (threadIdx.x < (unsigned)world) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    car_signal(P.flags[threadIdx.x], phase, rank, blk, epoch);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < world * nblk; i += blockDim.x)
    if (!car_wait(P.flags[rank], phase, i / nblk, i % nblk, epoch)) s_ok = 0;
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return s_ok != 0;
}

template <int W>
HS_DEVICE void sum_bf16x8(u16x8 (&v)[W], int n, float (&acc)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
  for (int p = 0; p < W; ++p)
    if (p < n)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf16_to_f32(v[p][e]);
}

// nvec = number of 16-byte (8 x bf16) vectors in the tensor
template <bool TWO_SHOT>
__global__ __launch_bounds__(CAR_THREADS) void car_kernel(CarPeers P, int rank, int world, size_t max_bytes,
                                                          const u16x8* __restrict__ inp, u16x8* __restrict__ out,
                                                          long nvec) {
  const int blk = blockIdx.x, nblk = gridDim.x;
  CarFlags* own = P.flags[rank];
  __shared__ unsigned int s_epoch;
  if (threadIdx.x == 0) s_epoch = own->counter[blk] + 1;
  __syncthreads();
  const unsigned int epoch = s_epoch;
  const size_t region = (epoch & 1) * max_bytes;
  // 1. stage the input into this rank's peer-visible region
  u16x8* mine = reinterpret_cast<u16x8*>(P.data[rank] + region);
  const long stride = (long)nblk * CAR_THREADS;
  for (long i = (long)blk * CAR_THREADS + threadIdx.x; i < nvec; i += stride) mine[i] = inp[i];
  if (!car_barrier(P, rank, world, 0, blk, nblk, epoch)) return;
  const u16x8* src[CAR_MAX_RANKS];
#pragma unroll
  for (int p = 0; p < CAR_MAX_RANKS; ++p)
    src[p] = reinterpret_cast<const u16x8*>(P.data[p < world ? p : 0] + region);
  if (!TWO_SHOT) {
    // 2. one-shot: reduce everything from every rank (rank order fixed -> identical on all ranks)
    for (long i = (long)blk * CAR_THREADS + threadIdx.x; i < nvec; i += stride) {
      u16x8 v[CAR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) v[p] = src[p][i];
      float acc[8];
      sum_bf16x8<CAR_MAX_RANKS>(v, world, acc);
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(acc[e]);
      out[i] = o;
    }
  } else {
    // 2. reduce-scatter: this rank owns chunk [c0, c1); result written in place
    const long chunk = (nvec + world - 1) / world;
    const long c0 = rank * chunk, c1 = min(nvec, c0 + chunk);
    u16x8* mine_w = mine;
    for (long i = c0 + (long)blk * CAR_THREADS + threadIdx.x; i < c1; i += stride) {
      u16x8 v[CAR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) v[p] = src[p][i];
      float acc[8];
      sum_bf16x8<CAR_MAX_RANKS>(v, world, acc);
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(acc[e]);
      mine_w[i] = o;
    }
    if (!car_barrier(P, rank, world, 1, blk, nblk, epoch)) return;
    // 3. all-gather: chunk p from rank p
    for (long i = (long)blk * CAR_THREADS + threadIdx.x; i < nvec; i += stride) {
      const int p = (int)(i / chunk);
      out[i] = src[p][i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) own->counter[blk] = epoch;
}

// ------------------------------------------------------------------ host side
static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("custom all-reduce: ") + what + ": " + hipGetErrorString(e));
}

void* car_create(int rank, int world, size_t max_bytes) {
  if (world < 1 || world > CAR_MAX_RANKS || rank < 0 || rank >= world)
    throw std::invalid_argument("custom all-reduce: bad rank/world");
  auto* st = new CarState();
  st->rank = rank;
  st->world = world;
  st->max_bytes = (max_bytes + 255) / 256 * 256;
  const size_t total = 2 * st->max_bytes + sizeof(CarFlags);
  hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&st->own), total, hipDeviceMallocUncached),
            "hipExtMallocWithFlags");
  hip_check(hipMemset(st->own, 0, total), "hipMemset");
  st->peers.data[rank] = st->own;
  st->peers.flags[rank] = reinterpret_cast<CarFlags*>(st->own + 2 * st->max_bytes);
  return st;
}

void car_get_handle(void* state, void* handle_out /* HIP_IPC_HANDLE_SIZE bytes */) {
  auto* st = static_cast<CarState*>(state);
  hipIpcMemHandle_t h;
  hip_check(hipIpcGetMemHandle(&h, st->own), "hipIpcGetMemHandle");
  std::memcpy(handle_out, &h, sizeof(h));
}

void car_open(void* state, int peer, const void* handle) {
  auto* st = static_cast<CarState*>(state);
  if (peer == st->rank) return;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  hip_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  st->peers.data[peer] = static_cast<unsigned char*>(p);
  st->peers.flags[peer] = reinterpret_cast<CarFlags*>(static_cast<unsigned char*>(p) + 2 * st->max_bytes);
  st->opened[peer] = true;
}

bool car_error(void* state) {
  auto* st = static_cast<CarState*>(state);
  unsigned int e = 0;
  hip_check(hipMemcpy(&e, &st->peers.flags[st->rank]->error, sizeof(e), hipMemcpyDeviceToHost), "hipMemcpy");
  return e != 0;
}

void car_destroy(void* state) {
  auto* st = static_cast<CarState*>(state);
  for (int p = 0; p < CAR_MAX_RANKS; ++p)
    if (st->opened[p]) (void)hipIpcCloseMemHandle(st->peers.data[p]);
  (void)hipFree(st->own);
  delete st;
}

size_t car_max_bytes(void* state) { return static_cast<CarState*>(state)->max_bytes; }

void launch_car(void* state, const void* inp, void* out, size_t bytes, bool two_shot, int blocks, hipStream_t s) {
  auto* st = static_cast<CarState*>(state);
  if (bytes > st->max_bytes || bytes % 16) throw std::invalid_argument("custom all-reduce: bad size");
  for (int p = 0; p < st->world; ++p)
    if (!st->peers.data[p]) throw std::runtime_error("custom all-reduce: peer buffers not opened");
  // one fixed grid for every call: per-block call counters stay equal on all ranks
  (void)blocks;
  blocks = CAR_BLOCKS;
  const long nvec = (long)(bytes / 16);
  if (two_shot)
    car_kernel<true><<<blocks, CAR_THREADS, 0, s>>>(st->peers, st->rank, st->world, st->max_bytes,
                                                      static_cast<const u16x8*>(inp), static_cast<u16x8*>(out), nvec);
  else
    car_kernel<false><<<blocks, CAR_THREADS, 0, s>>>(st->peers, st->rank, st->world, st->max_bytes,
                                                       static_cast<const u16x8*>(inp), static_cast<u16x8*>(out), nvec);
}

}  // namespace hipserve
