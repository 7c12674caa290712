// In-house tensor-parallel collectives over xGMI peer memory (SURVEY §2.E C1/C2,
// §5 "Distributed communication backend"). Decode-sized TP messages (16 KiB ..
// a few MiB) are latency-bound through RCCL's ring, which crosses one xGMI link
// per hop; on a fully connected 8xMI355X node every GPU can load from all 7 peers
// at once, so these kernels read the peers' buffers directly:
//
//   car_ar   bf16 all-reduce. one-shot (small): every rank reads ALL peers and
//            reduces everything locally (one barrier, 7 links busy in parallel);
//            two-shot (larger): reduce-scatter -> barrier -> all-gather, each link
//            carries 2/N of the message.
//   car_ag   all-gather of a [rows, cols] shard into [rows, world*cols] (the
//            vocab-parallel LM-head logits), one barrier.
//   car_norm the row-parallel projection epilogue of a decoder layer in ONE
//            kernel: local split-K partial sum -> cross-rank reduce-scatter (by
//            columns) -> residual add -> per-row sum of squares -> all-gather of
//            the new residual chunks -> RMSNorm. fp32 exchange keeps TP=N within
//            fp32 rounding of TP=1 (the partials are never rounded to bf16 before
//            the cross-rank sum); bf16 exchange halves the bytes (prefill chunks).
//
// Two grid classes per collective: decode-sized messages run on a 64-block grid
// (few blocks = few barrier pairs = lowest latency); prefill-sized ones (an 8K-token
// chunk of a 70B layer is a 128 MiB bf16 [8192, 8192] exchange) on a 512-block grid
// so every CU streams (the fixed 64-block car_norm was 754 us per 64 MiB
// call, as long as the GEMMs). Each class is an independent instance of the
// protocol below (own regions, flags and counters), so grids never mix.
// Whether a prefill-sized message goes through these kernels at all or through
// RCCL is decided per node by a start-up calibration (parallel/comm.py).
//
// Buffers: every rank owns ONE uncached (fine-grained) allocation holding, per
// collective kind, two data regions used alternately by call parity, plus a flag
// area; peers map it with HIP IPC. Inputs are staged into the rank's own region,
// so any tensor can be reduced and every call is hipGraph-capturable (all
// pointers fixed; the per-block call counters live on the device).
//
// Synchronisation is a PER-BLOCK PAIRED barrier: block b of rank r only signals
// and waits for block b of every peer (world flags per block, not world x grid).
// That is sufficient because every kernel assigns data to blocks by a mapping that
// does not depend on the message size (16-byte vector i -> block (i / GRAN) % NB;
// car_norm: row m -> block m % NB): the only remote reader of the bytes block b
// writes is block b of a peer, so "peer block b reached call k+1" proves it is done
// reading what block b will overwrite in call k+2 (regions alternate by parity).
// A block with nothing to move in a call skips its barriers (all ranks see the
// same size, so the pair skips together) and just advances its counter.
//
// Failure: every wait is bounded by a wall-clock timeout (s_memrealtime, 100 MHz).
// A timeout sets a sticky error word on this rank AND on every peer, plus a pinned
// host word the engine polls between steps; from then on every barrier of every
// rank fails fast (no further waiting, counters still advance) instead of pairing
// stale epochs — the engine sees car_error() and marks itself dead.
//
// Reference: vLLM's NCCL + custom all-reduce under `--tensor-parallel-size`
// (vllm-models/helm-chart/templates/model-deployments.yaml:37-38).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_NB_S = 64;      // decode-sized class grid (fixed per class: per-block epochs stay in lockstep)
constexpr int CAR_NB_L = 512;     // prefill-sized class grid: 2 blocks per CU
constexpr int CAR_NB_MAX = CAR_NB_L;
constexpr int CAR_T = 256;        // threads per block
constexpr int CAR_GRAN = CAR_T;   // 16-B vectors per block per grid-stride step
constexpr long CAR_MAX_ROWS = 65536;
constexpr long CAR_S_ROWS = 512;                // norm rows of the small class (decode batches)
constexpr size_t CAR_S_BYTES = 8u << 20;        // message bytes of the small class
// kinds: all-reduce small / large, all-gather, fused add+RMSNorm small / large
enum { K_AR_S = 0, K_AR_L = 1, K_AG = 2, K_NORM_S = 3, K_NORM_L = 4, K_NUM = 5 };

struct CarFlags {
  unsigned int flag[K_NUM][2][CAR_MAX_RANKS][CAR_NB_MAX];  // [kind][phase][src rank][block], stored by peers
  unsigned int counter[K_NUM][CAR_NB_MAX];                 // own per-block call counters
  unsigned int error;                                      // sticky: some rank timed out
};

struct CarPeers {
  unsigned char* base[CAR_MAX_RANKS];  // each rank's allocation (own one at [rank])
  CarFlags* flags[CAR_MAX_RANKS];
  unsigned int* host_error;            // pinned host word (device-mapped)
  size_t off[K_NUM];                   // region offset of each kind inside an allocation
  size_t bytes[K_NUM];                 // bytes of ONE parity region of each kind
  unsigned long long timeout;          // s_memrealtime ticks (100 MHz)
};

struct CarState {
  int rank = 0, world = 1;
  int nb_large = CAR_NB_L;  // grid of the prefill-sized class (smaller when ranks share a GPU)
  size_t max_bytes = 0;
  unsigned char* own = nullptr;
  CarPeers peers{};
  bool opened[CAR_MAX_RANKS] = {};
};

HS_DEVICE unsigned char* car_region(const CarPeers& P, int rank, int kind, unsigned int epoch) {
  return P.base[rank] + P.off[kind] + (epoch & 1) * P.bytes[kind];
}

// Epoch of this call for block `blk` (broadcast through LDS).
HS_DEVICE unsigned int car_epoch(const CarPeers& P, int rank, int kind, int blk, unsigned int* s_word) {
  if (threadIdx.x == 0) *s_word = P.flags[rank]->counter[kind][blk] + 1;
  __syncthreads();
  return *s_word;
}

HS_DEVICE void car_finish(const CarPeers& P, int rank, int kind, int blk, unsigned int epoch) {
  __syncthreads();
  if (threadIdx.x == 0) P.flags[rank]->counter[kind][blk] = epoch;
}

HS_DEVICE void car_raise(const CarPeers& P, int world) {
  for (int p = 0; p < world; ++p)
    __hip_atomic_store(&P.flags[p]->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(P.host_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Paired barrier: this block's stores become visible system-wide, then it signals
// block `blk` of every rank and waits until block `blk` of every rank signalled.
// Returns false (for the whole block) once the sticky error is set.
HS_DEVICE bool car_barrier(const CarPeers& P, int rank, int world, int kind, int phase, int blk,
                           unsigned int epoch, int* s_ok) {
  const int t = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (t == 0) *s_ok = 1;
  __syncthreads();
  CarFlags* own = P.flags[rank];
  if (t < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: the peers read our region
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&P.flags[t]->flag[kind][phase][rank][blk], epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      // the sticky error first: once set, no barrier pairs again (epochs may be skewed)
      if (__hip_atomic_load(&own->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
        // a peer timed out: make it visible to this rank's host too
        __hip_atomic_store(P.host_error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *s_ok = 0;
        break;
      }
      if ((int)(__hip_atomic_load(&own->flag[kind][phase][t][blk], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                epoch) >= 0)
        break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > P.timeout) {
        car_raise(P, world);
        *s_ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return *s_ok != 0;
}

template <int W>
HS_DEVICE u16x8 sum_bf16x8(const u16x8 (&v)[W], int n) {
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = bf16_to_f32(v[0][e]);
#pragma unroll
  for (int p = 1; p < W; ++p)
    if (p < n)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf16_to_f32(v[p][e]);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = f32_to_bf16(acc[e]);
  return o;
}

// ------------------------------------------------------------------ all-reduce
// nvec = 16-byte vectors in the tensor. Rank order of the sum is fixed, so every
// rank produces identical bits.
template <bool TWO_SHOT>
__global__ __launch_bounds__(CAR_T) void car_ar_kernel(CarPeers P, int kind, int NB, int rank, int world,
                                                       const u16x8* __restrict__ inp, u16x8* __restrict__ out,
                                                       long nvec) {
  __shared__ unsigned int s_epoch;
  __shared__ int s_ok;
  const int blk = blockIdx.x, t = threadIdx.x;
  const int K_AR = kind;
  const unsigned int epoch = car_epoch(P, rank, K_AR, blk, &s_epoch);
  if ((long)blk * CAR_GRAN >= nvec) {  // nothing of this size maps to this block (same on every rank)
    car_finish(P, rank, K_AR, blk, epoch);
    return;
  }
  u16x8* mine = reinterpret_cast<u16x8*>(car_region(P, rank, K_AR, epoch));
  const u16x8* src[CAR_MAX_RANKS];
#pragma unroll
  for (int p = 0; p < CAR_MAX_RANKS; ++p)
    src[p] = reinterpret_cast<const u16x8*>(car_region(P, p < world ? p : rank, K_AR, epoch));
  const long step = (long)NB * CAR_GRAN;
  for (long i = (long)blk * CAR_GRAN + t; i < nvec; i += step) mine[i] = inp[i];
  if (!car_barrier(P, rank, world, K_AR, 0, blk, epoch, &s_ok)) {
    car_finish(P, rank, K_AR, blk, epoch);
    return;
  }
  if (!TWO_SHOT) {
    for (long i = (long)blk * CAR_GRAN + t; i < nvec; i += step) {
      u16x8 v[CAR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) v[p] = src[p][i];
      out[i] = sum_bf16x8<CAR_MAX_RANKS>(v, world);
    }
  } else {
    const long chunk = (nvec + world - 1) / world;
    const long c0 = rank * chunk, c1 = min(nvec, c0 + chunk);
    // reduce-scatter: own chunk, in place in the own region (only this rank reads
    // its own chunk's staged values; peers read it after the next barrier)
    for (long i = (long)blk * CAR_GRAN + t; i < nvec; i += step) {
      if (i < c0 || i >= c1) continue;
      u16x8 v[CAR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) v[p] = src[p][i];
      mine[i] = sum_bf16x8<CAR_MAX_RANKS>(v, world);
    }
    if (!car_barrier(P, rank, world, K_AR, 1, blk, epoch, &s_ok)) {
      car_finish(P, rank, K_AR, blk, epoch);
      return;
    }
    for (long i = (long)blk * CAR_GRAN + t; i < nvec; i += step) out[i] = src[(int)(i / chunk)][i];
  }
  car_finish(P, rank, K_AR, blk, epoch);
}

// ------------------------------------------------------------------ all-gather
// inp: [rows, row_v] (V-sized elements, contiguous) -> out: [rows, world * row_v]
template <typename V>
__global__ __launch_bounds__(CAR_T) void car_ag_kernel(CarPeers P, int rank, int world, const V* __restrict__ inp,
                                                       V* __restrict__ out, long nv, long row_v) {
  __shared__ unsigned int s_epoch;
  __shared__ int s_ok;
  const int blk = blockIdx.x, t = threadIdx.x;
  const unsigned int epoch = car_epoch(P, rank, K_AG, blk, &s_epoch);
  if ((long)blk * CAR_GRAN >= nv) {
    car_finish(P, rank, K_AG, blk, epoch);
    return;
  }
  V* mine = reinterpret_cast<V*>(car_region(P, rank, K_AG, epoch));
  const long step = (long)CAR_NB_S * CAR_GRAN;
  for (long j = (long)blk * CAR_GRAN + t; j < nv; j += step) mine[j] = inp[j];
  if (car_barrier(P, rank, world, K_AG, 0, blk, epoch, &s_ok)) {
    const long orow = (long)world * row_v;
    for (long j = (long)blk * CAR_GRAN + t; j < nv; j += step) {
      const long r = j / row_v, c = j - r * row_v;
      V v[CAR_MAX_RANKS];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) v[p] = reinterpret_cast<const V*>(car_region(P, p, K_AG, epoch))[j];
#pragma unroll
      for (int p = 0; p < CAR_MAX_RANKS; ++p)
        if (p < world) out[r * orow + p * row_v + c] = v[p];
    }
  }
  car_finish(P, rank, K_AG, blk, epoch);
}

// ------------------------------------------------------------------ fused norm
// x: kIn == 0 -> fp32 split-K partials [S, M, N] (slice = M*N), kIn == 1 -> bf16 [M, N].
// Region of one parity: [A: M*N exchange values][B: M*N/world bf16 residual chunks][C: M fp32 sum of squares]
// Rows are dealt to blocks round-robin (row m -> block m % NB). Phase B (the
// reduce-scatter of one rank's column chunk, cv 16-B vectors wide) gives each row
// TPR = 64..256 threads so a 70B TP=8 chunk (cv = 128) keeps every lane busy with
// two rows per pass; a row's sum of squares is reduced wave by wave, in wave order
// (deterministic).
template <int kIn, bool kExF32, bool kWF32>
__global__ __launch_bounds__(CAR_T) void car_norm_kernel(CarPeers P, int kind, int NB, int rank, int world,
                                                         const void* __restrict__ x, int S,
                                                         unsigned short* __restrict__ residual,
                                                         const void* __restrict__ weight,
                                                         unsigned short* __restrict__ out, int M, int N, float eps) {
  __shared__ unsigned int s_epoch;
  __shared__ int s_ok;
  __shared__ float scratch[CAR_T / 64];
  const int blk = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int K_NORM = kind;
  const unsigned int epoch = car_epoch(P, rank, K_NORM, blk, &s_epoch);
  if (blk >= M) {  // no row maps to this block
    car_finish(P, rank, K_NORM, blk, epoch);
    return;
  }
  const int nv = N >> 3;            // 8-element vectors per row
  const int cv = nv / world;        // vectors of one rank's column chunk
  const int cN = cv * 8;
  const long aBytes = (long)M * N * (kExF32 ? 4 : 2);
  const long bBytes = (long)M * cN * 2;
  auto regA = [&](int p) { return car_region(P, p, K_NORM, epoch); };
  auto regB = [&](int p) { return car_region(P, p, K_NORM, epoch) + aBytes; };
  auto regC = [&](int p) { return reinterpret_cast<float*>(car_region(P, p, K_NORM, epoch) + aBytes + bBytes); };

  // A. local sum of this rank's partials -> own exchange region (all columns)
  for (int m = blk; m < M; m += NB) {
    for (int v = t; v < nv; v += CAR_T) {
      float h[8];
      if constexpr (kIn == 0) {
        f32x4 lo, hi;
        sum_slices8(lo, hi, static_cast<const float*>(x) + (long)m * N + v * 8, (long)M * N, S);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h[j] = lo[j];
          h[j + 4] = hi[j];
        }
      } else {
        const u16x8 b = reinterpret_cast<const u16x8*>(static_cast<const unsigned short*>(x) + (long)m * N)[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = bf16_to_f32(b[j]);
      }
      if constexpr (kExF32) {
        f32x4* d = reinterpret_cast<f32x4*>(regA(rank) + ((long)m * N + v * 8) * 4);
        d[0] = f32x4{h[0], h[1], h[2], h[3]};
        d[1] = f32x4{h[4], h[5], h[6], h[7]};
      } else {
        u16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = f32_to_bf16(h[j]);
        reinterpret_cast<u16x8*>(regA(rank))[(long)m * nv + v] = b;
      }
    }
  }
  if (!car_barrier(P, rank, world, K_NORM, 0, blk, epoch, &s_ok)) {
    car_finish(P, rank, K_NORM, blk, epoch);
    return;
  }
  // B. reduce-scatter by columns: this rank's chunk of every row of the block,
  //    rank-ordered sum, bf16 round (= the unfused GEMM output), residual add
  const int v0 = rank * cv;
  const int tpr = cv > 128 ? 256 : (cv > 64 ? 128 : 64);  // threads per row (whole waves)
  const int rpp = CAR_T / tpr, sub = t / tpr, lt = t - sub * tpr, wpr = tpr / 64;
  const int nrows = (M - blk + NB - 1) / NB;               // rows of this block
  for (int i0 = 0; i0 < nrows; i0 += rpp) {
    const int i = i0 + sub;
    const int m = blk + i * NB;
    float ss = 0.f;
    if (i < nrows) {
      for (int v = v0 + lt; v < v0 + cv; v += tpr) {
        float acc[8];
        if constexpr (kExF32) {
          f32x4 lo[CAR_MAX_RANKS], hi[CAR_MAX_RANKS];
#pragma unroll
          for (int p = 0; p < CAR_MAX_RANKS; ++p)
            if (p < world) {
              const f32x4* s = reinterpret_cast<const f32x4*>(regA(p) + ((long)m * N + v * 8) * 4);
              lo[p] = s[0];
              hi[p] = s[1];
            }
          f32x4 a = lo[0], b = hi[0];
#pragma unroll
          for (int p = 1; p < CAR_MAX_RANKS; ++p)
            if (p < world) {
              a += lo[p];
              b += hi[p];
            }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] = a[j];
            acc[j + 4] = b[j];
          }
        } else {
          u16x8 s[CAR_MAX_RANKS];
#pragma unroll
          for (int p = 0; p < CAR_MAX_RANKS; ++p)
            if (p < world) s[p] = reinterpret_cast<const u16x8*>(regA(p))[(long)m * nv + v];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = bf16_to_f32(s[0][j]);
#pragma unroll
          for (int p = 1; p < CAR_MAX_RANKS; ++p)
            if (p < world)
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[j] += bf16_to_f32(s[p][j]);
        }
        const u16x8 res = reinterpret_cast<const u16x8*>(residual + (long)m * N)[v];
        u16x8 r;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          r[j] = f32_to_bf16(bf16_to_f32(f32_to_bf16(acc[j])) + bf16_to_f32(res[j]));
          const float f = bf16_to_f32(r[j]);
          ss += f * f;
        }
        reinterpret_cast<u16x8*>(regB(rank))[(long)m * cv + (v - v0)] = r;
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) scratch[wave] = ss;
    __syncthreads();
    if (i < nrows && lt == 0) {
      float tot = 0.f;
      for (int w = sub * wpr; w < (sub + 1) * wpr; ++w) tot += scratch[w];
      regC(rank)[m] = tot;
    }
    __syncthreads();
  }
  if (!car_barrier(P, rank, world, K_NORM, 1, blk, epoch, &s_ok)) {
    car_finish(P, rank, K_NORM, blk, epoch);
    return;
  }
  // C. all-gather the residual chunks, total sum of squares (rank order), RMSNorm
  for (int m = blk; m < M; m += NB) {
    float ssum = 0.f;
    for (int p = 0; p < world; ++p) ssum += regC(p)[m];
    const float inv = rsqrtf(ssum / N + eps);
    for (int v = t; v < nv; v += CAR_T) {
      const int p = v / cv;
      const u16x8 r = reinterpret_cast<const u16x8*>(regB(p))[(long)m * cv + (v - p * cv)];
      reinterpret_cast<u16x8*>(residual + (long)m * N)[v] = r;
      u16x8 o;
      if constexpr (kWF32) {
        const f32x4* wp = reinterpret_cast<const f32x4*>(weight) + v * 2;
        const f32x4 w0 = wp[0], w1 = wp[1];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f32_to_bf16(bf16_to_f32(r[j]) * inv * w0[j]);
          o[j + 4] = f32_to_bf16(bf16_to_f32(r[j + 4]) * inv * w1[j]);
        }
      } else {
        const u16x8 w = reinterpret_cast<const u16x8*>(weight)[v];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f32_to_bf16(bf16_to_f32(r[j]) * inv * bf16_to_f32(w[j]));
      }
      reinterpret_cast<u16x8*>(out + (long)m * N)[v] = o;
    }
  }
  car_finish(P, rank, K_NORM, blk, epoch);
}

// ------------------------------------------------------------------ host side
static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("custom collectives: ") + what + ": " + hipGetErrorString(e));
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

void* car_create(int rank, int world, size_t max_bytes, int nb_large) {
  if (world < 1 || world > CAR_MAX_RANKS || rank < 0 || rank >= world)
    throw std::invalid_argument("custom collectives: bad rank/world");
  auto* st = new CarState();
  st->rank = rank;
  st->world = world;
  // every block of a call spins on its peers' block: all blocks of all ranks that
  // share a device must be resident at once (8 blocks of 256 threads per CU)
  st->nb_large = nb_large < CAR_NB_S ? CAR_NB_S : (nb_large > CAR_NB_MAX ? CAR_NB_MAX : nb_large);
  st->max_bytes = align_up(max_bytes, 256);
  const size_t B = st->max_bytes;
  // per-parity region of each kind: AR = message; AG = one shard; NORM = fp32
  // exchange (2B) + bf16 residual chunks (B) + per-row sums of squares. The small
  // class holds decode-sized messages only (SB = min(B, 8 MiB)).
  const size_t SB = B < CAR_S_BYTES ? B : CAR_S_BYTES;
  st->peers.bytes[K_AR_S] = SB;
  st->peers.bytes[K_AR_L] = B;
  st->peers.bytes[K_AG] = B;
  st->peers.bytes[K_NORM_S] = 3 * SB + align_up(CAR_S_ROWS * sizeof(float), 256);
  st->peers.bytes[K_NORM_L] = 3 * B + align_up(CAR_MAX_ROWS * sizeof(float), 256);
  size_t off = 0;
  for (int k = 0; k < K_NUM; ++k) {
    st->peers.off[k] = off;
    off += 2 * st->peers.bytes[k];
  }
  const size_t flags_off = off;
  const size_t total = flags_off + align_up(sizeof(CarFlags), 256);
  hip_check(hipExtMallocWithFlags(reinterpret_cast<void**>(&st->own), total, hipDeviceMallocUncached),
            "hipExtMallocWithFlags");
  hip_check(hipMemset(st->own, 0, total), "hipMemset");
  hip_check(hipHostMalloc(reinterpret_cast<void**>(&st->peers.host_error), sizeof(unsigned int),
                          hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc");
  *st->peers.host_error = 0;
  const char* to = std::getenv("HIPSERVE_CAR_TIMEOUT_S");
  const double secs = to ? std::atof(to) : 30.0;
  st->peers.timeout = (unsigned long long)(secs * 1e8);
  st->peers.base[rank] = st->own;
  st->peers.flags[rank] = reinterpret_cast<CarFlags*>(st->own + flags_off);
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
  st->peers.base[peer] = static_cast<unsigned char*>(p);
  st->peers.flags[peer] = reinterpret_cast<CarFlags*>(
      static_cast<unsigned char*>(p) + (reinterpret_cast<unsigned char*>(st->peers.flags[st->rank]) - st->own));
  st->opened[peer] = true;
}

// Host-side poll of the sticky error (pinned word: no device sync, safe between steps)
bool car_error(void* state) {
  auto* st = static_cast<CarState*>(state);
  return __atomic_load_n(st->peers.host_error, __ATOMIC_ACQUIRE) != 0;
}

void car_destroy(void* state) {
  auto* st = static_cast<CarState*>(state);
  for (int p = 0; p < CAR_MAX_RANKS; ++p)
    if (st->opened[p]) (void)hipIpcCloseMemHandle(st->peers.base[p]);
  (void)hipFree(st->own);
  (void)hipHostFree(st->peers.host_error);
  delete st;
}

size_t car_max_bytes(void* state) { return static_cast<CarState*>(state)->max_bytes; }

static CarState* ready(void* state) {
  auto* st = static_cast<CarState*>(state);
  for (int p = 0; p < st->world; ++p)
    if (!st->peers.base[p]) throw std::runtime_error("custom collectives: peer buffers not opened");
  return st;
}

void launch_car(void* state, const void* inp, void* out, size_t bytes, bool two_shot, int blocks, hipStream_t s) {
  auto* st = ready(state);
  (void)blocks;  // one fixed grid for every call
  if (bytes > st->max_bytes || bytes % 16) throw std::invalid_argument("custom all-reduce: bad size");
  const long nvec = (long)(bytes / 16);
  auto* i = static_cast<const u16x8*>(inp);
  auto* o = static_cast<u16x8*>(out);
  if (bytes <= st->peers.bytes[K_AR_S]) {
    if (two_shot) car_ar_kernel<true><<<CAR_NB_S, CAR_T, 0, s>>>(st->peers, K_AR_S, CAR_NB_S, st->rank, st->world, i, o, nvec);
    else car_ar_kernel<false><<<CAR_NB_S, CAR_T, 0, s>>>(st->peers, K_AR_S, CAR_NB_S, st->rank, st->world, i, o, nvec);
  } else {  // large messages: always reduce-scatter + all-gather (2/N of the bytes per link)
    const int nb = st->nb_large;
    car_ar_kernel<true><<<nb, CAR_T, 0, s>>>(st->peers, K_AR_L, nb, st->rank, st->world, i, o, nvec);
  }
}

void launch_car_all_gather(void* state, const void* inp, void* out, size_t shard_bytes, size_t row_bytes,
                           hipStream_t s) {
  auto* st = ready(state);
  if (shard_bytes > st->max_bytes || row_bytes == 0 || shard_bytes % row_bytes)
    throw std::invalid_argument("custom all-gather: bad size");
  if (row_bytes % 16 == 0)
    car_ag_kernel<u16x8><<<CAR_NB_S, CAR_T, 0, s>>>(st->peers, st->rank, st->world, static_cast<const u16x8*>(inp),
                                                  static_cast<u16x8*>(out), (long)(shard_bytes / 16),
                                                  (long)(row_bytes / 16));
  else if (row_bytes % 4 == 0)
    car_ag_kernel<unsigned int><<<CAR_NB_S, CAR_T, 0, s>>>(st->peers, st->rank, st->world,
                                                         static_cast<const unsigned int*>(inp),
                                                         static_cast<unsigned int*>(out), (long)(shard_bytes / 4),
                                                         (long)(row_bytes / 4));
  else if (row_bytes % 2 == 0)
    car_ag_kernel<unsigned short><<<CAR_NB_S, CAR_T, 0, s>>>(st->peers, st->rank, st->world,
                                                           static_cast<const unsigned short*>(inp),
                                                           static_cast<unsigned short*>(out),
                                                           (long)(shard_bytes / 2), (long)(row_bytes / 2));
  else
    throw std::invalid_argument("custom all-gather: rows must be a multiple of 2 bytes");
}

static bool norm_fits_class(const CarState* st, size_t B, long max_rows, int M, int N, bool exch_f32) {
  return M <= max_rows && N % (8 * st->world) == 0 && (size_t)M * N * (exch_f32 ? 4 : 2) <= 2 * B &&
         (size_t)M * N * 2 <= B;
}

// small class: decode batches (<= 512 rows that fit its 8 MiB regions)
static bool norm_small(const CarState* st, int M, int N, bool exch_f32) {
  const size_t SB = (st->peers.bytes[K_NORM_S] - align_up(CAR_S_ROWS * sizeof(float), 256)) / 3;
  return norm_fits_class(st, SB, CAR_S_ROWS, M, N, exch_f32);
}

bool car_norm_fits(void* state, int M, int N, bool exch_f32) {
  auto* st = static_cast<CarState*>(state);
  return norm_small(st, M, N, exch_f32) || norm_fits_class(st, st->max_bytes, CAR_MAX_ROWS, M, N, exch_f32);
}

void launch_car_add_rmsnorm(void* state, void* out, void* residual, const void* x, bool x_f32, int S,
                            const void* w, bool weight_f32, int M, int N, float eps, bool exch_f32, hipStream_t s) {
  auto* st = ready(state);
  if (!car_norm_fits(state, M, N, exch_f32)) throw std::invalid_argument("custom add+rmsnorm: message too large");
  auto* o = static_cast<unsigned short*>(out);
  auto* r = static_cast<unsigned short*>(residual);
  const bool small = norm_small(st, M, N, exch_f32);
#define CAR_NORM_LAUNCH(IN, EX, WF)                                                                             \
  do {                                                                                                         \
    const int nb = small ? CAR_NB_S : st->nb_large;                                                            \
    car_norm_kernel<IN, EX, WF><<<nb, CAR_T, 0, s>>>(st->peers, small ? K_NORM_S : K_NORM_L, nb, st->rank,      \
                                                     st->world, x, S, r, w, o, M, N, eps);                      \
  } while (0)
  if (x_f32) {
    if (exch_f32) { if (weight_f32) CAR_NORM_LAUNCH(0, true, true); else CAR_NORM_LAUNCH(0, true, false); }
    else { if (weight_f32) CAR_NORM_LAUNCH(0, false, true); else CAR_NORM_LAUNCH(0, false, false); }
  } else {
    if (exch_f32) { if (weight_f32) CAR_NORM_LAUNCH(1, true, true); else CAR_NORM_LAUNCH(1, true, false); }
    else { if (weight_f32) CAR_NORM_LAUNCH(1, false, true); else CAR_NORM_LAUNCH(1, false, false); }
  }
#undef CAR_NORM_LAUNCH
}

}  // namespace hipserve
