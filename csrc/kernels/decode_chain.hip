// Decode-layer GEMM chain in ONE launch (SURVEY §3.F hot loop; VERDICT r4 "next round"
// item 3): a row-parallel projection -> residual add -> RMSNorm -> the next projection,
//   o_proj   -> + residual -> RMSNorm(ln2)      -> gate|up with the SiLU-GLU epilogue
//   down     -> + residual -> RMSNorm(next ln1) -> the next layer's qkv (split-K partials)
// replacing decode_gemm (partials) -> splitk_add_rmsnorm -> decode_gemm: three launches
// and two kernel boundaries, during which the chip streams no weights.
//
//  * Blocks [0, nA) run the producer GEMM (decode_gemm.hip's packed body: 8 waves x 128
//    weight rows, K slice 256 * NSA), store their fp32 partial slabs and count into `done`.
//  * Blocks [nA, nA + nB) run the consumer GEMM. They issue their first two weight steps
//    and load the RMSNorm weight BEFORE waiting, so the weight stream starts while the
//    producers finish. The first tilesA * MT consumers then each reduce one unit (one
//    128-column tile x 16 rows: the S slabs summed in slice order + the residual, written
//    back in bf16 exactly as splitk_add_rmsnorm rounds, and the unit's per-row sums of
//    squares) once `done` == nA, and count into `rdone`. Every consumer waits for
//    `rdone`, forms each row's 1 / rms from the unit sums (fixed order) and stages
//    x = bf16(h * rs * w) into LDS instead of reading a materialised normalised copy.
//    The result equals the three-launch chain except where the reassociated sum of
//    squares moves 1 / rms by an ulp. (A per-tile last-arriver reducer — one block reading
//    all S slabs of its tile, 256 KB — took 9-12 us: too few blocks for the reduction;
//    the units spread it over 128 blocks of 64 KB each.)
//  * Hand-offs are write-through (cdna_hip_programming.md §6 Guideline 16 R1, the sc1
//    rows of the hand-off table): every handed-off byte (partial slabs, the new residual,
//    the tile sums) is stored sc1, every storing wave drains (s_waitcnt vmcnt(0)) before
//    the barrier behind which one lane adds to the counter, and EVERY load of those bytes
//    is an sc1 load — so no release fence (buffer_wbl2: ~10 us here with the slabs dirty
//    in L2) and no acquire fence is needed.
//  * No deadlock: producers never wait, and blocks are dispatched in index order, so
//    every producer is resident or finished before a consumer takes a slot. (At 64 rows
//    the norm staging needs ~142 VGPRs, so one block per CU: consumers start on the CUs
//    whose producers have retired; capping at 128 VGPRs for two blocks per CU spills.)
//    A consumer that polls 2^22 times anyway counts into `err` and proceeds (wrong
//    output, never a hang); the host checks `err` (tests, engine warm-up).
//  * The counters clean up after themselves: the last consumer past both waits (a third
//    counter) zeroes them; the buffer starts zeroed.
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

namespace {

constexpr int CH_ROW = 264;        // x ring row stride (bf16), as decode_gemm.hip
constexpr int CH_KMAX = 4096;      // consumer K (= producer N) held in LDS for the norm weight
constexpr int CH_SPIN_MAX = 1 << 22;

// sync words, each on its own 128-byte line: producers done, consumers past the wait,
// give-ups, reduction units done
constexpr int CH_DONE = 0, CH_PASSED = 32, CH_ERR = 64, CH_RDONE = 96, CH_WORDS = 128;

HS_DEVICE void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// the hand-off words are accessed as GLOBAL (address space 1) agent-scope atomics, never flat
typedef __attribute__((address_space(1))) int gint;
HS_DEVICE gint* gw(int* p) { return (gint*)p; }

// write-through hand-off stores / loads (sc1): buffer ops over a raw resource
constexpr int kSc1 = 16;  // buffer aux bit of sc1 on gfx950
HS_DEVICE __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// sum over S slabs (byte stride `slab`) of 8 consecutive fp32 at byte offset `off`, slab
// order 0, 1, ... (splitk_add_rmsnorm's order), every load sc1; batches of 8 in flight
HS_DEVICE void sum_slabs_sc1(f32x4& lo, f32x4& hi, __amdgpu_buffer_rsrc_t r, int off, int slab, int S) {
  for (int s0 = 0; s0 < S; s0 += 8) {
    u32x4 a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = off + min(s0 + j, S - 1) * slab;
      a[j] = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, kSc1);
      b[j] = __builtin_amdgcn_raw_buffer_load_b128(r, o + 16, 0, kSc1);
    }
    if (s0 == 0) {
      lo = __builtin_bit_cast(f32x4, a[0]);
      hi = __builtin_bit_cast(f32x4, b[0]);
    } else {
      lo += __builtin_bit_cast(f32x4, a[0]);
      hi += __builtin_bit_cast(f32x4, b[0]);
    }
#pragma unroll
    for (int j = 1; j < 8; ++j)
      if (s0 + j < S) {
        lo += __builtin_bit_cast(f32x4, a[j]);
        hi += __builtin_bit_cast(f32x4, b[j]);
      }
  }
}

template <int MT>
struct ChainLds {
  static constexpr int XR = 16 * MT;
  static constexpr int X = 2 * XR * CH_ROW;          // x ring (bf16)
  static constexpr int G = CH_KMAX;                  // norm weight (bf16)
  static constexpr int RS = 2 * 64;                  // 64 fp32 row scales
  static constexpr int TOTAL = X + G + RS;
};

// The packed decode GEMM main loop (decode_gemm_kernel<MT, 1, 8, NS, true, ...>): the
// weight ring 2 steps ahead, x through registers into a 2-slot LDS ring. kNorm: x rows
// are the residual h, staged as bf16(h * rs[row] * gamma[k]) (splitk_add_rmsnorm's
// rounding). kEarlyW: the weight loads go out before `pre_x` (the consumer's wait).
template <int MT, int NS, bool kNorm, bool kEarlyW, typename PreX>
HS_DEVICE void chain_gemm(f32x4 (&acc)[MT], unsigned short* xs, const unsigned short* wp,
                          const unsigned short* x, long x_stride, int M, int k0, const float* rsv,
                          const unsigned short* gl, PreX&& pre_x, __amdgpu_buffer_rsrc_t xr) {
  constexpr int XR = 16 * MT, NT = 512;
  constexpr int XPASS = XR * 32 / NT > 0 ? XR * 32 / NT : 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const unsigned short* wr = wp + (long)wave * (8 * 512) + lane * 8;
  u16x8 ring[3][8];
  u16x8 xv[XPASS];
  auto load_w = [&](int slot, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
      ring[slot][s] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(wr + (long)step * 32768 + 512 * s));
  };
  auto load_x = [&](int step) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      if (XR * 32 < NT && idx >= XR * 32) continue;
      const long e = (long)min(row, M - 1) * x_stride + k0 + step * 256 + col;
      if constexpr (kNorm)  // x = the residual another block just stored sc1: sc1 loads
        xv[p] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(e * 2), 0, kSc1));
      else
        xv[p] = *reinterpret_cast<const u16x8*>(x + e);
    }
  };
  auto store_x = [&](int buf, int step) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      if (XR * 32 < NT && idx >= XR * 32) continue;
      u16x8 v = xv[p];
      if constexpr (kNorm) {
        const float r = rsv[min(row, M - 1)];
        const u16x8 gm = *reinterpret_cast<const u16x8*>(gl + k0 + step * 256 + col);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) * r * bf16_to_f32(gm[j]));
      }
      *reinterpret_cast<u16x8*>(&xs[buf * XR * CH_ROW + row * CH_ROW + col]) = v;
    }
  };
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (kEarlyW) {
    load_w(0, 0);
    if (NS > 1) load_w(1, 1);
    pre_x();
    load_x(0);
    store_x(0, 0);
    if (NS > 1) load_x(1);
  } else {
    pre_x();
    load_x(0);
    store_x(0, 0);
    if (NS > 1) load_x(1);
    load_w(0, 0);
    if (NS > 1) load_w(1, 1);
  }
  __syncthreads();
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    if (st + 1 < NS) store_x((st + 1) % 2, st + 1);
    if (st + 2 < NS) {
      load_x(st + 2);
      load_w((st + 2) % 3, st + 2);
    }
    const unsigned short* xb = &xs[(st % 2) * XR * CH_ROW + c * CH_ROW + 8 * g];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xb + 16 * t * CH_ROW + 32 * s);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ring[st % 3][s]),
                                                         __builtin_bit_cast(bf16x8, b), acc[t], 0, 0, 0);
      }
    }
    if (st + 1 < NS) __syncthreads();
  }
}

struct ChainArgs {
  // producer: partials of xa . Wa^T, residual += their sum, per-tile row sums of squares
  const unsigned short* xa;
  long xa_stride;
  const unsigned short* wa;   // pack_decode_weight layout [NA/128][KA/256][8][8][64][8]
  float* wsa;                 // [SA, M, NA]
  unsigned short* residual;   // [M, NA] bf16, contiguous
  float* sq;                  // [tilesA, 64]
  int NA, KA, SA, tilesA;
  // consumer: x = RMSNorm(residual) * gamma, out = x . Wb^T
  const unsigned short* wb;   // packed (glu = true: gate/up interleaved per 128-row tile)
  const unsigned short* gamma;
  float eps;
  unsigned short* act;        // kGlu, SB == 1: act [M, NB/2]
  long act_stride;
  float* wsb;                 // !kGlu: partials [SB, M, NB]
  int NB, SB, tilesB;
  int* sync;
  int M;
  unsigned long long* dbg;    // optional, 8 per block: start, gemm done | wait done, end, role, reduce
                              // wait done, reduce done, rdone seen (s_memrealtime, 100 MHz)
};

template <int MT, int NSA, int NSB, bool kGlu>
__global__ __launch_bounds__(512) void decode_chain_kernel(ChainArgs a) {
  using L = ChainLds<MT>;
  constexpr int XR = L::XR;
  __shared__ __attribute__((aligned(16))) unsigned short lds[L::TOTAL];
  unsigned short* xs = lds;
  unsigned short* gl = lds + L::X;
  float* rsv = reinterpret_cast<float*>(lds + L::X + L::G);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int M = a.M;
  const int nA = a.tilesA * a.SA;
  f32x4 acc[MT];
  unsigned long long* dbg = a.dbg != nullptr && tid == 0 ? a.dbg + 8 * blockIdx.x : nullptr;
  if (dbg) dbg[0] = __builtin_amdgcn_s_memrealtime();

  if ((int)blockIdx.x < nA) {
    // ---------------- producer ----------------
    const int split = blockIdx.x / a.tilesA, tile = blockIdx.x - split * a.tilesA;
    const int N = a.NA, K = a.KA, S = a.SA;
    const unsigned short* wp = a.wa + ((long)tile * (K >> 8) + (long)split * NSA) * 32768;
    chain_gemm<MT, NSA, false, false>(acc, xs, wp, a.xa, a.xa_stride, M, split * 256 * NSA, nullptr, nullptr,
                                      [] {}, buf_rsrc(nullptr, 0));
    // partials stored write-through (sc1): no release fence, the counter add follows the
    // drain of every storing wave (Guideline 16 R1)
    const auto rws = buf_rsrc(a.wsa, (unsigned)((long)S * M * N * 4));
    const int n = tile * 128 + wave * 16 + 4 * g;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + c;
      if (m < M)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[t]), rws,
                                               (int)((((long)split * M + m) * N + n) * 4), 0, kSc1);
    }
    if (dbg) dbg[1] = __builtin_amdgcn_s_memrealtime();
    vm_drain();
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(gw(a.sync + CH_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (dbg) {
        dbg[2] = __builtin_amdgcn_s_memrealtime();
        dbg[3] = 0;
      }
    }
    return;
  }

  // ---------------- consumer ----------------
  const int bid = blockIdx.x - nA;
  const int nB = a.tilesB * a.SB;
  const int split = bid / a.tilesB, tile = bid - split * a.tilesB;
  const int N = a.NB, K = a.NA;
  const int kvec = K >> 3;
  // the norm weight does not depend on the producer: load it now, store it after the wait
  const u16x8 gv = *reinterpret_cast<const u16x8*>(a.gamma + (long)min(tid, kvec - 1) * 8);
  const unsigned short* wp = a.wb + ((long)tile * (K >> 8) + (long)split * NSB) * 32768;
  // bounded relaxed poll of one counter by one lane (sc1 loads), then the block barrier
  auto wait_count = [&](int word, int target) __attribute__((always_inline)) {
    if (tid == 0) {
      int spins = 0;
      while (__hip_atomic_load(gw(a.sync + word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > CH_SPIN_MAX) {
          __hip_atomic_fetch_add(gw(a.sync + CH_ERR), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  };
  const int units = a.tilesA * MT;  // (128-column tile, 16-row group) reduction units
  auto wait_rows = [&]() __attribute__((always_inline)) {
    if (bid < units) {
      // this consumer also reduces one unit: sum the S slabs in slice order, add the
      // residual, store it back (bf16, sc1) and the unit's per-row sums of squares
      wait_count(CH_DONE, nA);
      if (dbg) dbg[4] = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the sc1 loads below
      __syncthreads();
      const int ut = bid % a.tilesA, rg = bid / a.tilesA;
      const int NAc = a.NA;
      if (tid < 256) {
        const int row = rg * 16 + (tid >> 4), ch = tid & 15;
        const int col = ut * 128 + ch * 8;
        float ss = 0.f;
        if (row < M) {
          const auto rws = buf_rsrc(a.wsa, (unsigned)((long)a.SA * M * NAc * 4));
          const u16x8 res = *reinterpret_cast<const u16x8*>(a.residual + (long)row * NAc + col);
          f32x4 lo, hi;
          sum_slabs_sc1(lo, hi, rws, (int)(((long)row * NAc + col) * 4), (int)((long)M * NAc * 4), a.SA);
          u16x8 r;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float h = bf16_to_f32(f32_to_bf16(j < 4 ? lo[j] : hi[j - 4]));
            r[j] = f32_to_bf16(h + bf16_to_f32(res[j]));
            const float v = bf16_to_f32(r[j]);
            ss += v * v;
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r),
                                                 buf_rsrc(a.residual, (unsigned)((long)M * NAc * 2)),
                                                 (int)(((long)row * NAc + col) * 2), 0, kSc1);
        }
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        ss += __shfl_xor(ss, 8, 64);
        if (ch == 0)
          __hip_atomic_store(gw(reinterpret_cast<int*>(a.sq) + ut * 64 + row), __float_as_int(ss), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      vm_drain();
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(gw(a.sync + CH_RDONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (dbg) dbg[5] = __builtin_amdgcn_s_memrealtime();
    }
    wait_count(CH_RDONE, units);
    if (dbg) dbg[6] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 &&
        __hip_atomic_fetch_add(gw(a.sync + CH_PASSED), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nB - 1) {
      // every consumer is past both waits and every producer has counted: reset for the next call
      __hip_atomic_store(gw(a.sync + CH_DONE), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gw(a.sync + CH_RDONE), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gw(a.sync + CH_PASSED), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every load of the handed-off bytes below (tile sums, residual rows) is sc1: no
    // acquire fence (Guideline 16, the sc1 row of the hand-off table); this fence emits
    // nothing and only keeps the compiler from hoisting them above the wait
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (tid < kvec) *reinterpret_cast<u16x8*>(gl + tid * 8) = gv;
    __syncthreads();
    // 1 / rms per row: 8 threads per row sum the tile sums (fixed order)
    if (tid < XR * 8) {
      const int row = tid >> 3, j = tid & 7;
      float ss = 0.f;
      for (int t = j; t < a.tilesA; t += 8)
        ss += __int_as_float(__hip_atomic_load(gw(reinterpret_cast<int*>(a.sq) + t * 64 + row), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT));
      ss += __shfl_xor(ss, 1, 64);
      ss += __shfl_xor(ss, 2, 64);
      ss += __shfl_xor(ss, 4, 64);
      if (j == 0) rsv[row] = rsqrtf(ss / K + a.eps);
    }
    __syncthreads();
    if (dbg) dbg[1] = __builtin_amdgcn_s_memrealtime();
  };
  chain_gemm<MT, NSB, true, true>(acc, xs, wp, a.residual, a.NA, M, split * 256 * NSB, rsv, gl, wait_rows,
                                  buf_rsrc(a.residual, (unsigned)((long)M * a.NA * 2)));

  if constexpr (kGlu) {
    // rows of wave w: 0-3 gate row groups, 4-7 the matching up rows (decode_gemm.hip kGlu)
    constexpr int EW = 16 * MT;
    float* ex = reinterpret_cast<float*>(xs);
    __syncthreads();
    if (wave >= 4) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ex[((wave - 4) * 16 + 4 * g + j) * EW + 16 * t + c] = bf16_to_f32(f32_to_bf16(acc[t][j]));
    }
    __syncthreads();
    if (wave < 4) {
      const int I = N >> 1;
      const int col = tile * 64 + wave * 16 + 4 * g;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + c;
        if (m >= M || col >= I) continue;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = silu_mul1(f32_to_bf16(acc[t][j]), f32_to_bf16(ex[(wave * 16 + 4 * g + j) * EW + 16 * t + c]));
        uint2 v;
        v.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
        v.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *reinterpret_cast<uint2*>(a.act + (long)m * a.act_stride + col) = v;
      }
    }
  } else {
    const int n = tile * 128 + wave * 16 + 4 * g;
    if (n < N) {
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + c;
        if (m < M) *reinterpret_cast<f32x4*>(a.wsb + ((long)split * M + m) * N + n) = acc[t];
      }
    }
  }
  if (dbg) {
    dbg[2] = __builtin_amdgcn_s_memrealtime();
    dbg[3] = 2;
  }
}

template <int MT, int NSA, int NSB, bool kGlu>
void chain_launch(const ChainArgs& a, hipStream_t s) {
  const int grid = a.tilesA * a.SA + a.tilesB * a.SB;
  decode_chain_kernel<MT, NSA, NSB, kGlu><<<grid, 512, 0, s>>>(a);
}

template <int MT, int NSA, bool kGlu>
bool chain_b(const ChainArgs& a, int nsb, hipStream_t s) {
  switch (nsb) {
    case 2: chain_launch<MT, NSA, 2, kGlu>(a, s); return true;
    case 4: chain_launch<MT, NSA, 4, kGlu>(a, s); return true;
    case 8: chain_launch<MT, NSA, 8, kGlu>(a, s); return true;
    case 16: chain_launch<MT, NSA, 16, kGlu>(a, s); return true;
    default: return false;
  }
}

template <int MT, bool kGlu>
bool chain_a(const ChainArgs& a, int nsa, int nsb, hipStream_t s) {
  switch (nsa) {
    case 2: return chain_b<MT, 2, kGlu>(a, nsb, s);
    case 4: return chain_b<MT, 4, kGlu>(a, nsb, s);
    case 7: return chain_b<MT, 7, kGlu>(a, nsb, s);
    default: return false;
  }
}

}  // namespace

int decode_chain_sync_words(int) { return CH_WORDS; }

bool decode_chain_supported(int M, int NA, int KA, int SA, int NB, int SB, bool glu) {
  if (M < 17 || M > 64 || NA % 128 || NB % 128 || NA > CH_KMAX || NA % 256 || KA % (256 * SA) || NA % (256 * SB))
    return false;
  if (glu && SB != 1) return false;
  // every (tile, 16-row group) reduction unit needs a consumer block to run it
  if (NB / 128 * SB < NA / 128 * (M > 32 ? 4 : 2)) return false;
  const int nsa = KA / (256 * SA), nsb = NA / (256 * SB);
  return (nsa == 2 || nsa == 4 || nsa == 7) && (nsb == 2 || nsb == 4 || nsb == 8 || nsb == 16);
}

bool launch_decode_chain(const void* xa, long xa_stride, const void* wa, float* wsa, void* residual, float* sq,
                         int NA, int KA, int SA, const void* wb, const void* gamma, float eps, void* act,
                         long act_stride, float* wsb, int NB, int SB, bool glu, int* sync, int M, hipStream_t s,
                         unsigned long long* dbg) {
  if (!decode_chain_supported(M, NA, KA, SA, NB, SB, glu)) return false;
  ChainArgs a;
  a.xa = static_cast<const unsigned short*>(xa);
  a.xa_stride = xa_stride;
  a.wa = static_cast<const unsigned short*>(wa);
  a.wsa = wsa;
  a.residual = static_cast<unsigned short*>(residual);
  a.sq = sq;
  a.NA = NA;
  a.KA = KA;
  a.SA = SA;
  a.tilesA = NA / 128;
  a.wb = static_cast<const unsigned short*>(wb);
  a.gamma = static_cast<const unsigned short*>(gamma);
  a.eps = eps;
  a.act = static_cast<unsigned short*>(act);
  a.act_stride = act_stride;
  a.wsb = wsb;
  a.NB = NB;
  a.SB = SB;
  a.tilesB = NB / 128;
  a.sync = sync;
  a.M = M;
  a.dbg = dbg;
  const int nsa = KA / (256 * SA), nsb = NA / (256 * SB);
  if (M > 32) return glu ? chain_a<4, true>(a, nsa, nsb, s) : chain_a<4, false>(a, nsa, nsb, s);
  return glu ? chain_a<2, true>(a, nsa, nsb, s) : chain_a<2, false>(a, nsa, nsb, s);
}

}  // namespace hipserve
