// Decode GEMM with the layer's epilogue INSIDE the launch (fused decode layer v2,
// VERDICT r2 next-round item 2): a Llama decode layer becomes five kernels,
//   qkv GEMM [+ input RMSNorm on load] -> RoPE + paged-KV write in the fix-up,
//   paged attention,
//   o_proj GEMM -> residual add + per-tile sums of squares in the fix-up,
//   gate|up GEMM [+ post-attention RMSNorm on load] -> SiLU-GLU,
//   down GEMM -> residual add + per-tile sums of squares in the fix-up,
// instead of eight (v1: every split-K GEMM left fp32 partials for a separate
// epilogue kernel, profiles/r2_bench_llama3_8b_bf16_v10_trace.md: 3 epilogue
// kernels per layer, ~5.5 us each + a ~1.7 us launch boundary each).
//
// Split-K fix-up ("stream-K last arriver"): every workgroup of a 128-row weight
// tile writes its fp32 partial slab, then (every wave drained, barrier) lane 0
// releases at agent scope and draws a ticket from the tile's counter; the
// workgroup that draws S-1 acquires at agent scope and sums ALL S slabs in slice
// order 0..S-1 (the order of v1's epilogue kernels, so the sums are bit-identical)
// and runs the epilogue for the whole tile, then resets the counter for the next
// call / graph replay. Correct for any placement of a tile's slices over XCDs
// (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2 recipe); the
// slices of a tile are launched blockIdx-congruent mod 8 (slice-major grid with
// tiles % 8 == 0), so the last arriver's slab reads are normally same-XCD.
//
// RMSNorm on load: the residual-add epilogues leave the bf16 residual plus one fp32
// sum of squares per (row, 128-column tile); the consumer GEMM sums a row's tile
// partials (fixed order), forms inv = rsqrt(ss / K + eps) once per row in its
// prologue and stages x = bf16(residual * inv * w) into LDS — the rounding points of
// the unfused RMSNorm; only ss's summation order differs (a different fp32
// association: TP tests and the fused-vs-unfused tests allow for it).
//
// The GEMM body is decode_gemm.hip's packed kernel at RT = 1 (8 waves, 128 weight
// rows per workgroup; one tile = one 128-wide head for the RoPE epilogue).
#include "hipserve/common.h"
#include "hipserve/kernels.h"

namespace hipserve {

constexpr int DL_LDS_ROW = 264;  // 256 + 8 bf16 pad -> 528 B row stride (conflict-free ds_read_b128)
enum { FIX_ADD = 1, FIX_ROPE = 2, FIX_GLU = 3 };

template <int MT, int NSTEPS, int kFix, bool kNormIn>
__global__ __launch_bounds__(512) void dgf_kernel(DgfArgs A, const unsigned short* __restrict__ x, long x_stride,
                                                  const unsigned short* __restrict__ w, int M, int N, int K, int S,
                                                  int tiles) {
  constexpr int NW = 128, XR = 16 * MT, NT = 512, XPASS = XR * 32 / NT;
  __shared__ __attribute__((aligned(16))) unsigned short xs[2][XR * DL_LDS_ROW];
  __shared__ float s_inv[XR];
  __shared__ float s_red[8][XR];
  __shared__ __attribute__((aligned(16))) unsigned short s_nw[kNormIn ? 256 * NSTEPS : 8];  // norm weight slice
  __shared__ int s_ticket;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int split = blockIdx.x / tiles, tile = blockIdx.x - split * tiles;
  const int k0 = split * 256 * NSTEPS;
  const int nbase = tile * NW + wave * 16;
  // packed weight: [tile][kstep][row group = wave][slot s][lane][8]
  const unsigned short* wr = w + ((long)tile * (K >> 8) + (long)split * NSTEPS) * (NW * 256) + (long)wave * 4096 +
                             lane * 8;

  if constexpr (kNormIn) {
    if (tid < XR) {
      const int row = min(tid, M - 1);
      float ss = 0.f;
      for (int i = 0; i < A.Tin; ++i) ss += A.ss_in[(long)i * M + row];
      s_inv[tid] = rsqrtf(ss / K + A.eps);
    }
    for (int i = tid; i < 32 * NSTEPS; i += NT)
      reinterpret_cast<u16x8*>(s_nw)[i] = reinterpret_cast<const u16x8*>(A.norm_w + k0)[i];
  }
  u16x8 xv[XPASS];
  auto load_x = [&](int step) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      xv[p] = *reinterpret_cast<const u16x8*>(x + (long)min(row, M - 1) * x_stride + k0 + step * 256 + col);
    }
  };
  // step = the 256-k step whose x the buffer receives (for the norm weight slice)
  auto store_x = [&](int buf, int step) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) {
      const int idx = p * NT + tid, row = idx >> 5, col = (idx & 31) * 8;
      u16x8 v = xv[p];
      if constexpr (kNormIn) {
        const float iv = s_inv[row];
        const u16x8 nw = *reinterpret_cast<const u16x8*>(&s_nw[step * 256 + col]);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = f32_to_bf16(bf16_to_f32(v[j]) * iv * bf16_to_f32(nw[j]));
      }
      *reinterpret_cast<u16x8*>(&xs[buf][row * DL_LDS_ROW + col]) = v;
    }
  };

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 ring[3][8];
  auto load_w = [&](int slot, int step) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
      ring[slot][s] = __builtin_nontemporal_load(
          reinterpret_cast<const u16x8*>(wr + (long)step * (NW * 256) + 512 * s));
  };
  load_x(0);
  if constexpr (kNormIn) __syncthreads();  // s_inv, s_nw
  store_x(0, 0);
  if (NSTEPS > 1) load_x(1);
  load_w(0, 0);
  if (NSTEPS > 1) load_w(1, 1);
  __syncthreads();
#pragma unroll
  for (int st = 0; st < NSTEPS; ++st) {
    if (st + 1 < NSTEPS) store_x((st + 1) % 2, st + 1);
    if (st + 2 < NSTEPS) {
      load_x(st + 2);
      load_w((st + 2) % 3, st + 2);
    }
    const unsigned short* xb = &xs[st % 2][c * DL_LDS_ROW + 8 * g];
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u16x8 b = *reinterpret_cast<const u16x8*>(xb + 16 * t * DL_LDS_ROW + 32 * s);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ring[st % 3][s]),
                                                         __builtin_bit_cast(bf16x8, b), acc[t], 0, 0, 0);
      }
    if (st + 1 < NSTEPS) __syncthreads();
  }

  // C fragment: column m = 16t + c (token), rows n = nbase + 4g + j (output feature)
  const int n = nbase + 4 * g;
  if (S > 1) {
    // ---- publish this slice's slab, take a ticket; the last arriver reduces
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + c;
      if (m < M) *reinterpret_cast<f32x4*>(A.ws + ((long)split * M + m) * N + n) = acc[t];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_ticket = __hip_atomic_fetch_add(&A.counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_ticket != S - 1) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&A.counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // sum the S slabs in slice order (batches of 8 loads, no per-slab branch)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const float* p = A.ws + (long)min(16 * t + c, M - 1) * N + n;
      f32x4 tot;
      for (int s0 = 0; s0 < S; s0 += 8) {
        f32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const f32x4*>(p + (long)min(s0 + j, S - 1) * M * N);
        if (s0 == 0) tot = v[0];
        else tot += v[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)
          if (s0 + j < S) tot += v[j];
      }
      acc[t] = tot;
    }
  }

  // ---- epilogues on the complete tile (acc = sum over K)
  if constexpr (kFix == FIX_ADD) {
    // residual[m, n] = bf16(bf16(h) + residual); per-row partial sum of squares over the tile
    float ssm[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int m = 16 * t + c;
      ssm[t] = 0.f;
      if (m < M) {
        uint2* rp = reinterpret_cast<uint2*>(A.residual + (long)m * N + n);
        const uint2 rv = *rp;
        const unsigned short r0[4] = {(unsigned short)(rv.x & 0xffff), (unsigned short)(rv.x >> 16),
                                      (unsigned short)(rv.y & 0xffff), (unsigned short)(rv.y >> 16)};
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = f32_to_bf16(bf16_to_f32(f32_to_bf16(acc[t][j])) + bf16_to_f32(r0[j]));
          const float f = bf16_to_f32(o[j]);
          ssm[t] += f * f;
        }
        uint2 ov;
        ov.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
        ov.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *rp = ov;
      }
      // lanes c, c+16, c+32, c+48 hold the same row: fold the 4 lane groups
      ssm[t] += __shfl_xor(ssm[t], 16, 64);
      ssm[t] += __shfl_xor(ssm[t], 32, 64);
      if (g == 0) s_red[wave][16 * t + c] = ssm[t];
    }
    __syncthreads();
    if (tid < XR && tid < M) {
      float tot = 0.f;
#pragma unroll
      for (int wv = 0; wv < 8; ++wv) tot += s_red[wv][tid];
      A.ss_out[(long)tile * M + tid] = tot;
    }
  } else if constexpr (kFix == FIX_GLU) {
    // rows: waves 0-3 = 64 gate rows, waves 4-7 = the matching 64 up rows
    constexpr int EW = XR;
    float* ex = reinterpret_cast<float*>(&xs[0][0]);
    __syncthreads();  // every wave is done with the x ring
    if (wave >= 4) {
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ex[((wave - 4) * 16 + 4 * g + j) * EW + 16 * t + c] = bf16_to_f32(f32_to_bf16(acc[t][j]));
    }
    __syncthreads();
    if (wave < 4) {
      const int col = tile * 64 + wave * 16 + 4 * g;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + c;
        if (m >= M) continue;
        unsigned short o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = silu_mul1(f32_to_bf16(acc[t][j]), f32_to_bf16(ex[(wave * 16 + 4 * g + j) * EW + 16 * t + c]));
        uint2 v;
        v.x = (unsigned)o[0] | ((unsigned)o[1] << 16);
        v.y = (unsigned)o[2] | ((unsigned)o[3] << 16);
        *reinterpret_cast<uint2*>(A.out + (long)m * A.out_stride + col) = v;
      }
    }
  } else if constexpr (kFix == FIX_ROPE) {
    // the tile (128 features = 128 / D heads) through LDS as bf16-rounded floats,
    // then one 8-wide (pair) chunk per work item: bias, q/k RMSNorm, RoPE, stores
    float* tl = reinterpret_cast<float*>(&xs[0][0]);  // [128][XR]
    __syncthreads();
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nl = wave * 16 + 4 * g + j;
        float v = bf16_to_f32(f32_to_bf16(acc[t][j]));
        if (A.bias != nullptr) v = bf16_to_f32(f32_to_bf16(v + bf16_to_f32(A.bias[tile * NW + nl])));
        tl[nl * XR + 16 * t + c] = v;
      }
    __syncthreads();
    const int D = A.D, half = D >> 1, hpt = NW / D;
    const int mode = A.rope_mode;
    const int per_head = mode == 0 ? D / 16 : D / 8;  // chunks per head (a 2^k lane group)
    const int items = XR * hpt * per_head;
    for (int it = tid; it < items; it += NT) {
      const int cc = it % per_head, hl = (it / per_head) % hpt, m = it / (per_head * hpt);
      const bool live = m < M;
      const int mm = live ? m : M - 1;
      const int h = tile * hpt + hl;  // global head index: q heads, then k heads, then v heads
      const long pos = A.positions[mm];
      const long slot = A.slots[mm];
      const long blk = slot >= 0 ? slot / A.block_size : 0;
      const int off = slot >= 0 ? (int)(slot % A.block_size) : 0;
      const float* cs = A.cos_sin + pos * D;
      const float* src = tl + (long)hl * D * XR + mm;
      if (h >= A.nq + A.nkv) {  // V head: copy into the transposed cache block
        const int kh = h - A.nq - A.nkv;
        if (live && slot >= 0) {
          unsigned short* vc = A.v_cache + (blk * A.nkv + kh) * (long)D * A.block_size + off;
          const int d0 = mode == 0 ? cc * 8 : cc * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) vc[(d0 + j) * A.block_size] = f32_to_bf16(src[(d0 + j) * XR]);
          if (mode == 0)
#pragma unroll
            for (int j = 0; j < 8; ++j)
              vc[(half + d0 + j) * A.block_size] = f32_to_bf16(src[(half + d0 + j) * XR]);
        }
        continue;
      }
      const bool is_q = h < A.nq;
      unsigned short* dst = is_q ? A.q_out + (long)mm * A.q_stride + (long)h * D
                                 : A.k_cache + ((blk * A.nkv + (h - A.nq)) * A.block_size + off) * (long)D;
      const bool store = live && (is_q || slot >= 0);
      if (mode == 0) {
        float xa[8], ya[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xa[j] = src[(cc * 8 + j) * XR];
          ya[j] = src[(half + cc * 8 + j) * XR];
        }
        if (A.qw != nullptr) {  // per-head q / k RMSNorm (Qwen3) over the head's D values
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += xa[j] * xa[j] + ya[j] * ya[j];
          for (int o = per_head / 2; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
          const float inv = rsqrtf(ss / D + A.eps);
          const float* nwp = is_q ? A.qw : A.kw;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            xa[j] = bf16_to_f32(f32_to_bf16(xa[j] * inv * nwp[cc * 8 + j]));
            ya[j] = bf16_to_f32(f32_to_bf16(ya[j] * inv * nwp[half + cc * 8 + j]));
          }
        }
        u16x8 va, vb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float ra, rb;
          rope_rot(xa[j], ya[j], cs[cc * 8 + j], cs[half + cc * 8 + j], ra, rb);
          va[j] = f32_to_bf16(ra);
          vb[j] = f32_to_bf16(rb);
        }
        if (store) {
          *reinterpret_cast<u16x8*>(dst + cc * 8) = va;
          *reinterpret_cast<u16x8*>(dst + half + cc * 8) = vb;
        }
      } else {  // interleaved pairs (2i, 2i + 1): GGUF llama
        float xa[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xa[j] = src[(cc * 8 + j) * XR];
        u16x8 v;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int i = cc * 4 + p;
          float ra, rb;
          rope_rot(xa[2 * p], xa[2 * p + 1], cs[i], cs[half + i], ra, rb);
          v[2 * p] = f32_to_bf16(ra);
          v[2 * p + 1] = f32_to_bf16(rb);
        }
        if (store) *reinterpret_cast<u16x8*>(dst + cc * 8) = v;
      }
    }
  }
}

template <int MT, int kFix, bool kNormIn>
static bool dgf_steps(const DgfArgs& A, const void* x, long x_stride, const void* w, int M, int N, int K, int S,
                      hipStream_t s) {
  const int tiles = N / 128;
  auto* xi = static_cast<const unsigned short*>(x);
  auto* wi = static_cast<const unsigned short*>(w);
#define DGF_CASE(NS)                                                                                 \
  case NS:                                                                                           \
    dgf_kernel<MT, NS, kFix, kNormIn><<<tiles * S, 512, 0, s>>>(A, xi, x_stride, wi, M, N, K, S, tiles); \
    return true;
  switch (K / S / 256) {
    DGF_CASE(1)
    DGF_CASE(2)
    DGF_CASE(4)
    DGF_CASE(7)
    DGF_CASE(8)
    DGF_CASE(16)
    default: return false;
  }
#undef DGF_CASE
}

template <int kFix, bool kNormIn>
static bool dgf_mt(const DgfArgs& A, const void* x, long x_stride, const void* w, int M, int N, int K, int S,
                   hipStream_t s) {
  if (M <= 16) return dgf_steps<1, kFix, kNormIn>(A, x, x_stride, w, M, N, K, S, s);
  if (M <= 32) return dgf_steps<2, kFix, kNormIn>(A, x, x_stride, w, M, N, K, S, s);
  if (M <= 64) return dgf_steps<4, kFix, kNormIn>(A, x, x_stride, w, M, N, K, S, s);
  return false;
}

bool dgf_supported(int fix, bool norm_in, int M, int N, int K, int S) {
  if (M < 1 || M > 64 || N % 128 || K % 256 || S < 1 || K % (256 * S)) return false;
  const int ns = K / S / 256;
  if (ns != 1 && ns != 2 && ns != 4 && ns != 7 && ns != 8 && ns != 16) return false;
  if (fix == FIX_ADD) return !norm_in;
  return fix == FIX_ROPE || (fix == FIX_GLU && norm_in);
}

bool launch_dgf(int fix, bool norm_in, const DgfArgs& A, const void* x, long x_stride, const void* w, int M, int N,
                int K, int S, hipStream_t s) {
  if (!dgf_supported(fix, norm_in, M, N, K, S)) return false;
  if (fix == FIX_ADD) return dgf_mt<FIX_ADD, false>(A, x, x_stride, w, M, N, K, S, s);
  if (fix == FIX_GLU) return dgf_mt<FIX_GLU, true>(A, x, x_stride, w, M, N, K, S, s);
  if (norm_in) return dgf_mt<FIX_ROPE, true>(A, x, x_stride, w, M, N, K, S, s);
  return dgf_mt<FIX_ROPE, false>(A, x, x_stride, w, M, N, K, S, s);
}

}  // namespace hipserve
