// hipserve — host-side launchers of the gfx950 kernels. Raw pointers + stream
// only (no torch types) so each .hip translation unit compiles without the
// heavy ATen headers; csrc/torch_bindings.cpp validates tensors and calls these.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace hipserve {

// norm.hip — residual != nullptr selects the fused add (residual updated in place)
void launch_embed_rmsnorm(void* out, void* residual, const void* table, const long* ids, const long* src,
                          const long* tok, const void* w, bool weight_f32, int rows, int hidden, float eps,
                          hipStream_t s, float scale = 1.f, void* out8 = nullptr, float* xs8 = nullptr);
// out8 / xs8 (optional): out also as per-token e4m3 + row scale (= act_quant_fp8 of out)
void launch_rmsnorm(void* out, void* residual, const void* x, const void* w,
                    bool weight_f32, int rows, int hidden, long x_stride,
                    long out_stride, float eps, hipStream_t s, void* out8 = nullptr, float* xs8 = nullptr);
// per-head q/k RMSNorm inside the qkv rows, in place (fp32 weights [D], D <= 256)
void launch_qk_rmsnorm(void* qkv, long stride, const float* qw, const float* kw, int T, int nq, int nkv, int D,
                       float eps, hipStream_t s);

// activation.hip
void launch_silu_and_mul(void* out, const void* in, long rows, int inter,
                         long in_stride, long out_stride, hipStream_t s);
void launch_gelu_and_mul(void* out, const void* in, long rows, int inter,
                         long in_stride, long out_stride, hipStream_t s);

// rope_cache.hip
void launch_rope_cache(void* qkv, long qkv_stride, const long* positions,
                       const long* slots, const float* cos_sin, void* k_cache,
                       void* v_cache, int T, int nq, int nkv, int D,
                       int block_size, int mode, hipStream_t s, bool kv_f8 = false);

// attention_decode.hip
size_t paged_decode_smem_bytes(int D);
// fused decode: qkv split-K partials [S, B, N] -> RoPE(q, k) + KV write + attention
void launch_paged_decode_qkv(void* out, long out_stride, const float* ws, int S, int N, const long* positions,
                             const long* slots, const float* cos_sin, int mode, void* k_cache, void* v_cache,
                             const int* block_tables, int bt_stride, const int* context_lens, float* tmp_out,
                             float* tmp_ml, int B, int nq, int nkv, int D, int block_size, int part_size,
                             int max_parts, float scale, int window, hipStream_t s, void* out16 = nullptr,
                             const float* qw = nullptr, const float* kw = nullptr, float eps = 1e-6f);
// out16 (optional): f16 pair-order copy of out for a quantised o-projection (out's row stride)
void launch_paged_decode(void* out, long out_stride, const void* q, long q_stride,
                         const void* k_cache, const void* v_cache,
                         const int* block_tables, int bt_stride,
                         const int* context_lens, float* tmp_out, float* tmp_ml,
                         int B, int nq, int nkv, int D, int block_size,
                         int part_size, int max_parts, float scale, int window,
                         hipStream_t s, void* out16 = nullptr, bool kv_f8 = false);

// attention_prefill.hip — window > 0: sliding-window attention (keys within
// window - 1 positions before the query), 0 = full causal
void launch_prefill_attention(void* out, long out_stride, const void* q,
                              long q_stride, const void* k_cache,
                              const void* v_cache, const int* block_tables,
                              int bt_stride, const int* cu_q, const int* ctx_lens,
                              const int* tiles, int ntiles, int nq, int nkv, int D,
                              int block_size, float scale, int window, hipStream_t s, bool kv_f8 = false);

// sampling.hip
// ws: fp32 workspace of sample_workspace_floats(rows, V) for the multi-CU path
// (vocab >= 8192); nullptr selects the one-workgroup-per-row kernel.
size_t sample_workspace_floats(int rows, int V);
void launch_sample(long* out_tok, float* out_lp, const void* logits, bool is_bf16,
                   long stride, int rows, int V, const float* temperature,
                   const int* top_k, const float* top_p, const long* seeds,
                   const long* steps, float* ws, hipStream_t s, bool two_rounds = true);

// penalties.hip — device-side OpenAI penalties + top-n logprobs (graph-capturable).
// counts int32 [slots, V], seen bits [slots, ceil(V/32)]; slot < 0: row untouched.
void launch_penalty_apply(void* logits, bool is_bf16, long stride, int rows, int V, const int* slot,
                          const float* pres, const float* freq, const float* rep, const int* counts,
                          const unsigned int* seen, hipStream_t s);
void launch_penalty_update(const long* tok, const int* slot, int n, int* counts, unsigned int* seen, int V,
                           hipStream_t s);
void launch_penalty_init(int* counts, unsigned int* seen, int V, const int* slots, const int* off,
                         const int* n_prompt, const int* toks, int ninit, hipStream_t s);
void launch_top_logprobs(const void* logits, bool is_bf16, long stride, int rows, int V, const int* nreq,
                         int* out_ids, float* out_lp, int K, hipStream_t s);

// gguf.hip — qtype: 0 Q4_0, 1 Q4_1, 2 Q8_0, 3 Q4_K, 4 Q5_K, 5 Q6_K (repacked layouts)
void launch_gguf_gemm(void* out, float* ws, const void* x, long x_stride, long out_stride,
                      const void* q, const void* d, const void* m, int qtype, long row_bytes,
                      int M, int N, int K, int splits, hipStream_t s);
void launch_gguf_dequant(void* out, const void* q, const void* d, const void* m, int qtype,
                         long row_bytes, int N, int K, hipStream_t s);
// gguf_mfma.hip — decode GEMM v2 over the parts of a merged projection, weights in
// the tiled layout ([N/16][K/256][chunk]): out[:, col + n] (bf16, S == 1) or
// ws[S, M, Ntot] fp32 partials. M <= 64, parts' rows % 16 == 0.
struct GgufPart {
  const void* q;
  const float* rs;  // FP8 formats: per-row output scale
  int qtype;
  int rows;
  int col;
};
int gguf_tiled_chunk_bytes(int qtype);
// x16 (optional, M <= 64): x as f16 in the kernel's staging pair order {0,2,1,3,4,6,5,7}
// per aligned 8-run, row stride x_stride (decode_fused.hip producers write it)
void launch_gguf_gemm_parts(void* out, long out_stride, float* ws, const void* x, long x_stride,
                            const GgufPart* parts, int nparts, int M, int Ntot, int K, int S, hipStream_t s,
                            const void* x16 = nullptr);
void launch_gguf_dequant_tiled(void* out, const void* q, const float* rs, int qtype, int N, int K, hipStream_t s,
                               int pack = 0, int nrows = 0, bool kmajor = false);
// per-channel FP8 tiled part -> row-major [N, K] e4m3 bytes (N % 16 == 0, K % 256 == 0)
void launch_fp8_untile(void* out, const void* q, int N, int K, hipStream_t s);
// prefill GEMM straight from the tiled GGUF blocks on launch_x_f16_pairs' x16 / rsc (epi:
// PW_EPI_STORE / ADD / GLU / GEGLU; GLU: parts 0 / 1 = gate / up); false if the formats /
// shapes are not taken
bool launch_gguf_prefill(int epi, void* out, long ldo, const void* x16, const float* rsc, const GgufPart* parts,
                         int nparts, int M, int K, hipStream_t s);
// x [M, K] bf16 -> x16 [M, K] f16 (pair order, rows pre-scaled by 1 / rsc[m], powers of two)
void launch_x_f16_pairs(void* x16, float* rsc, const void* x, long ldx, int M, int K, hipStream_t s);
// quantised MoE experts (tiled layout per expert, stacked [E][N/16][K/256][chunk]) over
// moe_align tiles of 16/32/64 slots: out[slot, N] bf16 (S == 1) or ws[S, nslots, N] fp32.
// qtype: FP8 (rs [E, N]) or INT8 (the checkpoint expert formats). Returns false for an
// unsupported tile / qtype.
bool launch_qmoe_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* q,
                      const float* rs, int qtype, long w_estride, long rs_estride, const int* slots,
                      const int* tile_expert, int tiles_cap, int tile, int gather_k, int N, int K, int S,
                      hipStream_t s, bool kmajor = false, int glu = 0);

}  // namespace hipserve

namespace hipserve {
// skinny_gemm.hip — decode GEMM out[M,N] = x[M,K] . W[N,K]^T (M <= 64, K % (256*kw) == 0)
bool launch_skinny_gemm(void* out, const void* x, long x_stride, const void* w, long out_stride, int M,
                        int N, int K, int rt, int kw, hipStream_t s);

// allreduce.hip — custom all-reduce over HIP-IPC peer memory (one-shot / two-shot)
void* car_create(int rank, int world, size_t max_bytes, int nb_large);
void car_get_handle(void* state, void* handle_out);
void car_open(void* state, int peer, const void* handle);
bool car_error(void* state);
void car_destroy(void* state);
size_t car_max_bytes(void* state);
void launch_car(void* state, const void* inp, void* out, size_t bytes, bool two_shot, int blocks, hipStream_t s);
// [rows, row_bytes] shard of every rank -> out [rows, world * row_bytes] (rank-major within a row)
void launch_car_all_gather(void* state, const void* inp, void* out, size_t shard_bytes, size_t row_bytes,
                           hipStream_t s);
// Row-parallel projection epilogue: h = bf16(sum over ranks of (sum_s x[s])); residual = bf16(h + residual);
// out = rmsnorm(residual) * w. x: fp32 split-K partials [S, M, N] (x_f32) or bf16 [M, N] (S = 1).
// exch_f32: exchange fp32 partial sums (TP = N within fp32 rounding of TP = 1) or bf16 (half the bytes).
bool car_norm_fits(void* state, int M, int N, bool exch_f32);
void launch_car_add_rmsnorm(void* state, void* out, void* residual, const void* x, bool x_f32, int S,
                            const void* w, bool weight_f32, int M, int N, float eps, bool exch_f32, hipStream_t s);

// init.hip — on-device synthetic weights keyed by global coordinates (TP-invariant)
void launch_fill_uniform(void* out, long ld, int rows, int cols, long row0, long col0, long gcols,
                         unsigned int key, float scale, hipStream_t s);

// decode_gemm.hip — split-K LDS-shared decode GEMM (M <= 64, K % (256*S) == 0). S > 1 needs
// ws >= S*M*N fp32 and N % 8 == 0. Returns false for an uncompiled rt.
// packed = w in the pack_decode_weight layout ([ceil(N/128)][K/256][8][8][64][8] bf16).
// flags: DG_GLU (w packed with glu=true; out = act [M, N/2] = silu(gate) * up; packed only),
//        DG_PARTIAL (ws != nullptr: write the fp32 partials [S, M, N], no reduce launch).
// ws == nullptr requires S == 1 (bf16 out written directly).
constexpr int DG_GLU = 1, DG_PARTIAL = 2;
bool launch_decode_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w, int M,
                        int N, int K, int rt, int S, bool packed, int flags, hipStream_t s);


// prefill epilogues (prefill_gemm.hip FP8 kernel, prefill_gemm_packed.hip):
//   PG_EPI_STORE  C = bf16(acc)
//   PG_EPI_ADD    C (the residual, in place) = bf16(bf16(acc) + C)
//   PG_EPI_GLU    C = act [M, I] = silu(gate) * up of a merged [gate; up] weight
//   PG_EPI_GEGLU  as GLU with tanh-GELU(gate) * up (Gemma)
constexpr int PG_EPI_STORE = 0, PG_EPI_ADD = 1, PG_EPI_GLU = 2, PG_EPI_GEGLU = 3;
// prefill_gemm_packed.hip — C[M, N] = X[M, K] . W[N, K]^T with W in pack_decode_weight's
// layout (the decode GEMMs' copy; no second copy of the weight), K % 256 == 0, any M, N.
// wm = 1: 128 x 512 workgroup tiles, wm = 2: 256 x 256. bias (bf16 [N], STORE only) may be null.
//   PW_EPI_STORE / PW_EPI_ADD as PG_*; PW_EPI_GLU / PW_EPI_GEGLU: W packed with glu = true
//   (merged [gate; up], N = 2I, I % 64 == 0), C = act [M, I]
constexpr int PW_EPI_STORE = 0, PW_EPI_ADD = 1, PW_EPI_GLU = 2, PW_EPI_GEGLU = 3;
// grid_req <= 0: persistent (one workgroup per CU walking the tiles), else that many workgroups.
// rw: weight register sets in flight (2 or 4 32-deep slots ahead; 5 = 4 with each reload
// issued one MFMA group later).
// group (MoE experts, STORE / GLU): X = expert-sorted slots in 128 * wm-row tiles, m-tile tm
// uses expert tile_expert[tm]'s packed weight at Wp + e * estride; *num_tiles valid m-tiles.
struct PwGroup {
  const int* tile_expert;
  const int* num_tiles;
  long estride;  // elements between consecutive experts' packed weights
  // optional fused moe_gather: X is the token rows [x_rows, K] and slot row s of the
  // expert-sorted tiles reads token gather_slots[s] / gather_k (zeros for padding, -1)
  const int* gather_slots = nullptr;
  int gather_k = 1;
  int x_rows = 0;
};
bool launch_prefill_gemm_packed(int epi, void* C, long ldc, const void* X, long ldx, const void* Wp, int M, int N,
                                int K, const void* bias, int wm, int grid_req, hipStream_t s,
                                const PwGroup* group = nullptr, int rw = 4);
// FP8 (W8A8) form: A = per-token e4m3 activations [M, K] bytes (row scale xs[M]),
// B = e4m3 weights in the decode kernel's tiled layout (gguf_mfma.hip: [N/16][K/256]
// [4096 B]) as up to 4 parts stacked along N (each rows % 256 == 0; GLU: part 0 =
// gate, part 1 = up, equal rows % 128 == 0), per-row scale rs (x 256, the decode
// path's convention). C = epilogue(acc * xs[m] * rs[n] / 256). K % 256 == 0.
constexpr int kPgF8Parts = 4;
struct PgF8Part {
  const unsigned char* q;
  const float* rs;
  int rows;
  int tile0;  // first 256-column tile of the part (non-GLU)
};
struct PgF8 {
  PgF8Part p[kPgF8Parts];
  int n;
  const float* xs;
};
bool launch_prefill_gemm_f8(int epi, void* C, long ldc, const void* A, long lda, const PgF8& W, int M, int N, int K,
                            hipStream_t s);
// FP8 W8A8 decode GEMM (fp8_decode.hip), M <= 64: fp32 split-K partials
// ws[S, M, N] = (xq . wq^T over K slice s) * xs[m] * rs[n] / 256; (K / 256) / S in
// {1, 2, 3, 4, 6, 7, 8, 12, 14, 16, 21}; part rows % 16 == 0. W.xs = xs.
bool launch_fp8_decode_gemm(float* ws, const void* xq, const PgF8& W, int M, int N, int K, int S, hipStream_t s);
// act = silu / gelu_tanh(gate) * up of [gate | up] rows, written as per-token e4m3 q8 [rows,
// inter] + xs [rows] (and bf16 into out if non-null); inter / 8 <= 4096. activation.hip
bool launch_glu_quant(bool gelu, void* out, void* q8, float* xs, const void* in, long rows, int inter,
                      long in_stride, hipStream_t s);
// per-token dynamic e4m3 quantisation: xs[m] = max|x[m, :]| / 448, q = sat(x / xs)
void launch_act_quant_fp8(void* q, float* xs, const void* x, long x_stride, int M, int K, hipStream_t s);

// decode_fused.hip — split-K partial reductions fused with the next op of the layer
// ws: [S, M, N] fp32 partials. h = bf16(sum_s ws); residual = bf16(h + residual);
// out = rmsnorm(residual) * w  (bit-identical to splitk_reduce + fused_add_rmsnorm)
// out16 (optional): out also as f16 in the quantised GEMM's staging pair order (gguf_mfma.hip kX16)
// out8 / xs8 (optional): out also as per-token e4m3 + row scale for the W8A8 decode GEMM
// (fp8_decode.hip), bit-identical to act_quant_fp8 of out
void launch_splitk_add_rmsnorm(void* out, void* residual, const float* ws, int S, const void* w, bool weight_f32,
                               int M, int N, float eps, hipStream_t s, void* out16 = nullptr, void* out8 = nullptr,
                               float* xs8 = nullptr);
// sandwich norm (Gemma-3): residual = bf16(RMSNorm(bf16(sum_s ws)) * w_post + residual);
// out = RMSNorm(residual) * w_next (both weights bf16, or both fp32)
void launch_splitk_post_add_rmsnorm(void* out, void* residual, const float* ws, int S, const void* w_post,
                                    const void* w_next, bool weight_f32, int M, int N, float eps, hipStream_t s,
                                    void* out16 = nullptr, void* out8 = nullptr, float* xs8 = nullptr);
// qkv = bf16(sum_s ws) -> RoPE(q, k) -> q into qkv[:, :nq*D], k/v into the paged cache
// out[M, N] (bf16, row stride out_stride) = sum of the fp32 partials ws[S, M, N] (decode_gemm.hip)
void launch_splitk_reduce(void* out, long out_stride, const float* ws, int M, int N, int S, hipStream_t s);
// act[M, I] = GLU of the plain [gate | up] partials ws[S, M, 2I] (decode_fused.hip)
void launch_splitk_glu(void* act, long act_stride, const float* ws, int S, int M, int I, bool gelu, hipStream_t s,
                       void* act16 = nullptr);
// bias (bf16 [N]) and per-head q/k RMSNorm (fp32 weights [D], mode 0, D/16 a power of two)
// optional: nullptr skips them (Qwen2 / Qwen3 families)
void launch_splitk_rope_cache(void* qkv, long qkv_stride, const float* ws, int S, const long* positions,
                              const long* slots, const float* cos_sin, void* k_cache, void* v_cache, int T, int nq,
                              int nkv, int D, int block_size, int mode, hipStream_t s, const void* bias = nullptr,
                              const float* qw = nullptr, const float* kw = nullptr, float eps = 1e-6f,
                              bool kv_f8 = false);
void launch_pack_decode_weight(void* out, const void* w, int N, int K, bool glu, hipStream_t s, int batch = 1);
}  // namespace hipserve

namespace hipserve {
// moe.hip — tile in {16, 32, 64}
void launch_moe_topk_softmax(const void* logits, bool logits_f32, float* w, int* ids, int T, int E, int k,
                             bool renorm, hipStream_t s, int splits = 0);
void launch_moe_align(const int* ids, int npairs, int E, int tile, int* slots, int slots_cap, int* tile_expert,
                      int tiles_cap, int* num_tiles, int* pair_slot, int* group_end, hipStream_t s,
                      int* hist = nullptr);
// blocks of the multi-workgroup moe_align for npairs (1: the single-workgroup kernel);
// it needs hist = int32 [blocks * 128] scratch
int moe_align_blocks(int npairs);
// xs[slot, H] = x[slots[slot] / k] (zeros for padding slots): grouped-GEMM input rows
void launch_moe_gather(void* out, const void* x, long x_stride, const int* slots, int nslots, int k, int H,
                       hipStream_t s);
void launch_moe_gemm(void* out, long out_stride, const void* x, long x_stride, const void* w, const int* slots,
                     const int* tile_expert, int tiles_cap, int tile, int gather_k, int N, int K, hipStream_t s);
void launch_moe_combine(void* out, const void* y, const float* w, const int* pair_slot, int T, int k, int H,
                        hipStream_t s);
// out[t] = sum_j w[t, j] * bf16(sum_s ws[s, pair_slot[t*k + j], :]) — split-K partials of the w2 GEMM
void launch_moe_combine_partial(void* out, const float* ws, long slab, int S, const float* w, const int* pair_slot,
                                int T, int k, int H, hipStream_t s);
// combine (bf16 y [slots, H] when S == 0, fp32 partials [S, slots, H] else) + residual add +
// RMSNorm (norm_w bf16 or fp32 [H]) -> out [T, H], residual [T, H] in place
void launch_moe_combine_add_rmsnorm(void* out, void* residual, const void* y, long slab, int S, const float* w,
                                    const int* pair_slot, int T, int k, int H, const void* norm_w, bool norm_f32,
                                    float eps, hipStream_t s);
// decode_gemm.hip: expert GEMM on moe_align tiles (see there)
bool launch_moe_decode_gemm(void* out, long out_stride, float* ws, const void* x, long x_stride, const void* w,
                            long w_estride, const int* slots, const int* tile_expert, int tiles_cap, int tile,
                            int gather_k, int N, int K, int S, bool packed, bool glu, hipStream_t s);
}  // namespace hipserve

namespace hipserve {

// stage_copy.hip — up to 8 word-aligned copies in one dispatch; host_mask bit 2i / 2i+1
// marks copy i's src / dst as pinned host memory (device-mapped pointers).
constexpr int kMaxStageCopies = 8;
struct StageCopyArgs {
  void* dst[kMaxStageCopies];
  const void* src[kMaxStageCopies];
  long words[kMaxStageCopies];
  int n;
  unsigned int host_mask;
};
void launch_stage_copy(const StageCopyArgs& a, hipStream_t s);

}  // namespace hipserve

namespace hipserve {
// vision.hip — Qwen3-VL vision tower. residual != nullptr: residual = bf16(residual + x),
// out = LayerNorm(residual) (else LayerNorm(x)); bf16 weight / bias [C], C % 8 == 0.
void launch_layernorm(void* out, void* residual, const void* x, const void* w, const void* b, int rows, int C,
                      float eps, hipStream_t s);
void launch_gelu(void* x, long n, bool tanh_approx, hipStream_t s);
// qkv [T, 3 nh D]: 2D RoPE of q, k in place (fp32 table [T, D]), then bidirectional attention
// within each segment [cu[i], cu[i+1]) -> out [T, nh D]; tiles [ntiles, 2] = (segment, first row)
// in steps of 128 rows.
void launch_vision_attention(void* out, void* qkv, const float* cos_sin, const int* cu, const int* tiles,
                             int ntiles, int T, int nh, int D, float scale, hipStream_t s);
}  // namespace hipserve
