// torch.ops.hipserve.* — operator registration for the gfx950 kernel library.
//
// All ops write into caller-provided outputs (no allocation, no host sync), so
// the decode step can be captured into a hipGraph by torch.cuda.CUDAGraph.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "hipserve/kernels.h"

namespace {

hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

#define CHECK_DEV(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_ROWMAJOR(x) TORCH_CHECK((x).stride(-1) == 1, #x " must have unit inner stride")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")

static void e4m3_out_args(const c10::optional<at::Tensor>& out8, const c10::optional<at::Tensor>& xs8,
                          const at::Tensor& out, void** o8, float** x8, const char* who);

void rmsnorm(at::Tensor& out, const at::Tensor& x, const at::Tensor& weight, double eps,
             const c10::optional<at::Tensor>& out8, const c10::optional<at::Tensor>& xs8) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2, "rmsnorm expects 2-D [rows, hidden]");
  const int hidden = x.size(1);
  TORCH_CHECK(hidden % 8 == 0 && hidden <= 16384, "hidden must be a multiple of 8, <= 16384");
  TORCH_CHECK(weight.numel() == hidden && weight.is_contiguous());
  TORCH_CHECK(weight.scalar_type() == at::kBFloat16 || weight.scalar_type() == at::kFloat);
  void* o8;
  float* x8;
  e4m3_out_args(out8, xs8, out, &o8, &x8, "rmsnorm");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_rmsnorm(out.data_ptr(), nullptr, x.data_ptr(), weight.data_ptr(),
                           weight.scalar_type() == at::kFloat, x.size(0), hidden,
                           x.stride(0), out.stride(0), (float)eps, cur_stream(), o8, x8);
}

void fused_add_rmsnorm(at::Tensor& out, const at::Tensor& x, at::Tensor& residual,
                       const at::Tensor& weight, double eps, const c10::optional<at::Tensor>& out8,
                       const c10::optional<at::Tensor>& xs8) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_BF16(residual);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out); CHECK_CONTIG(residual);
  TORCH_CHECK(x.dim() == 2 && residual.sizes() == x.sizes());
  const int hidden = x.size(1);
  TORCH_CHECK(hidden % 8 == 0 && hidden <= 16384);
  TORCH_CHECK(weight.numel() == hidden && weight.is_contiguous());
  void* o8;
  float* x8;
  e4m3_out_args(out8, xs8, out, &o8, &x8, "fused_add_rmsnorm");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_rmsnorm(out.data_ptr(), residual.data_ptr(), x.data_ptr(), weight.data_ptr(),
                           weight.scalar_type() == at::kFloat, x.size(0), hidden,
                           x.stride(0), out.stride(0), (float)eps, cur_stream(), o8, x8);
}

// residual = bf16(table[id] * scale), out = RMSNorm(residual) * weight per row; id =
// ids[row], or tok[src[row]] where src[row] >= 0 (device-side decode lookahead ids);
// out8 / xs8 (optional): out also as per-token e4m3 + row scale (= act_quant_fp8 of out)
void embed_rmsnorm(at::Tensor& out, at::Tensor& residual, const at::Tensor& table, const at::Tensor& ids,
                   const c10::optional<at::Tensor>& src, const c10::optional<at::Tensor>& tok,
                   const at::Tensor& weight, double eps, double scale, const c10::optional<at::Tensor>& out8,
                   const c10::optional<at::Tensor>& xs8) {
  CHECK_DEV(table); CHECK_BF16(table); CHECK_BF16(out); CHECK_BF16(residual);
  CHECK_CONTIG(table); CHECK_CONTIG(out); CHECK_CONTIG(residual); CHECK_CONTIG(ids);
  TORCH_CHECK(table.dim() == 2 && out.dim() == 2 && residual.sizes() == out.sizes());
  const int hidden = table.size(1), rows = ids.numel();
  TORCH_CHECK(out.size(0) == rows && out.size(1) == hidden);
  TORCH_CHECK(hidden % 8 == 0 && hidden <= 16384);
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_cuda());
  TORCH_CHECK(src.has_value() == tok.has_value(), "src and tok come together");
  if (src.has_value()) {
    TORCH_CHECK(src->scalar_type() == at::kLong && tok->scalar_type() == at::kLong && src->numel() == rows);
    TORCH_CHECK(src->is_contiguous() && tok->is_contiguous() && src->is_cuda() && tok->is_cuda());
  }
  TORCH_CHECK(weight.numel() == hidden && weight.is_contiguous());
  TORCH_CHECK(weight.scalar_type() == at::kBFloat16 || weight.scalar_type() == at::kFloat);
  void* o8;
  float* x8;
  e4m3_out_args(out8, xs8, out, &o8, &x8, "embed_rmsnorm");
  c10::hip::HIPGuardMasqueradingAsCUDA g(table.device());
  hipserve::launch_embed_rmsnorm(out.data_ptr(), residual.data_ptr(), table.data_ptr(), ids.data_ptr<long>(),
                                 src.has_value() ? src->data_ptr<long>() : nullptr,
                                 tok.has_value() ? tok->data_ptr<long>() : nullptr, weight.data_ptr(),
                                 weight.scalar_type() == at::kFloat, rows, hidden, (float)eps, cur_stream(),
                                 (float)scale, o8, x8);
}

void silu_and_mul(at::Tensor& out, const at::Tensor& x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == 2 * out.size(1) && x.size(0) == out.size(0));
  TORCH_CHECK(out.size(1) % 8 == 0);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_silu_and_mul(out.data_ptr(), x.data_ptr(), x.size(0), out.size(1),
                                x.stride(0), out.stride(0), cur_stream());
}

// paged KV cache element type: bf16, or float8_e4m3fn (--kv-cache-dtype fp8: e4m3 with a
// per-tensor scale of 1, written rounded / read widened by the kernels); K and V alike
static bool kv_is_f8(const at::Tensor& k, const at::Tensor& v) {
  const auto t = k.scalar_type();
  TORCH_CHECK((t == at::kBFloat16 || t == at::kFloat8_e4m3fn) && v.scalar_type() == t,
              "KV cache: bf16 or float8_e4m3fn, K and V alike");
  return t == at::kFloat8_e4m3fn;
}

void rope_cache(at::Tensor& qkv, const at::Tensor& positions, const at::Tensor& slots,
                const at::Tensor& cos_sin, at::Tensor& k_cache, at::Tensor& v_cache,
                int64_t nq, int64_t nkv, int64_t head_dim, int64_t mode) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_ROWMAJOR(qkv);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= (nq + 2 * nkv) * head_dim);
  TORCH_CHECK(positions.scalar_type() == at::kLong && slots.scalar_type() == at::kLong);
  TORCH_CHECK(positions.numel() >= qkv.size(0) && slots.numel() >= qkv.size(0));
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == head_dim && cos_sin.is_contiguous());
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(3) == head_dim, "k_cache [blocks, nkv, bs, D]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == nkv && v_cache.size(2) == head_dim, "v_cache [blocks, nkv, D, bs]");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous());
  TORCH_CHECK(head_dim % 16 == 0 && (mode == 0 || mode == 1));
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  hipserve::launch_rope_cache(qkv.data_ptr(), qkv.stride(0), positions.data_ptr<int64_t>(),
                              slots.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                              k_cache.data_ptr(), v_cache.data_ptr(), qkv.size(0), nq, nkv,
                              head_dim, k_cache.size(2), mode, cur_stream(), kv_is_f8(k_cache, v_cache));
}

// the f16 pair-order copy of a bf16 [B, >= nq D] output (same shape and row stride) or null
static void* out16_ptr(const c10::optional<at::Tensor>& out16, const at::Tensor& out) {
  if (!out16.has_value() || !out16->defined()) return nullptr;
  TORCH_CHECK(out16->scalar_type() == at::kHalf && out16->device() == out.device() && out16->size(0) == out.size(0) &&
                  out16->size(1) == out.size(1) && out16->stride(0) == out.stride(0) && out16->stride(1) == 1,
              "out16: f16 with out's shape and row stride");
  return out16->data_ptr();
}

void paged_decode(at::Tensor& out, const at::Tensor& q, const at::Tensor& k_cache,
                  const at::Tensor& v_cache, const at::Tensor& block_tables,
                  const at::Tensor& context_lens, at::Tensor& tmp_out, at::Tensor& tmp_ml,
                  int64_t nq, int64_t nkv, int64_t part_size, double scale, int64_t window,
                  const c10::optional<at::Tensor>& out16) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_ROWMAJOR(q); CHECK_ROWMAJOR(out);
  const int D = k_cache.size(3), bs = k_cache.size(2);
  TORCH_CHECK(D == 64 || D == 96 || D == 128, "paged_decode: head_dim 64/96/128");
  TORCH_CHECK(window >= 0, "paged_decode: window >= 0");
  TORCH_CHECK(nq % nkv == 0 && nq / nkv <= 16, "paged_decode: GQA group <= 16");
  TORCH_CHECK(bs % 16 == 0 && (bs & (bs - 1)) == 0, "paged_decode: block_size a power of two >= 16");
  TORCH_CHECK(part_size % 128 == 0 && part_size / bs < 255);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && context_lens.scalar_type() == at::kInt);
  TORCH_CHECK(block_tables.stride(1) == 1);
  const int B = q.size(0);
  const int max_parts = tmp_ml.size(2);
  TORCH_CHECK(tmp_out.is_contiguous() && tmp_ml.is_contiguous());
  TORCH_CHECK(tmp_ml.dim() == 4 && tmp_ml.size(0) >= B && tmp_ml.size(1) == nq && tmp_ml.size(3) == 2);
  TORCH_CHECK(tmp_out.dim() == 4 && tmp_out.size(2) == max_parts && tmp_out.size(3) == D);
  TORCH_CHECK((long)max_parts * part_size >= (long)block_tables.size(1) * bs,
              "workspace partitions must cover block_tables capacity");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  hipserve::launch_paged_decode(out.data_ptr(), out.stride(0), q.data_ptr(), q.stride(0),
                                k_cache.data_ptr(), v_cache.data_ptr(),
                                block_tables.data_ptr<int>(), block_tables.stride(0),
                                context_lens.data_ptr<int>(), tmp_out.data_ptr<float>(),
                                tmp_ml.data_ptr<float>(), B, nq, nkv, D, bs, part_size,
                                max_parts, (float)scale, (int)window, cur_stream(), out16_ptr(out16, out),
                                kv_is_f8(k_cache, v_cache));
}

void paged_decode_qkv(at::Tensor& out, const at::Tensor& ws, int64_t splits, const at::Tensor& positions,
                      const at::Tensor& slots, const at::Tensor& cos_sin, at::Tensor& k_cache, at::Tensor& v_cache,
                      const at::Tensor& block_tables, const at::Tensor& context_lens, at::Tensor& tmp_out,
                      at::Tensor& tmp_ml, int64_t nq, int64_t nkv, int64_t part_size, double scale, int64_t window,
                      int64_t mode, const c10::optional<at::Tensor>& out16, const c10::optional<at::Tensor>& q_w,
                      const c10::optional<at::Tensor>& k_w, double eps) {
  CHECK_DEV(ws); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(!kv_is_f8(k_cache, v_cache), "paged_decode_qkv: bf16 KV cache only");
  const int D = k_cache.size(3), bs = k_cache.size(2);
  TORCH_CHECK(D == 64 || D == 128, "paged_decode_qkv: head_dim 64/128");
  const float *qwp = nullptr, *kwp = nullptr;
  if (q_w.has_value()) {  // per-head q / k RMSNorm before RoPE (Qwen3)
    TORCH_CHECK(k_w.has_value() && q_w->scalar_type() == at::kFloat && k_w->scalar_type() == at::kFloat &&
                q_w->numel() == D && k_w->numel() == D && q_w->is_contiguous() && k_w->is_contiguous(),
                "paged_decode_qkv: fp32 q/k norm weights [head_dim]");
    TORCH_CHECK(mode == 0, "paged_decode_qkv: q/k norm needs rotate-half RoPE (mode 0)");
    CHECK_DEV(*q_w); CHECK_DEV(*k_w);
    qwp = q_w->data_ptr<float>();
    kwp = k_w->data_ptr<float>();
  }
  TORCH_CHECK(window >= 0 && (mode == 0 || mode == 1));
  TORCH_CHECK(nq % nkv == 0 && nq / nkv <= 16, "paged_decode_qkv: GQA group <= 16");
  TORCH_CHECK(bs % 16 == 0 && (bs & (bs - 1)) == 0 && part_size % 128 == 0 && part_size / bs < 255);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && context_lens.scalar_type() == at::kInt);
  TORCH_CHECK(block_tables.stride(1) == 1);
  const int B = out.size(0);
  const long N = (nq + 2 * nkv) * D;
  TORCH_CHECK(out.size(1) >= nq * D);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * B * N);
  TORCH_CHECK(positions.scalar_type() == at::kLong && slots.scalar_type() == at::kLong);
  TORCH_CHECK(positions.numel() >= B && slots.numel() >= B);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == D && cos_sin.is_contiguous());
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && v_cache.dim() == 4 && v_cache.size(2) == D);
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous());
  const int max_parts = tmp_ml.size(2);
  TORCH_CHECK(tmp_out.is_contiguous() && tmp_ml.is_contiguous());
  TORCH_CHECK(tmp_ml.dim() == 4 && tmp_ml.size(0) >= B && tmp_ml.size(1) == nq && tmp_ml.size(3) == 2);
  TORCH_CHECK(tmp_out.dim() == 4 && tmp_out.size(2) == max_parts && tmp_out.size(3) == D);
  TORCH_CHECK((long)max_parts * part_size >= (long)block_tables.size(1) * bs,
              "workspace partitions must cover block_tables capacity");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
  hipserve::launch_paged_decode_qkv(out.data_ptr(), out.stride(0), ws.data_ptr<float>(), splits, N,
                                    positions.data_ptr<int64_t>(), slots.data_ptr<int64_t>(), cos_sin.data_ptr<float>(),
                                    mode, k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                    block_tables.stride(0), context_lens.data_ptr<int>(), tmp_out.data_ptr<float>(),
                                    tmp_ml.data_ptr<float>(), B, nq, nkv, D, bs, part_size, max_parts, (float)scale,
                                    (int)window, cur_stream(), out16_ptr(out16, out), qwp, kwp, (float)eps);
}

void prefill_attention(at::Tensor& out, const at::Tensor& q, const at::Tensor& k_cache,
                       const at::Tensor& v_cache, const at::Tensor& block_tables,
                       const at::Tensor& cu_q, const at::Tensor& ctx_lens,
                       const at::Tensor& tiles, int64_t nq, int64_t nkv, double scale, int64_t window) {
  CHECK_DEV(q); CHECK_BF16(q); CHECK_BF16(out); CHECK_ROWMAJOR(q); CHECK_ROWMAJOR(out);
  const int D = k_cache.size(3), bs = k_cache.size(2);
  TORCH_CHECK(D == 64 || D == 96 || D == 128, "prefill_attention: head_dim 64/96/128");
  TORCH_CHECK(window >= 0, "prefill_attention: window >= 0");
  TORCH_CHECK(bs % 16 == 0 && nq % nkv == 0);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && cu_q.scalar_type() == at::kInt &&
              ctx_lens.scalar_type() == at::kInt && tiles.scalar_type() == at::kInt);
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 2 && tiles.is_contiguous());
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  hipserve::launch_prefill_attention(out.data_ptr(), out.stride(0), q.data_ptr(), q.stride(0),
                                     k_cache.data_ptr(), v_cache.data_ptr(),
                                     block_tables.data_ptr<int>(), block_tables.stride(0),
                                     cu_q.data_ptr<int>(), ctx_lens.data_ptr<int>(),
                                     tiles.data_ptr<int>(), tiles.size(0), nq, nkv, D, bs,
                                     (float)scale, (int)window, cur_stream(), kv_is_f8(k_cache, v_cache));
}

// Per-head RMSNorm of q and k inside the merged qkv rows, in place (Qwen3 / Gemma-3).
void qk_rmsnorm(at::Tensor& qkv, const at::Tensor& q_w, const at::Tensor& k_w, int64_t nq, int64_t nkv,
                int64_t head_dim, double eps) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_ROWMAJOR(qkv);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= (nq + nkv) * head_dim && head_dim <= 256);
  TORCH_CHECK(q_w.scalar_type() == at::kFloat && k_w.scalar_type() == at::kFloat && q_w.is_contiguous() &&
              k_w.is_contiguous() && q_w.numel() == head_dim && k_w.numel() == head_dim,
              "qk_rmsnorm: fp32 [head_dim] weights");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  hipserve::launch_qk_rmsnorm(qkv.data_ptr(), qkv.stride(0), q_w.data_ptr<float>(), k_w.data_ptr<float>(),
                              qkv.size(0), nq, nkv, head_dim, (float)eps, cur_stream());
}

void gelu_and_mul(at::Tensor& out, const at::Tensor& x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.size(1) == 2 * out.size(1) && x.size(0) == out.size(0));
  TORCH_CHECK(out.size(1) % 8 == 0);
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_gelu_and_mul(out.data_ptr(), x.data_ptr(), x.size(0), out.size(1), x.stride(0), out.stride(0),
                                cur_stream());
}

void sample(at::Tensor& out_tok, at::Tensor& out_lp, const at::Tensor& logits,
            const at::Tensor& temperature, const at::Tensor& top_k, const at::Tensor& top_p,
            const at::Tensor& seeds, const at::Tensor& steps, bool two_rounds) {
  CHECK_DEV(logits); CHECK_ROWMAJOR(logits);
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat);
  TORCH_CHECK(out_tok.scalar_type() == at::kLong && out_lp.scalar_type() == at::kFloat);
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat &&
              top_k.scalar_type() == at::kInt && seeds.scalar_type() == at::kLong &&
              steps.scalar_type() == at::kLong);
  const int rows = logits.size(0);
  TORCH_CHECK(out_tok.numel() >= rows && temperature.numel() >= rows && top_k.numel() >= rows &&
              top_p.numel() >= rows && seeds.numel() >= rows && steps.numel() >= rows);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  // multi-CU sampler workspace (caching allocator: graph-capturable)
  const size_t wsn = hipserve::sample_workspace_floats(rows, logits.size(1));
  at::Tensor ws;
  if (wsn) ws = at::empty({(long)wsn}, logits.options().dtype(at::kFloat));
  hipserve::launch_sample(out_tok.data_ptr<int64_t>(), out_lp.numel() ? out_lp.data_ptr<float>() : nullptr,
                          logits.data_ptr(), logits.scalar_type() == at::kBFloat16,
                          logits.stride(0), rows, logits.size(1), temperature.data_ptr<float>(),
                          top_k.data_ptr<int>(), top_p.data_ptr<float>(), seeds.data_ptr<int64_t>(),
                          steps.data_ptr<int64_t>(), wsn ? ws.data_ptr<float>() : nullptr, cur_stream(),
                          two_rounds);
}

void gguf_gemm(at::Tensor& out, const at::Tensor& x, const at::Tensor& q, const at::Tensor& d,
               const at::Tensor& mn, int64_t qtype, int64_t row_bytes, int64_t N, int64_t K,
               at::Tensor& ws, int64_t splits) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(q.scalar_type() == at::kByte && q.is_contiguous());
  TORCH_CHECK(K % 256 == 0, "gguf_gemm: K must be a multiple of 256");
  TORCH_CHECK(x.size(1) >= K && out.size(1) >= N && out.size(0) == x.size(0));
  const int M = x.size(0);
  TORCH_CHECK(M <= 64, "gguf_gemm handles M <= 64 (use gguf_dequant + GEMM above)");
  TORCH_CHECK(x.stride(0) % 8 == 0, "x rows must be 16-byte aligned");
  TORCH_CHECK(qtype >= 0 && qtype <= 6);
  if (qtype <= 2) TORCH_CHECK(d.numel() >= N * (K / 32), "missing SoA scales");
  if (qtype == 1) TORCH_CHECK(mn.numel() >= N * (K / 32), "missing SoA mins");
  if (splits > 1) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= (long)splits * M * N,
                "gguf_gemm: split-K needs an fp32 workspace of splits*M*N (one slab per K slice)");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_gguf_gemm(out.data_ptr(), splits > 1 ? ws.data_ptr<float>() : nullptr, x.data_ptr(),
                             x.stride(0), out.stride(0), q.data_ptr(), d.numel() ? d.data_ptr() : nullptr,
                             mn.numel() ? mn.data_ptr() : nullptr, qtype, row_bytes, M, N, K,
                             splits, cur_stream());
}

// parts in the tiled layout (one uint8 tensor [N/16, K/256, chunk] each), their
// formats / rows / output columns. ws.numel() > 0: fp32 partials [S_actual, M, Ntot]
// (returned S_actual = ceil(nsb / ceil(nsb / S))); else bf16 out [M, >= Ntot], S == 1.
// kernel formats with a per-row fp32 output scale: FP8, FP8B, INT8C (gguf_tiles.h row_scaled)
static bool row_scaled_qt(int64_t qt) { return qt == 6 || qt == 7 || qt == 9; }

int64_t gguf_gemm_parts(at::Tensor& out, at::Tensor& ws, const at::Tensor& x, const std::vector<at::Tensor>& qs,
                        const std::vector<at::Tensor>& rss, const std::vector<int64_t>& qtypes, const std::vector<int64_t>& rows,
                        const std::vector<int64_t>& cols, int64_t Ntot, int64_t K, int64_t splits,
                        const c10::optional<at::Tensor>& x16) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x);
  const int np = qs.size();
  TORCH_CHECK(np >= 1 && np <= 4 && (int)qtypes.size() == np && (int)rss.size() == np && (int)rows.size() == np && (int)cols.size() == np,
              "gguf_gemm_parts: 1-4 parts");
  TORCH_CHECK(K % 256 == 0 && x.size(1) >= K && splits >= 1);
  const int M = x.size(0);
  TORCH_CHECK(M >= 1, "gguf_gemm_parts: M >= 1 (M > 64 sweeps 64-row tiles)");
  TORCH_CHECK(x.stride(0) % 8 == 0, "x rows must be 16-byte aligned");
  const int nsb = K / 256;
  const int per = (nsb + splits - 1) / splits;
  const int S = (nsb + per - 1) / per;
  hipserve::GgufPart P[4];
  for (int i = 0; i < np; ++i) {
    TORCH_CHECK(qtypes[i] >= 0 && qtypes[i] <= 9, "gguf_gemm_parts: kernel qtype 0-9");
    const bool fp8 = row_scaled_qt(qtypes[i]);
    TORCH_CHECK(!fp8 || (rss[i].scalar_type() == at::kFloat && rss[i].is_contiguous() && rss[i].numel() == rows[i] &&
                         rss[i].device() == x.device()), "FP8 / INT8C parts need an fp32 row scale per row");
    TORCH_CHECK(qs[i].scalar_type() == at::kByte && qs[i].is_contiguous() && qs[i].device() == x.device());
    TORCH_CHECK(cols[i] % 4 == 0 && rows[i] % 16 == 0 && rows[i] > 0 && cols[i] + rows[i] <= Ntot,
                "parts: 16-row multiples at 4-aligned columns inside Ntot");
    TORCH_CHECK(qs[i].numel() == rows[i] / 16 * nsb * hipserve::gguf_tiled_chunk_bytes(qtypes[i]),
                "part q is not a tiled [N/16, K/256, chunk] tensor of its format");
    P[i] = hipserve::GgufPart{qs[i].data_ptr(), fp8 ? rss[i].data_ptr<float>() : nullptr, (int)qtypes[i],
                              (int)rows[i], (int)cols[i]};
  }
  float* wp = nullptr;
  if (ws.numel() > 0) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= (long)S * M * Ntot,
                "gguf_gemm_parts: ws must hold S * M * Ntot fp32");
    TORCH_CHECK(ws.device() == x.device());
    wp = ws.data_ptr<float>();
  } else {
    TORCH_CHECK(S == 1, "gguf_gemm_parts: split-K needs a partial workspace");
    CHECK_BF16(out); CHECK_ROWMAJOR(out);
    TORCH_CHECK(out.size(0) == M && out.size(1) >= Ntot && out.stride(0) % 4 == 0 && out.device() == x.device());
  }
  const void* x16p = nullptr;
  if (x16.has_value() && x16->defined()) {  // f16 pair-order copy of x from the producer (M <= 64)
    TORCH_CHECK(x16->scalar_type() == at::kHalf && x16->size(0) == M && x16->size(1) >= K &&
                    x16->stride(0) == x.stride(0) && x16->stride(1) == 1 && x16->device() == x.device(),
                "gguf_gemm_parts: x16 f16 [M, >= K] with x's row stride");
    x16p = x16->data_ptr();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_gguf_gemm_parts(wp ? nullptr : out.data_ptr(), wp ? 0 : out.stride(0), wp, x.data_ptr(),
                                   x.stride(0), P, np, M, Ntot, K, splits, cur_stream(), x16p);
  return S;
}

// x [M, >= K] bf16 -> x16 [M, K] f16 in the GGUF kernels' pair order, each row scaled by
// 1 / rsc[m] (a power of two keeping it in the f16 range): the prefill GEMM's operand
void x_f16_pairs(at::Tensor& x16, at::Tensor& rsc, const at::Tensor& x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x);
  const int M = x.size(0), K = x16.size(1);
  TORCH_CHECK(x16.scalar_type() == at::kHalf && x16.is_contiguous() && x16.size(0) == M && K % 8 == 0 &&
                  x.size(1) >= K && x.stride(0) % 8 == 0 && x16.device() == x.device(),
              "x_f16_pairs: x16 f16 [M, K] contiguous, K % 8, 16-byte x rows");
  TORCH_CHECK(rsc.scalar_type() == at::kFloat && rsc.is_contiguous() && rsc.numel() >= M && rsc.device() == x.device(),
              "x_f16_pairs: rsc fp32 [M]");
  if (M == 0) return;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_x_f16_pairs(x16.data_ptr(), rsc.data_ptr<float>(), x.data_ptr(), x.stride(0), M, K, cur_stream());
}

// prefill GEMM on the tiled GGUF parts (gguf_mfma.hip qpf_kernel) over x16 / rsc from
// x_f16_pairs: epi 0 store at each part's column, 1 residual add (out += x . W^T, in
// place), 2 / 3 SiLU / GELU GLU of parts 0 (gate) and 1 (up) into out[M, rows]. Returns
// false when the kernel does not take it.
bool gguf_prefill(at::Tensor& out, const at::Tensor& x16, const at::Tensor& rsc, const std::vector<at::Tensor>& qs,
                  const std::vector<int64_t>& qtypes, const std::vector<int64_t>& rows, const std::vector<int64_t>& cols,
                  int64_t K, int64_t epi) {
  CHECK_DEV(x16); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  const int np = qs.size();
  TORCH_CHECK(np >= 1 && np <= 4 && (int)qtypes.size() == np && (int)rows.size() == np && (int)cols.size() == np,
              "gguf_prefill: 1-4 parts");
  TORCH_CHECK(x16.scalar_type() == at::kHalf && x16.is_contiguous() && x16.dim() == 2 && x16.size(1) == K &&
                  K % 256 == 0, "gguf_prefill: x16 f16 [M, K] contiguous (x_f16_pairs), K % 256");
  const int M = x16.size(0);
  TORCH_CHECK(rsc.scalar_type() == at::kFloat && rsc.is_contiguous() && rsc.numel() >= M && rsc.device() == x16.device(),
              "gguf_prefill: rsc fp32 [M]");
  const bool glu = epi == 2 || epi == 3;
  TORCH_CHECK(out.size(0) == M && out.stride(0) % 4 == 0 && out.device() == x16.device(), "gguf_prefill: out rows");
  const int nsb = K / 256;
  hipserve::GgufPart P[4];
  long ncols = 0;
  for (int i = 0; i < np; ++i) {
    TORCH_CHECK(qs[i].scalar_type() == at::kByte && qs[i].is_contiguous() && qs[i].device() == x16.device());
    TORCH_CHECK(rows[i] % 16 == 0 && rows[i] > 0 && cols[i] % 4 == 0, "gguf_prefill: 16-row parts, 4-aligned columns");
    TORCH_CHECK(qtypes[i] >= 0 && qtypes[i] <= 8 &&
                    qs[i].numel() == rows[i] / 16 * nsb * hipserve::gguf_tiled_chunk_bytes(qtypes[i]),
                "gguf_prefill: part q is not a tiled [N/16, K/256, chunk] tensor of its format");
    P[i] = hipserve::GgufPart{qs[i].data_ptr(), nullptr, (int)qtypes[i], (int)rows[i], (int)cols[i]};
    ncols = std::max(ncols, (long)(cols[i] + rows[i]));
  }
  TORCH_CHECK(out.size(1) >= (glu ? rows[0] : ncols), "gguf_prefill: out narrower than the parts");
  if (M == 0) return true;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x16.device());
  return hipserve::launch_gguf_prefill((int)epi, out.data_ptr(), out.stride(0), x16.data_ptr(), rsc.data_ptr<float>(),
                                       P, np, M, (int)K, cur_stream());
}

int64_t qmoe_gemm(at::Tensor& out, at::Tensor& ws, const at::Tensor& x, const at::Tensor& q, const at::Tensor& rs,
                  int64_t qtype, int64_t N, int64_t K, const at::Tensor& slots, const at::Tensor& tile_expert,
                  int64_t tile, int64_t gather_k, int64_t splits, bool kmajor, int64_t glu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x);
  TORCH_CHECK(qtype == 6 || qtype == 8 || qtype == 9, "qmoe_gemm: expert formats FP8 (per-row scale), INT8, INT8C");
  TORCH_CHECK(tile == 16 || tile == 32 || tile == 64, "qmoe_gemm: tile 16/32/64");
  TORCH_CHECK(N % 16 == 0 && K % 256 == 0 && x.size(1) >= K && x.stride(0) % 8 == 0, "qmoe_gemm: shapes");
  TORCH_CHECK(slots.scalar_type() == at::kInt && tile_expert.scalar_type() == at::kInt && slots.is_contiguous() &&
              tile_expert.is_contiguous() && slots.numel() == tile_expert.numel() * tile,
              "qmoe_gemm: int32 slots [tiles * tile] and tile_expert [tiles]");
  TORCH_CHECK(q.scalar_type() == at::kByte && q.is_contiguous() && q.dim() == 2 && q.device() == x.device(),
              "qmoe_gemm: q uint8 [E, expert bytes]");
  const long per_e = N / 16 * (K / 256) * hipserve::gguf_tiled_chunk_bytes(qtype);
  TORCH_CHECK(q.size(1) == per_e, "qmoe_gemm: q rows are not tiled [N/16, K/256, chunk] experts");
  const bool fp8 = qtype == 6 || qtype == 9;
  TORCH_CHECK(!fp8 || (rs.scalar_type() == at::kFloat && rs.is_contiguous() && rs.dim() == 2 &&
                       rs.size(0) == q.size(0) && rs.size(1) == N), "qmoe_gemm: FP8 / INT8C experts need rs [E, N] fp32");
  TORCH_CHECK(gather_k > 0 || x.size(0) >= slots.numel(), "qmoe_gemm: slot-indexed x needs a row per slot");
  const int nsb = K / 256;
  const int per = (nsb + splits - 1) / splits;
  const int S = (nsb + per - 1) / per;
  const long nslots = slots.numel();
  float* wp = nullptr;
  if (ws.numel() > 0) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= S * nslots * N &&
                ws.device() == x.device(), "qmoe_gemm: ws must hold S * slots * N fp32");
    wp = ws.data_ptr<float>();
  } else {
    TORCH_CHECK(S == 1, "qmoe_gemm: split-K needs a partial workspace");
    CHECK_BF16(out); CHECK_ROWMAJOR(out);
    TORCH_CHECK(out.size(0) == nslots && out.size(1) >= (glu ? N / 2 : N) && out.stride(0) % 4 == 0 &&
                out.device() == x.device());
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_qmoe_gemm(wp ? nullptr : out.data_ptr(), wp ? 0 : out.stride(0), wp, x.data_ptr(),
                                         x.stride(0), q.data_ptr(), fp8 ? rs.data_ptr<float>() : nullptr, qtype,
                                         per_e, fp8 ? N : 0, slots.data_ptr<int>(), tile_expert.data_ptr<int>(),
                                         tile_expert.numel(), tile, gather_k, N, K, splits, cur_stream(), kmajor,
                                         (int)glu),
              "qmoe_gemm: unsupported configuration");
  return S;
}

// pack 0: out row-major [N, K]; 1 / 2: the stacked matrices of `nrows` rows each (N = E nrows)
// in the pack_decode_weight layout (2: gate/up-interleaved), E copies back to back
void gguf_dequant_tiled(at::Tensor& out, const at::Tensor& q, const at::Tensor& rs, int64_t qtype, int64_t N,
                        int64_t K, int64_t pack, int64_t nrows, bool kmajor) {
  CHECK_DEV(q); CHECK_BF16(out);
  TORCH_CHECK(out.is_contiguous() && N % 16 == 0 && K % 256 == 0);
  TORCH_CHECK(pack >= 0 && pack <= 2, "gguf_dequant_tiled: pack 0, 1 or 2");
  if (pack == 0) {
    TORCH_CHECK(out.numel() >= N * K, "gguf_dequant_tiled: out [N, K]");
  } else {
    TORCH_CHECK(nrows > 0 && nrows % 16 == 0 && N % nrows == 0 && (pack == 1 || nrows % 128 == 0),
                "gguf_dequant_tiled: packed matrices of nrows rows (glu: nrows % 128 == 0)");
    TORCH_CHECK(out.numel() >= N / nrows * ((nrows + 127) / 128 * 128) * K, "gguf_dequant_tiled: packed out size");
  }
  TORCH_CHECK(qtype >= 0 && qtype <= 9 && q.scalar_type() == at::kByte && q.is_contiguous());
  TORCH_CHECK(q.numel() == N / 16 * (K / 256) * hipserve::gguf_tiled_chunk_bytes(qtype), "not a tiled tensor");
  TORCH_CHECK(!kmajor || nrows <= 0 || (nrows % 16 == 0 && N % nrows == 0), "gguf_dequant_tiled: k-major matrices of nrows rows");
  const bool fp8 = row_scaled_qt(qtype);
  TORCH_CHECK(!fp8 || (rs.scalar_type() == at::kFloat && rs.numel() == N), "FP8 / INT8C need an fp32 row scale");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  hipserve::launch_gguf_dequant_tiled(out.data_ptr(), q.data_ptr(), fp8 ? rs.data_ptr<float>() : nullptr,
                                      qtype, N, K, cur_stream(), (int)pack, (int)nrows, kmajor);
}

// per-channel FP8 tiled part q [N/16, K/256, 4096] -> out: row-major [N, K] e4m3 bytes
void fp8_untile(at::Tensor& out, const at::Tensor& q, int64_t N, int64_t K) {
  CHECK_DEV(q); CHECK_DEV(out);
  TORCH_CHECK(N % 16 == 0 && K % 256 == 0 && q.scalar_type() == at::kByte && q.is_contiguous() &&
              q.numel() == N * K, "fp8_untile: q must be a tiled FP8 part of N x K");
  TORCH_CHECK(out.is_contiguous() && out.element_size() == 1 && out.numel() == N * K, "fp8_untile: out [N, K] bytes");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "fp8_untile: 16-byte aligned out");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  hipserve::launch_fp8_untile(out.data_ptr(), q.data_ptr(), (int)N, (int)K, cur_stream());
}

void gguf_dequant(at::Tensor& out, const at::Tensor& q, const at::Tensor& d, const at::Tensor& mn,
                  int64_t qtype, int64_t row_bytes, int64_t N, int64_t K) {
  CHECK_DEV(q); CHECK_BF16(out); TORCH_CHECK(out.is_contiguous() && out.numel() >= N * K);
  TORCH_CHECK(q.scalar_type() == at::kByte && q.is_contiguous() && K % 256 == 0);
  TORCH_CHECK(qtype >= 0 && qtype <= 5);
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  hipserve::launch_gguf_dequant(out.data_ptr(), q.data_ptr(), d.numel() ? d.data_ptr() : nullptr,
                                mn.numel() ? mn.data_ptr() : nullptr, qtype, row_bytes, N, K,
                                cur_stream());
}

void skinny_gemm(at::Tensor& out, const at::Tensor& x, const at::Tensor& w, int64_t rt, int64_t kw) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out);
  CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out); CHECK_CONTIG(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) >= N);
  TORCH_CHECK(M >= 1 && M <= 64, "skinny_gemm: 1 <= M <= 64");
  TORCH_CHECK(kw >= 1 && K % (256 * kw) == 0, "skinny_gemm: K must be a multiple of 256*kw");
  TORCH_CHECK(x.stride(0) % 8 == 0, "x rows must be 16-byte aligned");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_skinny_gemm(out.data_ptr(), x.data_ptr(), x.stride(0), w.data_ptr(),
                                           out.stride(0), M, N, K, rt, kw, cur_stream()),
              "skinny_gemm: unsupported (rt, kw)");
}

// splits > 0: logits = the router decode GEMM's fp32 split-K partials, flat [splits, T, E]
// with T = w.size(0) (summed in order and rounded to bf16 in the kernel: no reduce launch)
void moe_topk_softmax(at::Tensor& w, at::Tensor& ids, const at::Tensor& logits, int64_t k, bool renorm,
                      int64_t splits) {
  CHECK_DEV(logits); CHECK_CONTIG(logits); CHECK_CONTIG(w); CHECK_CONTIG(ids);
  TORCH_CHECK(w.scalar_type() == at::kFloat && ids.scalar_type() == at::kInt);
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16);
  int T, E;
  if (splits > 0) {
    TORCH_CHECK(logits.scalar_type() == at::kFloat && w.dim() == 2, "moe_topk_softmax: fp32 partials, w [T, k]");
    T = w.size(0);
    TORCH_CHECK(T > 0 && logits.numel() % (splits * T) == 0, "moe_topk_softmax: partials [splits, T, E]");
    E = logits.numel() / (splits * T);
  } else {
    TORCH_CHECK(logits.dim() == 2, "moe_topk_softmax: logits [T, E]");
    T = logits.size(0);
    E = logits.size(1);
  }
  TORCH_CHECK(E <= 128, "moe: <= 128 experts");
  TORCH_CHECK(w.numel() >= T * k && ids.numel() >= T * k && k >= 1 && k <= E);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  hipserve::launch_moe_topk_softmax(logits.data_ptr(), logits.scalar_type() == at::kFloat, w.data_ptr<float>(),
                                    ids.data_ptr<int>(), T, E, k, renorm, cur_stream(), (int)splits);
}

int64_t car_create(int64_t rank, int64_t world, int64_t max_bytes, int64_t nb_large) {
  return reinterpret_cast<int64_t>(hipserve::car_create((int)rank, (int)world, (size_t)max_bytes, (int)nb_large));
}

at::Tensor car_handle(int64_t state) {
  auto t = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  hipserve::car_get_handle(reinterpret_cast<void*>(state), t.data_ptr());
  return t;
}

void car_open(int64_t state, int64_t peer, const at::Tensor& handle) {
  TORCH_CHECK(handle.device().is_cpu() && handle.numel() == 64 && handle.scalar_type() == at::kByte);
  auto h = handle.contiguous();
  hipserve::car_open(reinterpret_cast<void*>(state), (int)peer, h.data_ptr());
}

void car_all_reduce(int64_t state, const at::Tensor& inp, at::Tensor& out, bool two_shot) {
  CHECK_DEV(inp); CHECK_BF16(inp); CHECK_BF16(out); CHECK_CONTIG(inp); CHECK_CONTIG(out);
  TORCH_CHECK(inp.numel() == out.numel(), "car_all_reduce: size mismatch");
  const size_t bytes = inp.numel() * 2;
  TORCH_CHECK(bytes % 16 == 0 && bytes <= hipserve::car_max_bytes(reinterpret_cast<void*>(state)),
              "car_all_reduce: size must be a multiple of 16 B and fit the registered buffer");
  c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
  hipserve::launch_car(reinterpret_cast<void*>(state), inp.data_ptr(), out.data_ptr(), bytes, two_shot, 0,
                       cur_stream());
}

void car_all_gather(int64_t state, const at::Tensor& inp, at::Tensor& out) {
  CHECK_DEV(inp); CHECK_DEV(out); CHECK_CONTIG(inp); CHECK_CONTIG(out);
  TORCH_CHECK(inp.dim() == 2 && out.dim() == 2 && inp.size(0) == out.size(0) && inp.dtype() == out.dtype(),
              "car_all_gather: [rows, cols] -> [rows, world * cols]");
  TORCH_CHECK(out.size(1) % inp.size(1) == 0, "car_all_gather: out columns must be world * in columns");
  const size_t row = inp.size(1) * inp.element_size();
  const size_t bytes = row * inp.size(0);
  TORCH_CHECK(bytes <= hipserve::car_max_bytes(reinterpret_cast<void*>(state)), "car_all_gather: shard too large");
  if (bytes == 0) return;
  c10::hip::HIPGuardMasqueradingAsCUDA g(inp.device());
  hipserve::launch_car_all_gather(reinterpret_cast<void*>(state), inp.data_ptr(), out.data_ptr(), bytes, row,
                                  cur_stream());
}

bool car_norm_fits(int64_t state, int64_t M, int64_t N, bool exch_f32) {
  return hipserve::car_norm_fits(reinterpret_cast<void*>(state), (int)M, (int)N, exch_f32);
}

void car_add_rmsnorm(int64_t state, at::Tensor& out, at::Tensor& residual, const at::Tensor& x, int64_t splits,
                     const at::Tensor& weight, double eps, bool exch_f32) {
  CHECK_DEV(x); CHECK_BF16(out); CHECK_BF16(residual); CHECK_CONTIG(out); CHECK_CONTIG(residual); CHECK_CONTIG(x);
  TORCH_CHECK(residual.dim() == 2 && out.sizes() == residual.sizes(), "car_add_rmsnorm: out/residual [M, N]");
  const int M = residual.size(0), N = residual.size(1);
  const bool xf = x.scalar_type() == at::kFloat;
  TORCH_CHECK(xf || x.scalar_type() == at::kBFloat16, "car_add_rmsnorm: x fp32 partials or bf16");
  TORCH_CHECK(splits >= 1 && (xf || splits == 1), "car_add_rmsnorm: bf16 input has one slice");
  TORCH_CHECK(x.numel() == splits * (int64_t)M * N, "car_add_rmsnorm: x must hold splits * M * N values");
  TORCH_CHECK(weight.numel() == N && weight.is_contiguous() &&
              (weight.scalar_type() == at::kBFloat16 || weight.scalar_type() == at::kFloat));
  TORCH_CHECK(hipserve::car_norm_fits(reinterpret_cast<void*>(state), M, N, exch_f32),
              "car_add_rmsnorm: N must divide into 8-wide chunks per rank and the message fit the buffer");
  if (M == 0) return;
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_car_add_rmsnorm(reinterpret_cast<void*>(state), out.data_ptr(), residual.data_ptr(),
                                   x.data_ptr(), xf, (int)splits, weight.data_ptr(),
                                   weight.scalar_type() == at::kFloat, M, N, (float)eps, exch_f32, cur_stream());
}

static void check_pen_state(const at::Tensor& counts, const at::Tensor& seen, int V) {
  CHECK_DEV(counts); CHECK_CONTIG(counts); CHECK_CONTIG(seen);
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.dim() == 2 && counts.size(1) == V,
              "penalty counts: int32 [slots, V]");
  TORCH_CHECK(seen.scalar_type() == at::kInt && seen.dim() == 2 && seen.size(0) == counts.size(0) &&
              seen.size(1) == (V + 31) / 32, "penalty seen: int32 [slots, ceil(V/32)]");
}

void penalty_apply(at::Tensor& logits, const at::Tensor& slot, const at::Tensor& pres, const at::Tensor& freq,
                   const at::Tensor& rep, const at::Tensor& counts, const at::Tensor& seen) {
  CHECK_DEV(logits); CHECK_ROWMAJOR(logits);
  TORCH_CHECK(logits.dim() == 2 && (logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat));
  const int rows = logits.size(0), V = logits.size(1);
  check_pen_state(counts, seen, V);
  TORCH_CHECK(slot.scalar_type() == at::kInt && slot.numel() >= rows);
  TORCH_CHECK(pres.scalar_type() == at::kFloat && freq.scalar_type() == at::kFloat && rep.scalar_type() == at::kFloat);
  TORCH_CHECK(pres.numel() >= rows && freq.numel() >= rows && rep.numel() >= rows);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  hipserve::launch_penalty_apply(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, logits.stride(0), rows, V,
                                 slot.data_ptr<int>(), pres.data_ptr<float>(), freq.data_ptr<float>(),
                                 rep.data_ptr<float>(), counts.data_ptr<int>(),
                                 reinterpret_cast<const unsigned int*>(seen.data_ptr<int>()), cur_stream());
}

void penalty_update(const at::Tensor& tok, const at::Tensor& slot, at::Tensor& counts, at::Tensor& seen) {
  CHECK_DEV(tok);
  TORCH_CHECK(tok.scalar_type() == at::kLong && slot.scalar_type() == at::kInt && slot.numel() >= tok.numel());
  const int V = counts.size(1);
  check_pen_state(counts, seen, V);
  c10::hip::HIPGuardMasqueradingAsCUDA g(tok.device());
  hipserve::launch_penalty_update(tok.data_ptr<int64_t>(), slot.data_ptr<int>(), tok.numel(), counts.data_ptr<int>(),
                                  reinterpret_cast<unsigned int*>(seen.data_ptr<int>()), V, cur_stream());
}

void penalty_init(at::Tensor& counts, at::Tensor& seen, const at::Tensor& slots, const at::Tensor& off,
                  const at::Tensor& n_prompt, const at::Tensor& toks) {
  const int V = counts.size(1);
  check_pen_state(counts, seen, V);
  TORCH_CHECK(slots.scalar_type() == at::kInt && off.scalar_type() == at::kInt && n_prompt.scalar_type() == at::kInt &&
              toks.scalar_type() == at::kInt);
  const int n = slots.numel();
  TORCH_CHECK(off.numel() == n + 1 && n_prompt.numel() == n);
  c10::hip::HIPGuardMasqueradingAsCUDA g(counts.device());
  hipserve::launch_penalty_init(counts.data_ptr<int>(), reinterpret_cast<unsigned int*>(seen.data_ptr<int>()), V,
                                slots.data_ptr<int>(), off.data_ptr<int>(), n_prompt.data_ptr<int>(),
                                toks.data_ptr<int>(), n, cur_stream());
}

void top_logprobs(const at::Tensor& logits, const at::Tensor& nreq, at::Tensor& out_ids, at::Tensor& out_lp) {
  CHECK_DEV(logits); CHECK_ROWMAJOR(logits);
  TORCH_CHECK(logits.dim() == 2 && (logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat));
  const int rows = logits.size(0);
  TORCH_CHECK(nreq.scalar_type() == at::kInt && nreq.numel() >= rows);
  TORCH_CHECK(out_ids.scalar_type() == at::kInt && out_lp.scalar_type() == at::kFloat && out_ids.dim() == 2 &&
              out_ids.sizes() == out_lp.sizes() && out_ids.size(0) >= rows && out_ids.is_contiguous() &&
              out_lp.is_contiguous() && out_ids.size(1) <= 64);
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  hipserve::launch_top_logprobs(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, logits.stride(0), rows,
                                logits.size(1), nreq.data_ptr<int>(), out_ids.data_ptr<int>(),
                                out_lp.data_ptr<float>(), out_ids.size(1), cur_stream());
}

bool car_error(int64_t state) { return hipserve::car_error(reinterpret_cast<void*>(state)); }

void car_destroy(int64_t state) { hipserve::car_destroy(reinterpret_cast<void*>(state)); }

void fill_uniform(at::Tensor& out, int64_t row0, int64_t col0, int64_t gcols, int64_t key, double scale) {
  CHECK_DEV(out); CHECK_BF16(out);
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1, "fill_uniform: 2-D row-major view");
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  hipserve::launch_fill_uniform(out.data_ptr(), out.stride(0), out.size(0), out.size(1), row0, col0, gcols,
                                (unsigned int)(key & 0xffffffffu), (float)scale, cur_stream());
}

// Pinned host tensors are addressed through their device mapping; every pair must
// match in byte size (a multiple of 4) and be contiguous. Runs on `device`'s
// current stream.
void stage_copy(const std::vector<at::Tensor>& dst, const std::vector<at::Tensor>& src, int64_t device) {
  TORCH_CHECK(dst.size() == src.size() && dst.size() <= (size_t)hipserve::kMaxStageCopies,
              "stage_copy: matching lists of at most 8 tensors");
  hipserve::StageCopyArgs a{};
  a.n = (int)dst.size();
  auto addr = [](const at::Tensor& t, bool& host) -> void* {
    TORCH_CHECK(t.is_contiguous(), "stage_copy: tensors must be contiguous");
    if (t.is_cuda()) { host = false; return t.data_ptr(); }
    TORCH_CHECK(t.is_pinned(), "stage_copy: host tensors must be pinned");
    host = true;
    void* d = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&d, t.data_ptr(), 0) == hipSuccess && d,
                "stage_copy: pinned tensor has no device mapping");
    return d;
  };
  for (int i = 0; i < a.n; ++i) {
    const size_t nb = dst[i].nbytes();
    TORCH_CHECK(nb == src[i].nbytes() && nb % 4 == 0, "stage_copy: pair ", i, " byte sizes differ or not 4-aligned");
    bool hd = false, hs = false;
    a.dst[i] = addr(dst[i], hd);
    a.src[i] = addr(src[i], hs);
    a.words[i] = (long)(nb / 4);
    a.host_mask |= (hs ? 1u : 0u) << (2 * i);
    a.host_mask |= (hd ? 1u : 0u) << (2 * i + 1);
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)device);
  hipserve::launch_stage_copy(a, cur_stream());
}

void decode_gemm(at::Tensor& out, const at::Tensor& x, const at::Tensor& w, at::Tensor& ws, int64_t rt,
                 int64_t splits) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  CHECK_CONTIG(w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == N, "decode_gemm: shape mismatch");
  TORCH_CHECK(M >= 1 && M <= 64, "decode_gemm: 1 <= M <= 64");
  TORCH_CHECK(splits >= 1 && K % (256 * splits) == 0, "decode_gemm: K must be a multiple of 256*splits");
  TORCH_CHECK(N % 4 == 0 && out.stride(0) % 4 == 0 && x.stride(0) % 8 == 0, "decode_gemm: alignment");
  if (splits > 1) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * N && N % 8 == 0,
                "decode_gemm: fp32 workspace of S*M*N (N % 8 == 0) required for split-K");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_decode_gemm(out.data_ptr(), out.stride(0),
                                           splits > 1 ? ws.data_ptr<float>() : nullptr, x.data_ptr(), x.stride(0),
                                           w.data_ptr(), M, N, K, rt, splits, false, 0, cur_stream()),
              "decode_gemm: unsupported (rt, K/splits): rt in {1,2}, K/splits = 256*{1,2,4,7,8,12,16,21}");
}

// Packed weights: wp = pack_decode_weight(w[N, K]) (flat, ceil(N/128)*128*K bf16).
void decode_gemm_packed(at::Tensor& out, const at::Tensor& x, const at::Tensor& wp, at::Tensor& ws, int64_t N,
                        int64_t rt, int64_t splits) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(wp); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  CHECK_CONTIG(wp);
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 256 == 0 && wp.numel() == (N + 127) / 128 * 128 * K, "decode_gemm_packed: packed size mismatch");
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "decode_gemm_packed: out shape");
  TORCH_CHECK(M >= 1 && M <= 64, "decode_gemm_packed: 1 <= M <= 64");
  TORCH_CHECK(splits >= 1 && K % (256 * splits) == 0, "decode_gemm_packed: K must be a multiple of 256*splits");
  TORCH_CHECK(N % 4 == 0 && out.stride(0) % 4 == 0 && x.stride(0) % 8 == 0, "decode_gemm_packed: alignment");
  if (splits > 1) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * N && N % 8 == 0,
                "decode_gemm_packed: fp32 workspace of S*M*N (N % 8 == 0) required for split-K");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_decode_gemm(out.data_ptr(), out.stride(0),
                                           splits > 1 ? ws.data_ptr<float>() : nullptr, x.data_ptr(), x.stride(0),
                                           wp.data_ptr(), M, N, K, rt, splits, true, 0, cur_stream()),
              "decode_gemm_packed: unsupported (rt, K/splits)");
}

// Decode GEMM writing fp32 split-K partials ws[S, M, N] for a fused epilogue
// (splitk_add_rmsnorm / splitk_rope_cache).
void decode_gemm_partial(at::Tensor& ws, const at::Tensor& x, const at::Tensor& w, int64_t N, int64_t rt,
                         int64_t splits, bool packed) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_ROWMAJOR(x); CHECK_CONTIG(w);
  const int M = x.size(0), K = x.size(1);
  if (packed) {
    TORCH_CHECK(w.numel() == (N + 127) / 128 * 128 * K, "decode_gemm_partial: packed size mismatch");
  } else {
    TORCH_CHECK(w.dim() == 2 && w.size(0) == N && w.size(1) == K, "decode_gemm_partial: w [N, K]");
  }
  TORCH_CHECK(M >= 1 && M <= 64 && K % (256 * splits) == 0 && N % 8 == 0 && x.stride(0) % 8 == 0,
              "decode_gemm_partial: shape / alignment");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * N,
              "decode_gemm_partial: ws must hold S*M*N fp32");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_decode_gemm(nullptr, N, ws.data_ptr<float>(), x.data_ptr(), x.stride(0), w.data_ptr(),
                                           M, N, K, rt, splits, packed, hipserve::DG_PARTIAL, cur_stream()),
              "decode_gemm_partial: unsupported (rt, K/splits)");
}

// Merged gate|up decode GEMM with the SiLU-GLU fused: act[M, N/2] = silu(x Wg^T) * (x Wu^T),
// wp = pack_decode_weight(w, glu=true). splits > 1 needs ws of S*M*N fp32.
void decode_gemm_glu(at::Tensor& act, const at::Tensor& x, const at::Tensor& wp, at::Tensor& ws, int64_t N,
                     int64_t rt, int64_t splits) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(wp); CHECK_BF16(act); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(act);
  CHECK_CONTIG(wp);
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(N % 128 == 0 && wp.numel() == N * K && K % (256 * splits) == 0, "decode_gemm_glu: shapes");
  TORCH_CHECK(act.size(0) == M && act.size(1) == N / 2 && act.stride(0) % 8 == 0, "decode_gemm_glu: act [M, N/2]");
  TORCH_CHECK(M >= 1 && M <= 64 && x.stride(0) % 8 == 0, "decode_gemm_glu: 1 <= M <= 64");
  if (splits > 1) {
    TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * N,
                "decode_gemm_glu: ws must hold S*M*N fp32");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_decode_gemm(act.data_ptr(), act.stride(0), splits > 1 ? ws.data_ptr<float>() : nullptr,
                                           x.data_ptr(), x.stride(0), wp.data_ptr(), M, N, K, rt, splits, true,
                                           hipserve::DG_GLU, cur_stream()),
              "decode_gemm_glu: unsupported (rt, K/splits)");
}



// Prefill GEMM over the packed decode layout (prefill_gemm_packed.hip): wp =
// pack_decode_weight(w[N, K], glu) (flat, ceil(N/128)*128*K bf16). epi as the FP8 prefill GEMM (PG_EPI_*)
// (2 / 3 need the glu packing); bias (epi 0 only) bf16 [N] or None; wm 1 or 2.
void prefill_gemm_packed(at::Tensor& out, const at::Tensor& x, const at::Tensor& wp, int64_t N, int64_t epi,
                         const c10::optional<at::Tensor>& bias, int64_t wm, int64_t grid, int64_t rw) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(wp); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(wp.is_contiguous(), "prefill_gemm_packed: packed weight must be contiguous");
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 256 == 0 && wp.numel() == (N + 127) / 128 * 128 * K, "prefill_gemm_packed: wp = pack(w[N, K % 256])");
  TORCH_CHECK(x.stride(0) % 8 == 0 && out.stride(0) % 4 == 0, "prefill_gemm_packed: alignment");
  const bool glu = epi == 2 || epi == 3;
  TORCH_CHECK(out.size(0) == M && out.size(1) == (glu ? N / 2 : N), "prefill_gemm_packed: out shape");
  const void* bp = nullptr;
  if (bias.has_value()) {
    CHECK_BF16((*bias));
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "prefill_gemm_packed: bias [N]");
    bp = bias->data_ptr();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_prefill_gemm_packed((int)epi, out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0),
                                                   wp.data_ptr(), M, (int)N, K, bp, (int)wm, (int)grid, cur_stream(),
                                                   nullptr, (int)rw),
              "prefill_gemm_packed: unsupported (glu needs N % 128, bias only with epi 0, 32-bit offsets)");
}

// Grouped (MoE prefill experts) form: x = expert-sorted slot rows [cap, K] (moe_align
// with tile 128 * wm + moe_gather), wp = [E, packed expert] (pack_decode_weight per
// expert, glu for w13), tile_expert / num_tiles from moe_align. epi 0 or 2 / 3.
void prefill_gemm_packed_grouped(at::Tensor& out, const at::Tensor& x, const at::Tensor& wp, int64_t N, int64_t epi,
                                 const at::Tensor& tile_expert, const at::Tensor& num_tiles, int64_t wm, int64_t rw,
                                 const c10::optional<at::Tensor>& gather_slots, int64_t gather_k) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(wp); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  TORCH_CHECK(wp.dim() == 2 && wp.is_contiguous(), "prefill_gemm_packed_grouped: wp [E, packed]");
  // gather: x holds the token rows and slot row s reads x[gather_slots[s] / gather_k] (moe_align's slots)
  const bool gather = gather_slots.has_value() && gather_slots->numel() > 0;
  if (gather)
    TORCH_CHECK(gather_slots->scalar_type() == at::kInt && gather_slots->is_contiguous() &&
                    gather_slots->numel() == out.size(0) && gather_k >= 1 && x.stride(0) % 8 == 0,
                "prefill_gemm_packed_grouped: gather_slots [slot rows] int32, gather_k >= 1");
  const int M = gather ? out.size(0) : x.size(0), K = x.size(1);
  TORCH_CHECK(K % 256 == 0 && wp.size(1) == (N + 127) / 128 * 128 * K, "prefill_gemm_packed_grouped: wp per expert");
  TORCH_CHECK(M % (128 * wm) == 0 && tile_expert.numel() >= M / (128 * wm), "prefill_gemm_packed_grouped: tiles");
  TORCH_CHECK(tile_expert.scalar_type() == at::kInt && num_tiles.scalar_type() == at::kInt, "int32 tile tables");
  const bool glu = epi == 2 || epi == 3;
  TORCH_CHECK(epi == 0 || glu, "prefill_gemm_packed_grouped: store or glu epilogue");
  TORCH_CHECK(out.size(0) == M && out.size(1) == (glu ? N / 2 : N), "prefill_gemm_packed_grouped: out shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::PwGroup grp{tile_expert.data_ptr<int>(), num_tiles.data_ptr<int>(), (long)wp.size(1)};
  if (gather) {
    grp.gather_slots = gather_slots->data_ptr<int>();
    grp.gather_k = (int)gather_k;
    grp.x_rows = (int)x.size(0);
  }
  TORCH_CHECK(hipserve::launch_prefill_gemm_packed((int)epi, out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0),
                                                   wp.data_ptr(), M, (int)N, K, nullptr, (int)wm, 0, cur_stream(),
                                                   &grp, (int)rw),
              "prefill_gemm_packed_grouped: unsupported");
}

// FP8 W8A8 form: xq [M, K] uint8 e4m3 + xs [M] fp32 (act_quant_fp8), the weight as
// tiled FP8 parts (ops/quant.py QuantPart.from_fp8: q [N/16, K/256, 4096] uint8 and
// rs [N] fp32) stacked along N. epi 0 / 1 = store / residual add; 2 / 3: parts = (gate, up),
// out = act [M, I] = silu / gelu_tanh(gate) * up.
void prefill_gemm_f8(at::Tensor& out, const at::Tensor& xq, const at::Tensor& xs, const std::vector<at::Tensor>& q,
                     const std::vector<at::Tensor>& rs, int64_t epi) {
  CHECK_DEV(xq); CHECK_CONTIG(xq); CHECK_CONTIG(xs); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  TORCH_CHECK(xq.scalar_type() == at::kByte && xs.scalar_type() == at::kFloat, "prefill_gemm_f8: xq uint8, xs fp32");
  const int M = xq.size(0), K = xq.size(1);
  TORCH_CHECK(xs.numel() == M && K % 256 == 0 && out.stride(0) % 4 == 0, "prefill_gemm_f8: shapes");
  TORCH_CHECK(!q.empty() && q.size() <= (size_t)hipserve::kPgF8Parts && rs.size() == q.size(), "prefill_gemm_f8: parts");
  hipserve::PgF8 W{};
  W.n = (int)q.size();
  W.xs = xs.data_ptr<float>();
  int rows = 0;
  for (size_t i = 0; i < q.size(); ++i) {
    CHECK_CONTIG(q[i]); CHECK_CONTIG(rs[i]);
    const int n = rs[i].numel();
    TORCH_CHECK(q[i].scalar_type() == at::kByte && rs[i].scalar_type() == at::kFloat && q[i].numel() == (long)n * K,
                "prefill_gemm_f8: part ", i, " must be tiled FP8 [N/16, K/256, 4096] with rs [N]");
    W.p[i] = hipserve::PgF8Part{q[i].data_ptr<uint8_t>(), rs[i].data_ptr<float>(), n, rows / 256};
    rows += n;
  }
  const bool glu = epi == 2 || epi == 3;
  TORCH_CHECK(out.size(0) == M && out.size(1) == (glu ? rows / 2 : rows), "prefill_gemm_f8: out shape");
  c10::hip::HIPGuardMasqueradingAsCUDA g(xq.device());
  TORCH_CHECK(hipserve::launch_prefill_gemm_f8((int)epi, out.data_ptr(), out.stride(0), xq.data_ptr(), K, W, M, rows, K,
                                               cur_stream()),
              "prefill_gemm_f8: unsupported part shapes (rows % 256; GLU: two equal parts, rows % 128)");
}

// FP8 W8A8 decode form (fp8_decode.hip): fp32 split-K partials ws [S, M, N] of the
// per-token e4m3 activations xq / xs against the tiled FP8 parts, for the fused decode
// epilogues or splitk_reduce.
void fp8_decode_gemm(at::Tensor& ws, const at::Tensor& xq, const at::Tensor& xs, const std::vector<at::Tensor>& q,
                     const std::vector<at::Tensor>& rs, int64_t splits) {
  CHECK_DEV(xq); CHECK_CONTIG(xq); CHECK_CONTIG(xs); CHECK_CONTIG(ws);
  TORCH_CHECK(xq.scalar_type() == at::kByte && xs.scalar_type() == at::kFloat && ws.scalar_type() == at::kFloat,
              "fp8_decode_gemm: xq uint8, xs / ws fp32");
  const int M = xq.size(0), K = xq.size(1);
  TORCH_CHECK(xs.numel() == M && K % 256 == 0, "fp8_decode_gemm: shapes");
  TORCH_CHECK(!q.empty() && q.size() <= (size_t)hipserve::kPgF8Parts && rs.size() == q.size(), "fp8_decode_gemm: parts");
  hipserve::PgF8 W{};
  W.n = (int)q.size();
  W.xs = xs.data_ptr<float>();
  int rows = 0;
  for (size_t i = 0; i < q.size(); ++i) {
    CHECK_CONTIG(q[i]); CHECK_CONTIG(rs[i]);
    const int n = rs[i].numel();
    TORCH_CHECK(q[i].scalar_type() == at::kByte && rs[i].scalar_type() == at::kFloat && q[i].numel() == (long)n * K,
                "fp8_decode_gemm: part ", i, " must be tiled FP8 [N/16, K/256, 4096] with rs [N]");
    W.p[i] = hipserve::PgF8Part{q[i].data_ptr<uint8_t>(), rs[i].data_ptr<float>(), n, 0};
    rows += n;
  }
  TORCH_CHECK(ws.numel() >= splits * (long)M * rows, "fp8_decode_gemm: ws too small");
  c10::hip::HIPGuardMasqueradingAsCUDA g(xq.device());
  TORCH_CHECK(hipserve::launch_fp8_decode_gemm(ws.data_ptr<float>(), xq.data_ptr(), W, M, rows, K, (int)splits,
                                               cur_stream()),
              "fp8_decode_gemm: unsupported (M <= 256, part rows % 16, (K / 256) / splits in the kernel's step set)");
}

// [gate | up] rows -> per-token e4m3 act (q8 [rows, I] uint8, xs [rows] fp32), optionally
// the bf16 act too: glu_and_mul -> act_quant_fp8 in one pass
void glu_quant(const c10::optional<at::Tensor>& out, at::Tensor& q8, at::Tensor& xs, const at::Tensor& x, bool gelu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_CONTIG(q8); CHECK_CONTIG(xs);
  const long rows = x.size(0);
  const int inter = x.size(1) / 2;
  TORCH_CHECK(q8.scalar_type() == at::kByte && q8.size(0) == rows && q8.size(1) == inter &&
                  xs.scalar_type() == at::kFloat && xs.numel() == rows && x.stride(0) % 8 == 0,
              "glu_quant: q8 uint8 [rows, I], xs fp32 [rows]");
  void* o = nullptr;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(out->scalar_type() == at::kBFloat16 && out->is_contiguous() && out->size(0) == rows &&
                out->size(1) == inter, "glu_quant: out bf16 [rows, I]");
    o = out->data_ptr();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_glu_quant(gelu, o, q8.data_ptr(), xs.data_ptr<float>(), x.data_ptr(), rows, inter,
                                         x.stride(0), cur_stream()),
              "glu_quant: I % 8 == 0 and I <= 32768");
}

void act_quant_fp8(at::Tensor& xq, at::Tensor& xs, const at::Tensor& x) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_ROWMAJOR(x); CHECK_CONTIG(xq); CHECK_CONTIG(xs);
  const int M = x.size(0), K = x.size(1);
  TORCH_CHECK(xq.scalar_type() == at::kByte && xq.size(0) == M && xq.size(1) == K && xs.scalar_type() == at::kFloat &&
                  xs.numel() == M && K % 8 == 0 && x.stride(0) % 8 == 0,
              "act_quant_fp8: xq uint8 [M, K], xs fp32 [M], K % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_act_quant_fp8(xq.data_ptr(), xs.data_ptr<float>(), x.data_ptr(), x.stride(0), M, K, cur_stream());
}


static const void* opt_ptr(const c10::optional<at::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// optional per-token e4m3 copy (out8 uint8 like out, xs8 fp32 [M]) of a norm epilogue's output
static void e4m3_out_args(const c10::optional<at::Tensor>& out8, const c10::optional<at::Tensor>& xs8,
                          const at::Tensor& out, void** o8, float** x8, const char* who) {
  *o8 = nullptr;
  *x8 = nullptr;
  if (out8.has_value() && out8->defined()) {
    TORCH_CHECK(xs8.has_value() && xs8->defined(), who, ": out8 needs xs8");
    TORCH_CHECK(out8->scalar_type() == at::kByte && out8->sizes() == out.sizes() && out8->is_contiguous() &&
                    xs8->scalar_type() == at::kFloat && xs8->numel() == out.size(0) && xs8->is_contiguous(),
                who, ": out8 uint8 like out, xs8 fp32 [M]");
    *o8 = out8->data_ptr();
    *x8 = xs8->data_ptr<float>();
  }
}

void splitk_add_rmsnorm(at::Tensor& out, at::Tensor& residual, const at::Tensor& ws, int64_t splits,
                        const at::Tensor& weight, double eps, const c10::optional<at::Tensor>& out16,
                        const c10::optional<at::Tensor>& out8, const c10::optional<at::Tensor>& xs8) {
  CHECK_DEV(ws); CHECK_BF16(out); CHECK_BF16(residual); CHECK_CONTIG(out); CHECK_CONTIG(residual);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous());
  const int M = residual.size(0), N = residual.size(1);
  TORCH_CHECK(out.sizes() == residual.sizes() && ws.numel() >= splits * M * N && N % 8 == 0 && N <= 16384);
  TORCH_CHECK(weight.numel() == N && weight.is_contiguous() &&
              (weight.scalar_type() == at::kBFloat16 || weight.scalar_type() == at::kFloat));
  c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
  void* o16 = nullptr;
  if (out16.has_value() && out16->defined()) {
    TORCH_CHECK(out16->scalar_type() == at::kHalf && out16->sizes() == out.sizes() && out16->is_contiguous(),
                "splitk_add_rmsnorm: out16 f16 like out");
    o16 = out16->data_ptr();
  }
  void* o8;
  float* x8;
  e4m3_out_args(out8, xs8, out, &o8, &x8, "splitk_add_rmsnorm");
  hipserve::launch_splitk_add_rmsnorm(out.data_ptr(), residual.data_ptr(), ws.data_ptr<float>(), splits,
                                      weight.data_ptr(), weight.scalar_type() == at::kFloat, M, N, (float)eps,
                                      cur_stream(), o16, o8, x8);
}

void splitk_post_add_rmsnorm(at::Tensor& out, at::Tensor& residual, const at::Tensor& ws, int64_t splits,
                             const at::Tensor& w_post, const at::Tensor& w_next, double eps,
                             const c10::optional<at::Tensor>& out16, const c10::optional<at::Tensor>& out8,
                             const c10::optional<at::Tensor>& xs8) {
  CHECK_DEV(ws); CHECK_BF16(out); CHECK_BF16(residual); CHECK_CONTIG(out); CHECK_CONTIG(residual);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous());
  const int M = residual.size(0), N = residual.size(1);
  TORCH_CHECK(out.sizes() == residual.sizes() && ws.numel() >= splits * M * N && N % 8 == 0 && N <= 16384);
  TORCH_CHECK(w_post.numel() == N && w_next.numel() == N && w_post.is_contiguous() && w_next.is_contiguous() &&
                  w_post.scalar_type() == w_next.scalar_type() &&
                  (w_post.scalar_type() == at::kBFloat16 || w_post.scalar_type() == at::kFloat),
              "splitk_post_add_rmsnorm: both norm weights bf16 or both fp32 [N]");
  void* o16 = nullptr;
  if (out16.has_value() && out16->defined()) {
    TORCH_CHECK(out16->scalar_type() == at::kHalf && out16->sizes() == out.sizes() && out16->is_contiguous(),
                "splitk_post_add_rmsnorm: out16 f16 like out");
    o16 = out16->data_ptr();
  }
  void* o8;
  float* x8;
  e4m3_out_args(out8, xs8, out, &o8, &x8, "splitk_post_add_rmsnorm");
  c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
  hipserve::launch_splitk_post_add_rmsnorm(out.data_ptr(), residual.data_ptr(), ws.data_ptr<float>(), splits,
                                           w_post.data_ptr(), w_next.data_ptr(), w_post.scalar_type() == at::kFloat,
                                           M, N, (float)eps, cur_stream(), o16, o8, x8);
}

void splitk_rope_cache(at::Tensor& qkv, const at::Tensor& ws, int64_t splits, const at::Tensor& positions,
                       const at::Tensor& slots, const at::Tensor& cos_sin, at::Tensor& k_cache, at::Tensor& v_cache,
                       int64_t nq, int64_t nkv, int64_t head_dim, int64_t mode,
                       const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& q_w,
                       const c10::optional<at::Tensor>& k_w, double eps) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_ROWMAJOR(qkv);
  const int T = qkv.size(0);
  const long N = (nq + 2 * nkv) * head_dim;
  const void* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "splitk_rope_cache: bias bf16 [N]");
    bp = bias->data_ptr();
  }
  const float *qwp = nullptr, *kwp = nullptr;
  if (q_w.has_value()) {
    TORCH_CHECK(k_w.has_value() && q_w->scalar_type() == at::kFloat && k_w->scalar_type() == at::kFloat &&
                q_w->numel() == head_dim && k_w->numel() == head_dim && q_w->is_contiguous() && k_w->is_contiguous(),
                "splitk_rope_cache: fp32 q/k norm weights [head_dim]");
    const int lanes = (int)head_dim / 16;
    TORCH_CHECK(mode == 0 && (lanes == 4 || lanes == 8 || lanes == 16), "splitk_rope_cache: q/k norm needs mode 0, head_dim 64/128/256");
    qwp = q_w->data_ptr<float>();
    kwp = k_w->data_ptr<float>();
  }
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= N);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * T * N);
  TORCH_CHECK(positions.scalar_type() == at::kLong && slots.scalar_type() == at::kLong);
  TORCH_CHECK(positions.numel() >= T && slots.numel() >= T);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == head_dim && cos_sin.is_contiguous());
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(3) == head_dim, "k_cache [blocks, nkv, bs, D]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == nkv && v_cache.size(2) == head_dim, "v_cache [blocks, nkv, D, bs]");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous());
  TORCH_CHECK(head_dim % 16 == 0 && (mode == 0 || mode == 1));
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  hipserve::launch_splitk_rope_cache(qkv.data_ptr(), qkv.stride(0), ws.data_ptr<float>(), splits,
                                     positions.data_ptr<int64_t>(), slots.data_ptr<int64_t>(),
                                     cos_sin.data_ptr<float>(), k_cache.data_ptr(), v_cache.data_ptr(), T, nq, nkv,
                                     head_dim, k_cache.size(2), mode, cur_stream(), bp, qwp, kwp, (float)eps,
                                     kv_is_f8(k_cache, v_cache));
}

void splitk_reduce(at::Tensor& out, const at::Tensor& ws, int64_t splits) {
  CHECK_DEV(out); CHECK_BF16(out); CHECK_ROWMAJOR(out);
  const int M = out.size(0), N = out.size(1);
  TORCH_CHECK(N % 8 == 0 && out.stride(0) % 8 == 0, "splitk_reduce: N % 8 == 0");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * (long)N);
  c10::hip::HIPGuardMasqueradingAsCUDA g(out.device());
  hipserve::launch_splitk_reduce(out.data_ptr(), out.stride(0), ws.data_ptr<float>(), M, N, splits, cur_stream());
}

void splitk_glu(at::Tensor& act, const at::Tensor& ws, int64_t splits, bool gelu,
                const c10::optional<at::Tensor>& act16) {
  CHECK_DEV(act); CHECK_BF16(act); CHECK_ROWMAJOR(act);
  const int M = act.size(0), I = act.size(1);
  TORCH_CHECK(I % 8 == 0 && act.stride(0) % 8 == 0, "splitk_glu: I % 8 == 0");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous() && ws.numel() >= splits * M * 2L * I);
  c10::hip::HIPGuardMasqueradingAsCUDA g(act.device());
  void* a16 = nullptr;
  if (act16.has_value() && act16->defined()) {
    TORCH_CHECK(act16->scalar_type() == at::kHalf && act16->sizes() == act.sizes() &&
                    act16->stride(0) == act.stride(0) && act16->stride(1) == 1,
                "splitk_glu: act16 f16 like act");
    a16 = act16->data_ptr();
  }
  hipserve::launch_splitk_glu(act.data_ptr(), act.stride(0), ws.data_ptr<float>(), splits, M, I, gelu,
                              cur_stream(), a16);
}

// w [N, K], or a stack [E, N, K] (MoE experts: one launch, out = E packed copies back to back)
void pack_decode_weight(at::Tensor& out, const at::Tensor& w, bool glu) {
  CHECK_DEV(w); CHECK_BF16(w); CHECK_CONTIG(w); CHECK_BF16(out); CHECK_CONTIG(out);
  TORCH_CHECK((w.dim() == 2 || w.dim() == 3) && w.size(-1) % 256 == 0,
              "pack_decode_weight: w [N, K] or [E, N, K], K % 256 == 0");
  const long E = w.dim() == 3 ? w.size(0) : 1, N = w.size(-2), K = w.size(-1);
  TORCH_CHECK(out.numel() == E * ((N + 127) / 128 * 128 * K), "pack_decode_weight: out must hold E*ceil(N/128)*128*K");
  TORCH_CHECK(!glu || N % 128 == 0, "pack_decode_weight: glu packing needs N % 128 == 0");
  TORCH_CHECK(E <= 65535, "pack_decode_weight: at most 65535 stacked matrices");
  c10::hip::HIPGuardMasqueradingAsCUDA g(w.device());
  hipserve::launch_pack_decode_weight(out.data_ptr(), w.data_ptr(), N, K, glu, cur_stream(), (int)E);
}

void moe_align(const at::Tensor& ids, int64_t E, int64_t tile, at::Tensor& slots, at::Tensor& tile_expert,
               at::Tensor& num_tiles, at::Tensor& pair_slot, const c10::optional<at::Tensor>& group_end) {
  CHECK_DEV(ids);
  TORCH_CHECK(ids.scalar_type() == at::kInt && slots.scalar_type() == at::kInt &&
              tile_expert.scalar_type() == at::kInt && pair_slot.scalar_type() == at::kInt);
  TORCH_CHECK(E <= 128 && (tile == 16 || tile == 32 || tile == 64 || tile == 128 || tile == 256));
  const int npairs = ids.numel();
  TORCH_CHECK(slots.numel() >= npairs + E * (tile - 1) && slots.numel() % tile == 0,
              "slots capacity must cover padding and be a multiple of the tile");
  TORCH_CHECK(tile_expert.numel() * tile >= slots.numel() && pair_slot.numel() >= npairs);
  int* ge = nullptr;
  if (group_end.has_value() && group_end->numel() > 0) {
    TORCH_CHECK(group_end->scalar_type() == at::kInt && group_end->numel() >= E && group_end->is_contiguous());
    ge = group_end->data_ptr<int>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(ids.device());
  const int nb = hipserve::moe_align_blocks(npairs);
  at::Tensor hist;  // multi-workgroup form (prefill): per-block expert histograms
  if (nb > 1) hist = at::empty({(long)nb * 128}, ids.options().dtype(at::kInt));
  hipserve::launch_moe_align(ids.data_ptr<int>(), npairs, E, tile, slots.data_ptr<int>(), slots.numel(),
                             tile_expert.data_ptr<int>(), tile_expert.numel(), num_tiles.data_ptr<int>(),
                             pair_slot.data_ptr<int>(), ge, cur_stream(), nb > 1 ? hist.data_ptr<int>() : nullptr);
}

void moe_gather(at::Tensor& out, const at::Tensor& x, const at::Tensor& slots, int64_t k) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_CONTIG(out);
  TORCH_CHECK(slots.scalar_type() == at::kInt && slots.is_contiguous() && out.size(0) >= slots.numel());
  const int H = out.size(1);
  TORCH_CHECK(H % 8 == 0 && x.size(1) == H && x.stride(0) % 8 == 0, "moe_gather: H % 8 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_moe_gather(out.data_ptr(), x.data_ptr(), x.stride(0), slots.data_ptr<int>(), slots.numel(), k, H,
                              cur_stream());
}

void moe_gemm(at::Tensor& out, const at::Tensor& x, const at::Tensor& w, const at::Tensor& slots,
              const at::Tensor& tile_expert, int64_t tile, int64_t gather_k) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(out); CHECK_ROWMAJOR(x); CHECK_ROWMAJOR(out);
  CHECK_CONTIG(w);
  TORCH_CHECK(w.dim() == 3, "w [E, N, K]");
  const int N = w.size(1), K = w.size(2);
  TORCH_CHECK(K % 256 == 0 && x.size(1) >= K && out.size(1) >= N);
  TORCH_CHECK(out.size(0) >= slots.numel() && x.stride(0) % 8 == 0);
  TORCH_CHECK(tile_expert.numel() * tile >= slots.numel());
  TORCH_CHECK(gather_k > 0 || x.size(0) >= slots.numel(), "ungathered x needs one row per slot");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_moe_gemm(out.data_ptr(), out.stride(0), x.data_ptr(), x.stride(0), w.data_ptr(),
                            slots.data_ptr<int>(), tile_expert.data_ptr<int>(), slots.numel() / tile, tile,
                            gather_k, N, K, cur_stream());
}

void moe_combine(at::Tensor& out, const at::Tensor& y, const at::Tensor& w, const at::Tensor& pair_slot,
                 int64_t k) {
  CHECK_DEV(y); CHECK_BF16(y); CHECK_BF16(out); CHECK_CONTIG(y); CHECK_CONTIG(out);
  TORCH_CHECK(w.scalar_type() == at::kFloat && pair_slot.scalar_type() == at::kInt);
  const int T = out.size(0), H = out.size(1);
  TORCH_CHECK(y.size(1) == H && H % 8 == 0 && w.numel() >= T * k && pair_slot.numel() >= T * k);
  c10::hip::HIPGuardMasqueradingAsCUDA g(y.device());
  hipserve::launch_moe_combine(out.data_ptr(), y.data_ptr(), w.data_ptr<float>(), pair_slot.data_ptr<int>(), T, k,
                               H, cur_stream());
}

// Expert GEMM over moe_align tiles on the decode GEMM (decode_gemm.hip, kMoe).
// w: [E, ceil(N/128)*128*K] packed (pack_decode_weight per expert; glu = gate/up
// interleaved) or row-major [E, N, K]. out bf16: [slots, N] (glu: act [slots, N/2],
// splits must be 1); out fp32: partials [splits, slots, N] for moe_combine_partial.
void moe_decode_gemm(at::Tensor& out, const at::Tensor& x, const at::Tensor& w, const at::Tensor& slots,
                     const at::Tensor& tile_expert, int64_t tile, int64_t gather_k, int64_t N, int64_t splits,
                     bool packed, bool glu) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_ROWMAJOR(x); CHECK_CONTIG(w);
  TORCH_CHECK(slots.scalar_type() == at::kInt && tile_expert.scalar_type() == at::kInt && slots.is_contiguous());
  TORCH_CHECK(tile == 16 || tile == 32 || tile == 64, "moe_decode_gemm: tile in {16, 32, 64}");
  const long nslots = slots.numel();
  TORCH_CHECK(nslots % tile == 0 && tile_expert.numel() * tile >= nslots, "moe_decode_gemm: tiles");
  const int E = w.size(0);
  const long K = x.size(1);
  const long estride = packed ? (N + 127) / 128 * 128 * K : N * K;
  TORCH_CHECK(w.numel() == E * estride, "moe_decode_gemm: weight size != E * (packed) N * K");
  TORCH_CHECK(K % 256 == 0 && splits >= 1 && K % (256 * splits) == 0 && x.stride(0) % 8 == 0,
              "moe_decode_gemm: K must be a multiple of 256 * splits");
  TORCH_CHECK(gather_k > 0 || x.size(0) >= nslots, "moe_decode_gemm: ungathered x needs one row per slot");
  float* ws = nullptr;
  if (out.scalar_type() == at::kFloat) {
    TORCH_CHECK(!glu && out.is_contiguous() && out.numel() >= splits * nslots * N && N % 4 == 0,
                "moe_decode_gemm: fp32 partials [splits, slots, N]");
    ws = out.data_ptr<float>();
  } else {
    CHECK_BF16(out); CHECK_ROWMAJOR(out);
    TORCH_CHECK(splits == 1 && out.size(0) >= nslots && out.size(1) >= (glu ? N / 2 : N) && out.stride(0) % 4 == 0,
                "moe_decode_gemm: bf16 out [slots, N] (glu: [slots, N/2]) needs splits == 1");
    TORCH_CHECK(!glu || N % 128 == 0, "moe_decode_gemm: glu needs N % 128 == 0");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  TORCH_CHECK(hipserve::launch_moe_decode_gemm(out.data_ptr(), out.dim() == 2 ? out.stride(0) : N, ws, x.data_ptr(),
                                               x.stride(0), w.data_ptr(), estride, slots.data_ptr<int>(),
                                               tile_expert.data_ptr<int>(), nslots / tile, tile, gather_k, N, K,
                                               splits, packed, glu, cur_stream()),
              "moe_decode_gemm: unsupported K / splits (K / splits / 256 in {1,2,3,4,6,7,8,16}) or glu without packing");
}

void moe_combine_partial(at::Tensor& out, const at::Tensor& ws, const at::Tensor& w, const at::Tensor& pair_slot,
                         int64_t k) {
  CHECK_DEV(ws); CHECK_BF16(out); CHECK_CONTIG(out);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.dim() == 3 && ws.is_contiguous(), "ws [S, slots, H] fp32");
  TORCH_CHECK(w.scalar_type() == at::kFloat && pair_slot.scalar_type() == at::kInt);
  const int T = out.size(0), H = out.size(1);
  TORCH_CHECK(ws.size(2) == H && H % 8 == 0 && w.numel() >= T * k && pair_slot.numel() >= T * k);
  c10::hip::HIPGuardMasqueradingAsCUDA g(ws.device());
  hipserve::launch_moe_combine_partial(out.data_ptr(), ws.data_ptr<float>(), ws.stride(0), ws.size(0),
                                       w.data_ptr<float>(), pair_slot.data_ptr<int>(), T, k, H, cur_stream());
}

// moe_combine(_partial) + fused_add_rmsnorm in one launch (decode MoE tail, TP = 1):
// y bf16 [slots, H] (splits 0) or fp32 partials [splits, slots, H]; out = RMSNorm(residual
// += combine) * norm_w
void moe_combine_add_rmsnorm(at::Tensor& out, at::Tensor& residual, const at::Tensor& y, int64_t splits,
                             const at::Tensor& w, const at::Tensor& pair_slot, int64_t k, const at::Tensor& norm_w,
                             double eps) {
  CHECK_DEV(y); CHECK_BF16(out); CHECK_BF16(residual); CHECK_CONTIG(out); CHECK_CONTIG(residual); CHECK_CONTIG(y);
  TORCH_CHECK(w.scalar_type() == at::kFloat && pair_slot.scalar_type() == at::kInt);
  const int T = out.size(0), H = out.size(1);
  TORCH_CHECK(residual.sizes() == out.sizes() && H % 8 == 0 && H <= 16384 && w.numel() >= T * k &&
              pair_slot.numel() >= T * k, "moe_combine_add_rmsnorm: shapes");
  TORCH_CHECK(norm_w.numel() == H && norm_w.is_contiguous() &&
              (norm_w.scalar_type() == at::kBFloat16 || norm_w.scalar_type() == at::kFloat));
  long slab = 0;
  if (splits > 0) {
    TORCH_CHECK(y.scalar_type() == at::kFloat && y.dim() == 3 && y.size(0) >= splits && y.size(2) == H,
                "moe_combine_add_rmsnorm: partials [S, slots, H] fp32");
    slab = y.stride(0);
  } else {
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 2 && y.size(1) == H, "moe_combine_add_rmsnorm: y [slots, H]");
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(y.device());
  hipserve::launch_moe_combine_add_rmsnorm(out.data_ptr(), residual.data_ptr(), y.data_ptr(), slab, (int)splits,
                                           w.data_ptr<float>(), pair_slot.data_ptr<int>(), T, k, H, norm_w.data_ptr(),
                                           norm_w.scalar_type() == at::kFloat, (float)eps, cur_stream());
}

// ---- vision tower (vision.hip)
void layernorm(at::Tensor& out, const at::Tensor& x, const at::Tensor& w, const at::Tensor& b,
               const c10::optional<at::Tensor>& residual, double eps) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_CONTIG(x); CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && out.sizes() == x.sizes(), "layernorm: x, out [rows, C]");
  const int C = x.size(1);
  TORCH_CHECK(C % 8 == 0 && C <= 8192, "layernorm: C must be a multiple of 8, <= 8192");
  TORCH_CHECK(w.numel() == C && b.numel() == C && w.scalar_type() == at::kBFloat16 &&
              b.scalar_type() == at::kBFloat16 && w.is_contiguous() && b.is_contiguous(),
              "layernorm: bf16 weight and bias [C]");
  void* r = nullptr;
  if (residual.has_value()) {
    CHECK_BF16((*residual)); CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->sizes() == x.sizes(), "layernorm: residual [rows, C]");
    r = residual->data_ptr();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_layernorm(out.data_ptr(), r, x.data_ptr(), w.data_ptr(), b.data_ptr(), x.size(0), C, (float)eps,
                             cur_stream());
}

void gelu_(at::Tensor& x, bool tanh_approx) {
  CHECK_DEV(x); CHECK_BF16(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "gelu_: numel must be a multiple of 8");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  hipserve::launch_gelu(x.data_ptr(), x.numel(), tanh_approx, cur_stream());
}

void vision_attention(at::Tensor& out, at::Tensor& qkv, const at::Tensor& cos_sin, const at::Tensor& cu,
                      const at::Tensor& tiles, int64_t nh, int64_t D, double scale) {
  CHECK_DEV(qkv); CHECK_BF16(qkv); CHECK_BF16(out); CHECK_CONTIG(qkv); CHECK_CONTIG(out);
  TORCH_CHECK(D == 16 || D == 64 || D == 72 || D == 80 || D == 96 || D == 128,
              "vision_attention: head_dim must be one of 16, 64, 72, 80, 96, 128");
  const int T = qkv.size(0);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) == 3 * nh * D, "vision_attention: qkv [T, 3 * nh * D]");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == T && out.size(1) == nh * D, "vision_attention: out [T, nh * D]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() && cos_sin.dim() == 2 &&
              cos_sin.size(0) >= T && cos_sin.size(1) == D, "vision_attention: fp32 cos_sin [T, D]");
  TORCH_CHECK(cu.scalar_type() == at::kInt && tiles.scalar_type() == at::kInt && tiles.dim() == 2 &&
              tiles.size(1) == 2 && cu.is_contiguous() && tiles.is_contiguous(),
              "vision_attention: int32 cu_seqlens and tiles [n, 2]");
  c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  hipserve::launch_vision_attention(out.data_ptr(), qkv.data_ptr(), cos_sin.data_ptr<float>(), cu.data_ptr<int>(),
                                    tiles.data_ptr<int>(), tiles.size(0), T, nh, D, (float)scale, cur_stream());
}

}  // namespace

TORCH_LIBRARY(hipserve, m) {
  m.def("moe_topk_softmax(Tensor(a!) w, Tensor(b!) ids, Tensor logits, int k, bool renorm=True, int splits=0) -> ()");
  m.def("moe_combine_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor y, int splits, Tensor w, Tensor pair_slot, int k, Tensor norm_w, float eps) -> ()");
  m.def("moe_align(Tensor ids, int E, int tile, Tensor(a!) slots, Tensor(b!) tile_expert, Tensor(c!) num_tiles, Tensor(d!) pair_slot, Tensor(e!)? group_end=None) -> ()");
  m.def("moe_gather(Tensor(a!) out, Tensor x, Tensor slots, int k) -> ()");
  m.def("moe_gemm(Tensor(a!) out, Tensor x, Tensor w, Tensor slots, Tensor tile_expert, int tile, int gather_k) -> ()");
  m.def("moe_combine(Tensor(a!) out, Tensor y, Tensor w, Tensor pair_slot, int k) -> ()");
  m.def("moe_decode_gemm(Tensor(a!) out, Tensor x, Tensor w, Tensor slots, Tensor tile_expert, int tile, int gather_k, int N, int splits, bool packed, bool glu) -> ()");
  m.def("moe_combine_partial(Tensor(a!) out, Tensor ws, Tensor w, Tensor pair_slot, int k) -> ()");
  m.def("rmsnorm(Tensor(a!) out, Tensor x, Tensor weight, float eps, Tensor(b!)? out8=None, Tensor(c!)? xs8=None) -> ()");
  m.def("embed_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor table, Tensor ids, Tensor? src, Tensor? tok, "
        "Tensor weight, float eps, float scale=1.0, Tensor(c!)? out8=None, Tensor(d!)? xs8=None) -> ()");
  m.def("fused_add_rmsnorm(Tensor(a!) out, Tensor x, Tensor(b!) residual, Tensor weight, float eps, Tensor(c!)? out8=None, Tensor(d!)? xs8=None) -> ()");
  m.def("silu_and_mul(Tensor(a!) out, Tensor x) -> ()");
  m.def("rope_cache(Tensor(a!) qkv, Tensor positions, Tensor slots, Tensor cos_sin, Tensor(b!) k_cache, Tensor(c!) v_cache, int nq, int nkv, int head_dim, int mode) -> ()");
  m.def("paged_decode(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor context_lens, Tensor(b!) tmp_out, Tensor(c!) tmp_ml, int nq, int nkv, int part_size, float scale, int window=0, Tensor(d!)? out16=None) -> ()");
  m.def("prefill_attention(Tensor(a!) out, Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor cu_q, Tensor ctx_lens, Tensor tiles, int nq, int nkv, float scale, int window=0) -> ()");
  m.def("qk_rmsnorm(Tensor(a!) qkv, Tensor q_w, Tensor k_w, int nq, int nkv, int head_dim, float eps) -> ()");
  m.def("gelu_and_mul(Tensor(a!) out, Tensor x) -> ()");
  m.def("gguf_gemm(Tensor(a!) out, Tensor x, Tensor q, Tensor d, Tensor m, int qtype, int row_bytes, int N, int K, Tensor(b!) ws, int splits) -> ()");
  m.def("gguf_dequant(Tensor(a!) out, Tensor q, Tensor d, Tensor m, int qtype, int row_bytes, int N, int K) -> ()");
  // custom all-reduce control ops carry an opaque state handle: catch-all kernels
  m.def("gguf_gemm_parts(Tensor(a!) out, Tensor(b!) ws, Tensor x, Tensor[] qs, Tensor[] rss, int[] qtypes, int[] rows, int[] cols, int Ntot, int K, int splits, Tensor? x16=None) -> int", &gguf_gemm_parts);
  m.def("gguf_prefill(Tensor(a!) out, Tensor x16, Tensor rsc, Tensor[] qs, int[] qtypes, int[] rows, int[] cols, int K, int epi) -> bool", &gguf_prefill);
  m.def("x_f16_pairs(Tensor(a!) x16, Tensor(b!) rsc, Tensor x) -> ()", &x_f16_pairs);
  m.def("gguf_dequant_tiled(Tensor(a!) out, Tensor q, Tensor rs, int qtype, int N, int K, int pack=0, int nrows=0, bool kmajor=False) -> ()",
        &gguf_dequant_tiled);
  m.def("fp8_untile(Tensor(a!) out, Tensor q, int N, int K) -> ()", &fp8_untile);
  m.def("qmoe_gemm(Tensor(a!) out, Tensor(b!) ws, Tensor x, Tensor q, Tensor rs, int qtype, int N, int K, Tensor slots, Tensor tile_expert, int tile, int gather_k, int splits, bool kmajor=False, int glu=0) -> int", &qmoe_gemm);
  m.def("car_create(int rank, int world, int max_bytes, int nb_large=512) -> int", &car_create);
  m.def("car_handle(int state) -> Tensor", &car_handle);
  m.def("car_open(int state, int peer, Tensor handle) -> ()", &car_open);
  m.def("car_all_reduce(int state, Tensor inp, Tensor(a!) out, bool two_shot) -> ()", &car_all_reduce);
  m.def("car_all_gather(int state, Tensor inp, Tensor(a!) out) -> ()", &car_all_gather);
  m.def("car_norm_fits(int state, int M, int N, bool exch_f32) -> bool", &car_norm_fits);
  m.def("car_add_rmsnorm(int state, Tensor(a!) out, Tensor(b!) residual, Tensor x, int splits, Tensor weight, float eps, bool exch_f32) -> ()", &car_add_rmsnorm);
  m.def("car_error(int state) -> bool", &car_error);
  m.def("car_destroy(int state) -> ()", &car_destroy);
  m.def("fill_uniform(Tensor(a!) out, int row0, int col0, int gcols, int key, float scale) -> ()");
  m.def("stage_copy(Tensor(a!)[] dst, Tensor[] src, int device) -> ()", &stage_copy);
  m.def("decode_gemm(Tensor(a!) out, Tensor x, Tensor w, Tensor(b!) ws, int rt, int splits) -> ()");
  m.def("decode_gemm_packed(Tensor(a!) out, Tensor x, Tensor wp, Tensor(b!) ws, int N, int rt, int splits) -> ()");
  m.def("pack_decode_weight(Tensor(a!) out, Tensor w, bool glu=False) -> ()");
  m.def("decode_gemm_partial(Tensor(a!) ws, Tensor x, Tensor w, int N, int rt, int splits, bool packed) -> ()");
  m.def("decode_gemm_glu(Tensor(a!) act, Tensor x, Tensor wp, Tensor(b!) ws, int N, int rt, int splits) -> ()");
  m.def("prefill_gemm_packed(Tensor(a!) out, Tensor x, Tensor wp, int N, int epi, Tensor? bias=None, int wm=1, int grid=0, int rw=4) -> ()");
  m.def("prefill_gemm_packed_grouped(Tensor(a!) out, Tensor x, Tensor wp, int N, int epi, Tensor tile_expert, Tensor num_tiles, int wm=1, int rw=4, Tensor? gather_slots=None, int gather_k=1) -> ()");
  m.def("prefill_gemm_f8(Tensor(a!) out, Tensor xq, Tensor xs, Tensor[] q, Tensor[] rs, int epi) -> ()");
  m.def("fp8_decode_gemm(Tensor(a!) ws, Tensor xq, Tensor xs, Tensor[] q, Tensor[] rs, int splits) -> ()");
  m.def("glu_quant(Tensor(a!)? out, Tensor(b!) q8, Tensor(c!) xs, Tensor x, bool gelu) -> ()");
  m.def("act_quant_fp8(Tensor(a!) xq, Tensor(b!) xs, Tensor x) -> ()");
  m.def("splitk_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor ws, int splits, Tensor weight, float eps, Tensor(c!)? out16=None, Tensor(d!)? out8=None, Tensor(e!)? xs8=None) -> ()");
  m.def("splitk_post_add_rmsnorm(Tensor(a!) out, Tensor(b!) residual, Tensor ws, int splits, Tensor w_post, Tensor w_next, float eps, Tensor(c!)? out16=None, Tensor(d!)? out8=None, Tensor(e!)? xs8=None) -> ()");
  m.def("splitk_glu(Tensor(a!) act, Tensor ws, int splits, bool gelu, Tensor(b!)? act16=None) -> ()");
  m.def("paged_decode_qkv(Tensor(a!) out, Tensor ws, int splits, Tensor positions, Tensor slots, Tensor cos_sin, Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor block_tables, Tensor context_lens, Tensor(d!) tmp_out, Tensor(e!) tmp_ml, int nq, int nkv, int part_size, float scale, int window, int mode, Tensor(f!)? out16=None, Tensor? q_norm=None, Tensor? k_norm=None, float eps=1e-6) -> ()");
  m.def("splitk_reduce(Tensor(a!) out, Tensor ws, int splits) -> ()");
  m.def("splitk_rope_cache(Tensor(a!) qkv, Tensor ws, int splits, Tensor positions, Tensor slots, Tensor cos_sin, Tensor(b!) k_cache, Tensor(c!) v_cache, int nq, int nkv, int head_dim, int mode, Tensor? bias=None, Tensor? q_w=None, Tensor? k_w=None, float eps=1e-6) -> ()");
  m.def("skinny_gemm(Tensor(a!) out, Tensor x, Tensor w, int rt, int kw) -> ()");
  m.def("penalty_apply(Tensor(a!) logits, Tensor slot, Tensor pres, Tensor freq, Tensor rep, Tensor counts, Tensor seen) -> ()");
  m.def("penalty_update(Tensor tok, Tensor slot, Tensor(a!) counts, Tensor(b!) seen) -> ()");
  m.def("penalty_init(Tensor(a!) counts, Tensor(b!) seen, Tensor slots, Tensor off, Tensor n_prompt, Tensor toks) -> ()");
  m.def("top_logprobs(Tensor logits, Tensor nreq, Tensor(a!) out_ids, Tensor(b!) out_lp) -> ()");
  m.def("layernorm(Tensor(a!) out, Tensor x, Tensor w, Tensor b, Tensor(b!)? residual, float eps) -> ()");
  m.def("gelu_(Tensor(a!) x, bool tanh_approx) -> ()");
  m.def("vision_attention(Tensor(a!) out, Tensor(b!) qkv, Tensor cos_sin, Tensor cu, Tensor tiles, int nh, int D, float scale) -> ()");
  m.def("sample(Tensor(a!) out_tok, Tensor(b!) out_lp, Tensor logits, Tensor temperature, Tensor top_k, Tensor top_p, Tensor seeds, Tensor steps, bool two_rounds=True) -> ()");
}

TORCH_LIBRARY_IMPL(hipserve, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("embed_rmsnorm", &embed_rmsnorm);
  m.impl("layernorm", &layernorm);
  m.impl("gelu_", &gelu_);
  m.impl("vision_attention", &vision_attention);
  m.impl("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.impl("silu_and_mul", &silu_and_mul);
  m.impl("gelu_and_mul", &gelu_and_mul);
  m.impl("qk_rmsnorm", &qk_rmsnorm);
  m.impl("rope_cache", &rope_cache);
  m.impl("paged_decode", &paged_decode);
  m.impl("prefill_attention", &prefill_attention);
  m.impl("sample", &sample);
  m.impl("penalty_apply", &penalty_apply);
  m.impl("penalty_update", &penalty_update);
  m.impl("penalty_init", &penalty_init);
  m.impl("top_logprobs", &top_logprobs);
  m.impl("gguf_gemm", &gguf_gemm);
  m.impl("skinny_gemm", &skinny_gemm);
  m.impl("decode_gemm", &decode_gemm);
  m.impl("decode_gemm_packed", &decode_gemm_packed);
  m.impl("pack_decode_weight", &pack_decode_weight);
  m.impl("decode_gemm_partial", &decode_gemm_partial);
  m.impl("decode_gemm_glu", &decode_gemm_glu);
  m.impl("prefill_gemm_packed", &prefill_gemm_packed);
  m.impl("prefill_gemm_packed_grouped", &prefill_gemm_packed_grouped);
  m.impl("prefill_gemm_f8", &prefill_gemm_f8);
  m.impl("splitk_post_add_rmsnorm", &splitk_post_add_rmsnorm);
  m.impl("act_quant_fp8", &act_quant_fp8);
  m.impl("fp8_decode_gemm", &fp8_decode_gemm);
  m.impl("glu_quant", &glu_quant);
  m.impl("splitk_add_rmsnorm", &splitk_add_rmsnorm);
  m.impl("splitk_rope_cache", &splitk_rope_cache);
  m.impl("splitk_glu", &splitk_glu);
  m.impl("paged_decode_qkv", &paged_decode_qkv);
  m.impl("splitk_reduce", &splitk_reduce);
  m.impl("fill_uniform", &fill_uniform);
  m.impl("moe_topk_softmax", &moe_topk_softmax);
  m.impl("moe_combine_add_rmsnorm", &moe_combine_add_rmsnorm);
  m.impl("moe_align", &moe_align);
  m.impl("moe_gather", &moe_gather);
  m.impl("moe_gemm", &moe_gemm);
  m.impl("moe_combine", &moe_combine);
  m.impl("moe_decode_gemm", &moe_decode_gemm);
  m.impl("moe_combine_partial", &moe_combine_partial);
  m.impl("gguf_dequant", &gguf_dequant);
}
