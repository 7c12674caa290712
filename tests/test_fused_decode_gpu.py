"""Fused decode epilogues (csrc/kernels/decode_fused.hip + decode_gemm.hip partial
/ silu-x modes) must be BIT-identical to the unfused chains they replace, and the
fused decode forward of the model bit-identical to the unfused forward."""
import math

import pytest
import torch

from hipserve.ops import KernelOps, gemm
from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    return KernelOps()


def _partials(S, M, N, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(S, M, N, device=DEV, generator=g) * 0.5


@pytest.mark.parametrize("M,H", [(1, 4096), (64, 4096), (37, 2048), (8, 8192), (3, 1024), (64, 5376)])
@pytest.mark.parametrize("wf32", [False, True])
@pytest.mark.parametrize("lookahead", [False, True])
@pytest.mark.parametrize("scale", [1.0, 5376 ** 0.5])
def test_embed_rmsnorm_bit_exact(ops, M, H, wf32, lookahead, scale):
    """embed_rmsnorm (norm.hip gather mode) == id select + F.embedding (* the Gemma
    embedding scale, rounded to bf16) + clone + rmsnorm, bit for bit; with lookahead,
    rows with src >= 0 take tok[src]. Its e4m3 copy == act_quant_fp8 of the output."""
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M * 7 + H)
    V = 5000
    table = torch.randn(V, H, device=DEV, dtype=torch.bfloat16, generator=g)
    w = (torch.rand(H, device=DEV, generator=g) + 0.5)
    w = w if wf32 else w.to(torch.bfloat16)
    ids = torch.randint(0, V, (M,), device=DEV, generator=g)
    src = tok = None
    want_ids = ids
    if lookahead:
        tok = torch.randint(0, V, (80,), device=DEV, generator=g)
        src = torch.randint(-1, 80, (M,), device=DEV, generator=g)
        want_ids = torch.where(src >= 0, tok.index_select(0, src.clamp(min=0)), ids)
    sc = float(torch.tensor(scale, dtype=torch.bfloat16))
    h = torch.nn.functional.embedding(want_ids, table)
    if scale != 1.0:
        h = h * sc
    want = torch.empty_like(h)
    ops.rmsnorm(want, h, w, 1e-5)
    out = torch.full_like(h, float("nan"))
    res = torch.full_like(h, float("nan"))
    q8 = torch.empty(M, H, device=DEV, dtype=torch.uint8)
    s8 = torch.empty(M, device=DEV, dtype=torch.float32)
    torch.ops.hipserve.embed_rmsnorm(out, res, table, ids, src, tok, w, 1e-5, sc, q8, s8)
    assert torch.equal(res, h)
    assert torch.equal(out, want)
    xq, xs = pgemm.act_quant(out)
    assert torch.equal(q8, xq) and torch.equal(s8, xs)


@pytest.mark.parametrize("S,M,N", [(1, 5, 4096), (4, 64, 4096), (8, 17, 2048), (3, 1, 8192)])
@pytest.mark.parametrize("wf32", [False, True])
def test_splitk_add_rmsnorm_bit_exact(ops, S, M, N, wf32):
    ws = _partials(S, M, N, S * 100 + M)
    res0 = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, device=DEV, dtype=torch.float32 if wf32 else torch.bfloat16)
    # unfused: reduce -> bf16, fused add + rmsnorm
    h = ws[0].clone()
    for s in range(1, S):
        h = h + ws[s]
    h = h.to(torch.bfloat16)
    r1, o1 = res0.clone(), torch.empty_like(res0)
    ops.fused_add_rmsnorm(o1, h, r1, w, 1e-5)
    r2, o2 = res0.clone(), torch.empty_like(res0)
    torch.ops.hipserve.splitk_add_rmsnorm(o2, r2, ws.contiguous(), S, w, 1e-5)
    assert torch.equal(r1, r2) and torch.equal(o1, o2)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("S", [1, 4])
def test_splitk_rope_cache_bit_exact(ops, mode, S):
    T, nq, nkv, D, bs = 23, 32, 8, 128, 16
    N = (nq + 2 * nkv) * D
    ws = _partials(S, T, N, 7 + S)
    h = ws[0].clone()
    for s in range(1, S):
        h = h + ws[s]
    qkv1 = h.to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    slots = torch.randperm(64 * bs, device=DEV)[:T]
    slots[3] = -1
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    kc1 = torch.zeros(64, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc1 = torch.zeros(64, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    kc2, vc2 = kc1.clone(), vc1.clone()
    ops.rope_cache(qkv1, pos, slots, cs, kc1, vc1, nq, nkv, D, mode)
    qkv2 = torch.zeros(T, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.splitk_rope_cache(qkv2, ws.contiguous(), S, pos, slots, cs, kc2, vc2, nq, nkv, D, mode)
    assert torch.equal(qkv1[:, : nq * D], qkv2[:, : nq * D])
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)


@pytest.mark.parametrize("M", [1, 16, 40, 64])
@pytest.mark.parametrize("rt,S", [(1, 1), (2, 1), (1, 4), (2, 2)])
def test_glu_gemm_bit_exact(ops, M, rt, S):
    """gate|up decode GEMM with the SiLU-GLU epilogue == packed GEMM + silu_and_mul."""
    I, K = 1792, 4096
    N = 2 * I
    torch.manual_seed(M + S)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    gu = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    gemm.decode_gemm_packed(gu, x, gemm.pack(w), N, rt, S)
    want = torch.empty(M, I, device=DEV, dtype=torch.bfloat16)
    ops.silu_and_mul(want, gu)
    act = gemm.gemm_glu(x, w, (rt, S, gemm.pack(w, glu=True)))
    assert torch.equal(act, want)


def _small_model(ops, seed=0, family="llama"):
    from hipserve.config import PRESETS
    from hipserve.models.llama import LlamaModel
    from hipserve.parallel.comm import TPGroup

    cfg = PRESETS["llama-3-8b"].replace(hidden_size=1024, intermediate_size=3584, num_heads=8,
                                        num_kv_heads=2, num_layers=3, vocab_size=4096,
                                        max_position_embeddings=2048)
    if family == "qwen2":
        cfg = cfg.replace(family="qwen2", qkv_bias=True)
    elif family == "qwen3":
        cfg = cfg.replace(family="qwen3", qk_norm=True)
    elif family == "gemma3":  # sandwich norms, GeGLU, local/global layers, embedding scale, q/k norm
        cfg = cfg.replace(family="gemma3", qk_norm=True, hidden_act="gelu_tanh", sandwich_norm=True,
                          norm_offset=True, embed_scale=1024 ** 0.5, attn_scale=128 ** -0.5, sliding_window=96,
                          layer_windows=(96, 0, 96), rope_local_theta=1e4, rms_norm_eps=1e-6)
    elif family == "qwen3_moe":
        cfg = cfg.replace(family="qwen3_moe", architecture="mixtral", qk_norm=True, num_experts=8,
                          num_experts_per_tok=2, moe_intermediate_size=512)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, ops, max_pos=2048)
    m.allocate_random(seed=seed, std=0.05)
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    for lw in m.layers:  # non-trivial family extras
        if lw.bqkv is not None:
            lw.bqkv = (torch.randn(lw.bqkv.shape, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
        if lw.q_norm is not None:
            lw.q_norm = 1 + 0.2 * torch.randn(lw.q_norm.shape, device=DEV, generator=g)
            lw.k_norm = 1 + 0.2 * torch.randn(lw.k_norm.shape, device=DEV, generator=g)
        if lw.post_attn_norm is not None:
            for n in ("post_attn_norm", "post_ff_norm", "ln1", "ln2"):
                t = getattr(lw, n)
                setattr(lw, n, (1 + 0.2 * torch.randn(t.shape, device=DEV, generator=g)).to(t.dtype))
    return m, cfg


@pytest.mark.parametrize("bias,norm,D", [(True, False, 128), (False, True, 128), (True, True, 64),
                                         (False, True, 64)])
@pytest.mark.parametrize("S", [1, 3])
def test_splitk_rope_cache_extras_bit_exact(ops, bias, norm, D, S):
    """split-K RoPE epilogue with the Qwen2 bias and / or Qwen3 per-head q/k RMSNorm ==
    bf16 reduce -> bias add -> qk_rmsnorm -> rope_cache."""
    T, nq, nkv, bs = 29, 16, 4, 16
    N = (nq + 2 * nkv) * D
    ws = _partials(S, T, N, 11 + S + D)
    h = ws[0].clone()
    for s in range(1, S):
        h = h + ws[s]
    qkv1 = h.to(torch.bfloat16)
    b = (torch.randn(N, device=DEV) * 0.3).to(torch.bfloat16) if bias else None
    qw = 1 + 0.2 * torch.randn(D, device=DEV) if norm else None
    kw = 1 + 0.2 * torch.randn(D, device=DEV) if norm else None
    if bias:
        qkv1 += b
    if norm:
        ops.qk_rmsnorm(qkv1, qw, kw, nq, nkv, D, 1e-6)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    slots = torch.randperm(64 * bs, device=DEV)[:T]
    slots[5] = -1
    cs = ref.rope_cos_sin(D, 4096, 1e6).to(DEV)
    kc1 = torch.zeros(64, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc1 = torch.zeros(64, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    kc2, vc2 = kc1.clone(), vc1.clone()
    ops.rope_cache(qkv1, pos, slots, cs, kc1, vc1, nq, nkv, D, 0)
    qkv2 = torch.zeros(T, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.splitk_rope_cache(qkv2, ws.contiguous(), S, pos, slots, cs, kc2, vc2, nq, nkv, D, 0,
                                         b, qw, kw, 1e-6)
    assert torch.equal(qkv1[:, : nq * D], qkv2[:, : nq * D])
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)


@pytest.mark.parametrize("family", ["qwen2", "qwen3", "qwen3_moe", "gemma3"])
def test_fused_decode_forward_families_bit_exact(ops, family):
    test_fused_decode_forward_bit_exact(ops, "dgp", family)


@pytest.mark.parametrize("choices", ["dgp", "mixed"])
def test_fused_qkv_attention_forward_bit_exact(ops, choices):
    """The decode layer with qkv partials -> RoPE + KV write + attention in one kernel
    (paged_decode_qkv) vs the unfused path."""
    test_fused_decode_forward_bit_exact(ops, choices, qkv_attn=True)


@pytest.mark.parametrize("family", ["qwen3", "qwen3_moe"])
def test_fused_qkv_attention_qk_norm_forward_bit_exact(ops, family):
    """Qwen3 decode layer with the per-head q / k norm inside the fused attention vs the
    unfused path (and the model really takes the fused kernel)."""
    test_fused_decode_forward_bit_exact(ops, "dgp", family, qkv_attn=True)


@pytest.mark.parametrize("choices", ["dgp", "dg", "mixed"])
def test_fused_decode_forward_bit_exact(ops, choices, family="llama", qkv_attn=False):
    """Model forward on a decode batch: fused epilogues vs the unfused path."""
    from hipserve.models.llama import AttnMeta

    m, cfg = _small_model(ops, family=family)
    assert m.fused_family
    m.fused_qkv_attention = qkv_attn
    if qkv_attn and family in ("llama", "qwen3", "qwen3_moe"):
        assert m.fused_qkv_attn_ok()
        m.decode_partition = 2048  # one context partition: the fused kernel's regime
    old = dict(gemm.TUNER.table)
    try:
        gemm.TUNER.table.clear()
        shapes = m.gemm_shapes()
        for (N, K) in shapes:
            kind = "dgp" if choices == "dgp" or (choices == "mixed" and N != 1024) else "dg"
            for mm in gemm.TUNE_MS:
                S = 2 if K >= 1024 else 1
                gemm.TUNER.table[(mm, N, K)] = (kind, 1, S)
        if choices == "mixed":
            for mm in gemm.TUNE_MS:  # o_proj on hipBLASLt: unfused fallback for that op
                gemm.TUNER.table[(mm, 1024, 1024)] = "blas"
        m.pack_decode_weights(set(shapes))
        B, bs, D = 24, 16, cfg.head_dim
        ctx = torch.randint(1, 300, (B,), device=DEV, dtype=torch.int32)
        nblk = 64
        bt = torch.randperm(B * nblk, device=DEV).int().view(B, nblk)
        pos = (ctx - 1).long()
        slots = (bt.gather(1, (pos // bs).view(-1, 1).int()).view(-1).long() * bs + pos % bs)
        ids = torch.randint(0, cfg.vocab_size, (B,), device=DEV)
        kv1 = m.allocate_kv_cache(B * nblk, bs)
        for kc, vc in kv1:
            kc.normal_()
            vc.normal_()
        kv2 = [(k.clone(), v.clone()) for k, v in kv1]
        parts = math.ceil(nblk * bs / 512)
        mk = lambda: AttnMeta(num_prefill_tokens=0, num_decode=B, positions=pos, slot_mapping=slots,
                              bt_decode=bt, ctx_decode=ctx,
                              tmp_out=torch.empty(B, m.nq, parts, D, device=DEV),
                              tmp_ml=torch.empty(B, m.nq, parts, 2, device=DEV))
        m.fused_decode = False
        out1 = m.forward(ids, mk(), kv1).clone()
        m.fused_decode = True
        out2 = m.forward(ids, mk(), kv2).clone()
        assert torch.equal(out1, out2)
        for (k1, v1), (k2, v2) in zip(kv1, kv2):
            assert torch.equal(k1, k2) and torch.equal(v1, v2)
    finally:
        gemm.TUNER.table.clear()
        gemm.TUNER.table.update(old)


@pytest.mark.parametrize("S,part", [(1, 512), (4, 128), (2, 2048)])
@pytest.mark.parametrize("D", [128, 64])
def test_paged_decode_qkv_qk_norm_bit_exact(ops, S, part, D):
    """Qwen3's per-head q / k RMSNorm inside the fused decode attention == splitk_rope_cache
    (norm branch) followed by paged_decode, bit for bit."""
    test_paged_decode_qkv_bit_exact(ops, 0, S, part, D, qk_norm=True)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("S,part", [(1, 512), (4, 128), (3, 256)])
@pytest.mark.parametrize("D", [128, 64])
def test_paged_decode_qkv_bit_exact(ops, mode, S, part, D, qk_norm=False):
    """Fused qkv partials -> RoPE + KV write + attention == splitk_rope_cache followed
    by paged_decode, bit for bit (output and both caches), with split contexts
    (several partitions + reduce) and a padding row (slot -1)."""
    B, nq, nkv, bs = 9, 16, 4, 16
    nw = ((torch.rand(D, device=DEV, generator=torch.Generator(device=DEV).manual_seed(D)) + 0.5),
          (torch.rand(D, device=DEV, generator=torch.Generator(device=DEV).manual_seed(D + 1)) + 0.5)) \
        if qk_norm else (None, None)
    N = (nq + 2 * nkv) * D
    ws = _partials(S, B, N, 31 + S + D)
    nblk = 40
    ctx = torch.randint(1, nblk * bs, (B,), device=DEV, dtype=torch.int32)
    ctx[0] = 1
    ctx[1] = nblk * bs
    bt = torch.randperm(B * nblk, device=DEV).int().view(B, nblk)
    pos = (ctx - 1).long()
    slots = bt.gather(1, (pos // bs).view(-1, 1).int()).view(-1).long() * bs + pos % bs
    slots[4] = -1
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    kc1 = torch.randn(B * nblk, nkv, bs, D, device=DEV).to(torch.bfloat16)
    vc1 = torch.randn(B * nblk, nkv, D, bs, device=DEV).to(torch.bfloat16)
    kc2, vc2 = kc1.clone(), vc1.clone()
    parts = math.ceil(nblk * bs / part)
    mk = lambda: (torch.empty(B, nq, parts, D, device=DEV), torch.empty(B, nq, parts, 2, device=DEV))
    scale = D ** -0.5
    qkv = torch.zeros(B, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.splitk_rope_cache(qkv, ws.contiguous(), S, pos, slots, cs, kc1, vc1, nq, nkv, D, mode,
                                         None, nw[0], nw[1], 1e-6)
    out1 = torch.empty(B, nq * D, device=DEV, dtype=torch.bfloat16)
    t1, m1 = mk()
    ops.paged_decode(out1, qkv, kc1, vc1, bt, ctx, t1, m1, nq, nkv, part, scale)
    out2 = torch.empty(B, nq * D, device=DEV, dtype=torch.bfloat16)
    t2, m2 = mk()
    torch.ops.hipserve.paged_decode_qkv(out2, ws.contiguous(), S, pos, slots, cs, kc2, vc2, bt, ctx, t2, m2,
                                        nq, nkv, part, scale, 0, mode, None, nw[0], nw[1], 1e-6)
    assert torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    assert torch.equal(out1, out2)


@pytest.mark.parametrize("scheme,family", [("q4_k_m", "llama"), ("fp8", "llama"), ("fp8", "gemma3")])
@pytest.mark.parametrize("x16", [True, False])
def test_fused_decode_forward_quantised_bit_exact(ops, scheme, family, x16):
    """Quantised model (GGUF Q4_K_M / FP8 weights) at a 48-row decode batch: the fused
    forward (quantised GEMM partials -> fused epilogues; x16 = the producers' f16
    pair-order copy of x staged by the GEMM) is bit-identical to the unfused forward."""
    from hipserve.config import PRESETS
    from hipserve.models.llama import AttnMeta, LlamaModel
    from hipserve.parallel.comm import TPGroup

    cfg = PRESETS["llama-3-8b"].replace(hidden_size=1024, intermediate_size=3584, num_heads=8, num_kv_heads=2,
                                        num_layers=3, vocab_size=4096, max_position_embeddings=2048)
    if family == "gemma3":
        cfg = cfg.replace(family="gemma3", qk_norm=True, hidden_act="gelu_tanh", sandwich_norm=True,
                          norm_offset=True, embed_scale=1024 ** 0.5, attn_scale=128 ** -0.5, sliding_window=96,
                          layer_windows=(96, 0, 96), rope_local_theta=1e4, rms_norm_eps=1e-6)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, ops, max_pos=2048)
    m.allocate_random_quant(scheme, seed=3)
    m.X16 = x16
    B, bs, D = 48, 16, cfg.head_dim
    g = torch.Generator(device=DEV).manual_seed(5)
    ctx = torch.randint(1, 300, (B,), device=DEV, dtype=torch.int32, generator=g)
    nblk = 64
    bt = torch.randperm(B * nblk, device=DEV, generator=g).int().view(B, nblk)
    pos = (ctx - 1).long()
    slots = (bt.gather(1, (pos // bs).view(-1, 1).int()).view(-1).long() * bs + pos % bs)
    ids = torch.randint(0, cfg.vocab_size, (B,), device=DEV, generator=g)
    kv1 = m.allocate_kv_cache(B * nblk, bs)
    for kc, vc in kv1:
        kc.normal_(generator=g)
        vc.normal_(generator=g)
    kv2 = [(k.clone(), v.clone()) for k, v in kv1]
    parts = math.ceil(nblk * bs / 512)
    mk = lambda: AttnMeta(num_prefill_tokens=0, num_decode=B, positions=pos, slot_mapping=slots,
                          bt_decode=bt, ctx_decode=ctx, tmp_out=torch.empty(B, m.nq, parts, D, device=DEV),
                          tmp_ml=torch.empty(B, m.nq, parts, 2, device=DEV))
    m.fused_decode = False
    out1 = m.forward(ids, mk(), kv1).clone()
    m.fused_decode = True
    assert m._fused_ok(mk())
    out2 = m.forward(ids, mk(), kv2).clone()
    assert torch.equal(out1, out2)
    for (k1, v1), (k2, v2) in zip(kv1, kv2):
        assert torch.equal(k1, k2) and torch.equal(v1, v2)
