"""fp8 (e4m3) paged KV cache (--kv-cache-dtype fp8) on the gfx950 kernels.

Writers (rope_cache per-token / 16-token tile kernels, the decode layer's
splitk_rope_cache) must store exactly the e4m3 rounding of what the bf16 kernels store
(saturating RNE, per-tensor scale 1: ``reference.to_cache``); readers (paged decode,
prefill attention v1 / v2) widen e4m3 -> bf16 exactly, so they are checked against the
fp32 oracle run over the same e4m3 cache. vLLM semantics: ``--kv-cache-dtype fp8``
without calibrated scales."""
import math

import pytest
import torch

from hipserve.ops import KernelOps
from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
F8 = torch.float8_e4m3fn


@pytest.fixture(scope="module")
def ops():
    return KernelOps()


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    bad = (a - b).abs() > (atol + rtol * b.abs())
    assert not bad.any(), f"max err {(a - b).abs().max().item()}"


def _f8_caches(nblocks, nkv, bs, D, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(nblocks + bs + D)
    kc = ref.to_cache(torch.randn(nblocks, nkv, bs, D, device=DEV, generator=g) * scale, F8)
    vc = ref.to_cache(torch.randn(nblocks, nkv, D, bs, device=DEV, generator=g) * scale, F8)
    return kc, vc


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("T,layout", [(37, "random"), (300, "random"), (2500, "contig"), (2100, "aligned")])
def test_rope_cache_fp8_is_rounded_bf16(ops, mode, bs, T, layout):
    """e4m3 cache = to_cache(the bf16 kernel's cache), byte for byte; q identical. Values
    up to ~600 so the +-448 saturation is exercised."""
    torch.manual_seed(1)
    nq, nkv, D = 32, 8, 128
    qkv = (torch.randn(T, (nq + 2 * nkv) * D, device=DEV) * 150).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV)
    nb = max(64, (T + 2 * bs) // bs + 1)
    slots = torch.randperm(nb * bs, device=DEV)[:T] if layout == "random" else \
        torch.arange(T, device=DEV) + (5 if layout == "contig" else bs)
    slots[3] = -1
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    kb = torch.zeros(nb, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vb = torch.zeros(nb, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    k8 = torch.zeros(nb, nkv, bs, D, device=DEV, dtype=F8)
    v8 = torch.zeros(nb, nkv, D, bs, device=DEV, dtype=F8)
    q_b, q_8 = qkv.clone(), qkv.clone()
    ops.rope_cache(q_b, pos, slots, cs, kb, vb, nq, nkv, D, mode)
    ops.rope_cache(q_8, pos, slots, cs, k8, v8, nq, nkv, D, mode)
    assert torch.equal(q_b[:, : nq * D], q_8[:, : nq * D])
    assert torch.equal(k8.view(torch.uint8), ref.to_cache(kb, F8).view(torch.uint8))
    assert torch.equal(v8.view(torch.uint8), ref.to_cache(vb, F8).view(torch.uint8))
    assert (kb.float().abs() > 448).any()  # saturation exercised


@pytest.mark.parametrize("T,S", [(1, 1), (37, 4), (64, 3)])
@pytest.mark.parametrize("mode", [0, 1])
def test_splitk_rope_cache_fp8_is_rounded_bf16(T, S, mode):
    torch.manual_seed(2)
    nq, nkv, D, bs = 32, 8, 128, 16
    N = (nq + 2 * nkv) * D
    ws = torch.randn(S, T, N, device=DEV) * 40
    pos = torch.randint(0, 4000, (T,), device=DEV)
    slots = torch.randperm(32 * bs, device=DEV)[:T]
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    outs = {}
    for dt in (torch.bfloat16, F8):
        kc = torch.zeros(32, nkv, bs, D, device=DEV, dtype=dt)
        vc = torch.zeros(32, nkv, D, bs, device=DEV, dtype=dt)
        qkv = torch.empty(T, N, device=DEV, dtype=torch.bfloat16)
        torch.ops.hipserve.splitk_rope_cache(qkv, ws, S, pos, slots, cs, kc, vc, nq, nkv, D, mode)
        outs[dt] = (qkv, kc, vc)
    assert torch.equal(outs[F8][0][:, : nq * D], outs[torch.bfloat16][0][:, : nq * D])
    for i in (1, 2):
        assert torch.equal(outs[F8][i].view(torch.uint8), ref.to_cache(outs[torch.bfloat16][i], F8).view(torch.uint8))


@pytest.mark.parametrize("nq,nkv,D", [(32, 8, 128), (32, 16, 128), (32, 32, 64), (32, 32, 96)])
@pytest.mark.parametrize("part", [512, 2048])
@pytest.mark.parametrize("window", [0, 100])
def test_paged_decode_fp8_cache(ops, nq, nkv, D, part, window):
    torch.manual_seed(3)
    bs = 16
    ctx = [1, 17, 100, 600, 1300, 512, 33]
    B, max_blocks = len(ctx), 96
    kc, vc = _f8_caches(B * max_blocks, nkv, bs, D)
    bt = torch.randperm(B * max_blocks, device=DEV).int().view(B, max_blocks).contiguous()
    cl = torch.tensor(ctx, device=DEV, dtype=torch.int32)
    q = torch.randn(B, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
    max_parts = math.ceil(max_blocks * bs / part)
    tmp_out = torch.empty(B, nq, max_parts, D, device=DEV)
    tmp_ml = torch.empty(B, nq, max_parts, 2, device=DEV)
    out = torch.zeros(B, nq * D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    ops.paged_decode(out, q, kc, vc, bt, cl, tmp_out, tmp_ml, nq, nkv, part, scale, window)
    want = ref.paged_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cl.cpu(), nq, nkv, scale, window)
    _close(out.view(B, nq, D), want, atol=2e-2, rtol=2e-2)
    # the same cache widened to bf16 through the bf16 kernel: the same values; at head_dim 96
    # the e4m3 kernel also keeps the bf16 kernel's chunking, so the sums match bit for bit
    # (64 / 128 stream 64-key chunks: another fp32 summation order)
    out_b = torch.zeros_like(out)
    ops.paged_decode(out_b, q, kc.to(torch.bfloat16), vc.to(torch.bfloat16), bt, cl, tmp_out, tmp_ml, nq, nkv,
                     part, scale, window)
    if D == 96:
        assert torch.equal(out, out_b)
    else:
        _close(out, out_b, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("nq,nkv,D,v1", [(32, 8, 128, False), (32, 8, 128, True), (8, 1, 128, False),
                                         (16, 2, 64, False), (8, 8, 96, False)])
@pytest.mark.parametrize("window", [0, 200])
def test_prefill_attention_fp8_cache(ops, nq, nkv, D, v1, window, monkeypatch):
    monkeypatch.setenv("HIPSERVE_PREFILL_ATTN_V1", "1" if v1 else "0")
    torch.manual_seed(4)
    bs = 16
    seqs = [(1, 1), (37, 37), (300, 50), (1100, 1100), (1500, 333)]
    max_blocks = 1536 // bs
    kc, vc = _f8_caches(len(seqs) * max_blocks, nkv, bs, D)
    bt = torch.randperm(len(seqs) * max_blocks, device=DEV).int().view(len(seqs), max_blocks).contiguous()
    cu, tiles = [0], []
    for i, (c, ql) in enumerate(seqs):
        tiles += [(i, r) for r in range(0, ql, 128)]
        cu.append(cu[-1] + ql)
    T = cu[-1]
    q = torch.randn(T, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16) * 2
    cu_t = torch.tensor(cu, device=DEV, dtype=torch.int32)
    ctx_t = torch.tensor([c for c, _ in seqs], device=DEV, dtype=torch.int32)
    tiles_t = torch.tensor(tiles, device=DEV, dtype=torch.int32)
    out = torch.zeros(T, nq * D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    ops.prefill_attention(out, q, kc, vc, bt, cu_t, ctx_t, tiles_t, nq, nkv, scale, window)
    want = ref.prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu_t.cpu(), ctx_t.cpu(), nq, nkv, scale,
                                 window)
    _close(out.view(T, nq, D), want, atol=2e-2, rtol=2e-2)
    out_b = torch.zeros_like(out)
    ops.prefill_attention(out_b, q, kc.to(torch.bfloat16), vc.to(torch.bfloat16), bt, cu_t, ctx_t, tiles_t, nq, nkv,
                          scale, window)
    assert torch.equal(out, out_b)


def test_engine_fp8_kv_cache_graph_equals_eager():
    """Llama-3 architecture (2 layers) with an e4m3 cache: twice the KV blocks of the bf16
    cache in the same memory, hipGraph decode == eager decode token for token."""
    from hipserve.config import EngineConfig, PRESETS
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    dev = torch.device("cuda", 0)
    mcfg = PRESETS["llama-3-8b"].replace(name="llama-3-kvf8", num_layers=2, hidden_size=1024,
                                         intermediate_size=3584, num_heads=8, num_kv_heads=2,
                                         vocab_size=32000, max_position_embeddings=2048)
    prompts = [[1] + list(range(100, 400)), [1, 5, 6, 7], list(range(50, 90))]
    sp = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
    toks, bpb = {}, {}
    for kvd, eager in (("fp8", False), ("fp8", True), ("auto", False)):
        cfg = EngineConfig(model="llama-3-kvf8", load_format="dummy", device="cuda", max_num_seqs=8,
                           max_num_batched_tokens=256, max_model_len=1024, num_kv_blocks=256,
                           enforce_eager=eager, kv_cache_dtype=kvd)
        eng = LLMEngine(cfg, tp=TPGroup(0, 1, None, dev), model_cfg=mcfg)
        if kvd == "fp8":
            assert eng.runner.kv[0][0].dtype == F8
        bpb[kvd] = eng.runner.model.kv_bytes_per_block(16)
        toks[(kvd, eager)] = [r[0] for r in eng.generate(prompts, sp)]
        assert (eng.runner.stats["graph_steps"] > 0) != eager
        eng.shutdown()
        del eng
        torch.cuda.synchronize()
    assert toks[("fp8", False)] == toks[("fp8", True)]
    assert bpb["fp8"] * 2 == bpb["auto"]
    # the bf16 cache's first (prefill) token should mostly survive the K / V rounding
    same = sum(a[0] == b[0] for a, b in zip(toks[("fp8", False)], toks[("auto", False)]))
    assert same >= 2, (toks[("fp8", False)], toks[("auto", False)])
