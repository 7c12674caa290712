"""Long context (the reference's default model is the 128K
Gemma-3-27B, vllm-models/helm-chart/values.yaml:3): the attention kernels at 32K-token
contexts against the fp32 PyTorch reference — split-K paged decode with 64 partitions and
2,048-entry block tables, chunked prefill over a 32K prefix, sliding-window layers — and
the engine serving one 32K-token prompt end to end (chunked prefill vs one chunk)."""
import math

import pytest
import torch

from hipserve.ops import KernelOps
from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    return KernelOps()


def _close(a, b, atol, rtol):
    a, b = a.float(), b.float().to(a.device)
    bad = (a - b).abs() > (atol + rtol * b.abs())
    assert not bad.any(), f"max err {(a - b).abs().max().item()}"


def _caches(nblocks, nkv, bs, D):
    kc = torch.randn(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(nblocks, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    return kc, vc


@pytest.mark.parametrize("window", [0, 4096])
@pytest.mark.parametrize("part", [512, 2048])
def test_paged_decode_32k(ops, part, window):
    torch.manual_seed(21)
    nq, nkv, D, bs = 32, 8, 128, 16
    ctx = [32768, 32001, 17000, 5]
    B = len(ctx)
    max_blocks = 32768 // bs
    kc, vc = _caches(B * max_blocks, nkv, bs, D)
    bt = torch.randperm(B * max_blocks, device=DEV).int().view(B, max_blocks).contiguous()
    cl = torch.tensor(ctx, device=DEV, dtype=torch.int32)
    q = torch.randn(B, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
    max_parts = math.ceil(max_blocks * bs / part)
    tmp_out = torch.empty(B, nq, max_parts, D, device=DEV, dtype=torch.float32)
    tmp_ml = torch.empty(B, nq, max_parts, 2, device=DEV, dtype=torch.float32)
    out = torch.zeros(B, nq * D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    ops.paged_decode(out, q, kc, vc, bt, cl, tmp_out, tmp_ml, nq, nkv, part, scale, window)
    want = ref.paged_decode(q, kc, vc, bt, cl, nq, nkv, scale, window)  # fp32 math on the GPU
    _close(out.view(B, nq, D), want, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("window", [0, 4096])
def test_prefill_attention_32k_prefix(ops, window):
    """Chunks of new tokens at the end of 32K / 20K contexts (chunked prefill over a
    long prefix), plus a plain 4K prefill, in one varlen launch."""
    torch.manual_seed(22)
    nq, nkv, D, bs = 32, 8, 128, 16
    seqs = [(32768, 512), (20000, 300), (4096, 4096)]  # (context incl. the chunk, chunk length)
    max_blocks = 32768 // bs
    kc, vc = _caches(len(seqs) * max_blocks, nkv, bs, D)
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
    for s_, (c, ql) in enumerate(seqs):  # reference per sequence (bounded fp32 score matrices)
        q0, q1 = cu[s_], cu[s_ + 1]
        want = ref.prefill_attention(q[q0:q1], kc, vc, bt[s_:s_ + 1], torch.tensor([0, ql], device=DEV),
                                     ctx_t[s_:s_ + 1], nq, nkv, scale, window)
        _close(out[q0:q1].view(ql, nq, D), want, atol=2e-2, rtol=2e-2)


def test_engine_serves_32k_prompt():
    """One 32,000-token prompt through the engine: chunked prefill (4 chunks of 8,192
    over a growing prefix) vs one 32K chunk — first-token logits agree to bf16 noise and
    the greedy continuation (decode steps over a 32K context, hipGraph) matches."""
    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    prompt = torch.randint(3, 2000, (32000,), generator=torch.Generator().manual_seed(5)).tolist()

    def run(budget):
        cfg = EngineConfig(model="small-llama-long", device="cuda", dtype="bfloat16", max_num_seqs=4,
                           max_num_batched_tokens=budget, max_model_len=33000, num_kv_blocks=2200)
        eng = LLMEngine(cfg, tp=TPGroup(0, 1, None, torch.device("cuda", 0)))
        m = eng.runner.model
        logits = []
        orig = m.compute_logits

        def cap(h):
            out = orig(h)
            logits.append(out.float().clone())
            return out

        m.compute_logits = cap
        toks = eng.generate([prompt], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))[0][0]
        return toks, logits[0][-1], eng.runner.stats

    t_chunk, l_chunk, st = run(8192)
    t_one, l_one, _ = run(33000)
    assert len(t_chunk) == 8 and st["graph_steps"] >= 6
    err = (l_chunk - l_one).abs().max().item()
    assert err <= 0.05 * max(1.0, l_one.std().item()), err
    assert t_chunk[0] == t_one[0]
    assert sum(a == b for a, b in zip(t_chunk, t_one)) >= 6, (t_chunk, t_one)
