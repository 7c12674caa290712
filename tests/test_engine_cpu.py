"""Engine plumbing on CPU (reference ops): paged/chunked/batched generation must
equal a naive dense full-recompute forward of the same weights."""
import math

import pytest
import torch
import torch.nn.functional as F

from hipserve.config import EngineConfig
from hipserve.engine.llm_engine import LLMEngine
from hipserve.engine.request import SamplingParams
from hipserve.ops import reference as ref
from hipserve.parallel.comm import TPGroup


def make_engine(model="tiny-llama", **kw):
    base = dict(model=model, device="cpu", dtype="float32", max_num_seqs=8,
                max_num_batched_tokens=48, num_kv_blocks=256, max_model_len=512)
    base.update(kw)
    return LLMEngine(EngineConfig(**base), tp=TPGroup())


def dense_logits(model, ids, kv_dtype=None):
    """Naive causal forward over the whole sequence (no KV cache); kv_dtype: round the
    rotated K and the V rows through that cache element type (fp8 KV cache oracle)."""
    cfg = model.cfg
    x = model.embed[torch.tensor(ids)].float()
    T = len(ids)
    D, nq, nkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    pos = torch.arange(T)
    for lw in model.layers:
        h = ref.rmsnorm(x, lw.ln1, cfg.rms_norm_eps)
        qkv = h @ lw.wqkv.float().T
        q = qkv[:, : nq * D].view(T, nq, D)
        k = qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)
        v = qkv[:, (nq + nkv) * D:].view(T, nkv, D)
        q = ref.apply_rope(q, pos, model.cos_sin, cfg.rope_mode)
        k = ref.apply_rope(k, pos, model.cos_sin, cfg.rope_mode)
        if kv_dtype is not None:
            k, v = ref.to_cache(k, kv_dtype).float(), ref.to_cache(v, kv_dtype).float()
        G = nq // nkv
        k, v = k.repeat_interleave(G, 1), v.repeat_interleave(G, 1)
        s = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(D)
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool), 1), float("-inf"))
        o = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v).reshape(T, nq * D)
        x = x + o @ lw.wo.float().T
        h = ref.rmsnorm(x, lw.ln2, cfg.rms_norm_eps)
        if lw.router is not None:
            logits = h @ lw.router.float().T
            w, idx = torch.topk(torch.softmax(logits, -1), cfg.num_experts_per_tok, -1)
            w = w / w.sum(-1, keepdim=True)
            y = torch.zeros_like(x)
            for t in range(T):
                for j in range(cfg.num_experts_per_tok):
                    e = int(idx[t, j])
                    gu = h[t] @ lw.w13[e].float().T
                    I = gu.shape[0] // 2
                    y[t] += w[t, j] * (F.silu(gu[:I]) * gu[I:]) @ lw.w2[e].float().T
            x = x + y
        else:
            gu = h @ lw.wgu.float().T
            I = gu.shape[1] // 2
            x = x + (F.silu(gu[:, :I]) * gu[:, I:]) @ lw.wd.float().T
    x = ref.rmsnorm(x, model.norm, cfg.rms_norm_eps)
    return x[-1] @ model.lm_head.float().T


def assert_greedy(model, prompt, toks, tol=1e-4, kv_dtype=None):
    """Teacher-forced check: every generated token is an argmax (within fp32
    reduction-order noise) of the dense forward over the tokens before it."""
    ids = list(prompt)
    for i, t in enumerate(toks):
        lg = dense_logits(model, ids, kv_dtype)
        assert lg[t] >= lg.max() - tol, (i, t, int(torch.argmax(lg)), float(lg.max() - lg[t]))
        ids.append(t)


def dense_greedy(model, ids, n):
    ids = list(ids)
    out = []
    for _ in range(n):
        t = int(torch.argmax(dense_logits(model, ids)))
        out.append(t)
        ids.append(t)
    return out


@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_engine_matches_dense(model):
    eng = make_engine(model)
    for lw in eng.runner.model.layers:
        if lw.router is not None:
            # decisive routing: with std-0.02 routers the 2nd/3rd expert probabilities tie
            # to ~1e-5, below fp32 reduction-order noise between batched and dense forwards
            lw.router.mul_(50.0)
    prompts = [[1, 5, 9, 33, 70], list(range(3, 100)), [7] * 20, list(range(200, 261))]
    sp = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True)
    res = eng.generate(prompts, sp)
    for p, (toks, _, reason) in zip(prompts, res):
        assert reason == "length"
        assert_greedy(eng.runner.model, p, toks)


def test_engine_fp8_kv_cache_matches_dense():
    """--kv-cache-dtype fp8: e4m3 K / V blocks (a quarter of the fp32 bytes here, half of
    bf16 on the GPU) and generation equal to the dense forward whose K / V rows are
    rounded to e4m3 the same way (saturating, per-tensor scale 1), through chunked
    prefill and paged decode."""
    eng = make_engine(kv_cache_dtype="fp8", max_num_batched_tokens=32)
    m = eng.runner.model
    assert all(k.dtype == torch.float8_e4m3fn and v.dtype == torch.float8_e4m3fn for k, v in eng.runner.kv)
    ref_bytes = make_engine().runner.model.kv_bytes_per_block(16)
    assert m.kv_bytes_per_block(16) * 4 == ref_bytes
    prompts = [[1, 5, 9, 33, 70], list(range(3, 100)), list(range(200, 261))]
    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    for p, (toks, _, reason) in zip(prompts, eng.generate(prompts, sp)):
        assert reason == "length"
        assert_greedy(m, p, toks, kv_dtype=torch.float8_e4m3fn)
    with pytest.raises(ValueError):
        EngineConfig(kv_cache_dtype="int4")


def test_chunked_prefill_and_prefix_cache_consistent():
    eng = make_engine(max_num_batched_tokens=16)  # forces multi-step chunked prefill
    p = list(range(10, 120))
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    a = eng.generate([p], sp)[0][0]
    b = eng.generate([p], sp)[0][0]  # second time: prefix-cache hit
    assert a == b
    assert eng.blocks.prefix_hit_tokens >= 96
    assert_greedy(eng.runner.model, p, a)


def test_preemption_recompute_is_exact():
    # tiny pool: 4 seqs x ~10 blocks cannot all fit -> preemption + recompute
    eng = make_engine(num_kv_blocks=24, block_size=16, max_num_batched_tokens=64,
                      enable_prefix_caching=False)
    prompts = [list(range(5 + i, 85 + i)) for i in range(4)]
    sp = SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True)
    res = eng.generate(prompts, sp)
    assert eng.scheduler.num_preemptions > 0
    for p, r in zip(prompts, res):
        assert_greedy(eng.runner.model, p, r[0])


def test_stop_conditions():
    eng = make_engine()
    p = [1, 5, 9]
    free = eng.generate([p], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))[0][0]
    # stop token id
    r = eng.generate([p], SamplingParams(temperature=0.0, max_tokens=8, stop_token_ids=[free[2]]))[0]
    assert r[0] == free[:3] and r[2] == "stop"
    # max_tokens
    r = eng.generate([p], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))[0]
    assert len(r[0]) == 3 and r[2] == "length"


def test_stop_string():
    eng = make_engine()
    p = [1, 5, 9]
    full = eng.generate([p], SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True))[0][1]
    needle = full[4:7]
    r = eng.generate([p], SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True,
                                         stop=[needle]))[0]
    assert r[2] == "stop"
    assert needle not in r[1]
    assert full.startswith(r[1])


def test_seeded_sampling_reproducible():
    eng = make_engine()
    sp = SamplingParams(temperature=1.0, top_p=0.9, top_k=20, max_tokens=12, ignore_eos=True, seed=11)
    a = eng.generate([[1, 2, 3]], sp)[0][0]
    b = eng.generate([[1, 2, 3]], sp)[0][0]
    assert a == b


def test_penalties_and_logprobs():
    eng = make_engine()
    sp = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True, frequency_penalty=2.0, presence_penalty=2.0,
                        logprobs=3)
    toks = eng.generate([[1, 2, 3]], sp)[0][0]
    # a strong frequency penalty makes greedy avoid immediate repeats
    assert len(set(toks)) >= 6


def test_top_logprobs_are_raw_with_penalties():
    """top-n log-probs report the raw model distribution (vLLM's
    default raw-logprobs mode) even when penalties change what is sampled: the first
    step's top-5 of a heavily penalised request equals the unpenalised one's, while the
    penalised greedy pick avoids the prompt's tokens."""
    eng = make_engine()
    p = [1, 2, 3, 2, 3, 2, 3]
    plain = SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True, logprobs=5)
    pen = SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True, logprobs=5, repetition_penalty=50.0,
                         frequency_penalty=2.0)
    rids = [eng.add_request(None, p, sp).request_id for sp in (plain, pen)]
    tops, toks = {}, {}
    while eng.has_unfinished():
        for o in eng.step():
            toks[o.request_id] = o.new_token_ids
            tops[o.request_id] = o.logprobs[1] if o.logprobs else None
    a, b = tops[rids[0]], tops[rids[1]]
    assert a is not None and [t for t, _ in a] == [t for t, _ in b]
    assert all(abs(x - y) < 1e-5 for (_, x), (_, y) in zip(a, b))
    assert [v for _, v in a] == sorted((v for _, v in a), reverse=True)
    assert toks[rids[1]][0] not in p


def test_penalty_slots_cover_every_running_sequence():
    """more penalised requests than the old 256-slot pool, plus
    preemptions (a KV pool too small for all of them at once): every step finds a
    free penalty slot, preempted sequences give theirs back, nothing raises."""
    eng = make_engine(max_num_seqs=300, max_num_batched_tokens=2048, num_kv_blocks=330, max_model_len=64)
    sp = SamplingParams(temperature=0.0, max_tokens=24, ignore_eos=True, frequency_penalty=0.5,
                        repetition_penalty=1.2)
    out = eng.generate([[1 + i % 50, 2, 3, 4 + i % 7] for i in range(300)], sp)
    assert all(len(r[0]) == 24 for r in out)
    assert eng.scheduler.num_preemptions > 0
    assert len(eng.runner._free_pen) == eng.runner.pen_counts.shape[0]  # all returned


def test_prefill_pad_table():
    """Ragged-chunk padding table (model_runner.pad_table): each 256-row count maps to
    the fastest count at or above it, a larger one only when >3 % faster."""
    from hipserve.engine.model_runner import pad_table

    # hipBLASLt-like cliffs: 7424 / 7680 slower than 7936 / 8192 (profiles/r2_prefill_row_padding.md)
    t = {6912: 2.433, 7168: 2.245, 7424: 2.746, 7680: 2.72, 7936: 2.349, 8192: 2.32}
    assert pad_table(t) == {6912: 7168, 7424: 7936, 7680: 7936}
    assert pad_table({1024: 1.0, 1280: 1.0, 1536: 0.99}) == {}  # within 3 %: keep the smaller count
    assert pad_table({}) == {}


def test_default_prefill_budget_per_weight_format():
    """8192 prefill tokens per step by default, 16384 for GGUF weights (their per-step
    dequantise pass is amortised over twice the tokens); an explicit flag wins."""
    from hipserve.config import default_batched_tokens
    from hipserve.server.cli import build_parser, config_from_args

    assert default_batched_tokens("llama-3-8b") == 8192
    assert default_batched_tokens("llama-3-8b", quantization="fp8") == 8192
    assert default_batched_tokens("llama-3-8b", quantization="q4_k_m") == 16384
    assert default_batched_tokens("/models/Meta-Llama-3-8B.Q8_0.gguf") == 16384
    assert default_batched_tokens("qwen3-30b-a3b", quantization="int8") == 32768
    p = build_parser()
    assert config_from_args(p.parse_args(["--model", "llama-3-8b", "--device", "cpu"])).max_num_batched_tokens == 8192
    assert config_from_args(p.parse_args(["--model", "llama-3-8b", "--device", "cpu", "--quantization", "q8_0"])
                            ).max_num_batched_tokens == 16384
    assert config_from_args(p.parse_args(["--model", "llama-3-8b", "--device", "cpu", "--quantization", "q8_0",
                                          "--max-num-batched-tokens", "4096"])).max_num_batched_tokens == 4096


def test_checkpoint_quantization_detection(tmp_path):
    """INT8 / FP8 read from a local checkpoint's quantization_config (compressed-tensors
    groups, AWQ bits) pick the budget without a --quantization flag."""
    import json

    from hipserve.config import checkpoint_quantization, default_batched_tokens

    def ckpt(name, q):
        d = tmp_path / name
        d.mkdir()
        (d / "config.json").write_text(json.dumps({"model_type": "qwen3_moe", "quantization_config": q}))
        return str(d)

    ct8 = ckpt("ct8", {"quant_method": "compressed-tensors",
                       "config_groups": {"group_0": {"weights": {"num_bits": 8, "type": "int"}}}})
    fp8 = ckpt("fp8", {"quant_method": "compressed-tensors",
                       "config_groups": {"group_0": {"weights": {"num_bits": 8, "type": "float"}}}})
    awq = ckpt("awq", {"quant_method": "awq", "bits": 8})
    awq4 = ckpt("awq4", {"quant_method": "awq", "bits": 4})
    assert checkpoint_quantization(ct8) == "int8" and default_batched_tokens(ct8) == 32768
    assert checkpoint_quantization(fp8) == "fp8" and default_batched_tokens(fp8) == 8192
    assert checkpoint_quantization(awq) == "int8"
    assert checkpoint_quantization(awq4) is None
    assert checkpoint_quantization(str(tmp_path / "missing")) is None
    assert checkpoint_quantization("llama-3-8b") is None
