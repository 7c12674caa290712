"""GGUF tier on CPU: block codecs (bit layouts), file parser/writer, tokenizers,
and the engine running a synthetic GGUF llama (SURVEY §4.2, K14/K15 oracle)."""
import struct

import numpy as np
import pytest
import torch

from hipserve.config import PRESETS
from hipserve.weights import gguf as G


def _f16(x):
    return np.array([x], np.float16).view(np.uint8)


def test_q8_0_block_layout():
    blk = np.concatenate([_f16(0.5), np.arange(-16, 16, dtype=np.int8).view(np.uint8)])
    assert blk.size == 34
    np.testing.assert_allclose(G.dequantize(blk, G.Q8_0, 32), 0.5 * np.arange(-16, 16))


def test_q4_0_block_layout():
    qs = np.array([(j & 15) | (((15 - j) & 15) << 4) for j in range(16)], np.uint8)
    blk = np.concatenate([_f16(2.0), qs])
    y = G.dequantize(blk, G.Q4_0, 32)
    np.testing.assert_allclose(y[:16], 2.0 * (np.arange(16) - 8))       # low nibbles -> 0..15
    np.testing.assert_allclose(y[16:], 2.0 * (15 - np.arange(16) - 8))  # high nibbles -> 16..31


def test_q4_k_block_layout():
    # d=1, dmin=0.5; sub-block scales 1..8, mins 0..7 packed as get_scale_min_k4 expects
    sc = list(range(1, 9))
    mn = list(range(0, 8))
    s12 = np.zeros(12, np.uint8)
    for j in range(4):
        s12[j] = sc[j] | ((sc[j + 4] >> 4) << 6)
        s12[j + 4] = mn[j] | ((mn[j + 4] >> 4) << 6)
        s12[j + 8] = (sc[j + 4] & 0xF) | ((mn[j + 4] & 0xF) << 4)
    qs = np.array([(l % 16) | (((l + 3) % 16) << 4) for l in range(32)] * 4, np.uint8)
    blk = np.concatenate([_f16(1.0), _f16(0.5), s12, qs])
    y = G.dequantize(blk, G.Q4_K, 256).reshape(8, 32)
    for sub in range(8):
        q = (np.arange(32) % 16) if sub % 2 == 0 else ((np.arange(32) + 3) % 16)
        np.testing.assert_allclose(y[sub], sc[sub] * q - 0.5 * mn[sub])


def test_q6_k_block_layout():
    # all 6-bit values = 33 (-> +1), scales = index+1, d = 0.25
    ql = np.full(128, 0x11, np.uint8)            # low nibbles 1
    qh = np.full(64, 0b10101010, np.uint8)       # high 2 bits = 2 (-> +32)
    scl = np.arange(1, 17, dtype=np.int8).view(np.uint8)
    blk = np.concatenate([ql, qh, scl, _f16(0.25)])
    y = G.dequantize(blk, G.Q6_K, 256)
    want = 0.25 * np.repeat(np.arange(1, 17), 16) * 1.0
    np.testing.assert_allclose(y, want)


@pytest.mark.parametrize("qt,tol", [(G.Q8_0, 0.01), (G.Q4_0, 0.15), (G.Q4_1, 0.15), (G.Q4_K, 0.12),
                                    (G.Q5_K, 0.06), (G.Q6_K, 0.03), (G.F16, 1e-3), (G.BF16, 1e-2)])
def test_codec_roundtrip(qt, tol):
    if qt == G.Q4_1:
        pytest.skip("Q4_1 quantiser not provided (decode-only format)")
    x = np.random.default_rng(1).standard_normal(2048).astype(np.float32)
    y = G.dequantize(G.quantize(x, qt), qt, x.size)
    assert np.abs(x - y).mean() / np.abs(x).mean() < tol


def test_file_roundtrip_and_config(tmp_path):
    cfg = PRESETS["tiny-llama"]
    p = str(tmp_path / "m.gguf")
    G.write_synthetic_llama_gguf(p, cfg, G.Q4_K, mixed_k=True)
    gf = G.GGUFFile(p)
    mc = gf.model_config()
    assert (mc.hidden_size, mc.num_layers, mc.num_heads, mc.num_kv_heads, mc.head_dim) == \
        (cfg.hidden_size, cfg.num_layers, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim)
    assert mc.rope_mode == 1 and mc.vocab_size == cfg.vocab_size
    assert gf.tensors["blk.0.attn_v.weight"].type == G.Q6_K
    assert gf.tensors["blk.0.attn_q.weight"].type == G.Q4_K
    assert gf.tensors["blk.1.ffn_down.weight"].rows_cols == (cfg.hidden_size, cfg.intermediate_size)
    assert gf.data_offset % 32 == 0


def test_spm_tokenizer(tmp_path):
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{b:02X}>" for b in range(256)] + \
        ["▁", "h", "e", "l", "o", "he", "ll", "llo", "hello", "▁hello", "w", "r", "d", "▁w", "or", "ld", "▁wor", "▁world"]
    cfg = PRESETS["tiny-llama"].replace(vocab_size=len(toks))
    p = str(tmp_path / "t.gguf")
    G.write_synthetic_llama_gguf(p, cfg, G.Q8_0, vocab_tokens=toks)
    tk = G.GGUFTokenizer(G.GGUFFile(p))
    ids = tk.encode("hello world")
    assert ids[0] == 1
    assert [tk.tokens[i] for i in ids[1:]] == ["▁hello", "▁world"]
    assert tk.decode(ids) == " hello world"
    # unknown characters fall back to bytes
    ids = tk.encode("hé", add_special_tokens=False)
    assert tk.decode(ids) == " hé"


def test_engine_runs_gguf_on_cpu(tmp_path):
    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    from .test_engine_cpu import dense_greedy

    cfg = PRESETS["tiny-llama"]
    p = str(tmp_path / "m.gguf")
    G.write_synthetic_llama_gguf(p, cfg, G.Q8_0)
    eng = LLMEngine(EngineConfig(model=p, device="cpu", dtype="float32", num_kv_blocks=128,
                                 max_model_len=256, max_num_batched_tokens=32), tp=TPGroup())
    assert eng.runner.load_format == "gguf"
    assert eng.model_cfg.rope_mode == 1
    prompts = [[1, 300, 301, 302], list(range(260, 300))]
    res = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    for pr, r in zip(prompts, res):
        assert r[0] == dense_greedy(eng.runner.model, pr, 6)
    out = eng.generate(["hello"], SamplingParams(temperature=0.0, max_tokens=3, ignore_eos=True))
    assert len(out[0][0]) == 3


def test_synthetic_quant_engine_cpu():
    """--load-format dummy --quantization q4_k_m on the CPU plumbing engine: the
    random ggml blocks are dequantised to dense weights (same blocks as on GPU)."""
    import torch

    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    eng = LLMEngine(EngineConfig(model="tiny-llama", load_format="dummy", device="cpu", dtype="float32",
                                 num_kv_blocks=128, max_model_len=256, max_num_batched_tokens=64,
                                 max_num_seqs=4, extra={"quantization": "q4_k_m"}), tp=TPGroup())
    m = eng.runner.model
    assert m.cfg.rope_mode == 1 and isinstance(m.layers[0].wqkv, torch.Tensor)
    assert torch.isfinite(m.layers[0].wd).all()
    res = eng.generate([[1, 5, 6, 7]], SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    assert len(res[0][0]) == 6


def test_sub_scale_range_guard():
    """ops/quant.py sub_scale_ok: the v2 kernel's subnormal-integer dequant needs every
    block scale below 65504 / 2^(24 - shift); random synthetic blocks pass, a block with
    a huge scale sends the weight to the v1 kernel."""
    from hipserve.ops import quant as Q

    rng = np.random.default_rng(0)
    for qt in (G.Q4_K, G.Q5_K, G.Q6_K, G.Q8_0, G.Q4_0, G.Q4_1):
        raw = Q.random_blocks(rng, qt, 32, 512).copy()
        assert Q.sub_scale_ok(raw, qt), G.TYPE_NAMES.get(qt, qt)
        _, bb = G.BLOCK[qt]
        b = raw.reshape(-1, bb)
        off = 208 if qt == G.Q6_K else 0
        b[3, off:off + 2] = np.frombuffer(np.float16(8.0).tobytes(), np.uint8)  # one block, scale 8
        if qt in (G.Q4_K, G.Q5_K):
            b[3, 4:16] = 0xFF  # 6-bit scales at 63
        if qt == G.Q6_K:
            b[3, 192:208] = 100
        assert not Q.sub_scale_ok(raw, qt), G.TYPE_NAMES.get(qt, qt)
    assert Q.sub_scale_ok(np.zeros(0, np.uint8), G.Q4_K)
