"""GGUF dequant / dequant-MFMA GEMM kernels vs the numpy block decoders (T5)."""
import numpy as np
import pytest
import torch

from hipserve.ops import load_library
from hipserve.ops.quant import QuantWeight, dequantize, quant_linear
from hipserve.weights import gguf as G

pytestmark = pytest.mark.gpu
QTYPES = [G.Q4_0, G.Q8_0, G.Q4_K, G.Q5_K, G.Q6_K]


@pytest.fixture(scope="module", autouse=True)
def lib():
    load_library()


def _mat(N, K, seed=0):
    return np.random.default_rng(seed).standard_normal((N, K)).astype(np.float32) * 0.05


@pytest.mark.parametrize("qt", QTYPES)
def test_dequant_exact(qt):
    N, K = 48, 512
    w = _mat(N, K)
    qw = QuantWeight.from_float(w, qt, "cuda")
    ref = G.dequantize(G.quantize(w, qt), qt, N * K).reshape(N, K)
    got = dequantize(qw).float().cpu().numpy()
    want = torch.from_numpy(ref).to(torch.bfloat16).float().numpy()
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-6 + 1e-2 * np.abs(want).max())
    assert (got == want).mean() > 0.99


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("M", [1, 5, 17, 64])
@pytest.mark.parametrize("N,K", [(96, 256), (200, 1024), (4096, 512)])
def test_qgemm_matches_dequant_matmul(qt, M, N, K):
    w = _mat(N, K, seed=M)
    qw = QuantWeight.from_float(w, qt, "cuda")
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    y = quant_linear(x, qw).float()
    wd = torch.from_numpy(G.dequantize(G.quantize(w, qt), qt, N * K).reshape(N, K)).cuda()
    want = x.float() @ wd.to(torch.bfloat16).float().T
    err = (y - want).abs().max().item()
    assert err < 2e-2 * want.abs().max().item() + 1e-3, err


def test_mixed_parts_and_prefill_path():
    K = 512
    parts = [_mat(64, K, 1), _mat(32, K, 2), _mat(32, K, 3)]
    qw = QuantWeight.from_float(parts, G.Q4_K, "cuda")
    qw.parts[2] = QuantWeight.from_float(parts[2], G.Q6_K, "cuda").parts[0]  # Q4_K_M-style mix
    for M in (3, 130):  # fused decode path and dequant+hipBLASLt prefill path
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        y = quant_linear(x, qw).float()
        wd = torch.cat([torch.from_numpy(G.dequantize(G.quantize(p, t), t, p.size).reshape(p.shape))
                        for p, t in zip(parts, (G.Q4_K, G.Q4_K, G.Q6_K))]).cuda()
        want = x.float() @ wd.to(torch.bfloat16).float().T
        assert (y - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-3


def test_gguf_engine_on_gpu(tmp_path):
    from hipserve.config import PRESETS, EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    cfg = PRESETS["small-llama"]
    p = str(tmp_path / "small.gguf")
    G.write_synthetic_llama_gguf(p, cfg, G.Q4_K, mixed_k=True)
    eng = LLMEngine(EngineConfig(model=p, device="cuda", num_kv_blocks=256, max_model_len=1024,
                                 max_num_batched_tokens=256, max_num_seqs=8),
                    tp=TPGroup(0, 1, None, torch.device("cuda", 0)))
    assert isinstance(eng.runner.model.layers[0].wqkv, QuantWeight)
    res = eng.generate([[1] + list(range(300, 400)), [1, 5, 6]] * 3,
                       SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True))
    assert all(len(r[0]) == 10 for r in res)
    assert res[0][0] == res[2][0] == res[4][0]


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K, G.Q8_0, G.Q4_0])
def test_random_blocks_gemm(qt):
    """Synthetic GGUF blocks (ops/quant.random_blocks, the GGUF-tier benchmark
    weights): decode GEMM and prefill path vs x @ numpy-dequantised W."""
    from hipserve.ops.quant import random_blocks
    N, K = 320, 1024
    raw = random_blocks(np.random.default_rng(qt), qt, N, K)
    dense = G.dequantize(raw, qt, N * K).reshape(N, K)
    assert np.isfinite(dense).all() and 0.002 < np.abs(dense).mean() < 0.2
    qw = QuantWeight.from_raw([(qt, N, K, raw)], "cuda")
    want_w = torch.from_numpy(dense).cuda()
    for M in (4, 64, 200):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        y = quant_linear(x, qw).float()
        want = x.float() @ want_w.T
        assert (y - want).abs().max().item() < 2e-2 * want.abs().max().item() + 1e-3


def test_synthetic_q4_k_m_engine():
    """Engine with random-init Q4_K_M weights (bench.py --quantization q4_k_m) on the GPU."""
    from hipserve.config import PRESETS, EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    cfg = PRESETS["small-llama"]
    eng = LLMEngine(EngineConfig(model="small-llama", load_format="dummy", device="cuda", num_kv_blocks=256,
                                 max_model_len=1024, max_num_batched_tokens=256, max_num_seqs=8,
                                 extra={"quantization": "q4_k_m"}),
                    tp=TPGroup(0, 1, None, torch.device("cuda", 0)), model_cfg=cfg)
    m = eng.runner.model
    assert isinstance(m.layers[0].wqkv, QuantWeight) and m.cfg.rope_mode == 1
    assert [p.qtype for p in m.layers[0].wqkv.parts] == [G.Q4_K, G.Q4_K, G.Q6_K]
    res = eng.generate([[1] + list(range(300, 400)), [1, 5, 6]] * 3,
                       SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True))
    assert all(len(r[0]) == 10 for r in res)
    assert res[0][0] == res[2][0] == res[4][0]
