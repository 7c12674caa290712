"""GGUF prefill GEMM straight from the tiled blocks (gguf_mfma.hip qpg_kernel) vs a plain
PyTorch fp32 reference on the numpy block decoder's weights: plain store into part
columns (mixed formats, as Q4_K_M's q|k|v), residual add, SiLU / GELU GLU of gate / up
parts, ragged M / N, and rows beyond the f16 range (x_f16_pairs' power-of-two row
pre-scale, undone in the epilogue)."""
import numpy as np
import pytest
import torch

from hipserve.ops import load_library
from hipserve.ops import quant as Q
from hipserve.ops.quant import QuantWeight
from hipserve.weights import gguf as G

pytestmark = pytest.mark.gpu
QTYPES = [G.Q4_0, G.Q4_1, G.Q8_0, G.Q4_K, G.Q5_K, G.Q6_K]


@pytest.fixture(scope="module", autouse=True)
def lib():
    load_library()


def _mat(N, K, seed):
    return np.random.default_rng(seed).standard_normal((N, K)).astype(np.float32) * 0.05


def _raw(w, qt, seed=0):
    """ggml blocks of w (Q4_1 has no quantiser here: random valid blocks of its shape)."""
    if qt == G.Q4_1:
        return Q.random_blocks(np.random.default_rng(seed), qt, *w.shape)
    return G.quantize(w, qt)


def _ref_w(w, qt):
    """fp32 weights as the numpy block decoder reads the quantised blocks."""
    N, K = w.shape
    return torch.from_numpy(G.dequantize(_raw(w, qt), qt, N * K).reshape(N, K)).cuda()


def _qw(mats, qts):
    return QuantWeight.from_raw([(qt, m.shape[0], m.shape[1], _raw(m, qt)) for m, qt in zip(mats, qts)], "cuda")


def _args(qw):
    cols = np.cumsum([0] + [p.N for p in qw.parts])[:-1].tolist()
    return [p.q for p in qw.parts], [p.kqt for p in qw.parts], [p.N for p in qw.parts], cols


def _close(got, want, tol=1e-2):
    err = (got.float() - want).abs().max().item()
    assert err <= tol * want.abs().max().item() + 1e-3, (err, want.abs().max().item())


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("M,N,K", [(130, 272, 512), (1000, 512, 1024), (37, 1024, 256), (300, 4096, 512)])
def test_store(qt, M, N, K):
    w = _mat(N, K, M + N)
    qw = _qw([w], [qt])
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 0)
    _close(out, x.float() @ _ref_w(w, qt).T)


def test_mixed_formats_strided():
    """q | k | v with v in Q6_K (Q4_K_M), written at their columns of a wider output;
    x a strided view."""
    K, M = 768, 333
    mats = [_mat(512, K, 1), _mat(128, K, 2), _mat(128, K, 3)]
    qw = QuantWeight.from_float(mats[:2], G.Q4_K, "cuda")
    qw.parts.append(QuantWeight.from_float(mats[2], G.Q6_K, "cuda").parts[0])
    xb = torch.randn(M, K + 64, device="cuda", dtype=torch.bfloat16)
    x = xb[:, 16:16 + K]
    out = torch.full((M, 800), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 0)
    wd = torch.cat([_ref_w(m, t) for m, t in zip(mats, (G.Q4_K, G.Q4_K, G.Q6_K))])
    _close(out[:, :768], x.float() @ wd.T)
    assert out[:, 768:].isnan().all()  # untouched past the parts


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K])
def test_residual_add(qt):
    M, N, K = 517, 1024, 1024
    w = _mat(N, K, 9)
    qw = QuantWeight.from_float(w, qt, "cuda")
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    res0 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    res = res0.clone()
    assert torch.ops.hipserve.gguf_prefill(res, *Q.x_f16_pairs(x, K), *_args(qw), K, 1)
    h = (x.float() @ _ref_w(w, qt).T).to(torch.bfloat16).float()
    _close(res, h + res0.float(), tol=2e-2)


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q4_0, G.Q6_K])
@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,I", [(700, 384), (64, 1088)])
def test_glu(qt, act, M, I):
    K = 512
    g, u = _mat(I, K, 3), _mat(I, K, 4)
    qw = _qw([g, u], [qt, qt])
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.full((M, I), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 2 if act == "silu" else 3)
    gv = (x.float() @ _ref_w(g, qt).T).to(torch.bfloat16).float()
    uv = (x.float() @ _ref_w(u, qt).T).to(torch.bfloat16).float()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    _close(out, f(gv) * uv, tol=2e-2)


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K])
def test_f16_range_rescale(qt):
    """Rows with activations beyond the f16 range are pre-scaled by a power of two
    (x_f16_pairs) and stay exact; the other rows are unaffected."""
    M, N, K = 200, 256, 512
    w = _mat(N, K, 5)
    qw = QuantWeight.from_float(w, qt, "cuda")
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    x[3, 7] = 3.0e5
    x[150, :] *= 1.0e6
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 0)
    want = x.float() @ _ref_w(w, qt).T
    assert out.isfinite().all()
    for r in (3, 150, 0, 199):
        _close(out[r], want[r])


def test_rejects():
    K = 256
    qw = QuantWeight.from_float([_mat(64, K, 1), _mat(64, K, 2)], G.Q4_K, "cuda")
    qw.parts[1] = QuantWeight.from_float(_mat(64, K, 2), G.Q6_K, "cuda").parts[0]
    x = torch.randn(10, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(10, 64, device="cuda", dtype=torch.bfloat16)
    assert not torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 2)  # GLU over two formats


def test_x_f16_pairs():
    """The operand conversion: pair order {0, 2, 1, 3, 4, 6, 5, 7} per 8-run, every row
    scaled by 2^-k with max |x| 2^-k in [2^14, 2^15), rsc = 2^k."""
    M, K = 5, 512
    x = torch.randn(M, K + 8, device="cuda", dtype=torch.bfloat16)[:, :K]
    x[2] *= 1.0e6
    x16, rsc = Q.x_f16_pairs(x, K)
    perm = torch.tensor([0, 2, 1, 3, 4, 6, 5, 7], device="cuda")
    back = x16.float().view(M, K // 8, 8)[:, :, perm.argsort()].reshape(M, K) * rsc[:, None]
    assert torch.allclose(back, x.float(), rtol=1e-3, atol=1e-4 * x.float().abs().amax(1, keepdim=True).max().item())
    assert rsc[2].item() > 1.0 and x16.isfinite().all()
    # every row lands in [2^14, 2^15) (small rows are scaled up too), rsc a power of two
    amax = x16.float().abs().amax(1)
    assert ((amax >= 16384) & (amax < 32768)).all()
    assert (torch.frexp(rsc)[0] == 0.5).all()


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K])
def test_small_activations(qt):
    """1e-3-scale activations (all elements in the f16 subnormal range without the
    upward row scale) against the fp32 oracle at full relative accuracy."""
    M, N, K = 150, 256, 512
    w = _mat(N, K, 11)
    qw = QuantWeight.from_float(w, qt, "cuda")
    x = (torch.randn(M, K, device="cuda") * 1e-3).to(torch.bfloat16)
    x[5] *= 1e-3
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert torch.ops.hipserve.gguf_prefill(out, *Q.x_f16_pairs(x, K), *_args(qw), K, 0)
    want = x.float() @ _ref_w(w, qt).T
    for r in (0, 5, 77):
        _close(out[r], want[r])
