"""Quantised decode GEMM v3 (csrc/kernels/gguf_decode.hip: the x slice resident in LDS per
persistent workgroup, weight chunks streamed into registers three items ahead) vs a plain
PyTorch fp32 matmul of the numpy block decoder's weights, for every tiled format (GGUF
Q4_0 .. Q6_K, FP8 per-channel, INT8), every decode row bucket (1, 16, 33, 64 rows: MT =
1 / 2 / 4), split-K slices of every length (1 .. 11 super-chunks: item streams shorter
than the three-deep register rotation, slices past the LDS fall back to v2), mixed formats in one merged
weight (two launches into one output), parts whose rows are not a multiple of the
workgroup's rows. The v3 kernel is bit-identical to v2 on the same f16 operands (same
dequant, same MFMA order per accumulator), and rows past the f16 range take the
pre-scaled recompute (q3_slow)."""
import numpy as np
import pytest
import torch

from hipserve.ops import load_library
from hipserve.ops import quant as Q
from hipserve.ops.quant import QuantWeight
from hipserve.weights import gguf as G

pytestmark = pytest.mark.gpu
GGUF = [G.Q4_0, G.Q4_1, G.Q8_0, G.Q4_K, G.Q5_K, G.Q6_K]


@pytest.fixture(scope="module", autouse=True)
def lib():
    load_library()


def _rand_qw(specs, seed=0):
    rng = np.random.default_rng(seed)
    raws = [(t, n, k, Q.random_blocks(rng, t, n, k)) for t, n, k in specs]
    return QuantWeight.from_raw(raws, "cuda"), raws


def _dense(raws):
    return torch.cat([torch.from_numpy(G.dequantize(r, t, n * k).reshape(n, k)) for t, n, k, r in raws]).cuda()


def _x16(x):
    """bf16 x -> f16 in the quantised GEMMs' pair order {0, 2, 1, 3, 4, 6, 5, 7} per 8-run
    (what the decode producers write as out16 / act16)."""
    h = x.float().to(torch.float16).reshape(x.shape[0], -1, 8)
    return h[:, :, [0, 2, 1, 3, 4, 6, 5, 7]].reshape(x.shape).contiguous()


def _run(qw, x, S, x16):
    nsb = qw.K // 256
    per = -(-nsb // S)
    ny = -(-nsb // per)
    ws = torch.full((ny * x.shape[0] * qw.N,), float("nan"), dtype=torch.float32, device="cuda")
    Q._launch_v2(torch.empty(0, dtype=torch.bfloat16, device="cuda"), ws, x, qw, S, x16)
    return ws.view(ny, x.shape[0], qw.N)


@pytest.mark.parametrize("qt", GGUF)
@pytest.mark.parametrize("M", [1, 16, 33, 64])
def test_v3_formats_vs_fp32_and_v2(qt, M):
    K = 2048
    qw, raws = _rand_qw([(qt, 512, K), (qt, 80, K), (qt, 272, K)], seed=M + qt)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    want = x.float() @ _dense(raws).T
    tol = 1e-2 * want.abs().max().item() + 1e-3
    for S in (1, 3):
        v3 = _run(qw, x, S, _x16(x))
        assert torch.isfinite(v3).all()
        assert (v3.sum(0) - want).abs().max().item() < tol
        v2 = _run(qw, x, S, None)
        assert torch.equal(v3, v2), (S, (v3 - v2).abs().max().item())


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K])
@pytest.mark.parametrize("S", [1, 2, 3, 5, 7, 11])
def test_v3_every_slice_length(qt, S):
    """K slices of 1 .. 11 super-chunks at M = 64 (up to 4 run v3, longer ones v2), a
    Q4_K + Q6_K merged weight (two launches, one output)."""
    K, M = 2816, 64
    qw, raws = _rand_qw([(qt, 256, K), (G.Q6_K if qt == G.Q4_K else G.Q4_K, 128, K)], seed=S)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    want = x.float() @ _dense(raws).T
    got = _run(qw, x, S, _x16(x))
    assert torch.isfinite(got).all()
    assert (got.sum(0) - want).abs().max().item() < 1e-2 * want.abs().max().item() + 1e-3


@pytest.mark.parametrize("M", [1, 33, 64])
def test_v3_fp8_and_int8(M):
    """FP8 e4m3 (per-row scale) and INT8 (group scale + zero point) parts through v3."""
    N, K = 272, 1024
    torch.manual_seed(M)
    w = torch.randn(N, K, device="cuda") * 0.02
    s = w.abs().amax(1, keepdim=True) / 448.0
    q = (w / s).to(torch.float8_e4m3fn)
    f8 = QuantWeight([Q.QuantPart.from_fp8(q, s, "cuda")])
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    want = x.float() @ (q.float() * s).T
    got = _run(f8, x, 2, _x16(x)).sum(0)
    assert (got - want).abs().max().item() < 1e-2 * want.abs().max().item() + 1e-3
    qi = torch.randint(-128, 128, (N, K))
    sc = torch.rand(N, K // 32) * 2e-3 + 1e-4
    zp = torch.randint(-8, 8, (N, K // 32))
    i8 = QuantWeight([Q.QuantPart.from_int8((qi + 128).to(torch.uint8), sc, zp, "cuda")])
    wref = ((qi - zp.repeat_interleave(32, 1)).float() * sc.repeat_interleave(32, 1)).cuda()
    want = x.float() @ wref.T
    got = _run(i8, x, 1, _x16(x)).sum(0)
    assert (got - want).abs().max().item() < 1e-2 * want.abs().max().item() + 1e-4


@pytest.mark.parametrize("qt", [G.Q4_K, G.Q6_K])
@pytest.mark.parametrize("M", [16, 64])
def test_v3_beyond_f16_range(qt, M):
    """Rows past the f16 range are inf in x16: the waves whose accumulators come out
    non-finite recompute from the bf16 x with power-of-two row pre-scales; ordinary rows
    keep full accuracy, and the result equals v2's rerun bit for bit."""
    K = 2048
    qw, raws = _rand_qw([(qt, 512, K)], seed=3 + M)
    x = torch.randn(M, K, device="cuda")
    x[::5] *= 3e5
    x = x.to(torch.bfloat16)
    want = x.float() @ _dense(raws).T
    rowmax = want.abs().amax(1, keepdim=True)
    v3 = _run(qw, x, 2, _x16(x))
    assert torch.isfinite(v3).all()
    assert ((v3.sum(0) - want).abs() / rowmax).max().item() < 1e-2
    assert torch.equal(v3, _run(qw, x, 2, None))


def test_v3_bf16_store_and_disable(monkeypatch):
    """S == 1 writes bf16 directly (quant_linear's decode path with x16 is the partial
    path; here through _launch_v2 with an output); HIPSERVE_QGEMM3=0 at process start
    keeps v2 (checked by the launcher's env read only once: not toggled here)."""
    K, M = 1024, 48
    qw, raws = _rand_qw([(G.Q4_K, 384, K)], seed=5)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.full((M, qw.N), float("nan"), dtype=torch.bfloat16, device="cuda")
    Q._launch_v2(out, torch.empty(0, dtype=torch.float32, device="cuda"), x, qw, 1, _x16(x))
    want = x.float() @ _dense(raws).T
    assert (out.float() - want).abs().max().item() < 1e-2 * want.abs().max().item() + 1e-3
