"""FP8 W8A8 decode GEMM (csrc/kernels/fp8_decode.hip: per-token e4m3 activations x
per-channel e4m3 weights in the decode tiled layout on the scaled FP8 MFMA, fp32
split-K partials) against a plain PyTorch fp32 reference of the same op: the
reference dequantises the kernel's own e4m3 activations and the e4m3 weights and
multiplies in fp32 (products of two e4m3 values are exact in fp32, so only the
summation order differs). Multi-part weights (q | k | v-like), every m-tile width
(M 1..64), the K-slice counts the engine picks, and the quant_linear / quant_partial
wiring."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    from hipserve.ops import load_library

    load_library()


def _weight(g, rows, K):
    from hipserve.ops import quant as Q

    parts, deq = [], []
    for n in rows:
        w = (torch.rand(n, K, device=DEV, generator=g) * 2 - 1) * (0.02 + torch.rand(n, 1, device=DEV, generator=g))
        s = w.abs().amax(1, keepdim=True) / 448.0
        q = (w / s).to(torch.float8_e4m3fn)
        parts.append(Q.QuantPart.from_fp8(q, s, DEV))
        deq.append(q.float() * s)
    return Q.QuantWeight(parts), torch.cat(deq)


def _x(g, M, K):
    x = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1) * torch.logspace(-1, 1, M, device=DEV).unsqueeze(1)
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 65, 128, 200, 256])
@pytest.mark.parametrize("rows,K", [([512, 256, 256], 4096), ([768], 5376), ([256], 21504), ([1024, 1024], 1792)])
def test_fp8_decode_gemm_vs_fp32(M, rows, K):
    """M 65..256: the 8 / 16 x-tile bodies of the decode graph buckets above 64 rows."""
    from hipserve.ops import pgemm, quant as Q

    g = torch.Generator(device=DEV).manual_seed(M * 7 + K)
    w, wd = _weight(g, rows, K)
    assert Q.f8_decode_ok(w)
    x = _x(g, M, K)
    xq, xs = pgemm.act_quant(x)
    want = (xq.view(torch.float8_e4m3fn).float() * xs.unsqueeze(1)) @ wd.t()
    for S in sorted({Q.f8_decode_splits(w, M), 1 if (K // 256) in Q.F8D_STEPS else Q.f8_decode_splits(w, M)}):
        ws = torch.full((S * M * w.N,), float("nan"), device=DEV)
        torch.ops.hipserve.fp8_decode_gemm(ws, xq, xs, [p.q for p in w.parts], [p.rs for p in w.parts], S)
        got = ws.view(S, M, w.N).sum(0)
        scale = want.abs().amax(1, keepdim=True).clamp_min(1e-30)
        torch.testing.assert_close(got / scale, want / scale, rtol=0, atol=1e-4)


@pytest.mark.parametrize("M", [48, 256])
def test_quant_linear_and_partial_use_fp8_decode(M):
    """At decode sizes (up to 256 rows) quant_linear = the fused path's partials reduced
    by splitk_reduce (bit-identical), and both are W8A8."""
    from hipserve.ops import pgemm, quant as Q

    g = torch.Generator(device=DEV).manual_seed(9)
    w, wd = _weight(g, [512, 256, 256], 2048)
    x = _x(g, M, 2048)
    y = Q.quant_linear(x, w)
    ws, S = Q.quant_partial(x, w)
    r = torch.empty_like(y)
    torch.ops.hipserve.splitk_reduce(r, ws, S)
    assert torch.equal(y, r)
    xq, xs = pgemm.act_quant(x)
    want = (xq.view(torch.float8_e4m3fn).float() * xs.unsqueeze(1)) @ wd.t()
    torch.testing.assert_close(y.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())
    # vs the unquantised activations: e4m3 rounding of x only (~2-3 % RMS per element)
    rel = (y.float() - x.float() @ wd.t()).norm() / (x.float() @ wd.t()).norm()
    assert rel < 5e-2, rel


@pytest.mark.parametrize("post", [False, True])
@pytest.mark.parametrize("M,N", [(1, 5376), (48, 4096), (64, 2048)])
def test_norm_epilogue_e4m3_copy_is_act_quant(post, M, N):
    """splitk_add_rmsnorm / splitk_post_add_rmsnorm ``out8`` / ``xs8``: the per-token
    e4m3 copy of their bf16 output is bit-identical to act_quant_fp8 of that output."""
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M + N + post)
    S = 3
    ws = torch.randn(S * M * N, device=DEV, generator=g)
    res = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    w1 = (1 + 0.1 * torch.randn(N, device=DEV, generator=g)).to(torch.bfloat16)
    w2 = (1 + 0.1 * torch.randn(N, device=DEV, generator=g)).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    q8 = torch.empty(M, N, device=DEV, dtype=torch.uint8)
    s8 = torch.empty(M, device=DEV, dtype=torch.float32)
    if post:
        torch.ops.hipserve.splitk_post_add_rmsnorm(out, res, ws, S, w1, w2, 1e-6, None, q8, s8)
    else:
        torch.ops.hipserve.splitk_add_rmsnorm(out, res, ws, S, w1, 1e-6, None, q8, s8)
    xq, xs = pgemm.act_quant(out)
    assert torch.equal(q8, xq) and torch.equal(s8, xs)


@pytest.mark.parametrize("add", [False, True])
@pytest.mark.parametrize("M,N", [(3, 5376), (300, 4096), (1000, 1024)])
def test_rmsnorm_e4m3_copy_is_act_quant(add, M, N):
    """rmsnorm / fused_add_rmsnorm ``out8`` / ``xs8`` (the FP8 prefill GEMM's input,
    written by the norm instead of a separate act_quant_fp8 pass) is bit-identical to
    act_quant_fp8 of the bf16 output."""
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M + N + add)
    x = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    res = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    w = (1 + 0.1 * torch.randn(N, device=DEV, generator=g)).to(torch.bfloat16)
    out = torch.empty_like(x)
    q8 = torch.empty(M, N, device=DEV, dtype=torch.uint8)
    s8 = torch.empty(M, device=DEV, dtype=torch.float32)
    if add:
        torch.ops.hipserve.fused_add_rmsnorm(out, x, res, w, 1e-6, q8, s8)
    else:
        torch.ops.hipserve.rmsnorm(out, x, w, 1e-6, q8, s8)
    xq, xs = pgemm.act_quant(out)
    assert torch.equal(q8, xq) and torch.equal(s8, xs)