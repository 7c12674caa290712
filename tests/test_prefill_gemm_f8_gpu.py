"""FP8 W8A8 prefill GEMM (csrc/kernels/prefill_gemm.hip pgemm_f8_kernel, the scaled
e4m3 MFMA over the decode kernel's tiled FP8 weights) and the per-token dynamic
activation quantiser, each against a plain PyTorch fp32 reference of the same op:
the reference dequantises the kernel's own e4m3 activations (so only the GEMM is
compared) and the e4m3 weights, multiplies in fp32 and applies the same epilogue.
Ragged M, multi-part (q|k|v-like) weights, residual add, SiLU- and GELU-GLU."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    from hipserve.ops import load_library

    load_library()


def _fp8_weight(g, N, K):
    from hipserve.ops import quant as Q

    w = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1) * (0.02 + torch.rand(N, 1, device=DEV, generator=g))
    s = w.abs().amax(1, keepdim=True) / 448.0
    q = (w / s).to(torch.float8_e4m3fn)
    return Q.QuantPart.from_fp8(q, s, DEV), q.float() * s


def _weight(g, rows, K):
    from hipserve.ops import quant as Q

    parts = [_fp8_weight(g, n, K) for n in rows]
    return Q.QuantWeight([p for p, _ in parts]), torch.cat([d for _, d in parts])


def _x(g, M, K):
    x = torch.rand(M, K, device=DEV, generator=g) * 2 - 1
    x = x * torch.logspace(-2, 2, M, device=DEV).unsqueeze(1)  # rows of very different magnitude
    x[M // 2] = 0.0
    return x.to(torch.bfloat16)


def _deq_x(xq, xs):
    return xq.view(torch.float8_e4m3fn).float() * xs.unsqueeze(1)


def test_act_quant_fp8():
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(3)
    M, K = 777, 5376
    x = _x(g, M, K)
    x[5, 17] = 1.5e5  # beyond the f16 range: a per-row scale takes it
    xq, xs = pgemm.act_quant(x)
    amax = x.float().abs().amax(1)
    want_s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    torch.testing.assert_close(xs, want_s, rtol=1e-6, atol=0)
    ref = (x.float() / want_s.unsqueeze(1)).clamp(-448, 448).to(torch.float8_e4m3fn).float()
    got = xq.view(torch.float8_e4m3fn).float()
    assert torch.isfinite(got).all()
    diff = (got != ref)
    # x * (448 / max) vs x / (max / 448): a value on an e4m3 rounding midpoint may go either way
    assert diff.float().mean().item() < 5e-3
    step = torch.where(ref.abs() > 0, ref.abs() / 8, torch.full_like(ref, 2.0 ** -9))
    assert ((got - ref).abs() <= step + 1e-12)[diff].all()
    assert (got.abs().amax(1)[amax > 0] == 448).all()


@pytest.mark.parametrize("M,rows,K", [(300, [256], 256), (1000, [512, 256, 256], 1024), (2049, [768], 512),
                                      (4096, [1024, 256], 4096), (130, [256], 5376)])
def test_prefill_gemm_f8_store(M, rows, K):
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M + K)
    w, wd = _weight(g, rows, K)
    x = _x(g, M, K)
    xq, xs = pgemm.act_quant(x)
    out = torch.full((M, sum(rows)), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_f8(out, xq, xs, [p.q for p in w.parts], [p.rs for p in w.parts], 0)
    want = _deq_x(xq, xs) @ wd.t()
    scale = want.abs().amax(1, keepdim=True).clamp_min(1e-30)
    torch.testing.assert_close(out.float() / scale, want / scale, rtol=0, atol=1e-2)
    # the pgemm.f8_gemm wrapper (quantises x itself) gives the same result
    out2 = pgemm.f8_gemm(x, w)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("M,N,K", [(300, 256, 1024), (1000, 512, 512)])
def test_prefill_gemm_f8_residual_add(M, N, K):
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(5 + M)
    w, wd = _weight(g, [N], K)
    x = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    res0 = (torch.rand(M, N, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    xq, xs = pgemm.act_quant(x)
    res = res0.clone()
    torch.ops.hipserve.prefill_gemm_f8(res, xq, xs, [w.parts[0].q], [w.parts[0].rs], 1)
    h = (_deq_x(xq, xs) @ wd.t()).to(torch.bfloat16).float()
    want = (h + res0.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(res.float(), want, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,I,K", [(300, 128, 512), (1000, 384, 1024), (2049, 256, 256)])
def test_prefill_gemm_f8_glu(M, I, K, act):
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(11 + M + I)
    w, wd = _weight(g, [I, I], K)
    x = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    xq, xs = pgemm.act_quant(x)
    out = torch.full((M, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_f8(out, xq, xs, [p.q for p in w.parts], [p.rs for p in w.parts],
                                       2 if act == "silu" else 3)
    gu = (_deq_x(xq, xs) @ wd.t()).to(torch.bfloat16).float()
    gate = gu[:, :I]
    f = torch.nn.functional.silu(gate) if act == "silu" else torch.nn.functional.gelu(gate, approximate="tanh")
    want = f * gu[:, I:]
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())


def test_quant_linear_prefill_uses_f8():
    """quant_linear at prefill sizes runs the FP8 MFMA path, not a bf16 shadow."""
    from hipserve.ops import quant as Q

    g = torch.Generator(device=DEV).manual_seed(1)
    w, wd = _weight(g, [512, 256, 256], 2048)
    assert w.dense is None
    x = (torch.rand(1024, 2048, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    y = Q.quant_linear(x, w)
    want = x.float() @ wd.t()
    rel = (y.float() - want).norm() / want.norm()
    assert rel < 5e-2, rel  # e4m3 activations: ~2.6 % RMS relative rounding per element


@pytest.mark.parametrize("mode", ["scratch", "resident"])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_f8_gemm_library_path_matches_kernel(epi, mode, monkeypatch):
    """On hipBLASLt's FP8 GEMM (row-wise scales) f8_gemm reads the plain e4m3 weight —
    re-laid out per call from the tiled decode copy into a scratch (default: the tiled
    copy stays the only resident one) or a resident plain copy — + the elementwise
    epilogue; it matches the hand-written e4m3 kernel on the same per-token activations
    (fp32 accumulation of exact e4m3 products, bf16 outputs within a rounding step)."""
    from hipserve.ops import pgemm, quant as Q

    g = torch.Generator(device=DEV).manual_seed(21 + epi)
    rows = [512, 512] if epi >= 2 else [512, 256, 256]
    w, wd = _weight(g, rows, 1024)
    x = _x(g, 1024, 1024)
    n = rows[0] if epi >= 2 else sum(rows)
    res0 = (torch.rand(1024, n, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    a = res0.clone() if epi == 1 else None
    a = pgemm.f8_gemm(x, w, epi, a)
    monkeypatch.setattr(Q, "FP8_LIB", mode)
    added = Q.make_fp8_plain([w], DEV, 0)
    assert w.f8_scale is not None and (added > 0) == (mode == "resident")
    assert (getattr(w, "f8_plain", None) is not None) == (mode == "resident")
    plain = Q.f8_lib_weight(w)
    assert torch.equal(plain.view(torch.uint8), torch.cat([Q.fp8_plain(p) for p in w.parts]))
    assert torch.equal(plain.float() * w.f8_scale.reshape(-1, 1), wd)
    b = res0.clone() if epi == 1 else None
    b = pgemm.f8_gemm(x, w, epi, b)
    torch.testing.assert_close(b.float(), a.float(), rtol=2e-2, atol=2e-2 * a.float().abs().max().item())


@pytest.mark.parametrize("N,K", [(16, 256), (272, 5376), (4096, 1024)])
def test_fp8_untile_inverts_tiling(N, K):
    """fp8_untile (tiled FP8 part -> row-major e4m3 bytes) against the torch permutation
    of quant.fp8_plain, on random bytes (every position distinct enough to catch a
    misplaced 16-byte piece)."""
    from hipserve.ops import quant as Q

    g = torch.Generator(device=DEV).manual_seed(N + K)
    q = torch.randint(0, 256, (N // 16, K // 256, 4096), device=DEV, dtype=torch.uint8, generator=g)
    p = Q.QuantPart(Q.FP8, N, K, q, None, None, 0, tiled=True)
    out = torch.full((N, K), 7, device=DEV, dtype=torch.uint8)
    torch.ops.hipserve.fp8_untile(out, q, N, K)
    assert torch.equal(out, Q.fp8_plain(p))


@pytest.mark.parametrize("M,K", [(7, 5376), (64, 21504), (33, 512), (100, 4096)])
def test_act_quant_fp8_register_path(M, K):
    """Decode batch sizes take the single-pass act_quant kernel (row held in registers);
    it quantises exactly like the two-pass kernel (same scale, same conversion)."""
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M + K)
    x = _x(g, M, K)
    xq, xs = pgemm.act_quant(x)
    # the same rows inside a >= 512-row batch run the two-pass kernel
    big = torch.cat([x, torch.zeros(512, K, device=DEV, dtype=x.dtype)])
    bq, bs = pgemm.act_quant(big)
    assert torch.equal(xq, bq[:M]) and torch.equal(xs, bs[:M])
    assert torch.equal(bs[M:], torch.ones(512, device=DEV))


@pytest.mark.parametrize("gelu", [False, True])
@pytest.mark.parametrize("M,I", [(5, 21504), (256, 4096), (1000, 14336), (64, 384)])
def test_glu_quant_is_glu_then_act_quant(gelu, M, I):
    """glu_quant ([gate | up] -> per-token e4m3 act, the FP8 down projection's input) is
    bit-identical to glu_and_mul followed by act_quant_fp8, and its optional bf16 act
    to glu_and_mul."""
    from hipserve.ops import pgemm

    g = torch.Generator(device=DEV).manual_seed(M + I + gelu)
    gu = (torch.randn(M, 2 * I, device=DEV, generator=g) * 3).to(torch.bfloat16)
    act = torch.empty(M, I, device=DEV, dtype=torch.bfloat16)
    (torch.ops.hipserve.gelu_and_mul if gelu else torch.ops.hipserve.silu_and_mul)(act, gu)
    xq, xs = pgemm.act_quant(act)
    q8 = torch.empty(M, I, device=DEV, dtype=torch.uint8)
    s8 = torch.empty(M, device=DEV, dtype=torch.float32)
    a2 = torch.empty_like(act)
    torch.ops.hipserve.glu_quant(a2, q8, s8, gu, gelu)
    assert torch.equal(a2, act) and torch.equal(q8, xq) and torch.equal(s8, xs)
    torch.ops.hipserve.glu_quant(None, q8, s8, gu, gelu)
    assert torch.equal(q8, xq)
