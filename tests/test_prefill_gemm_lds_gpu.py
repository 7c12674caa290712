"""Prefill GEMM over the packed decode-weight layout with both operands staged by LDS-DMA
(csrc/kernels/prefill_gemm_lds.hip) vs a plain PyTorch fp32 reference of the same op:
plain store (+ bias), residual add, SiLU / GELU GLU, the grouped MoE mode over
moe_align's 256-row expert tiles; ragged M (below one 256-row tile, not a multiple of
it), N not a multiple of 128 (zero-padded packed rows) or of the 256-column tile (waves
past the last packed tile), K from one 256-deep packed step up (8 K steps: the LDS ring's
shortest pipeline), strided x. Asymmetric random operands catch transposed fragments and
swizzles; a NaN-filled output catches unwritten and out-of-range writes."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    from hipserve.ops import load_library

    load_library()


def _rnd(g, *s, scale=1.0):
    return ((torch.rand(*s, device=DEV, generator=g) * 2 - 1) * scale).to(torch.bfloat16)


def _pack(w, glu=False):
    N, K = w.shape
    wp = torch.empty(-(-N // 128) * 128 * K, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.pack_decode_weight(wp, w, glu)
    return wp


SHAPES = [(256, 256, 256), (300, 640, 1024), (1000, 200, 512), (77, 1536, 768), (2049, 384, 2048),
          (1, 128, 256), (8192, 512, 4096), (513, 4096, 14336)]


@pytest.mark.parametrize("var", [0, 1, 2, 3, 4])  # 8 waves: ring 4 / 5 slots, setprio off / on; 4: 4 waves
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_lds_store(M, N, K, var):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_lds(out, x, _pack(w), N, 0, variant=var)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


def test_lds_identity_asymmetric():
    """x = I (rows 0..255 of the identity) against an asymmetric W: out = W^T exactly, so
    a swapped fragment, a wrong swizzle or a transposed store shows as a moved value."""
    K, N = 256, 384
    x = torch.eye(256, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K) % 251 - 125).to(torch.bfloat16)
    out = torch.full((256, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_lds(out, x, _pack(w), N, 0)
    assert torch.equal(out, w.t()[:256].contiguous())
    out.fill_(float("nan"))
    torch.ops.hipserve.prefill_gemm_lds(out, x, _pack(w), N, 0, variant=4)
    assert torch.equal(out, w.t()[:256].contiguous())


def test_lds_store_bias_and_strided_x():
    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, K = 700, 896, 512
    xb = _rnd(g, M, K + 64)
    x = xb[:, 32:32 + K]  # row stride K + 64
    w, b = _rnd(g, N, K, scale=0.05), _rnd(g, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_lds(out, x, _pack(w), N, 0, b)
    want = x.float() @ w.float().t() + b.float()
    torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


@pytest.mark.parametrize("var", [0, 4])
@pytest.mark.parametrize("M,N,K", [(300, 512, 1024), (1000, 384, 512), (2049, 1024, 256), (8192, 4096, 4096)])
def test_lds_residual_add(M, N, K, var):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    res0 = _rnd(g, M, N)
    res = res0.clone()
    torch.ops.hipserve.prefill_gemm_lds(res, x, _pack(w), N, 1, variant=var)
    h = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    want = (h + res0.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(res.float(), want, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("var", [0, 4])
@pytest.mark.parametrize("act", ["silu", "gelu"])
@pytest.mark.parametrize("M,I,K", [(300, 256, 1024), (1000, 192, 512), (2049, 64, 256), (513, 1344, 768),
                                   (4096, 14336, 4096)])
def test_lds_glu(M, I, K, act, var):
    g = torch.Generator(device=DEV).manual_seed(11 + M)
    x, w = _rnd(g, M, K), _rnd(g, 2 * I, K, scale=0.05)
    out = torch.full((M, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_lds(out, x, _pack(w, glu=True), 2 * I, 2 if act == "silu" else 3, variant=var)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    want = f(gu[:, :I]) * gu[:, I:]
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())


@pytest.mark.parametrize("var", [0, 1, 2, 3, 4])
def test_lds_repeat_is_deterministic(var):
    """Back-to-back launches give bit-identical outputs (a DMA / read race would show as
    rare differing tiles), the same in every ring / priority variant."""
    g = torch.Generator(device=DEV).manual_seed(21)
    M, N, K = 4096, 2048, 2048
    x, wp = _rnd(g, M, K), _pack(_rnd(g, N, K, scale=0.05))
    ref = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_lds(ref, x, wp, N, 0, variant=0)
    out = torch.empty_like(ref)
    for _ in range(20):
        torch.ops.hipserve.prefill_gemm_lds(out, x, wp, N, 0, variant=var)
        assert torch.equal(out, ref)


@pytest.mark.parametrize("var", [0, 4])
@pytest.mark.parametrize("E,I,K,glu", [(8, 512, 1024, True), (8, 256, 512, False), (16, 128, 256, True)])
def test_lds_grouped_moe(E, I, K, glu, var):
    """Grouped expert GEMM over moe_align's expert-sorted 256-row tiles with each expert's
    weight in the packed decode layout, the valid tile count read on the device, vs a
    per-expert fp32 reference."""
    g = torch.Generator(device=DEV).manual_seed(E + I + K)
    T, k = 700, 2
    ids = torch.stack([torch.randperm(E, device=DEV, generator=g)[:k] for _ in range(T)]).int()
    N = 2 * I if glu else I
    w = _rnd(g, E, N, K, scale=0.05)
    wp = torch.stack([_pack(w[e], glu) for e in range(E)])
    x = _rnd(g, T, K)
    op = torch.ops.hipserve
    P, tile = T * k, 256
    cap = -(-(P + E * (tile - 1)) // tile) * tile
    slots = torch.empty(cap, dtype=torch.int32, device=DEV)
    tile_expert = torch.empty(cap // tile, dtype=torch.int32, device=DEV)
    ntiles = torch.empty(1, dtype=torch.int32, device=DEV)
    pair_slot = torch.empty(P, dtype=torch.int32, device=DEV)
    ends = torch.empty(E, dtype=torch.int32, device=DEV)
    op.moe_align(ids, E, tile, slots, tile_expert, ntiles, pair_slot, ends)
    xs = torch.empty(cap, K, dtype=torch.bfloat16, device=DEV)
    op.moe_gather(xs, x, slots, k)
    out = torch.full((cap, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    op.prefill_gemm_lds(out, xs, wp, N, 2 if glu else 0, None, tile_expert, ntiles, var)
    ps = pair_slot.long()
    for p in range(0, P, 37):  # a spread of pairs
        t, j = p // k, p % k
        e = int(ids[t, j])
        h = x[t].float() @ w[e].float().t()
        if glu:
            h = h.to(torch.bfloat16).float()
            want = torch.nn.functional.silu(h[:I]) * h[I:]
        else:
            want = h
        torch.testing.assert_close(out[ps[p]].float(), want, rtol=2e-2, atol=2e-2 * max(1.0, want.abs().max().item()))


def test_lds_rejects_bad_shapes():
    g = torch.Generator(device=DEV).manual_seed(3)
    x = _rnd(g, 64, 320)
    out = torch.empty(64, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):  # K % 256
        torch.ops.hipserve.prefill_gemm_lds(out, x, torch.empty(128 * 320, device=DEV, dtype=torch.bfloat16), 128, 0)
