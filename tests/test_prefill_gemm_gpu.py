"""Hand-written prefill GEMM (csrc/kernels/prefill_gemm.hip) vs a plain PyTorch fp32
reference of the same op: plain store, residual add and the SiLU-GLU epilogue, on
ragged row counts (M not a multiple of the 256-row tile) and K from one 64-deep tile
up. Asymmetric random operands catch transposed fragments / swizzles."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _lib():
    from hipserve.ops import load_library

    load_library()

SHAPES = [(256, 256, 64), (300, 512, 1024), (1000, 768, 2048), (2049, 1280, 512), (64, 1024, 4096),
          (8192, 512, 4096)]


def _rnd(g, *s, scale=1.0):
    return ((torch.rand(*s, device=DEV, generator=g) * 2 - 1) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("variant", [2])
@pytest.mark.parametrize("M,N,K", SHAPES + [(512, 256, 128), (700, 512, 192)])
def test_prefill_gemm_store(M, N, K, variant):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm(out, x, w, 0, variant)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


@pytest.mark.parametrize("variant", [2])
@pytest.mark.parametrize("M,N,K", SHAPES[:4])
def test_prefill_gemm_residual_add(M, N, K, variant):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    res0 = _rnd(g, M, N)
    res = res0.clone()
    torch.ops.hipserve.prefill_gemm(res, x, w, 1, variant)
    h = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    want = (h + res0.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(res.float(), want, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("variant,act", [(2, "silu"), (2, "gelu")])
@pytest.mark.parametrize("M,I,K", [(300, 256, 1024), (1000, 384, 512), (2049, 128, 256)])
def test_prefill_gemm_glu(M, I, K, variant, act):
    g = torch.Generator(device=DEV).manual_seed(11 + M)
    x, w = _rnd(g, M, K), _rnd(g, 2 * I, K, scale=0.05)
    out = torch.full((M, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm(out, x, w, 2 if act == "silu" else 3, variant)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    want = f(gu[:, :I]) * gu[:, I:]
    act = out
    torch.testing.assert_close(act.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())


@pytest.mark.parametrize("E,I,K,glu", [(8, 512, 1024, True), (8, 256, 512, False), (16, 128, 256, True)])
def test_prefill_gemm_grouped_moe(E, I, K, glu):
    """Grouped expert GEMM over moe_align's 256-row expert tiles (device offsets, no
    host sync) vs a per-expert fp32 reference."""
    g = torch.Generator(device=DEV).manual_seed(E + I + K)
    T, k = 700, 2
    ids = torch.stack([torch.randperm(E, device=DEV, generator=g)[:k] for _ in range(T)]).int()
    N = 2 * I if glu else I
    w = _rnd(g, E, N, K, scale=0.05)
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
    op.prefill_gemm_grouped(out, xs, w, tile_expert, 2 if glu else 0)
    ps = pair_slot.long()
    for p in range(0, P, 37):  # check a spread of pairs
        t, j = p // k, p % k
        e = int(ids[t, j])
        h = x[t].float() @ w[e].float().t()
        if glu:
            h = h.to(torch.bfloat16).float()
            want = torch.nn.functional.silu(h[:I]) * h[I:]
        else:
            want = h
        torch.testing.assert_close(out[ps[p]].float(), want, rtol=2e-2, atol=2e-2 * max(1.0, want.abs().max().item()))
