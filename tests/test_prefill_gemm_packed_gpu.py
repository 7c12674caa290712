"""Prefill GEMM over the packed decode-weight layout (csrc/kernels/prefill_gemm_packed.hip)
vs a plain PyTorch fp32 reference of the same op: plain store (+ bias), residual add and
the SiLU / GELU GLU epilogues, both workgroup shapes (wm = 1: 128 x 512, wm = 2: 256 x 256),
ragged M (not a multiple of the row tile, and fewer rows than one tile), N that is not a
multiple of 128 (zero-padded packed rows) or of the workgroup's 512 / 256 columns (waves
past the last weight tile), K from one 256-deep packed step up. Asymmetric random
operands catch transposed fragments and swizzles."""
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


SHAPES = [(256, 512, 256), (300, 640, 1024), (1000, 200, 512), (77, 1536, 768), (2049, 384, 2048),
          (1, 128, 256), (8192, 512, 4096)]


# grid: 0 = persistent (one workgroup per CU walking the tiles), 3 = three workgroups
# walking many tiles each (uneven counts), 1 << 30 = one tile per workgroup
@pytest.mark.parametrize("rw", [2, 4])  # weight slots in flight
@pytest.mark.parametrize("grid", [0, 3, 1 << 30])
@pytest.mark.parametrize("wm", [1, 2])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_packed_store(M, N, K, wm, grid, rw):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_packed(out, x, _pack(w), N, 0, None, wm, grid, rw)
    want = x.float() @ w.float().t()
    torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


@pytest.mark.parametrize("wm", [1, 2])
def test_packed_store_bias_and_strided_x(wm):
    g = torch.Generator(device=DEV).manual_seed(5)
    M, N, K = 700, 896, 512
    xb = _rnd(g, M, K + 64)
    x = xb[:, 32:32 + K]  # row stride K + 64
    w, b = _rnd(g, N, K, scale=0.05), _rnd(g, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_packed(out, x, _pack(w), N, 0, b, wm)
    want = x.float() @ w.float().t() + b.float()
    torch.testing.assert_close(out.float(), want, rtol=1e-2, atol=1e-2 * want.abs().max().item())


@pytest.mark.parametrize("wm", [1, 2])
@pytest.mark.parametrize("M,N,K", [(300, 512, 1024), (1000, 384, 512), (2049, 1024, 256)])
def test_packed_residual_add(M, N, K, wm):
    g = torch.Generator(device=DEV).manual_seed(7 + M)
    x, w = _rnd(g, M, K), _rnd(g, N, K, scale=0.05)
    res0 = _rnd(g, M, N)
    res = res0.clone()
    torch.ops.hipserve.prefill_gemm_packed(res, x, _pack(w), N, 1, None, wm, 7, 4)  # 7 workgroups: many tiles each
    h = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    want = (h + res0.float()).to(torch.bfloat16).float()
    torch.testing.assert_close(res.float(), want, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("rw", [2, 4])
@pytest.mark.parametrize("grid", [0, 5])
@pytest.mark.parametrize("wm,act", [(1, "silu"), (2, "silu"), (1, "gelu"), (2, "gelu")])
@pytest.mark.parametrize("M,I,K", [(300, 256, 1024), (1000, 192, 512), (2049, 64, 256), (513, 1344, 768)])
def test_packed_glu(M, I, K, wm, act, grid, rw):
    g = torch.Generator(device=DEV).manual_seed(11 + M)
    x, w = _rnd(g, M, K), _rnd(g, 2 * I, K, scale=0.05)
    out = torch.full((M, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.prefill_gemm_packed(out, x, _pack(w, glu=True), 2 * I, 2 if act == "silu" else 3, None, wm,
                                           grid, rw)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    want = f(gu[:, :I]) * gu[:, I:]
    torch.testing.assert_close(out.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())


def test_packed_rejects_bad_shapes():
    g = torch.Generator(device=DEV).manual_seed(3)
    x, w = _rnd(g, 64, 320), _rnd(g, 128, 320)
    out = torch.empty(64, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):  # K % 256
        torch.ops.hipserve.prefill_gemm_packed(out, x, torch.empty(128 * 320, device=DEV, dtype=torch.bfloat16),
                                               128, 0, None, 1)


@pytest.mark.parametrize("gather", [False, True])
@pytest.mark.parametrize("wm", [1, 2])
@pytest.mark.parametrize("E,I,K,glu", [(8, 512, 1024, True), (8, 256, 512, False), (16, 128, 256, True)])
def test_packed_grouped_moe(E, I, K, glu, wm, gather):
    """Grouped expert GEMM over moe_align's expert-sorted (128 * wm)-row tiles with each
    expert's weight in the packed decode layout (moe_packed: w13 GLU-interleaved), the
    valid tile count read on the device, vs a per-expert fp32 reference."""
    g = torch.Generator(device=DEV).manual_seed(E + I + K)
    T, k = 700, 2
    ids = torch.stack([torch.randperm(E, device=DEV, generator=g)[:k] for _ in range(T)]).int()
    N = 2 * I if glu else I
    w = _rnd(g, E, N, K, scale=0.05)
    wp = torch.stack([_pack(w[e], glu) for e in range(E)])
    x = _rnd(g, T, K)
    op = torch.ops.hipserve
    P, tile = T * k, 128 * wm
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
    op.prefill_gemm_packed_grouped(out, xs, wp, N, 2 if glu else 0, tile_expert, ntiles, wm)
    if gather:  # token rows read through the slot table inside the GEMM (moe_gather fused): bit-identical
        used = torch.arange(cap, device=DEV) < int(ntiles.item()) * tile
        fused = torch.full_like(out, float("nan"))
        op.prefill_gemm_packed_grouped(fused, x, wp, N, 2 if glu else 0, tile_expert, ntiles, wm, 4, slots, k)
        assert torch.equal(fused[used], out[used])
        assert bool((fused[used & (slots < 0)] == 0).all())  # padding slots multiply zero rows
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


@pytest.mark.parametrize("T,k,E,tile", [(700, 2, 8, 128), (8192, 8, 128, 128), (20000, 2, 8, 128), (9000, 8, 60, 16)])
def test_moe_align_layout(T, k, E, tile):
    """moe_align (single workgroup below 16K pairs, per-block histograms + scatter above):
    every pair has exactly one slot inside its expert's tile-padded segment, segments are in
    expert order, padding slots are -1, and the tile table / tile count / group ends match
    a host recount."""
    g = torch.Generator(device=DEV).manual_seed(T + E)
    logits = torch.randn(T, E, device=DEV, generator=g)
    ids = logits.topk(k, dim=-1).indices.int().contiguous()
    P = T * k
    cap = -(-(P + E * (tile - 1)) // tile) * tile
    op = torch.ops.hipserve
    slots = torch.empty(cap, dtype=torch.int32, device=DEV)
    tile_expert = torch.empty(cap // tile, dtype=torch.int32, device=DEV)
    ntiles = torch.empty(1, dtype=torch.int32, device=DEV)
    pair_slot = torch.empty(P, dtype=torch.int32, device=DEV)
    ends = torch.empty(E, dtype=torch.int32, device=DEV)
    op.moe_align(ids, E, tile, slots, tile_expert, ntiles, pair_slot, ends)
    flat = ids.view(-1).long().cpu()
    cnt = torch.bincount(flat, minlength=E)
    padded = (cnt + tile - 1) // tile * tile
    off = torch.cumsum(padded, 0) - padded
    assert int(ntiles.item()) == int(padded.sum()) // tile
    assert torch.equal(ends.cpu().long(), off + padded)
    s, ps, te = slots.cpu().long(), pair_slot.cpu().long(), tile_expert.cpu().long()
    assert torch.equal(s[ps], torch.arange(P))  # slots[pair_slot[p]] == p: a bijection on the real slots
    e_of = flat
    assert bool(((ps >= off[e_of]) & (ps < off[e_of] + cnt[e_of])).all())  # inside its expert's segment
    real = torch.zeros(cap, dtype=torch.bool)
    real[ps] = True
    assert bool((s[~real] == -1).all())
    want_te = torch.full((cap // tile,), -1, dtype=torch.long)
    for e in range(E):
        want_te[int(off[e]) // tile:int(off[e] + padded[e]) // tile] = e
    assert torch.equal(te, want_te)
