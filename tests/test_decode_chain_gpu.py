"""decode_chain (csrc/kernels/decode_chain.hip): producer GEMM -> residual add -> RMSNorm
-> consumer GEMM in one launch with in-launch hand-offs. Checked against the three-launch
chain it replaces (decode_gemm partials -> splitk_add_rmsnorm -> decode GEMM): the new
residual bit for bit, the consumer output within an ulp-level tolerance (only 1 / rms is
reassociated), and both against an fp32 PyTorch reference. Repeated and under a
concurrent stream's load, to catch stale hand-offs; the sync words must come back to
zero with no consumer having given up waiting."""
import pytest
import torch

from hipserve.ops import gemm, load_library

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS = 1e-5


@pytest.fixture(autouse=True, scope="module")
def _lib():
    load_library()


def _w(N, K, g, scale=0.02):
    return (torch.randn(N, K, device=DEV, generator=g) * scale).to(torch.bfloat16)


def _case(M, NA, KA, SA, NB, SB, glu, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    xa = torch.randn(M, KA, device=DEV, generator=g).to(torch.bfloat16)
    wa = _w(NA, KA, g)
    wb = _w(NB, NA, g)
    gamma = (torch.rand(NA, device=DEV, generator=g) + 0.5).to(torch.bfloat16)
    res0 = torch.randn(M, NA, device=DEV, generator=g).to(torch.bfloat16)
    return xa, wa, wb, gamma, res0


def _unfused(xa, wa_p, wb_p, gamma, res0, NA, SA, NB, SB, glu):
    op = torch.ops.hipserve
    M = xa.shape[0]
    wsa = torch.empty(SA * M * NA, device=DEV, dtype=torch.float32)
    op.decode_gemm_partial(wsa, xa, wa_p, NA, 1, SA, True)
    res = res0.clone()
    xn = torch.empty_like(res)
    op.splitk_add_rmsnorm(xn, res, wsa, SA, gamma, EPS)
    if glu:
        act = torch.empty(M, NB // 2, device=DEV, dtype=torch.bfloat16)
        op.decode_gemm_glu(act, xn, wb_p, torch.empty(0, device=DEV), NB, 1, 1)
        return res, act
    wsb = torch.empty(SB * M * NB, device=DEV, dtype=torch.float32)
    op.decode_gemm_partial(wsb, xn, wb_p, NB, 1, SB, True)
    return res, wsb.view(SB, M, NB).sum(0)


def _chain(xa, wa_p, wb_p, gamma, res, NA, SA, NB, SB, glu, sync):
    M = xa.shape[0]
    wsa = torch.empty(SA * M * NA, device=DEV, dtype=torch.float32)
    sq = torch.empty(NA // 128 * 64, device=DEV, dtype=torch.float32)
    if glu:
        act = torch.empty(M, NB // 2, device=DEV, dtype=torch.bfloat16)
        wsb = torch.empty(0, device=DEV)
    else:
        act = torch.empty(0, device=DEV, dtype=torch.bfloat16)
        wsb = torch.empty(SB * M * NB, device=DEV, dtype=torch.float32)
    torch.ops.hipserve.decode_chain(act, wsb, res, wsa, sq, sync, xa, wa_p, wb_p, gamma, SA, NB, SB, glu, EPS)
    return act if glu else wsb.view(SB, M, NB).sum(0)


def _fp32(xa, wa, wb, gamma, res0, glu):
    h = res0.float() + xa.float() @ wa.float().t()
    x = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + EPS) * gamma.float()
    y = x @ wb.float().t()
    if glu:
        I = y.shape[1] // 2
        y = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    return h, y


SHAPES = [
    # M, NA, KA, SA, NB, SB, glu
    (64, 4096, 4096, 8, 16384, 1, True),     # o_proj -> ln2 -> gate|up (Llama-3-8B widths, I = 8192)
    (64, 4096, 14336, 8, 6144, 4, False),    # down -> next ln1 -> qkv partials (Llama-3-8B)
    (48, 2048, 4096, 4, 8192, 2, False),
    (20, 4096, 4096, 8, 8192, 1, True),      # 17-32 rows: the 32-row body
    (33, 1024, 1792, 1, 4096, 1, True),      # K slice 7 steps, one slice
]


@pytest.mark.parametrize("M,NA,KA,SA,NB,SB,glu", SHAPES)
def test_decode_chain_matches_unfused(M, NA, KA, SA, NB, SB, glu):
    op = torch.ops.hipserve
    assert op.decode_chain_ok(M, NA, KA, SA, NB, SB, glu)
    xa, wa, wb, gamma, res0 = _case(M, NA, KA, SA, NB, SB, glu, M * 131 + NA + NB)
    wa_p, wb_p = gemm.pack(wa), gemm.pack(wb, glu=glu)
    # the glu packing pairs gate row i with up row i: the logical weight is [gate; up]
    res_u, out_u = _unfused(xa, wa_p, wb_p, gamma, res0, NA, SA, NB, SB, glu)
    sync = torch.zeros(4096, device=DEV, dtype=torch.int32)
    res = res0.clone()
    out = _chain(xa, wa_p, wb_p, gamma, res, NA, SA, NB, SB, glu, sync)
    torch.cuda.synchronize()
    assert torch.equal(res, res_u), "new residual must equal splitk_add_rmsnorm's bit for bit"
    d = (out.float() - out_u.float()).abs()
    scale = out_u.float().abs().max().item()
    assert d.max().item() <= 0.02 * scale, (d.max().item(), scale)
    assert (d > 1e-3 * scale).float().mean().item() < 0.02
    h32, y32 = _fp32(xa, wa, wb, gamma, res0, glu)
    assert (res.float() - h32).abs().max().item() <= 0.05 * h32.abs().max().item()
    e = (out.float() - y32).abs().max().item()
    assert e <= 0.03 * y32.abs().max().item() + 1e-3, e
    s = sync.cpu()
    assert s[64].item() == 0, "a consumer gave up waiting"
    assert s.abs().sum().item() == 0, "sync words must reset"


@pytest.mark.parametrize("M,NA,KA,SA,NB,SB,glu", [SHAPES[0], SHAPES[1]])
def test_decode_chain_repeated_under_load(M, NA, KA, SA, NB, SB, glu):
    """60 back-to-back launches (same buffers, sync words reused), half of them while
    another stream runs GEMMs (uneven CU load): every launch equals the first."""
    xa, wa, wb, gamma, res0 = _case(M, NA, KA, SA, NB, SB, glu, 7 + M)
    wa_p, wb_p = gemm.pack(wa), gemm.pack(wb, glu=glu)
    sync = torch.zeros(4096, device=DEV, dtype=torch.int32)
    res = res0.clone()
    first = _chain(xa, wa_p, wb_p, gamma, res, NA, SA, NB, SB, glu, sync).clone()
    res_first = res.clone()
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16) * 0.01
    b = torch.empty_like(a)
    side.wait_stream(torch.cuda.current_stream())
    outs = []
    for i in range(60):
        res.copy_(res0)
        if i % 2:
            with torch.cuda.stream(side):  # side-stream buffers only: no cross-stream reuse
                for _ in range(3):
                    torch.mm(a, a, out=b)
        outs.append((_chain(xa, wa_p, wb_p, gamma, res, NA, SA, NB, SB, glu, sync).clone(), res.clone()))
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(outs):
        assert torch.equal(r, res_first), f"launch {i}: residual differs"
        assert torch.equal(o, first), f"launch {i}: output differs"
    s = sync.cpu()
    assert s[64].item() == 0 and s.abs().sum().item() == 0


def test_decode_chain_graph_replay():
    """Captured once, replayed: the kernel resets its own counters, so every replay
    reduces and hands off again."""
    M, NA, KA, SA, NB, SB, glu = SHAPES[0]
    xa, wa, wb, gamma, res0 = _case(M, NA, KA, SA, NB, SB, glu, 99)
    wa_p, wb_p = gemm.pack(wa), gemm.pack(wb, glu=glu)
    sync = torch.zeros(4096, device=DEV, dtype=torch.int32)
    res = res0.clone()
    want = _chain(xa, wa_p, wb_p, gamma, res, NA, SA, NB, SB, glu, sync).clone()
    want_res = res.clone()
    wsa = torch.empty(SA * M * NA, device=DEV, dtype=torch.float32)
    sq = torch.empty(NA // 128 * 64, device=DEV, dtype=torch.float32)
    act = torch.empty(M, NB // 2, device=DEV, dtype=torch.bfloat16)
    e = torch.empty(0, device=DEV)
    res.copy_(res0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            torch.ops.hipserve.decode_chain(act, e, res, wsa, sq, sync, xa, wa_p, wb_p, gamma, SA, NB, SB, glu, EPS)
    for _ in range(10):
        res.copy_(res0)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(res, want_res) and torch.equal(act, want)
    assert sync.abs().sum().item() == 0
