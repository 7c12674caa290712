"""Numerics of every gfx950 kernel against the fp32 PyTorch reference."""
import math

import pytest
import torch

from hipserve.ops import KernelOps
from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    return KernelOps()


def _close(a, b, atol, rtol=0.0, frac=1.0):
    a, b = a.float().cpu(), b.float().cpu()
    bad = (a - b).abs() > (atol + rtol * b.abs())
    assert bad.float().mean().item() <= 1.0 - frac, f"max err {(a - b).abs().max().item()}"


@pytest.mark.parametrize("rows,hidden", [(7, 4096), (33, 8192), (3, 2048), (1, 64)])
@pytest.mark.parametrize("wf32", [False, True])
def test_rmsnorm(ops, rows, hidden, wf32):
    torch.manual_seed(0)
    x = torch.randn(rows, hidden, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(hidden, device=DEV, dtype=torch.float32 if wf32 else torch.bfloat16)
    out = torch.empty_like(x)
    ops.rmsnorm(out, x, w, 1e-5)
    _close(out, ref.rmsnorm(x.cpu(), w.cpu(), 1e-5), atol=2e-2, rtol=1e-2)
    # fused add
    r = torch.randn_like(x)
    r_ref = r.clone().cpu()
    ops.fused_add_rmsnorm(out, x, r, w, 1e-5)
    y_ref, rr = ref.fused_add_rmsnorm(x.cpu(), r_ref, w.cpu(), 1e-5)
    _close(r, rr, atol=1e-6)
    _close(out, y_ref, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("rows,inter", [(5, 14336), (64, 1792), (1, 8)])
def test_silu_and_mul(ops, rows, inter):
    x = torch.randn(rows, 2 * inter, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(rows, inter, device=DEV, dtype=torch.bfloat16)
    ops.silu_and_mul(out, x)
    _close(out, ref.silu_and_mul(x.cpu()), atol=1e-2, rtol=1e-2)


def _caches(nblocks, nkv, bs, D, fill=True):
    kc = torch.randn(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16) if fill else \
        torch.zeros(nblocks, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn(nblocks, nkv, D, bs, device=DEV, dtype=torch.bfloat16) if fill else \
        torch.zeros(nblocks, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    return kc, vc


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("T,layout", [(37, "random"), (300, "random"), (300, "contig"), (1000, "contig"),
                                      (300, "aligned"), (2500, "random"), (2500, "contig"), (2100, "aligned")])
def test_rope_cache(ops, mode, bs, T, layout):
    """Per-token kernel (T < 2048) and the 16-token tile kernel of prefill chunks
    (LDS-staged V, token-fastest V^T stores), scattered and contiguous slots
    (contig: a chunk starting mid-block; aligned: block-aligned, so whole tiles take the
    16-byte V^T store path), vs the fp32 oracle."""
    torch.manual_seed(1)
    nq, nkv, D = 32, 8, 128
    qkv = torch.randn(T, (nq + 2 * nkv) * D + 64, device=DEV, dtype=torch.bfloat16)[:, : (nq + 2 * nkv) * D]
    pos = torch.randint(0, 4000, (T,), device=DEV)
    nblk = max(64, (T + 2 * bs) // bs + 1)
    if layout == "random":
        slots = torch.randperm(nblk * bs, device=DEV)[:T]
    else:
        slots = torch.arange(T, device=DEV) + (5 if layout == "contig" else bs)
    slots[3] = -1
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    kc, vc = _caches(nblk, nkv, bs, D, fill=False)
    kc_r, vc_r, qkv_r = kc.cpu().clone(), vc.cpu().clone(), qkv.cpu().clone()
    ops.rope_cache(qkv, pos, slots, cs, kc, vc, nq, nkv, D, mode)
    ref.rope_cache(qkv_r, pos.cpu(), slots.cpu(), cs.cpu(), kc_r, vc_r, nq, nkv, D, mode)
    _close(qkv[:, : nq * D], qkv_r[:, : nq * D], atol=2e-2, rtol=1e-2)
    _close(kc, kc_r, atol=2e-2, rtol=1e-2)
    _close(vc, vc_r, atol=0)


@pytest.mark.parametrize("nq,nkv,D", [(32, 8, 128), (64, 8, 128), (32, 32, 64), (32, 4, 64), (32, 32, 96)])
@pytest.mark.parametrize("bs", [16, 32])
@pytest.mark.parametrize("part", [512, 2048])
@pytest.mark.parametrize("window", [0, 100])
def test_paged_decode(ops, nq, nkv, D, bs, part, window):
    """Split-K paged decode (incl. head_dim 96 and sliding-window layers: keys
    [ctx - window, ctx)) vs the fp32 oracle."""
    torch.manual_seed(2)
    ctx = [1, 17, 100, 600, 1300, 512, 33]
    B = len(ctx)
    max_blocks = 96
    nblocks = B * max_blocks
    kc, vc = _caches(nblocks, nkv, bs, D)
    perm = torch.randperm(nblocks, device=DEV).int()
    bt = perm.view(B, max_blocks).contiguous()
    cl = torch.tensor(ctx, device=DEV, dtype=torch.int32)
    q = torch.randn(B, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
    max_parts = math.ceil(max_blocks * bs / part)
    tmp_out = torch.empty(B, nq, max_parts, D, device=DEV, dtype=torch.float32)
    tmp_ml = torch.empty(B, nq, max_parts, 2, device=DEV, dtype=torch.float32)
    out = torch.zeros(B, nq * D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    out16 = torch.full((B, nq * D), float("nan"), device=DEV, dtype=torch.float16)
    ops.paged_decode(out, q, kc, vc, bt, cl, tmp_out, tmp_ml, nq, nkv, part, scale, window, out16)
    want = ref.paged_decode(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cl.cpu(), nq, nkv, scale, window)
    _close(out.view(B, nq, D), want, atol=2e-2, rtol=2e-2)
    # out16: the f16 pair-order copy {0, 2, 1, 3, 4, 6, 5, 7} of the bf16 output, exactly
    # (one- and multi-partition sequences: the attention and the merge kernel write it)
    h = out.float().to(torch.float16).view(B, -1, 8)[:, :, [0, 2, 1, 3, 4, 6, 5, 7]].reshape(B, -1)
    assert torch.equal(out16, h)


@pytest.mark.parametrize("nq,nkv,D,bs,v1", [(32, 8, 128, 16, False), (32, 8, 128, 16, True), (64, 8, 128, 16, False),
                                          (8, 1, 128, 32, False), (16, 8, 128, 16, False), (16, 2, 64, 16, False),
                                          (4, 4, 128, 16, False), (8, 8, 96, 16, False)])
@pytest.mark.parametrize("waves", ["4", "8"])
@pytest.mark.parametrize("window", [0, 200])
def test_prefill_attention(ops, nq, nkv, D, bs, v1, waves, window, monkeypatch):
    """v2 (LDS-shared K/V, GQA heads per workgroup: G = 2/4/8) and v1 (D = 64, MHA,
    or HIPSERVE_PREFILL_ATTN_V1) against the fp32 oracle, including long prompts
    (many 64-key tiles: the lazy rescale) and chunked prefill over a prefix."""
    monkeypatch.setenv("HIPSERVE_PREFILL_ATTN_V1", "1" if v1 else "0")
    monkeypatch.setenv("HIPSERVE_PREFILL_ATTN_WAVES", waves)
    torch.manual_seed(3)
    # (ctx_len, q_len): plain prefill, tiny, chunked prefill with prefix context, long
    seqs = [(1, 1), (37, 37), (200, 200), (300, 50), (129, 129), (1100, 1100), (1500, 333)]
    max_blocks = 1536 // bs
    nblocks = len(seqs) * max_blocks
    kc, vc = _caches(nblocks, nkv, bs, D)
    bt = torch.randperm(nblocks, device=DEV).int().view(len(seqs), max_blocks).contiguous()
    cu = [0]
    tiles = []
    for i, (c, ql) in enumerate(seqs):
        for r in range(0, ql, 128):
            tiles.append((i, r))
        cu.append(cu[-1] + ql)
    T = cu[-1]
    q = torch.randn(T, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16) * 2
    cu_t = torch.tensor(cu, device=DEV, dtype=torch.int32)
    ctx_t = torch.tensor([c for c, _ in seqs], device=DEV, dtype=torch.int32)
    tiles_t = torch.tensor(tiles, device=DEV, dtype=torch.int32)
    out = torch.zeros(T, nq * D, device=DEV, dtype=torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    ops.prefill_attention(out, q, kc, vc, bt, cu_t, ctx_t, tiles_t, nq, nkv, scale, window)
    want = ref.prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), cu_t.cpu(), ctx_t.cpu(), nq, nkv, scale,
                                 window)
    _close(out.view(T, nq, D), want, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,nq,nkv,D", [(37, 16, 8, 128), (5, 32, 4, 64), (64, 8, 8, 96), (3, 8, 2, 256)])
def test_qk_rmsnorm(ops, T, nq, nkv, D):
    """Per-head q/k RMSNorm in place inside the qkv rows; v untouched."""
    torch.manual_seed(11)
    W = (nq + 2 * nkv) * D
    qkv = torch.randn(T, W + 32, device=DEV, dtype=torch.bfloat16)[:, :W]
    qw = torch.rand(D, device=DEV) + 0.5
    kw = torch.rand(D, device=DEV) + 0.5
    want = qkv.cpu().clone()
    ref.qk_rmsnorm(want, qw.cpu(), kw.cpu(), nq, nkv, D, 1e-6)
    ops.qk_rmsnorm(qkv, qw, kw, nq, nkv, D, 1e-6)
    _close(qkv[:, : (nq + nkv) * D], want[:, : (nq + nkv) * D], atol=2e-2, rtol=1e-2)
    assert torch.equal(qkv[:, (nq + nkv) * D:].cpu(), want[:, (nq + nkv) * D:])


@pytest.mark.parametrize("rows,inter", [(5, 21504), (64, 1792), (1, 8)])
def test_gelu_and_mul(ops, rows, inter):
    x = torch.randn(rows, 2 * inter, device=DEV, dtype=torch.bfloat16) * 2
    out = torch.empty(rows, inter, device=DEV, dtype=torch.bfloat16)
    ops.gelu_and_mul(out, x)
    _close(out, ref.gelu_and_mul(x.cpu()), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sample(ops, dtype):
    torch.manual_seed(4)
    B, V = 12, 32000
    logits = (torch.randn(B, V, device=DEV) * 3).to(dtype)
    temp = torch.tensor([0.0, 1.0, 0.7, 1.0, 1.3, 0.9, 1.0, 0.5, 1.0, 2.0, 0.0, 1.0], device=DEV)
    top_k = torch.tensor([0, 0, 50, 1, 0, 20, 0, 0, 1000, 5, 0, 7], device=DEV, dtype=torch.int32)
    top_p = torch.tensor([1.0, 1.0, 1.0, 1.0, 0.9, 0.5, 0.1, 0.95, 0.8, 1.0, 1.0, 0.3], device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.long) * 7919 + 1
    steps = torch.arange(B, device=DEV, dtype=torch.long)
    tok = torch.empty(B, device=DEV, dtype=torch.long)
    lp = torch.empty(B, device=DEV, dtype=torch.float32)
    ops.sample(tok, lp, logits, temp, top_k, top_p, seeds, steps)
    rt, rlp = ref.sample(logits.cpu(), temp.cpu(), top_k.cpu(), top_p.cpu(), seeds.cpu(), steps.cpu())
    mism = (tok.cpu() != rt).sum().item()
    assert mism <= 1, (tok.cpu(), rt)
    ok = tok.cpu() == rt
    assert torch.allclose(lp.cpu()[ok], rlp[ok], atol=1e-3)
    # greedy rows must be exact
    assert tok[0].item() == int(logits[0].float().argmax())
    assert tok[3].item() == int(logits[3].float().argmax())  # top_k = 1


@pytest.mark.parametrize("V,scale", [(128256, 3.0), (128256, 0.05), (32000, 1.0), (9000, 8.0)])
def test_sample_multicu(ops, V, scale):
    """Multi-CU sampler (vocab >= 8192) vs the reference: greedy, temperature,
    top-k, top-p, both (incl. the nucleus moving past the top-k bin), and a
    clustered row (scale 0.05: nearly flat distribution, heavy key ties)."""
    torch.manual_seed(V + int(scale * 100))
    B = 14
    logits = (torch.randn(B, V, device=DEV) * scale).to(torch.bfloat16)
    logits[5, 1000:1010] = 30.0   # a very peaked row
    temp = torch.tensor([0.0, 1.0, 0.7, 1.0, 1.3, 0.9, 1.0, 0.5, 1.0, 2.0, 0.8, 1.0, 0.8, 1.1], device=DEV)
    top_k = torch.tensor([0, 0, 50, 1, 0, 20, 0, 0, 1000, 5, 0, 7, 40000, 3000], device=DEV, dtype=torch.int32)
    top_p = torch.tensor([1.0, 1.0, 1.0, 1.0, 0.9, 0.5, 0.1, 0.95, 0.8, 1.0, 0.95, 0.3, 0.95, 0.2], device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.long) * 7919 + 1
    steps = torch.arange(B, device=DEV, dtype=torch.long) + 3
    tok = torch.empty(B, device=DEV, dtype=torch.long)
    lp = torch.empty(B, device=DEV, dtype=torch.float32)
    ops.sample(tok, lp, logits, temp, top_k, top_p, seeds, steps)
    rt, rlp = ref.sample(logits.cpu(), temp.cpu(), top_k.cpu(), top_p.cpu(), seeds.cpu(), steps.cpu())
    assert ((tok.cpu() >= 0) & (tok.cpu() < V)).all()
    mism = (tok.cpu() != rt).sum().item()
    assert mism <= 1, (tok.cpu(), rt)
    ok = tok.cpu() == rt
    assert torch.allclose(lp.cpu()[ok], rlp[ok], atol=2e-3)
    assert tok[0].item() == int(logits[0].float().argmax())
    assert tok[3].item() == int(logits[3].float().argmax())
    # graph capture + replay gives the same draw
    g = torch.cuda.CUDAGraph()
    tok2 = torch.empty_like(tok)
    lp2 = torch.empty_like(lp)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.sample(tok2, lp2, logits, temp, top_k, top_p, seeds, steps)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        ops.sample(tok2, lp2, logits, temp, top_k, top_p, seeds, steps)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(tok2, tok)


def test_sample_nan_row_never_out_of_range(ops):
    V = 128256
    logits = torch.full((3, V), float("nan"), device=DEV, dtype=torch.bfloat16)
    temp = torch.tensor([0.0, 1.0, 0.7], device=DEV)
    top_k = torch.tensor([0, 0, 10], device=DEV, dtype=torch.int32)
    top_p = torch.tensor([1.0, 0.9, 0.9], device=DEV)
    tok = torch.empty(3, device=DEV, dtype=torch.long)
    lp = torch.empty(3, device=DEV)
    ops.sample(tok, lp, logits, temp, top_k, top_p, torch.zeros(3, device=DEV, dtype=torch.long),
               torch.zeros(3, device=DEV, dtype=torch.long))
    assert ((tok >= 0) & (tok < V)).all()


def test_sample_distribution(ops):
    """Empirical frequencies follow softmax(x/T) restricted to top-k."""
    V, N = 16, 4096
    base = torch.linspace(-2, 2, V)
    logits = base.repeat(N, 1).to(DEV)
    temp = torch.full((N,), 1.0, device=DEV)
    top_k = torch.full((N,), 8, device=DEV, dtype=torch.int32)
    top_p = torch.ones(N, device=DEV)
    seeds = torch.arange(N, device=DEV, dtype=torch.long)
    steps = torch.zeros(N, device=DEV, dtype=torch.long)
    tok = torch.empty(N, device=DEV, dtype=torch.long)
    lp = torch.empty(N, device=DEV)
    ops.sample(tok, lp, logits, temp, top_k, top_p, seeds, steps)
    cnt = torch.bincount(tok.cpu(), minlength=V).float() / N
    p = torch.softmax(base[8:], 0)
    assert cnt[:8].sum() == 0
    assert (cnt[8:] - p).abs().max() < 0.03


def _skinny_cases():
    """(N, K, rt, kw) with K divisible by the kernel's 256*kw K chunk."""
    return [(n, k, rt, kw)
            for n, k in [(4096, 4096), (200, 1024), (6144, 4096), (4096, 14336)]
            for rt, kw in [(1, 1), (1, 4), (1, 8), (2, 2), (2, 8)]
            if k % (256 * kw) == 0]


def _dg_cases(shapes, splits):
    """(N, K, splits) whose K slice is one of the compiled step counts (DG_STEPS)."""
    from hipserve.ops.gemm import DG_STEPS
    return [(n, k, s) for n, k in shapes for s in splits
            if k % (256 * s) == 0 and k // s // 256 in DG_STEPS]


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("N,K,rt,kw", _skinny_cases())
def test_skinny_gemm(ops, M, N, K, rt, kw):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.skinny_gemm(out, x, w, rt, kw)
    want = x.float() @ w.float().T
    _close(out, want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)


@pytest.mark.parametrize("M", [1, 20, 64])
@pytest.mark.parametrize("splits", [1, 4])
def test_splitk_bf16_gemm(ops, M, splits):
    from hipserve.ops.gemm import splitk_gemm
    N, K = 4096, 4096
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    splitk_gemm(out, x, w, splits)
    want = x.float() @ w.float().T
    _close(out, want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)


@pytest.mark.parametrize("M", [1, 7, 16, 23, 32, 50, 64])
@pytest.mark.parametrize("N,K,splits", _dg_cases([(4096, 4096), (1000, 512), (6144, 1792),
                                                  (4096, 3072), (4096, 5376)], [1, 2, 7, 8]))
@pytest.mark.parametrize("rt", [1, 2])
def test_decode_gemm(ops, M, N, K, rt, splits):
    """Split-K LDS-shared decode GEMM vs fp32 torch (incl. ragged M, N tails, strided x,
    and the 12/21-step K slices of Gemma-3's K = 3072 / 5376)."""
    from hipserve.ops.gemm import decode_gemm
    torch.manual_seed(M * 7 + N)
    xb = torch.randn(M, K + 64, device=DEV, dtype=torch.bfloat16)
    x = xb[:, :K]  # row stride != K
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    decode_gemm(out, x, w, rt, splits)
    assert not torch.isnan(out).any(), "unwritten outputs"
    want = x.float() @ w.float().T
    _close(out, want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)


@pytest.mark.parametrize("M", [1, 16, 23, 64])
@pytest.mark.parametrize("N,K,splits", _dg_cases([(4096, 4096), (1000, 512), (6144, 1792),
                                                  (4096, 14336), (4096, 5376)], [1, 2, 8]))
@pytest.mark.parametrize("rt", [1, 2])
def test_decode_gemm_packed(ops, M, N, K, rt, splits):
    """Packed-weight decode GEMM (pre-shuffled streaming layout, N padded to 128)
    vs fp32 torch; also checks the packing kernel against a torch permute."""
    from hipserve.ops import gemm
    torch.manual_seed(M * 11 + N + K)
    xb = torch.randn(M, K + 64, device=DEV, dtype=torch.bfloat16)
    x = xb[:, :K]
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    wp = gemm.pack(w)
    Np = -(-N // 128) * 128
    wpad = torch.zeros(Np, K, device=DEV, dtype=torch.bfloat16)
    wpad[:N] = w
    # [tile][kstep][rg][s][g][c][8] from (tile, rg, c, kstep, s, g, 8)
    want_p = wpad.view(Np // 128, 8, 16, K // 256, 8, 4, 8).permute(0, 3, 1, 4, 5, 2, 6).reshape(-1)
    assert torch.equal(wp, want_p)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    gemm.decode_gemm_packed(out, x, wp, N, rt, splits)
    assert not torch.isnan(out).any(), "unwritten outputs"
    want = x.float() @ w.float().T
    _close(out, want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)


@pytest.mark.parametrize("T,E,k,S", [(1, 8, 2, 1), (64, 128, 8, 4), (37, 64, 4, 8), (64, 16, 4, 2)])
def test_moe_topk_softmax_from_partials(ops, T, E, k, S):
    """The router's fp32 split-K partials summed inside the top-k kernel == splitk_reduce
    to bf16 + the top-k kernel over those logits, bit for bit (ids and weights)."""
    torch.manual_seed(T * 31 + E + S)
    ws = torch.randn(S, T, E, device=DEV) * 2
    logits = torch.empty(T, E, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.splitk_reduce(logits, ws.reshape(-1), S)
    w0 = torch.empty(T, k, device=DEV)
    i0 = torch.empty(T, k, device=DEV, dtype=torch.int32)
    torch.ops.hipserve.moe_topk_softmax(w0, i0, logits, k, True)
    w1 = torch.full((T, k), float("nan"), device=DEV)
    i1 = torch.full((T, k), -1, device=DEV, dtype=torch.int32)
    torch.ops.hipserve.moe_topk_softmax(w1, i1, ws.reshape(-1), k, True, S)
    assert torch.equal(i0, i1) and torch.equal(w0, w1)


@pytest.mark.parametrize("T,k,H", [(1, 8, 2048), (37, 8, 2048), (256, 2, 4096), (5, 4, 7168), (9, 2, 1024)])
@pytest.mark.parametrize("S", [0, 1, 3])
@pytest.mark.parametrize("wdt", [torch.bfloat16, torch.float32])
def test_moe_combine_add_rmsnorm_bit_exact(ops, T, k, H, S, wdt):
    """The one-kernel decode MoE tail == moe_combine(_partial) + fused_add_rmsnorm, bit for
    bit (norm output and the updated residual), for bf16 expert rows and fp32 partials."""
    torch.manual_seed(T + k + H + S)
    cap = T * k + 64
    pair_slot = torch.randperm(cap, device=DEV)[: T * k].int()
    w = torch.rand(T, k, device=DEV)
    y = (torch.randn(S, cap, H, device=DEV) if S else torch.randn(cap, H, device=DEV).to(torch.bfloat16))
    res = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    nw = (torch.rand(H, device=DEV) + 0.5).to(wdt)
    comb = torch.empty(T, H, device=DEV, dtype=torch.bfloat16)
    if S:
        torch.ops.hipserve.moe_combine_partial(comb, y, w, pair_slot, k)
    else:
        torch.ops.hipserve.moe_combine(comb, y, w, pair_slot, k)
    r0, o0 = res.clone(), torch.empty_like(res)
    ops.fused_add_rmsnorm(o0, comb, r0, nw, 1e-6)
    r1, o1 = res.clone(), torch.full_like(res, float("nan"))
    torch.ops.hipserve.moe_combine_add_rmsnorm(o1, r1, y, S, w, pair_slot, k, nw, 1e-6)
    assert torch.equal(r0, r1) and torch.equal(o0, o1)


@pytest.mark.parametrize("mode", ["packed", "rowmajor", "legacy"])
@pytest.mark.parametrize("T,E,k,norm", [(1, 8, 2, True), (13, 8, 2, True), (64, 8, 2, True), (200, 8, 2, True),
                                        (5, 4, 1, True), (3, 128, 8, True), (40, 128, 8, False), (9, 64, 4, False)])
def test_moe_kernels_match_reference(ops, T, E, k, norm, mode, monkeypatch):
    """HIP MoE (topk softmax, align, gathered GEMMs, combine) vs the torch path, for
    the expert decode GEMM on packed (GLU epilogue + split-K partial combine) and
    row-major weights, and the legacy 16-row gathered GEMM."""
    import types

    from hipserve.config import PRESETS
    from hipserve.models.llama import LayerWeights, LlamaModel
    from hipserve.parallel.comm import TPGroup

    cfg = PRESETS["tiny-mixtral"].replace(hidden_size=512, intermediate_size=768, num_experts=E,
                                          num_experts_per_tok=k, norm_topk_prob=norm)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, ops)
    torch.manual_seed(T)
    lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None,
                      # many experts: wider logits so the k-th / (k+1)-th choice never ties in bf16
                      router=torch.randn(E, 512, device=DEV, dtype=torch.bfloat16) * (0.2 if E <= 8 else 0.6),
                      w13=torch.randn(E, 1536, 512, device=DEV, dtype=torch.bfloat16) * 0.05,
                      w2=torch.randn(E, 512, 768, device=DEV, dtype=torch.bfloat16) * 0.05)
    x = torch.randn(T, 512, device=DEV, dtype=torch.bfloat16)
    if mode == "packed":
        assert m.pack_moe_weights() == 0  # no layers registered on the model: nothing packed
        m.layers = [lw]
        assert m.pack_moe_weights() > 0 and lw.moe_packed is not None
    elif mode == "legacy":
        monkeypatch.setattr(LlamaModel, "_moe_decode_ok", lambda self, lw: False)
    got = m.moe_hip(x, lw).float()
    ref_ops = types.SimpleNamespace(name="reference", silu_and_mul=ops.silu_and_mul)
    m.ops = ref_ops
    want = m.moe(x, lw).float()
    m.ops = ops
    _close(got, want, atol=3e-2 * want.abs().max().item() + 1e-3, frac=0.995)


@pytest.mark.parametrize("rows,cols,row0,col0,gcols", [(64, 96, 0, 0, 96), (300, 1000, 17, 5, 4096),
                                                       (1, 8192, 1000, 0, 8192)])
def test_fill_uniform_bit_exact(ops, rows, cols, row0, col0, gcols):
    """On-device synthetic init == its torch twin, bit for bit (strided view too)."""
    base = torch.zeros(rows, cols + 8, device=DEV, dtype=torch.bfloat16)
    view = base[:, 4:4 + cols]
    ops.fill_uniform(view, row0, col0, gcols, 987654321, 0.0346)
    want = ref.fill_uniform(torch.empty(rows, cols, dtype=torch.bfloat16), row0, col0, gcols, 987654321, 0.0346)
    assert torch.equal(view.cpu(), want)
    assert torch.count_nonzero(base[:, :4]) == 0 and torch.count_nonzero(base[:, 4 + cols:]) == 0


def test_stage_copy_host_device_roundtrip(ops):
    """Zero-copy staging kernel: pinned host -> device and device -> pinned host in one
    dispatch each, with mixed dtypes and sizes, matches torch copies; rewriting the host
    buffer between launches is seen by the next launch (no stale cached lines)."""
    h64 = torch.arange(300, dtype=torch.long).pin_memory()
    h32 = (torch.arange(5000, dtype=torch.int32) * 3).pin_memory()
    hf = torch.linspace(-1, 1, 17).pin_memory()
    d64 = torch.zeros(300, dtype=torch.long, device=DEV)
    d32 = torch.zeros(5000, dtype=torch.int32, device=DEV)
    df = torch.zeros(17, device=DEV)
    for it in range(3):
        h64.add_(7)
        h32[:4000].mul_(-1)
        torch.ops.hipserve.stage_copy([d64, d32[:4000], d32[4000:], df], [h64, h32[:4000], h32[4000:], hf], 0)
        torch.cuda.synchronize()
        assert torch.equal(d64.cpu(), h64) and torch.equal(d32.cpu(), h32) and torch.equal(df.cpu(), hf)
    out64 = torch.zeros(300, dtype=torch.long).pin_memory()
    outf = torch.zeros(17).pin_memory()
    d64.mul_(3)
    torch.ops.hipserve.stage_copy([out64, outf], [d64, df], 0)
    ev = torch.cuda.Event()
    ev.record()
    ev.synchronize()
    assert torch.equal(out64, h64 * 3) and torch.equal(outf, hf)


@pytest.mark.parametrize("V,dt", [(32000, torch.bfloat16), (128256, torch.bfloat16), (1000, torch.float32)])
def test_penalty_and_top_logprobs_kernels(V, dt):
    """csrc/kernels/penalties.hip vs the torch reference (hipserve/ops/reference.py):
    slot init from prompt + generated ids, in-graph updates, penalty application
    (rows without a slot untouched) and top-n logprobs with lowest-id tie breaks."""
    from hipserve.ops import load_library
    from hipserve.ops import reference as R

    load_library()
    op = torch.ops.hipserve
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(V)
    rows, slots = 6, 4
    words = (V + 31) // 32
    counts = torch.zeros(slots, V, dtype=torch.int32)
    seen = torch.zeros(slots, words, dtype=torch.int32)
    # init slots 0, 2, 3 from (prompt, generated) histories
    hist = [(torch.randint(0, V, (50,), generator=g), torch.randint(0, 200, (30,), generator=g))
            for _ in range(3)]
    sl = torch.tensor([0, 2, 3], dtype=torch.int32)
    toks = torch.cat([torch.cat([p, o]) for p, o in hist]).int()
    off = torch.tensor([0, 80, 160, 240], dtype=torch.int32)
    npr = torch.tensor([50, 50, 50], dtype=torch.int32)
    cd, sd = counts.to(dev), seen.to(dev)
    op.penalty_init(cd, sd, sl.to(dev), off.to(dev), npr.to(dev), toks.to(dev))
    R.penalty_init(counts, seen, sl, off, npr, toks)
    assert torch.equal(cd.cpu(), counts) and torch.equal(sd.cpu(), seen)
    # a sampled step updates the slots
    tok = torch.randint(0, V, (rows,), generator=g).long()
    slot = torch.tensor([0, -1, 2, 3, -1, -1], dtype=torch.int32)
    op.penalty_update(tok.to(dev), slot.to(dev), cd, sd)
    R.penalty_update(tok, slot, counts, seen)
    assert torch.equal(cd.cpu(), counts) and torch.equal(sd.cpu(), seen)
    # apply: row 3 has a slot but no active penalty (untouched), rows 1/4/5 no slot
    logits = (torch.randn(rows, V, generator=g) * 3).to(dt)
    pres = torch.tensor([0.5, 1.0, -0.7, 0.0, 0.0, 0.0])
    freq = torch.tensor([1.5, 1.0, 0.3, 0.0, 0.0, 0.0])
    rep = torch.tensor([1.3, 1.0, 0.8, 1.0, 1.0, 1.0])
    got = logits.to(dev)
    op.penalty_apply(got, slot.to(dev), pres.to(dev), freq.to(dev), rep.to(dev), cd, sd)
    want = logits.clone()
    R.penalty_apply(want, slot, pres, freq, rep, counts, seen)
    assert torch.equal(got.cpu()[[1, 3, 4, 5]], logits[[1, 3, 4, 5]])
    rel = 1e-5 if dt == torch.float32 else 2.0 ** -7  # one bf16 ulp
    assert ((got.cpu().float() - want.float()).abs() <= want.float().abs() * rel + 1e-5).all()
    # top-n logprobs (with forced ties in row 2); with fp32 logits, row 5's top entries
    # sit within one bf16 step of each other, increasing with id: the exact-value
    # order is the reverse of the id order
    want[2, 100:110] = want[2].max() + 1
    if dt == torch.float32:
        want[5, 300:310] = want[5].max() + 1 + torch.arange(10) * 1e-4
    got = want.to(dev)
    nreq = torch.tensor([5, 0, 20, 1, 3, 7], dtype=torch.int32)
    ids = torch.empty(rows, 20, dtype=torch.int32, device=dev)
    lps = torch.empty(rows, 20, dtype=torch.float32, device=dev)
    op.top_logprobs(got, nreq.to(dev), ids, lps)
    rid = torch.empty(rows, 20, dtype=torch.int32)
    rlp = torch.empty(rows, 20)
    R.top_logprobs(want, nreq, rid, rlp)
    assert torch.equal(ids.cpu(), rid)
    if dt == torch.float32:
        assert ids.cpu()[5, :7].tolist() == list(range(309, 302, -1))
    fin = torch.isfinite(rlp)
    assert torch.equal(torch.isfinite(lps.cpu()), fin)
    assert (lps.cpu()[fin] - rlp[fin]).abs().max().item() < 1e-3


@pytest.mark.parametrize("T,E,k,norm", [(700, 8, 2, True), (3000, 8, 2, True), (400, 128, 8, True), (300, 64, 4, False)])
def test_moe_grouped_prefill_vs_fp32(ops, T, E, k, norm):
    """Prefill MoE (routing kernel, moe_align, the two packed-layout grouped expert
    GEMMs with the token gather fused into the first and SiLU-GLU in its epilogue,
    combine) vs an fp32 reference of the same routed computation."""
    from hipserve.config import PRESETS
    from hipserve.models.llama import LayerWeights, LlamaModel
    from hipserve.parallel.comm import TPGroup

    H, I = 512, 768
    cfg = PRESETS["tiny-mixtral"].replace(hidden_size=H, intermediate_size=I, num_experts=E,
                                          num_experts_per_tok=k, norm_topk_prob=norm)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, ops)
    torch.manual_seed(T + E)
    lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None,
                      router=torch.randn(E, H, device=DEV, dtype=torch.bfloat16) * (0.2 if E <= 8 else 0.6),
                      w13=torch.randn(E, 2 * I, H, device=DEV, dtype=torch.bfloat16) * 0.05,
                      w2=torch.randn(E, H, I, device=DEV, dtype=torch.bfloat16) * 0.05)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    got = m.moe_grouped(x, lw).float()
    # fp32 reference, routing on the same bf16 router logits the kernel path sees
    logits = torch.nn.functional.linear(x, lw.router).float()
    wts, idx = torch.topk(torch.softmax(logits, -1), k, -1)
    if norm:
        wts = wts / wts.sum(-1, keepdim=True)
    xf, w13, w2 = x.float(), lw.w13.float(), lw.w2.float()
    want = torch.zeros(T, H, device=DEV)
    for e in range(E):
        rows, slot = (idx == e).nonzero(as_tuple=True)
        if rows.numel() == 0:
            continue
        gu = xf[rows] @ w13[e].T
        act = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
        want.index_add_(0, rows, (act @ w2[e].T) * wts[rows, slot].unsqueeze(-1))
    _close(got, want, atol=3e-2 * want.abs().max().item() + 1e-3, frac=0.995)
    # moe() takes this path for prefill-sized batches (beyond the decode kernels' range)
    calls = []
    orig = m.moe_grouped
    m.moe_grouped = lambda *a_: calls.append(1) or orig(*a_)
    from hipserve.models.llama import MOE_KERNEL_MAX_ROWS_PER_EXPERT
    x_big = torch.randn(MOE_KERNEL_MAX_ROWS_PER_EXPERT * E // k + 64, H, device=DEV, dtype=torch.bfloat16)
    m.moe(x_big, lw)
    assert calls, "prefill-sized MoE did not take the grouped path"


@pytest.mark.parametrize("M", [33, 50, 64])
@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("N,K,splits", [(6144, 4096, 4), (4096, 4096, 8), (1000, 512, 1), (4160, 1792, 1),
                                        (4096, 14336, 8)])
def test_decode_gemm_64_row_workgroups(ops, M, N, K, splits, packed):
    """rt = 3: 64-row workgroups (4 waves x 1 row group; a packed 128-row tile split over
    two workgroups), plain and as split-K partials, vs fp32 torch; N tails inside a
    packed tile's second half."""
    from hipserve.ops import gemm
    torch.manual_seed(M + N + K)
    xb = torch.randn(M, K + 64, device=DEV, dtype=torch.bfloat16)
    x = xb[:, :K]
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    want = x.float() @ w.float().T
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    if packed:
        gemm.decode_gemm_packed(out, x, gemm.pack(w), N, 3, splits)
    else:
        gemm.decode_gemm(out, x, w, 3, splits)
    assert not torch.isnan(out).any(), "unwritten outputs"
    _close(out, want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)
    ws = torch.full((splits * M * N,), float("nan"), device=DEV, dtype=torch.float32)
    torch.ops.hipserve.decode_gemm_partial(ws, x, gemm.pack(w) if packed else w, N, 3, splits, packed)
    _close(ws.view(splits, M, N).sum(0), want, atol=2e-2 * want.abs().max().item(), rtol=1e-2)
