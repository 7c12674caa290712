"""Fused decode layer v2 (csrc/kernels/decode_layer.hip): decode GEMMs whose split-K
fix-up runs the layer epilogue in the same launch (residual add + per-tile sums of
squares, RoPE + paged-KV write, SiLU-GLU) and RMSNorm-on-load of the GEMM input.

Every kernel is checked against a plain PyTorch fp32 reference of the same op
(bf16 rounding where the engine rounds), and against the v1 kernels it replaces:
the split-K sums are accumulated in the same slice order, so wherever no RMSNorm
sum of squares is involved the results are bit-identical to v1. The model forward
is compared with the v1 fused forward (tolerance: only the RMSNorm sums of squares
are associated differently), across hipGraph replays (tile counters reset)."""
import math

import pytest
import torch

from hipserve.ops import KernelOps, gemm
from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
op = None


@pytest.fixture(scope="module")
def ops():
    global op
    op = torch.ops.hipserve
    return KernelOps()


def _ctr():
    return torch.zeros(8192, dtype=torch.int32, device=DEV)


def _ws(S, M, N):
    return torch.empty(S * M * N, device=DEV, dtype=torch.float32) if S > 1 else torch.empty(0, device=DEV)


def _norm_in(M, K, g):
    """(residual, ss_in [T, M], norm weight, the bf16 normalised x the kernel must form)."""
    r = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (1 + 0.2 * torch.randn(K, device=DEV, generator=g)).to(torch.bfloat16)
    T = K // 128
    ss = r.float().pow(2).view(M, T, 128).sum(-1).t().contiguous()  # per-tile partials, like the ADD fix-up
    inv = torch.rsqrt(ss.sum(0) / K + 1e-5)
    xn = (r.float() * inv[:, None] * w.float()).to(torch.bfloat16)
    return r, ss, w, xn


@pytest.mark.parametrize("M", [1, 13, 32, 64])
@pytest.mark.parametrize("K,S", [(4096, 1), (4096, 8), (14336, 8), (14336, 7), (2048, 2)])
def test_dgf_add_vs_fp32_and_v1(ops, M, K, S):
    N = 4096
    g = torch.Generator(device=DEV).manual_seed(M * 31 + K + S)
    x = (torch.randn(M, K, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    res0 = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    wp = gemm.pack(w)
    res = res0.clone()
    ss = torch.full((N // 128, M), float("nan"), device=DEV)
    op.decode_gemm_fused(1, x, wp, N, S, _ws(S, M, N), _ctr(), None, None, 1e-5, res, ss, None, None, None, None,
                         None, None, 0, 0, 0, 0, 0, None, None, None)
    # fp32 reference with the engine's rounding points
    h = (x.float() @ w.float().t()).to(torch.bfloat16)
    want = (h.float() + res0.float()).to(torch.bfloat16)
    torch.testing.assert_close(res.float(), want.float(), rtol=8e-3, atol=8e-3)
    want_ss = res.float().pow(2).view(M, N // 128, 128).sum(-1).t()
    torch.testing.assert_close(ss, want_ss, rtol=1e-5, atol=1e-5)
    # v1: partials + splitk_add_rmsnorm -> the same residual bits
    ws1 = torch.empty(S * M * N, device=DEV, dtype=torch.float32)
    op.decode_gemm_partial(ws1, x, wp, N, 1, S, True)
    r1, o1 = res0.clone(), torch.empty_like(res0)
    op.splitk_add_rmsnorm(o1, r1, ws1, S, torch.ones(N, device=DEV, dtype=torch.bfloat16), 1e-5)
    assert torch.equal(r1, res)


@pytest.mark.parametrize("M", [1, 24, 64])
@pytest.mark.parametrize("S", [1, 4])
@pytest.mark.parametrize("norm_in", [False, True])
@pytest.mark.parametrize("mode,D,bias,qk", [(0, 128, False, False), (1, 128, False, False), (0, 64, True, False),
                                            (0, 128, True, True), (0, 64, False, True)])
def test_dgf_rope_vs_fp32(ops, M, S, norm_in, mode, D, bias, qk):
    nq, nkv, bs, K = 16, 4, 16, 2048
    N = (nq + 2 * nkv) * D
    g = torch.Generator(device=DEV).manual_seed(M * 7 + S + D + 3 * mode)
    if norm_in:
        x, ss_in, nw, xn = _norm_in(M, K, g)
    else:
        x = xn = (torch.randn(M, K, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
        ss_in = nw = None
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    b = (torch.randn(N, device=DEV, generator=g) * 0.3).to(torch.bfloat16) if bias else None
    qw = 1 + 0.2 * torch.randn(D, device=DEV, generator=g) if qk else None
    kw = 1 + 0.2 * torch.randn(D, device=DEV, generator=g) if qk else None
    pos = torch.randint(0, 4000, (M,), device=DEV, generator=g)
    slots = torch.randperm(64 * bs, device=DEV, generator=g)[:M]
    if M > 5:
        slots[5] = -1
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(DEV)
    kc = torch.zeros(64, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros(64, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
    q = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
    op.decode_gemm_fused(2, x, gemm.pack(w), N, S, _ws(S, M, N), _ctr(), ss_in, nw, 1e-6, None, None, q, pos, slots,
                         cs, kc, vc, nq, nkv, D, bs, mode, b, qw, kw)
    # reference: the unfused chain in fp32 with bf16 rounding points
    qkv = (xn.float() @ w.float().t()).to(torch.bfloat16)
    if bias:
        qkv = qkv + b
    if qk:
        ops.qk_rmsnorm(qkv, qw, kw, nq, nkv, D, 1e-6)
    kc1, vc1 = torch.zeros_like(kc), torch.zeros_like(vc)
    ref_ops = KernelOps()
    ref_ops.rope_cache(qkv, pos, slots, cs, kc1, vc1, nq, nkv, D, mode)
    tol = dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(q[:, : nq * D].float(), qkv[:, : nq * D].float(), **tol)
    torch.testing.assert_close(kc.float(), kc1.float(), **tol)
    torch.testing.assert_close(vc.float(), vc1.float(), **tol)
    if not norm_in and not qk:  # no sum of squares anywhere: bit-identical to v1
        ws1 = torch.empty(S * M * N, device=DEV, dtype=torch.float32)
        op.decode_gemm_partial(ws1, x, gemm.pack(w), N, 1, S, True)
        q2 = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
        op.splitk_rope_cache(q2, ws1, S, pos, slots, cs, kc2, vc2, nq, nkv, D, mode, b, None, None, 1e-6)
        assert torch.equal(q[:, : nq * D], q2[:, : nq * D])
        assert torch.equal(kc, kc2) and torch.equal(vc, vc2)


@pytest.mark.parametrize("M", [1, 16, 40, 64])
@pytest.mark.parametrize("S", [1, 2, 4])
def test_dgf_glu_vs_fp32(ops, M, S):
    I, K = 1792, 4096
    N = 2 * I
    g = torch.Generator(device=DEV).manual_seed(M + 100 * S)
    r, ss_in, nw, xn = _norm_in(M, K, g)
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
    act = torch.full((M, I), float("nan"), device=DEV, dtype=torch.bfloat16)
    op.decode_gemm_fused(3, r, gemm.pack(w, glu=True), N, S, _ws(S, M, N), _ctr(), ss_in, nw, 1e-5, None, None, act,
                         None, None, None, None, None, 0, 0, 0, 0, 0, None, None, None)
    gu = (xn.float() @ w.float().t()).to(torch.bfloat16).float()
    want = (torch.nn.functional.silu(gu[:, :I]).to(torch.bfloat16).float() * gu[:, I:])
    torch.testing.assert_close(act.float(), want, rtol=2e-2, atol=2e-3)


def _model(ops, family="llama"):
    from tests.test_fused_decode_gpu import _small_model

    m, cfg = _small_model(ops, family=family)
    return m, cfg


@pytest.mark.parametrize("family", ["llama", "qwen2", "qwen3"])
@pytest.mark.parametrize("B", [1, 24, 64])
def test_forward_v2_vs_v1(ops, family, B):
    """The v2 decode forward (5 kernels per layer) vs the v1 fused forward (8): the
    same hidden states and caches up to the RMSNorm sum-of-squares association;
    captured in a hipGraph and replayed (the tile counters must be reset by every
    replay's last arrivers)."""
    from hipserve.models.llama import AttnMeta

    m, cfg = _model(ops, family)
    old = dict(gemm.TUNER.table)
    try:
        gemm.TUNER.table.clear()
        shapes = m.gemm_shapes()
        for (N, K) in shapes:
            for mm in gemm.TUNE_MS:
                gemm.TUNER.table[(mm, N, K)] = ("dgp", 1, 2 if K >= 1024 else 1)
        m.pack_decode_weights(set(shapes))
        bs, D = 16, cfg.head_dim
        nblk = 40
        ctx = torch.randint(1, nblk * bs, (B,), device=DEV, dtype=torch.int32)
        bt = torch.randperm(B * nblk, device=DEV).int().view(B, nblk)
        pos = (ctx - 1).long()
        slots = bt.gather(1, (pos // bs).view(-1, 1).int()).view(-1).long() * bs + pos % bs
        ids = torch.randint(0, cfg.vocab_size, (B,), device=DEV)
        kv1 = m.allocate_kv_cache(B * nblk, bs)
        for kc, vc in kv1:
            kc.normal_()
            vc.normal_()
        kv2 = [(k.clone(), v.clone()) for k, v in kv1]
        parts = math.ceil(nblk * bs / 512)
        mk = lambda: AttnMeta(num_prefill_tokens=0, num_decode=B, positions=pos, slot_mapping=slots,
                              bt_decode=bt, ctx_decode=ctx, tmp_out=torch.empty(B, m.nq, parts, D, device=DEV),
                              tmp_ml=torch.empty(B, m.nq, parts, 2, device=DEV))
        m.fused_v2 = True
        assert m.v2_plan(B, mk()) is not None
        m.fused_v2 = False
        out1 = m.forward(ids, mk(), kv1).clone()
        m.fused_v2 = True
        out2 = m.forward(ids, mk(), kv2).clone()
        d = (out1.float() - out2.float()).abs()
        assert d.max().item() < 0.1 and d.mean().item() < 2e-3, (d.max().item(), d.mean().item())
        for (k1, v1), (k2, v2) in zip(kv1, kv2):  # bf16-ulp flips of a few cache entries at most
            for a, b in ((k1, k2), (v1, v2)):
                dd = (a.float() - b.float()).abs()
                assert dd.max().item() <= 0.0625 and (dd > 1e-2).float().mean().item() < 1e-4, dd.max().item()
        # hipGraph replays: bit-identical to the eager v2 forward every time
        meta = mk()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.forward(ids, meta, kv2)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out_g = m.forward(ids, meta, kv2)
        for _ in range(3):
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out_g, out2)
        assert int(m._dgf_counters.abs().sum()) == 0
    finally:
        gemm.TUNER.table.clear()
        gemm.TUNER.table.update(old)
        m.fused_v2 = type(m).fused_v2
