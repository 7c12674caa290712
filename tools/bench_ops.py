#!/usr/bin/env python3
"""Micro-benchmarks of individual hipserve kernels on the GPU (HIP-event timing,
median of N launches). Prints one JSON line per case.

    python tools/bench_ops.py [sample|decode|prefill|gemm|norm|all]
"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hipserve.ops import KernelOps  # noqa: E402

DEV = "cuda"


def timeit(fn, n=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    evs = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1000 for a, b in evs)
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)


def graph_time(fn, n=20, reps=5):
    """Device time per call with the calls captured in one hipGraph (how the
    engine's decode step runs them: no host launch cost)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    v = sorted(x.elapsed_time(y) for x, y in ts)
    return v[len(v) // 2] * 1000.0 / n


def bench_sample(ops):
    timer = graph_time if os.environ.get("BENCH_GRAPH", "1") == "1" else timeit
    for V, B in [(128256, 64), (128256, 256), (32000, 64), (128256, 1)]:
        logits = (torch.randn(B, V, device=DEV) * 3).to(torch.bfloat16)
        tok = torch.empty(B, dtype=torch.long, device=DEV)
        lp = torch.empty(B, device=DEV)
        for name, t, k, p in [("greedy", 0.0, 0, 1.0), ("temp", 0.8, 0, 1.0), ("top_p", 0.8, 0, 0.95),
                              ("top_k_p", 0.8, 50, 0.95)]:
            temp = torch.full((B,), t, device=DEV)
            tk = torch.full((B,), k, dtype=torch.int32, device=DEV)
            tp = torch.full((B,), p, device=DEV)
            seeds = torch.arange(B, device=DEV)
            steps = torch.zeros(B, dtype=torch.long, device=DEV)
            us = timer(lambda: ops.sample(tok, lp, logits, temp, tk, tp, seeds, steps))
            emit(op="sample", mode=name, V=V, B=B, us=round(us, 1), graph=timer is graph_time)


def bench_decode(ops):
    import os
    D = 128
    parts = [int(x) for x in os.environ.get("DECODE_PARTS", "512").split(",")]
    bss = [int(x) for x in os.environ.get("DECODE_BS", "16").split(",")]  # KV block sizes
    shapes = [(64, 1152, 32, 8), (64, 1280, 32, 8), (256, 1152, 32, 8), (1, 4096, 32, 8), (64, 4096, 64, 8)]
    if os.environ.get("DECODE_SHAPES"):  # "BxCTXxNQxNKV,..." e.g. 64x1152x32x4 (Qwen3-30B-A3B)
        shapes = [tuple(int(v) for v in sh.split("x")) for sh in os.environ["DECODE_SHAPES"].split(",")]
    for (B, ctx, nq, nkv), part, bs in [(c, p, b) for c in shapes for p in parts for b in bss]:
        mb = math.ceil(ctx / bs) + 1
        nblocks = B * mb
        # DECODE_COLD=1: rotate over enough KV copies (> 2x the 256 MB MALL) that every
        # call streams cold K / V, as in the engine (one step touches every layer's KV)
        # DECODE_KV=fp8: e4m3 cache (--kv-cache-dtype fp8), half the bytes
        f8 = os.environ.get("DECODE_KV") == "fp8"
        kvt = torch.float8_e4m3fn if f8 else torch.bfloat16
        byts = 2 * B * ctx * nkv * D * (1 if f8 else 2)
        ncopy = max(1, min(8, -(-(768 << 20) // byts))) if os.environ.get("DECODE_COLD") == "1" else 1
        kcs = [torch.randn(nblocks, nkv, bs, D, device=DEV).to(kvt) for _ in range(ncopy)]
        vcs = [torch.randn(nblocks, nkv, D, bs, device=DEV).to(kvt) for _ in range(ncopy)]
        bt = torch.randperm(nblocks, device=DEV).int().view(B, mb)
        cl = torch.full((B,), ctx, device=DEV, dtype=torch.int32)
        q = torch.randn(B, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
        mp = math.ceil(mb * bs / part)
        to = torch.empty(B, nq, mp, D, device=DEV)
        tm = torch.empty(B, nq, mp, 2, device=DEV)
        out = torch.empty(B, nq * D, device=DEV, dtype=torch.bfloat16)
        it = [0]

        def call():
            i = it[0] % ncopy
            it[0] += 1
            ops.paged_decode(out, q, kcs[i], vcs[i], bt, cl, to, tm, nq, nkv, part, 1 / math.sqrt(D))

        us = timeit(call)
        emit(op="paged_decode", kv="fp8" if f8 else "bf16", B=B, ctx=ctx, nq=nq, nkv=nkv, part=part, bs=bs, cold=ncopy > 1,
             nt=os.environ.get("HIPSERVE_DECODE_NT", "1"), us=round(us, 1), TBps=round(byts / us / 1e6, 2))
        del kcs, vcs


def bench_prefill(ops):
    D, bs = 128, 16
    shapes = [(1024, 8, 32, 8), (4096, 2, 32, 8), (8192, 1, 32, 8), (1024, 8, 8, 1)]
    if os.environ.get("BENCH_PREFILL_LONG"):
        shapes = [(1024, 8, 32, 8), (8192, 1, 32, 8), (32768, 1, 32, 8)]
    vers = os.environ.get("BENCH_PREFILL_VERS", "v2w4,v2w8,v1").split(",")
    for S, nseq, nq, nkv in shapes:
        mb = S // bs
        kvt = torch.float8_e4m3fn if os.environ.get("DECODE_KV") == "fp8" else torch.bfloat16
        kc = torch.randn(nseq * mb, nkv, bs, D, device=DEV).to(kvt)
        vc = torch.randn(nseq * mb, nkv, D, bs, device=DEV).to(kvt)
        bt = torch.arange(nseq * mb, device=DEV).int().view(nseq, mb)
        cu = torch.arange(0, (nseq + 1) * S, S, device=DEV, dtype=torch.int32)
        ctx = torch.full((nseq,), S, device=DEV, dtype=torch.int32)
        tiles = torch.tensor(sorted(((s, r) for s in range(nseq) for r in range(0, S, 128)), key=lambda t: -t[1]),
                             device=DEV, dtype=torch.int32)
        q = torch.randn(nseq * S, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
        out = torch.empty(nseq * S, nq * D, device=DEV, dtype=torch.bfloat16)
        flops = 4 * nseq * (S * S / 2) * D * nq
        for ver in vers:  # v1: per-wave L2 K/V reads (HIPSERVE_PREFILL_ATTN_V1=1)
            os.environ["HIPSERVE_PREFILL_ATTN_V1"] = "1" if ver == "v1" else "0"
            os.environ["HIPSERVE_PREFILL_ATTN_WAVES"] = "8" if ver == "v2w8" else "4"
            us = timeit(lambda: ops.prefill_attention(out, q, kc, vc, bt, cu, ctx, tiles, nq, nkv,
                                                      1 / math.sqrt(D)), n=10)
            emit(op="prefill_attention", ver=ver, S=S, nseq=nseq, nq=nq, nkv=nkv, us=round(us, 1),
                 TFLOPs=round(flops / us / 1e6, 1))
        os.environ.pop("HIPSERVE_PREFILL_ATTN_V1", None)


def bench_prefill_chunked(ops):
    """Chunked prefill attention: ``chunk`` new query rows at the end of a ``ctx``-token
    context per sequence (the shape of every step of a long prompt under an 8K token
    budget), TFLOP/s over the causal work of the chunk."""
    D, bs, nq, nkv = 128, 16, 32, 8
    for ctx_len, chunk, nseq in [(32768, 2048, 4), (32768, 8192, 1), (16384, 2048, 4), (8192, 2048, 4)]:
        mb = ctx_len // bs
        kc = torch.randn(nseq * mb, nkv, bs, D, device=DEV, dtype=torch.bfloat16)
        vc = torch.randn(nseq * mb, nkv, D, bs, device=DEV, dtype=torch.bfloat16)
        bt = torch.arange(nseq * mb, device=DEV).int().view(nseq, mb)
        cu = torch.arange(0, (nseq + 1) * chunk, chunk, device=DEV, dtype=torch.int32)
        ctx = torch.full((nseq,), ctx_len, device=DEV, dtype=torch.int32)
        tiles = torch.tensor(sorted(((s, r) for s in range(nseq) for r in range(0, chunk, 128)), key=lambda t: -t[1]),
                             device=DEV, dtype=torch.int32)
        q = torch.randn(nseq * chunk, (nq + 2 * nkv) * D, device=DEV, dtype=torch.bfloat16)
        out = torch.empty(nseq * chunk, nq * D, device=DEV, dtype=torch.bfloat16)
        flops = 4 * nseq * chunk * (ctx_len - chunk / 2) * D * nq
        us = timeit(lambda: ops.prefill_attention(out, q, kc, vc, bt, cu, ctx, tiles, nq, nkv, 1 / math.sqrt(D)), n=10)
        emit(op="prefill_attention_chunked", ctx=ctx_len, chunk=chunk, nseq=nseq, us=round(us, 1),
             TFLOPs=round(flops / us / 1e6, 1))
        del kc, vc, q, out


def bench_gemm(ops):
    for M in (1, 16, 64, 128, 256):
        for N, K, name in [(6144, 4096, "qkv"), (4096, 4096, "o"), (28672, 4096, "gate_up"),
                           (4096, 14336, "down"), (128256, 4096, "lm_head")]:
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
            us = timeit(lambda: torch.nn.functional.linear(x, w))
            emit(op="hipblaslt_linear", name=name, M=M, N=N, K=K, us=round(us, 1),
                 TBps=round(N * K * 2 / us / 1e6, 2))


def bench_norm(ops):
    for T, H in [(64, 4096), (8192, 4096)]:
        x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
        r = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
        w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        us = timeit(lambda: ops.fused_add_rmsnorm(out, x, r, w, 1e-5))
        emit(op="fused_add_rmsnorm", T=T, H=H, us=round(us, 1), TBps=round(4 * T * H * 2 / us / 1e6, 2))


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    ops = KernelOps()
    for name, fn in [("sample", bench_sample), ("decode", bench_decode), ("prefill", bench_prefill),
                     ("prefill_chunked", bench_prefill_chunked),
                     ("gemm", bench_gemm), ("norm", bench_norm)]:
        if which in ("all", name):
            fn(ops)




def bench_tune():
    from hipserve.ops import gemm
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]
    import time
    t0 = time.time()
    ms = [int(m) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 16, 32, 64]
    for r in gemm.TUNER.tune(shapes, torch.device("cuda"), ms):
        emit(op="gemm_tune", **r)
    emit(op="gemm_tune_total_s", seconds=round(time.time() - t0, 1))


def bench_gemm_sweep():
    """Every decode-GEMM candidate vs hipBLASLt, cold weights (tuner timing)."""
    import torch.nn.functional as F
    from hipserve.ops import gemm
    T = gemm.GemmTuner
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    ms = [int(m) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else [64]
    for N, K in shapes:
        ncopy = max(1, min(16, -(-gemm.COLD_BYTES // (N * K * 2))))
        ws_ = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(ncopy)]
        wp_ = [gemm.pack(w) for w in ws_]
        n = max(16, ncopy)
        for M in ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            res = {"blas": T._time(lambda i: F.linear(x, ws_[i % ncopy]), n=n)}
            for cfg in T.candidates(M, N, K, packed=True):
                res[str(cfg)] = T._time(lambda i: gemm.run_choice(cfg, out, x, ws_[i % ncopy], wp_[i % ncopy]), n=n)
            emit(op="gemm_sweep", M=M, N=N, K=K, **{k: round(v, 1) for k, v in sorted(res.items(), key=lambda kv: kv[1])[:10]})
        del ws_, wp_


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "sweep":
    KernelOps()
    bench_gemm_sweep()
    sys.exit(0)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "tune":
    KernelOps()
    bench_tune()
    sys.exit(0)


if __name__ == "__main__":
    main()
