#!/usr/bin/env python3
"""MALL (Infinity Cache) prefetch for the decode GEMMs, two questions:

1. Does a decode GEMM run faster when part of its weight is already in the 256 MiB
   MALL? For each Llama-3-8B decode shape at M = 64 (packed decode GEMM, fixed config),
   over weight copies rotated so every call is HBM-cold: the GEMM alone vs after a
   ``mall_prefetch`` of its first P MiB (GEMM time = (prefetch + GEMM) - prefetch).
2. Does the prefetch overlap with the short epilogue kernel that precedes the GEMM in
   a decode layer when it runs on a forked stream of the same hipGraph? Graph of
   [splitk_add_rmsnorm (M = 64, N = 4096, 4 slices) -> GEMM] vs the same with a
   prefetch of the GEMM's first P MiB on a side stream forked before the norm and joined
   before the GEMM.

    python tools/bench_prefetch.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hipserve.ops import gemm, load_library  # noqa: E402

SHAPES = {"qkv": (6144, 4096, 2, 4), "o": (4096, 4096, 1, 4), "gate_up": (28672, 4096, 1, 1),
          "down": (4096, 14336, 1, 8)}  # N, K, rt, splits
BLOCKS = int(os.environ.get("PREFETCH_BLOCKS", "512"))


def graph_us(build, n, reps=3):
    """µs per item of a graph that runs build() (n items)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        build()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        build()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, 1000 * a.elapsed_time(b))
    return best / n


def main():
    load_library()
    op = torch.ops.hipserve
    dev = torch.device("cuda", 0)
    M = 64
    x = torch.randn(M, 14336, device=dev, dtype=torch.bfloat16)
    # the epilogue kernel of the decode layer that precedes qkv / gate|up
    res = torch.randn(M, 4096, device=dev, dtype=torch.bfloat16)
    nout = torch.empty(M, 4096, device=dev, dtype=torch.bfloat16)
    part = torch.randn(4 * M * 4096, device=dev, dtype=torch.float32)
    lnw = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream()

    def norm():
        op.splitk_add_rmsnorm(nout, res, part, 4, lnw, 1e-5, None, None, None)

    for name, (N, K, rt, S) in SHAPES.items():
        nbytes = N * K * 2
        ncopy = max(2, min(12, (1536 << 20) // nbytes))
        ws_ = [gemm.pack(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        xs = x[:, :K]
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        wsb = torch.empty(S * M * N, device=dev, dtype=torch.float32)

        def g(i):
            op.decode_gemm_packed(out, xs, ws_[i], wsb, N, rt, S)

        row = {"proj": name, "MB": round(nbytes / 2**20, 1), "blocks": BLOCKS}
        cold = graph_us(lambda: [g(i) for i in range(ncopy)], ncopy)
        row["cold_us"] = round(cold, 2)
        seq = graph_us(lambda: [(norm(), g(i)) for i in range(ncopy)], ncopy)
        row["norm+gemm_us"] = round(seq, 2)
        for P in (8, 16, 32, 64):
            nb = min(nbytes, P << 20)

            def pf(i, nb=nb):
                op.mall_prefetch(ws_[i], nb, BLOCKS)

            t_pf = graph_us(lambda: [pf(i) for i in range(ncopy)], ncopy)
            t_pg = graph_us(lambda: [(pf(i), g(i)) for i in range(ncopy)], ncopy)

            def forked():
                for i in range(ncopy):
                    cur = torch.cuda.current_stream()
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        pf(i)
                    norm()
                    cur.wait_stream(side)
                    g(i)

            t_fork = graph_us(forked, ncopy)
            row[f"P{P}"] = {"prefetch_us": round(t_pf, 2), "gemm_after_prefetch_us": round(t_pg - t_pf, 2),
                            "norm||prefetch+gemm_us": round(t_fork, 2)}
        print(json.dumps(row), flush=True)
        del ws_
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
