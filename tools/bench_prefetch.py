#!/usr/bin/env python3
"""Does a decode GEMM start faster when the first part of its weight is already in the
256 MiB MALL (Infinity Cache)? Decode steps stream every weight once from HBM, and each
GEMM pays a ramp (first loads at HBM latency, per-CU bandwidth share) — if a weight
prefix read into the MALL ahead of the kernel (e.g. by a side-stream kernel while a
short epilogue kernel runs) removes part of that ramp, a prefetch branch in the decode
graph could hide it.

For each Llama-3-8B decode shape at M = 64 (packed decode GEMM, fixed config), over
copies of the weight rotated so every call is HBM-cold:
    cold      the GEMM alone
    touch     a read of the first P MiB of the weight copy alone
    touch+g   the read, then the GEMM (same graph)
GEMM time with a warm prefix = (touch+g) - touch.

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


def graph_us(fns, reps=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fns:
            f()
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
    return best / len(fns)


def main():
    load_library()
    dev = torch.device("cuda", 0)
    M = 64
    x = torch.randn(M, 14336, device=dev, dtype=torch.bfloat16)
    for name, (N, K, rt, S) in SHAPES.items():
        nbytes = N * K * 2
        ncopy = max(2, min(12, (1536 << 20) // nbytes))
        ws_ = [gemm.pack(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        xs = x[:, :K]
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ws = torch.empty(S * M * N, device=dev, dtype=torch.float32)
        sink = torch.empty(ncopy, device=dev, dtype=torch.float32)

        def gemm_fn(i):
            return lambda: torch.ops.hipserve.decode_gemm_packed(out, xs, ws_[i], ws, N, rt, S)

        cold = graph_us([gemm_fn(i) for i in range(ncopy)])
        row = {"proj": name, "MB": round(nbytes / 2**20, 1), "cold_us": round(cold, 2),
               "cold_TBps": round(nbytes / cold / 1e6, 2)}
        for P in (8, 16, 32, 64):
            n = min(ws_[0].numel(), (P << 20) // 2)

            def touch(i, n=n):
                # reads the first P MiB of copy i (fp32 view: one sum kernel)
                return lambda: torch.sum(ws_[i][:n].view(torch.float32), out=sink[i])

            t = graph_us([touch(i) for i in range(ncopy)])
            tg = graph_us([f for i in range(ncopy) for f in (touch(i), gemm_fn(i))]) * 2
            row[f"P{P}_touch_us"] = round(t, 2)
            row[f"P{P}_gemm_us"] = round(tg - t, 2)
        print(json.dumps(row), flush=True)
        del ws_
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
