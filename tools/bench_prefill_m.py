#!/usr/bin/env python3
"""Prefill GEMM time vs token count M (hipBLASLt heuristic choice): is a ragged last
chunk (M not a multiple of the 256-row tile) slower per row than a full one?

    python tools/bench_prefill_m.py [--ms 8192 7393 7424 ...]

One JSON line per M: the four Llama-3-8B projections chained 8 times (the way a
prefill step streams them), device ms per chain and us per 1K rows.
"""
import argparse
import json

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", type=int, nargs="+", default=[8192, 7393, 7424, 7456, 7680, 7936, 4096, 4000])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) * 0.02 for n, k in shapes]
    xs = {k: torch.randn(8192, k, device=dev, dtype=torch.bfloat16) for _, k in shapes}
    for M in a.ms:
        def chain():
            for _ in range(8):
                for w, (n, k) in zip(ws, shapes):
                    F.linear(xs[k][:M], w)
        chain()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            chain()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[1]
        flops = 8 * sum(2 * M * n * k for n, k in shapes)
        print(json.dumps({"M": M, "chain_ms": round(ms, 3), "us_per_1k_rows": round(1000 * ms / M * 1000 / 8, 1),
                          "PFLOPs": round(flops / ms / 1e12, 3)}), flush=True)


if __name__ == "__main__":
    main()
