#!/usr/bin/env python3
"""Decode-sized bf16 GEMMs above 64 rows (the graph buckets of max_num_seqs 256) on
hipBLASLt: the default heuristic pick vs the TunableOp-searched solution (every
hipBLASLt / rocBLAS algorithm, including split-K ones), Llama-3-8B projection shapes.
Each timing is one hipGraph replay of the layer's four GEMMs back to back over 4 layer
copies (1.7 GB of weights: HBM-cold, as in a decode step).

    python tools/bench_decode_blas.py
"""
import json
import os
import sys
import tempfile

import torch

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def graph_us(fn, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, 1000 * a.elapsed_time(b))
    return best


def main():
    dev = "cuda"
    L = 4
    ws = {k: [torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)]
          for k, (n, kk) in SHAPES.items()}
    tmp = tempfile.mkdtemp()
    for tuned in (False, True):
        if tuned:
            import torch.cuda.tunable as T
            T.enable(True)
            T.tuning_enable(True)
            T.set_filename(os.path.join(tmp, "tunableop.csv"))
        for M in (128, 256):
            xs = {k: torch.randn(M, kk, device=dev, dtype=torch.bfloat16) for k, (n, kk) in SHAPES.items()}
            if tuned:  # tune each shape eagerly (outside capture), then freeze
                T.tuning_enable(True)
                for k in SHAPES:
                    torch.nn.functional.linear(xs[k], ws[k][0])
                torch.cuda.synchronize()
                T.tuning_enable(False)
            row = {"M": M, "tuned": tuned}
            for k in SHAPES:
                us = graph_us(lambda k=k: [torch.nn.functional.linear(xs[k], w) for w in ws[k]]) / L
                n, kk = SHAPES[k]
                row[k] = {"us": round(us, 1), "TBps": round(n * kk * 2 / us / 1e6, 2)}
            row["layer_us"] = round(sum(row[k]["us"] for k in SHAPES), 1)
            print(json.dumps(row), flush=True)
    if os.path.exists(os.path.join(tmp, "tunableop.csv")):
        print(open(os.path.join(tmp, "tunableop.csv")).read(), flush=True)


if __name__ == "__main__":
    sys.exit(main())
