#!/usr/bin/env python3
"""Prefill GEMM operand layout on hipBLASLt: F.linear(x, W[N, K]) (the engine's plain copy)
against x @ Wt with Wt = W^T stored [K, N] contiguous, at prefill row counts, Llama-3-8B
projections. Rotates weight copies past the MALL like the engine (every layer's weights
are cold by the time it runs). Prints one JSON line per (shape, M)."""
import json
import sys

import torch
import torch.nn.functional as F


def timed(fn, n=20, reps=3):
    best = 1e30
    for _ in range(reps):
        fn(0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(i)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / n)
    return best


def main():
    ms = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2048, 8192]
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    for N, K in shapes:
        nc = max(2, -(-(512 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(nc)]
        wts = [w.t().contiguous() for w in ws]
        for M in ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            t_nt = timed(lambda i: F.linear(x, ws[i % nc]))
            t_nn = timed(lambda i: torch.matmul(x, wts[i % nc]))
            fl = 2.0 * M * N * K
            print(json.dumps({"N": N, "K": K, "M": M, "linear_ms": round(t_nt, 4), "nn_ms": round(t_nn, 4),
                              "linear_PF": round(fl / t_nt / 1e12, 3), "nn_PF": round(fl / t_nn / 1e12, 3)}),
                  flush=True)
        del ws, wts


if __name__ == "__main__":
    main()
