#!/usr/bin/env python3
"""Decode GEMM device time with cold weights (rotating copies > the 256 MB MALL) vs
hot weights (one copy, MALL-resident after the first call): how much of a small
projection's time is HBM latency / bandwidth that a MALL prefetch could hide.

    python tools/bench_mall.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipserve.ops import gemm  # noqa: E402
from hipserve.ops import load_library  # noqa: E402


def main():
    load_library()
    dev = torch.device("cuda", 0)
    M = 64
    for (N, K, cfg) in [(4096, 4096, ("dgp", 1, 8)), (6144, 4096, ("dgp", 2, 4)), (4096, 14336, ("dgp", 1, 8)),
                        (28672, 4096, ("dgp", 1, 1))]:
        ncopy = max(1, min(16, -(-gemm.COLD_BYTES // (N * K * 2))))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
        wp = [gemm.pack(w) for w in ws]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cold = gemm.GemmTuner._time(lambda i: gemm.run_choice(cfg, out, x, ws[i % ncopy], wp[i % ncopy]), n=32)
        hot = gemm.GemmTuner._time(lambda i: gemm.run_choice(cfg, out, x, ws[0], wp[0]), n=32)
        mb = N * K * 2 / 1e6
        print(json.dumps({"N": N, "K": K, "cfg": str(cfg), "MB": round(mb, 1), "cold_us": round(cold, 2),
                          "hot_us": round(hot, 2), "cold_TBps": round(mb / cold, 2), "hot_TBps": round(mb / hot, 2)}),
              flush=True)
        del ws, wp


if __name__ == "__main__":
    main()
