#!/usr/bin/env python3
"""Repeatability of the decode GEMM tuner's unit timings: the fused o_proj unit (GEMM +
split-K add + RMSNorm, Llama-3-8B 4096 x 4096 at 64 rows) for a few configs, timed in
interleaved rounds exactly as ops/gemm.py GemmTuner does.

    python tools/tune_probe.py [N K]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipserve.ops import gemm, load_library  # noqa: E402


@torch.inference_mode()
def main():
    load_library()
    N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4096, 4096)
    dev = torch.device("cuda", 0)
    M = 64
    ncopy = max(1, min(16, -(-gemm.COLD_BYTES // (N * K * 2))))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(ncopy)]
    wp = [gemm.pack(w) for w in ws]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    unit = gemm._Unit(("norm",), M, N, dev)
    cands = [c for c in gemm.GemmTuner.candidates(M, N, K, packed=True) if c[0] == "dgp"]
    times = {c: [] for c in cands}
    for _ in range(4):
        for c in cands:
            times[c].append(gemm.GemmTuner._time(lambda i, c=c: unit.fused(c, x, ws[i % ncopy], wp[i % ncopy]),
                                                 n=max(16, ncopy)))
    for c in sorted(cands, key=lambda c: sorted(times[c])[1]):
        print(json.dumps({"cfg": str(c), "us": [round(t, 2) for t in times[c]]}), flush=True)


if __name__ == "__main__":
    main()
