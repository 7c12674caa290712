#!/usr/bin/env python3
"""Workload for PMC passes over the GGUF prefill GEMM (scripts/pg_pmc.sh with
PMC_PY=tools/qpf_pmc.py): Llama-3-8B gate|up in Q4_K (or down in Q6_K with --down), M
tokens, GLU epilogue, a few launches after a warm-up."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipserve.ops import load_library  # noqa: E402
from hipserve.ops import quant as Q  # noqa: E402
from hipserve.weights import gguf as G  # noqa: E402


def main():
    load_library()
    M = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 8192
    down = "--down" in sys.argv
    rng = np.random.default_rng(0)
    if down:
        qw = Q.QuantWeight.from_raw([(G.Q6_K, 4096, 14336, Q.random_blocks(rng, G.Q6_K, 4096, 14336))], "cuda")
        epi = 0
    else:
        qw = Q.QuantWeight.from_raw([(G.Q4_K, 14336, 4096, Q.random_blocks(rng, G.Q4_K, 14336, 4096))] * 2, "cuda")
        epi = 2
    x = torch.randn(M, qw.K, device="cuda", dtype=torch.bfloat16)
    for _ in range(4):
        Q.qprefill(x, qw, epi)
    torch.cuda.synchronize()
    print("ok", M, "down" if down else "gate_up")


if __name__ == "__main__":
    main()
