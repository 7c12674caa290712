#!/usr/bin/env python3
"""hipBLASLt speed of the Llama-3-8B prefill GEMMs (M = 8192) by operand layout."""
import json

import torch
import torch.nn.functional as F

M, H, I = 8192, 4096, 14336
dev = "cuda"


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for name, (N, K) in {"qkv": (6144, H), "o": (H, H), "gu": (2 * I, H), "down": (H, I)}.items():
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    wt = w.t().contiguous()          # [K, N]
    xt = x.t().contiguous()          # [K, M]
    r = {"linear_x_wT": t(lambda: F.linear(x, w)),
         "mm_x_wt": t(lambda: x @ wt),
         "mm_w_xT(out^T)": t(lambda: w @ xt),
         "mm_w_xtview": t(lambda: torch.mm(w, x.t()))}
    fl = 2 * M * N * K
    print(json.dumps({"gemm": name, **{k: round(v, 4) for k, v in r.items()},
                      "best_PF": round(fl / (min(r.values()) * 1e-3) / 1e15, 3)}), flush=True)
