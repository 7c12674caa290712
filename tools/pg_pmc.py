#!/usr/bin/env python3
"""Minimal driver for PMC passes on one prefill-GEMM shape: 3 hipBLASLt calls then 3
hand-written packed prefill GEMM calls per variant in $PG_VARIANTS (p1 / p2 = wm; default p1) on the same operands, so one rocprofv3
--pmc pass gives per-dispatch counters of both kernels side by side.
usage: python tools/pg_pmc.py [M N K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from hipserve.ops import load_library

load_library()
M, N, K = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (8192, 28672, 4096)
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    F.linear(x, w)
torch.cuda.synchronize()
wp = None
for v in os.environ.get("PG_VARIANTS", "p1").split():
    for _ in range(3):
        if v.startswith("p"):  # packed-layout kernel (prefill_gemm_packed.hip), p1 / p2 = wm
            if wp is None:
                wp = torch.empty(-(-N // 128) * 128 * K, device="cuda", dtype=torch.bfloat16)
                torch.ops.hipserve.pack_decode_weight(wp, w, False)
            torch.ops.hipserve.prefill_gemm_packed(out, x, wp, N, 0, None, int(v[1]), 0, int(os.environ.get("PW_RW", "4")))
    torch.cuda.synchronize()
print("ok", M, N, K)
