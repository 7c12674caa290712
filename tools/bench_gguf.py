#!/usr/bin/env python3
"""GGUF decode-GEMM microbenchmark on one MI355X: the v1 per-part kernel
(csrc/kernels/gguf.hip) vs the v2 f16-MFMA kernel (csrc/kernels/gguf_mfma.hip)
on the Llama-3-8B Q4_K_M projection shapes, random valid ggml blocks.

    python tools/bench_gguf.py --m 1 16 64

One JSON line per (projection, M, kernel): µs per call and the weight-byte
bandwidth (TB/s) — decode GEMMs are bound by streaming the quantised weights.
Each M also sweeps the split-K factor (``--splits``, default 1 .. 32).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hipserve.ops import load_library  # noqa: E402
from hipserve.ops import quant as Q  # noqa: E402
from hipserve.weights import gguf as G  # noqa: E402

H, I, NQ, NKV, D, V = 4096, 14336, 32, 8, 128, 128256
SHAPES = {  # Q4_K_M: attn_v / ffn_down / output in Q6_K
    "qkv": [(G.Q4_K, NQ * D, H), (G.Q4_K, NKV * D, H), (G.Q6_K, NKV * D, H)],
    "o": [(G.Q4_K, H, NQ * D)],
    "gate_up": [(G.Q4_K, I, H), (G.Q4_K, I, H)],
    "down": [(G.Q6_K, H, I)],
    "lm_head": [(G.Q6_K, V, H)],
}


def _time(fn, reps=20, graph_reps=10):
    """Device µs per call: ``reps`` calls captured in one hipGraph (no host launch
    cost, like the engine's decode step), replayed ``graph_reps`` times."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(graph_reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / (reps * graph_reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16, 64])
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--splits", type=int, nargs="*", default=None)
    ap.add_argument("--fp8", action="store_true", help="FP8 e4m3 per-channel weights of the same shapes")
    ap.add_argument("--prefill", action="store_true",
                    help="M > 64: the prefill GEMM from the blocks (qpf) and the M-tiled dequant-MFMA kernel vs "
                         "dequant-to-scratch + hipBLASLt vs a bf16 shadow")
    ap.add_argument("--no-mtiled", action="store_true", help="--prefill: skip the (slow at large M) M-tiled kernel")
    ap.add_argument("--cold", action="store_true",
                    help="rotate every timed call over copies of the blocks (>= 768 MiB): HBM-cold weights, "
                         "as in a decode step, instead of MALL-resident ones")
    a = ap.parse_args()
    load_library()
    rng = np.random.default_rng(0)
    for name, specs in SHAPES.items():
        if a.only and name not in a.only:
            continue
        if a.fp8:
            parts = []
            for _, n, k in specs:
                w = torch.randn(n, k, device="cuda") * 0.02
                sc = w.abs().amax(1, keepdim=True) / 448.0
                parts.append(Q.QuantPart.from_fp8((w / sc).to(torch.float8_e4m3fn), sc, "cuda"))
                del w
            qw = Q.QuantWeight(parts)
        else:
            raws = [(t, n, k, Q.random_blocks(rng, t, n, k)) for t, n, k in specs]
            qw = Q.QuantWeight.from_raw(raws, "cuda")
            del raws
        for M in a.m:
            x = torch.randn(M, qw.K, device="cuda", dtype=torch.bfloat16)
            if a.prefill:
                out = torch.empty(M, qw.N, device="cuda", dtype=torch.bfloat16)
                dense = Q.dequantize(qw)
                buf = torch.empty_like(dense)

                def deq_blas():
                    off = 0
                    for p in qw.parts:
                        Q._dequant_into(buf[off:off + p.N], p)
                        off += p.N
                    return torch.nn.functional.linear(x, buf)

                cols = np.cumsum([0] + [p.N for p in qw.parts])[:-1].tolist()
                qargs = ([p.q for p in qw.parts], [p.kqt for p in qw.parts], [p.N for p in qw.parts], cols)
                act = torch.empty(M, qw.N // 2, device="cuda", dtype=torch.bfloat16)
                x16, rsc = Q.x_f16_pairs(x, qw.K)
                kerns = [("qpf_prefill", lambda: torch.ops.hipserve.gguf_prefill(out, x16, rsc, *qargs, qw.K, 0)),
                         ("qpf_prefill+x_conv", lambda: Q.qprefill(x, qw, 0, out))]
                if name == "gate_up":
                    kerns.append(("qpf_prefill_glu", lambda: torch.ops.hipserve.gguf_prefill(act, x16, rsc, *qargs, qw.K, 2)))
                if not a.no_mtiled:
                    kerns.append(("m_tiled_mfma", lambda: Q._launch_v2(out, Q._empty(x.device, torch.float32), x, qw, 1)))
                kerns += [("dequant+hipblaslt", deq_blas),
                          ("bf16_shadow_hipblaslt", lambda: torch.nn.functional.linear(x, dense))]
                for kern, fn in kerns:
                    us = _time(fn, reps=10, graph_reps=5)
                    print(json.dumps({"proj": name, "M": M, "kernel": kern, "us": round(us, 1),
                                      "TFLOPs": round(2 * M * qw.N * qw.K / us / 1e6, 1)}), flush=True)
                del dense, buf
                continue
            rows = []
            qw.groups
            ncopy = max(1, min(64, -(-(768 << 20) // qw.nbytes))) if a.cold else 1
            copies = [qw.v2_args[0]] + [[q.clone() for q in qw.v2_args[0]] for _ in range(ncopy - 1)]

            def timed(launch):  # µs per call, over the block copies
                return _time(lambda: [launch(qs) for qs in copies], reps=max(1, 20 // ncopy)) / ncopy

            rows.append(("v2_partial", Q.v2_splits(qw, M), _time(lambda: Q.quant_partial(x, qw))))
            x16 = None
            if 32 < M <= 64:  # x staged from a producer's f16 pair-order copy (out16 / act16)
                h = x.float().to(torch.float16).reshape(M, -1, 8)[:, :, [0, 2, 1, 3, 4, 6, 5, 7]].reshape(M, -1)
                x16 = h.contiguous()
                rows.append(("v2_partial_x16", Q.v2_splits(qw, M), _time(lambda: Q.quant_partial(x, qw, x16))))
            nsb = qw.K // 256
            e = Q._empty(x.device, torch.bfloat16)
            for Sx in sorted({-(-nsb // -(-nsb // S)) for S in (a.splits or (1, 2, 4, 8, 16, 32)) if S <= nsb}):
                ws = torch.empty(Sx * M * qw.N, dtype=torch.float32, device="cuda")
                rows.append((f"v2_S{Sx}", Sx, timed(lambda qs: Q._launch_v2(e, ws, x, qw, Sx, x16, qs))))
            del copies
            for kern, S, us in rows:
                print(json.dumps({"proj": name, "M": M, "kernel": kern, "splits": S, "us": round(us, 2),
                                  "weight_MB": round(qw.nbytes / 1e6, 2), "cold": a.cold,
                                  "TBps": round(qw.nbytes / us / 1e6, 3),
                                  "partial_MB": round(S * M * qw.N * 4 / 1e6, 2)}), flush=True)
        del qw
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
