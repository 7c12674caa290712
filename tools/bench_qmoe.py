"""Time the quantised expert GEMM (qmoe_gemm, gguf_mfma.hip MoE mode) of one
Qwen3-30B-A3B MoE layer at decode batch sizes: w13 (gathered token rows) and w2
(slot rows, split over K), INT8 (per-32-k scale / offset table) vs INT8C (per-channel,
row scale in the epilogue) vs FP8, at several K splits. Graph-timed over ``--layers``
distinct layers (their experts exceed the MALL); TB/s counts the bytes of the experts
that received tokens.

    python tools/bench_qmoe.py [--tokens 16,64,128] [--layers 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_ops import graph_time  # noqa: E402


def experts(E, N, K, kind, dev, g):
    from hipserve.ops import quant as Q
    parts = []
    for _ in range(E):
        wf = torch.randn(N, K, device=dev, generator=g) * 0.02
        s = wf.abs().amax(1, keepdim=True) / 127.0
        if kind == "fp8":
            s8 = wf.abs().amax(1, keepdim=True) / 448.0
            parts.append(Q.QuantPart.from_fp8((wf / s8).to(torch.float8_e4m3fn), s8, dev))
        else:
            q = torch.round(wf / s).clamp(-127, 127)
            parts.append(Q.QuantPart.from_int8((q + 128).to(torch.uint8), s, None, dev, channel=kind == "int8c"))
    return Q.QuantMoE(parts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="16,64,128")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--kinds", default="int8,int8c,fp8")
    ap.add_argument("--model", default="qwen3-30b-a3b")
    ap.add_argument("--kmajor", default="0,1", help="expert layouts timed: 0 row-group major, 1 super-chunk major")
    a = ap.parse_args()

    from hipserve.config import PRESETS
    from hipserve.ops import load_library

    load_library()
    op = torch.ops.hipserve
    dev = torch.device("cuda:0")
    cfg = PRESETS[a.model]
    E, H, I, k = cfg.num_experts, cfg.hidden_size, cfg.moe_intermediate_size or cfg.intermediate_size, \
        cfg.num_experts_per_tok
    g = torch.Generator(device=dev).manual_seed(0)
    f32 = torch.empty(0, dtype=torch.float32, device=dev)
    def kmaj(w):  # [E][N/16][K/256][chunk] -> [E][K/256][N/16][chunk]
        G, nsb = w.N // 16, w.K // 256
        return w.q.view(w.E, G, nsb, -1).transpose(1, 2).contiguous().view(w.E, -1)

    for kind, km in [(kd, int(m)) for kd in a.kinds.split(",") for m in a.kmajor.split(",")]:
        layers = [(experts(E, 2 * I, H, kind, dev, g), experts(E, H, I, kind, dev, g)) for _ in range(a.layers)]
        if km:
            for w13, w2 in layers:
                w13.q, w2.q = kmaj(w13), kmaj(w2)
        torch.cuda.synchronize()
        for T in [int(t) for t in a.tokens.split(",")]:
            P = T * k
            tile = 16 if P <= 8 * E else (32 if P <= 32 * E else 64)
            cap = -(-(P + E * (tile - 1)) // tile) * tile
            x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
            routes = []
            for _ in range(a.layers):
                ids = torch.topk(torch.rand(T, E, device=dev, generator=g), k, dim=-1).indices.int()
                slots = torch.empty(cap, dtype=torch.int32, device=dev)
                te = torch.empty(cap // tile, dtype=torch.int32, device=dev)
                nt = torch.empty(1, dtype=torch.int32, device=dev)
                ps = torch.empty(P, dtype=torch.int32, device=dev)
                op.moe_align(ids, E, tile, slots, te, nt, ps)
                routes.append((slots, te, int(torch.unique(ids).numel())))
            act_e = sum(r[2] for r in routes) / len(routes)
            w13_0, w2_0 = layers[0]
            b13 = w13_0.q.shape[1] * act_e
            b2 = w2_0.q.shape[1] * act_e
            gu = torch.empty(cap, 2 * I, device=dev, dtype=torch.bfloat16)
            act = torch.randn(cap, I, device=dev, dtype=torch.bfloat16)
            for S in (1, 2, 4):
                if (H // 256) % S:
                    continue
                ws = torch.empty(S, cap, 2 * I, device=dev) if S > 1 else f32
                it = [0]

                def f13():
                    i = it[0] = (it[0] + 1) % a.layers
                    w13 = layers[i][0]
                    sl, te, _ = routes[i]
                    op.qmoe_gemm(gu, ws, x, w13.q, w13.rs, w13.kqt, w13.N, w13.K, sl, te, tile, k, S, bool(km))
                us = graph_time(f13, n=4 * a.layers)
                print(json.dumps({"kind": kind, "kmajor": km, "T": T, "gemm": "w13", "S": S, "tile": tile, "active": act_e,
                                  "us": round(us, 2), "TBps": round(b13 / us / 1e6, 2)}), flush=True)
            for S in (1, 2, 3):
                if (I // 256) % S:
                    continue
                ws = torch.empty(S, cap, H, device=dev) if S > 1 else f32
                y = torch.empty(cap, H, device=dev, dtype=torch.bfloat16)
                it = [0]

                def f2():
                    i = it[0] = (it[0] + 1) % a.layers
                    w2 = layers[i][1]
                    sl, te, _ = routes[i]
                    op.qmoe_gemm(y, ws, act, w2.q, w2.rs, w2.kqt, w2.N, w2.K, sl, te, tile, 0, S, bool(km))
                us = graph_time(f2, n=4 * a.layers)
                print(json.dumps({"kind": kind, "kmajor": km, "T": T, "gemm": "w2", "S": S, "tile": tile, "active": act_e,
                                  "us": round(us, 2), "TBps": round(b2 / us / 1e6, 2)}), flush=True)
        del layers
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
