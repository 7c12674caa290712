#!/usr/bin/env python3
"""Decode GEMM chain (csrc/kernels/decode_chain.hip) vs the three launches it replaces,
at the Llama-3-8B decode shapes (M = 64), graph-captured, weights cycled over 4 copies
(> the 256 MB MALL) like a decode step streams them:

  o:    decode_gemm_partial(o_proj) -> splitk_add_rmsnorm -> decode_gemm_glu(gate|up)
  down: decode_gemm_partial(down)   -> splitk_add_rmsnorm -> decode_gemm_partial(qkv)

    python tools/bench_chain.py [--m 64]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipserve.ops import gemm, load_library  # noqa: E402

DEV = "cuda"


def graph_us(fn, iters=8, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(iters):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(iters):
                fn(i)
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / iters)
    return best


def timeline(name, run, blocks):
    """One launch with per-block timestamps (s_memrealtime, 100 MHz): when the producers'
    GEMMs end, when the reducers finish, when consumers start / pass the wait / end."""
    flush = torch.empty(1 << 28, device=DEV, dtype=torch.int32)
    dbg = torch.zeros(8 * blocks, device=DEV, dtype=torch.int64)
    for _ in range(3):
        flush.add_(1)
        run(dbg)
    torch.cuda.synchronize()
    d = dbg.view(-1, 8).cpu()
    t0 = d[:, 0].min().item()
    us = lambda v: round((v - t0) / 100.0, 2)  # noqa: E731
    prod, cons = d[d[:, 3] == 0], d[d[:, 3] == 2]
    out = {"timeline": name, "producers": len(prod), "consumers": len(cons),
           "prod_start_max": us(prod[:, 0].max().item()), "prod_gemm_end_med": us(prod[:, 1].median().item()),
           "prod_gemm_end_max": us(prod[:, 1].max().item()), "prod_exit_max": us(prod[:, 2].max().item()),
           "cons_start_min": us(cons[:, 0].min().item()), "cons_start_med": us(cons[:, 0].median().item()),
           "cons_start_max": us(cons[:, 0].max().item()), "cons_wait_end_min": us(cons[:, 1].min().item()),
           "cons_wait_end_max": us(cons[:, 1].max().item()), "cons_end_med": us(cons[:, 2].median().item()),
           "cons_end_max": us(cons[:, 2].max().item())}
    red = cons[cons[:, 4] > 0]
    out.update({"reducers": len(red), "red_wait_end_min": us(red[:, 4].min().item()),
                "red_wait_end_max": us(red[:, 4].max().item()), "red_end_min": us(red[:, 5].min().item()),
                "red_end_max": us(red[:, 5].max().item()), "rdone_seen_min": us(cons[:, 6].min().item()),
                "rdone_seen_max": us(cons[:, 6].max().item())})
    print(json.dumps(out), flush=True)
    del flush


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--copies", type=int, default=4)
    args = ap.parse_args()
    load_library()
    op = torch.ops.hipserve
    M, H, I, Q = args.m, 4096, 14336, 6144
    bf = dict(device=DEV, dtype=torch.bfloat16)
    nc = args.copies
    gamma = (torch.rand(H, device=DEV) + 0.5).to(torch.bfloat16)
    res = torch.randn(M, H, **bf)
    xn = torch.empty(M, H, **bf)
    sync = torch.zeros(4096, device=DEV, dtype=torch.int32)
    sq = torch.empty(H // 128 * 64, device=DEV, dtype=torch.float32)
    e = torch.empty(0, device=DEV)
    e16 = torch.empty(0, **bf)

    def pk(n, k, glu=False):
        return [gemm.pack((torch.randn(n, k, device=DEV) * 0.02).to(torch.bfloat16), glu=glu) for _ in range(nc)]

    # ---- o_proj -> ln2 -> gate|up ----
    wo, wgu = pk(H, H), pk(2 * I, H, glu=True)
    attn = torch.randn(M, H, **bf)
    act = torch.empty(M, I, **bf)
    ws8 = torch.empty(8 * M * H, device=DEV, dtype=torch.float32)
    ws_q = torch.empty(4 * M * Q, device=DEV, dtype=torch.float32)

    def o_unfused(i, rt=3, S=4):
        op.decode_gemm_partial(ws8, attn, wo[i % nc], H, rt, S, True)
        op.splitk_add_rmsnorm(xn, res, ws8, S, gamma, 1e-5)
        op.decode_gemm_glu(act, xn, wgu[i % nc], e, 2 * I, 1, 1)

    def o_chain(i, SA=8):
        op.decode_chain(act, e, res, ws8, sq, sync, attn, wo[i % nc], wgu[i % nc], gamma, SA, 2 * I, 1, True, 1e-5)

    rows = []
    rows.append({"chain": "o->ln2->gate|up", "path": "unfused rt3 S4", "us": graph_us(o_unfused)})
    rows.append({"chain": "o->ln2->gate|up", "path": "unfused rt1 S8",
                 "us": graph_us(lambda i: o_unfused(i, 1, 8))})
    for SA in (8, 4):
        rows.append({"chain": "o->ln2->gate|up", "path": f"decode_chain SA{SA}", "us": graph_us(lambda i: o_chain(i, SA))})
    # the parts alone
    timeline("o->ln2->gate|up", lambda dbg: op.decode_chain(act, e, res, ws8, sq, sync, attn, wo[1], wgu[1], gamma, 8,
                                                               2 * I, 1, True, 1e-5, dbg), H // 128 * 8 + 2 * I // 128)
    rows.append({"chain": "o->ln2->gate|up", "path": "gate|up glu alone",
                 "us": graph_us(lambda i: op.decode_gemm_glu(act, xn, wgu[i % nc], e, 2 * I, 1, 1))})
    del wo, wgu
    torch.cuda.empty_cache()

    # ---- down -> next ln1 -> qkv partials ----
    wd, wqkv = pk(H, I), pk(Q, H)
    a_in = torch.randn(M, I, **bf)

    def d_unfused(i):
        op.decode_gemm_partial(ws8, a_in, wd[i % nc], H, 1, 8, True)
        op.splitk_add_rmsnorm(xn, res, ws8, 8, gamma, 1e-5)
        op.decode_gemm_partial(ws_q, xn, wqkv[i % nc], Q, 1, 4, True)

    def d_chain(i):
        op.decode_chain(e16, ws_q, res, ws8, sq, sync, a_in, wd[i % nc], wqkv[i % nc], gamma, 8, Q, 4, False, 1e-5)

    timeline("down->ln1->qkv", lambda dbg: op.decode_chain(e16, ws_q, res, ws8, sq, sync, a_in, wd[1], wqkv[1], gamma,
                                                              8, Q, 4, False, 1e-5, dbg), H // 128 * 8 + Q // 128 * 4)
    rows.append({"chain": "down->ln1->qkv", "path": "unfused", "us": graph_us(d_unfused)})
    rows.append({"chain": "down->ln1->qkv", "path": "decode_chain SA8 SB4", "us": graph_us(d_chain)})
    torch.cuda.synchronize()
    err = int(sync[64].item())
    for r in rows:
        r["us"] = round(r["us"], 2)
        r["M"] = M
        print(json.dumps(r), flush=True)
    print(json.dumps({"sync_err": err, "sync_clean": int(sync.abs().sum().item()) == 0}), flush=True)


if __name__ == "__main__":
    main()
