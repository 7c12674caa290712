#!/usr/bin/env python3
"""Back-to-back hipGraph replay cost on one MI355X: how much device time separates
two consecutive graph launches, and what a replay costs on the host, for graphs of
N small kernels (a decode step is ~270 kernels).

    python tools/bench_graph_gap.py --kernels 274 --us 20

Prints one JSON line per configuration: device time per replay when replays run
back to back (events around R replays) vs the graph's own device time (events
around one replay at a time), and the host wall time of ``replay()``.
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=274)
    ap.add_argument("--elems", type=int, default=1 << 16, help="elements touched per kernel")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--event", action="store_true",
                    help="record a torch.cuda.Event after every replay, as the engine's launch() does")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.elems, device=dev)
    s = torch.cuda.Stream()
    graphs = []
    for par in range(2):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                x.mul_(1.0000001)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.kernels):
                x.mul_(1.0000001)
        graphs.append(g)
    torch.cuda.synchronize()
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    # one graph at a time (idle between): its own device time
    single = []
    for i in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        graphs[i & 1].replay()
        e1.record()
        torch.cuda.synchronize()
        single.append(e0.elapsed_time(e1))
    # back to back, alternating the two graph execs (the engine's parity graphs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = []
    e0.record()
    for i in range(a.reps):
        t = time.perf_counter()
        graphs[i & 1].replay()
        if a.event:
            torch.cuda.Event().record()
        host.append(time.perf_counter() - t)
    e1.record()
    torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) / a.reps
    single.sort()
    host.sort()
    print(json.dumps({"kernels": a.kernels, "event": a.event, "graph_device_ms": round(single[len(single) // 2], 4),
                      "back_to_back_ms_per_replay": round(b2b, 4),
                      "gap_us": round(1000 * (b2b - single[len(single) // 2]), 1),
                      "host_replay_us_p50": round(1e6 * host[len(host) // 2], 1)}), flush=True)


if __name__ == "__main__":
    main()
