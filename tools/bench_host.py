#!/usr/bin/env python3
"""Host-side ceiling of the serving path, no GPU needed.

The engine runs with a fake model runner whose "GPU" takes a fixed time per step
(``--decode-ms`` per decode step, ``--prefill-ms`` per prefill step) and returns
random tokens; everything else is the real serving path of bench.py: loadgen
process -> ingress emulator -> model-name router -> engine HTTP server (SSE) ->
engine loop with decode lookahead. If the host keeps up, a decode step takes
exactly ``--decode-ms``; the excess is host time the real GPU would sit idle for.

    python tools/bench_host.py --concurrency 64 --input-len 1024 --output-len 256 --decode-ms 4.5
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_fake_runner(decode_ms: float, prefill_ms: float, vocab: int, max_num_seqs: int, max_model_len: int,
                     num_blocks: int = 200000, block_size: int = 16):
    from hipserve.engine import model_runner as mr

    class FakeRunner(mr.ModelRunner):
        """ModelRunner.prepare (the real host batch builder) + a timed fake device."""

        def __init__(self, *a, **k):
            self.block_size = block_size
            self.max_model_len = max_model_len
            self.width = -(-max_model_len // block_size)
            self.num_blocks = num_blocks
            self.max_bs = max_num_seqs
            self.buckets = [b for b in mr.GRAPH_BUCKETS if b <= max_num_seqs] or [max_num_seqs]
            self.use_graphs = True
            self.gemm_report = []
            self.device_free_at = time.perf_counter()
            self.busy = 0.0
            self.rng = np.random.default_rng(0)
            self._free_pen = list(range(max_num_seqs))

        def _occupy(self, ms):
            now = time.perf_counter()
            start = max(now, self.device_free_at)
            self.device_free_at = start + ms / 1000.0
            self.busy += ms / 1000.0
            return self.device_free_at

        def launch(self, inp):
            return (self._occupy(decode_ms), inp.num_decode)

        def wait(self, handle):
            t, n = handle
            d = t - time.perf_counter()
            if d > 0:
                time.sleep(d)
            return self.rng.integers(10, vocab, n), np.zeros(n, np.float32), None

        def execute(self, inp):
            n = len(inp.logits_rows)
            if self.graph_eligible(inp):
                return self.wait(self.launch(inp))
            t = self._occupy(prefill_ms if inp.num_prefill_tokens else decode_ms)
            d = t - time.perf_counter()
            if d > 0:
                time.sleep(d)
            return self.rng.integers(10, vocab, n), np.zeros(n, np.float32), None

    return FakeRunner


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--decode-ms", type=float, default=4.5)
    ap.add_argument("--prefill-ms", type=float, default=90.0)
    ap.add_argument("--waves", type=int, default=2)
    ap.add_argument("--direct", action="store_true", help="loadgen -> engine port (no ingress / router)")
    a = ap.parse_args()

    from hipserve.bench.local_stack import GatewayStack, LoadgenProc, free_port, wait_http

    eport = free_port()
    stack = GatewayStack({"m": [eport]}).start()
    lg = LoadgenProc()
    from hipserve.config import PRESETS, EngineConfig
    from hipserve.engine import llm_engine
    from hipserve.parallel.comm import TPGroup

    mcfg = PRESETS["llama-3-8b"]
    max_len = a.input_len + a.output_len + 64
    llm_engine.ModelRunner = make_fake_runner(a.decode_ms, a.prefill_ms, mcfg.vocab_size, a.concurrency, max_len)
    cfg = EngineConfig(model="llama-3-8b", device="cpu", max_num_seqs=a.concurrency, max_model_len=max_len,
                       max_num_batched_tokens=8192)
    eng = llm_engine.LLMEngine(cfg, tp=TPGroup(), model_cfg=mcfg)
    eng.lookahead = True
    steps = []
    orig = eng._step_done

    def step_done(so, dt):
        steps.append((time.perf_counter(), len(so.prefill), len(so.decode)))
        orig(so, dt)

    eng._step_done = step_done
    arrivals = []
    orig_add = eng.add_request

    def add_request(*a, **k):
        arrivals.append(time.perf_counter())
        return orig_add(*a, **k)

    eng.add_request = add_request
    from hipserve.server.api_server import serve

    threading.Thread(target=lambda: asyncio.run(serve(eng, "127.0.0.1", eport, "m")), daemon=True).start()
    wait_http(f"http://127.0.0.1:{eport}/health", 60)
    t_all = []
    for w in range(a.waves):
        steps.clear()
        arrivals.clear()
        t0 = time.perf_counter()
        res = lg.wave(url=f"http://127.0.0.1:{eport}" if a.direct else stack.url, model="m", concurrency=a.concurrency, input_len=a.input_len,
                      output_len=a.output_len, vocab=100000, temperature=0.8, top_p=0.95)
        el = time.perf_counter() - t0
        t_all.append(el)
        dec = [steps[i][0] - steps[i - 1][0] for i in range(1, len(steps))
               if steps[i][1] == 0 and steps[i - 1][1] == 0 and steps[i][2] == a.concurrency]
        tok = sum(r["tokens"] for r in res)
        pre = [steps[i][0] - steps[i - 1][0] for i in range(1, len(steps)) if steps[i][1]]
        lead = steps[0][0] - t0 if steps else None
        tail = t0 + el - steps[-1][0] if steps else None
        out = {"wave": w, "elapsed_s": round(el, 3), "tok_per_s": round(tok / el, 1),
               "decode_steps": len(dec), "decode_step_ms_p50": round(1000 * statistics.median(dec), 3) if dec else None,
               "simulated_decode_ms": a.decode_ms,
               "p50_ttft_ms": round(1000 * statistics.median(r["ttft"] for r in res), 1),
               "first_step_at_ms": round(1000 * lead, 1), "after_last_step_ms": round(1000 * tail, 1),
               "steps": len(steps), "prefill_steps": len(pre) + 1,
               "first_arrival_ms": round(1000 * (arrivals[0] - t0), 1) if arrivals else None,
               "last_arrival_ms": round(1000 * (arrivals[-1] - t0), 1) if arrivals else None,
               "decode_total_ms": round(1000 * sum(dec), 1)}
        print(json.dumps(out), flush=True)
    lg.close()
    stack.stop()


if __name__ == "__main__":
    main()
