#!/usr/bin/env python3
"""Where a pipelined decode step's wall time goes: host engine phases vs device time.

Runs the bench's engine path shape (N concurrent requests, synthetic prompts, random
weights) with ``HIPSERVE_PROFILE=timing`` and reports, over the decode-only steady
state: wall ms per step (between consecutive ``step()`` returns) and
the host phases (schedule / prepare / launch / wait / process). ``wait`` is the time
the host blocks on the GPU: near zero means the host, not the GPU, paces the loop.

    python tools/decode_gap.py --model llama-3-8b --concurrency 64
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ["HIPSERVE_PROFILE"] = "timing"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--block-size", type=int, default=16)
    ap.add_argument("--decode-partition", type=int, default=512)
    a = ap.parse_args()
    import numpy as np
    import torch

    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    eng = LLMEngine(EngineConfig(model=a.model, load_format="dummy", device="cuda", max_num_seqs=a.concurrency,
                                 max_num_batched_tokens=8192, max_model_len=a.input_len + a.output_len + 16,
                                 block_size=a.block_size, decode_partition=a.decode_partition),
                    tp=TPGroup(0, 1, None, torch.device("cuda", 0)))
    rng = np.random.default_rng(0)
    sp = SamplingParams(temperature=0.8, top_p=0.95, max_tokens=a.output_len, ignore_eos=True)
    for _ in range(a.concurrency):
        eng.add_request(None, rng.integers(10, 30000, a.input_len).tolist(), sp)
    tr = eng.tracer
    stamps = []
    while eng.has_unfinished():
        outs = eng.step()
        stamps.append((time.perf_counter(), sum(len(o.new_token_ids) for o in outs), eng.runner.stats["graph_steps"]))
        if len(stamps) == 40:  # decode steady state from here: reset the phase counters
            base = {k: list(v) for k, v in tr.times.items()}
            t_base = stamps[-1][0]
            i_base = len(stamps)
        if len(stamps) == 40 + 150:
            break
    n = len(stamps) - i_base
    wall = (stamps[-1][0] - t_base) / n
    rep = {"steps": n, "wall_ms_per_step": round(1000 * wall, 3), "tokens_per_step": stamps[-1][1]}
    for k, (c, t) in tr.times.items():
        c0, t0 = base.get(k, [0, 0.0])
        if c - c0:
            rep[f"{k}_ms"] = round(1000 * (t - t0) / n, 3)
    print(json.dumps(rep), flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
