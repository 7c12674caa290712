#!/usr/bin/env python3
"""One rank of a TP=N engine whose ranks share ONE GPU (the 1-GPU box's stand-in
for a TP pod): every collective is the in-house HIP-IPC kernel set (fused
cross-rank add+RMSNorm, IPC logits all-gather), the process group is gloo, and
decode runs hipGraphs with one-step lookahead — the TP serving path.

Each rank is its own top-level process so each can run under its own profiler:

    RANK=0 WORLD_SIZE=2 MASTER_PORT=29555 rocprofv3 --kernel-trace --stats -d out/r0 -- \\
        python3 tools/tp_shared_gpu.py &
    RANK=1 WORLD_SIZE=2 MASTER_PORT=29555 rocprofv3 --kernel-trace --stats -d out/r1 -- \\
        python3 tools/tp_shared_gpu.py
    wait

Rank 0 prints one JSON line (decode tok/s of this shared-GPU setup — two ranks
time-slice one GPU, so it measures overheads and kernel shapes, not TP speed-up).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--layers", type=int, default=None, help="override num_layers (smaller trace)")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--input-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=128)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("LOCAL_RANK", "0")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist

    from hipserve.config import PRESETS, EngineConfig
    from hipserve.engine.llm_engine import LLMEngine, worker_loop
    from hipserve.engine.model_runner import ModelRunner
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import init_tp

    mcfg = PRESETS[a.model]
    if a.layers:
        mcfg = mcfg.replace(num_layers=a.layers)
    ecfg = EngineConfig(model=a.model, load_format="dummy", device="cuda", max_num_seqs=a.batch,
                        max_num_batched_tokens=8192, max_model_len=a.input_len + a.output_len + 16,
                        num_kv_blocks=a.batch * ((a.input_len + a.output_len) // 16 + 4) + 64,
                        tensor_parallel_size=world)
    tp = init_tp(world, backend="gloo", device_type="cuda")
    if rank != 0:
        worker_loop(ModelRunner(ecfg, mcfg, tp), tp)
    else:
        eng = LLMEngine(ecfg, tp=tp, model_cfg=mcfg)
        prompts = [[1] + [(7 * i + j) % 30000 + 10 for j in range(a.input_len - 1)] for i in range(a.batch)]
        sp = SamplingParams(temperature=0.0, max_tokens=a.output_len, ignore_eos=True)
        eng.generate(prompts[:2], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))  # warm-up
        for p in prompts:
            eng.add_request(None, p, sp)
        n_out, t_dec, t0 = 0, 0.0, time.perf_counter()
        while eng.has_unfinished():
            ts = time.perf_counter()
            outs = eng.step()
            new = sum(len(o.new_token_ids) for o in outs)
            if new >= a.batch // 2:  # a decode step of the full batch
                t_dec += time.perf_counter() - ts
                n_out += new
        wall = time.perf_counter() - t0
        print(json.dumps({"tp": world, "shared_gpu": True, "model": a.model, "layers": mcfg.num_layers,
                          "batch": a.batch, "decode_tok_per_s": round(n_out / max(t_dec, 1e-9), 1),
                          "wall_s": round(wall, 2), "graphs": len(eng.runner.graphs),
                          "lookahead": eng.lookahead, "custom_ar": tp.custom_ar is not None,
                          "stats": eng.runner.stats}), flush=True)
        eng.shutdown()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    # a normal interpreter exit (not os._exit): a profiler wrapping this rank
    # writes its trace from an exit handler


if __name__ == "__main__":
    main()
