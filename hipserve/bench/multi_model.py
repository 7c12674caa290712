"""Multi-model benchmark (BASELINE config 5): several engine pods behind the
model-name router and the ingress emulator, requests routed by ``body.model``.

The reference's multi-model setup is one vLLM Deployment per ``models[]`` entry
behind the OpenResty model-name router (vllm-models/helm-chart/templates/
model-gateway.yaml:14-82, values.yaml:1-12). Here every model is one
``python -m hipserve.server`` process (random-init weights, synthetic prompts);
on a one-GPU box they share the GPU, each with a fixed KV pool.

Phases: every model alone (per-model output tok/s and TTFT through the gateway),
then all models loaded at once (aggregate). One JSON line per phase.

    python -m hipserve.bench.multi_model --models llama-3-8b,mixtral-8x7b --out gpurun_out/mm.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

from .local_stack import ROOT, GatewayStack, LoadgenProc, free_port, wait_http


def vocab_of(model: str) -> int:
    from ..config import PRESETS

    cfg = PRESETS.get(model)
    return cfg.vocab_size if cfg else 32000


def start_engine(model: str, port: int, args) -> subprocess.Popen:
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "hipserve.server", "--model", model, "--served-model-name", model,
           "--load-format", "dummy", "--host", "127.0.0.1", "--port", str(port),
           "--num-kv-blocks", str(args.kv_blocks), "--max-num-seqs", str(max(args.concurrency, 8)),
           "--max-model-len", str(args.input_len + args.output_len + 64),
           "--log-level", "WARNING"]
    if args.device:
        cmd += ["--device", args.device]
    return subprocess.Popen(cmd, env=env)


def run_phase(url, models, args, name):
    """One wave set with every model in ``models`` loaded concurrently."""
    gens = {m: LoadgenProc() for m in models}
    results = {}

    def drive(m):
        kw = dict(url=url, model=m, concurrency=args.concurrency, input_len=args.input_len,
                  output_len=args.output_len, vocab=min(vocab_of(m), 100000),
                  temperature=0.8, top_p=0.95)
        for _ in range(args.warmup):
            gens[m].wave(**kw)
        t0 = time.perf_counter()
        res = []
        for _ in range(args.waves):
            res += gens[m].wave(**kw)
        results[m] = (res, time.perf_counter() - t0)

    try:
        th = [threading.Thread(target=drive, args=(m,)) for m in models]
        for t in th:
            t.start()
        for t in th:
            t.join()
    finally:
        for g in gens.values():
            g.close()
    out = {"phase": name, "models": {}}
    total_tok, wall = 0, 0.0
    for m, (res, el) in results.items():
        toks = sum(r["tokens"] for r in res)
        ttfts = sorted(r["ttft"] for r in res if r["ttft"] is not None)
        out["models"][m] = {"output_tok_per_s": round(toks / el, 1), "requests": len(res),
                            "p50_ttft_ms": round(1000 * ttfts[len(ttfts) // 2], 1) if ttfts else None,
                            "elapsed_s": round(el, 2)}
        total_tok += toks
        wall = max(wall, el)
    out["aggregate_output_tok_per_s"] = round(total_tok / wall, 1) if wall else 0.0
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="llama-3-8b,mixtral-8x7b")
    ap.add_argument("--kv-blocks", type=int, default=8192)
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--waves", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    models = [m for m in a.models.split(",") if m]
    engines, procs = {}, []
    stack = None
    lines = []
    try:
        for m in models:  # one at a time: the decode-GEMM tuners must not time each other
            port = free_port()
            p = start_engine(m, port, a)
            procs.append(p)
            wait_http(f"http://127.0.0.1:{port}/health", 1800, p)
            engines[m] = [port]
        stack = GatewayStack(engines).start()
        for m in models:
            lines.append(run_phase(stack.url, [m], a, f"{m} alone"))
            print(json.dumps(lines[-1]), flush=True)
        if len(models) > 1:
            lines.append(run_phase(stack.url, models, a, "all models concurrently"))
            print(json.dumps(lines[-1]), flush=True)
    finally:
        if stack is not None:
            stack.stop()
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    if a.out:
        with open(a.out, "w") as f:
            for ln in lines:
                f.write(json.dumps({**ln, "config": {"concurrency_per_model": a.concurrency,
                                                      "input_len": a.input_len, "output_len": a.output_len,
                                                      "path": "loadgen -> ingress emulator -> router -> engines",
                                                      "data": "synthetic prompts, random-init bf16 weights"}})
                        + "\n")


if __name__ == "__main__":
    main()
