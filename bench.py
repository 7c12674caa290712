#!/usr/bin/env python3
"""hipserve headline benchmark (BASELINE.json): output tok/s + p50 TTFT,
Llama-3-8B bf16 TP=1 per MI355X, synthetic prompts, random-init weights.

One rank per GPU (``torch.distributed.run --nproc-per-node N``); each rank is one
model replica (the k8s ``replicas`` DP of the reference chart,
vllm-models/helm-chart/templates/model-deployments.yaml:10), so per-GPU work is
fixed as N grows (weak scaling). A *step* is one closed-loop wave: every replica
receives ``--concurrency`` requests of ``--input-len`` random prompt tokens at
once and generates exactly ``--output-len`` tokens each (ignore_eos); the wave
includes scheduling, chunked prefill, decode hipGraphs, sampling and — with
``--path gateway`` (default) — the full HTTP path: client -> ingress emulator
(VirtualService rules from the rendered chart) -> model-name router -> engine
OpenAI server with SSE streaming.

Rank 0 prints ONE JSON line; value = total output tokens/s over all ranks
(time = max over ranks of the K timed waves, barrier + device sync on both sides).

Second phase, ``tp_strong`` (BASELINE.json's "Llama-3-70B TP=8 over xGMI" config,
VERDICT r2 next-round item 1): after the headline waves the SAME N ranks serve ONE
Llama-3-70B sharded TP=N (RCCL process group + the in-house IPC collectives), time
boxed (``--tp-budget-s``, 150 s); its tok/s, p50 TTFT and ms/step go under the
``tp_strong`` key of the same JSON line, with the observed process-group backend /
world size and whether the custom all-reduce was active. The driver's 1/2/4/8-GPU
runs therefore also measure the 70B strong-scaling curve. Each phase runs in a
child process per rank (the rank process itself never touches the GPU), so the 8B
engine's HBM (weights + a 0.9-of-HBM KV pool) is returned before the 70B loads.

``--tp T`` (T = the torchrun world size) instead serves ONE model sharded over the
T ranks — BASELINE.json's "Llama-3-70B TP=8 over xGMI" config:
``torchrun --nproc-per-node 8 bench.py --model llama-3-70b --tp 8``. Rank 0 runs
the engine, the HTTP stack and the load generator; ranks 1..T-1 run the TP worker
loop (hipserve/server/cli.py ``_worker``), exactly as a TP pod does.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "output tok/s + p50 TTFT through Istio GW, Llama-3-8B TP=1 and 70B TP=8"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=None)
    ap.add_argument("--path", choices=["engine", "gateway"], default="gateway")
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top-p", type=float, default=0.95)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--quantization", default=None, choices=["q4_k_m", "q8_0", "q4_0", "fp8", "int8"],
                    help="GGUF tier: random-init GGUF-quantised weights (BASELINE config: Llama-3-8B Q4_K_M)")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="paged KV cache element (fp8: e4m3, per-tensor scale 1; not the BASELINE config)")
    ap.add_argument("--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: fp32 on the host with gloo collectives (tests of the DP / TP paths)")
    ap.add_argument("--num-kv-blocks", type=int, default=None, help="KV pool size (default: from HBM)")
    ap.add_argument("--tp-phase", choices=["auto", "on", "off"], default="auto",
                    help="second phase: one --tp-model sharded over all N ranks (auto: on for the default "
                         "GPU headline run)")
    ap.add_argument("--tp-model", default="llama-3-70b")
    ap.add_argument("--tp-steps", type=int, default=2)
    ap.add_argument("--tp-warmup", type=int, default=1)
    ap.add_argument("--tp-budget-s", type=float, default=150.0)
    ap.add_argument("--result-file", default=None, help=argparse.SUPPRESS)  # child -> parent
    ap.add_argument("--deadline", type=float, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--request-rate", type=float, default=None,
                    help="gateway path: open-loop Poisson arrivals at this rate (req/s) for the timed "
                         "region (steps x concurrency requests) instead of closed-loop waves")
    return ap.parse_args()


def _self_launch(args) -> int:
    """``--gpus N`` without torchrun: start the documented multi-rank form as a
    CHILD process (one rank per GPU, 127.0.0.1 rendezvous) and return its exit
    code. Nothing here has touched the GPU yet."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


PEER_FAILED = 125  # exit code recorded for a phase child killed because a peer rank's child failed


def _peer_failures(fail_dir, rank) -> dict:
    """{rank: exit code} of the OTHER ranks whose child of this phase failed."""
    out = {}
    if fail_dir and os.path.isdir(fail_dir):
        for f in os.listdir(fail_dir):
            if f.startswith("rank") and f[4:].isdigit() and int(f[4:]) != rank:
                try:
                    with open(os.path.join(fail_dir, f)) as fh:
                        out[int(f[4:])] = int(fh.read().strip() or 1)
                except (OSError, ValueError):
                    out[int(f[4:])] = 1
    return out


def _run_child(argv, world, rank, local, port, result_file, timeout=None, fail_dir=None):
    """One phase as a child process of this rank (own process group on ``port``);
    returns (exit code, result dict or None). ``timeout``: kill the child's
    whole process group at that many seconds (exit code 124). ``fail_dir`` (one
    directory per phase shared by the node's ranks): a child that fails records its
    exit code there, and every rank kills its own child as soon as a peer's failure
    appears (exit code ``PEER_FAILED``) — the surviving ranks would otherwise sit in a
    collective with the dead one until the phase budget runs out."""
    import signal
    import subprocess

    env = dict(os.environ, HIPSERVE_BENCH_CHILD="1", WORLD_SIZE=str(world), RANK=str(rank),
               LOCAL_RANK=str(local), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in [k for k in env if k.startswith("TORCHELASTIC_")]:
        env.pop(k)  # the child's process group owns its own store (no torchrun agent store)
    cmd = [sys.executable, os.path.abspath(__file__)] + argv + ["--result-file", result_file]
    # the child's stdout goes to our stderr: the ONE JSON line on stdout is ours
    p = subprocess.Popen(cmd, env=env, stdout=sys.stderr, start_new_session=True)
    t_end = time.time() + timeout if timeout else None

    def kill():
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait()

    while True:
        try:
            rc = p.wait(timeout=0.5)
            break
        except subprocess.TimeoutExpired:
            pass
        if _peer_failures(fail_dir, rank):
            kill()
            rc = PEER_FAILED
            break
        if t_end is not None and time.time() > t_end:
            kill()
            rc = 124
            break
    if rc not in (0, 124, PEER_FAILED) and fail_dir:
        with open(os.path.join(fail_dir, f"rank{rank}"), "w") as f:
            f.write(str(rc))
    res = None
    if rank == 0 and os.path.exists(result_file):
        with open(result_file) as f:
            res = json.load(f)
        os.remove(result_file)
    return rc, res


def _strip(argv, names):
    """argv without the given ``--flag value`` / ``--flag=value`` options."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in names:
            skip = True
            continue
        if any(a.startswith(n + "=") for n in names):
            continue
        out.append(a)
    return out


def orchestrate(args) -> int:
    """Per-rank parent: phase 1 (the headline) and the optional TP phase, each as a
    child process; rank 0 prints the merged JSON line. Never touches the GPU."""
    import tempfile

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    tp_phase = args.tp_phase == "on" or (
        args.tp_phase == "auto" and args.device == "cuda" and args.tp == 1 and args.model == "llama-3-8b"
        and not args.quantization and not args.request_rate)
    dist = None
    ports = [_free_port(), _free_port()]
    # one directory shared by the node's ranks (single node: one rendezvous host), where
    # a rank whose phase child fails leaves its exit code for the others (_run_child)
    shared = tempfile.mkdtemp(prefix="hipserve_bench_fail_") if rank == 0 else None
    if world > 1:
        import datetime

        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=3600))
        lst = [(ports, shared)]
        dist.broadcast_object_list(lst, src=0)
        ports, shared = lst[0]
    fail1, fail2 = os.path.join(shared, "phase1"), os.path.join(shared, "phase2")
    if rank == 0:
        os.makedirs(fail1)
        os.makedirs(fail2)
    if dist is not None:
        dist.barrier()
    tmp = tempfile.mkdtemp(prefix="hipserve_bench_")
    argv = sys.argv[1:]
    rc1, res = _run_child(argv, world, rank, local, ports[0], os.path.join(tmp, "phase1.json"), fail_dir=fail1)
    if dist is not None:
        ok = [rc1 == 0] * world
        dist.all_gather_object(ok, rc1 == 0)
        rc1 = 0 if all(ok) else (rc1 or 1)
    if rc1 == 0 and tp_phase:
        t0 = time.time()
        argv2 = _strip(argv, {"--model", "--tp", "--steps", "--warmup", "--out", "--quantization",
                              "--request-rate", "--tp-phase", "--num-kv-blocks"})
        argv2 += ["--model", args.tp_model, "--tp", str(world), "--steps", str(args.tp_steps),
                  "--warmup", str(args.tp_warmup), "--tp-phase", "off",
                  "--deadline", str(t0 + args.tp_budget_s - 15)]
        if args.num_kv_blocks and args.device == "cpu":
            argv2 += ["--num-kv-blocks", str(args.num_kv_blocks)]
        rc2, tp = _run_child(argv2, world, rank, local, ports[1], os.path.join(tmp, "phase2.json"),
                             timeout=args.tp_budget_s, fail_dir=fail2)
        if dist is not None:
            dist.barrier()
        if rank == 0:
            failed = _peer_failures(fail2, -1)  # every rank whose child failed (rank 0's included)
            if rc2 != 0 or tp is None:
                if failed:
                    code = failed[min(failed)]
                    tp = {"model": args.tp_model, "tp": world, "status": f"failed (exit {code})",
                          "failed_ranks": {str(r): c for r, c in sorted(failed.items())}}
                else:
                    tp = {"model": args.tp_model, "tp": world,
                          "status": "timeout" if rc2 == 124 else f"failed (exit {rc2})"}
            tp["phase_wall_s"] = round(time.time() - t0, 1)
            res = dict(res or {}, tp_strong=tp)
    if rank == 0 and res is not None:
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if dist is not None:
        dist.destroy_process_group()
    import shutil

    shutil.rmtree(tmp, ignore_errors=True)
    if rank == 0:
        shutil.rmtree(shared, ignore_errors=True)
    return rc1


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(_self_launch(args))
    if args.gpus != int(world_env or "1"):
        raise SystemExit(f"--gpus {args.gpus} does not match the launched world size {world_env or 1}: "
                         "run one rank per GPU (torch.distributed.run --nproc-per-node N bench.py --gpus N)")
    if not os.environ.get("HIPSERVE_BENCH_CHILD"):
        sys.exit(orchestrate(args))
    run_phase(args)


def run_phase(args):
    """One benchmark phase on this rank (a child process of ``orchestrate``)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    if args.tp > 1 and args.tp != world:
        raise SystemExit(f"--tp {args.tp} needs a torchrun world size of {args.tp} (got {world})")
    tp_mode = args.tp > 1
    leader = not tp_mode or rank == 0
    stack = lg = None
    if args.path == "gateway" and leader:
        # client-side processes start BEFORE this process touches the GPU
        from hipserve.bench.local_stack import GatewayStack, LoadgenProc, free_port, wait_http

        eport = free_port()
        stack = GatewayStack({args.model: [eport]}).start()
        lg = LoadgenProc()

    from hipserve.config import EngineConfig, default_batched_tokens
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup, init_tp

    cuda = args.device == "cuda"
    tpg = None
    if tp_mode:
        tpg = init_tp(world, device_type=args.device)  # RCCL group + shm step ring + custom all-reduce
    elif world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if cuda:
            torch.cuda.set_device(local)
        dist.init_process_group("nccl" if cuda else "gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", local) if cuda else torch.device("cpu")
    cfg = EngineConfig(model=args.model, device=args.device, max_num_seqs=max(args.concurrency, 1),
                       dtype="bfloat16" if cuda else "float32", num_kv_blocks=args.num_kv_blocks,
                       kv_cache_dtype=args.kv_cache_dtype,
                       tensor_parallel_size=args.tp,
                       max_num_batched_tokens=args.max_num_batched_tokens or default_batched_tokens(
                           args.model, quantization=args.quantization),
                       max_model_len=args.input_len + args.output_len + 64,
                       enforce_eager=args.enforce_eager, seed=0 if tp_mode else rank,
                       load_format="dummy" if args.quantization else "auto",
                       extra={"quantization": args.quantization} if args.quantization else {})
    if tp_mode and not leader:
        from hipserve.engine.llm_engine import prepare_model, worker_loop
        from hipserve.engine.model_runner import ModelRunner

        wcfg, mcfg, _ = prepare_model(cfg, tpg)  # GGUF: the file's own hyper-parameters
        worker_loop(ModelRunner(wcfg, mcfg, tpg), tpg)
        dist.barrier()
        dist.destroy_process_group()
        return
    t0 = time.time()
    engine = LLMEngine(cfg, tp=tpg if tp_mode else TPGroup(0, 1, None, dev))
    init_s = time.time() - t0
    dp = world > 1 and not tp_mode  # independent replicas: cross-rank barriers and sums
    rng = np.random.default_rng(1234 + rank)
    V = engine.model_cfg.vocab_size

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    def barrier():
        sync()
        if dp:  # TP workers sit in their step loop: the engine's own collectives sync them
            dist.barrier()
        sync()

    if args.path == "gateway":
        import asyncio
        import threading

        from hipserve.server.api_server import serve

        def run_server():
            asyncio.run(serve(engine, "127.0.0.1", eport, args.model))

        threading.Thread(target=run_server, name="http", daemon=True).start()
        wait_http(f"http://127.0.0.1:{eport}/health", 120)

        def wave():
            res = lg.wave(url=stack.url, model=args.model, concurrency=args.concurrency,
                          input_len=args.input_len, output_len=args.output_len,
                          vocab=min(V, 100000), temperature=args.temperature, top_p=args.top_p)
            return sum(r["tokens"] for r in res), [r["ttft"] for r in res]
    else:
        def wave():
            prompts = [rng.integers(10, min(V, 100000), size=args.input_len).tolist()
                       for _ in range(args.concurrency)]
            sp = SamplingParams(temperature=args.temperature, top_p=args.top_p,
                                max_tokens=args.output_len, ignore_eos=True)
            t_start = time.monotonic()
            seqs = [engine.add_request(None, p, sp, arrival_time=t_start) for p in prompts]
            ntok = 0
            while engine.has_unfinished():
                for o in engine.step():
                    ntok += len(o.new_token_ids)
            return ntok, [s.first_token_time - s.arrival_time for s in seqs]

    steps = args.steps
    t_w = time.perf_counter()
    for _ in range(args.warmup):
        wave()
    if args.deadline and args.warmup:  # time-boxed phase: as many timed waves as fit (>= 1)
        per = (time.perf_counter() - t_w) / args.warmup
        steps = max(1, min(steps, int((args.deadline - time.time()) / max(per, 1e-3))))
    barrier()
    t0 = time.perf_counter()
    tok_total, ttfts, ol_summary = 0, [], None
    if args.request_rate and args.path == "gateway":
        res, _ = lg.open_loop(url=stack.url, model=args.model, rate=args.request_rate,
                              num_requests=args.steps * args.concurrency, input_len=args.input_len,
                              output_len=args.output_len, vocab=min(V, 100000), temperature=args.temperature,
                              top_p=args.top_p)
        tok_total, ttfts = sum(r["tokens"] for r in res), [r["ttft"] for r in res]
        from hipserve.bench.loadgen import summarize

        ol_summary = summarize(res, time.perf_counter() - t0)
    else:
        for _ in range(steps):
            n, tt = wave()
            tok_total += n
            ttfts += tt
    barrier()
    elapsed = time.perf_counter() - t0

    stats = torch.tensor([elapsed, float(tok_total)], dtype=torch.float64, device=dev)
    p50 = torch.tensor([statistics.median(ttfts)], dtype=torch.float64, device=dev)
    if dp:
        el = stats[:1].clone()
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        tk = stats[1:].clone()
        dist.all_reduce(tk, op=dist.ReduceOp.SUM)
        stats = torch.cat([el, tk])
        allp = [torch.zeros_like(p50) for _ in range(world)]
        dist.all_gather(allp, p50)
        p50 = torch.stack(allp).median()
    elapsed, tok_total = float(stats[0]), float(stats[1])
    value = tok_total / elapsed
    out = {
        "metric": "output tok/s through gateway (p50 TTFT reported)" if args.path == "gateway" else "output tok/s (engine, no HTTP)",
        "baseline_metric": BASELINE_METRIC,
        "value": round(value, 2),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if tp_mode else "weak",
        "vs_baseline": None,
        "dtype": ("bf16" if cuda else "fp32") if not args.quantization else (
            "bf16 activations, FP8 e4m3 weights (per-channel scales)" if args.quantization == "fp8"
            else "bf16 activations, INT8 weight-only (per-channel scales)" if args.quantization == "int8"
            else f"bf16 activations, GGUF {args.quantization.upper()} weights")
        + ("; fp8 e4m3 KV cache" if args.kv_cache_dtype == "fp8" else ""),
        "data": "synthetic prompts (random token ids), random-init weights",
        "p50_ttft_ms": round(1000 * float(p50), 2),
        "load": f"open-loop Poisson {args.request_rate} req/s" if args.request_rate else "closed-loop waves",
        "path": args.path,
        "config": {
            "model": args.model + ((" FP8" if args.quantization == "fp8" else " INT8" if args.quantization == "int8"
                                    else f" GGUF {args.quantization.upper()}")
                                   if args.quantization else ""),
            "tp": args.tp,
            "global_batch": args.concurrency * (world // args.tp),
            "seq_len": args.input_len + args.output_len,
            "input_len": args.input_len,
            "output_len": args.output_len,
            "concurrency_per_gpu": args.concurrency,
            "parallelism": f"tp{args.tp}" if tp_mode else (f"dp{world}" if world > 1 else "tp1"),
            "sampling": {"temperature": args.temperature, "top_p": args.top_p},
            "prefill_tokens_per_step": cfg.max_num_batched_tokens,
            **({"kv_cache_dtype": "fp8_e4m3"} if args.kv_cache_dtype == "fp8" else {}),
        },
        "engine_init_s": round(init_s, 1),
        "init_breakdown_s": getattr(engine.runner, "init_times", {}),
        "init_breakdown_s_per_rank": getattr(engine.runner, "init_times_ranks", None),
        "single_weight_layout": getattr(engine.runner, "single_layout", None),
        "packed_prefill_timing": getattr(engine.runner, "packed_prefill_report", None),
        "kv_blocks": engine.runner.num_blocks,
    }
    if args.quantization:  # resident bytes beyond the quantised weights, GGUF prefill path per shape
        out["quant_shadow_gb"] = round(getattr(engine.runner, "quant_shadow_bytes", 0) / 2**30, 2)
        out["gguf_prefill_timing"] = getattr(engine.runner, "qprefill_report", None)
    if engine.tracer.times:  # HIPSERVE_PROFILE=timing: host time per engine-step phase
        out["host_phase_ms"] = {k: {"calls": n, "avg": round(1000 * t / max(n, 1), 4)}
                                for k, (n, t) in engine.tracer.times.items()}
    if getattr(engine.runner, "moe_prefill_report", None) is not None:
        out["moe_prefill_timing"] = engine.runner.moe_prefill_report
    if ol_summary:  # open loop: TTFT tail and inter-token latency of every request
        out["open_loop"] = {"rate_req_s": args.request_rate, "requests": ol_summary["requests"],
                            **{k: round(ol_summary[k], 2) for k in ("p50_ttft_ms", "p90_ttft_ms", "p50_itl_ms",
                                                                    "p90_itl_ms") if ol_summary[k] is not None}}
    if tp_mode or args.deadline:
        out["tp_info"] = ({"pg_backend": tpg.backend, "pg_world_size": dist.get_world_size(),
                           "rccl": tpg.backend == "nccl", "custom_allreduce": tpg.custom_ar is not None,
                           "rccl_min_rows": tpg.rccl_min_rows, "collective_calibration": tpg.collective_report}
                          if tp_mode else {"pg_backend": None, "pg_world_size": 1, "rccl": False,
                                           "custom_allreduce": False})
        if args.deadline:  # the tp_strong record of orchestrate()
            out = {"model": args.model, "tp": args.tp, "status": "ok", "tok_s": out["value"],
                   "p50_ttft_ms": out["p50_ttft_ms"], "ms_per_step": out["ms_per_step"], "steps": steps,
                   "warmup": args.warmup, "global_batch": args.concurrency,
                   "input_len": args.input_len, "output_len": args.output_len,
                   "engine_init_s": out["engine_init_s"], "init_breakdown_s": out["init_breakdown_s"],
                   "init_breakdown_s_per_rank": out["init_breakdown_s_per_rank"],
                   "kv_blocks": out["kv_blocks"], **out["tp_info"]}
    if lg is not None:
        lg.close()
        stack.stop()
    if tp_mode:
        engine.shutdown()  # releases the workers from worker_loop
    if rank == 0:
        line = json.dumps(out)
        if args.result_file:
            with open(args.result_file, "w") as f:
                f.write(line + "\n")
        else:
            print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
            with open(os.path.splitext(args.out)[0] + "_gemm_tune.jsonl", "w") as f:
                for r in engine.runner.gemm_report + getattr(engine.runner, "gguf_split_report", []):
                    f.write(json.dumps(r) + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
