"""Engine command line.

Accepts the exact flags the reference charts pass to their engines:

* HF tier (vllm-models/helm-chart/templates/model-deployments.yaml:26-39):
  ``--model <hf id> --served-model-name <name> --host 0.0.0.0 --port 8080
  --gpu-memory-utilization 0.90 --tensor-parallel-size N --trust-remote-code``
* GGUF tier (ramalama-models/helm-chart/templates/model-deployments.yaml:26-35):
  ``llama-server --host 0.0.0.0 --port 8080 --model <path.gguf> --alias <name>``
  (``-m``, ``-c/--ctx-size``, ``-ngl`` are accepted too).

With ``--tensor-parallel-size N > 1`` this process becomes TP rank 0 (scheduler
+ HTTP) and spawns N-1 worker processes, one per GPU, that join an RCCL group.
"""
from __future__ import annotations

import argparse
import asyncio
import multiprocessing as mp
import os
import socket
import sys

from ..config import EngineConfig, default_batched_tokens


def build_parser(prog="hipserve") -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog=prog, description="hipserve OpenAI-compatible engine (MI355X)")
    ap.add_argument("--model", "-m", required=True, help="preset name, HF id/dir, or .gguf file")
    ap.add_argument("--served-model-name", "--alias", "-a", dest="served_model_name", default=None)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--tensor-parallel-size", "-tp", type=int, default=1)
    ap.add_argument("--trust-remote-code", action="store_true")
    ap.add_argument("--max-model-len", "--ctx-size", "-c", dest="max_model_len", type=int, default=None)
    ap.add_argument("--load-format", default="auto", choices=["auto", "dummy", "safetensors", "gguf"])
    ap.add_argument("--quantization", default=None, choices=["q4_k_m", "q8_0", "q4_0", "fp8", "int8"],
                    help="with --load-format dummy: random-init GGUF-quantised weights (GGUF tier benchmarks)")
    ap.add_argument("--dtype", default="bfloat16")
    ap.add_argument("--device", default=None, help="cuda (default when a GPU is visible) or cpu")
    ap.add_argument("--block-size", type=int, default=16)
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "bf16", "bfloat16", "fp8", "fp8_e4m3"],
                    help="paged KV cache element: auto (bf16) or fp8 (e4m3, per-tensor scale 1: 2x the KV blocks)")
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=None,
                    help="prefill token budget per step (default 8192; 16384 for GGUF weights)")
    ap.add_argument("--num-kv-blocks", type=int, default=None)
    ap.add_argument("--enable-prefix-caching", action=argparse.BooleanOptionalAction, default=True)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--n-gpu-layers", "-ngl", dest="ngl", type=int, default=None,
                    help="accepted for llama-server compatibility (all layers always run on the GPU)")
    ap.add_argument("--log-level", default=os.environ.get("HIPSERVE_LOG_LEVEL", "INFO"))
    ap.add_argument("--log-format", default=None, choices=["text", "json"],
                    help="text (default) or one JSON object per line (HIPSERVE_LOG_FORMAT)")
    return ap


def config_from_args(a) -> EngineConfig:
    device = a.device
    if device is None:
        import torch

        device = "cuda" if torch.cuda.is_available() else "cpu"
    dtype = a.dtype
    if device == "cpu" and dtype in ("auto",):
        dtype = "float32"
    return EngineConfig(
        model=a.model, served_model_name=a.served_model_name, tokenizer=a.tokenizer,
        load_format=a.load_format, dtype=dtype, device=device,
        tensor_parallel_size=a.tensor_parallel_size, gpu_memory_utilization=a.gpu_memory_utilization,
        max_model_len=a.max_model_len, block_size=a.block_size, max_num_seqs=a.max_num_seqs,
        max_num_batched_tokens=a.max_num_batched_tokens or default_batched_tokens(a.model, a.load_format,
                                                                                   a.quantization),
        num_kv_blocks=a.num_kv_blocks, kv_cache_dtype=getattr(a, "kv_cache_dtype", "auto"),
        enable_prefix_caching=a.enable_prefix_caching, enforce_eager=a.enforce_eager, seed=a.seed,
        trust_remote_code=a.trust_remote_code, host=a.host, port=a.port,
        extra={"quantization": a.quantization} if a.quantization else {})


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(cfg: EngineConfig, rank: int, world: int, port: int):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ..engine.llm_engine import prepare_model, worker_loop
    from ..engine.model_runner import ModelRunner
    from ..parallel.comm import init_tp
    from ..utils.faults import ParentWatch

    ParentWatch().start()  # rank 0 gone -> exit, never hold the GPU as an orphan
    tp = init_tp(world, device_type="cuda" if cfg.device == "cuda" else "cpu")
    cfg, mcfg, _ = prepare_model(cfg, tp)  # waits for rank 0's first-start download
    runner = ModelRunner(cfg, mcfg, tp)
    worker_loop(runner, tp)


def main(argv=None, prog="hipserve"):
    a = build_parser(prog).parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging(a.log_level, a.log_format)
    cfg = config_from_args(a)
    world = cfg.tensor_parallel_size
    procs = []
    if world > 1 and "RANK" not in os.environ:
        port = _free_port()
        ctx = mp.get_context("spawn")
        for r in range(1, world):
            p = ctx.Process(target=_worker, args=(cfg, r, world, port), daemon=True)
            p.start()
            procs.append(p)
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE=str(world),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from ..engine.llm_engine import LLMEngine
    from ..parallel.comm import init_tp
    from .api_server import serve

    tp = init_tp(world, device_type="cuda" if cfg.device == "cuda" else "cpu")
    engine = LLMEngine(cfg, tp=tp)
    names = (cfg.model,) if cfg.served_model_name else ()
    try:
        asyncio.run(serve(engine, cfg.host, cfg.port, cfg.model_name, extra_names=names,
                          worker_procs=procs))
    finally:
        engine.shutdown()
        for p in procs:
            p.join(timeout=10)


if __name__ == "__main__":
    sys.exit(main())
