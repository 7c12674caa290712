"""Prefill (large-M) GEMM solution selection.

Prefill projections are plain library GEMMs (M = the step's token budget, 8192 by
default): compute-bound, where MFMA tile shape, K-unroll and workgroup mapping decide
the throughput. The hipBLASLt heuristic's first pick is measurably off on gfx950 for
these shapes (Llama-3-8B gate|up at M=8192: 1.23 ms heuristic vs 0.91 ms for the best
rocBLAS/hipBLASLt solution, tools/tune_prefill_gemm.py), so the engine times the
candidate solutions of each exact (M, N, K) once at startup with PyTorch TunableOp and
keeps TunableOp enabled (tuning off) so every later ``F.linear`` of a tuned shape runs
the winner. The decode path is unaffected: its GEMMs are the hand-written decode
kernels (ops/gemm.py) baked into hipGraphs, and TunableOp only looks shapes up.

Results persist in a CSV keyed by the library versions (TunableOp's validators), so a
restart of the same image reads them instead of re-tuning; a version mismatch makes
TunableOp reject the file and the shapes are re-tuned.

Reference parity: vLLM (the reference's engine, ``vllm/vllm-openai:v0.11.0`` in
``vllm-models/helm-chart/values.yaml``) ships per-device GEMM/MoE tuning tables; this
is the MI355X equivalent for the library GEMMs.
"""
from __future__ import annotations

import logging
import os
import time

import torch
import torch.nn.functional as F

log = logging.getLogger("hipserve.prefill_tune")

TUNE_MS = 10          # per-solution tuning time budget (TunableOp max tuning duration)
TUNE_ITERS = 20
DEFAULT_FILE = os.environ.get(
    "HIPSERVE_TUNABLEOP_FILE",
    os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "tunableop_gfx950.csv"))


def model_prefill_shapes(mc, tp: int = 1) -> list[tuple[int, int]]:
    """(N, K) of a dense decoder layer's projections under TP (column-parallel qkv and
    gate|up, row-parallel o and down), for tools that have no model instance."""
    H, I = mc.hidden_size, mc.intermediate_size
    q = mc.num_heads * mc.head_dim // tp
    kv = max(mc.num_kv_heads // tp, 1) * mc.head_dim
    return sorted({(q + 2 * kv, H), (H, q), (2 * I // tp, H), (H, I // tp)})


def _sig(M: int, N: int, K: int) -> str:
    # F.linear(x[M,K], w[N,K]) is a TN GEMM with m=N, n=M, k=K in TunableOp's naming
    return f"tn_{N}_{M}_{K}_ld_{K}_{K}_{N}"


def _results() -> dict[str, tuple[str, float]]:
    out = {}
    for r in torch.cuda.tunable.get_results():
        op, param, sol, t = r
        if op.startswith("GemmTunableOp_BFloat16"):
            out[param] = (sol, float(t))
    return out


def _write(filename: str) -> None:
    """TunableOp's own file format: validator lines, then op,params,solution,ms."""
    os.makedirs(os.path.dirname(os.path.abspath(filename)), exist_ok=True)
    lines = [f"Validator,{k},{v}" for k, v in torch.cuda.tunable.get_validators()]
    lines += [f"{op},{param},{sol},{t}" for op, param, sol, t in torch.cuda.tunable.get_results()]
    tmp = filename + f".tmp{os.getpid()}"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, filename)


def tune(shapes, ms, device, filename: str | None = DEFAULT_FILE,
         duration_ms: float = TUNE_MS) -> list[dict]:
    """Tune bf16 ``F.linear`` for every (N, K) in ``shapes`` at every M in ``ms``;
    leaves TunableOp enabled with tuning off. Returns one record per shape."""
    T = torch.cuda.tunable
    T.enable(True)
    T.record_untuned_enable(False)
    if filename and os.path.exists(filename):
        if not T.read_file(filename):
            log.warning("tuning table %s rejected (library versions differ); re-tuning", filename)
    have = _results()
    todo = [(M, N, K) for M in ms for N, K in shapes if _sig(M, N, K) not in have]
    report = []
    if todo:
        T.set_max_tuning_duration(max(int(duration_ms), 1))
        T.set_max_tuning_iterations(TUNE_ITERS)
        T.tuning_enable(True)
        try:
            with torch.inference_mode():
                for M, N, K in todo:
                    t0 = time.time()
                    x = torch.randn(M, K, device=device, dtype=torch.bfloat16)
                    w = torch.randn(N, K, device=device, dtype=torch.bfloat16) * 0.02
                    F.linear(x, w)
                    torch.cuda.synchronize(device)
                    del x, w
                    report.append({"M": M, "N": N, "K": K, "tune_s": round(time.time() - t0, 2)})
        finally:
            T.tuning_enable(False)
        if filename:
            try:
                _write(filename)
            except OSError as e:  # read-only install: the table just is not persisted
                log.warning("could not write tuning table %s: %s", filename, e)
    have = _results()
    out = []
    for M in ms:
        for N, K in shapes:
            sol, t = have.get(_sig(M, N, K), ("Default", float("nan")))
            rec = {"M": M, "N": N, "K": K, "solution": sol, "ms": round(t, 4),
                   "PF": round(2 * M * N * K / t / 1e12, 3) if t == t and t > 0 else None}
            rec.update(next((r for r in report if (r["M"], r["N"], r["K"]) == (M, N, K)), {}))
            out.append(rec)
    return out


def disable() -> None:
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.enable(False)
