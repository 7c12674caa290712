"""Engine tracing and profiling hooks (SURVEY §5 "Tracing / profiling").

The reference passes no profiler flag to its engines
(vllm-models/helm-chart/templates/model-deployments.yaml:26-39,
ramalama-models/helm-chart/templates/model-deployments.yaml:27-35) and has no
tracing config at all. Here every engine step can be made visible three ways,
chosen once from the environment at engine construction (zero cost when off):

``HIPSERVE_PROFILE=ranges``
    roctx ranges around the engine phases (schedule / prepare / execute /
    launch / wait / process). ``rocprofv3 --marker-trace --kernel-trace`` then
    attributes every kernel to its engine phase and step.
``HIPSERVE_PROFILE=torch:<dir>[:<first>-<last>]``
    ``torch.profiler`` (CPU + HIP activities) over engine steps first..last
    (default 20-40), exported as a Chrome trace ``<dir>/hipserve_steps_<pid>.json``.
``HIPSERVE_PROFILE=timing``
    host wall time per engine phase accumulated in ``Tracer.times`` (name ->
    [calls, seconds]); ``tools/decode_gap.py`` uses it to split a decode step into
    host phases vs device time.
``HIPSERVE_STEP_LOG=<path>``
    one JSON line per engine step: step index, kind (prefill / mixed / decode),
    scheduled tokens and sequences, wall milliseconds, KV-pool usage, queue depths.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time

_NULL = contextlib.nullcontext()


def _roctx():
    """(push, pop) for roctx ranges, or None. torch's nvtx binding is roctx on ROCm."""
    try:
        import torch

        nv = torch.cuda.nvtx
        nv.range_push("hipserve-probe")
        nv.range_pop()
        return nv.range_push, nv.range_pop
    except Exception:
        return None


class _Range:
    __slots__ = ("push", "pop", "name")

    def __init__(self, push, pop, name):
        self.push, self.pop, self.name = push, pop, name

    def __enter__(self):
        self.push(self.name)
        return self

    def __exit__(self, *exc):
        self.pop()
        return False


class _Timed:
    __slots__ = ("acc", "name", "t0")

    def __init__(self, acc, name):
        self.acc, self.name = acc, name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        a = self.acc.setdefault(self.name, [0, 0.0])
        a[0] += 1
        a[1] += time.perf_counter() - self.t0
        return False


class Tracer:
    """Per-engine tracer. ``phase(name)`` is a context manager; ``step_done``
    is called once per engine step with its scheduling summary."""

    def __init__(self, mode: str = "", step_log: str | None = None):
        self.mode = mode or ""
        self.ranges = None
        self.profiler = None
        self.prof_dir = None
        self.prof_window = (20, 40)
        self.step = 0
        self._log = None
        self._lock = threading.Lock()
        self.times: dict | None = {} if self.mode == "timing" else None
        if self.mode == "ranges":
            self.ranges = _roctx()
        elif self.mode.startswith("torch:"):
            parts = self.mode.split(":")
            self.prof_dir = parts[1] or "."
            if len(parts) > 2 and "-" in parts[2]:
                a, b = parts[2].split("-", 1)
                self.prof_window = (int(a), int(b))
        if step_log:
            d = os.path.dirname(os.path.abspath(step_log))
            os.makedirs(d, exist_ok=True)
            self._log = open(step_log, "a", buffering=1)

    @classmethod
    def from_env(cls) -> "Tracer":
        return cls(os.environ.get("HIPSERVE_PROFILE", ""), os.environ.get("HIPSERVE_STEP_LOG") or None)

    @property
    def enabled(self) -> bool:
        return bool(self.ranges or self.prof_dir or self._log)

    def phase(self, name: str):
        if self.times is not None:
            return _Timed(self.times, name)
        if self.ranges is None:
            return _NULL
        return _Range(self.ranges[0], self.ranges[1], name)

    # ------------------------------------------------------------ per step
    def step_begin(self):
        if self.prof_dir is None:
            return
        a, b = self.prof_window
        if self.step == a and self.profiler is None:
            import torch.profiler as tp

            acts = [tp.ProfilerActivity.CPU]
            try:
                import torch

                if torch.cuda.is_available():
                    acts.append(tp.ProfilerActivity.CUDA)
            except Exception:
                pass
            self.profiler = tp.profile(activities=acts, record_shapes=False, with_stack=False)
            self.profiler.__enter__()

    def step_done(self, kind: str, num_tokens: int, num_seqs: int, wall_s: float,
                  kv_usage: float = 0.0, running: int = 0, waiting: int = 0):
        if self._log is not None:
            rec = {"step": self.step, "t": round(time.time(), 6), "kind": kind, "tokens": num_tokens,
                   "seqs": num_seqs, "ms": round(wall_s * 1000.0, 3), "kv_usage": round(kv_usage, 4),
                   "running": running, "waiting": waiting}
            with self._lock:
                self._log.write(json.dumps(rec) + "\n")
        if self.profiler is not None and self.step >= self.prof_window[1]:
            self.close_profiler()
        self.step += 1

    def close_profiler(self):
        if self.profiler is None:
            return None
        p, self.profiler = self.profiler, None
        p.__exit__(None, None, None)
        os.makedirs(self.prof_dir, exist_ok=True)
        path = os.path.join(self.prof_dir, f"hipserve_steps_{os.getpid()}.json")
        p.export_chrome_trace(path)
        self.prof_dir = None  # one window per process
        return path

    def close(self):
        self.close_profiler()
        if self._log is not None:
            self._log.close()
            self._log = None


def step_kind(num_prefill_tokens: int, num_decode: int) -> str:
    if num_prefill_tokens and num_decode:
        return "mixed"
    return "prefill" if num_prefill_tokens else "decode"
