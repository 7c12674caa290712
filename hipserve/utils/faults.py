"""Failure detection and test-only fault injection (SURVEY §5 "Failure detection /
recovery / fault injection").

The reference's only failure handling is Kubernetes probes (readiness/liveness
on ``/health``, vllm-models/helm-chart/templates/model-deployments.yaml:48-63;
none at all for the GGUF engines, ramalama-models/helm-chart/templates/
model-deployments.yaml:19-40) plus the Deployment controller restarting dead
pods. The engine itself must therefore turn every internal failure into either
a failing probe or a process exit. Detection pieces:

* ``WorkerMonitor`` (rank 0): polls the TP worker processes it spawned; when one
  exits, the engine is marked dead (``/health`` -> 503) and the pod process is
  terminated after a short grace period, so the pod restarts instead of hanging
  in a collective that can never complete.
* ``ParentWatch`` (TP workers): exits the worker when rank 0 disappears, so no
  orphan keeps holding a GPU.
* the engine-loop heartbeat watchdog lives in ``server/api_server.py``
  (``/health`` -> 503 "engine stalled" after ``HIPSERVE_STALL_TIMEOUT`` s).

Injection (tests and chaos drills only), ``HIPSERVE_FAULT`` = comma-separated
``[role:]kind@step[:arg]`` with role ``rank0`` | ``worker`` | ``any`` (default):

  ``raise@N``        the engine step N raises ``InjectedFault``
  ``stall@N:SECS``   step N sleeps SECS seconds (heartbeat stalls)
  ``exit@N[:CODE]``  the process exits with CODE (default 13) at step N
  ``init@0[:CODE]``  model-runner construction raises ``InjectedFault`` (or exits with
                     CODE): a rank that dies while its peers build their engines

Role ``rankK`` matches TP rank K of a sharded (TP > 1) engine only, e.g.
``rank3:init@0`` fails rank 3 of the 70B TP=8 phase of bench.py but none of the
unsharded DP replicas before it.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from dataclasses import dataclass

log = logging.getLogger("hipserve.faults")


class InjectedFault(RuntimeError):
    pass


@dataclass(frozen=True)
class FaultSpec:
    role: str
    kind: str
    step: int
    arg: float | None = None


def parse_faults(spec: str) -> list[FaultSpec]:
    out = []
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        role = "any"
        if ":" in item.split("@", 1)[0]:
            role, item = item.split(":", 1)
        if "@" not in item:
            raise ValueError(f"bad fault spec {item!r}: expected kind@step[:arg]")
        kind, rest = item.split("@", 1)
        arg = None
        if ":" in rest:
            rest, a = rest.split(":", 1)
            arg = float(a)
        if kind not in ("raise", "stall", "exit", "init"):
            raise ValueError(f"unknown fault kind {kind!r}")
        if role not in ("any", "rank0", "worker") and not (role.startswith("rank") and role[4:].isdigit()):
            raise ValueError(f"unknown fault role {role!r}")
        out.append(FaultSpec(role, kind, int(rest), arg))
    return out


class FaultInjector:
    """Fires the configured faults when ``on_step(role, step)`` reaches them."""

    def __init__(self, specs: list[FaultSpec] | None = None):
        self.specs = list(specs or [])
        self.fired: list[FaultSpec] = []

    @classmethod
    def from_env(cls) -> "FaultInjector":
        return cls(parse_faults(os.environ.get("HIPSERVE_FAULT", "")))

    @property
    def active(self) -> bool:
        return bool(self.specs)

    def on_init(self, tp_rank: int, tp_world: int):
        """Model-runner construction on TP rank ``tp_rank`` of ``tp_world``."""
        for f in self.specs:
            if f.kind != "init" or f in self.fired:
                continue
            role = f"rank{tp_rank}" if tp_world > 1 else None
            if f.role not in ("any", role, "rank0" if tp_rank == 0 else "worker"):
                continue
            self.fired.append(f)
            log.warning("fault injection: init on TP rank %d of %d", tp_rank, tp_world)
            if f.arg is not None:
                os._exit(int(f.arg))
            raise InjectedFault(f"injected fault in engine construction (TP rank {tp_rank} of {tp_world})")

    def on_step(self, role: str, step: int):
        if not self.specs:
            return
        for f in self.specs:
            if (f.kind == "init" or f.step != step or (f.role != "any" and f.role != role)
                    or f in self.fired):
                continue
            self.fired.append(f)
            log.warning("fault injection: %s@%d on %s", f.kind, f.step, role)
            if f.kind == "raise":
                raise InjectedFault(f"injected fault at step {step} ({role})")
            if f.kind == "stall":
                time.sleep(f.arg if f.arg is not None else 1.0)
            elif f.kind == "exit":
                os._exit(int(f.arg) if f.arg is not None else 13)


class WorkerMonitor(threading.Thread):
    """Rank-0 thread: ``on_death(proc)`` once when any watched process exits
    while the monitor is armed; then, if ``exit_after`` is not None, terminate
    this process with ``exit_code`` after that grace period (k8s restarts the pod)."""

    def __init__(self, procs, on_death=None, interval: float = 0.5, exit_after: float | None = 5.0,
                 exit_code: int = 70):
        super().__init__(name="hipserve-worker-monitor", daemon=True)
        self.procs = list(procs)
        self.on_death = on_death
        self.interval = interval
        self.exit_after = exit_after
        self.exit_code = exit_code
        self.dead = None
        self._halt = threading.Event()

    def stop(self):
        self._halt.set()

    def run(self):
        while not self._halt.wait(self.interval):
            for p in self.procs:
                code = p.exitcode if hasattr(p, "exitcode") else p.poll()
                if code is None:
                    continue
                if self._halt.is_set():
                    return
                self.dead = p
                log.error("TP worker %s exited with code %s: engine is dead", getattr(p, "pid", "?"), code)
                if self.on_death is not None:
                    try:
                        self.on_death(p)
                    except Exception:  # never let the monitor die silently
                        log.exception("on_death callback failed")
                if self.exit_after is not None:
                    time.sleep(self.exit_after)
                    os._exit(self.exit_code)
                return


class ParentWatch(threading.Thread):
    """Worker-side: exit when the parent (rank 0) process is gone."""

    def __init__(self, interval: float = 1.0, exit_code: int = 71):
        super().__init__(name="hipserve-parent-watch", daemon=True)
        self.ppid = os.getppid()
        self.interval = interval
        self.exit_code = exit_code

    def run(self):
        while True:
            time.sleep(self.interval)
            if os.getppid() != self.ppid:
                log.error("rank 0 (pid %d) is gone: TP worker exiting", self.ppid)
                os._exit(self.exit_code)


def stall_timeout() -> float:
    """Seconds without an engine-loop heartbeat (while work is pending) after
    which ``/health`` reports 503."""
    return float(os.environ.get("HIPSERVE_STALL_TIMEOUT", "120"))
