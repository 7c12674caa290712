"""Prometheus metrics for the engine (SURVEY §5 observability; the reference has
none — no scrape annotations in any template)."""
from __future__ import annotations

import time
from collections import deque

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

_LAT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
                7.5, 10.0, 20.0, 40.0, 80.0)


TTFT_WINDOW = 10000


class EngineMetrics:
    def __init__(self, model_name: str = "model"):
        self.registry = CollectorRegistry()
        r = self.registry
        lbl = ["model_name"]
        self.ttft = Histogram("hipserve_time_to_first_token_seconds", "TTFT", lbl, buckets=_LAT_BUCKETS, registry=r)
        self.itl = Histogram("hipserve_time_per_output_token_seconds", "inter-token latency", lbl,
                             buckets=_LAT_BUCKETS, registry=r)
        self.e2e = Histogram("hipserve_e2e_request_latency_seconds", "request latency", lbl,
                             buckets=_LAT_BUCKETS, registry=r)
        self.prompt_tokens = Counter("hipserve_prompt_tokens", "prefilled prompt tokens", lbl, registry=r)
        self.gen_tokens = Counter("hipserve_generation_tokens", "generated tokens", lbl, registry=r)
        self.finished = Counter("hipserve_request_success", "finished requests", lbl + ["finished_reason"],
                                registry=r)
        self.running = Gauge("hipserve_num_requests_running", "running", lbl, registry=r)
        self.waiting = Gauge("hipserve_num_requests_waiting", "waiting", lbl, registry=r)
        self.kv_usage = Gauge("hipserve_kv_cache_usage_perc", "KV block pool usage", lbl, registry=r)
        self.step_time = Histogram("hipserve_engine_step_seconds", "engine step wall time", lbl,
                                   buckets=_LAT_BUCKETS, registry=r)
        self.preemptions = Counter("hipserve_num_preemptions", "preempted sequences", lbl, registry=r)
        self.model_name = model_name
        # bound label children: .labels() is a dict lookup + lock per call, too slow
        # for the per-token path (64+ calls per decode step)
        m = {"model_name": model_name}
        self._ttft, self._itl, self._e2e = self.ttft.labels(**m), self.itl.labels(**m), self.e2e.labels(**m)
        self._prompt, self._gen = self.prompt_tokens.labels(**m), self.gen_tokens.labels(**m)
        self._running, self._waiting = self.running.labels(**m), self.waiting.labels(**m)
        self._kv, self._step = self.kv_usage.labels(**m), self.step_time.labels(**m)
        self._preempt = self.preemptions.labels(**m)
        self._pending_gen = 0
        self.num_steps = 0
        self.total_gen = 0
        self.total_prompt = 0
        # recent TTFTs for in-process summaries; bounded (a serving pod runs for weeks)
        self.ttfts: deque[float] = deque(maxlen=TTFT_WINDOW)

    def _l(self):
        return {"model_name": self.model_name}

    def on_arrival(self, seq):
        pass

    def on_step(self, so, dt, kv_usage, sched):
        self.num_steps += 1
        self._step.observe(dt)
        n_prompt = sum(s.num_tokens for s in so.prefill)
        self.total_prompt += n_prompt
        if n_prompt:
            self._prompt.inc(n_prompt)
        self._running.set(sched.num_running)
        self._waiting.set(sched.num_waiting)
        self._kv.set(kv_usage)
        if so.preempted:
            self._preempt.inc(len(so.preempted))
        self.flush()

    def flush(self):
        if self._pending_gen:
            self._gen.inc(self._pending_gen)
            self._pending_gen = 0

    def on_first_token(self, seq, now):
        t = now - seq.arrival_time
        self.ttfts.append(t)
        self._ttft.observe(t)
        self.total_gen += 1
        self._pending_gen += 1

    def on_token(self, seq, now):
        if seq.last_token_time is not None:
            self._itl.observe(now - seq.last_token_time)
        self.total_gen += 1
        self._pending_gen += 1

    def on_finish(self, seq, now):
        self._e2e.observe(now - seq.arrival_time)
        self.finished.labels(finished_reason=seq.finish_reason or "stop", **self._l()).inc()


def now() -> float:
    return time.monotonic()
