"""Prometheus metrics for the engine (SURVEY §5 observability; the reference has
none — no scrape annotations in any template)."""
from __future__ import annotations

import time

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram

_LAT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
                7.5, 10.0, 20.0, 40.0, 80.0)


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
        self.num_steps = 0
        self.total_gen = 0
        self.total_prompt = 0
        self.ttfts: list[float] = []

    def _l(self):
        return {"model_name": self.model_name}

    def on_arrival(self, seq):
        pass

    def on_step(self, so, dt, kv_usage, sched):
        self.num_steps += 1
        self.step_time.labels(**self._l()).observe(dt)
        n_prompt = sum(s.num_tokens for s in so.prefill)
        self.total_prompt += n_prompt
        self.prompt_tokens.labels(**self._l()).inc(n_prompt)
        self.running.labels(**self._l()).set(sched.num_running)
        self.waiting.labels(**self._l()).set(sched.num_waiting)
        self.kv_usage.labels(**self._l()).set(kv_usage)
        if so.preempted:
            self.preemptions.labels(**self._l()).inc(len(so.preempted))

    def on_first_token(self, seq, now):
        t = now - seq.arrival_time
        self.ttfts.append(t)
        self.ttft.labels(**self._l()).observe(t)
        self.total_gen += 1
        self.gen_tokens.labels(**self._l()).inc()

    def on_token(self, seq, now):
        if seq.last_token_time is not None:
            self.itl.labels(**self._l()).observe(now - seq.last_token_time)
        self.total_gen += 1
        self.gen_tokens.labels(**self._l()).inc()

    def on_finish(self, seq, now):
        self.e2e.labels(**self._l()).observe(now - seq.arrival_time)
        self.finished.labels(finished_reason=seq.finish_reason or "stop", **self._l()).inc()


def now() -> float:
    return time.monotonic()
