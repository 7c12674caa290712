"""Failure detection, fault injection and step tracing, on the CPU
engine: an injected engine-loop exception and a stalled step must turn /health
into 503 (what the chart's liveness probe acts on) and fail in-flight requests
with an error instead of hanging; a dying TP worker process must be noticed by
the rank-0 monitor; the step log records every engine step."""
import asyncio
import json
import multiprocessing as mp
import os
import time

import aiohttp
import pytest

from hipserve.config import EngineConfig
from hipserve.engine.llm_engine import LLMEngine
from hipserve.engine.request import SamplingParams
from hipserve.parallel.comm import TPGroup
from hipserve.utils.faults import (FaultInjector, FaultSpec, InjectedFault, WorkerMonitor,
                                   parse_faults)
from hipserve.utils.tracing import Tracer

from .test_server import start_engine_server


def _engine():
    return LLMEngine(EngineConfig(model="tiny-llama", device="cpu", dtype="float32", max_num_seqs=4,
                                  max_num_batched_tokens=64, num_kv_blocks=128, max_model_len=256),
                     tp=TPGroup())


def test_parse_faults():
    fs = parse_faults("raise@3, worker:exit@5:9,rank0:stall@2:0.5")
    assert fs == [FaultSpec("any", "raise", 3), FaultSpec("worker", "exit", 5, 9.0),
                  FaultSpec("rank0", "stall", 2, 0.5)]
    with pytest.raises(ValueError):
        parse_faults("explode@1")
    with pytest.raises(ValueError):
        parse_faults("raise")
    assert parse_faults("") == []


def test_injector_roles_and_once():
    inj = FaultInjector(parse_faults("worker:raise@1,stall@0:0.01"))
    t0 = time.monotonic()
    inj.on_step("rank0", 0)          # stall fires for any role
    assert time.monotonic() - t0 >= 0.01
    inj.on_step("rank0", 0)          # fires once only
    inj.on_step("rank0", 1)          # worker-only fault: not on rank 0
    with pytest.raises(InjectedFault):
        inj.on_step("worker", 1)
    inj.on_step("worker", 1)


def test_engine_step_fault_raises(monkeypatch):
    monkeypatch.setenv("HIPSERVE_FAULT", "raise@2")
    eng = _engine()
    eng.add_request(None, [1, 5, 6, 7], SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True))
    eng.step()
    eng.step()
    with pytest.raises(InjectedFault):
        eng.step()


def test_health_503_on_engine_death_and_stall(monkeypatch):
    async def main(fault, stall_timeout):
        monkeypatch.setenv("HIPSERVE_FAULT", fault)
        monkeypatch.setenv("HIPSERVE_STALL_TIMEOUT", str(stall_timeout))
        ae, runner, port = await start_engine_server()
        base = f"http://127.0.0.1:{port}"
        try:
            async with aiohttp.ClientSession() as s:
                assert (await s.get(base + "/health")).status == 200
                req = asyncio.ensure_future(s.post(base + "/v1/completions", json={
                    "prompt": [1, 5, 6, 7], "max_tokens": 20, "ignore_eos": True, "temperature": 0}))
                statuses = []
                for _ in range(60):
                    await asyncio.sleep(0.1)
                    statuses.append((await s.get(base + "/health")).status)
                    if statuses[-1] == 503:
                        break
                assert statuses[-1] == 503, statuses
                r = await asyncio.wait_for(req, 30)
                return r.status
        finally:
            ae.stop()
            await runner.cleanup()

    # engine-loop exception: the request fails with 500, /health stays 503
    assert asyncio.run(main("raise@1", 120)) == 500
    # stalled step (2 s) longer than the 0.5 s watchdog: /health 503 while stalled,
    # the request still completes afterwards
    assert asyncio.run(main("stall@1:2", 0.5)) == 200


def _exit_soon(code):
    time.sleep(0.3)
    os._exit(code)


def test_worker_monitor_detects_exit():
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_exit_soon, args=(7,))
    p.start()
    dead = []
    mon = WorkerMonitor([p], on_death=dead.append, interval=0.05, exit_after=None)
    mon.start()
    mon.join(timeout=30)
    p.join(5)
    assert dead == [p] and p.exitcode == 7


def test_worker_monitor_stop_is_silent():
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_exit_soon, args=(0,))
    p.start()
    dead = []
    mon = WorkerMonitor([p], on_death=dead.append, interval=0.05, exit_after=None)
    mon.start()
    mon.stop()          # orderly shutdown: workers exiting afterwards are not a failure
    p.join(5)
    mon.join(5)
    assert dead == []


def test_step_log(tmp_path, monkeypatch):
    path = tmp_path / "steps.jsonl"
    monkeypatch.setenv("HIPSERVE_STEP_LOG", str(path))
    monkeypatch.delenv("HIPSERVE_FAULT", raising=False)
    eng = _engine()
    res = eng.generate([[1, 5, 6, 7, 8, 9]], SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    assert len(res[0][0]) == 5
    eng.shutdown()
    recs = [json.loads(x) for x in path.read_text().splitlines()]
    assert [r["step"] for r in recs] == list(range(len(recs)))
    assert recs[0]["kind"] == "prefill" and recs[0]["tokens"] == 6
    assert all(r["kind"] == "decode" and r["tokens"] == 1 for r in recs[1:])
    assert len(recs) == 5


def test_tracer_off_is_noop():
    t = Tracer("")
    assert not t.enabled
    with t.phase("x"):
        pass
    t.step_begin()
    t.step_done("decode", 1, 1, 0.001)
    t.close()


def test_torch_profiler_window(tmp_path, monkeypatch):
    monkeypatch.setenv("HIPSERVE_PROFILE", f"torch:{tmp_path}:1-2")
    monkeypatch.delenv("HIPSERVE_STEP_LOG", raising=False)
    monkeypatch.delenv("HIPSERVE_FAULT", raising=False)
    eng = _engine()
    eng.generate([[1, 5, 6, 7]], SamplingParams(temperature=0.0, max_tokens=5, ignore_eos=True))
    eng.shutdown()
    traces = list(tmp_path.glob("hipserve_steps_*.json"))
    assert len(traces) == 1 and traces[0].stat().st_size > 0
