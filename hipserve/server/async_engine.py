"""Asyncio front of the engine: the engine loop runs in its own thread (GPU work
is launched from there, the GIL is released while the device runs), the HTTP
side submits requests and receives per-step output batches through
``loop.call_soon_threadsafe`` — one cross-thread hop per engine step, not per
token."""
from __future__ import annotations

import asyncio
import logging
import os
import queue
import threading
import time
import traceback

from ..engine.llm_engine import LLMEngine
from ..engine.request import RequestOutput, SamplingParams

log = logging.getLogger("hipserve.engine")

# Idle-arrival coalescing: when requests arrive at an idle engine (nothing running or in
# flight), the engine keeps admitting arrivals before its first step until they pause for
# COALESCE_GAP, the waiting prompts fill one prefill step, or COALESCE_MAX has passed. A
# burst of requests (OpenWebUI fan-out, the bench's closed-loop waves through three HTTP
# hops: 64 arrivals over ~20 ms) otherwise starts with a one-request prefill step and
# needs one prefill step more than its tokens fill (profiles/r6_burst_coalescing.md).
# A lone request waits at most COALESCE_GAP. 0 disables. (2 ms measured too short: a
# burst's first request, on a kept-alive connection, leads the rest by several ms)
COALESCE_GAP = float(os.environ.get("HIPSERVE_COALESCE_GAP_MS", "5")) / 1000.0
COALESCE_MAX = float(os.environ.get("HIPSERVE_COALESCE_MAX_MS", "20")) / 1000.0


class EngineDeadError(RuntimeError):
    pass


class AsyncEngine:
    def __init__(self, engine: LLMEngine, loop: asyncio.AbstractEventLoop | None = None):
        self.engine = engine
        self.loop = loop
        self._submit: queue.SimpleQueue = queue.SimpleQueue()
        self._wake = threading.Event()
        self._queues: dict[str, asyncio.Queue] = {}
        self._stop = False
        self.error: BaseException | None = None
        self.thread: threading.Thread | None = None
        self.heartbeat = time.monotonic()
        self.steps = 0

    def start(self, loop: asyncio.AbstractEventLoop | None = None):
        self.loop = loop or asyncio.get_event_loop()
        self.thread = threading.Thread(target=self._run, name="hipserve-engine", daemon=True)
        self.thread.start()

    def stop(self):
        self._stop = True
        self._wake.set()
        if self.thread:
            self.thread.join(timeout=10)

    @property
    def alive(self) -> bool:
        return self.thread is not None and self.thread.is_alive() and self.error is None

    def mark_dead(self, exc: BaseException):
        """Declare the engine dead from outside the engine thread (e.g. a TP
        worker exited: the engine thread may be stuck in a collective forever).
        ``/health`` turns 503 and every waiting request gets an error."""
        if self.error is None:
            self.error = exc
            log.error("engine marked dead: %s", exc)
            if self.loop is not None:
                self.loop.call_soon_threadsafe(self._fail_all, exc)

    # ------------------------------------------------------------ engine thread
    def _run(self):
        eng = self.engine
        try:
            while not self._stop:
                self.heartbeat = time.monotonic()
                idle = not eng.has_unfinished()
                if self._drain() and idle:
                    self._coalesce()
                if not eng.has_unfinished():
                    self._wake.wait(timeout=0.5)
                    self._wake.clear()
                    continue
                outs = eng.step()
                self.steps += 1
                if outs:
                    self.loop.call_soon_threadsafe(self._dispatch, outs)
        except BaseException as e:  # surface to /health and every waiter
            self.error = e
            log.error("engine loop died: %s", traceback.format_exc())
            self.loop.call_soon_threadsafe(self._fail_all, e)

    def _coalesce(self):
        """The engine was idle and requests arrived: admit further arrivals until they
        pause for COALESCE_GAP, the waiting prompt tokens fill one prefill step, or
        COALESCE_MAX has passed since the first."""
        sch = self.engine.scheduler
        if COALESCE_MAX <= 0 or COALESCE_GAP <= 0:
            return
        t0 = last = time.monotonic()
        while not self._stop:
            if sum(s.num_uncomputed for s in sch.waiting) >= sch.max_tokens:
                return
            now = time.monotonic()
            left = min(COALESCE_GAP - (now - last), COALESCE_MAX - (now - t0))
            if left <= 0:
                return
            self._wake.wait(timeout=left)
            self._wake.clear()
            if self._drain():
                last = time.monotonic()

    def _drain(self) -> int:
        """Moves submitted requests / aborts into the engine; returns the requests added."""
        added = 0
        while True:
            try:
                kind, args = self._submit.get_nowait()
            except queue.Empty:
                return added
            if kind == "add":
                added += 1
                rid, prompt, params, arrival = args
                try:
                    self.engine.add_request(rid, prompt, params, arrival_time=arrival)
                except Exception as e:  # validation errors go back to the request
                    self.loop.call_soon_threadsafe(self._deliver_error, rid, e)
            elif kind == "abort":
                self.engine.abort(args)

    # ------------------------------------------------------------ loop side
    def _dispatch(self, outs: list[RequestOutput]):
        for o in outs:
            q = self._queues.get(o.request_id)
            if q is not None:
                q.put_nowait(o)
                if o.finished:
                    self._queues.pop(o.request_id, None)

    def _deliver_error(self, rid, e):
        q = self._queues.pop(rid, None)
        if q is not None:
            q.put_nowait(e)

    def _fail_all(self, e):
        for q in self._queues.values():
            q.put_nowait(EngineDeadError(str(e)))
        self._queues.clear()

    async def generate(self, request_id: str, prompt, params: SamplingParams):
        """Async iterator of RequestOutput deltas for one request."""
        if self.error is not None:
            raise EngineDeadError(str(self.error))
        q: asyncio.Queue = asyncio.Queue()
        self._queues[request_id] = q
        self._submit.put(("add", (request_id, prompt, params, time.monotonic())))
        self._wake.set()
        try:
            while True:
                o = await q.get()
                if isinstance(o, BaseException):
                    raise o
                yield o
                if o.finished:
                    return
        except (asyncio.CancelledError, GeneratorExit):
            self.abort(request_id)
            raise
        finally:
            self._queues.pop(request_id, None)

    def abort(self, request_id: str):
        if request_id in self._queues:
            self._queues.pop(request_id, None)
        self._submit.put(("abort", request_id))
        self._wake.set()
