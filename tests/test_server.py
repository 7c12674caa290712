"""OpenAI API of the engine pod, alone and behind ingress -> router (CPU tiny model)."""
import asyncio
import json

import aiohttp
import pytest
from aiohttp import web

from hipserve.config import EngineConfig
from hipserve.engine.llm_engine import LLMEngine
from hipserve.gateway.ingress import IngressEmulator, load_rules
from hipserve.gateway.router import ModelRouter
from hipserve.parallel.comm import TPGroup
from hipserve.server.api_server import OpenAIServer
from hipserve.server.async_engine import AsyncEngine

from .test_gateway import VS


async def start_engine_server(name="tiny", model="tiny-llama"):
    eng = LLMEngine(EngineConfig(model=model, served_model_name=name, device="cpu", dtype="float32",
                                 max_num_seqs=8, max_num_batched_tokens=64, num_kv_blocks=256,
                                 max_model_len=512), tp=TPGroup())
    ae = AsyncEngine(eng)
    ae.start(asyncio.get_running_loop())
    srv = OpenAIServer(ae, name, eng.max_model_len)
    runner = web.AppRunner(srv.app())
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    return ae, runner, port


async def sse_events(resp):
    out = []
    async for line in resp.content:
        line = line.strip()
        if line.startswith(b"data: "):
            d = line[6:]
            if d == b"[DONE]":
                out.append("[DONE]")
            else:
                out.append(json.loads(d))
    return out


def test_openai_endpoints():
    async def main():
        ae, runner, port = await start_engine_server()
        base = f"http://127.0.0.1:{port}"
        async with aiohttp.ClientSession() as s:
            assert (await s.get(base + "/health")).status == 200
            j = await (await s.get(base + "/v1/models")).json()
            assert j["data"][0]["id"] == "tiny"
            # completions: text prompt, non-streaming
            r = await s.post(base + "/v1/completions", json={"model": "tiny", "prompt": "hello",
                                                             "max_tokens": 5, "temperature": 0})
            j = await r.json()
            assert r.status == 200, j
            assert j["object"] == "text_completion" and j["usage"]["completion_tokens"] <= 5
            # token-id prompt, streaming, with usage
            r = await s.post(base + "/v1/completions", json={
                "model": "tiny", "prompt": [1, 5, 6, 7], "max_tokens": 6, "stream": True,
                "ignore_eos": True, "temperature": 0, "stream_options": {"include_usage": True}})
            ev = await sse_events(r)
            assert ev[-1] == "[DONE]"
            assert ev[-2]["usage"]["completion_tokens"] == 6
            fin = [e for e in ev[:-2] if e["choices"][0]["finish_reason"]]
            assert fin and fin[-1]["choices"][0]["finish_reason"] == "length"
            # chat streaming
            r = await s.post(base + "/v1/chat/completions", json={
                "model": "tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 4,
                "stream": True, "ignore_eos": True})
            ev = await sse_events(r)
            assert ev[0]["choices"][0]["delta"]["role"] == "assistant"
            assert ev[-1] == "[DONE]"
            # chat non-streaming with n=2
            r = await s.post(base + "/v1/chat/completions", json={
                "model": "tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 3,
                "n": 2, "ignore_eos": True})
            j = await r.json()
            assert len(j["choices"]) == 2 and j["choices"][0]["message"]["role"] == "assistant"
            # errors: unknown model (404), bad body (400), too long prompt (400)
            r = await s.post(base + "/v1/completions", json={"model": "other", "prompt": "x"})
            assert r.status == 404
            r = await s.post(base + "/v1/completions", data=b"{")
            assert r.status == 400
            r = await s.post(base + "/v1/completions", json={"prompt": [3] * 600})
            assert r.status == 400
            # tokenize + metrics
            j = await (await s.post(base + "/tokenize", json={"prompt": "ab"})).json()
            assert j["count"] == 3
            m = await (await s.get(base + "/metrics")).text()
            assert "hipserve_generation_tokens" in m
        ae.stop()
        await runner.cleanup()

    asyncio.run(main())


def test_full_path_ingress_router_two_models():
    """client -> ingress (VirtualService rules) -> router (body.model) -> engine pods."""
    async def main():
        ae1, r1, p1 = await start_engine_server("llama", "tiny-llama")
        ae2, r2, p2 = await start_engine_server("mixtral", "tiny-mixtral")
        router = ModelRouter([("llama", [f"127.0.0.1:{p1}"]), ("mixtral", [f"127.0.0.1:{p2}"])])
        await router.start("127.0.0.1", 0)
        ing = IngressEmulator(load_rules(VS), {"api-gateway": ("127.0.0.1", router.port)})
        await ing.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{ing.port}"
        async with aiohttp.ClientSession() as s:
            j = await (await s.get(base + "/v1/models")).json()
            assert [m["id"] for m in j["data"]] == ["llama", "mixtral"]
            for name in ("llama", "mixtral"):
                r = await s.post(base + "/v1/chat/completions", json={
                    "model": name, "messages": [{"role": "user", "content": "hey"}],
                    "max_tokens": 5, "stream": True, "ignore_eos": True})
                ev = await sse_events(r)
                assert ev[-1] == "[DONE]" and ev[0]["model"] == name
            # concurrent streams through the whole path
            async def one(i):
                r = await s.post(base + "/v1/completions", json={
                    "model": "llama", "prompt": [1, i + 3, 7], "max_tokens": 8, "stream": True,
                    "ignore_eos": True})
                ev = await sse_events(r)
                return sum(1 for e in ev if e != "[DONE]" and e["choices"])
            counts = await asyncio.gather(*[one(i) for i in range(12)])
            assert all(c == 8 for c in counts)
        for x in (ing, router):
            await x.stop()
        for ae, rr in ((ae1, r1), (ae2, r2)):
            ae.stop()
            await rr.cleanup()

    asyncio.run(main())


def test_bad_request_fields_are_400_and_engine_survives():
    """out-of-range / mistyped sampling fields used to reach the
    engine thread and kill it. Each must be a 400; the engine stays healthy."""
    async def main():
        ae, runner, port = await start_engine_server()
        base = f"http://127.0.0.1:{port}"
        bad_completions = [{"seed": 2 ** 64}, {"seed": "x"}, {"top_k": 2 ** 40}, {"logprobs": 10 ** 6},
                           {"temperature": "hot"}, {"stop": 5}, {"n": 0}, {"max_tokens": -3},
                           {"presence_penalty": float("inf")}, {"stop_token_ids": "1,2"},
                           {"prompt": [1, 5, 10 ** 9], "stream": True}, {"prompt": [], "stream": True}]
        bad_chat = [{"logprobs": True, "top_logprobs": "abc"}, {"logprobs": 3},
                    {"messages": [{"role": "user", "content": [
                        {"type": "text", "text": "what is this?"},
                        {"type": "image_url", "image_url": {"url": "data:image/png;base64,AAAA"}}]}]},
                    {"messages": [{"role": "user", "content": 7}], "stream": True}]
        async with aiohttp.ClientSession() as s:
            for extra in bad_completions:
                body = {"model": "tiny", "prompt": [1, 5, 6], "max_tokens": 3, **extra}
                r = await s.post(base + "/v1/completions", json=body)
                assert r.status == 400, (extra, r.status, await r.text())
            for extra in bad_chat:
                body = {"model": "tiny", "messages": [{"role": "user", "content": "hi"}], "max_tokens": 3, **extra}
                r = await s.post(base + "/v1/chat/completions", json=body)
                assert r.status == 400, (extra, r.status, await r.text())
            assert (await s.get(base + "/health")).status == 200
            r = await s.post(base + "/v1/completions", json={"model": "tiny", "prompt": [1, 5, 6], "max_tokens": 3,
                                                              "seed": 2 ** 63 - 1, "n": 2, "logprobs": 2})
            assert r.status == 200, await r.text()
            assert ae.alive
        ae.stop()
        await runner.cleanup()

    asyncio.run(main())


def test_client_disconnect_aborts_generation():
    """a client that goes away mid-stream (through the router) must
    abort the generation in the engine, not run on to max_tokens."""
    async def main():
        ae, r1, p1 = await start_engine_server("llama", "tiny-llama")
        router = ModelRouter([("llama", [f"127.0.0.1:{p1}"])])
        await router.start("127.0.0.1", 0)
        eng = ae.engine
        reader, writer = await asyncio.open_connection("127.0.0.1", router.port)
        body = json.dumps({"model": "llama", "prompt": [1, 5, 6], "max_tokens": 480, "stream": True,
                           "ignore_eos": True}).encode()
        writer.write(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                     b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
        await writer.drain()
        got = b""
        while got.count(b"data: ") < 3:
            got += await reader.read(4096)
        assert eng.has_unfinished()
        writer.transport.abort()  # RST: the client is gone
        for _ in range(200):
            await asyncio.sleep(0.05)
            if not eng.has_unfinished():
                break
        assert not eng.has_unfinished(), "generation kept running after the client disconnected"
        assert eng.metrics.total_gen < 480
        await router.stop()
        ae.stop()
        await r1.cleanup()

    asyncio.run(main())


def test_asyncio_debug_mode_clean(caplog):
    """The request path under asyncio debug mode (SURVEY §5 race detection: "CPU-side
    asyncio debug mode"): concurrent streaming and non-streaming requests plus a client
    that disconnects mid-stream leave no never-retrieved task exception, no coroutine
    that was never awaited and no non-threadsafe loop call from the engine thread."""
    import gc
    import logging
    import warnings

    async def main():
        loop = asyncio.get_running_loop()
        loop.slow_callback_duration = 10.0  # CPU model steps are slow; only correctness is checked
        ae, runner, port = await start_engine_server()
        base = f"http://127.0.0.1:{port}"
        async with aiohttp.ClientSession() as s:
            async def stream(i):
                r = await s.post(base + "/v1/chat/completions", json={
                    "model": "tiny", "messages": [{"role": "user", "content": f"hi {i}"}], "max_tokens": 5,
                    "stream": True, "ignore_eos": True})
                return await sse_events(r)

            async def plain(i):
                r = await s.post(base + "/v1/completions", json={"model": "tiny", "prompt": [1, 2, i + 3],
                                                                 "max_tokens": 4, "ignore_eos": True})
                return await r.json()

            res = await asyncio.gather(*[stream(i) for i in range(4)], *[plain(i) for i in range(4)])
            assert all(r[-1] == "[DONE]" for r in res[:4])
            assert all(r["usage"]["completion_tokens"] == 4 for r in res[4:])
            # a client that goes away mid-stream
            reader, writer = await asyncio.open_connection("127.0.0.1", port)
            body = json.dumps({"model": "tiny", "prompt": [5, 6], "max_tokens": 200, "stream": True,
                               "ignore_eos": True}).encode()
            writer.write(b"POST /v1/completions HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                         b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
            await writer.drain()
            await reader.readline()
            writer.close()
            await asyncio.sleep(0.3)
            assert (await s.get(base + "/health")).status == 200
        ae.stop()
        await runner.cleanup()

    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)  # "coroutine ... was never awaited"
        with caplog.at_level(logging.WARNING, logger="asyncio"):
            asyncio.run(main(), debug=True)
            gc.collect()
    bad = [r for r in caplog.records if r.name == "asyncio" and r.levelno >= logging.WARNING
           and "took" not in r.getMessage()]
    assert not bad, [r.getMessage() for r in bad]


def test_idle_arrival_coalescing(monkeypatch):
    """Requests that reach an idle engine a few ms apart start together: the loop keeps
    admitting arrivals until they pause (COALESCE_GAP) or fill a prefill step, so the
    first step is not a lone one-request prefill (profiles/r6_burst_coalescing.md)."""
    import threading
    import time

    from hipserve.server import async_engine as AE

    class Seq:
        num_uncomputed = 100

    class Sched:
        def __init__(self):
            self.waiting = []
            self.max_tokens = 1000

    class Eng:
        def __init__(self):
            self.scheduler = Sched()
            self.steps = []

        def has_unfinished(self):
            return bool(self.scheduler.waiting)

        def add_request(self, rid, prompt, params, arrival_time=None):
            self.scheduler.waiting.append(Seq())

        def step(self):
            self.steps.append(len(self.scheduler.waiting))
            self.scheduler.waiting.clear()
            return []

    monkeypatch.setattr(AE, "COALESCE_GAP", 0.05)
    monkeypatch.setattr(AE, "COALESCE_MAX", 1.0)
    eng = Eng()
    ae = AE.AsyncEngine(eng)
    ae.loop = None

    def feed(n, gap):
        for i in range(n):
            ae._submit.put(("add", (str(i), [1], None, time.monotonic())))
            ae._wake.set()
            time.sleep(gap)

    t = threading.Thread(target=ae._run, daemon=True)
    t.start()
    feed(5, 0.01)  # 5 arrivals 10 ms apart: one step of 5
    time.sleep(0.3)
    assert eng.steps == [5], eng.steps
    feed(12, 0.005)  # 12 x 100 prompt tokens > the 1000-token budget: the step starts at 10
    time.sleep(0.3)
    assert eng.steps[1] == 10 and sum(eng.steps) == 17, eng.steps
    ae._stop = True
    ae._wake.set()
    t.join(2)
