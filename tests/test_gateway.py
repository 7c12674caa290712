"""Router + ingress emulator + engine server over real sockets."""
import asyncio
import json
import time

import aiohttp
import pytest
from aiohttp import web

from hipserve.gateway.ingress import IngressEmulator, load_rules
from hipserve.gateway.router import ModelRouter

VS = """
apiVersion: networking.istio.io/v1alpha3
kind: VirtualService
metadata: {name: vs}
spec:
  hosts: ["*"]
  gateways: [gw]
  http:
  - match: [{uri: {exact: /v1/models}}]
    route: [{destination: {host: api-gateway, port: {number: 8080}}}]
  - match: [{uri: {prefix: /v1/}}]
    route: [{destination: {host: api-gateway.ns.svc.cluster.local, port: {number: 8080}}}]
  - match: [{uri: {prefix: /health}}]
    route: [{destination: {host: api-gateway, port: {number: 8080}}}]
  - match: [{uri: {prefix: /}}]
    route: [{destination: {host: webui, port: {number: 8080}}}]
"""


async def fake_upstream(tag, sse_delay=0.0, status=200):
    seen = []

    async def any_(request):
        body = await request.read()
        seen.append((request.path, len(body)))
        if request.path.endswith("/stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(request)
            await resp.write(f"data: {tag}-1\n\n".encode())
            await asyncio.sleep(sse_delay)
            await resp.write(f"data: {tag}-2\n\n".encode())
            await resp.write_eof()
            return resp
        return web.json_response({"who": tag, "n": len(body)}, status=status)

    app = web.Application(client_max_size=1 << 30)
    app.router.add_route("*", "/{tail:.*}", any_)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    return runner, port, seen


def run(coro):
    return asyncio.run(coro)


def test_router_contract():
    async def main():
        ra, pa, seen_a = await fake_upstream("A")
        rb, pb, seen_b = await fake_upstream("B", status=404)
        router = ModelRouter([("alpha", [f"http://127.0.0.1:{pa}"]), ("beta", [f"127.0.0.1:{pb}"]),
                              ("dead", ["127.0.0.1:1"])])
        await router.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{router.port}"
        async with aiohttp.ClientSession() as s:
            r = await s.get(base + "/v1/models")
            j = await r.json()
            assert [m["id"] for m in j["data"]] == ["alpha", "beta", "dead"]
            assert all(m["object"] == "model" for m in j["data"])
            r = await s.get(base + "/health")
            assert r.status == 200 and await r.text() == "OK"
            r = await s.post(base + "/v1/chat/completions", json={"model": "alpha"})
            assert (await r.json())["who"] == "A"
            # upstream status passes through (reference Python router turned it into 502)
            r = await s.post(base + "/v1/chat/completions", json={"model": "beta"})
            assert r.status == 404 and (await r.json())["who"] == "B"
            # unknown model and missing body -> default = first model
            r = await s.post(base + "/v1/completions", json={"model": "nope"})
            assert (await r.json())["who"] == "A"
            r = await s.post(base + "/v1/completions", data=b"not json")
            assert (await r.json())["who"] == "A"
            # 3 MiB body still routed by model (nginx spilled >16 KiB bodies to disk -> default)
            big = {"model": "beta", "prompt": "x" * (3 << 20)}
            r = await s.post(base + "/v1/completions", json=big)
            assert r.status == 404 and (await r.json())["n"] > (3 << 20)
            # chunked request body
            async def gen():
                yield json.dumps({"model": "alpha", "p": "y" * 100000}).encode()
            r = await s.post(base + "/v1/completions", data=gen())
            assert (await r.json())["who"] == "A"
            # dead upstream -> 502
            r = await s.post(base + "/v1/completions", json={"model": "dead"})
            assert r.status == 502
        assert router.routed["alpha"] >= 3
        await router.stop()
        await ra.cleanup()
        await rb.cleanup()

    run(main())


def test_router_streams_without_buffering():
    async def main():
        ra, pa, _ = await fake_upstream("A", sse_delay=0.5)
        router = ModelRouter([("alpha", [f"127.0.0.1:{pa}"])])
        await router.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as s:
            t0 = time.monotonic()
            r = await s.post(f"http://127.0.0.1:{router.port}/v1/stream", json={"model": "alpha"})
            first = await r.content.readuntil(b"\n\n")
            t_first = time.monotonic() - t0
            rest = await r.content.read()
            t_all = time.monotonic() - t0
        assert first == b"data: A-1\n\n" and b"A-2" in rest
        assert t_first < 0.3 < t_all
        await router.stop()
        await ra.cleanup()

    run(main())


def test_ingress_rules_and_replicas():
    async def main():
        rt, prt, _ = await fake_upstream("ROUTER")
        ui, pui, _ = await fake_upstream("UI")
        r1, p1, s1 = await fake_upstream("R1")
        r2, p2, s2 = await fake_upstream("R2")
        ing = IngressEmulator(load_rules(VS), {"api-gateway:8080": ("127.0.0.1", prt),
                                               "webui": ("127.0.0.1", pui)})
        await ing.start("127.0.0.1", 0)
        base = f"http://127.0.0.1:{ing.port}"
        async with aiohttp.ClientSession() as s:
            for path, who in [("/v1/models", "ROUTER"), ("/v1/chat/completions", "ROUTER"),
                              ("/health", "ROUTER"), ("/", "UI"), ("/c/abc", "UI")]:
                r = await s.post(base + path, json={})
                assert (await r.json())["who"] == who, path
        # round-robin over replicas of one model (k8s Service semantics)
        router = ModelRouter([("m", [f"127.0.0.1:{p1}", f"127.0.0.1:{p2}"])])
        await router.start("127.0.0.1", 0)
        async with aiohttp.ClientSession() as s:
            for _ in range(4):
                await s.post(f"http://127.0.0.1:{router.port}/v1/x", json={"model": "m"})
        assert len(s1) == 2 and len(s2) == 2
        for x in (ing, router):
            await x.stop()
        for x in (rt, ui, r1, r2):
            await x.cleanup()

    run(main())
