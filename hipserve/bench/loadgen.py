"""OpenAI streaming load generator: output tok/s, TTFT, ITL
measured client-side, i.e. through whatever sits in front of the engine
(ingress emulator -> router -> engine, or a real Istio gateway URL).

Closed-loop "waves": ``concurrency`` requests sent at once, each a synthetic
prompt of ``input_len`` random token ids asking for exactly ``output_len`` tokens
(``ignore_eos``). CLI: ``python -m hipserve.bench.loadgen --url http://host:port``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import statistics
import time

import aiohttp


def request_body(model, prompt, output_len, temperature, top_p, seed=None) -> bytes:
    body = {"model": model, "prompt": prompt, "max_tokens": output_len, "stream": True,
            "ignore_eos": True, "temperature": temperature, "top_p": top_p,
            "stream_options": {"include_usage": True}}
    if seed is not None:
        body["seed"] = seed
    return json.dumps(body, separators=(",", ":")).encode()


_JSON = {"Content-Type": "application/json"}


async def one_request(session, url, model, prompt, output_len, temperature, top_p, seed=None, body=None):
    """One streaming completion; ``body`` = the pre-encoded request (a client
    has its request ready before the clock starts). Token events are counted
    without decoding their JSON; only the final usage event is parsed."""
    if body is None:
        body = request_body(model, prompt, output_len, temperature, top_p, seed)
    t0 = time.perf_counter()
    ttft = None
    last = t0
    itls = []
    ntok = 0
    usage = None
    async with session.post(url + "/v1/completions", data=body, headers=_JSON) as r:
        if r.status != 200:
            raise RuntimeError(f"HTTP {r.status}: {(await r.text())[:300]}")
        buf = b""
        async for chunk in r.content.iter_any():
            buf += chunk
            if b"\n\n" not in buf:
                continue
            *events, buf = buf.split(b"\n\n")
            now = time.perf_counter()
            for ev in events:
                if not ev.startswith(b"data: ") or ev == b"data: [DONE]":
                    continue
                if b'"usage"' in ev:
                    j = json.loads(ev[6:])
                    if j.get("usage"):
                        usage = j["usage"]
                    if not j.get("choices"):
                        continue
                elif b'"choices":[]' in ev:
                    continue
                if ttft is None:
                    ttft = now - t0
                else:
                    itls.append(now - last)
                last = now
                ntok += 1
    n = usage["completion_tokens"] if usage else ntok
    return {"ttft": ttft, "tokens": n, "latency": time.perf_counter() - t0, "itl": itls}


def make_prompts(rng: random.Random, concurrency: int, input_len: int, vocab: int) -> list[list[int]]:
    """Synthetic prompts: uniform random token ids in [10, vocab)."""
    import numpy as np

    g = np.random.default_rng(rng.getrandbits(63))
    return g.integers(10, vocab, size=(concurrency, input_len)).tolist()


async def wave(url, model, concurrency, input_len, output_len, vocab, temperature=0.8, top_p=0.95,
               rng=None, session=None, prompts=None, bodies=None):
    rng = rng or random.Random(0)
    if prompts is None and bodies is None:
        prompts = make_prompts(rng, concurrency, input_len, vocab)
    if bodies is None:
        bodies = [request_body(model, p, output_len, temperature, top_p) for p in prompts]
    own = session is None
    if own:
        session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                        connector=aiohttp.TCPConnector(limit=0))
    try:
        res = await asyncio.gather(*[one_request(session, url, model, None, output_len, temperature, top_p,
                                                 body=b) for b in bodies])
    finally:
        if own:
            await session.close()
    return res


async def open_loop(url, model, rate, num_requests, input_len, output_len, vocab, temperature=0.8, top_p=0.95,
                    rng=None, session=None, burstiness=1.0):
    """Open-loop arrivals: ``num_requests`` requests with gamma-distributed
    inter-arrival gaps of mean 1/``rate`` seconds (burstiness 1.0 = Poisson), each
    sent at its arrival time whether or not earlier ones finished — TTFT then
    reflects queueing under a realistic load instead of one synchronised wave."""
    import numpy as np

    rng = rng or random.Random(0)
    g = np.random.default_rng(rng.getrandbits(63))
    bodies = [request_body(model, p, output_len, temperature, top_p)
              for p in make_prompts(rng, num_requests, input_len, vocab)]
    shape = 1.0 / burstiness
    gaps = g.gamma(shape, 1.0 / (rate * shape), size=num_requests) if rate > 0 else np.zeros(num_requests)
    own = session is None
    if own:
        session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                        connector=aiohttp.TCPConnector(limit=0))
    try:
        t0 = time.perf_counter()
        at = np.cumsum(gaps)

        async def fire(i):
            d = t0 + at[i] - time.perf_counter()
            if d > 0:
                await asyncio.sleep(d)
            return await one_request(session, url, model, None, output_len, temperature, top_p, body=bodies[i])

        res = await asyncio.gather(*[fire(i) for i in range(num_requests)])
        return res, time.perf_counter() - t0
    finally:
        if own:
            await session.close()


def summarize(results, elapsed):
    toks = sum(r["tokens"] for r in results)
    ttfts = sorted(r["ttft"] for r in results if r["ttft"] is not None)
    itls = sorted(x for r in results for x in r["itl"])
    pct = lambda xs, q: xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None  # noqa: E731
    return {"requests": len(results), "output_tokens": toks, "elapsed_s": elapsed,
            "output_tok_per_s": toks / elapsed if elapsed > 0 else 0.0,
            "p50_ttft_ms": 1000 * statistics.median(ttfts) if ttfts else None,
            "p90_ttft_ms": 1000 * pct(ttfts, 0.9) if ttfts else None,
            "p50_itl_ms": 1000 * statistics.median(itls) if itls else None,
            "p90_itl_ms": 1000 * pct(itls, 0.9) if itls else None}


async def run(url, model, concurrency, input_len, output_len, vocab, waves, warmup, **kw):
    rng = random.Random(1234)
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                     connector=aiohttp.TCPConnector(limit=0)) as s:
        for _ in range(warmup):
            await wave(url, model, concurrency, input_len, output_len, vocab, rng=rng, session=s, **kw)
        t0 = time.perf_counter()
        res = []
        for _ in range(waves):
            res += await wave(url, model, concurrency, input_len, output_len, vocab, rng=rng, session=s, **kw)
        return summarize(res, time.perf_counter() - t0)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--model", default=None)
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--input-len", type=int, default=1024)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=32000)
    ap.add_argument("--waves", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--request-rate", type=float, default=None,
                    help="open loop: mean arrivals per second (Poisson; --burstiness for gamma) instead of waves")
    ap.add_argument("--num-requests", type=int, default=256, help="open loop: requests to send")
    ap.add_argument("--burstiness", type=float, default=1.0)
    a = ap.parse_args(argv)

    async def go():
        model = a.model
        if model is None:
            async with aiohttp.ClientSession() as s:
                j = await (await s.get(a.url + "/v1/models")).json()
                model = j["data"][0]["id"]
        if a.request_rate is not None:
            res, el = await open_loop(a.url, model, a.request_rate, a.num_requests, a.input_len, a.output_len,
                                      a.vocab, burstiness=a.burstiness)
            return {**summarize(res, el), "mode": "open-loop", "request_rate": a.request_rate}
        return await run(a.url, model, a.concurrency, a.input_len, a.output_len, a.vocab, a.waves, a.warmup)

    print(json.dumps(asyncio.run(go())))




def _bodies(rng, key):
    model, conc, inp, out, vocab, temp, top_p = key
    return [request_body(model, p, out, temp, top_p) for p in make_prompts(rng, conc, inp, vocab)]


def serve_stdio():
    """Line-oriented JSON command loop (used by bench.py so the client runs in its
    own process and never competes with the engine for the GIL)."""
    import sys

    loop = asyncio.new_event_loop()
    session = None
    rng = random.Random(1234)
    pending = None  # (shape key, prompts) of the NEXT wave, generated while idle:
    # a client has its prompts ready; building them is not part of the timed wave
    for line in sys.stdin:
        cmd = json.loads(line)
        if cmd["op"] == "quit":
            break
        if session is None:
            async def mk():
                return aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                             connector=aiohttp.TCPConnector(limit=0))
            session = loop.run_until_complete(mk())
        if cmd["op"] == "open":
            try:
                res, el = loop.run_until_complete(open_loop(
                    cmd["url"], cmd["model"], cmd["rate"], cmd["num_requests"], cmd["input_len"],
                    cmd["output_len"], cmd["vocab"], cmd.get("temperature", 0.8), cmd.get("top_p", 0.95),
                    rng=rng, session=session, burstiness=cmd.get("burstiness", 1.0)))
                out = {"ok": True, "results": res, "elapsed": el}
            except Exception as e:
                out = {"ok": False, "error": repr(e)}
            sys.stdout.write(json.dumps(out) + "\n")
            sys.stdout.flush()
            continue
        if cmd["op"] == "wave":
            key = (cmd["model"], cmd["concurrency"], cmd["input_len"], cmd["output_len"], cmd["vocab"],
                   cmd.get("temperature", 0.8), cmd.get("top_p", 0.95))
            bodies = pending[1] if pending is not None and pending[0] == key else _bodies(rng, key)
            t0 = time.perf_counter()
            try:
                res = loop.run_until_complete(wave(cmd["url"], cmd["model"], cmd["concurrency"],
                                                   cmd["input_len"], cmd["output_len"], cmd["vocab"],
                                                   cmd.get("temperature", 0.8), cmd.get("top_p", 0.95),
                                                   rng=rng, session=session, bodies=bodies))
                out = {"ok": True, "results": res, "elapsed": time.perf_counter() - t0}
            except Exception as e:
                out = {"ok": False, "error": repr(e)}
            sys.stdout.write(json.dumps(out) + "\n")
            sys.stdout.flush()
            pending = (key, _bodies(rng, key))
    if session is not None:
        loop.run_until_complete(session.close())


if __name__ == "__main__":
    import sys as _sys

    if "--serve" in _sys.argv:
        serve_stdio()
    else:
        main()
