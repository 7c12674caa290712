"""OpenAI-compatible HTTP server of one model pod (container port 8080).

Endpoints: ``GET /health`` (engine-loop liveness, used by the
chart's readiness/liveness/startup probes), ``GET /v1/models``,
``POST /v1/completions``, ``POST /v1/chat/completions`` (both with SSE
``stream: true``), ``GET /metrics`` (Prometheus), ``POST /tokenize``,
``POST /detokenize``, ``GET /version``.

Replaces the engines the reference launches: ``vllm/vllm-openai:v0.11.0``
(vllm-models/helm-chart/templates/model-deployments.yaml:26-39) and
``llama-server`` (ramalama-models/helm-chart/templates/model-deployments.yaml:26-35).
"""
from __future__ import annotations

import asyncio
import contextlib
import json
import logging
import time
import uuid

from aiohttp import web
from prometheus_client import CONTENT_TYPE_LATEST, generate_latest

from .. import __version__
from ..engine.request import SamplingParams
from ..utils.faults import stall_timeout
from .async_engine import AsyncEngine, EngineDeadError

log = logging.getLogger("hipserve.server")


def _err(status: int, msg: str, typ: str = "invalid_request_error", code=None):
    return web.json_response({"error": {"message": msg, "type": typ, "param": None,
                                        "code": code if code is not None else status}},
                             status=status)


def _dumps(o) -> str:
    return json.dumps(o, separators=(",", ":"), ensure_ascii=False)


def _has_images(msgs) -> bool:
    return any(isinstance(m, dict) and isinstance(m.get("content"), list)
               and any(isinstance(p, dict) and p.get("type") in ("image_url", "image") for p in m["content"])
               for m in msgs)


class OpenAIServer:
    def __init__(self, aengine: AsyncEngine, model_name: str, max_model_len: int,
                 extra_names: tuple = ()):
        self.ae = aengine
        self.engine = aengine.engine
        self.model_name = model_name
        self.names = {model_name, *extra_names}
        self.max_model_len = max_model_len
        self.created = int(time.time())
        self.tokenizer = self.engine.tokenizer
        self.stall_timeout = stall_timeout()

    # ------------------------------------------------------------ app
    def app(self) -> web.Application:
        app = web.Application(client_max_size=256 * 1024 * 1024)
        app.add_routes([
            web.get("/health", self.health),
            web.get("/v1/models", self.models),
            web.get("/version", self.version),
            web.get("/metrics", self.metrics),
            web.post("/v1/completions", self.completions),
            web.post("/v1/chat/completions", self.chat),
            web.post("/tokenize", self.tokenize),
            web.post("/detokenize", self.detokenize),
        ])
        return app

    async def health(self, request):
        if not self.ae.alive:
            return web.Response(status=503, text="engine dead")
        # stuck-loop watchdog: a running engine refreshes its heartbeat every step
        if self.engine.has_unfinished() and time.monotonic() - self.ae.heartbeat > self.stall_timeout:
            return web.Response(status=503, text="engine stalled")
        return web.Response(status=200, text="OK")

    async def version(self, request):
        return web.json_response({"version": __version__, "engine": "hipserve"})

    async def models(self, request):
        data = [{"id": n, "object": "model", "created": self.created, "owned_by": "hipserve",
                 "root": self.engine.cfg.model, "max_model_len": self.max_model_len}
                for n in sorted(self.names)]
        return web.json_response({"object": "list", "data": data})

    async def metrics(self, request):
        body = generate_latest(self.engine.metrics.registry)
        return web.Response(body=body, headers={"Content-Type": CONTENT_TYPE_LATEST})

    async def tokenize(self, request):
        body = await request.json()
        if "messages" in body:
            ids = self.tokenizer.encode_chat(body["messages"])
        else:
            ids = self.tokenizer.encode(body.get("prompt", ""), body.get("add_special_tokens", True))
        return web.json_response({"tokens": ids, "count": len(ids), "max_model_len": self.max_model_len})

    async def detokenize(self, request):
        body = await request.json()
        return web.json_response({"prompt": self.tokenizer.decode(body.get("tokens", []))})

    # ------------------------------------------------------------ helpers
    def _check_model(self, body):
        m = body.get("model")
        if m is not None and m not in self.names:
            return _err(404, f"The model `{m}` does not exist.", "NotFoundError", 404)
        return None

    def _params(self, body, chat: bool) -> SamplingParams:
        mt = body.get("max_completion_tokens") if chat else None
        if mt is None:
            mt = body.get("max_tokens")
        if mt is None:
            mt = self.max_model_len if chat else 16
        lp = body.get("logprobs")
        if chat:  # chat: logprobs is a bool, top_logprobs the count (>= 1 reported)
            if lp is not None and not isinstance(lp, bool):
                raise ValueError("logprobs must be a boolean for chat completions")
            tl = body.get("top_logprobs")
            lp = (1 if tl is None else tl) if lp else None
        stop_ids = body.get("stop_token_ids") or []
        if not isinstance(stop_ids, list):
            raise ValueError("stop_token_ids must be a list of integers")

        def opt(key, default):
            v = body.get(key)
            return default if v is None else v

        # SamplingParams coerces and range-checks every field (ValueError -> 400)
        return SamplingParams(
            temperature=opt("temperature", 1.0), top_p=opt("top_p", 1.0), top_k=opt("top_k", 0),
            max_tokens=mt, min_tokens=opt("min_tokens", 0), stop=opt("stop", []),
            stop_token_ids=stop_ids, ignore_eos=bool(body.get("ignore_eos", False)),
            seed=body.get("seed"), presence_penalty=opt("presence_penalty", 0.0),
            frequency_penalty=opt("frequency_penalty", 0.0),
            repetition_penalty=opt("repetition_penalty", 1.0), logprobs=lp, n=opt("n", 1))

    def _check_prompt(self, ids):
        """The engine's add_request checks, run in the handler so that a bad prompt
        is a 400 before any SSE header goes out (not a truncated stream)."""
        if not ids:
            raise ValueError("empty prompt")
        V = self.engine.model_cfg.vocab_size
        for t in ids:
            if isinstance(t, bool) or not isinstance(t, int) or not 0 <= t < V:
                raise ValueError(f"prompt token id out of range [0, {V})")

    async def _encode_images(self, msgs, vcfg):
        """Chat messages with image parts -> MultiModalPrompt: the template with one
        image marker per part, the images fetched / decoded / patchified off the event
        loop (worker thread), each marker's pad token expanded to the image's merged
        patch count."""
        from ..multimodal import MultiModalPrompt, expand_image_tokens, load_image, preprocess_image

        ids, urls = self.tokenizer.encode_chat_mm(msgs, vcfg)
        allow_local = bool(self.engine.cfg.extra.get("allow_local_media", False))

        def work():
            return [preprocess_image(load_image(u, allow_local=allow_local), vcfg) for u in urls]

        images = await asyncio.get_running_loop().run_in_executor(None, work)
        return MultiModalPrompt(expand_image_tokens(ids, images, vcfg), images)

    def _clip_max_tokens(self, params: SamplingParams, n_prompt: int):
        room = self.max_model_len - n_prompt
        if room <= 0:
            raise ValueError(f"This model's maximum context length is {self.max_model_len} tokens, "
                             f"but the prompt has {n_prompt} tokens.")
        params.max_tokens = min(params.max_tokens, room)

    async def _run_many(self, prompts, params: SamplingParams, base_id):
        """Fan out prompts x n into engine requests; returns list of (index, gen)."""
        gens = []
        idx = 0
        for p in prompts:
            for j in range(params.n):
                sp = params
                if params.n > 1:
                    seed = None if params.seed is None else ((params.seed + j + (1 << 63)) % (1 << 64)) - (1 << 63)
                    sp = SamplingParams(**{**params.__dict__, "n": 1, "seed": seed})
                gens.append((idx, self.ae.generate(f"{base_id}-{idx}", p, sp)))
                idx += 1
        return gens

    # ------------------------------------------------------------ completions
    def _prompts(self, body):
        p = body.get("prompt")
        if p is None:
            raise ValueError("prompt is required")
        if isinstance(p, str):
            return [p]
        if isinstance(p, list) and p and all(isinstance(x, int) for x in p):
            return [p]
        if isinstance(p, list) and all(isinstance(x, (str, list)) for x in p) and p:
            return p
        raise ValueError("prompt must be a string, a list of strings, a token list or a list of token lists")

    async def completions(self, request: web.Request):
        try:
            body = await request.json()
        except Exception:
            return _err(400, "invalid JSON body")
        bad = self._check_model(body)
        if bad:
            return bad
        try:
            params = self._params(body, chat=False)
            prompts = [self.tokenizer.encode(p) if isinstance(p, str) else list(p)
                       for p in self._prompts(body)]
            for p in prompts:
                self._check_prompt(p)
                self._clip_max_tokens(params, len(p))
        except (ValueError, TypeError) as e:
            return _err(400, str(e))
        rid = f"cmpl-{uuid.uuid4().hex}"
        created = int(time.time())
        model = body.get("model") or self.model_name
        stream = bool(body.get("stream", False))
        include_usage = bool((body.get("stream_options") or {}).get("include_usage", False))
        n_prompt_total = sum(len(p) for p in prompts) * params.n
        gens = await self._run_many(prompts, params, rid)
        if stream:
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                               "Cache-Control": "no-cache", "X-Accel-Buffering": "no"})
            await resp.prepare(request)
            n_out = 0
            # per-token SSE events are the HTTP side's hot path (it shares the
            # interpreter with the engine loop): splice pre-serialised constant
            # parts around the per-token fields instead of json.dumps of a dict
            head = 'data: {"id":%s,"object":"text_completion","created":%d,"model":%s,"choices":[{"index":' % (
                _dumps(rid), created, _dumps(model))
            try:
                async with contextlib.aclosing(_merge(gens)) as merged:
                    async for idx, o in merged:
                        n_out += len(o.new_token_ids)
                        if params.logprobs is not None and o.logprobs:
                            ch = {"index": idx, "text": o.new_text, "finish_reason": o.finish_reason if o.finished else None,
                                  "logprobs": {"tokens": [self.tokenizer.decode(o.new_token_ids)],
                                               "token_logprobs": [o.logprobs[0]]}}
                            chunk = {"id": rid, "object": "text_completion", "created": created,
                                     "model": model, "choices": [ch]}
                            await resp.write(("data: " + _dumps(chunk) + "\n\n").encode())
                            continue
                        fin = _dumps(o.finish_reason) if o.finished else "null"
                        await resp.write(f'{head}{idx},"text":{_dumps(o.new_text)},"logprobs":null,'
                                         f'"finish_reason":{fin}}}]}}\n\n'.encode())
                if include_usage:
                    u = {"id": rid, "object": "text_completion", "created": created, "model": model,
                         "choices": [], "usage": _usage(n_prompt_total, n_out)}
                    await resp.write(("data: " + _dumps(u) + "\n\n").encode())
            except (EngineDeadError, ValueError) as e:
                await resp.write(("data: " + _dumps({"error": {"message": str(e)}}) + "\n\n").encode())
            await resp.write(b"data: [DONE]\n\n")
            await resp.write_eof()
            return resp
        try:
            results = await _collect(gens)
        except EngineDeadError as e:
            return _err(500, str(e), "InternalServerError")
        except ValueError as e:
            return _err(400, str(e))
        choices, n_out = [], 0
        for idx in sorted(results):
            text, toks, reason, lps = results[idx]
            n_out += len(toks)
            ch = {"index": idx, "text": text, "logprobs": None, "finish_reason": reason}
            if params.logprobs is not None:
                ch["logprobs"] = {"tokens": [self.tokenizer.decode([t]) for t in toks],
                                  "token_logprobs": lps}
            choices.append(ch)
        return web.json_response({"id": rid, "object": "text_completion", "created": created,
                                  "model": model, "choices": choices,
                                  "usage": _usage(n_prompt_total, n_out)})

    # ------------------------------------------------------------ chat
    async def chat(self, request: web.Request):
        try:
            body = await request.json()
        except Exception:
            return _err(400, "invalid JSON body")
        bad = self._check_model(body)
        if bad:
            return bad
        msgs = body.get("messages")
        if not isinstance(msgs, list) or not msgs:
            return _err(400, "messages must be a non-empty list")
        try:
            params = self._params(body, chat=True)
            vcfg = self.engine.model_cfg.vision
            if vcfg is not None and _has_images(msgs):
                prompt = await self._encode_images(msgs, vcfg)
                ids = prompt.ids
            else:
                ids = prompt = self.tokenizer.encode_chat(msgs, add_generation_prompt=True)
            self._check_prompt(ids)
            self._clip_max_tokens(params, len(ids))
        except (ValueError, TypeError) as e:
            return _err(400, str(e))
        except Exception as e:  # template errors
            return _err(400, f"chat template error: {e}")
        rid = f"chatcmpl-{uuid.uuid4().hex}"
        created = int(time.time())
        model = body.get("model") or self.model_name
        stream = bool(body.get("stream", False))
        include_usage = bool((body.get("stream_options") or {}).get("include_usage", False))
        gens = await self._run_many([prompt], params, rid)
        n_prompt = len(ids) * params.n
        if stream:
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                               "Cache-Control": "no-cache", "X-Accel-Buffering": "no"})
            await resp.prepare(request)
            base = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model}
            first = b"".join(
                ("data: " + _dumps({**base, "choices": [{"index": i, "delta": {"role": "assistant", "content": ""},
                                                         "logprobs": None, "finish_reason": None}]})
                 + "\n\n").encode() for i in range(len(gens)))
            await resp.write(first)
            n_out = 0
            head = 'data: {"id":%s,"object":"chat.completion.chunk","created":%d,"model":%s,"choices":[{"index":' % (
                _dumps(rid), created, _dumps(model))
            try:
                async with contextlib.aclosing(_merge(gens)) as merged:
                    async for idx, o in merged:
                        n_out += len(o.new_token_ids)
                        delta = '{"content":%s}' % _dumps(o.new_text) if (o.new_text or not o.finished) else "{}"
                        fin = _dumps(o.finish_reason) if o.finished else "null"
                        await resp.write(f'{head}{idx},"delta":{delta},"logprobs":null,'
                                         f'"finish_reason":{fin}}}]}}\n\n'.encode())
                if include_usage:
                    await resp.write(("data: " + _dumps({**base, "choices": [],
                                                         "usage": _usage(n_prompt, n_out)}) + "\n\n").encode())
            except (EngineDeadError, ValueError) as e:
                await resp.write(("data: " + _dumps({"error": {"message": str(e)}}) + "\n\n").encode())
            await resp.write(b"data: [DONE]\n\n")
            await resp.write_eof()
            return resp
        try:
            results = await _collect(gens)
        except EngineDeadError as e:
            return _err(500, str(e), "InternalServerError")
        except ValueError as e:
            return _err(400, str(e))
        choices, n_out = [], 0
        for idx in sorted(results):
            text, toks, reason, lps = results[idx]
            n_out += len(toks)
            ch = {"index": idx, "message": {"role": "assistant", "content": text},
                  "logprobs": None, "finish_reason": reason}
            if params.logprobs:
                ch["logprobs"] = {"content": [{"token": self.tokenizer.decode([t]), "logprob": lp}
                                              for t, lp in zip(toks, lps)]}
            choices.append(ch)
        return web.json_response({"id": rid, "object": "chat.completion", "created": created,
                                  "model": model, "choices": choices,
                                  "usage": _usage(n_prompt, n_out)})


def _usage(p, c):
    return {"prompt_tokens": p, "completion_tokens": c, "total_tokens": p + c}


async def _merge(gens):
    """Interleave several async generators, yielding (index, output)."""
    if len(gens) == 1:
        idx, g = gens[0]
        try:
            async for o in g:
                yield idx, o
        finally:  # client gone / handler failed: AsyncEngine.generate aborts the request
            await g.aclose()
        return
    q: asyncio.Queue = asyncio.Queue()
    done = object()

    async def pump(idx, g):
        try:
            async for o in g:
                await q.put((idx, o))
        except BaseException as e:
            await q.put((idx, e))
        finally:
            await q.put((idx, done))

    tasks = [asyncio.ensure_future(pump(i, g)) for i, g in gens]
    remaining = len(tasks)
    try:
        while remaining:
            idx, o = await q.get()
            if o is done:
                remaining -= 1
            elif isinstance(o, BaseException):
                raise o
            else:
                yield idx, o
    finally:
        for t in tasks:
            t.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        for _, g in gens:
            await g.aclose()


async def _collect(gens):
    res = {}
    async for idx, o in _merge(gens):
        r = res.setdefault(idx, ["", [], None, []])
        r[0] += o.new_text
        r[1].extend(o.new_token_ids)
        if o.logprobs:
            r[3].append(o.logprobs[0])
        if o.finished:
            r[2] = o.finish_reason
    return {k: tuple(v) for k, v in res.items()}


async def serve(engine, host: str, port: int, model_name: str, ready: asyncio.Event | None = None,
                extra_names: tuple = (), worker_procs=(), death_grace_s: float = 5.0):
    """Serve until the engine dies. ``worker_procs``: TP worker processes to watch;
    if one exits the engine is marked dead (/health 503) and this process exits
    after ``death_grace_s`` so Kubernetes restarts the pod."""
    loop = asyncio.get_running_loop()
    ae = AsyncEngine(engine)
    ae.start(loop)
    monitor = None
    if worker_procs:
        from ..utils.faults import WorkerMonitor

        monitor = WorkerMonitor(
            worker_procs, exit_after=death_grace_s,
            on_death=lambda p: ae.mark_dead(EngineDeadError(
                f"TP worker pid {getattr(p, 'pid', '?')} exited with code {getattr(p, 'exitcode', '?')}")))
        monitor.start()
    srv = OpenAIServer(ae, model_name, engine.max_model_len, extra_names)
    runner = web.AppRunner(srv.app(), access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, host, port, reuse_port=True, backlog=4096)
    await site.start()
    log.info("hipserve serving %s on %s:%d", model_name, host, port)
    if ready is not None:
        ready.set()
    try:
        while ae.alive or ae.error is None and ae.thread is None:
            await asyncio.sleep(1.0)
        if ae.error is not None:
            # keep serving 503 on /health so k8s restarts the pod
            await asyncio.sleep(3600 * 24 * 365)
    finally:
        if monitor is not None:
            monitor.stop()
        ae.stop()
        await runner.cleanup()
