"""Model-name router: the OpenAI-compatible API gateway in front of the model
pods.

Same routing contract as both reference routers:
  * ``GET /v1/models`` answered statically from configuration, never touching an
    engine (vllm-models/helm-chart/templates/model-gateway.yaml:29-49;
    ramalama-models/helm-chart/templates/api-gateway.yaml:43-61);
  * ``GET /health`` -> ``200 OK`` (model-gateway.yaml:84-86; api-gateway.yaml:32-36);
  * anything else is proxied to the backend whose name equals the JSON body's
    ``model`` field, else to the FIRST configured model
    (model-gateway.yaml:20-22,51-75; api-gateway.yaml:26,68-77).
Beyond the reference: streaming relay, any body size, status pass-through,
several replicas per model (round-robin, like a k8s Service), request counters.
"""
from __future__ import annotations

import itertools
import json
import os
import time
from urllib.parse import urlparse

from .proxy import HTTPProxy, Request, Response


def parse_upstream(u: str):
    if "://" not in u:
        u = "http://" + u
    p = urlparse(u)
    return p.hostname, p.port or 80


class ModelRouter(HTTPProxy):
    def __init__(self, backends: list[tuple[str, list[str]]], owned_by: str = "hipserve",
                 created: int | None = None):
        super().__init__("router")
        if not backends:
            raise ValueError("router needs at least one model backend")
        self.order = [name for name, _ in backends]
        self.backends = {name: [parse_upstream(u) for u in ups] for name, ups in backends}
        self.rr = {name: itertools.cycle(range(len(ups))) for name, ups in self.backends.items()}
        self.default = self.order[0]
        self.owned_by = owned_by
        self.created = created
        self.routed = {name: 0 for name in self.order}

    def pick(self, name: str):
        ups = self.backends[name]
        return ups[next(self.rr[name])] if len(ups) > 1 else ups[0]

    def models_body(self) -> bytes:
        created = self.created if self.created is not None else int(time.time())
        data = [{"id": n, "object": "model", "created": created, "owned_by": self.owned_by}
                for n in self.order]
        return json.dumps({"object": "list", "data": data}).encode()

    async def route(self, req: Request):
        path = req.path
        if path == "/v1/models" and req.method in ("GET", "HEAD"):
            return Response(200, self.models_body())
        if path == "/health":
            return Response(200, b"OK", content_type="text/plain")
        name = self.default
        if req.body:
            body = req.json()
            if isinstance(body, dict):
                m = body.get("model")
                if isinstance(m, str) and m in self.backends:
                    name = m
        self.routed[name] += 1
        return self.pick(name)


def backends_from_env(env: dict | None = None) -> list[tuple[str, list[str]]]:
    """``HIPSERVE_BACKENDS`` = JSON list of {"name", "url" | "urls"} (the chart
    renders it from .Values.models, like the reference's BACKENDS dict)."""
    env = env or os.environ
    raw = env.get("HIPSERVE_BACKENDS")
    if not raw and env.get("HIPSERVE_BACKENDS_FILE"):
        with open(env["HIPSERVE_BACKENDS_FILE"]) as f:
            raw = f.read()
    if not raw:
        return []
    out = []
    for b in json.loads(raw):
        urls = b.get("urls") or [b["url"]]
        out.append((b["name"], urls))
    return out
