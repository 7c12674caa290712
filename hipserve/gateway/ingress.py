"""Istio ingress emulator for local / offline runs.

Applies the ``http`` match rules of a rendered Istio ``VirtualService`` exactly
as Envoy would for these charts: rules in order, first match wins; ``exact``,
``prefix`` and ``regex`` URI matches; destination ``host`` (short name or FQDN
``<svc>.<ns>.svc.cluster.local``) + ``port.number``. Service names are resolved
through a map to local ``host:port`` pairs, which stands in for kube-proxy.

This is what "through the Istio gateway" means for measurements taken without a
cluster: the same route table the reference installs
(vllm-models/helm-chart/templates/gateway.yaml:16-57,
ramalama-models/helm-chart/templates/gateway.yaml:16-41) sits in the path.
"""
from __future__ import annotations

import re

import yaml

from .proxy import HTTPProxy, Request, Response


class Rule:
    def __init__(self, matches, host, port):
        self.matches = matches  # list of (kind, value)
        self.host = host
        self.port = port

    def hit(self, path: str) -> bool:
        if not self.matches:
            return True
        for kind, val in self.matches:
            if kind == "exact" and path == val:
                return True
            if kind == "prefix" and path.startswith(val):
                return True
            if kind == "regex" and re.fullmatch(val, path):
                return True
        return False


def rules_from_virtualservice(docs) -> list[Rule]:
    rules = []
    for d in docs:
        if not d or d.get("kind") != "VirtualService":
            continue
        for http in d.get("spec", {}).get("http", []):
            matches = []
            for m in http.get("match", []) or []:
                uri = m.get("uri", {})
                for kind in ("exact", "prefix", "regex"):
                    if kind in uri:
                        matches.append((kind, uri[kind]))
            dest = http["route"][0]["destination"]
            rules.append(Rule(matches, dest["host"], int(dest.get("port", {}).get("number", 80))))
    return rules


def load_rules(path_or_text: str) -> list[Rule]:
    if "\n" not in path_or_text:
        with open(path_or_text) as f:
            path_or_text = f.read()
    return rules_from_virtualservice(list(yaml.safe_load_all(path_or_text)))


class IngressEmulator(HTTPProxy):
    def __init__(self, rules: list[Rule], services: dict[str, tuple[str, int]]):
        super().__init__("ingress")
        self.rules = rules
        self.services = services

    def resolve(self, host: str, port: int):
        for key in (f"{host}:{port}", host, host.split(".")[0] + f":{port}", host.split(".")[0]):
            if key in self.services:
                return self.services[key]
        return None

    async def route(self, req: Request):
        for r in self.rules:
            if r.hit(req.path):
                dest = self.resolve(r.host, r.port)
                if dest is None:
                    return Response(503, b'{"error":"no healthy upstream"}')
                return dest
        return Response(404, b'{"error":"no route"}')
