"""``python -m hipserve.gateway router|ingress`` — see router.py / ingress.py."""
import argparse
import asyncio
import logging
import multiprocessing as mp
import os
import sys

from .ingress import IngressEmulator, load_rules
from .router import ModelRouter, backends_from_env, parse_upstream


def _build(a):
    if a.cmd == "router":
        backends = []
        for spec in a.backend or []:
            name, _, urls = spec.partition("=")
            backends.append((name, urls.split(",")))
        backends = backends or backends_from_env()
        return ModelRouter(backends)
    services = {}
    for spec in a.service or []:
        name, _, url = spec.partition("=")
        services[name] = parse_upstream(url)
    return IngressEmulator(load_rules(a.virtualservice), services)


async def _serve(a):
    proxy = _build(a)
    host, _, port = a.listen.rpartition(":")
    await proxy.start(host or "0.0.0.0", int(port))
    logging.getLogger("hipserve.gateway").info("%s listening on %s", a.cmd, a.listen)
    await asyncio.Event().wait()


def _run(a):
    asyncio.run(_serve(a))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="hipserve-gateway")
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("router", help="model-name router (OpenAI API gateway)")
    r.add_argument("--listen", default=f"0.0.0.0:{os.environ.get('PORT', '8080')}")
    r.add_argument("--backend", action="append", help="NAME=URL[,URL...] (first = default model)")
    r.add_argument("--workers", type=int, default=int(os.environ.get("HIPSERVE_GATEWAY_WORKERS", "1")))
    i = sub.add_parser("ingress", help="Istio VirtualService emulator")
    i.add_argument("--listen", default="0.0.0.0:8080")
    i.add_argument("--virtualservice", required=True, help="rendered YAML file with the VirtualService")
    i.add_argument("--service", action="append", help="HOST[:PORT]=URL (k8s Service -> local address)")
    i.add_argument("--workers", type=int, default=1)
    ap.add_argument("--log-level", default="INFO")
    ap.add_argument("--log-format", default=None, choices=["text", "json"],
                    help="text (default) or one JSON object per line (HIPSERVE_LOG_FORMAT)")
    a = ap.parse_args(argv)
    from ..utils.logs import setup_logging
    setup_logging(a.log_level, a.log_format)
    if a.workers > 1:  # SO_REUSEPORT worker processes, like nginx workers
        procs = [mp.get_context("fork").Process(target=_run, args=(a,)) for _ in range(a.workers)]
        for p in procs:
            p.start()
        for p in procs:
            p.join()
    else:
        _run(a)


if __name__ == "__main__":
    sys.exit(main())
