"""Run the chart-defined serving path locally, without a cluster.

The hf-models chart is rendered with tools/helmlite.py; its Istio VirtualService
feeds the ingress emulator and the model list feeds the model-name router, each
in its own process (like the pods they stand in for). Engines are either given
(already listening on known ports) or started here as ``python -m
hipserve.server`` subprocesses.

    python -m hipserve.bench.local_stack --model tiny-llama --device cpu --port 8080
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_next_port = [0]


def _bindable(p: int) -> bool:
    s = socket.socket()
    try:
        s.bind(("127.0.0.1", p))
        return True
    except OSError:
        return False
    finally:
        s.close()


def free_port() -> int:
    """A free localhost port. Under torchrun (WORLD_SIZE > 1) every local rank scans
    its own disjoint range, so the N replicas of a DP bench starting at the same
    moment never pick the same port between probe and bind (the kernel's bind(0)
    can hand the port one rank just released to the next)."""
    world = int(os.environ.get("WORLD_SIZE", "1") or 1)
    if world > 1:
        base = 30000 + 200 * int(os.environ.get("LOCAL_RANK", "0") or 0)
        while _next_port[0] < 200:
            p = base + _next_port[0]
            _next_port[0] += 1
            if _bindable(p):
                return p
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def render_hf_chart(models: list[dict], namespace: str = "default", extra: dict | None = None):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from helmlite import manifests, render_chart

    vals = {"models": models}
    vals.update(extra or {})
    return manifests(render_chart(os.path.join(ROOT, "deploy/charts/hf-models"), vals,
                                  namespace=namespace))


def wait_http(url: str, timeout: float = 600.0, proc: subprocess.Popen | None = None):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"process for {url} exited with {proc.returncode}")
        try:
            with urllib.request.urlopen(url, timeout=2) as r:
                if r.status == 200:
                    return
        except Exception:
            pass
        time.sleep(0.2)
    raise TimeoutError(url)


class GatewayStack:
    """ingress emulator -> model-name router -> engines, all on 127.0.0.1."""

    def __init__(self, engines: dict[str, list[int]], namespace: str = "default"):
        self.engines = engines
        self.namespace = namespace
        self.router_port = free_port()
        self.ingress_port = free_port()
        self.procs: list[subprocess.Popen] = []
        self.tmp = tempfile.mkdtemp(prefix="hipserve-stack-")

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.ingress_port}"

    def start(self):
        models = [{"huggingfaceId": name, "modelName": name, "gpuRequestCount": 1} for name in self.engines]
        docs = render_hf_chart(models, self.namespace)
        vs = [d for d in docs if d["kind"] == "VirtualService"]
        prefix = "hipserve"
        vs_path = os.path.join(self.tmp, "virtualservice.yaml")
        with open(vs_path, "w") as f:
            yaml.safe_dump_all([{k: v for k, v in d.items() if k != "__source"} for d in vs], f)
        env = dict(os.environ)
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        router_cmd = [sys.executable, "-m", "hipserve.gateway", "router",
                      "--listen", f"127.0.0.1:{self.router_port}"]
        for name, ports in self.engines.items():
            router_cmd += ["--backend", name + "=" + ",".join(f"127.0.0.1:{p}" for p in ports)]
        ingress_cmd = [sys.executable, "-m", "hipserve.gateway", "ingress",
                       "--listen", f"127.0.0.1:{self.ingress_port}", "--virtualservice", vs_path,
                       "--service", f"{prefix}-api-gateway=127.0.0.1:{self.router_port}",
                       "--service", f"{prefix}-webui=127.0.0.1:{self.router_port}"]
        for cmd in (router_cmd, ingress_cmd):
            self.procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL,
                                               stderr=subprocess.DEVNULL))
        wait_http(f"http://127.0.0.1:{self.router_port}/health", 60, self.procs[0])
        wait_http(self.url + "/health", 60, self.procs[1])
        return self

    def stop(self):
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        self.procs = []


class LoadgenProc:
    """The load generator in its own process, driven over stdin/stdout."""

    def __init__(self):
        import json  # noqa: F401

        env = dict(os.environ)
        env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
        self.p = subprocess.Popen([sys.executable, "-m", "hipserve.bench.loadgen", "--serve"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env, text=True)

    def wave(self, **kw):
        import json

        self.p.stdin.write(json.dumps({"op": "wave", **kw}) + "\n")
        self.p.stdin.flush()
        line = self.p.stdout.readline()
        if not line:
            raise RuntimeError("load generator died")
        out = json.loads(line)
        if not out["ok"]:
            raise RuntimeError(out["error"])
        return out["results"]

    def open_loop(self, **kw):
        """Open-loop arrivals (loadgen.open_loop); returns (results, elapsed_s)."""
        import json

        self.p.stdin.write(json.dumps({"op": "open", **kw}) + "\n")
        self.p.stdin.flush()
        out = json.loads(self.p.stdout.readline() or '{"ok": false, "error": "load generator died"}')
        if not out["ok"]:
            raise RuntimeError(out["error"])
        return out["results"], out["elapsed"]

    def close(self):
        try:
            self.p.stdin.write('{"op": "quit"}\n')
            self.p.stdin.flush()
            self.p.wait(timeout=10)
        except Exception:
            self.p.kill()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", action="append", required=True, help="preset / path (repeatable)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--port", type=int, default=8080, help="ingress port")
    ap.add_argument("engine_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    engines, procs = {}, []
    for m in a.model:
        port = free_port()
        name = os.path.basename(m).replace(".gguf", "")
        cmd = [sys.executable, "-m", "hipserve.server", "--model", m, "--served-model-name", name,
               "--host", "127.0.0.1", "--port", str(port)] + (["--device", a.device] if a.device else []) \
            + a.engine_args
        procs.append(subprocess.Popen(cmd, env=env))
        engines[name] = [port]
    for (name, ports), p in zip(engines.items(), procs):
        wait_http(f"http://127.0.0.1:{ports[0]}/health", 1800, p)
    st = GatewayStack(engines)
    st.ingress_port = a.port
    st.start()
    print(f"stack ready: {st.url}  models={list(engines)}", flush=True)
    try:
        while all(p.poll() is None for p in procs):
            time.sleep(1)
    except KeyboardInterrupt:
        pass
    finally:
        st.stop()
        for p in procs:
            p.terminate()


if __name__ == "__main__":
    main()
