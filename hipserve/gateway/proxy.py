"""Minimal streaming HTTP/1.1 reverse proxy on raw asyncio streams.

Shared core of the model-name router (``router.py``) and the ingress emulator
(``ingress.py``). Built to fix the reference routers' defects:
  * bodies of any size are read completely (Content-Length or chunked) before
    routing — no 8-16 KiB buffer spill that silently routes to the default model,
    no 1 MiB 413;
  * responses are relayed byte-for-byte as they arrive (SSE token streams are
    never buffered), with no read timeout on long generations;
  * upstream status codes (4xx/5xx) are passed through unchanged — only a
    connection failure becomes 502;
  * concurrent clients (asyncio), keep-alive on the client side, and
    ``SO_REUSEPORT`` so several worker processes can share one port.
"""
from __future__ import annotations

import asyncio
import json
import logging
import socket
import time
from dataclasses import dataclass, field

log = logging.getLogger("hipserve.gateway")
access_log = logging.getLogger("hipserve.access")  # one INFO line per proxied request

_HOP = {b"connection", b"keep-alive", b"proxy-connection", b"te", b"trailer", b"upgrade"}


@dataclass
class Request:
    method: str
    target: str
    version: str
    headers: list[tuple[bytes, bytes]]
    body: bytes
    peer: str = ""

    @property
    def path(self) -> str:
        return self.target.split("?", 1)[0]

    def header(self, name: bytes) -> bytes | None:
        name = name.lower()
        for k, v in self.headers:
            if k.lower() == name:
                return v
        return None

    def json(self):
        try:
            return json.loads(self.body) if self.body else None
        except Exception:
            return None


@dataclass
class Response:
    status: int
    body: bytes
    content_type: str = "application/json"
    headers: list = field(default_factory=list)


_REASONS = {200: "OK", 400: "Bad Request", 404: "Not Found", 413: "Payload Too Large",
            500: "Internal Server Error", 502: "Bad Gateway", 503: "Service Unavailable"}


class BadRequest(Exception):
    pass


async def read_request(reader: asyncio.StreamReader, max_body: int) -> Request | None:
    try:
        head = await reader.readuntil(b"\r\n\r\n")
    except asyncio.IncompleteReadError:
        return None
    except asyncio.LimitOverrunError:
        raise BadRequest("header too large")
    lines = head[:-4].split(b"\r\n")
    try:
        method, target, version = lines[0].decode("latin-1").split(" ", 2)
    except ValueError:
        raise BadRequest("bad request line")
    headers = []
    for ln in lines[1:]:
        if not ln:
            continue
        k, _, v = ln.partition(b":")
        headers.append((k.strip(), v.strip()))
    req = Request(method, target, version, headers, b"")
    te = req.header(b"transfer-encoding")
    if te and b"chunked" in te.lower():
        parts = []
        total = 0
        while True:
            size_line = await reader.readuntil(b"\r\n")
            size = int(size_line.split(b";")[0].strip() or b"0", 16)
            if size == 0:
                # trailers until blank line
                while (await reader.readuntil(b"\r\n")) != b"\r\n":
                    pass
                break
            total += size
            if total > max_body:
                raise BadRequest("body too large")
            parts.append(await reader.readexactly(size))
            await reader.readexactly(2)
        req.body = b"".join(parts)
        req.headers = [(k, v) for k, v in req.headers if k.lower() != b"transfer-encoding"]
    else:
        cl = req.header(b"content-length")
        n = int(cl) if cl else 0
        if n > max_body:
            raise BadRequest("body too large")
        if n:
            req.body = await reader.readexactly(n)
    return req


def _keepalive(req: Request) -> bool:
    c = (req.header(b"connection") or b"").lower()
    if req.version == "HTTP/1.0":
        return c == b"keep-alive"
    return c != b"close"


def render_response(resp: Response, keep_alive: bool) -> bytes:
    hdr = [f"HTTP/1.1 {resp.status} {_REASONS.get(resp.status, 'OK')}",
           f"Content-Type: {resp.content_type}", f"Content-Length: {len(resp.body)}",
           "Connection: keep-alive" if keep_alive else "Connection: close"]
    for k, v in resp.headers:
        hdr.append(f"{k}: {v}")
    return ("\r\n".join(hdr) + "\r\n\r\n").encode() + resp.body


class HTTPProxy:
    """Subclasses implement ``route(req) -> Response | (host, port)``."""

    max_body = 1 << 31
    upstream_connect_timeout = 10.0

    def __init__(self, name: str = "proxy"):
        self.name = name
        self.server: asyncio.AbstractServer | None = None
        self.requests = 0
        self.errors = 0

    async def route(self, req: Request):
        raise NotImplementedError

    async def handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        peer = writer.get_extra_info("peername")
        peer = peer[0] if peer else ""
        sock = writer.get_extra_info("socket")
        if sock is not None:
            try:
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        try:
            while True:
                try:
                    req = await read_request(reader, self.max_body)
                except BadRequest as e:
                    code = 413 if "large" in str(e) else 400
                    writer.write(render_response(Response(code, json.dumps({"error": str(e)}).encode()), False))
                    await writer.drain()
                    return
                if req is None:
                    return
                req.peer = peer
                self.requests += 1
                ka = _keepalive(req)
                dest = await self.route(req)
                if isinstance(dest, Response):
                    writer.write(render_response(dest, ka))
                    await writer.drain()
                else:
                    ok = await self._forward(req, dest, writer, ka)
                    if not ok:
                        return
                if not ka:
                    return
        except (ConnectionResetError, BrokenPipeError, asyncio.IncompleteReadError):
            return
        except Exception:
            log.exception("%s: handler error", self.name)
        finally:
            try:
                writer.close()
            except Exception:
                pass

    async def _forward(self, req: Request, dest, writer: asyncio.StreamWriter, ka: bool) -> bool:
        host, port = dest
        t0 = time.monotonic()
        try:
            ur, uw = await asyncio.wait_for(asyncio.open_connection(host, port, limit=1 << 20),
                                            self.upstream_connect_timeout)
        except Exception as e:
            self.errors += 1
            body = json.dumps({"error": f"upstream {host}:{port} unavailable: {e}"}).encode()
            writer.write(render_response(Response(502, body), ka))
            await writer.drain()
            return True
        us = uw.get_extra_info("socket")
        if us is not None:
            try:
                us.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            except OSError:
                pass
        try:
            lines = [f"{req.method} {req.target} HTTP/1.1".encode()]
            for k, v in req.headers:
                kl = k.lower()
                if kl in _HOP or kl in (b"host", b"content-length"):
                    continue
                lines.append(k + b": " + v)
            lines.append(f"Host: {host}:{port}".encode())
            lines.append(b"Connection: close")
            lines.append(f"Content-Length: {len(req.body)}".encode())
            lines.append(f"X-Forwarded-For: {req.peer}".encode())
            lines.append(b"X-Real-IP: " + req.peer.encode())
            uw.write(b"\r\n".join(lines) + b"\r\n\r\n" + req.body)
            await uw.drain()
            head = await ur.readuntil(b"\r\n\r\n")
            hl = head[:-4].split(b"\r\n")
            status_line = hl[0]
            out = [status_line.replace(b"HTTP/1.0", b"HTTP/1.1", 1)]
            delimited = False
            for ln in hl[1:]:
                k, _, v = ln.partition(b":")
                kl = k.strip().lower()
                if kl in (b"connection", b"keep-alive"):
                    continue
                if kl in (b"content-length",) or (kl == b"transfer-encoding" and b"chunked" in v.lower()):
                    delimited = True
                out.append(ln)
            client_ka = ka and delimited
            out.append(b"Connection: keep-alive" if client_ka else b"Connection: close")
            writer.write(b"\r\n".join(out) + b"\r\n\r\n")
            # relay the body as it arrives (SSE chunks are forwarded immediately);
            # drain after every chunk so a client that went away is noticed at once
            # (asyncio drops writes to a closed transport silently): the upstream
            # connection is then closed, which aborts the generation in the engine
            while True:
                data = await ur.read(1 << 16)
                if not data:
                    break
                if writer.transport.is_closing():
                    raise ConnectionResetError("client disconnected")
                writer.write(data)
                await writer.drain()
            await writer.drain()
            self.on_done(req, dest, time.monotonic() - t0, status_line)
            return client_ka
        except Exception as e:
            self.errors += 1
            log.warning("%s: upstream %s:%s failed: %s", self.name, host, port, e)
            return False
        finally:
            try:
                uw.close()
            except Exception:
                pass

    def on_done(self, req, dest, dt, status_line):
        access_log.info("%s %s %s %s -> %s:%s %s %.1fms", self.name, req.peer, req.method, req.target, dest[0], dest[1],
                  status_line.decode("latin-1"), 1000 * dt)

    async def start(self, host: str, port: int, reuse_port: bool = True):
        self.server = await asyncio.start_server(self.handle, host, port, reuse_port=reuse_port,
                                                 backlog=4096, limit=1 << 20)
        return self.server

    @property
    def port(self) -> int:
        return self.server.sockets[0].getsockname()[1]

    async def stop(self):
        if self.server:
            self.server.close()
            await self.server.wait_closed()
