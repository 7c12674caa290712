"""Process logging setup for the engine and the gateway (SURVEY.md §5 observability:
"router access logs with upstream + latency; JSON logs").

``text`` (default): ``time LEVEL logger: message``. ``json``: one JSON object per line —
``ts`` (RFC 3339, UTC), ``level``, ``logger``, ``msg``, plus ``rank`` under tensor
parallelism and ``exc`` for exceptions — the shape cluster log collectors (Fluent Bit,
Vector, Loki) parse without a per-service regex. Chosen by ``--log-format`` or
``HIPSERVE_LOG_FORMAT``.
"""
from __future__ import annotations

import datetime
import json
import logging
import os

FORMATS = ("text", "json")


class JsonFormatter(logging.Formatter):
    def __init__(self, rank: int | None = None):
        super().__init__()
        self.rank = rank

    def format(self, record: logging.LogRecord) -> str:
        ts = datetime.datetime.fromtimestamp(record.created, tz=datetime.timezone.utc)
        out = {"ts": ts.isoformat(timespec="milliseconds").replace("+00:00", "Z"), "level": record.levelname,
               "logger": record.name, "msg": record.getMessage()}
        if self.rank is not None:
            out["rank"] = self.rank
        if record.exc_info:
            out["exc"] = self.formatException(record.exc_info)
        return json.dumps(out, ensure_ascii=False)


def setup_logging(level: str = "INFO", fmt: str | None = None) -> None:
    """Configure the root logger once per process (replaces any handler set before)."""
    fmt = (fmt or os.environ.get("HIPSERVE_LOG_FORMAT", "text")).lower()
    if fmt not in FORMATS:
        raise ValueError(f"log format must be one of {FORMATS}, got {fmt!r}")
    handler = logging.StreamHandler()
    if fmt == "json":
        rank = os.environ.get("RANK")
        handler.setFormatter(JsonFormatter(int(rank) if rank is not None and rank.isdigit() else None))
    else:
        handler.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    root.addHandler(handler)
    root.setLevel(level.upper())
