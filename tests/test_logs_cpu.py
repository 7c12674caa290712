"""JSON / text log formats of the engine and gateway processes (hipserve/utils/logs.py)."""
import io
import json
import logging

import pytest

from hipserve.utils.logs import JsonFormatter, setup_logging


@pytest.fixture(autouse=True)
def _restore_root_logger():
    root = logging.getLogger()
    handlers, level = list(root.handlers), root.level
    yield
    for h in list(root.handlers):
        root.removeHandler(h)
    for h in handlers:
        root.addHandler(h)
    root.setLevel(level)


def _capture(fmt, monkeypatch, rank=None):
    if rank is None:
        monkeypatch.delenv("RANK", raising=False)
    else:
        monkeypatch.setenv("RANK", str(rank))
    setup_logging("INFO", fmt)
    buf = io.StringIO()
    handler = logging.getLogger().handlers[0]
    handler.stream = buf
    return buf


def test_json_lines(monkeypatch):
    buf = _capture("json", monkeypatch, rank=3)
    logging.getLogger("hipserve.test").info("served %d tokens", 42)
    try:
        raise ValueError("boom")
    except ValueError:
        logging.getLogger("hipserve.test").exception("failed")
    lines = [json.loads(x) for x in buf.getvalue().strip().splitlines()]
    assert lines[0]["msg"] == "served 42 tokens" and lines[0]["level"] == "INFO"
    assert lines[0]["logger"] == "hipserve.test" and lines[0]["rank"] == 3
    assert lines[0]["ts"].endswith("Z") and "T" in lines[0]["ts"]
    assert lines[1]["level"] == "ERROR" and "ValueError: boom" in lines[1]["exc"]


def test_text_default_and_env(monkeypatch):
    monkeypatch.setenv("HIPSERVE_LOG_FORMAT", "text")
    buf = _capture(None, monkeypatch)
    logging.getLogger("hipserve.test").warning("plain")
    assert buf.getvalue().rstrip().endswith("WARNING hipserve.test: plain")
    assert not isinstance(logging.getLogger().handlers[0].formatter, JsonFormatter)
    monkeypatch.setenv("HIPSERVE_LOG_FORMAT", "json")
    setup_logging("INFO")
    assert isinstance(logging.getLogger().handlers[0].formatter, JsonFormatter)
    with pytest.raises(ValueError):
        setup_logging("INFO", "xml")
