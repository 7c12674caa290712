"""Persisted start-up tuning tables (hipserve/ops/tune_cache.py): keyed by a device /
kernel-build fingerprint, merged on write, tuples restored on read, disabled by
HIPSERVE_TUNE_CACHE=0. The GPU is faked (no device here): the fingerprint is pinned."""
import json
import os

import pytest
import torch

from hipserve.ops import gemm
from hipserve.ops import tune_cache as TC


@pytest.fixture
def cache(tmp_path, monkeypatch):
    monkeypatch.setenv("HIPSERVE_TUNE_CACHE", str(tmp_path))
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(TC, "fingerprint", lambda device: "fp0")
    TC._STATE.clear()
    TC._DIRTY.clear()
    yield tmp_path
    TC._STATE.clear()
    TC._DIRTY.clear()


def test_roundtrip_and_merge(cache):
    dev = torch.device("cuda", 0)
    assert TC.get(dev, "decode_gemm", [64, 6144, 4096, None]) is None
    TC.put(dev, "decode_gemm", [64, 6144, 4096, None], {"best": ("dgp", 1, 4), "bp": None, "row": {"M": 64}})
    TC.flush()
    # another process added a row meanwhile: a flush merges instead of overwriting
    p = cache / "fp0.json"
    disk = json.loads(p.read_text())
    disk.setdefault("gguf_splits", {})["[1]"] = {"S": 8}
    p.write_text(json.dumps(disk))
    TC.put(dev, "decode_gemm", [64, 4096, 4096, ["norm"]], {"best": "blas", "bp": None, "row": {}})
    TC.flush()
    TC._STATE.clear()  # a fresh process
    h = TC.get(dev, "decode_gemm", [64, 6144, 4096, None])
    assert TC.tup(h["best"]) == ("dgp", 1, 4)
    assert TC.get(dev, "decode_gemm", [64, 4096, 4096, ("norm",)])["best"] == "blas"
    assert TC.get(dev, "gguf_splits", [1]) == {"S": 8}
    assert not [f for f in os.listdir(cache) if ".tmp" in f]


def test_disabled(cache, monkeypatch):
    monkeypatch.setenv("HIPSERVE_TUNE_CACHE", "0")
    dev = torch.device("cuda", 0)
    TC.put(dev, "x", [1], 1)
    TC.flush()
    assert TC.get(dev, "x", [1]) is None and not os.listdir(cache)


def test_gemm_tuner_reuses_cached_shapes(cache, monkeypatch):
    """A shape whose every M bucket is cached is not timed again: the table, the packed
    fallback choice and the report come from the cache."""
    dev = torch.device("cuda", 0)
    for M in (1, 64):
        TC.put(dev, gemm.TC_KIND, [M, 256, 512, None],
               {"best": ["dgp", 3, 2], "bp": [["dgp", 3, 2], 4.5], "row": {"M": M, "N": 256, "K": 512}})
    t = gemm.GemmTuner()

    def boom(*a, **k):
        raise AssertionError("timed a cached shape")
    monkeypatch.setattr(gemm.GemmTuner, "_time", staticmethod(boom))
    rep = t.tune([(256, 512)], dev, ms=[1, 64])
    assert t.table[(64, 256, 512)] == ("dgp", 3, 2) and t.best_packed[(1, 256, 512)] == (("dgp", 3, 2), 4.5)
    assert len(rep) == 2 and all(r["cached"] for r in rep)
    assert (256, 512) in t.packed_shapes()
