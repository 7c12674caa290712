"""Start-up tuning tables persisted per (device, kernel build).

The engine times its decode GEMM configs (ops/gemm.py GemmTuner), the quantised decode
split-K factors (ops/quant.py tune_splits), the packed-vs-hipBLASLt prefill units
(ops/pgemm.py tune_packed) and the prefill row padding (engine/model_runner.py) at every
start: ~10 s for Llama-3-8B, ~17 s for Llama-3-70B at TP=1 — inside the 150 s start-up
budget of a TP=8 pod (the reference's startup probe window,
/root/reference/vllm-models/helm-chart/templates/model-deployments.yaml:37-38) it is the
largest item after the weights. The results depend only on the device and on the
kernels, so they are stored in one JSON file per fingerprint:

    $HIPSERVE_TUNE_CACHE/<fingerprint>.json     (default ~/.cache/hipserve/tune)

fingerprint = sha1(device capability, CU count, HBM GiB, torch version, hipserve/_C.so bytes,
the kernel-choice knobs of ``TUNING_KNOBS`` that are set): a new GPU model, a driver-visible
CU count change, a rebuilt kernel library or a start with other knob values re-tunes.
``HIPSERVE_TUNE_CACHE=0`` disables the cache (every start times everything); deleting the
directory (or one ``<fingerprint>.json``) invalidates it. The charts put it on the model
volume so a restarted pod skips the timing (deploy/charts/*/templates/model-deployments.yaml). Writers
merge with the file on disk and replace it atomically, so TP ranks sharing a volume
never leave a torn table behind.
"""
from __future__ import annotations

import hashlib
import json
import logging
import os

import torch

log = logging.getLogger("hipserve.tune_cache")

_STATE: dict = {}  # fingerprint -> {kind: {key: value}}
_DIRTY: set = set()


def cache_dir() -> str | None:
    d = os.environ.get("HIPSERVE_TUNE_CACHE", os.path.join(os.path.expanduser("~"), ".cache", "hipserve", "tune"))
    return None if d in ("", "0") else d


def _lib_digest() -> str:
    from . import library_path  # the kernel library
    p = library_path()
    h = hashlib.sha1()
    if p and os.path.exists(p):
        with open(p, "rb") as f:
            for blk in iter(lambda: f.read(1 << 22), b""):
                h.update(blk)
    return h.hexdigest()


_FP: dict = {}

# knobs that change a tuner's candidate set or the kernels a timed unit runs: a start
# with other values must not reuse tables timed under these (docs/ENV.md)
TUNING_KNOBS = ("HIPSERVE_FP8_DECODE", "HIPSERVE_FP8_PREFILL", "HIPSERVE_FP8_PREFILL_LIB",
                "HIPSERVE_FUSED_DECODE", "HIPSERVE_FUSED_QKV_ATTN", "HIPSERVE_MOE_PACK",
                "HIPSERVE_MOE_PACKED_PREFILL", "HIPSERVE_PW_GRID", "HIPSERVE_PW_RW", "HIPSERVE_PW_WM",
                "HIPSERVE_QGEMM_X16", "HIPSERVE_QPREFILL", "HIPSERVE_QPREFILL_MAX_M",
                "HIPSERVE_QUANT_SHADOW", "HIPSERVE_SINGLE_LAYOUT")


def knob_values() -> dict:
    return {k: os.environ[k] for k in TUNING_KNOBS if k in os.environ}


def fingerprint(device) -> str:
    idx = torch.device(device).index or 0
    knobs = knob_values()
    key = (idx, json.dumps(knobs, sort_keys=True))
    fp = _FP.get(key)
    if fp is None:
        # not the marketing name: it reads "" under rocprofv3, which would make profiled
        # runs miss the tables of unprofiled ones (and re-tune with tracing overhead)
        pr = torch.cuda.get_device_properties(idx)
        ident = [list(torch.cuda.get_device_capability(idx)), pr.multi_processor_count,
                 round(pr.total_memory / 2**30), torch.__version__, _lib_digest()]
        if knobs:  # default settings keep the knob-free fingerprint of earlier tables
            ident.append(sorted(knobs.items()))
        fp = _FP[key] = hashlib.sha1(json.dumps(ident).encode()).hexdigest()[:16]
    return fp


def _path(fp: str) -> str | None:
    d = cache_dir()
    return os.path.join(d, fp + ".json") if d else None


def _table(fp: str) -> dict:
    t = _STATE.get(fp)
    if t is None:
        t = {}
        p = _path(fp)
        if p and os.path.exists(p):
            try:
                with open(p) as f:
                    t = json.load(f)
            except (OSError, ValueError) as e:
                log.warning("tuning cache %s unreadable (%s): re-tuning", p, e)
                t = {}
        _STATE[fp] = t
    return t


def _key(key) -> str:
    return json.dumps(key, separators=(",", ":"))


def tup(v):
    """JSON lists back to the tuples the tuners key and compare on."""
    return tuple(tup(x) for x in v) if isinstance(v, list) else v


def get(device, kind: str, key):
    """The stored value for (kind, key) on this device / kernel build, or None."""
    if cache_dir() is None or not torch.cuda.is_available():
        return None
    return _table(fingerprint(device)).get(kind, {}).get(_key(key))


def put(device, kind: str, key, value) -> None:
    if cache_dir() is None or not torch.cuda.is_available():
        return
    fp = fingerprint(device)
    _table(fp).setdefault(kind, {})[_key(key)] = value
    _DIRTY.add(fp)


def flush() -> None:
    """Write the tables changed since the last flush (merged with what other processes
    wrote meanwhile; atomic replace). A read-only cache directory only logs."""
    for fp in list(_DIRTY):
        p = _path(fp)
        _DIRTY.discard(fp)
        if p is None:
            continue
        try:
            os.makedirs(os.path.dirname(p), exist_ok=True)
            merged = {}
            if os.path.exists(p):
                try:
                    with open(p) as f:
                        merged = json.load(f)
                except (OSError, ValueError):
                    merged = {}
            for kind, rows in _STATE[fp].items():
                merged.setdefault(kind, {}).update(rows)
            tmp = f"{p}.tmp{os.getpid()}"
            with open(tmp, "w") as f:
                json.dump(merged, f)
            os.replace(tmp, p)
            _STATE[fp] = merged
        except OSError as e:
            log.warning("could not write tuning cache %s: %s", p, e)
