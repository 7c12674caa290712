"""First start of a model pod: populate the PVC-backed Hugging Face cache BEFORE
anything reads the model's config or tokenizer.

The reference's golden path is ``--model <huggingfaceId>``: the engine downloads
the checkpoint into the per-model PVC mounted at ``/root/.cache/huggingface`` and
later restarts reuse it
(vllm-models/helm-chart/templates/model-deployments.yaml:27-28,45-47,64-70;
vllm-models/README.md:13-15,203). ``materialize`` turns such an id into a local
snapshot directory:

* local directories, ``.gguf`` files and preset names pass through unchanged;
* the snapshot is the one ``refs/main`` names (the revision the Hub client last
  resolved), not whichever directory sorts first;
* a snapshot is used offline only when it is COMPLETE: config.json plus every
  shard that ``model.safetensors.index.json`` lists (or, without an index, every
  ``*.safetensors`` present), each with an intact header and all the bytes its
  header promises. A pod killed half-way through the first download (liveness,
  OOM, node drain) therefore re-enters the download on restart — the Hub client
  resumes and skips what is there — instead of crash-looping on a missing shard;
* otherwise TP rank 0 downloads (token from ``HUGGING_FACE_HUB_TOKEN`` /
  ``HF_TOKEN``) and publishes its progress in a status file next to the cache;
  the other ranks of the pod poll that file (no bounded collective: a 140 GB 70B
  first download may take longer than any process-group timeout);
* ``--load-format dummy`` fetches only the JSON configs + tokenizer, and may fall
  back to a built-in preset's architecture (random weights) when even that
  fails. Without ``dummy`` a failed download is fatal (the pod crash-loops, like
  vLLM) unless ``HIPSERVE_HUB_DUMMY_FALLBACK=1`` opts in — a pod must never
  answer under a real model's name with random weights by accident; under the
  fallback the model is served as ``<preset>-random``, never as the Hub id.

``HIPSERVE_SNAPSHOT_DOWNLOAD=module:function`` replaces
``huggingface_hub.snapshot_download`` (an internal mirror, or the tests).
"""
from __future__ import annotations

import glob
import importlib
import json
import logging
import os
import struct
import time
import uuid

log = logging.getLogger("hipserve.hub")

WEIGHT_PATTERNS = ["*.json", "*.safetensors", "tokenizer*", "*.model", "*.tiktoken", "*.txt"]
CONFIG_PATTERNS = ["*.json", "tokenizer*", "*.model", "*.tiktoken"]
INDEX = "model.safetensors.index.json"


class DummyFallback(str):
    """A preset name returned instead of a snapshot path: the caller serves the
    preset architecture with random weights under ``served_name``."""

    served_name: str


def is_hub_id(model: str) -> bool:
    return ("/" in model and not os.path.exists(model) and not model.endswith(".gguf")
            and not model.startswith((".", "/", "~")) and model.count("/") == 1)


def _downloader():
    spec = os.environ.get("HIPSERVE_SNAPSHOT_DOWNLOAD")
    if spec:
        mod, _, fn = spec.partition(":")
        return getattr(importlib.import_module(mod), fn)
    from huggingface_hub import snapshot_download

    return snapshot_download


def _token():
    return os.environ.get("HUGGING_FACE_HUB_TOKEN") or os.environ.get("HF_TOKEN") or None


def safetensors_intact(path: str) -> bool:
    """True if ``path`` is a whole safetensors file: an 8-byte header length, a JSON
    header, and at least as many data bytes as the largest tensor offset needs."""
    try:
        size = os.path.getsize(path)
        if size < 8:
            return False
        with open(path, "rb") as f:
            (n,) = struct.unpack("<Q", f.read(8))
            if n > size - 8 or n > (100 << 20):
                return False
            head = json.loads(f.read(n))
        end = max((int(v["data_offsets"][1]) for k, v in head.items()
                   if k != "__metadata__" and isinstance(v, dict) and "data_offsets" in v), default=0)
        return 8 + n + end <= size
    except (OSError, ValueError, KeyError, TypeError, struct.error):
        return False


def weight_files(d: str) -> list[str]:
    """Shard paths of a snapshot: the index's weight_map when there is one (missing
    shards included, so a caller can tell), else the ``*.safetensors`` present."""
    idx = os.path.join(d, INDEX)
    if os.path.exists(idx):
        with open(idx) as f:
            wm = json.load(f).get("weight_map", {})
        return [os.path.join(d, s) for s in sorted(set(wm.values()))]
    return sorted(glob.glob(os.path.join(d, "*.safetensors")))


def snapshot_problem(d: str | None, need_weights: bool) -> str | None:
    """Why snapshot ``d`` cannot be served offline, or None when it is complete."""
    if not d or not os.path.exists(os.path.join(d, "config.json")):
        return "no config.json"
    if not need_weights:
        return None
    try:
        files = weight_files(d)
    except (OSError, ValueError) as e:
        return f"unreadable {INDEX}: {e}"
    if not files:
        return "no *.safetensors"
    for f in files:
        if not os.path.exists(f):
            return f"missing shard {os.path.basename(f)}"
        if not safetensors_intact(f):
            return f"truncated shard {os.path.basename(f)}"
    return None


def cached_snapshot(model: str, need_weights: bool) -> str | None:
    from ..config import _hf_cache_dir

    d = _hf_cache_dir(model)
    return d if snapshot_problem(d, need_weights) is None else None


def drop_truncated(d: str | None) -> list[str]:
    """Delete the truncated shards of snapshot ``d`` (and, for the Hub cache's
    symlinks, the blob each points to) so the next download fetches them again: the
    Hub client skips a file that already exists in the snapshot, truncated or not, so
    leaving it would turn a killed download into a permanent crash loop."""
    gone = []
    if not d or not os.path.isdir(d):
        return gone
    try:
        files = weight_files(d)
    except (OSError, ValueError):
        return gone
    for f in files:
        if os.path.lexists(f) and not safetensors_intact(f):
            if os.path.islink(f):
                blob = os.path.realpath(f)
                if os.path.exists(blob):
                    os.remove(blob)
            os.remove(f)
            gone.append(os.path.basename(f))
    if gone:
        log.warning("re-downloading truncated shards: %s", ", ".join(gone))
    return gone


def download(model: str, need_weights: bool) -> str:
    from ..config import _hf_cache_dir

    fn = _downloader()
    patterns = WEIGHT_PATTERNS if need_weights else CONFIG_PATTERNS
    if need_weights:
        drop_truncated(_hf_cache_dir(model))
    log.info("downloading %s from the Hugging Face Hub (%s)", model, "weights" if need_weights else "config")
    path = fn(model, allow_patterns=patterns, token=_token())
    why = snapshot_problem(path, need_weights)
    if why is not None:
        raise RuntimeError(f"download of {model} finished incomplete: {why}")
    return path


def _status_path(nonce: str) -> str:
    home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    d = os.path.join(home, "hub")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f".hipserve-download-{nonce}.json")


def _write_status(fname: str, **kw):
    tmp = f"{fname}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(dict(kw, t=time.time()), f)
    os.replace(tmp, fname)  # atomic: a poller never reads half a file


def _wait_status(path: str, model: str, timeout: float, poll: float = 1.0) -> dict:
    t0 = last = time.monotonic()
    while True:
        try:
            with open(path) as f:
                st = json.load(f)
            if st.get("state") in ("done", "failed"):
                return st
        except (OSError, ValueError):
            pass
        now = time.monotonic()
        if now - t0 > timeout:
            return {"state": "failed", "error": f"rank 0 did not finish downloading {model} in {timeout:.0f} s"}
        if now - last > 60:
            log.info("waiting for rank 0 to download %s (%.0f s)", model, now - t0)
            last = now
        time.sleep(poll)


def _fallback(model: str, load_format: str, served_name: str | None, err) -> str:
    from ..config import PRESETS, preset_key

    key = preset_key(model)
    allowed = load_format == "dummy" or os.environ.get("HIPSERVE_HUB_DUMMY_FALLBACK", "0") == "1"
    if key in PRESETS and allowed:
        out = DummyFallback(key)
        out.served_name = served_name or f"{key}-random"
        log.warning("%s: not in the cache and not downloadable (%s); serving the %s architecture with "
                    "RANDOM weights as %r", model, err, key, out.served_name)
        return out
    hint = " (HIPSERVE_HUB_DUMMY_FALLBACK=1 or --load-format dummy serves the preset with random weights)" \
        if key in PRESETS else ""
    raise FileNotFoundError(f"model {model!r}: not in the Hugging Face cache and the download failed: {err}{hint}")


def materialize(model: str, load_format: str = "auto", tp=None, served_name: str | None = None) -> str:
    """Local path (or preset name) for ``model``; collective over ``tp`` (every
    rank of the pod calls it with the same arguments)."""
    if not is_hub_id(model):
        return model
    need_weights = load_format not in ("dummy",)
    rank = tp.rank if tp is not None else 0
    world = tp.world_size if tp is not None else 1
    timeout = float(os.environ.get("HIPSERVE_DOWNLOAD_TIMEOUT_S", 24 * 3600))
    path, err = None, None
    if rank == 0:
        from ..config import _hf_cache_dir

        why = snapshot_problem(_hf_cache_dir(model), need_weights)
        if why is None:
            path = _hf_cache_dir(model)
            msg = ("ok", path)
        else:
            log.info("%s: cached snapshot unusable (%s)", model, why)
            msg = ("downloading", uuid.uuid4().hex[:16])
    else:
        msg = None
    if world > 1:
        msg = tp.broadcast_obj(msg)  # immediate: rank 0 has not started downloading yet
    if msg[0] == "ok":
        path = msg[1]
    elif rank == 0:
        status = _status_path(msg[1]) if world > 1 else None
        if status:
            _write_status(status, state="downloading", model=model)
        try:
            path = download(model, need_weights)
        except Exception as e:  # no network / unknown repo / auth / incomplete
            err = e
        if status:
            _write_status(status, state="done" if path else "failed", path=path, error=str(err) if err else None)
    else:
        st = _wait_status(_status_path(msg[1]), model, timeout)
        path = st.get("path") if st["state"] == "done" else None
        err = st.get("error")
    if world > 1:
        tp.barrier()  # everyone has the answer; rank 0 may delete the status file
        if rank == 0 and msg[0] == "downloading":
            try:
                os.remove(_status_path(msg[1]))
            except OSError:
                pass
    if path is not None:
        return path
    return _fallback(model, load_format, served_name, err or "download failed on rank 0")
