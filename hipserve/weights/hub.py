"""First start of a model pod: populate the PVC-backed Hugging Face cache BEFORE
anything reads the model's config or tokenizer.

The reference's golden path is ``--model <huggingfaceId>``: the engine downloads
the checkpoint into the per-model PVC mounted at ``/root/.cache/huggingface`` and
later restarts reuse it
(vllm-models/helm-chart/templates/model-deployments.yaml:27-28,45-47,64-70;
vllm-models/README.md:13-15). ``materialize`` turns such an id into a local
snapshot directory:

* local directories, ``.gguf`` files and preset names pass through unchanged;
* a Hub id already in the cache (complete: config + weights) is used offline;
* otherwise TP rank 0 downloads (token from ``HUGGING_FACE_HUB_TOKEN`` /
  ``HF_TOKEN``) while the other ranks of the pod wait on the CPU group — exactly
  one download per pod; the others then read the same cache;
* ``--load-format dummy`` fetches only the JSON configs + tokenizer;
* an id that matches a built-in preset (``meta-llama/Meta-Llama-3-8B`` ->
  ``llama-3-8b``) and cannot be downloaded (air-gapped box) falls back to the
  preset with random weights, loudly.

``HIPSERVE_SNAPSHOT_DOWNLOAD=module:function`` replaces
``huggingface_hub.snapshot_download`` (an internal mirror, or the tests).
"""
from __future__ import annotations

import glob
import importlib
import logging
import os

log = logging.getLogger("hipserve.hub")

WEIGHT_PATTERNS = ["*.json", "*.safetensors", "tokenizer*", "*.model", "*.tiktoken", "*.txt"]
CONFIG_PATTERNS = ["*.json", "tokenizer*", "*.model", "*.tiktoken"]


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


def cached_snapshot(model: str, need_weights: bool) -> str | None:
    from ..config import _hf_cache_dir

    d = _hf_cache_dir(model)
    if not d or not os.path.exists(os.path.join(d, "config.json")):
        return None
    if need_weights and not glob.glob(os.path.join(d, "*.safetensors")):
        return None
    return d


def download(model: str, need_weights: bool) -> str:
    fn = _downloader()
    patterns = WEIGHT_PATTERNS if need_weights else CONFIG_PATTERNS
    log.info("downloading %s from the Hugging Face Hub (%s)", model, "weights" if need_weights else "config")
    return fn(model, allow_patterns=patterns, token=_token())


def materialize(model: str, load_format: str = "auto", tp=None) -> str:
    """Local path (or preset name) for ``model``; collective over ``tp`` (every
    rank of the pod calls it with the same arguments)."""
    if not is_hub_id(model):
        return model
    need_weights = load_format not in ("dummy",)
    rank = tp.rank if tp is not None else 0
    world = tp.world_size if tp is not None else 1
    path, err = cached_snapshot(model, need_weights), None
    if path is None and rank == 0:
        try:
            path = download(model, need_weights)
        except Exception as e:  # no network / unknown repo / auth
            err = e
    if world > 1:
        tp.barrier()  # the other ranks wait for rank 0's download, then read the cache
        if path is None and rank != 0:
            path = cached_snapshot(model, need_weights)
    if path is not None:
        return path
    from ..config import PRESETS, preset_key

    key = preset_key(model)
    if key in PRESETS:
        log.warning("%s: not in the cache and not downloadable (%s); serving the %s architecture with "
                    "RANDOM weights (--load-format dummy)", model, err or "download failed on rank 0", key)
        return key
    raise FileNotFoundError(f"model {model!r}: not in the Hugging Face cache and the download failed: {err}")
