"""A stand-in for ``huggingface_hub.snapshot_download`` (no network here): plugged
in through ``HIPSERVE_SNAPSHOT_DOWNLOAD=tests.fake_hub:snapshot_download``.

``FAKE_HUB_REPOS`` maps repo ids to the preset whose shapes the fake checkpoint
gets; every call is appended to ``FAKE_HUB_LOG`` (one line per download, from any
process) and the snapshot is written where the real client puts it:
``$HF_HOME/hub/models--<org>--<name>/snapshots/<rev>/`` plus ``refs/main``.

Failure modes of a real first start, for the cache-hardening tests:
* ``FAKE_HUB_SHARDS=n``: write n shards + ``model.safetensors.index.json``;
* ``FAKE_HUB_INTERRUPT=k``: die (raise) after writing k shards — the pod killed
  mid-download; like the real client, a later call resumes (skips shards that
  are already in the snapshot — complete or not) and finishes;
* ``FAKE_HUB_DELAY=s``: the download takes s seconds (slower than a collective
  timeout)."""
import fnmatch
import json
import os
import time


def _tokenizer(path, vocab_size):
    from tokenizers import Tokenizer, models, pre_tokenizers

    vocab = {f"t{i}": i for i in range(vocab_size)}
    vocab["<s>"], vocab["</s>"], vocab["<unk>"] = 1, 2, 0
    tk = Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tk.save(os.path.join(path, "tokenizer.json"))
    with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<s>", "eos_token": "</s>", "add_bos_token": True,
                   "chat_template": "{% for m in messages %}{{ m['content'] }} {% endfor %}"}, f)


def _sharded(snap, cfg, tensors, n, interrupt):
    """n shards + index; stop (raise) after ``interrupt`` newly written shards."""
    from safetensors.torch import save_file

    from hipserve.weights.hub import safetensors_intact
    from hipserve.weights.safetensors_loader import save_hf_checkpoint

    save_hf_checkpoint(snap, cfg, {})  # config.json (and an empty model.safetensors)
    os.remove(os.path.join(snap, "model.safetensors"))
    names = sorted(tensors)
    parts = [names[i::n] for i in range(n)]
    files = [f"model-{i + 1:05d}-of-{n:05d}.safetensors" for i in range(n)]
    with open(os.path.join(snap, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {}, "weight_map": {k: files[i] for i, p in enumerate(parts) for k in p}}, f)
    wrote = 0
    for fn, p in zip(files, parts):
        path = os.path.join(snap, fn)
        if os.path.exists(path):
            continue  # like the real client: a file already in the snapshot is not re-fetched
        if interrupt is not None and wrote >= interrupt:
            raise RuntimeError("connection reset (pod killed mid-download)")
        save_file({k: tensors[k].contiguous() for k in p}, path)
        wrote += 1


def snapshot_download(repo_id, allow_patterns=None, token=None, **kw):
    repos = json.loads(os.environ["FAKE_HUB_REPOS"])
    if repo_id not in repos:
        raise RuntimeError(f"404: {repo_id}")
    with open(os.environ["FAKE_HUB_LOG"], "a") as f:
        f.write(f"{os.getpid()} {repo_id} {','.join(allow_patterns or [])}\n")
    time.sleep(float(os.environ.get("FAKE_HUB_DELAY", "0")))
    from hipserve.config import PRESETS
    from hipserve.weights.safetensors_loader import random_hf_tensors, save_hf_checkpoint

    cfg = PRESETS[repos[repo_id]]
    home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    repo = os.path.join(home, "hub", "models--" + repo_id.replace("/", "--"))
    rev = "0123abcd"
    snap = os.path.join(repo, "snapshots", rev)
    os.makedirs(os.path.join(repo, "refs"), exist_ok=True)
    with open(os.path.join(repo, "refs", "main"), "w") as f:
        f.write(rev)
    weights = not allow_patterns or any(fnmatch.fnmatch("model.safetensors", p) for p in allow_patterns)
    nshards = int(os.environ.get("FAKE_HUB_SHARDS", "0"))
    if weights and nshards:
        os.makedirs(snap, exist_ok=True)
        _tokenizer(snap, cfg.vocab_size)
        intr = os.environ.get("FAKE_HUB_INTERRUPT")
        _sharded(snap, cfg, random_hf_tensors(cfg, seed=5), nshards, int(intr) if intr else None)
        return snap
    save_hf_checkpoint(snap, cfg, random_hf_tensors(cfg, seed=5))
    if not weights:
        os.remove(os.path.join(snap, "model.safetensors"))
    _tokenizer(snap, cfg.vocab_size)
    return snap
