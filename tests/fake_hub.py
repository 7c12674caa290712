"""A stand-in for ``huggingface_hub.snapshot_download`` (no network here): plugged
in through ``HIPSERVE_SNAPSHOT_DOWNLOAD=tests.fake_hub:snapshot_download``.

``FAKE_HUB_REPOS`` maps repo ids to the preset whose shapes the fake checkpoint
gets; every call is appended to ``FAKE_HUB_LOG`` (one line per download, from any
process) and the snapshot is written where the real client puts it:
``$HF_HOME/hub/models--<org>--<name>/snapshots/<rev>/``."""
import fnmatch
import json
import os


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


def snapshot_download(repo_id, allow_patterns=None, token=None, **kw):
    repos = json.loads(os.environ["FAKE_HUB_REPOS"])
    if repo_id not in repos:
        raise RuntimeError(f"404: {repo_id}")
    with open(os.environ["FAKE_HUB_LOG"], "a") as f:
        f.write(f"{os.getpid()} {repo_id} {','.join(allow_patterns or [])}\n")
    from hipserve.config import PRESETS
    from hipserve.weights.safetensors_loader import random_hf_tensors, save_hf_checkpoint

    cfg = PRESETS[repos[repo_id]]
    home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    snap = os.path.join(home, "hub", "models--" + repo_id.replace("/", "--"), "snapshots", "0123abcd")
    save_hf_checkpoint(snap, cfg, random_hf_tensors(cfg, seed=5))
    if allow_patterns and not any(fnmatch.fnmatch("model.safetensors", p) for p in allow_patterns):
        os.remove(os.path.join(snap, "model.safetensors"))
    _tokenizer(snap, cfg.vocab_size)
    return snap
