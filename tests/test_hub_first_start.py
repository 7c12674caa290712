"""First start of an HF-tier pod on an empty PVC: ``--model
<huggingfaceId>`` must download into ``HF_HOME`` BEFORE the model config and the
tokenizer are resolved (reference golden path:
vllm-models/helm-chart/templates/model-deployments.yaml:27-28,45-47,64-70), for
ids that are not presets and for ids that happen to match one, with exactly one
download per TP pod. The Hub client is replaced by tests/fake_hub.py (no network)."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from hipserve.config import EngineConfig
from hipserve.engine.request import SamplingParams

REPOS = {"acme/tiny-chat": "tiny-llama", "meta-llama/Meta-Llama-3-8B": "tiny-llama"}
SP = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
PROMPTS = [[1, 5, 9, 33], list(range(3, 40))]


@pytest.fixture
def hub(tmp_path, monkeypatch):
    log = tmp_path / "downloads.log"
    log.write_text("")
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hf"))
    monkeypatch.setenv("FAKE_HUB_REPOS", json.dumps(REPOS))
    monkeypatch.setenv("FAKE_HUB_LOG", str(log))
    monkeypatch.setenv("HIPSERVE_SNAPSHOT_DOWNLOAD", "tests.fake_hub:snapshot_download")
    return log


def _cfg(model, tp=1, **kw):
    return EngineConfig(model=model, device="cpu", dtype="float32", num_kv_blocks=128, max_model_len=256,
                        max_num_batched_tokens=64, max_num_seqs=4, tensor_parallel_size=tp, **kw)


def _engine(model, **kw):
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.parallel.comm import TPGroup

    return LLMEngine(_cfg(model, **kw), tp=TPGroup())


def test_first_start_non_preset_id(hub):
    from hipserve.tokenizer import HFTokenizer

    eng = _engine("acme/tiny-chat")
    assert isinstance(eng.tokenizer, HFTokenizer)
    assert eng.model_cfg.hidden_size == 128 and eng.runner.load_format == "safetensors"
    assert eng.cfg.model_name == "acme/tiny-chat"  # served under the Hub id, not the snapshot path
    out = eng.generate(PROMPTS, SP)
    assert all(len(r[0]) == 6 for r in out)
    assert len(hub.read_text().splitlines()) == 1
    _engine("acme/tiny-chat")  # pod restart: the PVC cache is reused, no second download
    assert len(hub.read_text().splitlines()) == 1


def test_first_start_preset_matching_id(hub):
    """An id that matches a preset must still be downloaded first: its config and
    tokenizer come from the checkpoint (here: tiny shapes), not the preset and
    not the synthetic byte tokenizer."""
    from hipserve.tokenizer import HFTokenizer

    eng = _engine("meta-llama/Meta-Llama-3-8B")
    assert isinstance(eng.tokenizer, HFTokenizer)
    assert eng.model_cfg.hidden_size == 128 and eng.model_cfg.vocab_size == 512
    assert eng.tokenizer.encode("t7 t9", add_special_tokens=False) == [7, 9]
    assert len(hub.read_text().splitlines()) == 1


def test_dummy_load_format_fetches_config_only(hub):
    eng = _engine("acme/tiny-chat", load_format="dummy")
    assert eng.model_cfg.hidden_size == 128
    line = hub.read_text().splitlines()[0]
    assert "*.safetensors" not in line


def test_offline_fallbacks(hub, monkeypatch):
    """a failed download of a real model is fatal — no silent
    random weights under the Hub id. The preset fallback is opt-in (dummy load
    format or HIPSERVE_HUB_DUMMY_FALLBACK=1) and never serves under the Hub id."""
    monkeypatch.setenv("FAKE_HUB_REPOS", "{}")  # every download fails (air-gapped box)
    with pytest.raises(FileNotFoundError, match="HIPSERVE_HUB_DUMMY_FALLBACK"):
        _engine("acme/tiny-llama")  # maps to the tiny-llama preset, but no opt-in
    with pytest.raises(FileNotFoundError):
        _engine("acme/not-a-preset")
    eng = _engine("acme/tiny-llama", load_format="dummy")
    assert eng.runner.load_format == "dummy" and eng.cfg.model_name == "tiny-llama-random"
    monkeypatch.setenv("HIPSERVE_HUB_DUMMY_FALLBACK", "1")
    eng = _engine("acme/tiny-llama", served_model_name="chat")
    assert eng.runner.load_format == "dummy" and eng.cfg.model_name == "chat"
    with pytest.raises(FileNotFoundError):
        _engine("acme/not-a-preset")


def test_interrupted_download_resumes(hub, monkeypatch):
    """a pod killed mid-download leaves a partial snapshot (config +
    index + some shards). The restart must see it as incomplete, resume the
    download and serve — not crash-loop on the missing shard."""
    from hipserve.weights.hub import cached_snapshot, snapshot_problem

    monkeypatch.setenv("FAKE_HUB_SHARDS", "3")
    monkeypatch.setenv("FAKE_HUB_INTERRUPT", "1")
    with pytest.raises(FileNotFoundError, match="connection reset"):
        _engine("acme/tiny-chat")
    from hipserve.config import _hf_cache_dir

    snap = _hf_cache_dir("acme/tiny-chat")
    assert snap and "missing shard" in snapshot_problem(snap, True)
    assert cached_snapshot("acme/tiny-chat", True) is None
    monkeypatch.delenv("FAKE_HUB_INTERRUPT")
    eng = _engine("acme/tiny-chat")  # restart: resumes, then serves
    assert len(hub.read_text().splitlines()) == 2
    assert snapshot_problem(snap, True) is None
    got = [r[0] for r in eng.generate(PROMPTS, SP)]
    want = [r[0] for r in _engine(snap, served_model_name="x").generate(PROMPTS, SP)]
    assert got == want
    _engine("acme/tiny-chat")  # complete now: no third download
    assert len(hub.read_text().splitlines()) == 2


def test_truncated_shard_is_redownloaded(hub, monkeypatch):
    from hipserve.config import _hf_cache_dir
    from hipserve.weights.hub import snapshot_problem

    monkeypatch.setenv("FAKE_HUB_SHARDS", "2")
    _engine("acme/tiny-chat")
    snap = _hf_cache_dir("acme/tiny-chat")
    shard = os.path.join(snap, "model-00002-of-00002.safetensors")
    with open(shard, "r+b") as f:
        f.truncate(os.path.getsize(shard) - 100)
    assert "truncated" in snapshot_problem(snap, True)
    # the client skips files already in the snapshot (tests/fake_hub.py, like the real
    # one): the engine must drop the truncated shard itself before re-downloading
    _engine("acme/tiny-chat")
    assert len(hub.read_text().splitlines()) == 2 and snapshot_problem(snap, True) is None


def test_snapshot_follows_refs_main(tmp_path, monkeypatch):
    from hipserve.config import _hf_cache_dir

    monkeypatch.setenv("HF_HOME", str(tmp_path))
    repo = tmp_path / "hub" / "models--acme--x"
    for rev in ("aaaa", "ffff"):
        (repo / "snapshots" / rev).mkdir(parents=True)
        (repo / "snapshots" / rev / "config.json").write_text("{}")
    (repo / "refs").mkdir()
    (repo / "refs" / "main").write_text("ffff\n")
    assert _hf_cache_dir("acme/x").endswith("ffff")
    (repo / "refs" / "main").write_text("aaaa")
    assert _hf_cache_dir("acme/x").endswith("aaaa")
    (repo / "refs" / "main").write_text("gone")  # dangling ref: newest snapshot
    os.utime(repo / "snapshots" / "aaaa", (1, 1))
    assert _hf_cache_dir("acme/x").endswith("ffff")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, env, q):
    os.environ.update(env, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist

    from hipserve.engine.llm_engine import LLMEngine, prepare_model, worker_loop
    from hipserve.engine.model_runner import ModelRunner
    from hipserve.parallel.comm import init_tp

    tp = init_tp(world, backend="gloo", device_type="cpu")
    cfg = _cfg("acme/tiny-chat", tp=world)
    try:
        if rank == 0:
            eng = LLMEngine(cfg, tp=tp)
            res = eng.generate(PROMPTS, SP)
            eng.shutdown()
            q.put([r[0] for r in res])
        else:
            wcfg, mcfg, _ = prepare_model(cfg, tp)
            worker_loop(ModelRunner(wcfg, mcfg, tp), tp)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)


@pytest.mark.parametrize("slow", [False, True])
def test_first_start_tp2_downloads_once(hub, monkeypatch, slow):
    """slow: the download outlasts the process groups' collective timeout (8 s
    here; a 140 GB 70B first download vs the 600 s default) — the non-zero rank
    polls rank 0's status file instead of sitting in one bounded barrier."""
    if slow:
        monkeypatch.setenv("HIPSERVE_DIST_TIMEOUT_S", "8")
        monkeypatch.setenv("FAKE_HUB_DELAY", "14")
        monkeypatch.setenv("FAKE_HUB_SHARDS", "2")
    keys = ("HF_HOME", "FAKE_HUB_REPOS", "FAKE_HUB_LOG", "HIPSERVE_SNAPSHOT_DOWNLOAD", "HIPSERVE_DIST_TIMEOUT_S",
            "FAKE_HUB_DELAY", "FAKE_HUB_SHARDS")
    env = {k: os.environ[k] for k in keys if k in os.environ}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, env, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=240)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert len(hub.read_text().splitlines()) == 1  # rank 0 downloaded, rank 1 waited
    monkeypatch.delenv("FAKE_HUB_DELAY", raising=False)
    want = [r[0] for r in _engine("acme/tiny-chat").generate(PROMPTS, SP)]
    assert got == want
    assert len(hub.read_text().splitlines()) == 1  # the cache was complete: no second download
