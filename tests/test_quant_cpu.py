"""GGUF prefill routing on the CPU (no GPU needed): which prefill path a quantised
weight takes (hipserve/ops/quant.py qprefill_ok: prefill-sized batches on device
tensors without a bf16 shadow, GLU only over one format, the start-up timing in
``auto``)."""
import numpy as np
import pytest
import torch

from hipserve.ops import quant as Q
from hipserve.weights import gguf as G


@pytest.fixture(scope="module", autouse=True)
def lib():
    try:  # the gfx950 library loads without a GPU (op registration only)
        from hipserve.ops import load_library
        load_library()
    except Exception:
        pass


def _qw(qts, N=64, K=256):
    rng = np.random.default_rng(0)
    return Q.QuantWeight.from_raw([(qt, N, K, Q.random_blocks(rng, qt, N, K)) for qt in qts], "cpu")


def test_qprefill_not_taken_on_cpu_tensors():
    w = _qw([G.Q4_K])
    assert not Q.qprefill_ok(w, 1024)
    assert not Q.qprefill_ok(w, 1024, glu=True)


def test_qprefill_needs_prefill_rows_and_no_shadow(monkeypatch):
    w = _qw([G.Q4_K, G.Q4_K])
    monkeypatch.setattr(torch.Tensor, "is_cuda", property(lambda self: True))  # routing only
    monkeypatch.setattr(Q, "QPREFILL_MODE", "1")
    if not hasattr(torch.ops.hipserve, "gguf_prefill"):
        return  # extension not built in this environment: the predicate is False by design
    assert not Q.qprefill_ok(w, Q.MAX_FUSED_M)          # decode-sized batch
    assert Q.qprefill_ok(w, Q.MAX_FUSED_M + 1)
    assert Q.qprefill_ok(w, 4096, glu=True)              # two parts of one format and size
    w3 = _qw([G.Q4_K, G.Q6_K])
    assert not Q.qprefill_ok(w3, 4096, glu=True)          # GLU over two formats
    w.dense = torch.empty(0)
    assert not Q.qprefill_ok(w, 4096)                     # a resident bf16 shadow wins


def test_qprefill_auto_follows_start_up_timing(monkeypatch):
    w = _qw([G.Q4_K])
    monkeypatch.setattr(torch.Tensor, "is_cuda", property(lambda self: True))
    if not hasattr(torch.ops.hipserve, "gguf_prefill"):
        return
    monkeypatch.setattr(Q, "QPREFILL_MODE", "auto")
    monkeypatch.setattr(Q, "QPF_CHOICE", {Q._sig(w): False})
    assert not Q.qprefill_ok(w, 4096)                     # timed slower than dequant + hipBLASLt
    assert Q.qprefill_ok(w, 4096, timed=False)
    monkeypatch.setattr(Q, "QPF_CHOICE", {})
    assert Q.qprefill_ok(w, 4096)                         # untimed shapes take the block kernel
    monkeypatch.setattr(Q, "QPREFILL", False)
    assert not Q.qprefill_ok(w, 4096, timed=False)        # HIPSERVE_QPREFILL=0
