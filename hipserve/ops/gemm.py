"""bf16 linear layers: hipBLASLt (``F.linear``) or the hand-written skinny MFMA
GEMM (``csrc/kernels/skinny_gemm.hip``) for decode batches.

The choice is made per (M, N, K) by timing both on the device once, before the
decode hipGraphs are captured (``GemmTuner.tune``); the captured graphs then bake
in the winner. Nothing is dispatched per call at run time except a dict lookup.
"""
from __future__ import annotations

import logging

import torch
import torch.nn.functional as F

log = logging.getLogger("hipserve.gemm")

SKINNY_CONFIGS = [(1, 1), (1, 2), (1, 4), (1, 8), (1, 16), (2, 1), (2, 2), (2, 4), (2, 8)]
# split-K MFMA GEMM with an LDS-staged x chunk shared by 64 rows (gguf.hip, qtype 6 = bf16)
SPLITK_CONFIGS = [1, 2, 4, 8]
_EMPTY = {}
TUNE_MS = [1, 2, 4, 8, 16, 24, 32, 48, 64]


class GemmTuner:
    def __init__(self):
        self.table: dict[tuple, object] = {}
        self.report: list[dict] = []

    def choose(self, M: int, N: int, K: int):
        if M > 64:
            return "blas"
        for m in TUNE_MS:
            if m >= M:
                return self.table.get((m, N, K), "blas")
        return "blas"

    @staticmethod
    def _time(fn, n=16, reps=5):
        """Device time per call inside a hipGraph (how decode runs), so host
        launch cost — which differs between hipBLASLt and our ops — is excluded."""
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        v = sorted(x.elapsed_time(y) for x, y in ts)
        del g
        return v[len(v) // 2] * 1000.0 / n

    @torch.inference_mode()
    def tune(self, shapes, device, ms=None):
        # inference mode like the engine's graph capture: the generator state tensors a
        # capture registers must not switch between inference and normal tensors
        ms = [m for m in (ms or TUNE_MS) if m <= 64]
        for (N, K) in sorted(set(shapes)):
            w = torch.randn(N, K, device=device, dtype=torch.bfloat16)
            for M in ms:
                x = torch.randn(M, K, device=device, dtype=torch.bfloat16)
                out = torch.empty(M, N, device=device, dtype=torch.bfloat16)
                best, best_t = "blas", self._time(lambda: F.linear(x, w))
                t_blas = best_t
                for rt, kw in SKINNY_CONFIGS:
                    if K % (256 * kw):
                        continue
                    t = self._time(lambda: torch.ops.hipserve.skinny_gemm(out, x, w, rt, kw))
                    if t < best_t * 0.97:
                        best, best_t = (rt, kw), t
                for sp in SPLITK_CONFIGS:
                    if (K // 256) < sp:
                        continue
                    t = self._time(lambda: splitk_gemm(out, x, w, sp))
                    if t < best_t * 0.97:
                        best, best_t = ("splitk", sp), t
                self.table[(M, N, K)] = best
                self.report.append({"M": M, "N": N, "K": K, "blas_us": round(t_blas, 1),
                                    "best": str(best), "best_us": round(best_t, 1)})
            del w
        return self.report


TUNER = GemmTuner()


def _empty(device):
    e = _EMPTY.get(device)
    if e is None:
        e = _EMPTY[device] = (torch.empty(0, dtype=torch.int16, device=device),
                              torch.empty(0, dtype=torch.float32, device=device))
    return e


def splitk_gemm(out, x, w, splits):
    M, K = x.shape
    N = w.shape[0]
    e16, e32 = _empty(x.device)
    ws = torch.empty(M, N, dtype=torch.float32, device=x.device) if splits > 1 else e32
    torch.ops.hipserve.gguf_gemm(out, x, w.view(torch.uint8), e16, e16, 6, 2 * K, N, K, ws, splits)
    return out


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    M = x.shape[0]
    if M <= 64 and x.is_cuda and TUNER.table:
        c = TUNER.choose(M, w.shape[0], w.shape[1])
        if c != "blas" and x.stride(1) == 1 and x.stride(0) % 8 == 0:
            out = torch.empty(M, w.shape[0], device=x.device, dtype=x.dtype)
            if c[0] == "splitk":
                return splitk_gemm(out, x, w, c[1])
            torch.ops.hipserve.skinny_gemm(out, x, w, c[0], c[1])
            return out
    return F.linear(x, w)
