"""LLMEngine: request lifecycle around scheduler + model runner.

``step()`` = schedule -> (broadcast to TP workers) -> execute -> append sampled
tokens -> stop checks (EOS / stop ids / stop strings / max_tokens / max_model_len)
-> incremental detokenisation -> ``RequestOutput`` deltas for the API server.
"""
from __future__ import annotations

import itertools
import random
import time

import numpy as np

from ..config import EngineConfig, ModelConfig, resolve_model_config
from ..parallel.comm import TPGroup, get_tp
from ..tokenizer import IncrementalDetokenizer, get_tokenizer
from ..utils.faults import FaultInjector
from ..utils.tracing import Tracer, step_kind
from .block_manager import BlockManager
from .metrics import EngineMetrics
from .model_runner import ModelRunner
from .request import RequestOutput, SamplingParams, Sequence, Status
from .scheduler import ScheduledSeq, Scheduler, SchedulerOutput

PLACEHOLDER = -1  # output token whose value is still on the GPU (decode lookahead)


def prepare_model(cfg: EngineConfig, tp: TPGroup, model_cfg: ModelConfig | None = None):
    """(cfg, model config, tokenizer) of a pod's model, in the order a first start
    needs: the Hub id is materialised into the (PVC-backed) HF cache first — rank 0
    downloads, the other TP ranks wait — and only then are the config and the
    tokenizer read from it. Collective: every TP rank calls it."""
    from ..weights.hub import DummyFallback, materialize

    path = materialize(cfg.model, cfg.load_format, tp, cfg.served_model_name)
    if isinstance(path, DummyFallback):  # opted-in random weights: never under the Hub id's name
        cfg = cfg.replace(model=str(path), served_model_name=path.served_name, load_format="dummy",
                          tokenizer=cfg.tokenizer if cfg.tokenizer and cfg.tokenizer != cfg.model else None)
    elif path != cfg.model:
        cfg = cfg.replace(model=path, served_model_name=cfg.served_model_name or cfg.model,
                          tokenizer=cfg.tokenizer if cfg.tokenizer and cfg.tokenizer != cfg.model else None)
    mcfg = model_cfg or resolve_model_config(cfg.model, cfg.served_model_name)
    if cfg.extra.get("quantization") and cfg.extra["quantization"] not in ("fp8", "int8") and cfg.load_format == "dummy":
        # synthetic GGUF tier: ggml llama weights use interleaved-pair RoPE
        mcfg = mcfg.replace(rope_mode=1)
    tokenizer = get_tokenizer(cfg.model, mcfg, cfg.tokenizer)
    if getattr(tokenizer, "model_config_override", None):
        mcfg = tokenizer.model_config_override
    return cfg, mcfg, tokenizer


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tp: TPGroup | None = None,
                 model_cfg: ModelConfig | None = None):
        self.tp = tp or get_tp()
        self.cfg, self.model_cfg, self.tokenizer = prepare_model(cfg, self.tp, model_cfg)
        cfg = self.cfg
        self.runner = ModelRunner(cfg, self.model_cfg, self.tp)
        self.max_model_len = self.runner.max_model_len
        self.blocks = BlockManager(self.runner.usable_blocks, cfg.block_size, cfg.enable_prefix_caching)
        self.scheduler = Scheduler(self.blocks, cfg.max_num_seqs, cfg.max_num_batched_tokens,
                                   self.max_model_len)
        self.seqs: dict[str, Sequence] = {}
        self.detok: dict[str, IncrementalDetokenizer] = {}
        self._ids = itertools.count()
        self.metrics = EngineMetrics(model_name=cfg.model_name)
        self.eos_ids = tuple(self.tokenizer.eos_token_ids or self.model_cfg.eos_token_id or ())
        self.last_step_time = time.monotonic()
        self.lookahead = bool(cfg.extra.get("decode_lookahead", True)) and self.runner.use_graphs
        self._inflight = None
        self.tracer = Tracer.from_env()
        self.faults = FaultInjector.from_env()
        self.step_no = 0

    # ---------------------------------------------------------------- requests
    def new_request_id(self) -> str:
        return f"req-{next(self._ids)}"

    def add_request(self, request_id: str | None, prompt, params: SamplingParams,
                    arrival_time: float | None = None) -> Sequence:
        from ..multimodal import MultiModalPrompt, mm_state

        request_id = request_id or self.new_request_id()
        images = None
        if isinstance(prompt, MultiModalPrompt):
            images = prompt.images or None
            prompt = prompt.ids
        if isinstance(prompt, str):
            ids = self.tokenizer.encode(prompt)
        else:
            ids = [int(t) for t in prompt]
        if not ids:
            raise ValueError("empty prompt")
        V = self.model_cfg.vocab_size
        if any(t < 0 or t >= V for t in ids):
            raise ValueError(f"prompt token id out of range [0, {V})")
        if len(ids) >= self.max_model_len:
            raise ValueError(f"prompt has {len(ids)} tokens; max_model_len is {self.max_model_len}")
        seq = Sequence(request_id, ids, params, eos_token_ids=self.eos_ids)
        vcfg = self.model_cfg.vision
        if images:
            if vcfg is None or self.runner.model.visual is None:
                raise ValueError("this model has no vision encoder: image inputs are not supported")
            seq.mm = mm_state(ids, images, vcfg)
        elif vcfg is not None and vcfg.image_token_id in ids:
            raise ValueError("image placeholder tokens in a prompt without images")
        if arrival_time is not None:
            seq.arrival_time = arrival_time
        seq.seed = params.seed if params.seed is not None else random.getrandbits(62)
        self.seqs[request_id] = seq
        self.detok[request_id] = IncrementalDetokenizer(self.tokenizer, ids)
        self.scheduler.add(seq)
        self.metrics.on_arrival(seq)
        return seq

    def abort(self, request_id: str):
        seq = self.scheduler.abort(request_id)
        if seq is not None:
            self.runner.release(seq)
        self.seqs.pop(request_id, None)
        self.detok.pop(request_id, None)
        return seq

    def has_unfinished(self) -> bool:
        return self.scheduler.has_unfinished() or self._inflight is not None

    # ---------------------------------------------------------------- stepping
    def step(self) -> list[RequestOutput]:
        """One engine iteration. Decode-only batches are pipelined one step deep
        (``decode_lookahead``): step k+1 is scheduled with a placeholder for each
        sequence's not-yet-known token, staged and launched on the GPU — its input
        ids are taken on the device from step k's sampler output — BEFORE step k's
        tokens are read back and processed on the host. The host bookkeeping
        (stop checks, detokenisation, streaming) then overlaps GPU work instead of
        leaving the GPU idle between steps. Anything else (prefill, admissions,
        preemption, penalties, logprobs) runs synchronously."""
        self.faults.on_step("rank0", self.step_no)
        self.tp.check()  # a timed-out TP collective on any rank: raise -> engine dead
        self.step_no += 1
        tr = self.tracer
        if self._inflight is not None:
            return self._step_pipelined()
        with tr.phase("schedule"):
            so = self.scheduler.schedule()
        outputs: list[RequestOutput] = []
        for s in so.preempted:
            if s.status == Status.FINISHED:
                outputs.append(self._finish_output(s))
            else:  # recompute rebuilds the penalty slot from its ids (pen_init)
                self.runner.release(s)
        if so.empty:
            return outputs
        t0 = time.monotonic()
        tr.step_begin()
        with tr.phase("prepare"):
            inp = self.runner.prepare(so)
        if self.lookahead and self.runner.graph_eligible(inp):
            with tr.phase("launch"):
                self._inflight = self._launch(so, inp, t0)
            return outputs
        if self.tp.world_size > 1:
            self.tp.broadcast_obj(("step", inp))
        sampled = self._commit(so)
        with tr.phase("execute"):
            toks, lps, top = self.runner.execute(inp)
        now = time.monotonic()
        self._step_done(so, now - t0)
        with tr.phase("process"):
            outputs += self._process(so, sampled, toks, lps, top, now)
        return outputs

    def _step_done(self, so, dt):
        self.metrics.on_step(so, dt, self.blocks.usage(), self.scheduler)
        if self.tracer.enabled:
            npf = sum(s.num_tokens for s in so.prefill)
            self.tracer.step_done(step_kind(npf, len(so.decode)), so.num_tokens,
                                  len(so.prefill) + len(so.decode), dt, self.blocks.usage(),
                                  self.scheduler.num_running, self.scheduler.num_waiting)

    # -- pipelined decode ---------------------------------------------------
    def _launch(self, so, inp, t0, src=None):
        inp.src = src
        if self.tp.world_size > 1:
            self.tp.broadcast_obj(("step", inp))
        sampled = self._commit(so)
        return (so, sampled, self.runner.launch(inp), t0)

    def _step_pipelined(self) -> list[RequestOutput]:
        so, sampled, handle, t0 = self._inflight
        tr = self.tracer
        with tr.phase("schedule"):
            nxt = self._schedule_lookahead(sampled)
        t1 = time.monotonic()
        self._inflight = None
        if nxt is not None:
            so2, src = nxt
            tr.step_begin()
            with tr.phase("prepare"):
                inp = self.runner.prepare(so2)
            with tr.phase("launch"):
                self._inflight = self._launch(so2, inp, t1, src)
        with tr.phase("wait"):
            toks, lps, top = self.runner.wait(handle)
        now = time.monotonic()
        self._step_done(so, now - t0)
        with tr.phase("process"):
            return self._process(so, sampled, toks, lps, top, now)

    def _schedule_lookahead(self, sampled):
        """Next decode-only batch while the previous step is still in flight, or
        None when the batch composition cannot be predicted without its tokens."""
        sch = self.scheduler
        if sch.waiting or not sch.running:
            return None
        row = {id(seq): j for j, (seq, _) in enumerate(sampled)}
        so = SchedulerOutput()
        src = []
        for seq in sch.running:
            j = row.get(id(seq))
            if j is None or seq.is_prefill:
                return None
            p = seq.params
            n_out = len(seq.output_token_ids)
            if (p.max_tokens is not None and n_out >= p.max_tokens) or seq.num_tokens >= self.max_model_len:
                continue  # finishes with the in-flight token: not scheduled again
            target = seq.num_computed_tokens + 1
            if not self.blocks.can_grow(seq, target):
                return None
            self.blocks.grow(seq, target)
            so.decode.append(ScheduledSeq(seq, seq.num_computed_tokens, target))
            src.append(j)
        if not so.decode or len(so.decode) > self.runner.max_graph_batch:
            return None
        return so, np.array(src, dtype=np.int64)

    # -- bookkeeping ----------------------------------------------------------
    def _commit(self, so):
        """At launch: KV of the scheduled tokens counts as computed; each sampling
        sequence gets a placeholder output token (filled in by ``_process``)."""
        sampled = []
        for ss in so.prefill + so.decode:
            seq = ss.seq
            samples = ss.samples
            seq.num_computed_tokens = ss.end
            if samples:
                seq.output_token_ids.append(PLACEHOLDER)
                seq.output_logprobs.append(0.0)
                sampled.append((seq, len(seq.output_token_ids) - 1))
        return sampled

    def _process(self, so, sampled, toks, lps, top, now):
        outputs = []
        for k, (seq, idx) in enumerate(sampled):
            if seq.status == Status.FINISHED or seq.request_id not in self.seqs:
                continue  # finished / aborted while this step was in flight
            top_k = None
            if top is not None and seq.params.logprobs:
                n = seq.params.logprobs
                top_k = [(int(i), float(v)) for i, v in zip(top[0][k][:n], top[1][k][:n])]
            outputs.append(self._append(seq, idx, int(toks[k]), float(lps[k]), top_k, now))
        for ss in so.prefill + so.decode:
            if ss.seq.status != Status.FINISHED:
                self.blocks.register(ss.seq)
        self.last_step_time = now
        self.metrics.flush()
        return outputs

    def _append(self, seq: Sequence, idx: int, tok: int, lp: float, top, now: float) -> RequestOutput:
        p = seq.params
        if seq.first_token_time is None:
            seq.first_token_time = now
            self.metrics.on_first_token(seq, now)
        else:
            self.metrics.on_token(seq, now)
        seq.last_token_time = now
        seq.output_token_ids[idx] = tok
        seq.output_logprobs[idx] = lp
        reason = None
        n_out = idx + 1
        if not p.ignore_eos and tok in seq.eos_token_ids and n_out > p.min_tokens:
            reason = "stop"
        elif tok in p.stop_token_ids and n_out > p.min_tokens:
            reason = "stop"
            seq.stop_reason = tok
        skip_text = reason == "stop" and (tok in seq.eos_token_ids or tok in p.stop_token_ids)
        text = "" if skip_text else self.detok[seq.request_id].add([tok])
        if p.stop and reason is None:
            full = seq.output_text + text
            for st in p.stop:
                j = full.find(st, max(0, len(seq.output_text) - len(st)))
                if j >= 0:
                    text = full[len(seq.output_text):j] if j >= len(seq.output_text) else ""
                    full = full[:j]
                    reason = "stop"
                    seq.stop_reason = st
                    break
        seq.output_text += text
        if reason is None and p.max_tokens is not None and n_out >= p.max_tokens:
            reason = "length"
        if reason is None and seq.num_prompt_tokens + n_out >= self.max_model_len:
            reason = "length"
        out = RequestOutput(seq.request_id, [tok], text, reason is not None, reason,
                            seq.num_prompt_tokens, n_out, [lp] if top is None else [lp, top],
                            seq.output_text)
        if reason is not None:
            del seq.output_token_ids[n_out:]  # drop a look-ahead placeholder
            del seq.output_logprobs[n_out:]
            self.scheduler.finish(seq, reason)
            self.runner.release(seq)
            self.metrics.on_finish(seq, now)
            self.seqs.pop(seq.request_id, None)
            self.detok.pop(seq.request_id, None)
        return out

    def _finish_output(self, seq: Sequence) -> RequestOutput:
        self.runner.release(seq)
        self.seqs.pop(seq.request_id, None)
        self.detok.pop(seq.request_id, None)
        return RequestOutput(seq.request_id, [], "", True, seq.finish_reason or "length",
                             seq.num_prompt_tokens, len(seq.output_token_ids), None, seq.output_text)

    # ---------------------------------------------------------------- offline
    def generate(self, prompts, params: SamplingParams | list[SamplingParams]):
        """Blocking batch generation; returns {request_id: (token_ids, text, reason)}."""
        if not isinstance(params, list):
            params = [params] * len(prompts)
        order = []
        for p, sp in zip(prompts, params):
            order.append(self.add_request(None, p, sp).request_id)
        res = {rid: [[], "", None] for rid in order}
        while self.has_unfinished():
            for o in self.step():
                r = res[o.request_id]
                r[0].extend(o.new_token_ids)
                r[1] += o.new_text
                if o.finished:
                    r[2] = o.finish_reason
        return [tuple(res[rid]) for rid in order]

    def shutdown(self):
        self.tracer.close()
        if self.tp.world_size > 1 and self.tp.is_first:
            self.tp.broadcast_obj(("stop", None))


def worker_loop(runner: ModelRunner, tp: TPGroup, faults: FaultInjector | None = None):
    """TP ranks > 0: execute whatever rank 0 schedules until told to stop."""
    faults = faults or FaultInjector.from_env()
    step = 0
    while True:
        kind, inp = tp.broadcast_obj(None)
        if kind == "stop":
            return
        faults.on_step("worker", step)
        tp.check()
        step += 1
        if runner.graph_eligible(inp):
            runner.launch(inp)  # no host readback on workers: keep the GPU queue fed
        else:
            runner.execute(inp)
