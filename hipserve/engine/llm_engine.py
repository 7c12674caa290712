"""LLMEngine: request lifecycle around scheduler + model runner.

``step()`` = schedule -> (broadcast to TP workers) -> execute -> append sampled
tokens -> stop checks (EOS / stop ids / stop strings / max_tokens / max_model_len)
-> incremental detokenisation -> ``RequestOutput`` deltas for the API server.
"""
from __future__ import annotations

import itertools
import random
import time

from ..config import EngineConfig, ModelConfig, resolve_model_config
from ..parallel.comm import TPGroup, get_tp
from ..tokenizer import IncrementalDetokenizer, get_tokenizer
from .block_manager import BlockManager
from .metrics import EngineMetrics
from .model_runner import ModelRunner
from .request import RequestOutput, SamplingParams, Sequence, Status
from .scheduler import Scheduler


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tp: TPGroup | None = None,
                 model_cfg: ModelConfig | None = None):
        self.cfg = cfg
        self.tp = tp or get_tp()
        self.model_cfg = model_cfg or resolve_model_config(cfg.model, cfg.served_model_name)
        self.tokenizer = get_tokenizer(cfg.model, self.model_cfg, cfg.tokenizer)
        if getattr(self.tokenizer, "model_config_override", None):
            self.model_cfg = self.tokenizer.model_config_override
        self.runner = ModelRunner(cfg, self.model_cfg, self.tp)
        self.max_model_len = self.runner.max_model_len
        self.blocks = BlockManager(self.runner.usable_blocks, cfg.block_size, cfg.enable_prefix_caching)
        self.scheduler = Scheduler(self.blocks, cfg.max_num_seqs, cfg.max_num_batched_tokens,
                                   self.max_model_len)
        self.seqs: dict[str, Sequence] = {}
        self.detok: dict[str, IncrementalDetokenizer] = {}
        self._ids = itertools.count()
        self.metrics = EngineMetrics()
        self.eos_ids = tuple(self.tokenizer.eos_token_ids or self.model_cfg.eos_token_id or ())
        self.last_step_time = time.monotonic()

    # ---------------------------------------------------------------- requests
    def new_request_id(self) -> str:
        return f"req-{next(self._ids)}"

    def add_request(self, request_id: str | None, prompt, params: SamplingParams,
                    arrival_time: float | None = None) -> Sequence:
        request_id = request_id or self.new_request_id()
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
        self.seqs.pop(request_id, None)
        self.detok.pop(request_id, None)
        return seq

    def has_unfinished(self) -> bool:
        return self.scheduler.has_unfinished()

    # ---------------------------------------------------------------- stepping
    def step(self) -> list[RequestOutput]:
        so = self.scheduler.schedule()
        outputs: list[RequestOutput] = []
        for s in so.preempted:
            if s.status == Status.FINISHED:
                outputs.append(self._finish_output(s))
        if so.empty:
            return outputs
        t0 = time.monotonic()
        inp = self.runner.prepare(so)
        if self.tp.world_size > 1:
            self.tp.broadcast_obj(("step", inp))
        toks, lps, top = self.runner.execute(inp)
        now = time.monotonic()
        self.metrics.on_step(so, now - t0, self.blocks.usage(), self.scheduler)
        k = 0
        for ss in so.prefill + so.decode:
            seq = ss.seq
            seq.num_computed_tokens = ss.end
            self.blocks.register(seq)
            if not ss.samples:
                continue
            tok = int(toks[k])
            lp = float(lps[k])
            top_k = None
            if top is not None and seq.params.logprobs:
                n = seq.params.logprobs
                top_k = [(int(i), float(v)) for i, v in zip(top[0][k][:n], top[1][k][:n])]
            k += 1
            outputs.append(self._append(seq, tok, lp, top_k, now))
        self.last_step_time = now
        return outputs

    def _append(self, seq: Sequence, tok: int, lp: float, top, now: float) -> RequestOutput:
        p = seq.params
        if seq.first_token_time is None:
            seq.first_token_time = now
            self.metrics.on_first_token(seq, now)
        else:
            self.metrics.on_token(seq, now)
        seq.last_token_time = now
        seq.output_token_ids.append(tok)
        seq.output_logprobs.append(lp)
        reason = None
        n_out = len(seq.output_token_ids)
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
        if reason is None and seq.num_tokens >= self.max_model_len:
            reason = "length"
        out = RequestOutput(seq.request_id, [tok], text, reason is not None, reason,
                            seq.num_prompt_tokens, n_out, [lp] if top is None else [lp, top],
                            seq.output_text)
        if reason is not None:
            self.scheduler.finish(seq, reason)
            self.metrics.on_finish(seq, now)
            self.seqs.pop(seq.request_id, None)
            self.detok.pop(seq.request_id, None)
        return out

    def _finish_output(self, seq: Sequence) -> RequestOutput:
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
        if self.tp.world_size > 1 and self.tp.is_first:
            self.tp.broadcast_obj(("stop", None))


def worker_loop(runner: ModelRunner, tp: TPGroup):
    """TP ranks > 0: execute whatever rank 0 schedules until told to stop."""
    while True:
        kind, inp = tp.broadcast_obj(None)
        if kind == "stop":
            return
        runner.execute(inp)
