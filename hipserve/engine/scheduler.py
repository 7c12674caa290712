"""Continuous-batching scheduler with chunked prefill, prefix caching and
recompute preemption (SURVEY §3.C engine core, §7.4 hard part 4).

Each step builds one batch under a token budget (``max_num_batched_tokens``):
running sequences first (1 token per decoding sequence, the next chunk for a
sequence still in prefill), then newly admitted ones (their prompt minus any
prefix-cache hit, chunked to the remaining budget). When the KV pool runs dry
the most recently admitted running sequence is preempted (blocks freed, state
reset to recompute) — FCFS fairness, no swap space needed with 288 GB HBM.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field

from .block_manager import BlockManager
from .request import Sequence, Status


@dataclass
class ScheduledSeq:
    seq: Sequence
    start: int            # first token index computed this step
    end: int              # one past the last token index computed this step

    @property
    def num_tokens(self) -> int:
        return self.end - self.start

    @property
    def samples(self) -> bool:
        """The step's last row is the sequence's last known token -> sample."""
        return self.end == self.seq.num_tokens


@dataclass
class SchedulerOutput:
    prefill: list[ScheduledSeq] = field(default_factory=list)
    decode: list[ScheduledSeq] = field(default_factory=list)
    preempted: list[Sequence] = field(default_factory=list)

    @property
    def num_tokens(self) -> int:
        return sum(s.num_tokens for s in self.prefill) + len(self.decode)

    @property
    def empty(self) -> bool:
        return not self.prefill and not self.decode


class Scheduler:
    def __init__(self, blocks: BlockManager, max_num_seqs: int, max_num_batched_tokens: int,
                 max_model_len: int):
        self.blocks = blocks
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []
        self.num_preemptions = 0

    def add(self, seq: Sequence):
        seq.status = Status.WAITING
        self.waiting.append(seq)

    def abort(self, request_id: str) -> Sequence | None:
        for q in (self.running, self.waiting):
            for s in list(q):
                if s.request_id == request_id:
                    q.remove(s)
                    self.blocks.free(s)
                    s.status = Status.FINISHED
                    s.finish_reason = "abort"
                    return s
        return None

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.running)

    @property
    def num_running(self):
        return len(self.running)

    @property
    def num_waiting(self):
        return len(self.waiting)

    def _preempt(self, seq: Sequence, out: SchedulerOutput):
        self.running.remove(seq)
        self.blocks.free(seq)
        seq.num_computed_tokens = 0
        seq.status = Status.PREEMPTED
        self.waiting.appendleft(seq)
        out.preempted.append(seq)
        self.num_preemptions += 1

    def schedule(self) -> SchedulerOutput:
        out = SchedulerOutput()
        budget = self.max_tokens
        scheduled_ids = set()
        # ---- 1. running sequences (FCFS order; victims taken from the tail)
        i = 0
        while i < len(self.running) and budget > 0:
            seq = self.running[i]
            n = min(seq.num_uncomputed, budget) if seq.is_prefill else 1
            target = seq.num_computed_tokens + n
            while not self.blocks.can_grow(seq, target):
                victim = self.running[-1]
                if victim is seq:
                    break
                self._preempt(victim, out)
            if not self.blocks.can_grow(seq, target):
                self._preempt(seq, out)
                continue
            self.blocks.grow(seq, target)
            ss = ScheduledSeq(seq, seq.num_computed_tokens, target)
            (out.prefill if seq.is_prefill else out.decode).append(ss)
            scheduled_ids.add(id(seq))
            budget -= n
            i += 1
        # ---- 2. admit waiting sequences (no admission in a step that preempted)
        if not out.preempted:
            while self.waiting and budget > 0 and len(self.running) < self.max_num_seqs:
                seq = self.waiting[0]
                if seq.num_computed_tokens == 0 and not seq.block_ids:
                    self.blocks.match_prefix(seq)
                n = min(seq.num_uncomputed, budget)
                target = seq.num_computed_tokens + n
                # the watermark protects RUNNING sequences' growth: with nothing running
                # (and nothing admitted yet this step) it would only block admission
                # forever for a chunk that fits the free pool exactly
                idle = not self.running and not out.prefill
                if not self.blocks.can_grow(seq, target, watermark=not idle):
                    if not self.running and not out.prefill:
                        # nothing else can free memory: the request can never fit
                        if not self.blocks.can_grow(seq, target):
                            self.waiting.popleft()
                            self.blocks.free(seq)
                            seq.status = Status.FINISHED
                            seq.finish_reason = "length"
                            out.preempted.append(seq)
                            continue
                    self.blocks.free(seq)  # undo prefix hit, retry next step
                    seq.num_computed_tokens = 0
                    break
                self.waiting.popleft()
                self.blocks.grow(seq, target)
                seq.status = Status.RUNNING
                self.running.append(seq)
                out.prefill.append(ScheduledSeq(seq, seq.num_computed_tokens, target))
                budget -= n
        return out

    def finish(self, seq: Sequence, reason: str):
        seq.status = Status.FINISHED
        seq.finish_reason = reason
        if seq in self.running:
            self.running.remove(seq)
        self.blocks.free(seq)
