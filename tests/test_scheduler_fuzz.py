"""Property-based fuzzing of the continuous-batching scheduler over the native
block pool (SURVEY §5 "race detection / sanitizers": hypothesis fuzzing of
scheduler invariants). Random arrivals (with shared prompt prefixes, so the
prefix cache is hit), aborts and steps on a deliberately tiny KV pool, so
preemption and the can-never-fit path run; the engine's commit is simulated.

Invariants checked after every step:
* the step's token count is within ``max_num_batched_tokens`` and the running set
  within ``max_num_seqs``;
* every scheduled sequence owns blocks covering its scheduled range, and its
  range starts at its computed-token count;
* each block's refcount equals the number of live sequences holding it;
* after draining, every request finished and all blocks are back in the pool.
"""
import random

import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from hipserve.engine.block_manager import BlockManager  # noqa: E402
from hipserve.engine.request import SamplingParams, Sequence, Status  # noqa: E402
from hipserve.engine.scheduler import Scheduler  # noqa: E402

NUM_BLOCKS, BS, MAX_SEQS, MAX_TOKENS, MAX_LEN = 24, 4, 4, 16, 64

ops = st.lists(st.one_of(
    st.tuples(st.just("add"), st.integers(1, 40), st.integers(1, 12), st.integers(0, 2)),
    st.tuples(st.just("step")),
    st.tuples(st.just("abort"), st.integers(0, 50)),
), min_size=1, max_size=60)


def _check(sch: Scheduler, bm: BlockManager, live: dict):
    held = {}
    for s in live.values():
        for b in s.block_ids:
            held[b] = held.get(b, 0) + 1
    for b in range(NUM_BLOCKS):
        assert bm.pool.refcount(b) == held.get(b, 0), (b, bm.pool.refcount(b), held.get(b, 0))
    assert len(sch.running) <= MAX_SEQS


def _step(sch: Scheduler, bm: BlockManager, live: dict, rng: random.Random, limits: dict):
    so = sch.schedule()
    assert so.num_tokens <= MAX_TOKENS
    for s in so.preempted:
        if s.status == Status.FINISHED:  # can never fit the pool: finished with "length"
            live.pop(s.request_id, None)
    for ss in so.prefill + so.decode:
        seq = ss.seq
        assert ss.start == seq.num_computed_tokens and ss.end > ss.start
        assert len(seq.block_ids) * BS >= ss.end
        samples = ss.samples
        seq.num_computed_tokens = ss.end
        if samples:
            seq.output_token_ids.append(rng.randrange(5))
            if len(seq.output_token_ids) >= limits[seq.request_id] or seq.num_tokens >= MAX_LEN:
                sch.finish(seq, "length")
                live.pop(seq.request_id, None)
    for ss in so.prefill + so.decode:
        if ss.seq.status != Status.FINISHED:
            bm.register(ss.seq)
    _check(sch, bm, live)
    return so


@settings(max_examples=150, deadline=None)
@given(ops, st.integers(0, 2**31 - 1))
def test_scheduler_invariants(program, seed):
    rng = random.Random(seed)
    bm = BlockManager(NUM_BLOCKS, BS, prefix_caching=True)
    sch = Scheduler(bm, MAX_SEQS, MAX_TOKENS, MAX_LEN)
    live, limits, order = {}, {}, []
    prefixes = [[7] * 12, [1, 2, 3, 4] * 3, list(range(20, 32))]
    for i, op in enumerate(program):
        if op[0] == "add":
            _, n, max_out, fam = op
            toks = (prefixes[fam] + [rng.randrange(5) for _ in range(n)])[: MAX_LEN - 1]
            rid = f"r{i}"
            seq = Sequence(rid, toks, SamplingParams(max_tokens=max_out))
            live[rid], limits[rid] = seq, max_out
            order.append(rid)
            sch.add(seq)
        elif op[0] == "abort" and order:
            rid = order[op[1] % len(order)]
            if sch.abort(rid) is not None:
                live.pop(rid, None)
            _check(sch, bm, live)
        else:
            _step(sch, bm, live, rng, limits)
    for _ in range(2000):  # drain
        if not sch.has_unfinished():
            break
        _step(sch, bm, live, rng, limits)
    assert not sch.has_unfinished() and not live
    assert bm.num_free() == NUM_BLOCKS


def test_idle_admission_ignores_watermark():
    """with nothing running, a first chunk that fits the free pool only
    WITHOUT the watermark used to be neither finished nor admitted — retried
    every step forever, blocking the FCFS queue. It must be admitted."""
    bm = BlockManager(NUM_BLOCKS, BS, prefix_caching=False)
    sch = Scheduler(bm, MAX_SEQS, 1000, 1000)
    # exactly the whole pool: fits without the watermark, not with it
    seq = Sequence("r0", list(range(NUM_BLOCKS * BS - 1)), SamplingParams(max_tokens=1))
    sch.add(seq)
    so = sch.schedule()
    assert [s.seq.request_id for s in so.prefill] == ["r0"]
    assert not so.preempted


def test_incremental_prefix_registration_matches():
    """BlockManager.register hashes only the newly filled blocks (chained from the
    last call); a later sequence with the same prefix must still hit every block."""
    bm = BlockManager(16, 4, prefix_caching=True)
    a = Sequence("a", list(range(10, 20)), SamplingParams(max_tokens=8))
    bm.grow(a, 10)
    a.num_computed_tokens = 10
    bm.register(a)                      # blocks 0-1 (8 tokens)
    a.output_token_ids += [7, 8, 9]
    bm.grow(a, 13)
    a.num_computed_tokens = 13
    bm.register(a)                      # block 2 (prompt tail + outputs)
    b = Sequence("b", list(range(10, 20)) + [7, 8, 9, 5], SamplingParams(max_tokens=1))
    bm.match_prefix(b)
    assert b.num_computed_tokens == 12 and b.block_ids == a.block_ids[:3]
