"""Request / sequence state and sampling parameters (OpenAI request surface)."""
from __future__ import annotations

import enum
import time
import math
from dataclasses import dataclass, field

INT32_MAX = (1 << 31) - 1
MAX_LOGPROBS = 20   # OpenAI's top_logprobs limit; also the sampler kernel's top-n capacity
MAX_N = 128
MAX_STOP = 64


def _int(name: str, v, lo: int, hi: int) -> int:
    if isinstance(v, bool) or not isinstance(v, (int, float, str)):
        raise ValueError(f"{name} must be an integer")
    try:
        if isinstance(v, float):
            if not v.is_integer():
                raise ValueError
            v = int(v)
        else:
            v = int(v)
    except (ValueError, OverflowError):
        raise ValueError(f"{name} must be an integer") from None
    if not lo <= v <= hi:
        raise ValueError(f"{name} must be in [{lo}, {hi}]")
    return v


def _float(name: str, v, lo: float, hi: float) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float, str)):
        raise ValueError(f"{name} must be a number")
    try:
        v = float(v)
    except ValueError:
        raise ValueError(f"{name} must be a number") from None
    if not math.isfinite(v) or not lo <= v <= hi:
        raise ValueError(f"{name} must be in [{lo}, {hi}]")
    return v


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    max_tokens: int = 16
    min_tokens: int = 0
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    logprobs: int | None = None
    n: int = 1

    def __post_init__(self):
        """Coerce and range-check every field: a value that reaches the engine
        thread unchecked (a 2**64 seed in the int64 seed array, a string logprobs
        count) would raise inside ``step()`` and kill the engine for every
        request, so bad requests fail here with ValueError (HTTP 400)."""
        if isinstance(self.stop, str):
            self.stop = [self.stop]
        if not isinstance(self.stop, (list, tuple)) or not all(isinstance(s, str) for s in self.stop):
            raise ValueError("stop must be a string or a list of strings")
        self.stop = [s for s in self.stop if s]
        if len(self.stop) > MAX_STOP:
            raise ValueError(f"at most {MAX_STOP} stop strings")
        self.temperature = _float("temperature", self.temperature, 0.0, 1e4)
        self.top_p = _float("top_p", self.top_p, 0.0, 1.0)
        if self.top_p <= 0.0:
            raise ValueError("top_p must be in (0, 1]")
        self.top_k = _int("top_k", self.top_k, -1, INT32_MAX)
        if self.top_k < 0:
            self.top_k = 0
        if self.max_tokens is not None:
            self.max_tokens = _int("max_tokens", self.max_tokens, 1, INT32_MAX)
        self.min_tokens = _int("min_tokens", self.min_tokens, 0, INT32_MAX)
        self.stop_token_ids = [_int("stop_token_ids", t, 0, INT32_MAX) for t in (self.stop_token_ids or [])]
        self.ignore_eos = bool(self.ignore_eos)
        if self.seed is not None:
            self.seed = _int("seed", self.seed, -(1 << 63), (1 << 63) - 1)
        self.presence_penalty = _float("presence_penalty", self.presence_penalty, -2.0, 2.0)
        self.frequency_penalty = _float("frequency_penalty", self.frequency_penalty, -2.0, 2.0)
        self.repetition_penalty = _float("repetition_penalty", self.repetition_penalty, 1e-3, 100.0)
        if self.logprobs is not None:
            self.logprobs = _int("logprobs", self.logprobs, 0, MAX_LOGPROBS)
        self.n = _int("n", self.n, 1, MAX_N)

    @property
    def greedy(self) -> bool:
        return self.temperature <= 1e-5

    @property
    def has_penalties(self) -> bool:
        return (self.presence_penalty != 0.0 or self.frequency_penalty != 0.0
                or self.repetition_penalty != 1.0)


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    PREEMPTED = 2
    FINISHED = 3


@dataclass
class Sequence:
    request_id: str
    prompt_token_ids: list[int]
    params: SamplingParams
    eos_token_ids: tuple = ()
    arrival_time: float = field(default_factory=time.monotonic)
    output_token_ids: list[int] = field(default_factory=list)
    output_logprobs: list[float] = field(default_factory=list)
    status: Status = Status.WAITING
    block_ids: list[int] = field(default_factory=list)
    num_computed_tokens: int = 0        # tokens whose KV is in the cache
    num_cached_prefix: int = 0          # tokens served from the prefix cache
    finish_reason: str | None = None
    stop_reason: object = None
    first_token_time: float | None = None
    last_token_time: float | None = None
    seed: int = 0
    pen_slot: int | None = None         # device penalty-state slot (ModelRunner), while it has penalties
    mm: object = None                   # multimodal.MMState of a prompt with images
    # detokenizer state
    output_text: str = ""
    _decoded_upto: int = 0
    _prefix_offset: int = 0
    _read_offset: int = 0

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    @property
    def num_prompt_tokens(self) -> int:
        return len(self.prompt_token_ids)

    def all_token_ids(self) -> list[int]:
        return self.prompt_token_ids + self.output_token_ids

    def token_at(self, i: int) -> int:
        n = len(self.prompt_token_ids)
        return self.prompt_token_ids[i] if i < n else self.output_token_ids[i - n]

    @property
    def num_uncomputed(self) -> int:
        return self.num_tokens - self.num_computed_tokens

    @property
    def is_prefill(self) -> bool:
        """True while prompt (or recomputed) tokens remain; decode = exactly the
        last sampled token is missing from the KV cache."""
        return self.num_uncomputed > 1 or not self.output_token_ids

    @property
    def finished(self) -> bool:
        return self.status == Status.FINISHED


@dataclass
class RequestOutput:
    request_id: str
    new_token_ids: list[int]
    new_text: str
    finished: bool
    finish_reason: str | None = None
    num_prompt_tokens: int = 0
    num_output_tokens: int = 0
    logprobs: list[float] | None = None
    text: str = ""
