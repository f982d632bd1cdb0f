"""Engine-side request state and per-step outputs.

Internal request model of the reference spec (design.md:645-678:
InferenceRequest{id, request_type, tokens, params, created_at, deadline, ...},
InferenceParams{max_tokens, temperature, top_p, stop_sequences}) re-expressed
for a continuous-batching engine. Token-id stop sequences go to the C++
scheduler; string stop sequences are matched by the incremental detokenizer.
"""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field
from typing import Any, Callable, List, Optional


class RequestType(str, enum.Enum):
    Generate = "generate"
    Chat = "chat"
    Embeddings = "embeddings"


@dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    stop: List[str] = field(default_factory=list)
    stop_token_ids: List[List[int]] = field(default_factory=list)
    ignore_eos: bool = False
    min_tokens: int = 0
    seed: Optional[int] = None
    logprobs: bool = False


# finish reason codes shared with csrc/runtime/scheduler.h (SeqFinish)
FINISH_NONE, FINISH_STOP, FINISH_LENGTH, FINISH_STOP_SEQ, FINISH_ABORT, FINISH_EMBED = 0, 1, 2, 3, 4, 5
FINISH_NAMES = {FINISH_STOP: "stop", FINISH_LENGTH: "length", FINISH_STOP_SEQ: "stop_sequence",
                FINISH_ABORT: "abort", FINISH_EMBED: "stop"}


@dataclass
class RequestOutput:
    request_id: str
    new_token_ids: List[int]
    new_text: str
    finished: bool
    finish_reason: Optional[str] = None
    prompt_tokens: int = 0
    completion_tokens: int = 0
    cached_tokens: int = 0
    logprobs: Optional[List[float]] = None
    embedding: Optional[List[float]] = None
    error: Optional[str] = None
    error_code: Optional[str] = None
    # time.monotonic() when this output's tokens reached the host (Req 5.1 delivery
    # delay = socket write time - t_tokens; CLOCK_MONOTONIC is system-wide, so it holds
    # across replica processes)
    t_tokens: float = 0.0
    # the native SSE token event of this output, already framed as one HTTP/1.1 chunk
    # (encoded by the replica process that produced it, so the HTTP process only
    # writes bytes: server/replica.py encode_sse_chunk); None: encode on the server
    sse: Optional[bytes] = None


@dataclass
class EngineRequest:
    request_id: str
    seq_id: int
    prompt_ids: List[int]
    params: SamplingParams
    priority: int = 1
    kind: RequestType = RequestType.Generate
    arrival_time: float = field(default_factory=time.monotonic)
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    output_ids: List[int] = field(default_factory=list)
    detok: Any = None
    finished: bool = False
    finish_reason: Optional[str] = None
    cached_tokens: int = 0
    embed_acc_row: int = -1
    user_data: Any = None

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival_time
