"""Request batcher (Req 2, requirements.md:39-49; design.md:227-267;
Properties 4-5).

Two modes behind one interface:

* ``continuous`` (default): admission is per-request and the engine's C++
  StepScheduler forms a new ragged batch every iteration, so no padding ever
  exists (padding_ratio == 0). The batcher only forwards.
* ``static``: the spec's window batcher. Requests collected for at most
  ``batch_timeout_ms`` or until ``max_batch_size`` (whichever first) form one
  InferenceBatch, padded to the longest member with ``padding_token_id`` and a
  0/1 attention mask; each BatchedRequest keeps its original/padded length.
  High-priority requests jump to the front of the *next* batch (Req 2.4). The
  batch is dispatched to one replica as a unit (all members admitted in the
  same engine step) -- the engine itself still runs ragged kernels, the padded
  tensors are the API contract and feed the Req 2.5 log line.
"""
from __future__ import annotations

import asyncio
import logging
import time
import uuid
from dataclasses import dataclass, field
from typing import Any, List, Optional

log = logging.getLogger("xgserve.batcher")


@dataclass
class BatchedRequest:
    id: str
    original_length: int
    padded_length: int
    payload: Any = None


@dataclass
class InferenceBatch:
    id: str
    requests: List[BatchedRequest]
    input_ids: List[List[int]]
    attention_mask: List[List[int]]
    max_new_tokens: int
    created_at: float = field(default_factory=time.monotonic)

    @property
    def size(self) -> int:
        return len(self.requests)

    @property
    def padding_ratio(self) -> float:
        tot = sum(len(r) for r in self.input_ids)
        return 0.0 if tot == 0 else 1.0 - sum(r.original_length for r in self.requests) / tot

    @property
    def avg_seq_len(self) -> float:
        return sum(r.original_length for r in self.requests) / max(1, len(self.requests))


def build_batch(items: List[tuple], padding_token_id: int = 0, max_sequence_length: Optional[int] = None) -> InferenceBatch:
    """items: (id, token_ids, max_new_tokens, payload). Pads to the longest sequence."""
    seqs = [list(t[1])[: max_sequence_length] if max_sequence_length else list(t[1]) for t in items]
    L = max((len(s) for s in seqs), default=0)
    ids, mask, reqs = [], [], []
    for (rid, _, _, payload), s in zip(items, seqs):
        n = len(s)
        ids.append(s + [padding_token_id] * (L - n))
        mask.append([1] * n + [0] * (L - n))
        reqs.append(BatchedRequest(rid, n, L, payload))
    return InferenceBatch(str(uuid.uuid4()), reqs, ids, mask, max((t[2] for t in items), default=0))


class RequestBatcher:
    """Window batcher for static mode (asyncio; one consumer)."""

    def __init__(self, max_batch_size: int = 32, batch_timeout_ms: float = 50.0, max_sequence_length: int = 8192,
                 padding_token_id: int = 0):
        self.max_batch_size = max_batch_size
        self.batch_timeout_ms = batch_timeout_ms
        self.max_sequence_length = max_sequence_length
        self.padding_token_id = padding_token_id
        self._pending: List[tuple] = []
        self._first_at: Optional[float] = None
        self._cv: Optional[asyncio.Condition] = None
        self.batches_formed = 0

    def _cond(self) -> asyncio.Condition:
        if self._cv is None:
            self._cv = asyncio.Condition()
        return self._cv

    def set_limits(self, max_batch_size: int, batch_timeout_ms: float):
        self.max_batch_size, self.batch_timeout_ms = max_batch_size, batch_timeout_ms

    async def add_request(self, rid: str, token_ids: List[int], max_new_tokens: int, payload=None,
                          high_priority: bool = False) -> None:
        cv = self._cond()
        async with cv:
            item = (rid, token_ids, max_new_tokens, payload)
            if high_priority:
                # ahead of every non-high item still waiting -> next batch (Req 2.4)
                k = 0
                while k < len(self._pending) and getattr(self._pending[k][3], "high", False):
                    k += 1
                self._pending.insert(k, item)
            else:
                self._pending.append(item)
            if self._first_at is None:
                self._first_at = time.monotonic()
            cv.notify_all()

    def pending_count(self) -> int:
        return len(self._pending)

    def current_batch_size(self) -> int:
        return min(len(self._pending), self.max_batch_size)

    async def get_batch(self, timeout: Optional[float] = None) -> Optional[InferenceBatch]:
        """Block until a batch is due: max_batch_size pending, or the window of the
        oldest pending request has elapsed. None if `timeout` passes with nothing pending."""
        cv = self._cond()
        deadline = None if timeout is None else time.monotonic() + timeout
        async with cv:
            while True:
                now = time.monotonic()
                if self._pending:
                    due = self._first_at + self.batch_timeout_ms / 1000.0
                    if len(self._pending) >= self.max_batch_size or now >= due:
                        return self._take()
                    wait = due - now
                else:
                    if deadline is not None and now >= deadline:
                        return None
                    wait = None if deadline is None else deadline - now
                try:
                    await asyncio.wait_for(cv.wait(), timeout=wait)
                except asyncio.TimeoutError:
                    pass

    def _take(self) -> InferenceBatch:
        items = self._pending[: self.max_batch_size]
        self._pending = self._pending[self.max_batch_size:]
        self._first_at = time.monotonic() if self._pending else None
        b = build_batch(items, self.padding_token_id, self.max_sequence_length)
        self.batches_formed += 1
        log.info("batch formed id=%s size=%d avg_seq_len=%.1f padding_overhead=%.3f", b.id, b.size, b.avg_seq_len,
                 b.padding_ratio)
        return b
