"""InferenceWorker: the spec'd batch-level worker interface on top of an engine.

The reference specifies (design.md:310-361; Req 7, requirements.md:100-110)

    trait InferenceWorker { initialize(); infer(batch) -> BatchResult; shutdown();
                            status() -> WorkerStatus; model_info() -> ModelInfo }

with ``BatchResult{batch_id, results: Vec<RequestResult>, inference_time,
tokens_generated}`` holding exactly one ``RequestResult`` per input request
(Property 21) and per-request failure isolation (Property 22).

Here the engines are iteration-level (continuous batching): ``infer`` admits
every member of an :class:`~xgserve.server.batcher.InferenceBatch` at once
(un-padded: ``original_length`` tokens each, the padding is an API artefact)
and steps the engine until all of them finished, so a static batch is simply
a burst of requests that share engine steps. A request that fails is returned
with ``finish_reason="error"`` and its message; its batch-mates are unaffected.
Works with :class:`LLMEngine` and :class:`MockEngine` alike.
"""
from __future__ import annotations

import copy
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from .request import SamplingParams


@dataclass
class RequestResult:
    request_id: str
    tokens: List[int]
    text: str
    finish_reason: str
    prompt_tokens: int
    completion_tokens: int
    error: Optional[str] = None
    error_code: Optional[str] = None


@dataclass
class BatchResult:
    batch_id: str
    results: List[RequestResult]
    inference_time: float  # seconds
    tokens_generated: int


@dataclass
class WorkerState:
    """design.md:290-297 WorkerStatus (the router keeps the live copy)."""
    id: int
    ready: bool
    active_batches: int
    memory_used: int
    memory_available: int
    is_healthy: bool
    last_health_check: float


@dataclass
class ModelInfo:
    name: str
    vocab_size: int
    hidden_size: int
    max_model_len: int
    eos_token_ids: List[int] = field(default_factory=list)
    num_blocks: int = 0


class WorkerError(RuntimeError):
    """WorkerError (error.rs:115-128): ModelNotLoaded / Shutdown / InferenceFailed / OutOfMemory."""

    def __init__(self, kind: str, message: str = ""):
        super().__init__(f"{kind}: {message}" if message else kind)
        self.kind = kind


class InferenceWorker:
    """One model replica behind the spec'd batch interface.

    ``engine_factory`` builds the engine on ``initialize()`` (e.g.
    ``lambda: make_engine(engine_spec(...))``), so construction is cheap and
    loading errors surface from ``initialize`` as ``WorkerError("ModelLoad")``.
    """

    def __init__(self, engine_factory: Callable[[], object], worker_id: int = 0):
        self._factory = engine_factory
        self.id = worker_id
        self.engine = None
        self._lock = threading.Lock()  # one infer() at a time drives the engine
        self._active = 0
        self._shutdown = False
        self._last_check = 0.0

    # -- lifecycle ------------------------------------------------------------
    def initialize(self) -> None:
        if self.engine is not None:
            return
        try:
            self.engine = self._factory()
        except Exception as e:  # noqa: BLE001 - reported as the spec's load error
            raise WorkerError("ModelLoad", str(e)) from e
        self._shutdown = False

    def shutdown(self) -> None:
        with self._lock:
            eng, self.engine = self.engine, None
            self._shutdown = True
        stop = getattr(eng, "stop_followers", None)
        if stop is not None:
            stop()

    # -- inference ------------------------------------------------------------
    def infer(self, batch, params: Optional[SamplingParams] = None,
              per_request: Optional[Dict[str, SamplingParams]] = None, max_steps: int = 1 << 30) -> BatchResult:
        """Run one InferenceBatch to completion. ``params`` defaults to greedy with
        ``batch.max_new_tokens``; ``per_request`` overrides it by request id."""
        if self._shutdown:
            raise WorkerError("Shutdown")
        if self.engine is None:
            raise WorkerError("ModelNotLoaded")
        base = params or SamplingParams(max_tokens=max(1, int(batch.max_new_tokens)), temperature=0.0)
        t0 = time.perf_counter()
        with self._lock:
            self._active += 1
            try:
                return self._run(batch, base, per_request or {}, max_steps, t0)
            finally:
                self._active -= 1

    def _run(self, batch, base, per_request, max_steps, t0) -> BatchResult:
        eng = self.engine
        order: List[str] = []
        res: Dict[str, RequestResult] = {}
        for br, ids in zip(batch.requests, batch.input_ids):
            rid = br.id
            order.append(rid)
            prompt = list(ids[: br.original_length])
            p = copy.deepcopy(per_request.get(rid, base))
            try:
                eng.add_request(rid, prompt, p)
            except Exception as e:  # noqa: BLE001 - rejected alone (Property 22)
                res[rid] = RequestResult(rid, [], "", "error", len(prompt), 0, error=str(e),
                                         error_code="invalid_request")
                continue
            res[rid] = RequestResult(rid, [], "", "", len(prompt), 0)
        pending = {rid for rid in order if not res[rid].finish_reason}
        steps = 0
        while pending and steps < max_steps:
            try:
                outs = eng.step()
            except Exception as e:  # noqa: BLE001 - a failed step fails the requests still running
                for rid in list(pending):
                    r = res[rid]
                    r.finish_reason, r.error, r.error_code = "error", f"Inference failed: {e}", "inference_failed"
                    eng.abort(rid)
                pending.clear()
                break
            steps += 1
            for o in outs:
                r = res.get(o.request_id)
                if r is None or o.request_id not in pending:
                    continue
                r.tokens.extend(o.new_token_ids)
                r.text += o.new_text
                r.completion_tokens = max(r.completion_tokens, o.completion_tokens or len(r.tokens))
                if o.finished:
                    r.finish_reason = o.finish_reason or "stop"
                    if getattr(o, "error", None):
                        r.error, r.error_code = o.error, getattr(o, "error_code", None) or "inference_failed"
                    pending.discard(o.request_id)
        for rid in pending:  # step cap hit
            eng.abort(rid)
            res[rid].finish_reason = "length"
        results = [res[rid] for rid in order]
        return BatchResult(batch.id, results, time.perf_counter() - t0,
                           sum(len(r.tokens) for r in results))

    # -- introspection ----------------------------------------------------------
    def status(self) -> WorkerState:
        self._last_check = time.time()
        eng = self.engine
        if eng is None:
            return WorkerState(self.id, False, 0, 0, 0, False, self._last_check)
        st = eng.stats()
        return WorkerState(self.id, True, self._active, int(st.get("memory_used", 0)),
                           int(st.get("memory_available", 0)), not self._shutdown, self._last_check)

    def model_info(self) -> ModelInfo:
        if self.engine is None:
            raise WorkerError("ModelNotLoaded")
        from ..server.replica import engine_info
        i = engine_info(self.engine)
        return ModelInfo(i["model"], i["vocab_size"], i["hidden_size"], i["max_model_len"], i["eos_token_ids"],
                         i["num_blocks"])
