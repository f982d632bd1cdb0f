"""InferenceServer: the control plane (tasks.md:298-312).

Owns the admission path and the replica pool:

  HTTP handler -> C++ RequestValidator (400) -> tokenizer -> degradation gate
  (503) -> C++ PriorityQueueManager (503 + Retry-After on backpressure) ->
  dispatcher -> C++ ReplicaRouter.select(strategy, memory estimate) ->
  replica (engine loop in a thread or a per-GPU process group) -> outputs hop
  onto the event loop -> TokenStreamer (SSE) or the request's future.

Background tasks: the dispatcher (event driven), the queue-timeout sweeper
(408, Req 3.3 / Property 8), the health checker (heartbeat age + process
liveness; failed replicas leave the routing pool, not-yet-started requests are
re-dispatched, streaming ones get an error event, the replica is restarted --
Req 6.4/6.5, 7.4, 9.4), the degradation monitor (design.md:921-944), and
optional static-mode batching (Req 2). Admin operations: hot config reload
(Req 10.5) and model hot-swap (Req 13: load new replica set, atomically switch
new traffic, drain the old set, then shut it down; failure keeps the old model).
"""
from __future__ import annotations

import asyncio
import copy
import logging
import threading
import time
from typing import Any, Dict, List, Optional

from .. import _runtime as R
from ..core.errors import (ApiError, ApiInternal, ApiQueueFull, ApiTimeout, ApiValidationError, ConfigError,
                           ValidationError)
from ..core.types import Priority, new_request_id
from ..core.wire import FinishReason, TokenEvent, Usage
from ..engine.request import RequestOutput, RequestType, SamplingParams
from ..obs import trace
from ..obs.metrics import MetricsCollector
from ..router import Router
from .batcher import RequestBatcher
from .config import ServerConfig, apply_hot_reload
from .degradation import DegradationLevel
from .replica import InProcessReplica, ProcessReplica, Replica, engine_spec
from .streamer import StreamSender, TokenStreamer

log = logging.getLogger("xgserve.server")

_FINISH = {"stop": FinishReason.Stop, "length": FinishReason.Length, "stop_sequence": FinishReason.StopSequence}


class ServiceUnavailable(ApiError):
    status = 503
    error_type = "server_error"
    code = "service_unavailable"

    def __init__(self, message: str, code: str = "service_unavailable", retry_after: float = 1.0):
        super().__init__(message, code=code, retry_after=retry_after)


def sse_chunk(ev: TokenEvent) -> bytes:
    """A TokenEvent's SSE bytes framed as one HTTP/1.1 chunk (direct socket writes)."""
    body = ev.sse()
    return b"%x\r\n%s\r\n" % (len(body), body)


class RemoteSender:
    """Stream sender of a request admitted by an HTTP front-end process
    (server/frontend.py): its final done / error event goes to that process."""

    def __init__(self, hub, wid: int, rid: str):
        self.hub, self.wid, self.rid = hub, wid, rid
        self.closed = False

    def send(self, ev: TokenEvent) -> None:
        if not self.closed:
            self.hub.send(self.wid, ("ev", self.rid, ev_to_tuple(ev)))

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self.hub.send(self.wid, ("close", self.rid))


# unread bytes a native SSE client may leave in its transport before the stream is cut
WIRE_MAX_BUFFERED = 4 << 20


class RemoteWire:
    """`ServerRequest.wire` of a native SSE stream held by a front-end process: token
    chunks are batched to that process, which writes them to the client socket."""

    def __init__(self, hub, wid: int, rid: str):
        self.hub, self.wid, self.rid = hub, wid, rid
        self.conn = hub.conns.get(wid)  # the front end's batching pipe end (frontend._Conn)

    def is_closing(self) -> bool:
        return False

    def send(self, chunk: bytes, t_tokens: float) -> None:
        c = self.conn
        if c is not None:  # appended in order with the request's other events
            c.pending.append(("tok", self.rid, chunk, t_tokens))
            if not c._flush_armed:
                c._flush_armed = True
                c.loop.call_soon(c.flush)


def ev_to_tuple(ev: TokenEvent) -> tuple:
    u = ev.usage
    return (ev.type, ev.token, ev.index, ev.logprob, ev.finish_reason.value if ev.finish_reason else None,
            (u.prompt_tokens, u.completion_tokens) if u is not None else None, ev.message, ev.code)


def ev_from_tuple(t: tuple) -> TokenEvent:
    typ, token, index, logprob, fr, u, message, code = t
    return TokenEvent(typ, token=token, index=index, logprob=logprob,
                      finish_reason=FinishReason(fr) if fr is not None else None,
                      usage=Usage.new(*u) if u is not None else None, message=message, code=code)


class ServerRequest:
    """One admitted request (the spec's InferenceRequest, design.md:645-678)."""

    def __init__(self, rid: str, kind: RequestType, prompt_ids: List[int], params: SamplingParams, priority: int,
                 stream: bool, loop: asyncio.AbstractEventLoop):
        self.id = rid
        self.kind = kind
        self.prompt_ids = prompt_ids
        self.params = params
        self.priority = int(priority)
        self.stream = stream
        # native SSE stream (/generate, /chat): replicas pre-encode its token events and,
        # once the response has started, _handle_outputs writes them straight to `wire`
        # (the client transport) -- no per-token queue hop or coroutine wake-up
        self.sse_native = False
        self.wire = None
        self.remote_wid: Optional[int] = None  # admitting front-end process (server/frontend.py)
        self.future: Optional[asyncio.Future] = None if stream else loop.create_future()
        self.sender: Optional[StreamSender] = None
        self.token_stream = None
        self.high = False
        self.text_parts: List[str] = []
        self.logprobs: List[float] = []
        self.completion_tokens = 0
        self.cached_tokens = 0
        self.embedding: Optional[List[float]] = None
        self.finish_reason: Optional[FinishReason] = None
        self.started = False
        self.finished = False
        self.replica: Optional[int] = None
        self.created = time.monotonic()
        self.dispatched_at: Optional[float] = None
        self.first_token_at: Optional[float] = None
        self.last_token_at: Optional[float] = None
        self.attempts = 0
        self.span = None
        self.qspan = None
        self.espan = None

    @property
    def prompt_tokens(self) -> int:
        return len(self.prompt_ids)

    @property
    def text(self) -> str:
        return "".join(self.text_parts)

    def usage(self) -> Usage:
        return Usage.new(self.prompt_tokens, self.completion_tokens)


class InferenceServer:
    def __init__(self, cfg: ServerConfig, engine=None):
        """`engine`: optional pre-built engine served by one in-process replica (tests/bench)."""
        self.cfg = cfg
        self.metrics = MetricsCollector()
        self.streamer = TokenStreamer()
        self.streamer.on_disconnect = self.cancel
        self.queue = R.PriorityQueueManager(self._qcfg(cfg))
        self.validator = R.RequestValidator(self._vcfg(cfg))
        self.router = Router(cfg.scheduler.strategy)
        self.batcher = RequestBatcher(cfg.batcher.max_batch_size, cfg.batcher.batch_timeout_ms,
                                      cfg.batcher.max_sequence_length, cfg.batcher.padding_token_id)
        self.replicas: Dict[int, Replica] = {}
        self.routable: List[int] = []
        self.inflight: Dict[str, ServerRequest] = {}
        self.queued: Dict[str, ServerRequest] = {}
        self.level = DegradationLevel.Normal
        self.accepting = False
        self.model_name = cfg.worker.model
        self.model_info: dict = {}
        self.tokenizer = None
        self._engine = engine
        self.fault: Optional[dict] = None  # MockEngine fault-injection knobs for new replicas (tests)
        self._next_replica_id = 0
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._loop_thread: Optional[int] = None
        self._wake: Optional[asyncio.Event] = None
        self._tasks: List[asyncio.Task] = []
        self._swap_lock: Optional[asyncio.Lock] = None
        self._reduced = False
        self.swaps = 0
        self.dispatched: Dict[int, int] = {}  # requests sent per replica id (first sends and re-dispatches)
        self.hub = None  # FrontendHub when HTTP runs in front-end processes (api.frontends > 1)
        trace.configure(cfg.observability.tracing, cfg.observability.trace_sample_rate)

    # ------------------------------------------------------------------ config helpers
    @staticmethod
    def _qcfg(cfg: ServerConfig):
        q = R.QueueConfig()
        q.high_watermark = cfg.queue.high_watermark
        q.low_watermark = cfg.queue.low_watermark
        q.request_timeout_s = cfg.queue.request_timeout_s
        q.max_queue_size = cfg.queue.max_queue_size
        q.aging_s = cfg.queue.aging_s
        return q

    @staticmethod
    def _vcfg(cfg: ServerConfig):
        v = R.ValidatorConfig()
        s = cfg.validator
        v.max_context_tokens, v.max_output_tokens = s.max_context_tokens, s.max_output_tokens
        v.min_temperature, v.max_temperature = s.min_temperature, s.max_temperature
        v.min_top_p, v.max_top_p = s.min_top_p, s.max_top_p
        return v

    # ------------------------------------------------------------------ lifecycle
    async def start(self, ready_timeout: Optional[float] = None) -> None:
        self._loop = asyncio.get_running_loop()
        self._loop_thread = threading.get_ident()
        self._wake = asyncio.Event()
        self._swap_lock = asyncio.Lock()
        ids = await self._spawn_set(self.cfg, ready_timeout)
        self._activate(ids)
        self.accepting = True
        self._tasks = [asyncio.create_task(self._dispatch_loop(), name="dispatch"),
                       asyncio.create_task(self._sweeper_loop(), name="sweeper"),
                       asyncio.create_task(self._health_loop(), name="health"),
                       asyncio.create_task(self._degradation_loop(), name="degradation"),
                       asyncio.create_task(self._lag_loop(), name="loop-lag")]
        if self.cfg.batcher.mode == "static":
            self._tasks.append(asyncio.create_task(self._batch_loop(), name="batcher"))
        log.info("server ready: model=%s replicas=%d tp=%d", self.model_name, len(ids), self.cfg.worker.tp)

    def _gpu_list(self, w) -> List[int]:
        if w.gpus:
            return [int(x) for x in str(w.gpus).split(",") if x.strip() != ""]
        return list(range(w.replicas * w.tp))

    def _make_replica(self, rid: int, spec: dict, gpus: List[int], w) -> Replica:
        if self._engine is not None:
            return InProcessReplica(rid, spec, self._on_replica_event, engine=self._engine)
        if w.in_process:
            if spec.get("tp", 1) != 1:
                raise ConfigError("in-process replicas support tp == 1 only")
            if not w.mock and w.device is None:
                spec = dict(spec, device=None)
            return InProcessReplica(rid, spec, self._on_replica_event)
        return ProcessReplica(rid, spec, self._on_replica_event, gpus=gpus, loop=self._loop)

    async def _spawn_set(self, cfg: ServerConfig, ready_timeout: Optional[float]) -> List[int]:
        w = cfg.worker
        spec = engine_spec(w, cfg.cache, cfg.spec, self.fault, cfg.batcher)
        gpus = self._gpu_list(w)
        n = 1 if self._engine is not None else w.replicas
        new: List[Replica] = []
        for i in range(n):
            rid = self._next_replica_id
            self._next_replica_id += 1
            r = self._make_replica(rid, spec, gpus[i * w.tp:(i + 1) * w.tp] or list(range(w.tp)), w)
            self.replicas[rid] = r
            new.append(r)
            r.start()
        timeout = ready_timeout or (60.0 if w.mock else 1800.0)
        oks = await asyncio.gather(*[asyncio.to_thread(r.wait_ready, timeout) for r in new])
        if not all(oks):
            errs = [f"replica {r.id}: {r.error or 'not ready in time'}" for r, ok in zip(new, oks) if not ok]
            for r in new:
                await asyncio.to_thread(r.shutdown, 5.0)
                self.replicas.pop(r.id, None)
            raise ApiInternal("; ".join(errs), code="model_load_failed")
        info = new[0].info
        self.model_info = info
        self.model_name = info.get("model", w.model)
        self.tokenizer = self._build_tokenizer(cfg, info)
        if self.hub is not None:
            self.hub.broadcast_state()
        self._spec = spec
        self._engine = None  # a pre-built engine is used once
        return [r.id for r in new]

    def _build_tokenizer(self, cfg: ServerConfig, info: dict):
        from ..engine.tokenizer import SyntheticTokenizer, load_tokenizer
        w = cfg.worker
        if w.mock:
            return SyntheticTokenizer(info.get("vocab_size", 1000), 1, info.get("eos_token_ids", [2]))
        eng = getattr(self.replicas[min(self.replicas)], "engine", None)
        if eng is not None and hasattr(eng, "tokenizer"):
            return eng.tokenizer
        from ..models import get_config
        return load_tokenizer(get_config(w.checkpoint or w.model), w.checkpoint)

    def _activate(self, ids: List[int]) -> None:
        for rid in ids:
            r = self.replicas[rid]
            self.router.register(rid, int(r.stats.get("memory_available", 1 << 40)) if r.stats else 1 << 40)
        self.routable = list(ids)

    async def shutdown(self, drain_timeout: float = 30.0) -> None:
        """Graceful: stop admitting, let queued + in-flight requests finish (bounded), stop replicas."""
        self.accepting = False
        t_end = time.monotonic() + drain_timeout
        while (self.inflight or not self.queue.is_empty()) and time.monotonic() < t_end:
            await asyncio.sleep(0.05)
        for _id, sreq, _p, _t in self.queue.drain():
            self.queued.pop(sreq.id, None)
            self._fail(sreq, ServiceUnavailable("Server shutting down", code="shutting_down"))
        for sreq in list(self.inflight.values()):
            self._abort_on_replica(sreq)
            self._fail(sreq, ServiceUnavailable("Server shutting down", code="shutting_down"))
        for t in self._tasks:
            t.cancel()
        await asyncio.gather(*self._tasks, return_exceptions=True)
        await asyncio.gather(*[asyncio.to_thread(r.shutdown, 10.0) for r in self.replicas.values()])
        self.replicas.clear()

    # ------------------------------------------------------------------ admission
    def validate_generate(self, prompt: str, max_tokens: int, temperature: float, top_p: float) -> None:
        self._raise_validation(self.validator.validate_generate(prompt, max_tokens, temperature, top_p))

    def validate_chat(self, contents: List[str], max_tokens: int, temperature: float, top_p: float) -> None:
        self._raise_validation(self.validator.validate_chat(contents, max_tokens, temperature, top_p))

    def validate_embeddings(self, inputs: List[str]) -> None:
        self._raise_validation(self.validator.validate_embeddings(inputs))

    @staticmethod
    def _raise_validation(res) -> None:
        if res is None:
            return
        raise ApiValidationError(ValidationError(res["kind"], res["message"], field=res["field"] or None,
                                                 reason=res["reason"] or None, actual=res["actual"],
                                                 limit=res["limit"]))

    def encode(self, text: str) -> List[int]:
        return self.tokenizer.encode(text)

    def admit(self, kind: RequestType, prompt_ids: List[int], params: SamplingParams,
              priority: int = Priority.Normal, stream: bool = False, rid: Optional[str] = None,
              sse_native: bool = False, remote: Optional[tuple] = None) -> ServerRequest:
        """Gate + enqueue. Raises ApiError (400 / 503). sse_native: the response is the
        native SSE format (token events pre-encoded by the replica). remote = (hub,
        front-end id): the request belongs to an HTTP front-end process; its events
        and result are routed there (server/frontend.py)."""
        if not self.accepting:
            self.metrics.record_rejection("shutting_down")
            raise ServiceUnavailable("Server is not accepting requests", code="shutting_down")
        if self.router.num_healthy() == 0:
            self.metrics.record_rejection("no_healthy_replica")
            raise ServiceUnavailable("No healthy replica available", code="no_replica")
        if not self.level.admits(int(priority)):
            self.metrics.record_rejection(f"degradation_{self.level.name}")
            raise ServiceUnavailable(f"Server under memory pressure ({self.level.name})", code="overloaded",
                                     retry_after=self.cfg.queue.retry_after_s)
        mml = int(self.model_info.get("max_model_len", 1 << 30))
        limit = mml if kind == RequestType.Embeddings else mml - 1
        if len(prompt_ids) > limit:
            raise ApiValidationError(ValidationError.token_limit_exceeded(len(prompt_ids), limit))
        sreq = ServerRequest(rid or new_request_id(), kind, prompt_ids, params, int(priority), stream, self._loop)
        if remote is not None:
            hub, wid = remote
            sreq.remote_wid = wid  # cancelled if that front end dies (FrontendHub._front_end_lost)
            if stream:
                sreq.sender = RemoteSender(hub, wid, sreq.id)
                self.streamer.register(sreq.id, sreq.sender)
                sreq.sse_native = sse_native
                if sse_native:
                    sreq.wire = RemoteWire(hub, wid, sreq.id)
            else:
                sreq.future.add_done_callback(lambda f, s_=sreq: hub.send_result(wid, s_, f))
        elif stream:
            sreq.sender, sreq.token_stream = self.streamer.create_stream(sreq.id)
            sreq.sse_native = sse_native
        if not self.queue.enqueue(sreq.id, sreq, int(priority)):
            if stream:
                self.streamer.discard(sreq.id)
            self.metrics.record_rejection("queue_full")
            raise ApiQueueFull(retry_after=self.cfg.queue.retry_after_s)
        sreq.qspan = trace.start_span("queue", request_id=sreq.id, priority=int(priority))
        self.queued[sreq.id] = sreq
        self._record_queue_depth()
        self._wake.set()
        return sreq

    # ---- async facade: the HTTP handlers' interface, also served to front-end
    # processes over IPC (server/frontend.py FrontendClient implements the same)
    async def aadmit(self, *a, **kw) -> ServerRequest:
        return self.admit(*a, **kw)

    async def astats(self) -> dict:
        return self.stats()

    async def ahealth(self) -> dict:
        return self.health()

    async def ametrics_text(self) -> str:
        self.check_health()
        return self.metrics.prometheus()

    async def areload_config(self, patch) -> dict:
        return self.reload_config(patch)

    async def acfg(self) -> dict:
        return self.cfg.to_dict()

    async def amodel_state(self) -> dict:
        return {"model": self.model_name, "info": self.model_info, "swaps": self.swaps}

    async def areplica_state(self) -> dict:
        return {"replicas": self.stats()["replicas"], "routable": list(self.routable)}

    def cancel(self, rid: str) -> None:
        """Client disconnect or caller timeout: remove from the queue or abort in the engine."""
        sreq = self.queued.pop(rid, None)
        if sreq is not None:
            self.queue.cancel(rid)
            self._record_queue_depth()
            sreq.finished = True
            trace.end_span(sreq.qspan, outcome="cancelled")
            return
        sreq = self.inflight.get(rid)
        if sreq is not None:
            self._abort_on_replica(sreq)
            self._finalize(sreq)
            trace.end_span(sreq.espan, outcome="cancelled")

    def _abort_on_replica(self, sreq: ServerRequest) -> None:
        r = self.replicas.get(sreq.replica) if sreq.replica is not None else None
        if r is not None:
            r.abort(sreq.id)

    def _record_queue_depth(self) -> None:
        h, n, l, _ = self.queue.queue_depth()
        self.metrics.record_queue_depth(h, n, l)

    # ------------------------------------------------------------------ dispatch
    def _mem_estimate(self, sreq: ServerRequest) -> int:
        per_tok = int(self.model_info.get("kv_bytes_per_token", 0))
        return per_tok * (sreq.prompt_tokens + (0 if sreq.kind == RequestType.Embeddings else sreq.params.max_tokens))

    def _pick(self, sreq: ServerRequest) -> int:
        rid = self.router.select(self._mem_estimate(sreq) if self.router.strategy == "memory_aware" else 0)
        if rid < 0:
            return -1
        cap = self.cfg.scheduler.max_inflight_per_replica
        if len(self.replicas[rid].inflight) < cap:
            return rid
        for other in self.routable:  # selected one is saturated: any healthy replica with room
            r = self.replicas.get(other)
            if r is not None and other in self._healthy_ids() and len(r.inflight) < cap:
                return other
        return -1

    def _healthy_ids(self) -> set:
        return {s["id"] for s in self.router.statuses() if s["healthy"]}

    def _send_to(self, sreq: ServerRequest, rid: int) -> None:
        r = self.replicas[rid]
        sreq.replica = rid
        sreq.attempts += 1
        sreq.dispatched_at = time.monotonic()
        self.inflight[sreq.id] = sreq
        r.inflight[sreq.id] = sreq
        self.router.add_active(rid, 1)
        self.dispatched[rid] = self.dispatched.get(rid, 0) + 1
        trace.end_span(sreq.qspan, replica=rid)
        sreq.espan = trace.start_span("engine", parent=sreq.qspan, request_id=sreq.id, replica=rid)
        r.submit(sreq.id, sreq.prompt_ids, copy.copy(sreq.params), sreq.priority, sreq.kind.value, sreq.sse_native)

    async def _dispatch_loop(self) -> None:
        while True:
            try:
                await asyncio.wait_for(self._wake.wait(), timeout=0.05)
            except asyncio.TimeoutError:
                pass
            self._wake.clear()
            self._dispatch_ready()

    def _dispatch_ready(self) -> None:
        static = self.cfg.batcher.mode == "static"
        while not self.queue.is_empty():
            head = self.queue.peek_id()
            sreq = self.queued.get(head) if head is not None else None
            if sreq is None:  # stale entry (cancelled concurrently)
                self.queue.dequeue_one()
                continue
            if not static:
                rid = self._pick(sreq)
                if rid < 0:
                    break
            item = self.queue.dequeue_one()
            self.queued.pop(item[0], None)
            if static:
                sreq.high = sreq.priority == Priority.High
                self._loop.create_task(self.batcher.add_request(sreq.id, sreq.prompt_ids, sreq.params.max_tokens,
                                                                sreq, high_priority=sreq.high))
            else:
                self._send_to(sreq, rid)
        self._record_queue_depth()

    async def _batch_loop(self) -> None:
        """Static batching: one window batch -> one replica, all members admitted together."""
        while True:
            b = await self.batcher.get_batch(timeout=0.5)
            if b is None:
                continue
            self.metrics.record_batch(b.size, b.padding_ratio)
            live = [br.payload for br in b.requests if not br.payload.finished]
            if not live:
                continue
            rid = -1
            while rid < 0:
                rid = self._pick(live[0])
                if rid < 0:
                    await asyncio.sleep(0.01)
            for sreq in live:
                self._send_to(sreq, rid)

    # ------------------------------------------------------------------ replica events
    def _on_replica_event(self, rid: int, kind: str, payload: Any) -> None:
        loop = self._loop
        if loop is None or loop.is_closed():
            return
        if threading.get_ident() == self._loop_thread:  # a reader on the loop itself (ProcessReplica)
            self._handle_event(rid, kind, payload)
            return
        try:
            loop.call_soon_threadsafe(self._handle_event, rid, kind, payload)
        except RuntimeError:
            pass

    def _handle_event(self, rid: int, kind: str, payload: Any) -> None:
        if kind == "out":
            self._handle_outputs(rid, payload)
        elif kind == "hb":
            r = self.replicas.get(rid)
            if r is not None and rid in self.routable:
                self.router.update(rid, len(r.inflight), payload.get("memory_used", 0),
                                   payload.get("memory_available", 0))
        elif kind == "fatal":
            r = self.replicas.get(rid)
            if r is not None and r.ready.is_set() and rid in self.routable:
                log.error("replica %d reported fatal error: %s", rid, payload)
                self._on_replica_failure(r)

    def _wire_ok(self, sreq: ServerRequest, w) -> bool:
        """May a token chunk go straight to this client transport? Direct writes skip
        aiohttp's drain, so a client that stays connected but stops reading would
        grow the transport buffer for the whole generation: past WIRE_MAX_BUFFERED
        unread bytes the stream fails as a slow consumer and its sequence is aborted."""
        if w.is_closing():
            return False
        if w.get_write_buffer_size() <= WIRE_MAX_BUFFERED:
            return True
        log.warning("request %s: client not reading (%d bytes unsent), stream cut", sreq.id,
                    w.get_write_buffer_size())
        self.metrics.record_error("slow_consumer")
        sreq.wire = None
        self.streamer.fail_stream(sreq.id, "client is not reading the stream", "slow_consumer")
        self.cancel(sreq.id)
        return False

    def _handle_outputs(self, rid: int, outs: List[RequestOutput]) -> None:
        now = time.monotonic()
        n_tok = 0
        n_wire, t_wire = 0, 0.0
        inflight = self.inflight
        itl: List[float] = []
        for o in outs:
            sreq = inflight.get(o.request_id)
            if sreq is None or sreq.replica != rid:
                continue
            w = sreq.wire
            if (w is not None and o.sse is not None and not o.finished and sreq.last_token_at is not None
                    and not o.logprobs and o.embedding is None):
                # steady-state token of a native SSE stream (the per-token hot path at node
                # scale): the replica encoded the chunk; account it and pass it on
                n_tok += 1
                itl.append(now - sreq.last_token_at)
                sreq.last_token_at = now
                sreq.completion_tokens = o.completion_tokens
                if w.__class__ is RemoteWire:
                    w.send(o.sse, o.t_tokens)
                elif self._wire_ok(sreq, w):
                    w.write(o.sse)
                    n_wire += 1
                    t_wire = o.t_tokens
                continue
            if o.error:
                self._finalize(sreq)
                self.metrics.record_error(o.error_code or "inference_failed")
                self._fail(sreq, ApiInternal(o.error.removeprefix("Inference failed: ")
                                             if o.error_code == "inference_failed" else o.error,
                                             code=o.error_code or "inference_failed"))
                continue
            if o.new_token_ids:
                n_tok += len(o.new_token_ids)
                if sreq.first_token_at is None:
                    sreq.first_token_at = now
                    self.metrics.record_ttft(now - sreq.created)
                elif sreq.last_token_at is not None:
                    itl.append(now - sreq.last_token_at)
                sreq.last_token_at = now
                sreq.started = True
                sreq.completion_tokens = o.completion_tokens or (sreq.completion_tokens + len(o.new_token_ids))
                if o.logprobs:
                    sreq.logprobs.extend(o.logprobs)
                if sreq.sender is not None:
                    if o.new_text:
                        w = sreq.wire
                        if w is not None:  # direct: write the (pre-encoded) chunk to the socket now
                            chunk = o.sse if o.sse is not None else sse_chunk(TokenEvent.tok(
                                o.new_text, sreq.completion_tokens - 1, o.logprobs[-1] if o.logprobs else None))
                            if w.__class__ is RemoteWire:
                                w.send(chunk, o.t_tokens)  # the front end writes it and times the delivery
                            elif self._wire_ok(sreq, w):
                                w.write(chunk)
                                n_wire += 1
                                t_wire = o.t_tokens
                        else:
                            ev = TokenEvent.tok(o.new_text, sreq.completion_tokens - 1,
                                                o.logprobs[-1] if o.logprobs else None)
                            ev.t_tokens = o.t_tokens  # not serialised: delivery-delay measurement (Req 5.1)
                            sreq.sender.send(ev)
                else:
                    sreq.text_parts.append(o.new_text)
            elif o.new_text:
                if sreq.sender is not None:
                    ev = TokenEvent.tok(o.new_text, max(0, sreq.completion_tokens - 1))
                    if sreq.wire is not None:
                        if sreq.wire.__class__ is RemoteWire:
                            sreq.wire.send(sse_chunk(ev), o.t_tokens)
                        elif self._wire_ok(sreq, sreq.wire):
                            sreq.wire.write(sse_chunk(ev))
                    else:
                        sreq.sender.send(ev)
                else:
                    sreq.text_parts.append(o.new_text)
            if o.embedding is not None:
                sreq.embedding = o.embedding
            if o.finished:
                if o.finish_reason == "abort":
                    continue  # aborted by us (cancel/timeout) -- already answered
                sreq.cached_tokens = o.cached_tokens
                sreq.finish_reason = _FINISH.get(o.finish_reason or "stop", FinishReason.Stop)
                self._finalize(sreq)
                self._complete(sreq)
        if n_tok:
            self.metrics.record_inference(0, n_tok)
        if itl:
            self.metrics.record_itl_many(itl)
        if n_wire and t_wire:
            self.metrics.record_delivery(time.monotonic() - t_wire, n_wire)

    def _finalize(self, sreq: ServerRequest) -> None:
        if sreq.finished:
            return
        sreq.finished = True
        self.inflight.pop(sreq.id, None)
        r = self.replicas.get(sreq.replica) if sreq.replica is not None else None
        if r is not None and r.inflight.pop(sreq.id, None) is not None:
            self.router.add_active(r.id, -1)
        self.metrics.record_inference(sreq.prompt_tokens, 0)
        if sreq.cached_tokens:
            self.metrics.record_cache_access(True, sreq.cached_tokens)
        self.metrics.record_cache_access(False, max(0, sreq.prompt_tokens - sreq.cached_tokens))
        self._wake.set()

    def _complete(self, sreq: ServerRequest) -> None:
        trace.end_span(sreq.espan, completion_tokens=sreq.completion_tokens, finish=sreq.finish_reason.value)
        if sreq.sender is not None:
            try:
                self.streamer.close_stream(sreq.id, sreq.finish_reason, sreq.usage())
            except Exception:
                pass
        elif sreq.future is not None and not sreq.future.done():
            sreq.future.set_result(sreq)

    def _fail(self, sreq: ServerRequest, err: ApiError) -> None:
        sreq.finished = True
        trace.end_span(sreq.espan or sreq.qspan, error=err.code)
        if sreq.sender is not None:
            self.streamer.fail_stream(sreq.id, err.message, err.code)
        elif sreq.future is not None and not sreq.future.done():
            sreq.future.set_exception(err)

    # ------------------------------------------------------------------ background loops
    async def _sweeper_loop(self) -> None:
        while True:
            await asyncio.sleep(0.1)
            expired = self.queue.remove_expired()
            for _id, sreq, _p, _t in expired:
                self.queued.pop(sreq.id, None)
                self.metrics.record_error("timeout")
                self._fail(sreq, ApiTimeout())
            if expired:
                self._record_queue_depth()
            if not self.queue.is_empty():
                self._wake.set()

    async def _health_loop(self) -> None:
        while True:
            await asyncio.sleep(self.cfg.scheduler.health_check_interval_s)
            self.check_health()

    def check_health(self) -> None:
        hb_timeout = self.cfg.scheduler.heartbeat_timeout_s
        healthy = self._healthy_ids()
        specs = [r.stats.get("speculative") for r in self.replicas.values() if r.stats.get("speculative")]
        if specs:
            sfs = [x["speedup_factor"] for x in specs if x.get("speedup_factor") is not None]
            self.metrics.set_spec_totals(sum(x["draft_tokens_proposed"] for x in specs),
                                         sum(x["draft_tokens_accepted"] for x in specs),
                                         sum(sfs) / len(sfs) if sfs else None)
        for rid in list(self.routable):
            r = self.replicas.get(rid)
            if r is None:
                continue
            alive = r.is_alive() and r.heartbeat_age() < hb_timeout
            st = r.stats or {}
            self.metrics.record_worker_status(rid, {"healthy": alive, "active": len(r.inflight),
                                                    "kv_usage": st.get("kv_usage", 0.0),
                                                    "memory_used": st.get("memory_used", 0),
                                                    "memory_available": st.get("memory_available", 0),
                                                    "restarts": r.restarts, "kind": r.kind})
            if alive:
                self.router.update(rid, len(r.inflight), st.get("memory_used", 0), st.get("memory_available", 0))
                if rid not in healthy and not getattr(r, "restarting", False):
                    self.router.set_healthy(rid, True)
            elif rid in healthy:
                self._on_replica_failure(r)

    def _on_replica_failure(self, r: Replica) -> None:
        log.error("replica %d unhealthy (alive=%s hb_age=%.1fs); removing from routing pool", r.id, r.is_alive(),
                  r.heartbeat_age())
        self.metrics.record_error("worker_failed")
        self.router.set_healthy(r.id, False)
        reqs = list(r.inflight.values())
        r.inflight.clear()
        for sreq in reqs:
            self.inflight.pop(sreq.id, None)
            if not sreq.started and sreq.attempts < 3 and self.accepting:
                sreq.replica = None  # re-dispatch on a healthy replica
                if self.queue.enqueue(sreq.id, sreq, int(Priority.High)):
                    self.queued[sreq.id] = sreq
                    continue
            sreq.finished = True
            self._fail(sreq, ApiInternal("worker failed", code="worker_failed"))
        self._record_queue_depth()
        self._wake.set()
        if self.cfg.scheduler.restart_failed and r.restarts < self.cfg.scheduler.max_restarts:
            r.restarting = True
            self._loop.create_task(self._restart(r))

    async def _restart(self, old: Replica) -> None:
        await asyncio.to_thread(old.shutdown, 2.0)
        w = self.cfg.worker
        spec = old.spec
        if isinstance(old, ProcessReplica):
            r: Replica = ProcessReplica(old.id, spec, self._on_replica_event, gpus=old.gpus, loop=self._loop)
        else:
            r = InProcessReplica(old.id, spec, self._on_replica_event)
        r.restarts = old.restarts + 1
        self.replicas[old.id] = r
        r.start()
        ok = await asyncio.to_thread(r.wait_ready, 60.0 if w.mock else 1800.0)
        if ok and old.id in self.routable:
            log.warning("replica %d restarted (%d/%d)", r.id, r.restarts, self.cfg.scheduler.max_restarts)
            self.router.set_healthy(r.id, True)
            self._wake.set()
        else:
            log.error("replica %d failed to restart: %s", r.id, r.error)

    async def _lag_loop(self, period: float = 0.02) -> None:
        """Event-loop lag probe: everything on the serve path (outputs, SSE writes,
        admission) runs on this loop, so a late wake-up is delay every stream sees."""
        while True:
            t = time.monotonic()
            await asyncio.sleep(period)
            self.metrics.record_loop_lag(max(0.0, time.monotonic() - t - period))

    async def _degradation_loop(self) -> None:
        while True:
            await asyncio.sleep(0.5)
            self.update_degradation()

    def memory_pressure(self) -> float:
        healthy = self._healthy_ids()
        us = [self.replicas[i].stats.get("kv_usage", 0.0) for i in self.routable
              if i in healthy and i in self.replicas and self.replicas[i].stats]
        return min(us) if us else 0.0

    def update_degradation(self, pressure: Optional[float] = None) -> DegradationLevel:
        d = self.cfg.degradation
        p = self.memory_pressure() if pressure is None else pressure
        lvl = DegradationLevel.from_memory_pressure(p, d.reduce_batch_at, d.aggressive_evict_at,
                                                    d.reject_low_priority_at, d.emergency_at)
        if lvl != self.level:
            log.warning("degradation level %s -> %s (memory pressure %.2f)", self.level.name, lvl.name, p)
        w = self.cfg.worker
        if lvl >= DegradationLevel.ReducedBatchSize and not self._reduced:
            for i in self.routable:
                self.replicas[i].set_limits(max(1, w.max_num_seqs // 2), w.max_num_batched_tokens)
            self._reduced = True
        elif lvl == DegradationLevel.Normal and self._reduced:
            for i in self.routable:
                self.replicas[i].set_limits(w.max_num_seqs, w.max_num_batched_tokens)
            self._reduced = False
        if lvl >= DegradationLevel.AggressiveCacheEviction and lvl != self.level:
            for i in self.routable:
                self.replicas[i].clear_cache()
        self.level = lvl
        return lvl

    # ------------------------------------------------------------------ admin
    def reload_config(self, patch: Dict[str, Dict[str, Any]]) -> dict:
        new = apply_hot_reload(self.cfg, patch)
        self.queue.set_config(self._qcfg(new))
        self.validator.set_config(self._vcfg(new))
        if new.scheduler.strategy != self.cfg.scheduler.strategy:
            self.router.set_strategy(new.scheduler.strategy)
        self.batcher.set_limits(new.batcher.max_batch_size, new.batcher.batch_timeout_ms)
        if (new.worker.max_num_seqs, new.worker.max_num_batched_tokens) != \
                (self.cfg.worker.max_num_seqs, self.cfg.worker.max_num_batched_tokens):
            for i in self.routable:
                self.replicas[i].set_limits(new.worker.max_num_seqs, new.worker.max_num_batched_tokens)
        self.cfg = new
        if self.hub is not None:
            self.hub.broadcast_state()
        log.info("config reloaded: %s", patch)
        return {k: v for k, v in new.to_dict().items() if k in patch}

    async def swap_model(self, worker_patch: Dict[str, Any], ready_timeout: Optional[float] = None) -> dict:
        """Req 13: load the new model on a fresh replica set, switch new requests
        atomically, drain in-flight requests on the old set, then unload it."""
        async with self._swap_lock:
            new_cfg = copy.deepcopy(self.cfg)
            errors: List[str] = []
            from .config import _set
            for k, v in worker_patch.items():
                _set(new_cfg, "worker", k, v, errors, "swap")
            errors += new_cfg.validate()
            if errors:
                raise ConfigError("; ".join(errors))
            old_ids = list(self.routable)
            old_name, old_info, old_tok = self.model_name, self.model_info, self.tokenizer
            try:
                ids = await self._spawn_set(new_cfg, ready_timeout)
            except ApiError:
                self.model_name, self.model_info, self.tokenizer = old_name, old_info, old_tok
                raise
            # atomic switch (single-threaded event loop): new traffic -> new set
            for rid in old_ids:
                self.router.unregister(rid)
            self._activate(ids)
            self.cfg = new_cfg
            self.metrics = MetricsCollector()  # stats reset after a swap (Req 13.5)
            self.swaps += 1
            if self.hub is not None:
                self.hub.broadcast_state()
            self._wake.set()
            self._loop.create_task(self._drain_and_stop(old_ids))
            log.info("model swapped: %s -> %s", old_name, self.model_name)
            return {"previous_model": old_name, "model": self.model_name, "replicas": ids}

    def _free_gpus(self, n: int) -> List[int]:
        """The n lowest GPU indices no live process replica holds, taken from the
        configured `worker.gpus` list, else from the GPUs this node has (mock
        replicas touch no GPU: any index). ConfigError when fewer are free."""
        used = {g for r in self.replicas.values() for g in (getattr(r, "gpus", None) or [])}
        w = self.cfg.worker
        if w.gpus:
            pool = self._gpu_list(w)
        elif w.mock:
            pool = list(range(len(used) + n))
        else:
            import torch  # device_count() does not initialise the GPU in this process
            pool = list(range(torch.cuda.device_count()))
        cand = [g for g in pool if g not in used]
        if len(cand) < n:
            raise ConfigError(f"need {n} free GPU(s), only {len(cand)} of {len(pool)} are free")
        return cand[:n]

    async def add_replicas(self, count: int = 1, gpus: Optional[List[int]] = None,
                           ready_timeout: Optional[float] = None) -> dict:
        """Req 7.5: start `count` more replicas of the serving model at runtime and
        route to them once ready; traffic on the existing replicas is untouched.
        The swap lock is held only while GPUs are reserved and processes started,
        and again while the ready replicas are registered -- not across the load."""
        w = self.cfg.worker
        max_count = 64 if w.mock else 8
        if count < 1 or count > max_count:
            raise ConfigError(f"count must be in [1, {max_count}]")
        async with self._swap_lock:
            spec = self._spec
            tp = max(1, int(w.tp))
            if gpus is not None and len(gpus) != count * tp:
                raise ConfigError(f"need {count * tp} GPU ids for {count} replica(s) of tp={tp}, got {len(gpus)}")
            if gpus is not None:
                held = {g for r in self.replicas.values() for g in (getattr(r, "gpus", None) or [])}
                if held & set(gpus):
                    raise ConfigError(f"GPU(s) {sorted(held & set(gpus))} already hold a replica")
            gl = list(gpus) if gpus is not None else (self._free_gpus(count * tp) if not w.in_process else [])
            new: List[Replica] = []
            for i in range(count):
                rid = self._next_replica_id
                self._next_replica_id += 1
                r = self._make_replica(rid, spec, gl[i * tp:(i + 1) * tp] or list(range(tp)), w)
                self.replicas[rid] = r  # reserves its GPUs for concurrent calls
                new.append(r)
                r.start()
            model_at_start = self.model_name
        timeout = ready_timeout or (60.0 if w.mock else 1800.0)
        oks = await asyncio.gather(*[asyncio.to_thread(r.wait_ready, timeout) for r in new])
        async with self._swap_lock:
            swapped = self.model_name != model_at_start
            if not all(oks) or swapped:
                errs = ([f"replica {r.id}: {r.error or 'not ready in time'}" for r, ok in zip(new, oks) if not ok]
                        or ["the serving model was swapped while the replicas loaded"])
                for r in new:
                    await asyncio.to_thread(r.shutdown, 5.0)
                    self.replicas.pop(r.id, None)
                raise ApiInternal("; ".join(errs), code="replica_start_failed")
            for r in new:
                self.router.register(r.id, int(r.stats.get("memory_available", 1 << 40)) if r.stats else 1 << 40)
                self.routable.append(r.id)
            self.cfg.worker.replicas = len(self.routable)
            self._wake.set()
            log.info("replicas added: %s (now %d)", [r.id for r in new], len(self.routable))
            return {"added": [r.id for r in new], "replicas": list(self.routable)}

    async def remove_replicas(self, ids: Optional[List[int]] = None, count: int = 1) -> dict:
        """Req 7.5: take replicas out of routing at runtime (default: the newest
        `count`), let their in-flight requests finish, then stop them. Queued
        requests are dispatched to the remaining replicas; at least one stays."""
        async with self._swap_lock:
            if ids is None:
                ids = list(self.routable[-count:]) if count >= 1 else []
            ids = [int(i) for i in ids]
            bad = [i for i in ids if i not in self.routable]
            if bad:
                raise ConfigError(f"unknown or inactive replica id(s) {bad}; active: {self.routable}")
            if not ids or len(ids) >= len(self.routable):
                raise ConfigError("removal would leave no replica serving")
            for rid in ids:
                self.router.unregister(rid)
                self.routable.remove(rid)
            self.cfg.worker.replicas = len(self.routable)
            self._wake.set()
            self._loop.create_task(self._drain_and_stop(ids))
            log.info("replicas removed: %s (now %d)", ids, len(self.routable))
            return {"removed": ids, "replicas": list(self.routable)}

    async def _drain_and_stop(self, ids: List[int], timeout: float = 600.0) -> None:
        t_end = time.monotonic() + timeout
        olds = [self.replicas[i] for i in ids if i in self.replicas]
        while any(r.inflight for r in olds) and time.monotonic() < t_end:
            await asyncio.sleep(0.05)
        for r in olds:
            for sreq in list(r.inflight.values()):
                r.abort(sreq.id)
                self._finalize(sreq)
                self._fail(sreq, ApiInternal("model swapped", code="model_swapped"))
            await asyncio.to_thread(r.shutdown, 10.0)
            self.replicas.pop(r.id, None)

    # ------------------------------------------------------------------ views
    def stats(self) -> dict:
        snap = self.metrics.snapshot()
        h, n, l, t = self.queue.queue_depth()
        reps = []
        healthy = self._healthy_ids()
        for s in self.router.statuses():
            r = self.replicas.get(s["id"])
            st = dict(r.stats) if r is not None and r.stats else {}
            reps.append({"id": s["id"], "healthy": s["healthy"], "active_requests": len(r.inflight) if r else 0,
                         "memory_used": s["memory_used"], "memory_available": s["memory_available"],
                         "kind": r.kind if r else None, "restarts": r.restarts if r else 0,
                         "requests_dispatched": self.dispatched.get(s["id"], 0),
                         "heartbeat_age_s": r.heartbeat_age() if r else None, "engine": st})
        return {"model": self.model_name, "metrics": snap,
                "queue_depth": {"high": h, "normal": n, "low": l, "total": t},
                "accepting": self.queue.is_accepting(),
                "active_requests": len(self.inflight), "active_streams": self.streamer.active_streams(),
                "replicas": reps, "replicas_healthy": len(healthy & set(self.routable)),
                "strategy": self.router.strategy, "batcher": {"mode": self.cfg.batcher.mode,
                                                              "batches_formed": self.batcher.batches_formed},
                "degradation": {"level": self.level.name, "memory_pressure": self.memory_pressure()},
                "model_swaps": self.swaps}

    def health(self) -> dict:
        n = len(self._healthy_ids() & set(self.routable))
        status = "ok" if n == len(self.routable) and n > 0 else ("degraded" if n > 0 else "unhealthy")
        return {"status": status, "model": self.model_name, "replicas_healthy": n,
                "replicas_total": len(self.routable), "degradation": self.level.name}
