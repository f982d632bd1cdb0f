"""Sharded HTTP front end: `api.frontends` > 1 HTTP processes over one orchestrator.

At node scale one asyncio process cannot write every token event of every
stream: 8 replicas x ~150 steps/s x 64 rows is ~77k SSE events/s, and each is a
socket send on the serving loop (profiles/r3_frontend.md). With `frontends = N`
the serving process keeps the control plane -- C++ priority queue + backpressure,
C++ router, replicas, health, degradation, hot reload, hot swap, metrics -- and N
front-end processes own the client sockets:

  client --HTTP--> front end k (SO_REUSEPORT: the kernel spreads connections)
      parse + validate (C++ validator) + tokenize locally
      "admit" ---pipe---> hub (orchestrator process): queue / 400 / 503 decision
  replicas --outputs--> hub: per step, each stream's token chunk (pre-encoded by
      the replica, RequestOutput.sse) is appended to its front end's batch; one
      pipe message per front end per loop iteration
  front end k: writes each chunk straight to its client's socket (no per-token
      queue hop), done / error events and non-stream results come the same way.

The hub's per-token work is a dict lookup and a list append; the socket sends,
HTTP parsing, JSON and tokenization run in N processes. Everything a handler
needs (`aadmit`, `astats`, `ahealth`, `ametrics_text`, admin calls, `cancel`,
`metrics.*`) has the same interface here (FrontendClient) as on InferenceServer,
so server/app.py serves both modes unchanged. Front ends report request
metrics and Req 5.1 delivery delays (measured at their socket writes) to the hub.
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import multiprocessing as mp
import os
import pickle
import select
import signal
import struct
import threading
import time
from typing import Any, Dict, List, Optional

from ..core.errors import ApiError, ApiValidationError, ValidationError
from ..core.wire import FinishReason, TokenEvent, Usage
from .streamer import TokenStreamer

log = logging.getLogger("xgserve.frontend")


def error_to_tuple(e: BaseException) -> tuple:
    if isinstance(e, ApiError):
        return (e.status, e.error_type, e.code, e.message, e.retry_after)
    return (500, "server_error", "internal_error", f"Internal server error: {e}", None)


class RemoteApiError(ApiError):
    """An ApiError raised in the hub, re-raised in the front end (same status / body)."""

    def __init__(self, status: int, error_type: str, code: str, message: str, retry_after):
        self.status = status
        self.error_type = error_type
        super().__init__(message, code=code, retry_after=retry_after)


def _unframe(chunk: bytes) -> bytes:
    """HTTP/1.1 chunk -> its payload (b"<hex>\\r\\n<payload>\\r\\n")."""
    i = chunk.index(b"\r\n")
    return chunk[i + 2:len(chunk) - 2]


_HDR = struct.Struct("<I")


class _Conn:
    """One duplex pipe end, serviced ON the event loop: a reader callback (no reader
    thread re-hopping onto the loop and contending for the GIL) hands decoded
    message batches to `on_msgs`; `send` batches messages and flushes once per loop
    iteration. (A writer thread doing the pickling and the pipe write measured
    slower on an 8-core host: one more thread holding the GIL beside the loop.)

    The socket is NON-BLOCKING with our own length-prefixed frames: a flush writes
    what the kernel takes and leaves the rest to a loop writer callback, so a peer
    that is itself busy writing (both ends flushing batches larger than the socket
    buffer) can never block this loop -- each side keeps reading while its own
    bytes wait (blocking send_bytes on both ends could deadlock)."""

    READ_CHUNK = 1 << 20

    def __init__(self, conn, loop: asyncio.AbstractEventLoop, on_msgs, name: str):
        self.conn = conn  # keeps the descriptor open
        self.fd = conn.fileno()
        os.set_blocking(self.fd, False)
        self.loop = loop
        self.on_msgs = on_msgs
        self.pending: List[tuple] = []
        self._flush_armed = False
        self.closed = False
        self.name = name
        self._rbuf = bytearray()
        self._wbuf = bytearray()
        self._writer_on = False
        loop.add_reader(self.fd, self._readable)

    def _readable(self) -> None:
        eof = False
        while True:
            try:
                data = os.read(self.fd, self.READ_CHUNK)
            except (BlockingIOError, InterruptedError):
                break
            except OSError:
                eof = True
                break
            if not data:
                eof = True
                break
            self._rbuf += data
        self._deliver()
        if eof:
            self._eof()

    def _deliver(self) -> None:
        buf, off, n = self._rbuf, 0, len(self._rbuf)
        frames = []
        while n - off >= 4:
            (ln,) = _HDR.unpack_from(buf, off)
            if n - off - 4 < ln:
                break
            frames.append(bytes(buf[off + 4:off + 4 + ln]))
            off += 4 + ln
        if off:
            del buf[:off]
        for f in frames:
            self.on_msgs(pickle.loads(f))

    def _eof(self) -> None:
        self.closed = True
        self.loop.remove_reader(self.fd)
        if self._writer_on:
            self.loop.remove_writer(self.fd)
            self._writer_on = False
        self._wbuf.clear()
        self.on_msgs([("eof",)])

    def send(self, msg: tuple) -> None:
        self.pending.append(msg)
        if not self._flush_armed:
            self._flush_armed = True
            self.loop.call_soon(self.flush)

    def flush(self) -> None:
        self._flush_armed = False
        if not self.pending or self.closed:
            self.pending = []
            return
        msgs, self.pending = self.pending, []
        payload = pickle.dumps(msgs, protocol=pickle.HIGHEST_PROTOCOL)
        self._wbuf += _HDR.pack(len(payload))
        self._wbuf += payload
        self._write_some()

    def _write_some(self) -> None:
        try:
            while self._wbuf:
                k = os.write(self.fd, self._wbuf)
                del self._wbuf[:k]
        except (BlockingIOError, InterruptedError):
            pass
        except OSError:  # peer gone: the reader sees the EOF
            self.closed = True
            self._wbuf.clear()
        if self._wbuf and not self._writer_on:
            self.loop.add_writer(self.fd, self._write_some)
            self._writer_on = True
        elif not self._wbuf and self._writer_on:
            self.loop.remove_writer(self.fd)
            self._writer_on = False

    @property
    def buffered(self) -> int:
        """Bytes flushed but not yet taken by the kernel."""
        return len(self._wbuf)

    def close(self, timeout: float = 5.0) -> None:
        """Flush, then give the socket up to `timeout` to take the rest (shutdown)."""
        self.flush()
        t_end = time.monotonic() + timeout
        while self._wbuf and not self.closed and time.monotonic() < t_end:
            select.select([], [self.fd], [], 0.05)
            self._write_some()


# ---------------------------------------------------------------------------- hub
class FrontendHub:
    """The orchestrator side: one pipe per front-end process."""

    def __init__(self, srv, n: int):
        self.srv = srv
        self.n = n
        self.conns: Dict[int, _Conn] = {}
        self.procs: List[mp.Process] = []

    # respawns of one front end within RESPAWN_WINDOW_S before the hub gives up and
    # shuts the server down (a crash loop must not leave a healthy-looking hub that
    # nothing listens for)
    MAX_RESPAWNS = 5
    RESPAWN_WINDOW_S = 60.0

    def start(self) -> None:
        self.srv.hub = self
        self.procs = [None] * self.n
        self._respawns: Dict[int, List[float]] = {}
        for wid in range(self.n):
            self._spawn(wid)

    def _spawn(self, wid: int) -> None:
        ctx = mp.get_context("spawn")
        loop = asyncio.get_running_loop()
        a, b = ctx.Pipe(duplex=True)
        p = ctx.Process(target=frontend_main, args=(wid, self.srv.cfg, self._state(), b), daemon=True,
                        name=f"xgs-frontend{wid}")
        p.start()
        b.close()
        self.procs[wid] = p
        self.conns[wid] = _Conn(a, loop, lambda msgs, w=wid: self._on_msgs(w, msgs), f"hub-frontend{wid}")

    def _front_end_lost(self, wid: int) -> None:
        """An unexpected front-end exit: its clients' sockets died with it, so every
        request it admitted is cancelled (queued ones leave the queue, running ones
        are aborted in their engine -- no decoding for clients that are gone); then a
        fresh front end takes the port share (bounded respawns, else shut down)."""
        srv = self.srv
        lost = [rid for rid, r in list(srv.queued.items()) + list(srv.inflight.items())
                if getattr(r, "remote_wid", None) == wid]
        for rid in lost:
            srv.streamer.discard(rid)
            srv.cancel(rid)
        log.error("front end %d exited: cancelled %d of its requests", wid, len(lost))
        now = time.monotonic()
        hist = [t for t in self._respawns.get(wid, []) if now - t < self.RESPAWN_WINDOW_S]
        if len(hist) >= self.MAX_RESPAWNS:
            log.error("front end %d keeps exiting (%d respawns in %.0f s): shutting down", wid, len(hist),
                      self.RESPAWN_WINDOW_S)
            os.kill(os.getpid(), signal.SIGTERM)
            return
        self._respawns[wid] = hist + [now]
        p = self.procs[wid]
        if p is not None:
            p.join(0.1)
        self._spawn(wid)

    def _state(self) -> dict:
        s = self.srv
        return {"model_name": s.model_name, "model_info": s.model_info, "cfg": s.cfg}

    def broadcast_state(self) -> None:
        st = self._state()
        for c in self.conns.values():
            c.send(("state", st))

    def send(self, wid: int, msg: tuple) -> None:
        c = self.conns.get(wid)
        if c is not None:
            c.send(msg)

    def send_result(self, wid: int, sreq, fut: asyncio.Future) -> None:
        if fut.cancelled():
            return
        e = fut.exception()
        if e is not None:
            self.send(wid, ("res", sreq.id, False, error_to_tuple(e)))
            return
        r = sreq
        self.send(wid, ("res", sreq.id, True, {
            "id": r.id, "text": r.text, "finish_reason": r.finish_reason.value if r.finish_reason else "stop",
            "prompt_tokens": r.prompt_tokens, "completion_tokens": r.completion_tokens,
            "embedding": r.embedding, "logprobs": list(r.logprobs)}))

    def _on_msgs(self, wid: int, msgs: List[tuple]) -> None:
        srv = self.srv
        m = srv.metrics
        for msg in msgs:
            op = msg[0]
            if op == "admit":
                _, rid, kind, ids, params, prio, stream, sse_native = msg
                try:
                    srv.admit(kind, ids, params, prio, stream=stream, rid=rid, sse_native=sse_native,
                              remote=(self, wid))
                    self.send(wid, ("admitted", rid, True, None))
                except Exception as e:  # noqa: BLE001 - every rejection goes back to the client
                    self.send(wid, ("admitted", rid, False, error_to_tuple(e)))
            elif op == "cancel":  # client gone / caller timeout: drop the stream, abort the sequence
                srv.streamer.disconnect(msg[1])
            elif op == "rpc":
                asyncio.get_running_loop().create_task(self._rpc(wid, msg[1], msg[2], msg[3]))
            elif op == "m":  # front-end HTTP metrics: (kind, args)
                getattr(m, msg[1])(*msg[2])
            elif op == "eof":
                self.conns.pop(wid, None)
                if getattr(self, "stopping", False):
                    log.info("front end %d stopped", wid)
                else:
                    self._front_end_lost(wid)

    # admin calls whose bad input is a 400 on the single-process server (app.py)
    _INVALID = {"areload_config": "config", "swap_model": "model", "add_replicas": "replicas",
                "remove_replicas": "replicas"}

    async def _rpc(self, wid: int, cid: int, name: str, args: tuple) -> None:
        from ..core.errors import ConfigError
        try:
            res = await getattr(self.srv, name)(*args)
            self.send(wid, ("rpc", cid, True, res))
        except (ValueError, ConfigError) as e:
            field = self._INVALID.get(name)
            err = ApiValidationError(ValidationError.invalid_parameter(field, str(e))) if field else e
            self.send(wid, ("rpc", cid, False, error_to_tuple(err)))
        except Exception as e:  # noqa: BLE001
            self.send(wid, ("rpc", cid, False, error_to_tuple(e)))

    def stop(self, timeout: float = 10.0) -> None:
        self.stopping = True  # front-end EOFs from here on are the requested shutdown
        for c in self.conns.values():
            c.send(("stop",))
            c.close()
        t_end = time.monotonic() + timeout
        for p in self.procs:
            if p is None:
                continue
            p.join(max(0.1, t_end - time.monotonic()))
            if p.is_alive():
                p.terminate()
                p.join(2.0)


async def run_hub(srv, n: int) -> None:
    """The serving process with N front ends: start the replicas, then the front
    ends (they bind the port with SO_REUSEPORT), run until SIGINT / SIGTERM, then
    shut down gracefully (front ends first: no new requests)."""
    await srv.start()
    hub = FrontendHub(srv, n)
    hub.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, stop.set)
    log.info("serving on %s:%d through %d front-end processes", srv.cfg.api.host, srv.cfg.api.port, n)
    await stop.wait()
    await asyncio.to_thread(hub.stop)
    await srv.shutdown(drain_timeout=1.0)


# ---------------------------------------------------------------------------- front end
class _ForwardMetrics:
    """The handlers' `srv.metrics` calls, forwarded to the hub's collector; Req 5.1
    delivery samples are aggregated per loop iteration."""

    def __init__(self, client: "FrontendClient"):
        self._c = client

    def request_started(self):
        self._c.send(("m", "request_started", ()))

    def request_finished(self):
        self._c.send(("m", "request_finished", ()))

    def record_request(self, endpoint, status, dur):
        self._c.send(("m", "record_request", (endpoint, status, dur)))

    def record_error(self, code):
        self._c.send(("m", "record_error", (code,)))

    def record_delivery(self, s: float, n: int = 1):
        self._c.send(("m", "record_delivery", (s, n)))


class _ProxyRequest:
    """Front-end view of an admitted request (the handlers' ServerRequest)."""

    def __init__(self, rid: str, stream: bool, sse_native: bool, loop):
        self.id = rid
        self.stream = stream
        self.sse_native = sse_native
        self.wire = None
        self.qspan = None
        self.future: Optional[asyncio.Future] = None if stream else loop.create_future()
        self.sender = self.token_stream = None


class _RawToken:
    """A pre-encoded native SSE token event (queued until the handler switches the
    stream to direct socket writes)."""
    type = "token"

    def __init__(self, body: bytes, t_tokens: float):
        self._body = body
        self.t_tokens = t_tokens

    def sse(self) -> bytes:
        return self._body


class _Result:
    def __init__(self, d: dict):
        self.id = d["id"]
        self.text = d["text"]
        self.finish_reason = FinishReason(d["finish_reason"])
        self.prompt_tokens = d["prompt_tokens"]
        self.completion_tokens = d["completion_tokens"]
        self.embedding = d["embedding"]
        self.logprobs = d["logprobs"]

    def usage(self) -> Usage:
        return Usage.new(self.prompt_tokens, self.completion_tokens)


class FrontendClient:
    """InferenceServer's handler interface inside a front-end process."""

    def __init__(self, wid: int, state: dict, conn):
        self.wid = wid
        self._conn_raw = conn
        self.conn: Optional[_Conn] = None
        self.metrics = _ForwardMetrics(self)
        self.streamer = TokenStreamer()
        self.streamer.on_disconnect = self.cancel
        self.reqs: Dict[str, _ProxyRequest] = {}
        self._pending: Dict[Any, asyncio.Future] = {}
        self._cids = itertools.count()
        self.accepting = False
        self.replicas: dict = {}
        self.inflight = self.reqs
        self._deliv = [0.0, 0, False]  # sum of delays, count, flush armed
        self._apply_state(state)

    # ---- state
    def _apply_state(self, st: dict) -> None:
        from .. import _runtime as R
        from .orchestrator import InferenceServer
        self.cfg = st["cfg"]
        self.model_name = st["model_name"]
        self.model_info = st["model_info"]
        self.validator = R.RequestValidator(InferenceServer._vcfg(self.cfg))
        self.tokenizer = self._build_tokenizer()

    def _build_tokenizer(self):
        from ..engine.tokenizer import SyntheticTokenizer, load_tokenizer
        w = self.cfg.worker
        info = self.model_info
        if w.mock:
            return SyntheticTokenizer(info.get("vocab_size", 1000), 1, info.get("eos_token_ids", [2]))
        from ..models import get_config
        return load_tokenizer(get_config(w.checkpoint or w.model), w.checkpoint)

    # ---- lifecycle (build_app's startup / cleanup hooks)
    async def start(self) -> None:
        self.loop = asyncio.get_running_loop()
        self.conn = _Conn(self._conn_raw, self.loop, self._on_msgs, f"frontend{self.wid}-reader")
        self.accepting = True

    async def shutdown(self, drain_timeout: float = 1.0) -> None:
        self.accepting = False
        if self.conn is not None:
            self.conn.close(1.0)

    def send(self, msg: tuple) -> None:
        if self.conn is not None:
            self.conn.send(msg)

    # ---- local work: validation and tokenization
    def validate_generate(self, prompt, max_tokens, temperature, top_p) -> None:
        from .orchestrator import InferenceServer
        InferenceServer._raise_validation(self.validator.validate_generate(prompt, max_tokens, temperature, top_p))

    def validate_chat(self, contents, max_tokens, temperature, top_p) -> None:
        from .orchestrator import InferenceServer
        InferenceServer._raise_validation(self.validator.validate_chat(contents, max_tokens, temperature, top_p))

    def validate_embeddings(self, inputs) -> None:
        from .orchestrator import InferenceServer
        InferenceServer._raise_validation(self.validator.validate_embeddings(inputs))

    def encode(self, text: str) -> List[int]:
        return self.tokenizer.encode(text)

    # ---- hub calls
    async def aadmit(self, kind, prompt_ids, params, priority=1, stream: bool = False, rid: Optional[str] = None,
                     sse_native: bool = False) -> _ProxyRequest:
        from ..core.types import new_request_id
        rid = rid or new_request_id()
        p = _ProxyRequest(rid, stream, sse_native, self.loop)
        if stream:
            p.sender, p.token_stream = self.streamer.create_stream(rid)
        self.reqs[rid] = p
        fut = self.loop.create_future()
        self._pending[("a", rid)] = fut
        self.send(("admit", rid, kind, list(prompt_ids), params, int(priority), bool(stream), bool(sse_native)))
        ok, err = await fut
        if not ok:
            self.reqs.pop(rid, None)
            self.streamer.discard(rid)
            raise RemoteApiError(*err)
        return p

    def cancel(self, rid: str) -> None:
        self.send(("cancel", rid))
        p = self.reqs.pop(rid, None)
        if p is not None and p.future is not None and not p.future.done():
            p.future.cancel()

    async def _call(self, name: str, *args):
        cid = next(self._cids)
        fut = self.loop.create_future()
        self._pending[("r", cid)] = fut
        self.send(("rpc", cid, name, args))
        ok, res = await fut
        if not ok:
            raise RemoteApiError(*res)
        return res

    async def astats(self) -> dict:
        return await self._call("astats")

    async def ahealth(self) -> dict:
        return await self._call("ahealth")

    async def ametrics_text(self) -> str:
        return await self._call("ametrics_text")

    async def areload_config(self, patch) -> dict:
        return await self._call("areload_config", patch)

    async def acfg(self) -> dict:
        return await self._call("acfg")

    async def amodel_state(self) -> dict:
        return await self._call("amodel_state")

    async def areplica_state(self) -> dict:
        return await self._call("areplica_state")

    async def swap_model(self, patch) -> dict:
        return await self._call("swap_model", patch)

    async def add_replicas(self, count, gpus=None) -> dict:
        return await self._call("add_replicas", count, gpus)

    async def remove_replicas(self, ids=None, count=1) -> dict:
        return await self._call("remove_replicas", ids, count)

    # ---- hub -> front end
    def _on_msgs(self, msgs: List[tuple]) -> None:
        reqs = self.reqs
        now = time.monotonic()
        dsum, dn = 0.0, 0
        for msg in msgs:
            op = msg[0]
            if op == "tok":
                _, rid, chunk, t_tok = msg
                p = reqs.get(rid)
                if p is None:
                    continue
                w = p.wire
                if w is not None:
                    if w.is_closing():
                        continue
                    if w.get_write_buffer_size() > WIRE_MAX_BUFFERED:  # client not reading: cut the stream
                        p.wire = None
                        self.metrics.record_error("slow_consumer")
                        self.streamer.fail_stream(rid, "client is not reading the stream", "slow_consumer")
                        self.cancel(rid)
                        continue
                    w.write(chunk)
                    if t_tok:
                        dsum += now - t_tok
                        dn += 1
                elif p.sender is not None:
                    p.sender.send(_RawToken(_unframe(chunk), t_tok))
            elif op == "ev":
                p = reqs.get(msg[1])
                if p is not None and p.sender is not None:
                    from .orchestrator import ev_from_tuple
                    p.sender.send(ev_from_tuple(msg[2]))
            elif op == "close":
                p = reqs.pop(msg[1], None)
                if p is not None and p.sender is not None:
                    self.streamer._senders.pop(msg[1], None)
                    p.sender.close()
            elif op == "res":
                _, rid, ok, payload = msg
                p = reqs.pop(rid, None)
                if p is not None and p.future is not None and not p.future.done():
                    if ok:
                        p.future.set_result(_Result(payload))
                    else:
                        p.future.set_exception(RemoteApiError(*payload))
            elif op == "admitted":
                fut = self._pending.pop(("a", msg[1]), None)
                if fut is not None and not fut.done():
                    fut.set_result((msg[2], msg[3]))
            elif op == "rpc":
                fut = self._pending.pop(("r", msg[1]), None)
                if fut is not None and not fut.done():
                    fut.set_result((msg[2], msg[3]))
            elif op == "state":
                self._apply_state(msg[1])
            elif op in ("stop", "eof"):
                os.kill(os.getpid(), signal.SIGINT)  # web.run_app's graceful exit
        if dn:  # Req 5.1 delay of the tokens written now (mean of this batch, weighted by count)
            self.metrics.record_delivery(dsum / dn, dn)


from .orchestrator import WIRE_MAX_BUFFERED  # noqa: E402  (shared slow-consumer bound)


def frontend_main(wid: int, cfg, state: dict, conn) -> None:
    """Entry point of a front-end process: the same aiohttp app, bound with
    SO_REUSEPORT next to its siblings, over a FrontendClient."""
    import sys
    from aiohttp import web
    from .app import build_app
    logging.basicConfig(level=os.environ.get("XGS_LOG_LEVEL", "WARNING"),
                        format=f"[frontend {wid}] %(levelname)s %(message)s")
    sys.setswitchinterval(0.0005)
    client = FrontendClient(wid, state, conn)
    app = build_app(client)
    web.run_app(app, host=cfg.api.host, port=cfg.api.port, reuse_port=True, handler_cancellation=True,
                access_log=None, print=None)
