"""HTTP API (Req 1, requirements.md:26-37; design.md:125-155; Req 11 wire format).

Endpoints
  POST /generate, /chat, /embeddings     reference wire format (core/wire.py)
  GET  /server/stats                     JSON snapshot (Req 8.2)
  GET  /metrics                          Prometheus text (Req 8.1)
  GET  /health                           200 ok|degraded, 503 unhealthy
  POST /admin/config                     hot reload (Req 10.5)
  POST /admin/model                      model hot-swap (Req 13)
  GET|POST /admin/replicas               list / add / remove replicas at runtime (Req 7.5)
  GET  /debug/traces                     recent request spans (Req 8.5)
  POST /v1/completions, /v1/chat/completions, /v1/embeddings, GET /v1/models
                                         OpenAI-compatible aliases

`stream: true` answers with Server-Sent Events: one `token` event per decoded
text delta, then a final `done` (finish_reason + usage) or `error` event
(Properties 13-15). The SSE response is only committed once the first event
exists, so a request that times out in the queue still gets a real 408. A
client disconnect aborts the sequence in its engine (Req 5.4).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from typing import Optional

from aiohttp import web

from ..core.errors import ApiError, ApiInternal, ApiValidationError, ConfigError, ValidationError
from ..core.types import Priority
from ..core.wire import (ChatChoice, ChatMessage, ChatRequest, ChatResponse, EmbeddingData, EmbeddingsRequest,
                         EmbeddingsResponse, FinishReason, GenerateChoice, GenerateRequest, GenerateResponse, Role,
                         TokenEvent, Usage)
from ..engine.request import RequestType, SamplingParams
from ..obs import trace
from .orchestrator import InferenceServer, ServerRequest, sse_chunk

log = logging.getLogger("xgserve.http")

SERVER_KEY = web.AppKey("server", InferenceServer)


def _json(data, status: int = 200, headers=None) -> web.Response:
    return web.Response(text=json.dumps(data, separators=(",", ":")), status=status,
                        content_type="application/json", headers=headers)


def _error_response(e: ApiError) -> web.Response:
    headers = None
    if e.status == 503:
        headers = {"Retry-After": str(max(1, int(round(e.retry_after or 1))))}
    return _json(e.to_response(), status=e.status, headers=headers)


@web.middleware
async def error_middleware(request: web.Request, handler):
    srv: InferenceServer = request.app[SERVER_KEY]
    t0 = time.monotonic()
    endpoint = request.match_info.route.resource.canonical if request.match_info.route.resource else request.path
    status = 500
    srv.metrics.request_started()
    try:
        resp = await handler(request)
        status = resp.status
        return resp
    except ApiError as e:
        status = e.status
        srv.metrics.record_error(e.code)
        return _error_response(e)
    except ValidationError as e:
        status = 400
        srv.metrics.record_error(e.kind)
        return _error_response(ApiValidationError(e))
    except web.HTTPException as e:
        status = e.status
        raise
    except asyncio.CancelledError:
        status = 499
        raise
    except Exception as e:  # noqa: BLE001
        log.exception("unhandled error on %s", request.path)
        srv.metrics.record_error("internal_error")
        return _error_response(ApiInternal(str(e)))
    finally:
        srv.metrics.request_finished()
        if endpoint not in ("/metrics", "/health"):
            srv.metrics.record_request(endpoint, status, time.monotonic() - t0)


async def _body(request: web.Request) -> bytes:
    return await request.read()


def _params(max_tokens, temperature, top_p, stop, seed=None, ignore_eos=False, logprobs=False) -> SamplingParams:
    return SamplingParams(max_tokens=int(max_tokens), temperature=float(temperature), top_p=float(top_p),
                          stop=list(stop), seed=seed, ignore_eos=ignore_eos, logprobs=logprobs)


async def _await_result(request: web.Request, srv: InferenceServer, sreq: ServerRequest) -> ServerRequest:
    try:
        return await asyncio.wait_for(asyncio.shield(sreq.future), timeout=srv.cfg.api.request_timeout_s)
    except asyncio.TimeoutError:
        srv.cancel(sreq.id)
        from ..core.errors import ApiTimeout
        raise ApiTimeout()
    except asyncio.CancelledError:
        srv.cancel(sreq.id)  # client went away: free the sequence
        raise


async def _sse(request: web.Request, srv: InferenceServer, sreq: ServerRequest, fmt=None) -> web.StreamResponse:
    """Stream TokenEvents. `fmt(ev) -> bytes|None` re-encodes for the OpenAI aliases."""
    it = sreq.token_stream.__aiter__()
    resp: Optional[web.StreamResponse] = None
    sspan = trace.start_span("stream", parent=sreq.qspan, request_id=sreq.id)
    try:
        first = await asyncio.wait_for(it.__anext__(), timeout=srv.cfg.api.request_timeout_s)
        if first.type == "error" and first.code == "timeout":
            from ..core.errors import ApiTimeout
            raise ApiTimeout()
        if first.type == "error" and first.code in ("shutting_down", "no_replica"):
            from .orchestrator import ServiceUnavailable
            raise ServiceUnavailable(first.message, code=first.code)
        resp = web.StreamResponse(status=200, headers={"Content-Type": "text/event-stream",
                                                       "Cache-Control": "no-cache", "X-Request-Id": sreq.id})
        await resp.prepare(request)
        batch = [first] + sreq.token_stream.take_ready()
        n = 0
        while True:
            # coalesce whatever is queued into one write (one wake-up per backlog, not per token)
            data = b"".join(d for d in ((e.sse() if fmt is None else fmt(e)) for e in batch) if d)
            if data:
                await resp.write(data)
                now = time.monotonic()
                for e in batch:
                    t_tok = getattr(e, "t_tokens", 0.0)
                    if t_tok:
                        srv.metrics.record_delivery(now - t_tok)
            n += len(batch)
            if batch[-1].type in ("done", "error"):
                break
            if (sreq.sse_native and sreq.wire is None and request.transport is not None
                    and resp.headers.get("Transfer-Encoding", "").lower() == "chunked"):
                # (the wire bytes are pre-framed HTTP/1.1 chunks: an HTTP/1.0 client gets an
                # unchunked, close-delimited body, so it stays on the queued resp.write path)
                # the response has started (headers flushed): from here on the server's
                # output handler writes this stream's token chunks straight to the
                # socket; only the final done / error event comes through the queue.
                # Events queued meanwhile go out first, in order, in this same step.
                tail = sreq.token_stream.take_ready()
                toks = [e for e in tail if e.type == "token"]
                if toks:
                    request.transport.write(b"".join(sse_chunk(e) for e in toks))
                    n += len(toks)
                sreq.wire = request.transport
                rest = [e for e in tail if e.type != "token"]
                if rest:
                    batch = rest
                    continue
            ev = await it.__anext__()
            batch = [ev] + sreq.token_stream.take_ready()
        if fmt is not None:
            await resp.write(b"data: [DONE]\n\n")
        await resp.write_eof()
        trace.end_span(sspan, events=n)
        return resp
    except StopAsyncIteration:
        if resp is not None:
            await resp.write_eof()
            return resp
        raise ApiInternal("stream closed")
    except asyncio.TimeoutError:
        srv.cancel(sreq.id)
        from ..core.errors import ApiTimeout
        raise ApiTimeout()
    except (ConnectionResetError, asyncio.CancelledError) as e:
        srv.streamer.disconnect(sreq.id)  # -> srv.cancel -> engine abort (Req 5.4)
        trace.end_span(sspan, disconnected=True)
        if isinstance(e, asyncio.CancelledError):
            raise
        return resp
    except Exception as e:
        if resp is not None and type(e).__name__ in ("ClientConnectionResetError", "ClientConnectionError"):
            srv.streamer.disconnect(sreq.id)
            return resp
        raise


# ---------------------------------------------------------------------- core endpoints
async def handle_generate(request: web.Request) -> web.StreamResponse:
    srv: InferenceServer = request.app[SERVER_KEY]
    with trace.span("validate", endpoint="/generate"):
        req = GenerateRequest.parse(await _body(request))
        srv.validate_generate(req.prompt, req.max_tokens, req.temperature, req.top_p)
    ids = srv.encode(req.prompt)
    sp = _params(req.max_tokens, req.temperature, req.top_p, req.stop_sequences, req.seed, req.ignore_eos, req.logprobs)
    sreq = await srv.aadmit(RequestType.Generate, ids, sp, req.priority if req.priority is not None else Priority.Normal,
                     stream=req.stream, sse_native=req.stream)
    if req.stream:
        return await _sse(request, srv, sreq)
    r = await _await_result(request, srv, sreq)
    resp = GenerateResponse.build(srv.model_name, [GenerateChoice(r.text, 0, r.finish_reason)], r.usage(), rid=r.id)
    return _json(resp.to_dict())


async def handle_chat(request: web.Request) -> web.StreamResponse:
    srv: InferenceServer = request.app[SERVER_KEY]
    with trace.span("validate", endpoint="/chat"):
        req = ChatRequest.parse(await _body(request))
        srv.validate_chat([m.content for m in req.messages], req.max_tokens, req.temperature, req.top_p)
    ids = srv.encode(srv.tokenizer.apply_chat_template(req.messages))
    sp = _params(req.max_tokens, req.temperature, req.top_p, req.stop_sequences, req.seed, req.ignore_eos)
    sreq = await srv.aadmit(RequestType.Chat, ids, sp, Priority.Normal, stream=req.stream, sse_native=req.stream)
    if req.stream:
        return await _sse(request, srv, sreq)
    r = await _await_result(request, srv, sreq)
    resp = ChatResponse.build(srv.model_name, [ChatChoice(0, ChatMessage(Role.Assistant, r.text), r.finish_reason)],
                              r.usage(), rid=r.id)
    return _json(resp.to_dict())


async def _embed(srv: InferenceServer, inputs, request) -> tuple:
    srv.validate_embeddings(inputs)
    sreqs = []
    try:
        for t in inputs:
            sreqs.append(await srv.aadmit(RequestType.Embeddings, srv.encode(t), SamplingParams(max_tokens=0),
                                          Priority.Normal))
        done = await asyncio.gather(*[_await_result(request, srv, s) for s in sreqs])
    except BaseException:
        for s in sreqs:
            srv.cancel(s.id)
        raise
    data = [EmbeddingData(list(r.embedding or []), i) for i, r in enumerate(done)]
    return data, Usage.new(sum(r.prompt_tokens for r in done), 0)


async def handle_embeddings(request: web.Request) -> web.Response:
    srv: InferenceServer = request.app[SERVER_KEY]
    req = EmbeddingsRequest.parse(await _body(request))
    data, usage = await _embed(srv, req.into_vec(), request)
    return _json(EmbeddingsResponse(data, req.model or srv.model_name, usage).to_dict())


async def handle_stats(request: web.Request) -> web.Response:
    return _json(await request.app[SERVER_KEY].astats())


async def handle_metrics(request: web.Request) -> web.Response:
    srv: InferenceServer = request.app[SERVER_KEY]
    return web.Response(text=await srv.ametrics_text(), content_type="text/plain",
                        headers={"X-Prometheus-Format": "0.0.4"})


async def handle_health(request: web.Request) -> web.Response:
    h = await request.app[SERVER_KEY].ahealth()
    return _json(h, status=200 if h["status"] != "unhealthy" else 503)


async def handle_traces(request: web.Request) -> web.Response:
    n = int(request.query.get("n", "100"))
    return _json({"spans": trace.recent(n)})


# ---------------------------------------------------------------------- admin
async def handle_admin_config(request: web.Request) -> web.Response:
    srv: InferenceServer = request.app[SERVER_KEY]
    if request.method == "GET":
        return _json(await srv.acfg())
    try:
        patch = json.loads(await _body(request))
        if not isinstance(patch, dict) or not all(isinstance(v, dict) for v in patch.values()):
            raise ValueError("expected {section: {key: value}}")
        applied = await srv.areload_config(patch)
    except (ValueError, ConfigError) as e:
        raise ApiValidationError(ValidationError.invalid_parameter("config", str(e)))
    return _json({"status": "ok", "applied": applied})


async def handle_admin_model(request: web.Request) -> web.Response:
    srv: InferenceServer = request.app[SERVER_KEY]
    if request.method == "GET":
        return _json(await srv.amodel_state())
    try:
        patch = json.loads(await _body(request))
        if not isinstance(patch, dict):
            raise ValueError("expected an object of worker settings, e.g. {\"model\": \"llama3-8b\"}")
        res = await srv.swap_model(patch)
    except (ValueError, ConfigError) as e:
        raise ApiValidationError(ValidationError.invalid_parameter("model", str(e)))
    return _json({"status": "ok", **res})


async def handle_admin_replicas(request: web.Request) -> web.Response:
    """GET: the replica set. POST {"action": "add", "count": n, "gpus": [..]} or
    {"action": "remove", "ids": [..]} / {"action": "remove", "count": n}."""
    srv: InferenceServer = request.app[SERVER_KEY]
    if request.method == "GET":
        return _json(await srv.areplica_state())
    try:
        d = json.loads(await _body(request))
        if not isinstance(d, dict) or d.get("action") not in ("add", "remove"):
            raise ValueError('expected {"action": "add"|"remove", ...}')
        count = d.get("count", 1)
        if not isinstance(count, int) or isinstance(count, bool):
            raise ValueError("count must be an integer")
        if d["action"] == "add":
            gpus = d.get("gpus")
            if gpus is not None and not (isinstance(gpus, list) and all(isinstance(g, int) for g in gpus)):
                raise ValueError("gpus must be a list of integers")
            res = await srv.add_replicas(count, gpus)
        else:
            ids = d.get("ids")
            if ids is not None and not (isinstance(ids, list) and all(isinstance(i, int) for i in ids)):
                raise ValueError("ids must be a list of integers")
            res = await srv.remove_replicas(ids, count)
    except (ValueError, ConfigError) as e:
        raise ApiValidationError(ValidationError.invalid_parameter("replicas", str(e)))
    return _json({"status": "ok", **res})


# ---------------------------------------------------------------------- OpenAI aliases
def _oa_stop(d: dict):
    s = d.get("stop")
    if s is None:
        return d.get("stop_sequences", [])
    return [s] if isinstance(s, str) else s


def _oa_finish(ev: TokenEvent):
    return ev.finish_reason.value if ev.finish_reason != FinishReason.StopSequence else "stop"


async def handle_v1_completions(request: web.Request) -> web.StreamResponse:
    srv: InferenceServer = request.app[SERVER_KEY]
    d = json.loads(await _body(request) or b"{}")
    if not isinstance(d, dict):
        raise ValidationError.invalid_json("invalid type: expected a JSON object")
    p = d.get("prompt")
    if isinstance(p, list) and len(p) == 1 and isinstance(p[0], str):
        p = p[0]
    body = {k: v for k, v in d.items() if k in ("max_tokens", "temperature", "top_p", "stream", "seed", "priority")}
    body["prompt"] = p if p is not None else None
    if body["prompt"] is None:
        body.pop("prompt")
    body["stop_sequences"] = _oa_stop(d)
    req = GenerateRequest.parse(body)
    srv.validate_generate(req.prompt, req.max_tokens, req.temperature, req.top_p)
    sp = _params(req.max_tokens, req.temperature, req.top_p, req.stop_sequences, req.seed)
    sreq = await srv.aadmit(RequestType.Generate, srv.encode(req.prompt), sp,
                     req.priority if req.priority is not None else Priority.Normal, stream=req.stream)
    created = int(time.time())
    if req.stream:
        def fmt(ev: TokenEvent):
            if ev.type == "error":
                return ev.sse()
            ch = {"text": ev.token if ev.type == "token" else "", "index": 0,
                  "finish_reason": _oa_finish(ev) if ev.type == "done" else None}
            return b"data: " + json.dumps({"id": sreq.id, "object": "text_completion", "created": created,
                                           "model": srv.model_name, "choices": [ch]}).encode() + b"\n\n"
        return await _sse(request, srv, sreq, fmt)
    r = await _await_result(request, srv, sreq)
    out = GenerateResponse.build(srv.model_name, [GenerateChoice(r.text, 0, r.finish_reason)], r.usage(),
                                 rid=r.id).to_dict()
    out["choices"][0]["finish_reason"] = "stop" if r.finish_reason == FinishReason.StopSequence else \
        r.finish_reason.value
    return _json(out)


async def handle_v1_chat(request: web.Request) -> web.StreamResponse:
    srv: InferenceServer = request.app[SERVER_KEY]
    d = json.loads(await _body(request) or b"{}")
    if not isinstance(d, dict):
        raise ValidationError.invalid_json("invalid type: expected a JSON object")
    body = {k: v for k, v in d.items() if k in ("messages", "max_tokens", "temperature", "top_p", "stream", "seed")}
    if "max_completion_tokens" in d and "max_tokens" not in body:
        body["max_tokens"] = d["max_completion_tokens"]
    body["stop_sequences"] = _oa_stop(d)
    req = ChatRequest.parse(body)
    srv.validate_chat([m.content for m in req.messages], req.max_tokens, req.temperature, req.top_p)
    sp = _params(req.max_tokens, req.temperature, req.top_p, req.stop_sequences, req.seed)
    sreq = await srv.aadmit(RequestType.Chat, srv.encode(srv.tokenizer.apply_chat_template(req.messages)), sp,
                     Priority.Normal, stream=req.stream)
    created = int(time.time())
    if req.stream:
        def fmt(ev: TokenEvent):
            if ev.type == "error":
                return ev.sse()
            delta = {"content": ev.token} if ev.type == "token" else {}
            ch = {"index": 0, "delta": delta, "finish_reason": _oa_finish(ev) if ev.type == "done" else None}
            return b"data: " + json.dumps({"id": sreq.id, "object": "chat.completion.chunk", "created": created,
                                           "model": srv.model_name, "choices": [ch]}).encode() + b"\n\n"
        return await _sse(request, srv, sreq, fmt)
    r = await _await_result(request, srv, sreq)
    out = ChatResponse.build(srv.model_name, [ChatChoice(0, ChatMessage(Role.Assistant, r.text), r.finish_reason)],
                             r.usage(), rid=r.id).to_dict()
    out["choices"][0]["finish_reason"] = "stop" if r.finish_reason == FinishReason.StopSequence else \
        r.finish_reason.value
    return _json(out)


async def handle_v1_embeddings(request: web.Request) -> web.Response:
    return await handle_embeddings(request)


async def handle_v1_models(request: web.Request) -> web.Response:
    srv: InferenceServer = request.app[SERVER_KEY]
    return _json({"object": "list", "data": [{"id": srv.model_name, "object": "model", "owned_by": "xgserve",
                                              "max_model_len": srv.model_info.get("max_model_len")}]})


# ---------------------------------------------------------------------- app factory
def build_app(srv: InferenceServer) -> web.Application:
    app = web.Application(middlewares=[error_middleware], client_max_size=srv.cfg.api.max_request_size)
    app[SERVER_KEY] = srv
    r = app.router
    r.add_post("/generate", handle_generate)
    r.add_post("/chat", handle_chat)
    r.add_post("/embeddings", handle_embeddings)
    r.add_get("/server/stats", handle_stats)
    r.add_get("/metrics", handle_metrics)
    r.add_get("/health", handle_health)
    r.add_get("/debug/traces", handle_traces)
    r.add_route("*", "/admin/config", handle_admin_config)
    r.add_route("*", "/admin/model", handle_admin_model)
    r.add_route("*", "/admin/replicas", handle_admin_replicas)
    r.add_post("/v1/completions", handle_v1_completions)
    r.add_post("/v1/chat/completions", handle_v1_chat)
    r.add_post("/v1/embeddings", handle_v1_embeddings)
    r.add_get("/v1/models", handle_v1_models)

    async def on_startup(app):
        if not srv.accepting and not srv.replicas:
            await srv.start()

    async def on_cleanup(app):
        await srv.shutdown(drain_timeout=srv.cfg.api.request_timeout_s if srv.inflight else 1.0)

    app.on_startup.append(on_startup)
    app.on_cleanup.append(on_cleanup)
    return app


def serve(srv: InferenceServer) -> None:
    """Blocking: run the HTTP server until SIGINT/SIGTERM, then shut down gracefully."""
    import sys
    # replica reader threads unpickle outputs; they must hand the GIL back to the
    # event loop quickly (token delivery, Req 5.1), not after the default 5 ms
    sys.setswitchinterval(0.0005)
    app = build_app(srv)
    web.run_app(app, host=srv.cfg.api.host, port=srv.cfg.api.port, handler_cancellation=True,
                access_log=None, print=lambda *a: log.info(*a) if a else None)
