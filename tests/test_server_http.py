"""HTTP integration tests against the in-process app with the MockEngine
(SURVEY.md 4.3 "Integration" + "Fault injection"; Properties 2, 3, 8, 13-15,
18, 22, 28-29)."""
from __future__ import annotations

import asyncio
import json
import time

import pytest

from _server_util import mock_config, parse_sse, run_with_client


def _gen(client, **body):
    body.setdefault("prompt", "hello world")
    return client.post("/generate", data=json.dumps(body))


def test_generate_roundtrip():
    async def fn(c, srv):
        r = await _gen(c, max_tokens=8, temperature=0.0)
        assert r.status == 200
        d = await r.json()
        assert d["object"] == "text_completion" and d["model"] == "mock"
        assert len(d["id"]) == 36
        ch = d["choices"][0]
        assert ch["finish_reason"] == "length" and ch["index"] == 0 and isinstance(ch["text"], str)
        u = d["usage"]
        assert u["completion_tokens"] == 8 and u["total_tokens"] == u["prompt_tokens"] + 8
        assert u["prompt_tokens"] == len(srv.encode("hello world"))
        # determinism: same prompt -> same text
        d2 = await (await _gen(c, max_tokens=8)).json()
        assert d2["choices"][0]["text"] == ch["text"]
        return True

    assert run_with_client(mock_config(), fn)


def test_generate_stream_events():
    """Property 13/14: token events carry token+index, final done has finish_reason + usage."""
    async def fn(c, srv):
        r = await _gen(c, max_tokens=6, stream=True)
        assert r.status == 200
        assert r.headers["Content-Type"].startswith("text/event-stream")
        evs = parse_sse(await r.read())
        toks = [e for e in evs if e["type"] == "token"]
        assert evs[-1]["type"] == "done"
        assert evs[-1]["finish_reason"] == "length"
        assert evs[-1]["usage"]["completion_tokens"] == 6
        assert all(isinstance(e["token"], str) and isinstance(e["index"], int) for e in toks)
        assert [e["index"] for e in toks] == sorted(e["index"] for e in toks)
        nonstream = await (await _gen(c, max_tokens=6)).json()
        assert "".join(e["token"] for e in toks) == nonstream["choices"][0]["text"]
        return True

    assert run_with_client(mock_config(), fn)


def test_chat_and_embeddings_and_aliases():
    async def fn(c, srv):
        r = await c.post("/chat", data=json.dumps({"messages": [{"role": "user", "content": "hi"}],
                                                   "max_tokens": 4}))
        d = await r.json()
        assert r.status == 200 and d["object"] == "chat.completion"
        assert d["choices"][0]["message"]["role"] == "assistant"
        r = await c.post("/embeddings", data=json.dumps({"input": ["a b", "c d e"]}))
        d = await r.json()
        assert r.status == 200 and d["object"] == "list" and len(d["data"]) == 2
        assert d["data"][1]["index"] == 1 and d["data"][0]["object"] == "embedding"
        v = d["data"][0]["embedding"]
        assert abs(sum(x * x for x in v) - 1.0) < 1e-4
        r = await c.post("/embeddings", data=json.dumps({"input": "single"}))
        assert len((await r.json())["data"]) == 1
        r = await c.post("/v1/completions", data=json.dumps({"prompt": "x", "max_tokens": 3, "stop": "zz"}))
        assert r.status == 200 and (await r.json())["usage"]["completion_tokens"] == 3
        r = await c.post("/v1/chat/completions", data=json.dumps({"messages": [{"role": "user", "content": "x"}],
                                                                  "max_tokens": 3, "stream": True}))
        evs = parse_sse(await r.read())
        assert evs[-1]["type"] == "[DONE]" and evs[-2]["choices"][0]["finish_reason"] == "length"
        r = await c.get("/v1/models")
        assert (await r.json())["data"][0]["id"] == "mock"
        return True

    assert run_with_client(mock_config(), fn)


@pytest.mark.parametrize("body,code", [
    ("{not json", "invalid_json"),
    (json.dumps({"max_tokens": 3}), "missing_field"),
    (json.dumps({"prompt": "   \t"}), "empty_prompt"),
    (json.dumps({"prompt": "x", "temperature": 2.5}), "invalid_parameter"),
    (json.dumps({"prompt": "x", "top_p": -0.1}), "invalid_parameter"),
    (json.dumps({"prompt": "x", "max_tokens": 5000}), "invalid_parameter"),
    (json.dumps({"prompt": "x", "max_tokens": -1}), "invalid_json"),
    (json.dumps({"prompt": "x", "priority": "Urgent"}), "invalid_json"),
    (json.dumps({"prompt": "x" * 40000}), "token_limit_exceeded"),
])
def test_invalid_requests_400(body, code):
    """Property 2/3: malformed / out-of-range -> 400 with message, type, code."""
    async def fn(c, srv):
        r = await c.post("/generate", data=body)
        d = await r.json()
        assert r.status == 400, d
        e = d["error"]
        assert e["type"] == "invalid_request_error" and e["code"] == code and e["message"].startswith(
            "Validation error: ")
        return True

    assert run_with_client(mock_config(), fn)


def test_priority_spellings_accepted():
    async def fn(c, srv):
        for p in ("High", "low", "Normal"):
            r = await _gen(c, max_tokens=1, priority=p)
            assert r.status == 200
        return True

    assert run_with_client(mock_config(), fn)


def test_queue_full_503_with_retry_after():
    cfg = mock_config(queue={"high_watermark": 2, "low_watermark": 1, "max_queue_size": 2},
                      scheduler={"max_inflight_per_replica": 1}, worker={"mock_latency_ms": 20.0})

    async def fn(c, srv):
        rs = await asyncio.gather(*[_gen(c, max_tokens=5) for _ in range(8)])
        st = [r.status for r in rs]
        assert 503 in st and 200 in st
        bad = [r for r in rs if r.status == 503][0]
        assert bad.headers["Retry-After"] == "1"
        d = await bad.json()
        assert d["error"]["type"] == "rate_limit_error" and d["error"]["code"] == "queue_full"
        return True

    assert run_with_client(cfg, fn)


def test_queue_timeout_408():
    """Property 8: a request waiting longer than the queue timeout gets 408."""
    cfg = mock_config(queue={"request_timeout_s": 0.2}, scheduler={"max_inflight_per_replica": 1},
                      worker={"mock_latency_ms": 20.0})

    async def fn(c, srv):
        first = asyncio.create_task(_gen(c, max_tokens=30))
        await asyncio.sleep(0.05)
        r = await _gen(c, max_tokens=5)
        assert r.status == 408
        d = await r.json()
        assert d["error"]["type"] == "timeout_error" and d["error"]["code"] == "timeout"
        rs = await _gen(c, max_tokens=2, stream=True)  # streaming request timing out in the queue: still 408
        assert rs.status == 408
        assert (await first).status == 200
        return True

    assert run_with_client(cfg, fn)


def test_client_disconnect_aborts_generation():
    """Req 5.4: dropping an SSE connection aborts the sequence in the engine."""
    cfg = mock_config(worker={"mock_latency_ms": 5.0})

    async def fn(c, srv):
        r = await _gen(c, max_tokens=2000, stream=True, ignore_eos=True)
        assert r.status == 200
        await r.content.readline()
        r.close()
        for _ in range(200):
            await asyncio.sleep(0.02)
            eng = srv.replicas[0].engine
            if not srv.inflight and not eng.requests:
                return True
        raise AssertionError(f"still in flight: {list(srv.inflight)}")

    assert run_with_client(cfg, fn)


def test_failure_isolation():
    """Property 22: a failing request errors alone; its batch-mates complete."""
    async def fn(c, srv):
        bad, good = await asyncio.gather(_gen(c, prompt="x __FAIL__ y", max_tokens=4), _gen(c, max_tokens=4))
        assert bad.status == 500
        e = (await bad.json())["error"]
        assert e["type"] == "server_error" and e["code"] == "inference_failed"
        assert good.status == 200
        r = await _gen(c, prompt="__FAIL__", stream=True)
        evs = parse_sse(await r.read())
        assert evs[-1]["type"] == "error" and evs[-1]["code"] == "inference_failed" and "message" in evs[-1]
        return True

    assert run_with_client(mock_config(), fn)


def test_stats_metrics_health():
    async def fn(c, srv):
        await _gen(c, max_tokens=3)
        d = await (await c.get("/server/stats")).json()
        assert d["model"] == "mock" and d["replicas"][0]["healthy"]
        assert d["metrics"]["requests_total"] >= 1 and d["metrics"]["generation_tokens_total"] >= 3
        assert set(d["queue_depth"]) == {"high", "normal", "low", "total"}
        t = await (await c.get("/metrics")).text()
        assert "xgs_requests_total{endpoint=\"/generate\",status=\"200\"} 1" in t
        assert "xgs_ttft_seconds_bucket" in t and "xgs_worker_healthy{worker=\"0\"} 1" in t
        h = await (await c.get("/health")).json()
        assert h["status"] == "ok" and h["replicas_healthy"] == 1
        tr = await (await c.get("/debug/traces")).json()
        assert {"queue", "engine"} <= {s["name"] for s in tr["spans"]}
        return True

    assert run_with_client(mock_config(), fn)


def test_hot_reload_config():
    async def fn(c, srv):
        r = await c.post("/admin/config", data=json.dumps({"scheduler": {"strategy": "round_robin"},
                                                          "queue": {"high_watermark": 1500, "max_queue_size": 3000}}))
        assert r.status == 200, await r.text()
        assert srv.router.strategy == "round_robin" and srv.queue.config().high_watermark == 1500
        r = await c.post("/admin/config", data=json.dumps({"api": {"port": 1}}))
        assert r.status == 400
        r = await c.post("/admin/config", data=json.dumps({"validator": {"max_output_tokens": 4}}))
        assert r.status == 200
        assert (await _gen(c, max_tokens=5)).status == 400
        return True

    assert run_with_client(mock_config(), fn)


def test_model_hot_swap_drains_old():
    """Property 28: in-flight requests finish on the old model; new ones see the new model."""
    cfg = mock_config(worker={"mock_latency_ms": 5.0})

    async def fn(c, srv):
        old = asyncio.create_task(_gen(c, max_tokens=40))
        await asyncio.sleep(0.05)
        r = await c.post("/admin/model", data=json.dumps({"model": "mock-b"}))
        assert r.status == 200, await r.text()
        assert (await r.json())["model"] == "mock-b"
        d_old = await (await old).json()
        assert d_old["usage"]["completion_tokens"] == 40
        d_new = await (await _gen(c, max_tokens=2)).json()
        assert d_new["model"] == "mock-b"
        for _ in range(100):
            if len(srv.replicas) == 1:
                break
            await asyncio.sleep(0.02)
        assert list(srv.replicas) == [1]
        return True

    assert run_with_client(cfg, fn)


def test_hot_swap_failure_keeps_old_model():
    """Property 29: a failed swap leaves the original model serving without interruption."""
    async def fn(c, srv):
        r = await c.post("/admin/model", data=json.dumps({"model": "no-such-model", "mock": False}))
        assert r.status in (400, 500)
        assert (await (await _gen(c, max_tokens=2)).json())["model"] == "mock"
        return True

    assert run_with_client(mock_config(), fn)


def test_static_batching_mode():
    cfg = mock_config(batcher={"mode": "static", "max_batch_size": 4, "batch_timeout_ms": 30.0})

    async def fn(c, srv):
        rs = await asyncio.gather(*[_gen(c, max_tokens=2) for _ in range(4)])
        assert all(r.status == 200 for r in rs)
        assert srv.batcher.batches_formed >= 1
        return True

    assert run_with_client(cfg, fn)


def test_hung_replica_detected_and_requests_redispatched():
    """Req 9.4: a replica that stops heartbeating leaves the pool; every request it
    held that had not started streaming is reassigned, so all of them succeed."""
    cfg = mock_config(worker={"replicas": 2, "mock_latency_ms": 2.0},
                      scheduler={"heartbeat_timeout_s": 0.5, "restart_failed": False, "strategy": "round_robin"})

    async def fn(c, srv):
        srv.replicas[0].inject_hang()
        t0 = time.monotonic()
        rs = await asyncio.gather(*[_gen(c, max_tokens=3) for _ in range(6)])
        assert [r.status for r in rs] == [200] * 6
        h = await (await c.get("/health")).json()
        assert h["status"] == "degraded" and h["replicas_healthy"] == 1
        assert time.monotonic() - t0 < 5.0
        assert (await _gen(c, max_tokens=2)).status == 200
        srv.replicas[0].engine.hang = False
        return True

    assert run_with_client(cfg, fn)


def test_collective_timeout_fails_step_and_restarts_replica():
    """A TP peer-wait timeout (CustomAllReduceTimeout) is fatal for the replica: the
    in-flight request gets an error (never stale numbers), the replica is restarted
    and serves again."""
    cfg = mock_config(worker={"replicas": 1, "mock_latency_ms": 5.0},
                      scheduler={"restart_failed": True, "max_restarts": 2, "health_check_interval_s": 0.1})

    async def fn(c, srv):
        assert (await _gen(c, max_tokens=2)).status == 200
        old = srv.replicas[0]
        old.inject_collective_timeout()
        r = await _gen(c, max_tokens=50)
        assert r.status == 500, await r.text()
        t0 = time.monotonic()
        while srv.replicas[0] is old or not srv.replicas[0].ready.is_set():
            assert time.monotonic() - t0 < 10.0
            await asyncio.sleep(0.05)
        assert srv.replicas[0].restarts == 1
        for _ in range(50):
            r = await _gen(c, max_tokens=2)
            if r.status == 200:
                break
            await asyncio.sleep(0.1)
        assert r.status == 200
        return True

    assert run_with_client(cfg, fn)


def test_runtime_add_remove_replicas_without_dropping_traffic():
    """Req 7.5: POST /admin/replicas adds and removes replicas while requests flow;
    every request succeeds and the new replica takes traffic."""
    cfg = mock_config(worker={"replicas": 2, "mock_latency_ms": 2.0}, scheduler={"strategy": "round_robin"})

    async def fn(c, srv):
        stop = asyncio.Event()
        statuses = []

        async def traffic():
            while not stop.is_set():
                rs = await asyncio.gather(*[_gen(c, max_tokens=4) for _ in range(4)])
                statuses.extend(r.status for r in rs)

        task = asyncio.create_task(traffic())
        await asyncio.sleep(0.1)
        r = await c.post("/admin/replicas", data=json.dumps({"action": "add", "count": 1}))
        d = await r.json()
        assert r.status == 200, d
        new_id = d["added"][0]
        assert sorted(d["replicas"]) == [0, 1, new_id]
        for _ in range(200):
            if srv.replicas[new_id].loop.steps > 0:
                break
            await asyncio.sleep(0.05)
        assert srv.replicas[new_id].loop.steps > 0  # the new replica serves traffic
        r = await c.post("/admin/replicas", data=json.dumps({"action": "remove", "ids": [0]}))
        d = await r.json()
        assert r.status == 200, d
        assert sorted(d["replicas"]) == [1, new_id]
        await asyncio.sleep(0.3)
        stop.set()
        await task
        assert statuses and all(st == 200 for st in statuses), statuses
        h = await (await c.get("/health")).json()
        assert h["status"] == "ok" and h["replicas_total"] == 2
        g = await (await c.get("/admin/replicas")).json()
        assert sorted(g["routable"]) == [1, new_id]
        # cannot remove every replica; bad ids are rejected
        r = await c.post("/admin/replicas", data=json.dumps({"action": "remove", "ids": [1, new_id]}))
        assert r.status == 400
        r = await c.post("/admin/replicas", data=json.dumps({"action": "remove", "ids": [99]}))
        assert r.status == 400
        for _ in range(200):
            if 0 not in srv.replicas:
                break
            await asyncio.sleep(0.05)
        assert 0 not in srv.replicas  # drained and stopped
        return True

    assert run_with_client(cfg, fn)


def test_degradation_rejects_low_priority():
    async def fn(c, srv):
        p = {"v": 0.92}
        srv.memory_pressure = lambda: p["v"]  # what the replicas' KV usage would report
        srv.update_degradation()
        r = await _gen(c, max_tokens=1, priority="Low")
        assert r.status == 503 and r.headers.get("Retry-After")
        assert (await _gen(c, max_tokens=1, priority="High")).status == 200
        p["v"] = 0.99
        srv.update_degradation()
        assert (await _gen(c, max_tokens=1, priority="High")).status == 503
        p["v"] = 0.1
        srv.update_degradation()
        assert (await _gen(c, max_tokens=1)).status == 200
        return True

    cfg = mock_config()
    assert run_with_client(cfg, fn)


def test_token_delivery_delay_is_measured():
    """Req 5.1: the server records token-on-host -> SSE-write delay per token event."""
    async def fn(c, srv):
        r = await c.post("/generate", data=json.dumps({"prompt": "hello", "max_tokens": 8, "stream": True}))
        assert r.status == 200
        await r.read()
        st = await (await c.get("/server/stats")).json()
        d = st["metrics"]["token_delivery_ms"]
        assert d["n"] >= 7 and 0 <= d["p50"] <= d["p99"] <= d["max"]
        assert d["p99"] < 1000.0
        text = await (await c.get("/metrics")).text()
        assert "xgs_token_delivery_seconds_count" in text
        return True

    assert run_with_client(mock_config(), fn)
