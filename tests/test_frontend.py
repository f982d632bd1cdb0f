"""Sharded HTTP front end (api.frontends > 1, server/frontend.py): the serving
process keeps the control plane, N front-end processes (SO_REUSEPORT) own the
client sockets. Every endpoint must behave exactly as the single-process server:
streams (native and OpenAI), plain results, 400 / 503 errors raised in either
process, embeddings, stats / metrics / admin calls, client disconnect -> abort,
and the native SSE bytes equal core.wire's encoding."""
from __future__ import annotations

import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import time

import aiohttp
import pytest

from _server_util import parse_sse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def server():
    port = _free_port()
    cmd = [sys.executable, "-m", "xgserve", "serve", "--host", "127.0.0.1", "--port", str(port), "--mock",
           "--replicas", "2", "--frontends", "3", "--log-level", "WARNING", "--set", "worker.mock_latency_ms=3",
           "--set", "queue.max_queue_size=64", "--set", "queue.high_watermark=48", "--set", "queue.low_watermark=8"]
    p = subprocess.Popen(cmd, cwd=ROOT, start_new_session=True, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    url = f"http://127.0.0.1:{port}"

    async def ready():
        t_end = time.monotonic() + 120
        async with aiohttp.ClientSession() as s:
            while time.monotonic() < t_end:
                try:
                    async with s.get(url + "/health") as r:
                        if r.status == 200:
                            return True
                except aiohttp.ClientError:
                    pass
                await asyncio.sleep(0.3)
        return False

    try:
        assert asyncio.run(ready()), "server did not come up"
        yield url
    finally:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait(10)


def _run(coro):
    return asyncio.run(coro)


def test_stream_and_plain_agree(server):
    async def main():
        async with aiohttp.ClientSession() as s:
            body = {"prompt": "the quick brown fox", "max_tokens": 24, "stream": True, "ignore_eos": True}
            async with s.post(server + "/generate", json=body) as r:
                assert r.status == 200 and r.headers["Content-Type"].startswith("text/event-stream")
                evs = parse_sse(await r.read())
            body["stream"] = False
            async with s.post(server + "/generate", json=body) as r:
                plain = await r.json()
        return evs, plain

    evs, plain = _run(main())
    toks = [e for e in evs if e["type"] == "token"]
    assert evs[-1]["type"] == "done" and evs[-1]["usage"]["completion_tokens"] == 24
    assert "".join(e["token"] for e in toks) == plain["choices"][0]["text"]  # deterministic mock
    idx = [e["index"] for e in toks]
    assert idx == sorted(idx) and len(set(idx)) == len(idx) and idx[-1] == 23


def test_many_concurrent_streams_land_on_every_front_end(server):
    async def one(s, i):
        body = {"prompt": f"stream {i}", "max_tokens": 16, "stream": True, "ignore_eos": True}
        async with s.post(server + "/generate", json=body) as r:
            evs = parse_sse(await r.read())
        return evs

    async def main():
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0, force_close=True)) as s:
            return await asyncio.gather(*[one(s, i) for i in range(40)])

    for evs in _run(main()):
        assert evs[-1]["type"] == "done" and evs[-1]["usage"]["completion_tokens"] == 16


def test_errors_from_front_end_and_hub(server):
    async def main():
        out = {}
        async with aiohttp.ClientSession() as s:
            async with s.post(server + "/generate", json={"prompt": "   ", "max_tokens": 4}) as r:
                out["empty"] = (r.status, await r.json())          # validated in the front end
            async with s.post(server + "/generate", data=b"{nope") as r:
                out["json"] = (r.status, await r.json())
            async with s.post(server + "/generate", json={"prompt": "x" * 40000, "max_tokens": 4}) as r:
                out["long"] = (r.status, await r.json())
            async with s.post(server + "/admin/config", json={"queue": {"bogus": 1}}) as r:
                out["cfg"] = (r.status, await r.json())             # rejected in the hub
        return out

    out = _run(main())
    assert out["empty"][0] == 400 and out["empty"][1]["error"]["code"] == "empty_prompt"
    assert out["json"][0] == 400
    assert out["long"][0] == 400 and out["long"][1]["error"]["type"] == "invalid_request_error"
    assert out["cfg"][0] == 400 and out["cfg"][1]["error"]["code"] == "invalid_parameter"


def test_queue_full_is_503_with_retry_after(server):
    async def main():
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0)) as s:
            async def post():
                async with s.post(server + "/generate", json={"prompt": "q", "max_tokens": 1500,
                                                              "ignore_eos": True}) as r:
                    return r.status, dict(r.headers)
            tasks = [asyncio.create_task(post()) for _ in range(240)]
            res = await asyncio.gather(*tasks)
        return res

    res = _run(main())
    codes = [c for c, _ in res]
    assert 503 in codes and 200 in codes, codes
    assert all("Retry-After" in h for c, h in res if c == 503)


def test_embeddings_chat_openai_and_admin(server):
    async def main():
        out = {}
        async with aiohttp.ClientSession() as s:
            async with s.post(server + "/embeddings", json={"input": ["a b", "c d e"]}) as r:
                out["emb"] = (r.status, await r.json())
            async with s.post(server + "/chat", json={"messages": [{"role": "user", "content": "hi"}],
                                                      "max_tokens": 6, "stream": True}) as r:
                out["chat"] = parse_sse(await r.read())
            async with s.post(server + "/v1/completions", json={"prompt": "hi", "max_tokens": 5, "stream": True}) as r:
                out["oa"] = (await r.read()).decode()
            async with s.get(server + "/server/stats") as r:
                out["stats"] = await r.json()
            async with s.get(server + "/metrics") as r:
                out["metrics"] = await r.text()
            async with s.get(server + "/admin/replicas") as r:
                out["reps"] = await r.json()
            async with s.get(server + "/admin/model") as r:
                out["model"] = await r.json()
        return out

    out = _run(main())
    assert out["emb"][0] == 200 and len(out["emb"][1]["data"]) == 2
    assert out["chat"][-1]["type"] == "done"
    assert out["oa"].rstrip().endswith("data: [DONE]") and "text_completion" in out["oa"]
    m = out["stats"]["metrics"]
    assert m["requests_total"] >= 3 and m["generation_tokens_total"] > 0
    assert m["token_delivery_ms"]["n"] > 0  # delivery delays reported by the front ends
    assert "xgs_requests_total" in out["metrics"]
    assert len(out["reps"]["routable"]) == 2 and out["model"]["model"]


def test_client_disconnect_aborts(server):
    async def main():
        async with aiohttp.ClientSession() as s:
            r = await s.post(server + "/generate", json={"prompt": "abort me", "max_tokens": 4000,
                                                         "stream": True, "ignore_eos": True})
            await r.content.readline()
            r.close()  # client goes away mid-stream
            await asyncio.sleep(1.0)
            async with s.get(server + "/server/stats") as st:
                return await st.json()

    stats = _run(main())
    assert sum(r["active_requests"] for r in stats["replicas"]) == 0


def test_frontend_count_auto():
    """api.frontends = 0 (default): two front ends for GPU process replicas (Req 5.1 at one
    replica's token rate, profiles/r3_frontend.md), one for mock / in-process / CPU serving;
    an explicit count wins; negative counts are rejected."""
    from xgserve.server.config import ServerConfig
    c = ServerConfig()
    assert c.api.frontends == 0
    assert c.api.resolved_frontends(c.worker) == 2
    c.worker.mock = True
    assert c.api.resolved_frontends(c.worker) == 1
    c.worker.mock = False
    c.worker.in_process = True
    assert c.api.resolved_frontends(c.worker) == 1
    c.worker.in_process = False
    c.worker.device = "cpu"
    assert c.api.resolved_frontends(c.worker) == 1
    c.api.frontends = 3
    assert c.api.resolved_frontends(c.worker) == 3
    c.api.frontends = -1
    assert any("api.frontends" in e for e in c.validate())
