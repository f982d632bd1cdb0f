"""The round-3 serving fixes, end to end:

* an HTTP/1.0 client asking for `stream: true` gets a clean close-delimited SSE
  body (no chunk-size lines: the pre-framed HTTP/1.1 wire path is only for chunked
  responses, server/app.py) -- through the in-process server and the sharded
  front ends;
* a front end killed mid-stream (SIGKILL) has its requests cancelled in the
  engine, a fresh front end takes over its port share, /health stays truthful and
  new requests are served (server/frontend.py `_front_end_lost`);
* a client that stays connected but stops reading is cut once its unsent bytes
  pass WIRE_MAX_BUFFERED: error event, sequence aborted in the engine
  (orchestrator `_wire_ok`)."""
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
import psutil
import pytest

from _server_util import mock_config, parse_sse, run_with_client

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


async def _http10(host: str, port: int, body: dict) -> tuple:
    """One HTTP/1.0 POST /generate on a raw socket; the body ends at connection close."""
    data = json.dumps(body).encode()
    r, w = await asyncio.open_connection(host, port)
    w.write(b"POST /generate HTTP/1.0\r\nHost: test\r\nContent-Type: application/json\r\n"
            + f"Content-Length: {len(data)}\r\n\r\n".encode() + data)
    await w.drain()
    raw = await asyncio.wait_for(r.read(), 60)
    w.close()
    head, _, payload = raw.partition(b"\r\n\r\n")
    return head.decode("latin-1"), payload


def _check_clean_sse(head: str, payload: bytes, n: int):
    assert head.startswith("HTTP/1.") and " 200 " in head.split("\r\n")[0], head
    assert "chunked" not in head.lower(), head
    # every non-empty line of the body is an SSE field: no hex chunk-size framing
    for line in payload.decode().split("\n"):
        assert line == "" or line.startswith("data: "), repr(line)
    evs = parse_sse(payload)
    toks = [e for e in evs if e["type"] == "token"]
    assert evs[-1]["type"] == "done" and evs[-1]["usage"]["completion_tokens"] == n, evs[-3:]
    # (a token whose text is an incomplete UTF-8 sequence is carried by the next event)
    idx = [e["index"] for e in toks]
    assert idx == sorted(set(idx)) and idx[-1] == n - 1 and len(idx) >= n - 4, idx


BODY = {"prompt": "an http/1.0 streaming client", "max_tokens": 40, "stream": True, "ignore_eos": True}


def test_http10_stream_in_process():
    cfg = mock_config()

    async def fn(client, srv):
        head, payload = await _http10(client.server.host, client.server.port, BODY)
        _check_clean_sse(head, payload, 40)

    run_with_client(cfg, fn)


def _start_server(*extra):
    port = _free_port()
    cmd = [sys.executable, "-m", "xgserve", "serve", "--host", "127.0.0.1", "--port", str(port), "--mock",
           "--replicas", "1", "--in-process", "--log-level", "WARNING", *extra]
    p = subprocess.Popen(cmd, cwd=ROOT, start_new_session=True, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
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

    if not asyncio.run(ready()):
        p.kill()
        raise AssertionError("server did not come up: " + p.stderr.read().decode()[-2000:])
    return p, port, url


def _stop(p):
    os.killpg(p.pid, signal.SIGTERM)
    try:
        p.wait(30)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait(10)


def _front_ends(p) -> list:
    """The server's front-end processes (multiprocessing spawn children)."""
    out = []
    for c in psutil.Process(p.pid).children(recursive=True):
        try:
            cl = " ".join(c.cmdline())
        except psutil.Error:
            continue
        if "spawn_main" in cl and "resource_tracker" not in cl:
            out.append(c)
    return out


def test_http10_stream_through_front_ends():
    p, port, _ = _start_server("--frontends", "2")
    try:
        for _ in range(4):  # SO_REUSEPORT spreads connections: exercise both front ends
            head, payload = asyncio.run(_http10("127.0.0.1", port, BODY))
            _check_clean_sse(head, payload, 40)
    finally:
        _stop(p)


def test_front_end_killed_mid_stream():
    p, port, url = _start_server("--frontends", "2", "--set", "worker.mock_latency_ms=20")
    try:
        fes = _front_ends(p)
        assert len(fes) == 2, fes

        async def main():
            n = 10
            body = {"prompt": "a long stream", "max_tokens": 3000, "stream": True, "ignore_eos": True}
            sessions = [aiohttp.ClientSession(connector=aiohttp.TCPConnector(force_close=True)) for _ in range(n)]
            resps = [await s.post(url + "/generate", json=body) for s in sessions]
            for r in resps:
                assert r.status == 200
                await r.content.readline()  # the stream is running
            async with aiohttp.ClientSession() as s:
                async with s.get(url + "/server/stats") as r:
                    before = (await r.json())["active_requests"]
            assert before == n
            os.kill(fes[0].pid, signal.SIGKILL)
            # the killed front end's streams end at once; the others keep streaming
            dead, alive = [], []
            for r in resps:
                try:
                    await asyncio.wait_for(r.content.readline(), 2.0)
                    await asyncio.wait_for(r.content.readline(), 2.0)
                    alive.append(r)
                except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionError):
                    dead.append(r)
            # (a stream that only looked alive on already-buffered bytes is re-checked below)
            t_end = time.monotonic() + 20
            stats = None
            async with aiohttp.ClientSession() as s:
                while time.monotonic() < t_end:
                    async with s.get(url + "/server/stats") as r:
                        stats = await r.json()
                    live = 0
                    for r in alive:
                        try:
                            await asyncio.wait_for(r.content.readline(), 0.5)
                            live += 1
                        except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionError):
                            pass
                    if stats["active_requests"] == live and live < n:
                        break
                    await asyncio.sleep(0.2)
                assert stats is not None and stats["active_requests"] < n, stats
                assert stats["active_requests"] == live, (stats["active_requests"], live, len(dead))
                # a fresh front end took the port share; health is truthful; service continues
                t_end = time.monotonic() + 30
                while time.monotonic() < t_end and len(_front_ends(p)) != 2:
                    await asyncio.sleep(0.2)
                assert len(_front_ends(p)) == 2 and fes[0].pid not in {f.pid for f in _front_ends(p)}
                async with s.get(url + "/health") as r:
                    assert r.status == 200 and (await r.json())["status"] == "ok"
                for _ in range(4):
                    async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(force_close=True)) as s2:
                        async with s2.post(url + "/generate", json={"prompt": "after", "max_tokens": 8,
                                                                    "ignore_eos": True}) as r:
                            assert r.status == 200
                            assert (await r.json())["usage"]["completion_tokens"] == 8
            for s in sessions:
                await s.close()

        asyncio.run(main())
    finally:
        _stop(p)


def test_slow_consumer_is_cut_and_aborted():
    """A transport whose unsent bytes exceed WIRE_MAX_BUFFERED: the stream fails with
    a slow_consumer error event and the sequence is aborted in the engine."""
    from xgserve.server import orchestrator as O
    cfg = mock_config(worker={"mock_latency_ms": 10.0})

    class StuckTransport:
        def is_closing(self):
            return False

        def get_write_buffer_size(self):
            return O.WIRE_MAX_BUFFERED + 1

        def write(self, data):
            raise AssertionError("a cut stream must not be written")

    async def fn(client, srv):
        body = {"prompt": "slow reader", "max_tokens": 2000, "stream": True, "ignore_eos": True}
        async with client.post("/generate", json=body) as r:
            assert r.status == 200
            await r.content.readline()
            sreq = next(iter(srv.inflight.values()))
            rid = sreq.id
            assert srv._wire_ok(sreq, StuckTransport()) is False
            raw = await asyncio.wait_for(r.read(), 10)
        evs = parse_sse(raw)
        assert evs and evs[-1]["type"] == "error" and evs[-1]["code"] == "slow_consumer", evs[-2:]
        t_end = time.monotonic() + 5
        while time.monotonic() < t_end and rid in srv.inflight:
            await asyncio.sleep(0.05)
        assert rid not in srv.inflight
        eng = srv.replicas[0].engine  # the in-process replica's MockEngine
        t_end = time.monotonic() + 5
        while time.monotonic() < t_end and eng.requests:
            await asyncio.sleep(0.05)
        assert not eng.requests  # the sequence left the engine ...
        g0 = eng.stats_counters["generation_tokens"]
        await asyncio.sleep(0.3)
        assert eng.stats_counters["generation_tokens"] == g0  # ... and nothing decodes for it any more

    run_with_client(cfg, fn)
