"""Helpers to run the HTTP app in-process for integration tests (no pytest-asyncio)."""
from __future__ import annotations

import asyncio
import json
from typing import Any, Awaitable, Callable, Dict, List, Optional

from aiohttp.test_utils import TestClient, TestServer

from xgserve.server.app import build_app
from xgserve.server.config import load_config
from xgserve.server.orchestrator import InferenceServer


def mock_config(**sections) -> Any:
    base = {"worker": {"mock": True, "model": "mock", "in_process": True, "mock_latency_ms": 1.0, "replicas": 1},
            "scheduler": {"health_check_interval_s": 0.1, "heartbeat_timeout_s": 2.0}}
    for sec, kv in sections.items():
        base.setdefault(sec, {}).update(kv)
    return load_config(env={}, overrides=base)


def run_with_client(cfg, fn: Callable[[TestClient, InferenceServer], Awaitable[Any]], engine=None,
                    fault: Optional[dict] = None, timeout: float = 60.0):
    async def main():
        srv = InferenceServer(cfg, engine=engine)
        srv.fault = fault
        app = build_app(srv)
        client = TestClient(TestServer(app))
        await client.start_server()
        try:
            return await asyncio.wait_for(fn(client, srv), timeout)
        finally:
            await client.close()

    return asyncio.run(main())


def parse_sse(raw: bytes) -> List[Dict]:
    events = []
    for chunk in raw.decode().split("\n\n"):
        chunk = chunk.strip()
        if not chunk.startswith("data: "):
            continue
        body = chunk[len("data: "):]
        if body == "[DONE]":
            events.append({"type": "[DONE]"})
            continue
        events.append(json.loads(body))
    return events
