#!/usr/bin/env python3
"""Serve-path benchmark: N concurrent SSE streams against `python -m xgserve serve`
(BASELINE.json config 1 on the CPU, and the HTTP path of config 3 on a GPU).

    python bench/serve_bench.py --launch "--model gpt2 --device cpu --in-process" \
        --concurrency 8 --prompt-len 128 --output-len 64 --duration 30
    python bench/serve_bench.py --url http://127.0.0.1:8000 --concurrency 64 ...

Each client is a closed loop: POST /generate {"stream": true, "ignore_eos": true}
with a synthetic ASCII prompt (one token per byte with the synthetic tokenizer of
random-init models, so --prompt-len is exact) and staggered max_tokens (uniform on
[1, 2*output_len], mean output_len, as bench.py), reads the SSE events, and
starts the next request when `done` arrives. After --warmup seconds it measures
for --duration seconds:
  * output tok/s seen by the clients (token events received in the window),
  * TTFT (request sent -> first token event) p50 / p99,
  * inter-token gap at the client p50 / p99,
  * Req 5.1 token delivery delay (token on the server host -> SSE event written;
    server-side histogram, /server/stats token_delivery_ms) p50 / p99 / max vs 10 ms,
  * Req 8.4 prompt vs generation tokens/s from the server's own counters.
Prints ONE JSON line. `--launch` starts the server as a child process on a free
port (127.0.0.1) and stops it afterwards.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import shlex
import socket
import string
import subprocess
import sys
import time

import aiohttp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pct(xs, q):
    if not xs:
        return None
    v = sorted(xs)
    return v[min(len(v) - 1, max(0, int(round(q * len(v))) - 1))]


async def _wait_ready(url: str, timeout: float) -> None:
    t_end = time.monotonic() + timeout
    async with aiohttp.ClientSession() as s:
        while time.monotonic() < t_end:
            try:
                async with s.get(url + "/health") as r:
                    if r.status == 200:
                        return
            except aiohttp.ClientError:
                pass
            await asyncio.sleep(0.5)
    raise RuntimeError(f"server at {url} not ready after {timeout:.0f} s")


async def run_clients(a, url: str, first: int, n: int, t0: float, t1: float) -> dict:
    """Clients [first, first + n) of the closed loop; measures in [t0, t1) (monotonic)."""
    rng = random.Random(1234 + first)
    st = {"tokens": 0, "ttft": [], "itl": [], "requests": 0, "errors": 0}
    lens = [max(1, int(round(1 + (2 * a.output_len - 1) * (i + 0.5) / a.concurrency))) for i in range(a.concurrency)]

    def prompt() -> str:
        return "".join(rng.choice(string.ascii_lowercase) for _ in range(max(1, a.prompt_len - 1)))

    async def client(i: int, s: aiohttp.ClientSession):
        max_tokens = lens[i]
        while time.monotonic() < t1:
            body = {"prompt": prompt(), "max_tokens": max_tokens, "temperature": 0.0, "stream": True,
                    "ignore_eos": True}
            sent = time.monotonic()
            last = None
            last_idx = -1
            try:
                async with s.post(url + "/generate", json=body) as r:
                    if r.status != 200:
                        st["errors"] += 1
                        await r.read()
                        await asyncio.sleep(0.05)
                        continue
                    async for raw in r.content:
                        if not raw.startswith(b"data: "):
                            continue
                        now = time.monotonic()
                        in_win = t0 <= now < t1
                        if raw.startswith(b'data: {"type":"token"'):
                            if last is None:
                                if in_win and t0 <= sent:
                                    st["ttft"].append(now - sent)
                            elif in_win:
                                st["itl"].append(now - last)
                            last = now
                            # an event carries the tokens since the previous one (a token whose
                            # text is an incomplete UTF-8 sequence rides the next event): count
                            # by the event's index, the generated-token position
                            i = raw.rfind(b'"index":')
                            idx = int(raw[i + 8:raw.index(b"}", i)].split(b",")[0]) if i >= 0 else last_idx + 1
                            if in_win:
                                st["tokens"] += idx - last_idx
                            last_idx = idx
                        else:
                            ev = json.loads(raw[6:])
                            if ev["type"] == "error":
                                st["errors"] += 1
                            elif in_win:
                                st["requests"] += 1
                            break
            except aiohttp.ClientError:
                st["errors"] += 1
            max_tokens = a.output_len  # later requests: the mean length (bench.py replaces the same way)

    conn = aiohttp.TCPConnector(limit=0)
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None), connector=conn) as s:
        await asyncio.gather(*[client(first + i, s) for i in range(n)])
    return st


def _proc_main(a, url, first, n, t0, t1, q):
    q.put(asyncio.run(run_clients(a, url, first, n, t0, t1)))


async def _stats(url: str) -> dict:
    async with aiohttp.ClientSession() as s:
        async with s.get(url + "/server/stats") as r:
            return await r.json()


def run(a, url: str) -> dict:
    """Client processes (--procs) so the load generator never is the bottleneck."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    t_start = time.monotonic() + 2.0  # processes up
    t0, t1 = t_start + a.warmup, t_start + a.warmup + a.duration
    P = max(1, min(a.procs, a.concurrency))
    per = [a.concurrency // P + (1 if i < a.concurrency % P else 0) for i in range(P)]
    firsts = [sum(per[:i]) for i in range(P)]
    ps = [ctx.Process(target=_proc_main, args=(a, url, firsts[i], per[i], t0, t1, q)) for i in range(P)]
    for p in ps:
        p.start()
    time.sleep(max(0.0, t0 - time.monotonic()))
    s0 = asyncio.run(_stats(url))
    time.sleep(max(0.0, t1 - time.monotonic()))
    s1 = asyncio.run(_stats(url))
    parts = [q.get(timeout=a.duration + 600) for _ in ps]
    for p in ps:
        p.join(60)
    st = {"tokens": sum(x["tokens"] for x in parts), "ttft": sum((x["ttft"] for x in parts), []),
          "itl": sum((x["itl"] for x in parts), []), "requests": sum(x["requests"] for x in parts),
          "errors": sum(x["errors"] for x in parts), "t0": t0, "t1": t1}
    return _report(a, st, s0, s1)


def _replica_delta(s0, s1, win) -> list:
    """Per replica over the window: engine steps/s, mean tokens per step and, with
    XGS_STEP_TIMING=1 in the server's env, host seconds per phase per step."""
    out = []
    r0 = {r["id"]: r.get("engine", {}) for r in s0.get("replicas", [])}
    for r in s1.get("replicas", []):
        e1, e0 = r.get("engine", {}), r0.get(r["id"], {})
        if not e1 or not e0:
            continue
        steps = e1.get("steps", 0) - e0.get("steps", 0)
        d = {"id": r["id"], "steps_per_s": round(steps / win, 2),
             "gen_tokens_per_step": round((e1.get("generation_tokens", 0) - e0.get("generation_tokens", 0))
                                          / max(1, steps), 2)}
        for key in ("loop_time_s", "step_timing_s"):
            if key in e1 and key in e0 and steps:
                d[key.replace("_s", "_ms_per_step")] = {k: round(1000 * (v - e0[key].get(k, 0.0)) / steps, 4)
                                                        for k, v in e1[key].items()}
        out.append(d)
    return out


def _replica_requests(s0, s1) -> dict:
    """Requests the router sent to each replica during the window (id -> count) and
    the spread of that split: max / mean - 1 (0 = perfectly even)."""
    r0 = {r["id"]: r.get("requests_dispatched", 0) for r in s0.get("replicas", [])}
    per = {str(r["id"]): r.get("requests_dispatched", 0) - r0.get(r["id"], 0) for r in s1.get("replicas", [])}
    mean = sum(per.values()) / max(1, len(per))
    return {"per_replica": per, "imbalance": round(max(per.values()) / mean - 1, 4) if per and mean > 0 else None}


def _report(a, st, s0, s1) -> dict:
    win = st["t1"] - st["t0"]
    m0, m1 = s0["metrics"], s1["metrics"]
    dp = m1["prompt_tokens_total"] - m0["prompt_tokens_total"]
    dg = m1["generation_tokens_total"] - m0["generation_tokens_total"]
    dl = m1.get("token_delivery_ms", {})
    ms = lambda x: None if x is None else round(1000 * x, 3)  # noqa: E731
    return {
        "metric": "serve_output_tokens_per_sec", "value": round(st["tokens"] / win, 2), "unit": "tokens/s",
        "window_s": round(win, 2), "concurrency": a.concurrency, "prompt_len": a.prompt_len,
        "output_len": a.output_len, "requests_completed": st["requests"], "errors": st["errors"],
        "ttft_p50_ms": ms(_pct(st["ttft"], 0.5)), "ttft_p99_ms": ms(_pct(st["ttft"], 0.99)),
        "client_itl_p50_ms": ms(_pct(st["itl"], 0.5)), "client_itl_p99_ms": ms(_pct(st["itl"], 0.99)),
        "token_delivery_ms": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in dl.items()},
        "req_5_1_delivery_within_10ms": (dl.get("p99") is not None and dl["p99"] <= 10.0),
        "server_prompt_tokens_per_sec": round(dp / win, 2), "server_generation_tokens_per_sec": round(dg / win, 2),
        "event_loop_lag_ms": m1.get("event_loop_lag_ms"), "client_procs": a.procs,
        "replica_window": _replica_delta(s0, s1, win),
        "replica_requests": _replica_requests(s0, s1),
        "model": s1.get("model"),
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", help="an already running server, e.g. http://127.0.0.1:8000")
    ap.add_argument("--launch", help="start `python -m xgserve serve <ARGS>` (quoted) on a free port")
    ap.add_argument("--concurrency", type=int, default=8)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=64)
    ap.add_argument("--warmup", type=float, default=5.0)
    ap.add_argument("--duration", type=float, default=20.0)
    ap.add_argument("--ready-timeout", type=float, default=900.0)
    ap.add_argument("--procs", type=int, default=4, help="client processes")
    ap.add_argument("--out", help="also append the JSON line to this file")
    ap.add_argument("--label", help="added to the JSON line (bench/scale.sh)")
    a = ap.parse_args()
    if bool(a.url) == bool(a.launch):
        ap.error("give exactly one of --url / --launch")
    proc = None
    url = a.url
    try:
        if a.launch:
            port = _free_port()
            cmd = [sys.executable, "-m", "xgserve", "serve", "--host", "127.0.0.1", "--port", str(port)]
            cmd += shlex.split(a.launch)
            proc = subprocess.Popen(cmd, cwd=ROOT, start_new_session=True)
            url = f"http://127.0.0.1:{port}"
        asyncio.run(_wait_ready(url, a.ready_timeout))
        res = run(a, url)
        if a.label:
            res["label"] = a.label
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
        return 0 if res["errors"] == 0 else 1
    finally:
        if proc is not None:
            proc.terminate()
            try:
                proc.wait(60)
            except subprocess.TimeoutExpired:
                proc.kill()


if __name__ == "__main__":
    sys.exit(main())
