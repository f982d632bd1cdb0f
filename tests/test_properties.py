"""Property tests (hypothesis, >= 100 examples) for the native runtime core and
wire layer. Each test names the reference property it checks:
models.rs:444-475 (Property 25 round trips), validator.rs:337-435 (Properties
1-3 + token_count), design.md:686-856 (Properties 4-8, 9-12, 13-15, 16-19,
23-24, 26-27)."""
from __future__ import annotations

import json
import math
import os
import string
import uuid

import pytest
from hypothesis import HealthCheck, assume, given, settings
from hypothesis import strategies as st

from xgserve import _runtime as R
from xgserve.core.errors import ApiInternal, ApiQueueFull, ApiTimeout, ApiValidationError, ConfigError, ValidationError
from xgserve.core.types import Priority
from xgserve.core.wire import (ChatChoice, ChatMessage, ChatResponse, EmbeddingData, EmbeddingsResponse, ErrorResponse,
                               FinishReason, GenerateChoice, GenerateRequest, GenerateResponse, Role, TokenEvent, Usage)

S = settings(max_examples=100, deadline=None, suppress_health_check=[HealthCheck.too_slow])

# ----------------------------------------------------------------------------- generators (models.rs:334-441)
usage_st = st.builds(lambda p, c: Usage.new(p, c), st.integers(0, 100000), st.integers(0, 100000))
finish_st = st.sampled_from(list(FinishReason))
role_st = st.sampled_from(list(Role))
text_st = st.text(max_size=200)
msg_st = st.builds(ChatMessage, role_st, text_st)
model_st = st.text(alphabet=string.ascii_letters + string.digits + "_", min_size=1, max_size=50)
id_st = st.builds(lambda: str(uuid.uuid4()))
f32_st = st.floats(-1.0, 1.0, width=32, exclude_max=True)


@S
@given(id_st, st.integers(0, 2**40), model_st,
       st.lists(st.builds(GenerateChoice, text_st, st.integers(0, 10), finish_st), min_size=1, max_size=4), usage_st)
def test_prop25_generate_response_roundtrip(rid, created, model, choices, usage):
    r = GenerateResponse(rid, "text_completion", created, model, choices, usage)
    assert GenerateResponse.from_dict(json.loads(json.dumps(r.to_dict()))) == r


@S
@given(id_st, st.integers(0, 2**40), model_st,
       st.lists(st.builds(ChatChoice, st.integers(0, 10), msg_st, finish_st), min_size=1, max_size=4), usage_st)
def test_prop25_chat_response_roundtrip(rid, created, model, choices, usage):
    r = ChatResponse(rid, "chat.completion", created, model, choices, usage)
    assert ChatResponse.from_dict(json.loads(json.dumps(r.to_dict()))) == r


@S
@given(st.lists(st.builds(EmbeddingData, st.lists(f32_st, min_size=1, max_size=99), st.integers(0, 100)),
                min_size=1, max_size=5), model_st, usage_st)
def test_prop25_embeddings_response_roundtrip(data, model, usage):
    r = EmbeddingsResponse(data, model, usage)
    assert EmbeddingsResponse.from_dict(json.loads(json.dumps(r.to_dict()))) == r


@S
@given(text_st, text_st, text_st)
def test_prop24_25_error_response(message, etype, code):
    r = ErrorResponse.new(message, etype, code)
    d = json.loads(json.dumps(r.to_dict()))
    assert set(d["error"]) == {"message", "type", "code"}
    assert ErrorResponse.from_dict(d) == r


# ----------------------------------------------------------------------------- validator (validator.rs:337-435)
V = R.RequestValidator()
valid_prompt = st.text(min_size=1, max_size=2000).filter(lambda s: s.strip() != "")


@S
@given(valid_prompt, st.integers(0, 4096), st.floats(0.0, 2.0, width=32), st.floats(0.0, 1.0, width=32))
def test_prop1_valid_generate_accepted(p, mt, t, tp):
    assume(len(p.encode()) <= 8192 * 4 and p.strip())
    assert V.validate_generate(p, mt, t, tp) is None


@S
@given(st.lists(st.builds(lambda c: c, valid_prompt), min_size=1, max_size=5), st.integers(0, 4096),
       st.floats(0.0, 2.0, width=32), st.floats(0.0, 1.0, width=32))
def test_prop1_valid_chat_accepted(contents, mt, t, tp):
    assert V.validate_chat(contents, mt, t, tp) is None


@S
@given(st.sampled_from(["", "   ", "\t\n", "　", "   "]))
def test_empty_prompt_rejected(p):
    r = V.validate_generate(p, 10, 1.0, 1.0)
    assert r["kind"] == "empty_prompt" and r["message"] == "Empty prompt not allowed"


@S
@given(st.one_of(st.floats(-10.0, -0.01), st.floats(2.01, 10.0)))
def test_prop2_invalid_temperature_rejected(t):
    r = V.validate_generate("hi", 10, t, 1.0)
    assert r["kind"] == "invalid_parameter" and r["field"] == "temperature"
    assert r["message"].startswith("Invalid parameter 'temperature': must be between 0 and 2, got ")


@S
@given(st.one_of(st.floats(-10.0, -0.01), st.floats(1.01, 10.0)))
def test_prop2_invalid_top_p_rejected(p):
    r = V.validate_generate("hi", 10, 1.0, p)
    assert r["kind"] == "invalid_parameter" and r["field"] == "top_p"


@S
@given(st.integers(35000, 40000))
def test_prop3_oversized_prompt_rejected(n):
    r = V.validate_generate("a" * n, 10, 1.0, 1.0)
    assert r["kind"] == "token_limit_exceeded"
    assert r["message"] == f"Token limit exceeded: {(n + 3) // 4} tokens > 8192 max"


@S
@given(st.text(max_size=5000))
def test_token_count_proportional(s):
    n = len(s.encode())
    assert V.token_count(s) == (0 if n == 0 else (n + 3) // 4)


def test_nan_rejected_and_f32_display():
    assert V.validate_generate("x", 1, float("nan"), 1.0)["field"] == "temperature"
    assert R.rust_f32_display(2.5) == "2.5" and R.rust_f32_display(-0.01) == "-0.01"


@S
@given(st.dictionaries(st.sampled_from(["max_tokens", "temperature", "top_p", "stream", "prompt"]),
                       st.one_of(st.none(), st.booleans(), st.text(max_size=5), st.floats(allow_nan=False),
                                 st.integers(-5, 10))))
def test_prop2_wire_parse_strictness(d):
    """Any parse either succeeds with correctly-typed fields or raises ValidationError."""
    try:
        r = GenerateRequest.parse(json.dumps(d))
    except ValidationError as e:
        assert e.kind in ("invalid_json", "missing_field")
        return
    assert isinstance(r.prompt, str) and isinstance(r.max_tokens, int) and r.max_tokens >= 0
    assert isinstance(r.stream, bool)


# ----------------------------------------------------------------------------- queue (queue.rs; Properties 6-8)
def _queue(hw=1000, lw=500, mx=2000, timeout=30.0):
    c = R.QueueConfig()
    c.high_watermark, c.low_watermark, c.max_queue_size, c.request_timeout_s = hw, lw, mx, timeout
    q = R.PriorityQueueManager(c)
    q.set_manual_clock(True, 0.0)
    return q


@S
@given(st.lists(st.sampled_from([0, 1, 2]), max_size=200))
def test_prop6_priority_ordering(prios):
    q = _queue()
    for i, p in enumerate(prios):
        assert q.enqueue(str(i), i, p)
    out = q.dequeue_batch(len(prios) + 5)
    got = [(it[2], it[1]) for it in out]
    assert got == sorted(got, key=lambda x: (-x[0], x[1]))


@S
@given(st.integers(2, 60), st.lists(st.booleans(), max_size=300))
def test_prop7_backpressure_hysteresis(hw, ops):
    lw = hw // 2
    q = _queue(hw, lw, 10 * hw)
    active = False
    n = 0
    for i, enq in enumerate(ops):
        if enq:
            ok = q.enqueue(str(i), None, 1)
            assert ok == (not active)
            if ok:
                n += 1
        elif n:
            q.dequeue_one()
            n -= 1
        if not active and n > hw:
            active = True
        elif active and n < lw:
            active = False
        assert q.is_accepting() == (not active)
        assert q.total_depth() == n


def test_prop7_default_boundaries():
    q = _queue()
    for i in range(1001):
        assert q.enqueue(str(i), None, 1)
    assert not q.is_accepting() and not q.enqueue("x", None, 1)
    for _ in range(501):
        q.dequeue_one()
    assert q.total_depth() == 500 and not q.is_accepting()
    q.dequeue_one()
    assert q.total_depth() == 499 and q.is_accepting()


@S
@given(st.lists(st.tuples(st.floats(0, 10), st.sampled_from([0, 1, 2])), min_size=1, max_size=40), st.floats(0.5, 5))
def test_prop8_timeouts(arrivals, timeout):
    q = _queue(timeout=timeout)
    t = 0.0
    stamps = {}
    for i, (dt, p) in enumerate(arrivals):
        t += dt
        q.advance_clock(dt)
        q.enqueue(str(i), i, p)
        stamps[str(i)] = t
    q.advance_clock(timeout * 0.999)
    now = t + timeout * 0.999
    expired = {it[0] for it in q.remove_expired()}
    assert expired == {k for k, s in stamps.items() if now - s > timeout}
    left = {it[0] for it in q.drain()}
    assert left.isdisjoint(expired) and left | expired == set(stamps)


def test_queue_cancel():
    q = _queue()
    q.enqueue("a", 1, 1)
    q.enqueue("b", 2, 2)
    assert q.cancel("a")[0] == "a" and q.cancel("a") is None
    assert q.total_depth() == 1


# ----------------------------------------------------------------------------- batcher (Properties 4-5)
@S
@given(st.lists(st.lists(st.integers(0, 50000), min_size=1, max_size=64), min_size=1, max_size=32))
def test_prop5_padding(seqs):
    from xgserve.server.batcher import build_batch
    b = build_batch([(str(i), s, 8, None) for i, s in enumerate(seqs)], padding_token_id=0)
    L = max(len(s) for s in seqs)
    assert all(len(r) == L for r in b.input_ids)
    for s, r, m, br in zip(seqs, b.input_ids, b.attention_mask, b.requests):
        assert br.original_length == len(s) and br.padded_length == L
        assert r[:len(s)] == s and m == [1] * len(s) + [0] * (L - len(s))


@settings(max_examples=25, deadline=None)
@given(st.integers(1, 32))
def test_prop4_batch_formation(n):
    import asyncio
    from xgserve.server.batcher import RequestBatcher

    async def run():
        b = RequestBatcher(max_batch_size=32, batch_timeout_ms=20.0)
        for i in range(n):
            await b.add_request(str(i), [1, 2], 4)
        batch = await b.get_batch(timeout=1.0)
        return batch.size

    assert asyncio.run(run()) == n


# ----------------------------------------------------------------------------- prefix cache (Properties 9-11)
@S
@given(st.lists(st.integers(0, 7), min_size=16, max_size=120), st.lists(st.integers(0, 7), max_size=60))
def test_prop9_prefix_reuse(prefix, suffix):
    a = R.BlockAllocator(64)
    c = R.PrefixCache(a, 16, 64)
    n_pages = len(prefix) // 16
    blocks = [a.alloc() for _ in range(n_pages)]
    c.insert(prefix, blocks)
    got = c.match(prefix + suffix, len(prefix) + len(suffix))
    assert got[:n_pages] == blocks


@S
@given(st.integers(2, 20), st.lists(st.integers(0, 19), min_size=1, max_size=60))
def test_prop10_11_lru_eviction_and_touch(n_entries, accesses):
    a = R.BlockAllocator(64)
    c = R.PrefixCache(a, 16, 64)
    keys = []
    for e in range(n_entries):
        k = [e * 100 + j for j in range(16)]
        b = a.alloc()
        c.insert(k, [b])
        a.decref(b)  # cache-only reference
        keys.append((k, b))
    for i in accesses:
        i %= n_entries
        before = c.last_access_of(keys[i][1])
        c.match(keys[i][0], 16)
        assert c.last_access_of(keys[i][1]) >= before  # Property 11
    order = sorted(range(n_entries), key=lambda i: c.last_access_of(keys[i][1]))
    ev = c.evict(1)
    assert ev == 1
    lru = order[0]
    assert c.last_access_of(keys[lru][1]) == 0  # the least recently used entry went first (Property 10)
    assert c.stats()["eviction_count"] >= 1


def test_prop10_memory_limit_enforced():
    a = R.BlockAllocator(64)
    c = R.PrefixCache(a, 16, 8)
    for e in range(20):
        b = a.alloc()
        c.insert([e * 100 + j for j in range(16)], [b])
        a.decref(b)
    assert c.stats()["entries"] <= 8


@S
@given(st.lists(st.tuples(st.integers(0, 5), st.integers(1, 4), st.booleans()), min_size=1, max_size=40),
       st.integers(1, 30))
def test_prop10_evictable_count_and_lru_order_under_sharing(ops_, n_evict):
    """Branching prefixes, some pages still referenced by 'sequences': the O(1)
    evictable count equals a brute-force count, eviction never frees a page a
    sequence holds, and it frees leaves oldest-access first."""
    a = R.BlockAllocator(512)
    c = R.PrefixCache(a, 4, 512)
    held = []
    for i, (branch, pages, keep) in enumerate(ops_):
        toks = [branch] * 4 + [1000 + i * 10 + j for j in range(4 * (pages - 1))]
        blocks = c.match(toks, len(toks), False)
        for b in blocks:
            a.incref(b)
        while len(blocks) < pages:
            blocks.append(a.alloc())
        c.insert(toks, blocks)
        for b in blocks:
            if keep:
                held.append(b)
            else:
                a.decref(b)
    cached = [b for b in range(512) if c.last_access_of(b) > 0]
    assert c.evictable() == sum(1 for b in cached if a.refcount(b) == 1)
    ev = c.evict(n_evict)
    assert all(a.refcount(b) >= 1 for b in held)  # pages a sequence holds survive
    cached2 = [b for b in range(512) if c.last_access_of(b) > 0]
    assert len(cached) - len(cached2) == ev
    assert c.evictable() == sum(1 for b in cached2 if a.refcount(b) == 1)


def test_eviction_scales_with_cache_size():
    """A full 64K-page cache: single-page evictions (what every page allocation
    does once the pool is full) must not walk the tree -- 2000 of them well under a
    second (a whole-tree walk per eviction would take minutes)."""
    import time
    n = 1 << 16
    a = R.BlockAllocator(n)
    c = R.PrefixCache(a, 16, n)
    for s_ in range(n // 32):  # 2048 sequences x 32 pages
        toks = [s_ * 7 + 1] + list(range(2, 16 * 32 + 1))
        blocks = [a.alloc() for _ in range(32)]
        c.insert(toks, blocks)
        for b in blocks:
            a.decref(b)
    assert c.evictable() == n and a.num_free() == 0
    t0 = time.perf_counter()
    for _ in range(2000):
        assert c.evict(1) == 1
    assert time.perf_counter() - t0 < 1.0
    assert c.evictable() == n - 2000 and a.num_free() == 2000


# ----------------------------------------------------------------------------- KV serialisation (Property 12)
@S
@given(st.integers(1, 3), st.integers(0, 4), st.sampled_from(["bfloat16", "float16", "float32"]), st.integers(0, 9999))
def test_prop12_cache_entry_roundtrip(L, pages, dt, seed):
    import torch
    from xgserve.engine.kv_io import CacheEntry, deserialize, serialize
    g = torch.Generator().manual_seed(seed)
    kv = torch.randn(L, 2, pages, 2, 16, 8, generator=g).to(getattr(torch, dt))
    key = [int(x) for x in torch.randint(0, 1000, (pages * 16,), generator=g)]
    e = CacheEntry(key, kv, len(key), "m", 16)
    assert deserialize(serialize(e)).equivalent(e)


def test_prop12_engine_export_import_reuses_kv():
    import torch
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    from xgserve.engine.kv_io import deserialize, serialize
    mk = lambda: LLMEngine(EngineConfig(model="llama-tiny", device="cpu", dtype="float32", num_blocks=64,
                                        max_num_seqs=4, max_num_batched_tokens=128, use_graphs=False, seed=5))
    a, b = mk(), mk()
    prompt = list(range(10, 60))
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    want = a.generate([prompt], sp)[0]
    e = deserialize(serialize(a.export_prefix(prompt)))
    assert e.token_count == 48
    assert b.import_prefix(e) == 3
    got = b.generate([prompt], sp)[0]
    assert got == want
    assert b.sched.cache_stats()["hit_tokens"] >= 48


# ----------------------------------------------------------------------------- SSE events (Properties 13-15)
@S
@given(text_st, st.integers(0, 10**6), st.one_of(st.none(), st.floats(-100, 0)))
def test_prop13_token_event(tok, idx, lp):
    raw = TokenEvent.tok(tok, idx, lp).sse()
    assert raw.startswith(b"data: ") and raw.endswith(b"\n\n")
    d = json.loads(raw[6:-2])
    assert d["type"] == "token" and d["token"] == tok and d["index"] == idx
    assert ("logprob" in d) == (lp is not None)


@S
@given(finish_st, usage_st)
def test_prop14_done_event(fr, u):
    d = json.loads(TokenEvent.done(fr, u).sse()[6:-2])
    assert d["finish_reason"] in ("stop", "length", "stop_sequence")
    assert set(d["usage"]) == {"prompt_tokens", "completion_tokens", "total_tokens"}


@S
@given(text_st, text_st)
def test_prop15_error_event(m, c):
    d = json.loads(TokenEvent.error(m, c).sse()[6:-2])
    assert d == {"type": "error", "message": m, "code": c}


# ----------------------------------------------------------------------------- routing (Properties 16-19)
@S
@given(st.lists(st.tuples(st.integers(0, 50), st.integers(0, 10**9), st.booleans()), min_size=1, max_size=12),
       st.integers(0, 10**9))
def test_prop16_to_19_routing(workers, need):
    from xgserve.router import Router
    for strat in ("least_loaded", "memory_aware", "round_robin"):
        r = Router(strat)
        for i, (act, mem, healthy) in enumerate(workers):
            r.register(i, mem)
            r.update(i, act, 0, mem)
            r.set_healthy(i, healthy)
        sel = r.select(need)
        healthy_ids = [i for i, w in enumerate(workers) if w[2]]
        if not healthy_ids:
            assert sel == -1
            continue
        if strat == "least_loaded":
            assert sel in healthy_ids and workers[sel][0] == min(workers[i][0] for i in healthy_ids)
        elif strat == "memory_aware":
            fits = [i for i in healthy_ids if workers[i][1] >= need]
            assert (sel == -1) if not fits else (sel in fits)
        else:
            assert sel in healthy_ids
        # Property 19: a recovered worker becomes eligible again
        for i in range(len(workers)):
            r.set_healthy(i, i == 0)
        r.update(0, 0, 0, 10**10)
        assert r.select(0) == 0


# ----------------------------------------------------------------------------- API errors (Property 24)
def test_prop24_api_error_mapping():
    ve = ValidationError.empty_prompt()
    cases = [(ApiValidationError(ve), 400, "invalid_request_error"), (ApiQueueFull(), 503, "rate_limit_error"),
             (ApiTimeout(), 408, "timeout_error"), (ApiInternal("boom"), 500, "server_error")]
    for e, status, typ in cases:
        d = e.to_response()
        assert e.status == status and d["error"]["type"] == typ and set(d["error"]) == {"message", "type", "code"}
    assert ApiQueueFull().message == "Queue full , server is overloaded"
    assert ApiInternal("x").message == "Internal server error: x"


# ----------------------------------------------------------------------------- config (Properties 26-27)
@S
@given(st.one_of(st.none(), st.integers(1001, 5000)), st.one_of(st.none(), st.integers(1001, 5000)),
       st.one_of(st.none(), st.integers(1001, 5000)))
def test_prop26_config_precedence(f, e, c):
    import tempfile
    from xgserve.server.config import load_config
    path = None
    if f is not None:
        fd, path = tempfile.mkstemp(suffix=".toml")
        with os.fdopen(fd, "w") as fh:
            fh.write(f"[queue]\nhigh_watermark = {f}\nmax_queue_size = 100000\n")
    env = {"XGS_QUEUE__HIGH_WATERMARK": str(e), "XGS_QUEUE__MAX_QUEUE_SIZE": "100000"} if e is not None else {}
    cli = [f"queue.high_watermark={c}", "queue.max_queue_size=100000"] if c is not None else []
    try:
        cfg = load_config(path, env=env, cli=cli, overrides={"worker": {"mock": True}})
    finally:
        if path:
            os.unlink(path)
    expect = c if c is not None else e if e is not None else f if f is not None else 1000
    assert cfg.queue.high_watermark == expect


@pytest.mark.parametrize("cli", [["queue.high_watermark=-1"], ["scheduler.strategy=fastest"],
                                 ["worker.tp=0"], ["batcher.mode=dynamic"], ["nosuch.key=1"], ["queue.bogus=1"],
                                 ["worker.quantization=q4"], ["queue.low_watermark=abc"]])
def test_prop27_invalid_config_rejected(cli):
    from xgserve.server.config import load_config
    with pytest.raises(ConfigError):
        load_config(env={}, cli=cli, overrides={"worker": {"mock": True}})


def test_prop27_cli_exit_code(tmp_path):
    import subprocess
    import sys
    bad = tmp_path / "bad.toml"
    bad.write_text("[queue]\nhigh_watermark = -5\n[scheduler]\nstrategy = \"nope\"\n")
    p = subprocess.run([sys.executable, "-m", "xgserve", "check-config", "--config", str(bad), "--mock"],
                       capture_output=True, text=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert p.returncode == 2
    assert "high_watermark" in p.stderr and "strategy" in p.stderr


def test_priority_parse():
    assert Priority.parse("High") == Priority.High and Priority.parse("low") == Priority.Low
    with pytest.raises(ValueError):
        Priority.parse("URGENT")


def test_weight_quantizers_roundtrip():
    """INT8 / INT4 weight-only quantizers (Req 10.3): codes in range, dequantisation
    within half a step of the input, and the int4 pair-interleaved packing (element
    2j at bits 4j, element 2j + 1 at bits 16 + 4j of each word) decodes by hand."""
    import torch
    from xgserve.ops.linear import (WQ_INT4, WQ_INT8, dequantize_weight, quantize_weight)
    g = torch.Generator().manual_seed(3)
    w = torch.randn(48, 384, generator=g)
    q, s = quantize_weight(w, WQ_INT8)
    assert q.dtype == torch.uint8 and s.shape == (48,) and int(q.view(torch.int8).abs().max()) <= 127
    assert float(((dequantize_weight(q, s, WQ_INT8) - w).abs() - s[:, None] / 2).max()) <= 1e-6
    q4, s4 = quantize_weight(w, WQ_INT4)
    assert q4.shape == (48, 192) and s4.shape == (3, 48)
    d = dequantize_weight(q4, s4, WQ_INT4)
    step = s4.t().repeat_interleave(128, dim=1)
    assert float(((d - w).abs() - step / 2).max()) <= 1e-5
    word = int(q4[5, 4:8].view(torch.int32)[0]) & 0xFFFFFFFF  # k = 8 .. 15 of row 5
    for j in range(4):
        for h in range(2):
            u = (word >> (4 * j + 16 * h)) & 15
            assert abs((u - 8) * float(s4[0, 5]) - float(d[5, 8 + 2 * j + h])) < 1e-6
