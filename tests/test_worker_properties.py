"""Spec properties 20-23 (design.md:800-826) and the InferenceWorker batch interface
(design.md:310-361): worker count, exactly-N batch results, failure isolation,
response format -- against the MockEngine and a tiny CPU Llama engine."""
from __future__ import annotations

import json

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from _server_util import mock_config, run_with_client
from xgserve.engine.mock import MockEngine
from xgserve.engine.request import SamplingParams
from xgserve.engine.worker import BatchResult, InferenceWorker, WorkerError
from xgserve.server.batcher import build_batch

_prompt = st.lists(st.integers(5, 900), min_size=1, max_size=24)


def _mock_worker(**kw):
    w = InferenceWorker(lambda: MockEngine(**kw))
    w.initialize()
    return w


@settings(max_examples=100, deadline=None)
@given(prompts=st.lists(_prompt, min_size=1, max_size=12), max_new=st.integers(1, 12))
def test_prop21_batch_returns_exactly_n_results(prompts, max_new):
    """Property 21: a batch of N requests yields exactly N results, one per request, in order."""
    w = _mock_worker()
    items = [(f"r{i}", p, max_new, None) for i, p in enumerate(prompts)]
    batch = build_batch(items, padding_token_id=0)
    res = w.infer(batch)
    assert isinstance(res, BatchResult) and res.batch_id == batch.id
    assert [r.request_id for r in res.results] == [f"r{i}" for i in range(len(prompts))]
    for r, p in zip(res.results, prompts):
        assert r.finish_reason == "length" and len(r.tokens) == max_new == r.completion_tokens
        assert r.prompt_tokens == len(p)  # padding is not fed to the engine
    assert res.tokens_generated == max_new * len(prompts)
    assert res.inference_time >= 0


@settings(max_examples=100, deadline=None)
@given(prompts=st.lists(_prompt, min_size=2, max_size=10), bad=st.data())
def test_prop22_failure_isolated_within_batch(prompts, bad):
    """Property 22: one failing request errors alone; its batch-mates complete."""
    w = _mock_worker()
    marker = w.engine.fail_marker_ids
    j = bad.draw(st.integers(0, len(prompts) - 1))
    prompts = [list(p) for p in prompts]
    prompts[j] = prompts[j] + marker
    batch = build_batch([(f"r{i}", p, 4, None) for i, p in enumerate(prompts)])
    res = w.infer(batch)
    assert len(res.results) == len(prompts)
    for i, r in enumerate(res.results):
        if i == j:
            assert r.finish_reason == "error" and r.error and r.error_code == "inference_failed"
        else:
            assert r.error is None and r.finish_reason == "length" and len(r.tokens) == 4


def test_worker_lifecycle_errors_status_and_info():
    w = InferenceWorker(lambda: MockEngine(model_name="m"), worker_id=3)
    batch = build_batch([("a", [5, 6], 2, None)])
    with pytest.raises(WorkerError, match="ModelNotLoaded"):
        w.infer(batch)
    assert not w.status().ready
    w.initialize()
    s = w.status()
    assert s.ready and s.is_healthy and s.id == 3 and s.active_batches == 0
    info = w.model_info()
    assert info.name == "m" and info.vocab_size == 1000
    assert len(w.infer(batch).results) == 1
    w.shutdown()
    with pytest.raises(WorkerError, match="Shutdown"):
        w.infer(batch)
    bad = InferenceWorker(lambda: (_ for _ in ()).throw(RuntimeError("no such checkpoint")))
    with pytest.raises(WorkerError, match="ModelLoad"):
        bad.initialize()


def test_worker_step_exception_fails_running_requests_only():
    class Boom(MockEngine):
        def step(self):
            raise RuntimeError("device lost")

    w = InferenceWorker(lambda: Boom())
    w.initialize()
    res = w.infer(build_batch([("a", [5], 3, None), ("b", [6], 3, None)]))
    assert [r.finish_reason for r in res.results] == ["error", "error"]
    assert all("device lost" in r.error for r in res.results)


def test_worker_over_cpu_llama_engine_matches_generate():
    """The same interface over the real engine (tiny Llama, CPU, fp32): results equal generate()."""
    from xgserve.engine import EngineConfig, LLMEngine
    eng_cfg = EngineConfig(model="llama-tiny", device="cpu", dtype="float32", use_graphs=False, num_blocks=256,
                           max_num_seqs=8, max_model_len=256)
    w = InferenceWorker(lambda: LLMEngine(eng_cfg))
    w.initialize()
    prompts = [[5, 9, 13, 2 + i] * (i + 1) for i in range(4)]
    res = w.infer(build_batch([(f"q{i}", p, 6, None) for i, p in enumerate(prompts)]))
    ref = w.engine.generate(prompts, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    for r, want in zip(res.results, ref):
        if r.finish_reason == "length":
            assert r.tokens == want
        else:  # an EOS stop comes earlier than the ignore_eos reference
            assert r.finish_reason == "stop" and want[: len(r.tokens)] == r.tokens


@settings(max_examples=6, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(n=st.integers(1, 4))
def test_prop20_worker_count(n):
    """Property 20: N configured workers -> N replicas spawned and reporting ready."""
    async def fn(c, srv):
        h = await (await c.get("/health")).json()
        s = await (await c.get("/server/stats")).json()
        assert h["replicas_total"] == n and h["replicas_healthy"] == n
        assert len(s["replicas"]) == n
        return True

    assert run_with_client(mock_config(worker={"replicas": n}), fn)


@settings(max_examples=100, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(reqs=st.lists(st.tuples(st.sampled_from(["generate", "chat"]),
                               st.text(st.characters(min_codepoint=32, max_codepoint=126), min_size=1, max_size=40)
                               .filter(lambda s: s.strip()),
                               st.integers(1, 16)), min_size=1, max_size=100))
def test_prop23_response_format(reqs):
    """Property 23: every successful response has id/object/created/model/choices/usage."""
    async def fn(c, srv):
        for kind, text, mt in reqs:
            if kind == "generate":
                r = await c.post("/generate", data=json.dumps({"prompt": text, "max_tokens": mt}))
            else:
                r = await c.post("/chat", data=json.dumps({"messages": [{"role": "user", "content": text}],
                                                           "max_tokens": mt}))
            assert r.status == 200
            d = await r.json()
            assert isinstance(d["id"], str) and isinstance(d["object"], str)
            assert isinstance(d["created"], int) and isinstance(d["model"], str)
            assert isinstance(d["choices"], list) and len(d["choices"]) >= 1
            u = d["usage"]
            assert all(isinstance(u[k], int) for k in ("prompt_tokens", "completion_tokens", "total_tokens"))
            assert u["total_tokens"] == u["prompt_tokens"] + u["completion_tokens"]
            assert u["completion_tokens"] == mt
        return True

    assert run_with_client(mock_config(), fn)
