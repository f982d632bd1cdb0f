"""Server with real engines on CPU and with per-process replicas:

* BASELINE config 1 analogue: GPT-2 (tiny dims) served over HTTP on the CPU;
  outputs must equal the engine's offline greedy generation.
* process replicas (spawned workers): crash -> detection -> restart (Req 7.4).
* TP=2 replica as two gloo-connected processes (leader + follower) serving
  HTTP requests; greedy output equals a TP=1 engine with the same weights.
"""
from __future__ import annotations

import asyncio
import json
import time

import pytest

from _server_util import mock_config, run_with_client
from xgserve.server.config import load_config


def _cpu_cfg(model, **worker):
    w = {"model": model, "device": "cpu", "quantization": "fp32", "num_blocks": 128, "max_num_seqs": 8,
         "max_num_batched_tokens": 256, "use_graphs": False, "in_process": True}
    w.update(worker)
    return load_config(env={}, overrides={"worker": w, "scheduler": {"health_check_interval_s": 0.2,
                                                                      "heartbeat_timeout_s": 30.0}})


@pytest.mark.parametrize("model", ["gpt2-tiny", "llama-tiny", "mixtral-tiny"])
def test_cpu_engine_over_http_matches_offline(model):
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    ref = LLMEngine(EngineConfig(model=model, device="cpu", dtype="float32", num_blocks=128, max_num_seqs=8,
                                 max_num_batched_tokens=256, use_graphs=False))
    prompt = "The quick brown fox"
    ids = ref.tokenizer.encode(prompt)
    want = ref.generate([ids], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))[0]
    want_text = ref.tokenizer.decode(want)

    async def fn(c, srv):
        rs = await asyncio.gather(*[c.post("/generate", data=json.dumps(
            {"prompt": prompt, "max_tokens": 12, "temperature": 0.0, "ignore_eos": True})) for _ in range(3)])
        for r in rs:
            d = await r.json()
            assert r.status == 200, d
            assert d["choices"][0]["text"] == want_text
            assert d["usage"]["prompt_tokens"] == len(ids)
        r = await c.post("/embeddings", data=json.dumps({"input": ["abc", "defg"]}))
        d = await r.json()
        assert r.status == 200 and len(d["data"][0]["embedding"]) == srv.model_info["hidden_size"]
        return True

    assert run_with_client(_cpu_cfg(model), fn, timeout=300)


def test_process_replica_crash_restart():
    cfg = mock_config(worker={"in_process": False, "replicas": 1, "mock_latency_ms": 2.0},
                      scheduler={"health_check_interval_s": 0.1, "heartbeat_timeout_s": 3.0,
                                 "restart_failed": True, "max_restarts": 2})

    async def fn(c, srv):
        r = await c.post("/generate", data=json.dumps({"prompt": "x", "max_tokens": 3}))
        assert r.status == 200
        rep = srv.replicas[0]
        assert rep.kind == "process"
        stream = await c.post("/generate", data=json.dumps({"prompt": "y", "max_tokens": 4000, "stream": True,
                                                            "ignore_eos": True}))
        await stream.content.readline()
        t0 = time.monotonic()
        rep.kill()
        body = await stream.read()
        assert b'"code":"worker_failed"' in body
        for _ in range(600):
            await asyncio.sleep(0.05)
            if srv.health()["status"] == "ok" and srv.replicas[0] is not rep:
                break
        assert srv.health()["status"] == "ok", srv.health()
        assert srv.replicas[0].restarts == 1
        r = await c.post("/generate", data=json.dumps({"prompt": "x", "max_tokens": 3}))
        assert r.status == 200
        assert time.monotonic() - t0 < 60
        return True

    assert run_with_client(cfg, fn, timeout=120)


@pytest.mark.parametrize("model,moe_comm,overlap", [("llama-tiny-gqa8", "alltoall", False),
                                                    ("llama-tiny-gqa8", "alltoall", True),
                                                    ("mixtral-tiny", "alltoall", False),
                                                    ("mixtral-tiny", "allreduce", False)])
def test_tp2_process_replica_gloo_matches_tp1(tmp_path, monkeypatch, model, moe_comm, overlap):
    """TP=2 (two processes over gloo; leader broadcasts step plans; Mixtral
    experts split 4+4 with all-to-all or all-reduce combine) serving HTTP gives
    the same greedy text as a TP=1 engine on the same safetensors checkpoint.
    `overlap`: every step takes the chunk-pipelined all-reduce path
    (LlamaLayer._forward_tp_overlap, 3 token chunks, async all-reduces)."""
    if overlap:  # read by the replica processes at import
        monkeypatch.setenv("XGS_TUNE", "tp_overlap_min_tokens=1|tp_overlap_chunks=3")
    import torch
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    from xgserve.models import build_model, get_config, save_checkpoint
    ck = str(tmp_path / "ckpt")
    save_checkpoint(build_model(get_config(model), "cpu", torch.float32, seed=3), ck)
    ref = LLMEngine(EngineConfig(model=model, checkpoint=ck, device="cpu", dtype="float32", num_blocks=128,
                                 max_num_seqs=8, max_num_batched_tokens=256, use_graphs=False))
    prompts = ["tensor parallel", "over gloo on the host cpu"]
    want = [ref.tokenizer.decode(ref.generate([ref.tokenizer.encode(p)], SamplingParams(
        max_tokens=10, temperature=0.0, ignore_eos=True))[0]) for p in prompts]
    cfg = _cpu_cfg(model, in_process=False, tp=2, checkpoint=ck, random_init=False, moe_comm=moe_comm)
    cfg.scheduler.heartbeat_timeout_s = 60.0

    async def fn(c, srv):
        rs = await asyncio.gather(*[c.post("/generate", data=json.dumps(
            {"prompt": p, "max_tokens": 10, "temperature": 0.0, "ignore_eos": True})) for p in prompts])
        got = [(await r.json())["choices"][0]["text"] for r in rs]
        assert got == want
        return True

    assert run_with_client(cfg, fn, timeout=300)
