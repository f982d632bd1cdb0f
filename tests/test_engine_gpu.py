"""Engine on the GPU: HIP-kernel model forward vs the fp32 PyTorch reference,
graph replay == eager, chunked prefill == one-shot prefill, prefix-cache hits."""
from dataclasses import replace

import pytest
import torch

from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
from xgserve.models import build_model, get_config
from xgserve.models.reference import reference_logits
from xgserve.ops import _native

pytestmark = pytest.mark.gpu


def _engine(model, **kw):
    base = dict(model=model.cfg.name, device="cuda:0", num_blocks=512, max_num_seqs=16,
                max_num_batched_tokens=2048, max_model_len=1024, graph_batch_sizes=[1, 2, 4, 8])
    base.update(kw)
    return LLMEngine(EngineConfig(**base), model=model)


@pytest.fixture(scope="module")
def llama_small():
    _native.kernels()
    cfg = replace(get_config("llama3-8b"), num_layers=2, name="llama3-8b-2l")
    return build_model(cfg, device="cuda:0", seed=3)


def test_prefill_logits_match_reference(llama_small):
    eng = _engine(llama_small, use_graphs=False)
    prompt = [128000] + list(range(1000, 1100))
    ref = reference_logits(llama_small, prompt)[-1].float()
    # run one step by hand and capture logits through the runner
    eng.add_request("a", prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    plan = eng.sched.schedule()
    from xgserve.models.base import AttnMeta
    import numpy as np
    r = eng.runner
    dev = "cuda:0"
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    meta = AttnMeta(num_tokens=int(plan["num_tokens"]), num_decodes=0, positions=t(plan["positions"]),
                    slot_mapping=t(plan["slot_mapping"]), pre_block_tables=t(plan["block_tables"]).view(1, -1),
                    pre_qsl=t(plan["query_start_loc"]), pre_seq_lens=t(plan["seq_lens"]),
                    pre_max_q=int(plan["q_lens"].max()))
    h = llama_small(t(plan["input_ids"]), meta, r.kv_caches)
    logits = llama_small.compute_logits(h[-1:]).float()[0]
    rel = (logits - ref).norm() / ref.norm()
    assert rel < 2e-2, float(rel)


@pytest.mark.parametrize("n_prompts", [1, 3, 8])
def test_graph_decode_equals_eager(llama_small, n_prompts):
    prompts = [[128000] + list(range(200 + 7 * i, 260 + 11 * i)) for i in range(n_prompts)]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    a = _engine(llama_small, use_graphs=True).generate(prompts, sp)
    b = _engine(llama_small, use_graphs=False).generate(prompts, sp)
    assert a == b


@pytest.mark.parametrize("budget", [48, 128, 2048])
def test_chunked_prefill_matches_reference(llama_small, budget):
    """Chunked prefill (chunks attend to the paged prefix) -- fast skinny path for
    small chunks, hipBLASLt for large -- against the dense fp32 reference."""
    prompt = [128000] + list(range(3000, 3700))
    ref = reference_logits(llama_small, prompt)[-1].float().cpu()
    eng = _engine(llama_small, max_num_batched_tokens=budget, use_graphs=False)
    eng.runner.capture_logits = True
    eng.add_request("c", prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    while eng.has_work():
        eng.step()
    got = eng.runner.last_logits[-1]
    assert float((got - ref).norm() / ref.norm()) < 2e-2


def test_prefix_cache_hit_same_tokens(llama_small):
    eng = _engine(llama_small)
    p = [128000] + list(range(5000, 5300))
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    first = eng.generate([p], sp)
    second = eng.generate([p], sp)
    assert first == second
    assert eng.stats()["cache"]["hit_tokens"] >= 256


def test_sampling_seeded_reproducible(llama_small):
    eng = _engine(llama_small)
    p = [[128000, 11, 12, 13]] * 3
    sp = SamplingParams(max_tokens=10, temperature=0.9, top_p=0.95, seed=7, ignore_eos=True)
    a = eng.generate(p, sp)
    b = eng.generate(p, sp)
    assert a == b
    assert a[0] == a[1] == a[2]


def test_mixtral_small_runs_and_matches_reference():
    cfg = replace(get_config("mixtral-8x7b"), num_layers=1, intermediate_size=1792, name="mixtral-1l")
    m = build_model(cfg, device="cuda:0", seed=5)
    eng = _engine(m, use_graphs=True)
    prompt = [1] + list(range(100, 160))
    ref = reference_logits(m, prompt)[-1].float()
    out = eng.generate([prompt], SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert len(out[0]) == 4
    assert out[0][0] == int(ref.argmax()) or float(ref.topk(2).values.diff().abs()) < 0.05


def test_embeddings_request(llama_small):
    from xgserve.engine import RequestType
    eng = _engine(llama_small)
    eng.add_request("e1", [128000, 5, 6, 7, 8], SamplingParams(max_tokens=0), kind=RequestType.Embeddings)
    outs = []
    while eng.has_work():
        outs += eng.step()
    emb = [o for o in outs if o.request_id == "e1"][0].embedding
    v = torch.tensor(emb)
    assert v.shape[0] == llama_small.cfg.hidden_size
    assert abs(float(v.norm()) - 1.0) < 1e-3


def test_speculative_self_draft_on_gpu(llama_small):
    """Draft == target weights on the GPU (graphs on): nearly every draft token is
    accepted and the output tracks plain greedy decoding (bf16 verify rows go
    through the prefill kernel, plain decode through the decode kernel, so a rare
    near-tie may flip late tokens)."""
    prompts = [[128000] + list(range(300 + 13 * i, 340 + 13 * i)) for i in range(4)]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    want = _engine(llama_small).generate(prompts, sp)
    eng = _engine(llama_small, draft_model=llama_small, num_speculative_tokens=3)
    got = eng.generate(prompts, sp)
    st = eng.stats()["speculative"]
    assert st["acceptance_rate"] > 0.8, st
    assert st["mean_tokens_per_verify"] > 2.5, st
    assert [g[0] for g in got] == [w[0] for w in want]  # first token: the same prefill
    assert all(len(g) == 16 for g in got)


def test_http_server_with_gpu_engine(llama_small):
    """The HTTP layer over a real HIP engine replica (in-process)."""
    import asyncio
    import json
    import sys
    import os
    sys.path.insert(0, os.path.dirname(__file__))
    from _server_util import run_with_client
    from xgserve.server.config import load_config
    eng = _engine(llama_small)
    cfg = load_config(env={}, overrides={"worker": {"model": "llama3-8b", "in_process": True}})

    async def fn(c, srv):
        rs = await asyncio.gather(*[c.post("/generate", data=json.dumps(
            {"prompt": f"hello {i}", "max_tokens": 8, "temperature": 0.0, "ignore_eos": True})) for i in range(4)])
        for r in rs:
            d = await r.json()
            assert r.status == 200, d
            assert d["usage"]["completion_tokens"] == 8
        r = await c.post("/generate", data=json.dumps({"prompt": "stream me", "max_tokens": 5, "stream": True,
                                                       "ignore_eos": True}))
        body = await r.read()
        assert b'"type":"done"' in body
        r = await c.post("/embeddings", data=json.dumps({"input": ["a", "bb"]}))
        d = await r.json()
        assert r.status == 200 and len(d["data"][0]["embedding"]) == 4096
        return True

    assert run_with_client(cfg, fn, engine=eng, timeout=300)


def _run_async_vs_sync(model, async_, staggered, temperature):
    eng = _engine(model, async_schedule=async_)
    assert eng._async == async_
    outs = {}
    for i in range(4):
        eng.add_request(f"r{i}", [128000] + list(range(400 + 9 * i, 430 + 13 * i)),
                        SamplingParams(max_tokens=(5 + 3 * i) if staggered else 10, temperature=temperature,
                                       ignore_eos=True, seed=11 + i))
    n = 0
    while eng.has_work():
        for o in eng.step():
            outs.setdefault(o.request_id, []).extend(o.new_token_ids)
        n += 1
        if staggered and n == 4:  # arrivals while a lookahead step is in flight
            for i in range(4, 7):
                eng.add_request(f"r{i}", [128000] + list(range(700 + 5 * i, 720 + 5 * i)),
                                SamplingParams(max_tokens=9, temperature=temperature, ignore_eos=True,
                                               seed=11 + i))
    return outs, eng


@pytest.mark.parametrize("temperature", [0.0, 0.8])
def test_async_schedule_matches_sync(llama_small, temperature):
    """Asynchronous scheduling (step N+1 planned and launched before step N's
    tokens reach the host; decode ids substituted on the GPU from the previous
    graph step's sampled tokens) reproduces the synchronous loop exactly when the
    steps' batch composition is the same: greedy and seeded sampling."""
    a, _ = _run_async_vs_sync(llama_small, False, False, temperature)
    b, eng = _run_async_vs_sync(llama_small, True, False, temperature)
    assert a == b
    assert all(len(v) == 10 for v in b.values())
    assert eng.sched.num_inflight() == 0 and eng.sched.num_running() == 0


def test_async_schedule_staggered_tokens_are_reference_argmax(llama_small):
    """Staggered lengths (rows finishing while their successor step is already in
    flight) and mid-run arrivals change step composition, hence bf16 rounding, so
    each greedy token is checked against the fp32 reference instead: an argmax up
    to a bf16-sized near-tie, with exact requested lengths."""
    b, eng = _run_async_vs_sync(llama_small, True, True, 0.0)
    assert all(len(b[f"r{i}"]) == (5 + 3 * i if i < 4 else 9) for i in range(7))
    prompts = {f"r{i}": [128000] + list(range(400 + 9 * i, 430 + 13 * i)) for i in range(4)}
    prompts.update({f"r{i}": [128000] + list(range(700 + 5 * i, 720 + 5 * i)) for i in range(4, 7)})
    for rid, gen in b.items():
        p = prompts[rid]
        ref = reference_logits(llama_small, p + gen[:-1]).float()
        for i, tok in enumerate(gen):
            row = ref[len(p) - 1 + i]
            assert float(row.max() - row[tok]) < 0.15, (rid, i)
    assert eng.sched.num_inflight() == 0 and eng.sched.num_running() == 0


def _run_stall_free(model, chunk, temperature=0.0):
    """16 rows decoding while prompts arrive: with decode_prefill_cap = chunk every
    prompt is prefilled in chunk-sized pieces that ride on the decode steps."""
    eng = _engine(model, decode_prefill_cap=chunk, graph_batch_sizes=[1, 2, 4, 8, 16, 24, 32],
                  max_num_seqs=32)
    prompts, outs = {}, {}
    for i in range(16):
        p = [128000] + list(range(900 + 3 * i, 940 + 3 * i))
        prompts[f"d{i}"] = p
        eng.add_request(f"d{i}", p, SamplingParams(max_tokens=24, temperature=temperature, ignore_eos=True,
                                                  seed=5 + i))
    n = 0
    while eng.has_work():
        for o in eng.step():
            outs.setdefault(o.request_id, []).extend(o.new_token_ids)
        n += 1
        if n in (3, 6):  # long prompts arriving while the rows decode
            for j in range(2):
                rid = f"p{n}-{j}"
                p = [128000] + list(range(2000 + 50 * n + 7 * j, 2000 + 50 * n + 7 * j + 300 + 37 * j))
                prompts[rid] = p
                eng.add_request(rid, p, SamplingParams(max_tokens=6, temperature=temperature, ignore_eos=True,
                                                      seed=50 + n + j))
    return prompts, outs, eng


def test_stall_free_mixed_graphs_match_reference(llama_small):
    """Mixed steps (decode rows + one <= 128-token prompt chunk) replay the captured
    mixed graphs on the gemm_mw path; every greedy token is the fp32 reference's
    argmax up to a bf16 near-tie, with exact lengths."""
    prompts, outs, eng = _run_stall_free(llama_small, 128)
    assert eng.runner.mixed_graphs, "no mixed graphs captured"
    assert eng.runner.mixed_replays >= 6, eng.runner.mixed_replays
    for rid, gen in outs.items():
        assert len(gen) == (24 if rid.startswith("d") else 6), rid
        p = prompts[rid]
        ref = reference_logits(llama_small, p + gen[:-1]).float()
        for i, tok in enumerate(gen):
            row = ref[len(p) - 1 + i]
            assert float(row.max() - row[tok]) < 0.15, (rid, i)
    assert eng.sched.num_inflight() == 0 and eng.sched.num_running() == 0


def test_stall_free_sampling_seeded(llama_small):
    """Seeded sampling through the mixed graphs is reproducible run to run."""
    _, a, _ = _run_stall_free(llama_small, 128, temperature=0.8)
    _, b, eng = _run_stall_free(llama_small, 128, temperature=0.8)
    assert a == b
    assert eng.runner.mixed_replays >= 6


def test_whole_prompt_mixed_graphs_on_library_gemms(llama_small):
    """decode_prefill_cap = 512: a whole prompt (<= 512 tokens) rides one decode step as
    a captured mixed graph whose GEMMs are the library ones (rows > MW_MAX_TOKENS); every
    greedy token is the fp32 reference's argmax up to a bf16 near-tie."""
    prompts, outs, eng = _run_stall_free(llama_small, 512)
    assert eng.runner.mixed_chunk == 512 and eng.runner.mixed_graphs
    assert eng.runner.mixed_replays >= 3, eng.runner.mixed_replays
    for rid, gen in outs.items():
        assert len(gen) == (24 if rid.startswith("d") else 6), rid
        p = prompts[rid]
        ref = reference_logits(llama_small, p + gen[:-1]).float()
        for i, tok in enumerate(gen):
            row = ref[len(p) - 1 + i]
            assert float(row.max() - row[tok]) < 0.15, (rid, i)
    assert eng.sched.num_inflight() == 0 and eng.sched.num_running() == 0
