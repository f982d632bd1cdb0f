"""Tensor parallelism on the MI355X kernels: TP=2 as two processes sharing the one
GPU of a gpurun box (per-rank shards of real Llama-3-8B layer shapes loaded from
a safetensors checkpoint; gloo carries the plan broadcast and the RCCL-shaped
collectives, the one-shot IPC all-reduce carries the decode all-reduces).

Checks, against the fp32 PyTorch reference forward of the unsharded model:
  * prefill logits (a 300-token prompt: hipBLASLt GEMMs, prefill attention on
    half the heads, and the chunk-pipelined all-reduce path) within bf16 error;
  * every greedily decoded token (eager -- gloo is not graph-capturable; sharded
    m64g GEMMs, custom all-reduce, vocab-parallel LM head gather) is an argmax
    of the reference logits at its position, up to a bf16-sized near-tie.
Multi-GPU xGMI performance is not measured here (one GPU per box)."""
import os
import socket
from dataclasses import replace

import pytest
import torch

pytestmark = pytest.mark.gpu

PROMPTS = [[1] + list(range(1000, 1299)), [1] + list(range(50, 90))]  # ids < the 32k vocab
N_GEN = 8


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(model):
    from xgserve.models import get_config
    if model == "llama":
        return replace(get_config("llama3-8b"), num_layers=2, vocab_size=32000, name="tp-test")
    return replace(get_config("mixtral-8x7b"), num_layers=2, intermediate_size=1792, name="tp-test")


def _rank_main(rank, world, port, ck, moe_comm, q, env=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    os.environ.update(env or {})
    try:
        from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
        from xgserve.parallel.state import destroy_distributed, init_distributed
        torch.cuda.set_device(0)
        init_distributed(tp_size=world, backend="gloo", device=torch.device("cuda", 0), timeout_s=120)
        eng = LLMEngine(EngineConfig(model="tp-test", checkpoint=ck, tp=world, device="cuda:0",
                                     num_blocks=256, max_num_seqs=8, max_num_batched_tokens=1024,
                                     max_model_len=512, moe_comm=moe_comm))
        temp = float(os.environ.get("XGS_TEST_TEMPERATURE", "0"))
        if rank == 0:
            sp = SamplingParams(max_tokens=N_GEN, temperature=temp, top_p=0.95 if temp > 0 else 1.0, seed=11,
                                ignore_eos=True)
            if os.environ.get("XGS_TEST_STAGGER") == "1":
                # the second prompt arrives while the first decodes: its prompt step is an
                # eager MIXED step, launched asynchronously under TP (followers sample too)
                res = {"a": [], "b": []}
                eng.add_request("a", PROMPTS[0], sp)
                n = 0
                while eng.has_work() or n < 3:
                    for o in eng.step():
                        res[o.request_id].extend(o.new_token_ids)
                    n += 1
                    if n == 3:
                        eng.add_request("b", PROMPTS[1], sp)
                outs = [res["a"], res["b"]]
            else:
                outs = eng.generate(PROMPTS, sp)
            eng.stop_followers()
            mode = {"custom_ar": eng.custom_ar is not None, "graphs": bool(eng.runner.graphs), "async": eng._async,
                    "gemm_ar": eng.custom_ar is not None and eng.custom_ar.gemm_ar is not None
                    and eng.custom_ar.gemm_ar_allowed(),
                    "fused": eng.model._fused_ok, "samples": eng.runner.sample_log}
            q.put(("ok", outs, mode))
        else:
            eng.follower_loop()
            if eng.runner.sample_log is not None:
                q.put(("samples", rank, eng.runner.sample_log))
        torch.cuda.synchronize()
        destroy_distributed()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put(("err", f"rank {rank}: {e}\n{traceback.format_exc()}", None))
        raise


_UNFUSED = {"XGS_TUNE": "fused_decode=0|async_sched=0"}
_GG_AR = {"XGS_TUNE": "gemm_ar_shared=1"}


@pytest.mark.parametrize("model,moe_comm,world,env", [
    ("llama", "alltoall", 2, None), ("llama", "alltoall", 2, _UNFUSED), ("llama", "alltoall", 4, None),
    # the Llama-3-70B TP8 decode collective (8 peers, one kv head per rank): 8 processes
    # share the GPU with one hardware queue each, so every rank's kernels are co-resident
    ("llama", "alltoall", 8, {"GPU_MAX_HW_QUEUES": "1"}),
    ("mixtral", "alltoall", 2, None), ("mixtral", "allreduce", 2, None), ("mixtral", "auto", 2, None),
    ("mixtral", "alltoall", 2, {"XGS_TUNE": "ep_exact_min_pairs=0"}),
    # an arrival while decoding: the asynchronous eager mixed step under TP
    ("llama", "alltoall", 2, {"XGS_TEST_STAGGER": "1"}), ("llama", "alltoall", 4, {"XGS_TEST_STAGGER": "1"}),
    # the all-reduce inside the O / down GEMM launches (GG_AR; on separate GPUs the
    # default, here forced on for ranks sharing the GPU): graphs + async scheduling,
    # O and down at different tile widths over consecutive layers
    ("llama", "alltoall", 2, _GG_AR), ("llama", "alltoall", 2, dict(_GG_AR, XGS_TEST_STAGGER="1")),
    ("llama", "alltoall", 4, _GG_AR)])
def test_tp2_on_one_gpu_matches_fp32_reference(tmp_path, model, moe_comm, world, env):
    """Llama: TP attention + MLP shards; by default the fused TP decode layer (one
    custom all-reduce launch per row-parallel projection reduces the split-K
    partials, sums across ranks, adds the residual and emits the next norm's
    statistics), IPC LM-head gather, HIP graphs and asynchronous scheduling with
    the followers substituting their own sampled tokens; _UNFUSED is the eager
    unfused chain. Mixtral: TP=2 attention, EP=2 experts (4 + 4) exchanged by
    all-to-all (HIP dispatch kernels, fixed-capacity or count-exact splits) or
    combined by all-reduce, or "auto" (all-reduce on the custom IPC kernel for the
    decode steps, all-to-all for the prompt step)."""
    from xgserve.models import build_model, save_checkpoint
    from xgserve.models.reference import reference_logits
    from xgserve.ops import _native
    _native.kernels()
    cfg = _cfg(model)
    full = build_model(cfg, device="cuda:0", seed=7)
    ck = str(tmp_path / "ckpt")
    save_checkpoint(full, ck)

    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, ck, moe_comm, q, env)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        kind, outs, mode = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert kind == "ok", outs
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert mode["custom_ar"], mode  # decode all-reduces on the IPC kernels
    if model == "llama" and (env is None or "XGS_TEST_STAGGER" in env or env is _GG_AR):
        assert mode["graphs"] and mode["async"] and mode["fused"], mode
    # GG_AR is engaged exactly when forced on (ranks share this box's GPU)
    assert mode["gemm_ar"] == ("gemm_ar_shared=1" in (env or {}).get("XGS_TUNE", "")), mode

    base = None
    if model == "mixtral":
        # top-2 routing turns bf16-level differences into expert flips, so the bf16
        # TP=1 engine (same weights, same GPU) is the baseline: TP=2 must follow it
        # token for token until they first differ, and may differ only at a near-tie
        from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
        eng = LLMEngine(EngineConfig(model="tp-test", device="cuda:0", num_blocks=256, max_num_seqs=8,
                                     max_num_batched_tokens=1024, max_model_len=512), model=full)
        base = eng.generate(PROMPTS, SamplingParams(max_tokens=N_GEN, temperature=0.0, ignore_eos=True))
    for j, (prompt, gen) in enumerate(zip(PROMPTS, outs)):
        assert len(gen) == N_GEN
        ref = reference_logits(full, prompt + gen[:-1]).float()  # [L, V] fp32, unsharded
        for i, tok in enumerate(gen):
            row = ref[len(prompt) - 1 + i]
            gap = float(row.max() - row[tok])
            if base is not None and base[j][:i + 1] == gen[:i + 1]:
                continue  # identical to the TP=1 engine so far
            assert gap < 0.15, (i, tok, int(row.argmax()), gap)
            if base is not None:
                break  # diverged from TP=1 at a near-tie: later tokens have other prefixes


@pytest.mark.parametrize("world", [2, 4])
def test_tp_followers_sample_the_leaders_tokens(tmp_path, world):
    """Asynchronous scheduling under TP at temperature > 0: every rank
    samples the decode ids of the next step itself (graph steps and asynchronous
    eager mixed steps), from the same all-gathered logits, the leader's broadcast
    sampling rows and per-request seeds -- so every rank must draw exactly the
    leader's tokens, step by step, or the ranks' KV caches would silently diverge."""
    from xgserve.models import build_model, save_checkpoint
    from xgserve.ops import _native
    _native.kernels()
    cfg = _cfg("llama")
    ck = str(tmp_path / "ckpt")
    save_checkpoint(build_model(cfg, device="cuda:0", seed=7), ck)
    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env = {"XGS_TEST_STAGGER": "1", "XGS_TEST_TEMPERATURE": "0.8", "XGS_TEST_SAMPLE_LOG": "1"}
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, ck, "alltoall", q, env)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = []
    try:
        for _ in range(world):
            msgs.append(q.get(timeout=240))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    lead = [m for m in msgs if m[0] == "ok"]
    assert len(lead) == 1, msgs
    _, outs, mode = lead[0]
    assert all(len(g) == N_GEN for g in outs)
    assert mode["graphs"] and mode["async"], mode
    logs = {m[1]: m[2] for m in msgs if m[0] == "samples"}
    assert sorted(logs) == list(range(1, world)), msgs
    ref = mode["samples"]
    assert len(ref) >= N_GEN // 2  # graph + async steps were logged
    for r, lg in logs.items():
        assert lg == ref, (r, next((i, a, b) for i, (a, b) in enumerate(zip(lg, ref)) if a != b) if lg != ref else None)
