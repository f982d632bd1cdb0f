"""Tensor / expert parallelism at full degree on the CPU (gloo, one process per
rank): TP=4 and TP=8 of a GQA model with 8 kv heads (TP=8 -> ONE kv head per
rank, the Llama-3-70B TP8 layout) and a vocabulary that does not divide by the
TP degree (the vocab-parallel LM head pads to V_pad and the gather trims it);
Mixtral-style EP=4 (8 experts, 2 per rank) with both exchange modes, the
all_to_all one both with fixed-capacity and with count-exact splits.

Every rank loads its shard of the same safetensors checkpoint; the leader
drives the engine and the followers mirror its plans. Each greedily decoded
token must be the argmax of the unsharded fp32 reference logits at its
position, up to an fp32-rounding-sized near-tie (TP only changes the order of
fp32 sums). Reference: design.md:1046-1053 (multi-worker coordination tests)."""
from __future__ import annotations

import os
import socket
from dataclasses import replace

import pytest
import torch

PROMPTS = [[1] + list(range(10, 70)), [1, 5, 6, 7, 8]]
N_GEN = 6


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(kind):
    from xgserve.models import get_config
    if kind == "gqa8":
        return replace(get_config("llama-tiny-gqa8"), vocab_size=509, name="tp-cpu-test", dtype="float32")
    return replace(get_config("mixtral-tiny"), vocab_size=509, name="tp-cpu-test", dtype="float32")


def _rank_main(rank, world, port, ck, moe_comm, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    if moe_comm == "alltoall-exact":  # every step on the count-exact (packed) EP dispatch
        os.environ["XGS_TUNE"] = "ep_exact_min_pairs=0"
        moe_comm = "alltoall"
    torch.set_num_threads(1)
    try:
        from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
        from xgserve.parallel.state import destroy_distributed, init_distributed
        init_distributed(tp_size=world, backend="gloo", device=torch.device("cpu"), timeout_s=120)
        eng = LLMEngine(EngineConfig(model="tp-cpu-test", checkpoint=ck, tp=world, device="cpu", dtype="float32",
                                     num_blocks=64, max_num_seqs=4, max_num_batched_tokens=128, max_model_len=256,
                                     moe_comm=moe_comm, use_graphs=False))
        info = (eng.model.V_pad, eng.model.num_kv_heads_local, eng.model.layers[0].qkv.shape[0])
        if rank == 0:
            outs = eng.generate(PROMPTS, SamplingParams(max_tokens=N_GEN, temperature=0.0, ignore_eos=True))
            eng.stop_followers()
            q.put((rank, "ok", outs, info))
        else:
            eng.follower_loop()
            q.put((rank, "ok", None, info))
        destroy_distributed()
    except Exception as e:  # noqa: BLE001 - reported to the parent
        import traceback
        q.put((rank, "err", f"{e}\n{traceback.format_exc()}", None))


@pytest.mark.parametrize("kind,world,moe_comm", [("gqa8", 4, "alltoall"), ("gqa8", 8, "alltoall"),
                                                 ("mixtral", 4, "alltoall"), ("mixtral", 4, "alltoall-exact"),
                                                 ("mixtral", 2, "alltoall-exact"), ("mixtral", 4, "allreduce"),
                                                 ("mixtral", 2, "auto")])
def test_tp_full_degree_matches_fp32_reference(tmp_path, kind, world, moe_comm):
    from xgserve.models import build_model, save_checkpoint
    from xgserve.models.reference import reference_logits
    cfg = _cfg(kind)
    full = build_model(cfg, device="cpu", dtype=torch.float32, seed=11)
    ck = str(tmp_path / "ckpt")
    save_checkpoint(full, ck)

    ctx = torch.multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, ck, moe_comm, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = {}
        for _ in procs:
            rank, kind_, payload, info = q.get(timeout=240)
            res[rank] = (kind_, payload, info)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = {r: v[1] for r, v in res.items() if v[0] != "ok"}
    assert not errs, errs
    V_pad, hkv_local, qkv_rows = res[0][2]
    assert V_pad % world == 0 and V_pad >= cfg.vocab_size and V_pad != cfg.vocab_size  # padding exercised
    if kind == "gqa8":
        assert hkv_local == cfg.num_kv_heads // world
        assert qkv_rows == (cfg.num_heads // world + 2 * hkv_local) * cfg.head_dim
    outs = res[0][1]
    for prompt, gen in zip(PROMPTS, outs):
        assert len(gen) == N_GEN
        ref = reference_logits(full, prompt + gen[:-1]).float()
        for i, tok in enumerate(gen):
            row = ref[len(prompt) - 1 + i]
            assert tok < cfg.vocab_size
            assert float(row.max() - row[tok]) < 1e-3, (i, tok, int(row.argmax()))
