#!/usr/bin/env python3
"""Headline benchmark: whole-node output tokens/s (+ p50 TTFT) of Llama-3-8B
serving with continuous batching (BASELINE.json config 3: 64 concurrent
synthetic requests per GPU), one DP replica per GPU.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--concurrency 64]
                  [--prompt-len 512] [--output-len 256] [--model llama3-8b]

For N > 1 launch one rank per GPU (torch.distributed.run); ranks are
independent replicas (weak scaling: per-GPU work is fixed) and only meet at the
timing barriers. A "step" is one engine iteration (scheduler + forward of the
packed decode/prefill batch + sampling), the unit the engine serves in.
Weights are random-init bf16 of the full architecture, prompts are synthetic
token ids; finished requests are immediately replaced so the concurrency stays
at --concurrency. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import numpy as np


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0, help="(debug) torch.profiler over N timed steps")
    return ap.parse_args()


def main():
    a = parse()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch
    import torch.distributed as dist
    from xgserve.parallel.state import init_distributed
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams

    world = int(os.environ.get("WORLD_SIZE", "1"))
    st = init_distributed(tp_size=1)
    rank = st.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    max_len = a.prompt_len + 2 * a.output_len + 16
    ecfg = EngineConfig(model=a.model, device=str(dev), max_num_seqs=max(64, a.concurrency),
                        max_num_batched_tokens=a.max_batched_tokens, max_model_len=max_len,
                        use_graphs=not a.no_graphs, enable_prefix_cache=not a.no_prefix_cache,
                        graph_batch_sizes=[b for b in [1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128]
                                           if b <= max(64, a.concurrency)], seed=rank)
    eng = LLMEngine(ecfg)
    V = eng.mcfg.vocab_size
    rng = random.Random(1234 + rank)

    counter = [0]
    arrival = {}
    first_tok = {}

    def submit(max_tokens):
        rid = f"r{rank}-{counter[0]}"
        counter[0] += 1
        # random token prompts: no accidental prefix sharing across requests
        prompt = [rng.randrange(10, V - 10) for _ in range(a.prompt_len)]
        eng.add_request(rid, prompt, SamplingParams(max_tokens=max_tokens, temperature=0.0, ignore_eos=True))
        arrival[rid] = time.perf_counter()

    # staggered output lengths (uniform on [1, 2*output_len], mean output_len) ->
    # requests finish and get replaced continuously from the first steps on
    for i in range(a.concurrency):
        submit(max(1, int(round(1 + (2 * a.output_len - 1) * (i + 0.5) / a.concurrency))))

    def run_step():
        outs = eng.step()
        now = time.perf_counter()
        n_tok = 0
        for o in outs:
            n_tok += len(o.new_token_ids)
            if o.new_token_ids and o.request_id not in first_tok:
                first_tok[o.request_id] = now
            if o.finished:
                submit(a.output_len)
        return n_tok

    for _ in range(a.warmup):
        run_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start_wall = time.perf_counter()
    tokens = 0
    first_before = set(first_tok)
    for _ in range(a.steps):
        tokens += run_step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start_wall
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ttfts = [first_tok[r] - arrival[r] for r in first_tok if r not in first_before]
    p50_local = float(np.median(ttfts)) if ttfts else float("nan")

    t = torch.tensor([elapsed, float(tokens), p50_local], dtype=torch.float64, device=dev)
    if world > 1:
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, tokens, p50 = mx[0].item(), sm[1].item(), sm[2].item() / world
    else:
        p50 = p50_local
    if rank == 0:
        value = tokens / elapsed
        st_ = eng.stats()
        print(json.dumps({
            "metric": "output_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random-token prompts, random-init weights)",
            "ttft_p50_ms": round(1000 * p50, 2) if p50 == p50 else None,
            "config": {"model": a.model, "global_batch": a.concurrency * world,
                       "seq_len": a.prompt_len + a.output_len, "prompt_len": a.prompt_len,
                       "output_len": a.output_len, "parallelism": f"dp{world}",
                       "concurrency_per_gpu": a.concurrency},
            "detail": {"preemptions": st_["preemptions"], "kv_blocks": st_["kv_blocks_total"],
                       "decode_steps_total": st_["decode_steps"], "steps_total": st_["steps"]},
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
