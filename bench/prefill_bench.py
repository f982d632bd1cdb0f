#!/usr/bin/env python3
"""Prefill attention (K5) throughput on one MI355X: one sequence of L new tokens
(no cached prefix) over the paged KV cache, causal, for L in --lens, Llama-3-8B
(32 q / 8 kv heads) and Llama-3-70B (64 / 8) head layouts, every GQA head-group
width `gh` (query heads per workgroup). TFLOP/s counts the causal work:
4 * Hq * D * L (L + 1) / 2. Also --ttft: end-to-end batch-1 TTFT of one
--ttft-len-token prompt through the engine (random-init Llama-3-8B, bf16)."""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve import ops  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402


def bench_attn(L, Hq, Hkv, D, gh, iters=20, bs=16):
    n_pages = (L + bs - 1) // bs
    kc = (torch.randn(n_pages, Hkv, bs, D, device="cuda") * 0.5).bfloat16()
    vc = torch.randn(n_pages, Hkv, bs, D, device="cuda").bfloat16()
    bt = torch.randperm(n_pages, device="cuda", dtype=torch.int32)[None, :].contiguous()
    q = torch.randn(L, Hq, D, device="cuda").bfloat16()
    qsl = torch.tensor([0, L], dtype=torch.int32, device="cuda")
    sl = torch.tensor([L], dtype=torch.int32, device="cuda")
    out = torch.empty_like(q)
    fn = lambda: ops.prefill_attention(q, kc, vc, bt, qsl, sl, L, 1.0 / math.sqrt(D), out=out, gh=gh)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1000.0
    flops = 4.0 * Hq * D * L * (L + 1) / 2
    return us, flops / us / 1e6


def ttft(L):
    from xgserve.engine import EngineConfig, LLMEngine, SamplingParams
    eng = LLMEngine(EngineConfig(model="llama3-8b", max_num_seqs=4, max_num_batched_tokens=max(8192, L),
                                 max_model_len=L + 16, graph_batch_sizes=[1]))
    res = []
    for it in range(4):
        prompt = torch.randint(10, 128000, (L,)).tolist()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.add_request(f"t{it}", prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
        done = False
        while not done:
            for o in eng.step():
                if o.new_token_ids:
                    done = True
        res.append(1000 * (time.perf_counter() - t0))
        eng.clear_prefix_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", type=int, nargs="*", default=[512, 2048, 8192])
    ap.add_argument("--gh", type=int, nargs="+", default=[0, 4, -44, -84, -82, -1284, -1282, -1281])
    ap.add_argument("--ttft-len", type=int, default=8000)
    ap.add_argument("--no-ttft", action="store_true")
    a = ap.parse_args()
    kernels()
    for name, Hq, Hkv in (("llama3-8b", 32, 8), ("llama3-70b", 64, 8)):
        for L in a.lens:
            for gh in a.gh:
                us, tf = bench_attn(L, Hq, Hkv, 128, gh)
                print(json.dumps({"op": "prefill_attention", "heads": name, "L": L, "gh": gh, "us": round(us, 1),
                                  "TFLOP/s": round(tf, 1)}), flush=True)
    if not a.no_ttft:
        r = ttft(a.ttft_len)
        print(json.dumps({"op": "ttft_batch1", "model": "llama3-8b", "prompt_len": a.ttft_len,
                          "ttft_ms": [round(x, 2) for x in r], "ttft_ms_best_of_last3": round(min(r[1:]), 2)}),
              flush=True)


if __name__ == "__main__":
    main()
