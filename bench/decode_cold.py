#!/usr/bin/env python3
"""Decode attention at 64 concurrent with a COLD Infinity Cache: the engine reads
each layer's K/V once per step (5.4 GB per step for Llama-3-8B at ~640 keys), but a
micro-benchmark that repeats one layer's 168 MB keeps it in the 256 MB Infinity Cache
and reads high. Here the timed calls rotate over --caches independent paged caches
(> 1 GB together), like the engine's walk over its 32 layers.
Prints one JSON line per (form, splits): us per call and K/V TB/s."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve import ops  # noqa: E402
from xgserve.ops.linear import PendingSum  # noqa: E402


def make_cache(B, lens, Hkv, D, bs, dev, g):
    pages = [(int(L) + bs - 1) // bs for L in lens]
    NB = sum(pages) + 8
    kc = (torch.randn(NB, Hkv, bs, D, device=dev) * 0.5).bfloat16()
    vc = torch.randn(NB, Hkv, bs, D, device=dev).bfloat16()
    perm = torch.randperm(NB, generator=g).tolist()
    W = max(pages)
    bt = torch.zeros(B, W, dtype=torch.int32)
    i = 0
    for b, n in enumerate(pages):
        bt[b, :n] = torch.tensor(perm[i:i + n])
        i += n
    return kc, vc, bt.to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--L", type=int, default=768)
    ap.add_argument("--stagger", type=int, default=256)
    ap.add_argument("--caches", type=int, default=7)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--iters", type=int, default=70)
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--depth", type=int, nargs="+", default=[2])
    ap.add_argument("--arrange", default="random", choices=["random", "pair", "sorted"],
                    help="sequence order: random lengths; pair = seq b and b + B/2 complement each other "
                         "(short + long); sorted = ascending")
    ap.add_argument("--graph", action="store_true",
                    help="time `iters` calls captured in one HIP graph (device time; an eager Python loop is "
                         "host-bound below ~10 us per call)")
    ap.add_argument("--probe", action="store_true",
                    help="anatomy: also time the kernel without its prologue (11), key loop (12), both (13)")
    a = ap.parse_args()
    if a.probe:  # the probe kernels live only in a probe build of _kernels.so
        from xgserve import _build
        _build.build_kernels(probes=True)
    dev, Hq, Hkv, D, bs = "cuda", 32, 8, 128, a.bs
    B = a.B
    g = torch.Generator().manual_seed(0)
    lens = (a.L - torch.randint(0, max(a.stagger, 1), (B,), generator=g)).int()
    if a.arrange != "random":
        srt = torch.sort(lens).values
        if a.arrange == "sorted":
            lens = srt
        else:  # b < B/2 takes the i-th shortest, b + B/2 the i-th longest
            lens = torch.cat([srt[: B // 2], srt[B // 2:].flip(0)]).int()
    caches = [make_cache(B, lens, Hkv, D, bs, dev, g) for _ in range(a.caches)]
    lens = lens.to(dev)
    pos = (lens - 1).int()
    cs = torch.randn(a.L + 16, D, device=dev)
    pend = PendingSum(torch.randn(4, B, (Hq + 2 * Hkv) * D, device=dev), 4)
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    ws = ops.attention.DecodeWorkspace(B, Hq, D, 16, dev)
    nbytes = int(lens.sum().item()) * Hkv * D * 2 * 2
    sc = 1 / math.sqrt(D)
    slots = []
    for kc, vc, bt in caches:
        slots.append((bt.gather(1, (pos // bs).long().view(B, 1)).view(B) * bs + pos % bs).int())

    def run(i, S, dp):
        kc, vc, bt = caches[i % len(caches)]
        ops.decode_attention_fused(pend, pos, slots[i % len(caches)], cs, kc, vc, bt, lens, Hq, sc, S, ws, out=out,
                                   depth=dp)

    depths = list(a.depth) + ([11, 12, 13] if a.probe else [])
    for S, dp, mode in [(S, dp, m) for S in a.splits for dp in depths for m in ("warm", "cold")]:
        if True:
            f = (lambda i: run(0, S, dp)) if mode == "warm" else (lambda i: run(i, S, dp))
            for i in range(2 * len(caches)):
                f(i)
            torch.cuda.synchronize()
            body = lambda: [f(i) for i in range(a.iters)]  # noqa: E731
            if a.graph:
                gs = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(gs):
                    with torch.cuda.graph(g, stream=gs):
                        body()
                torch.cuda.synchronize()
                body = g.replay
                body()
                torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            body()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1000.0
            print(json.dumps({"op": "decode_attention_fq", "cache": mode, "B": B, "L": a.L, "stagger": a.stagger, "bs": bs,
                              "splits": S, "depth": dp, "arrange": a.arrange, "graph": a.graph, "us": round(us, 2), "TB/s": round(nbytes / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
