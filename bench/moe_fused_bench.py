#!/usr/bin/env python3
"""Mixtral decode expert GEMMs in the forms the fused decode layer runs them, graph-
timed with cold weights (two copies of the layer's experts, alternated):

  w13 : grouped gemm_m64g, SiLU gate in the epilogue, x rows gathered by the layout
  w2  : grouped gemm_m64g with the MoE combine into the residual stream in the launch
        (GG_MOE_RESID), split-K S

Sweeps w13 cfg and w2 (nw, cfg, S) at T tokens (default 1, k = 2) and prints the
fastest configurations next to the shipped ones (xgserve/ops/moe.py).

  python bench/moe_fused_bench.py --T 1
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve.ops import moe as MO  # noqa: E402
from xgserve.ops._native import kernels, stream_ptr  # noqa: E402


def graph_time(fns, iters=32):
    for f in fns:
        f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(iters):
                fns[i % len(fns)]()
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1000.0 / (reps * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[1])
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    kn = kernels()
    dev = torch.device("cuda")
    E, H, F, k = 8, 4096, 14336, 2
    copies = 2
    w13s = [(torch.randn(E, 2 * F, H, device=dev) * 0.02).bfloat16() for _ in range(copies)]
    w2s = [(torch.randn(E, H, F, device=dev) * 0.02).bfloat16() for _ in range(copies)]
    for T in a.T:
        torch.manual_seed(T)
        ids = torch.stack([torch.randperm(E, device=dev)[:k] for _ in range(T)]).int()
        topw = torch.softmax(torch.randn(T, k, device=dev), -1)
        x = torch.randn(T, H, device=dev).bfloat16()
        sorted_rows, offs, dest = MO.moe_align(ids, E, 0)
        P = sorted_rows.shape[0]
        act = torch.empty(P, F, dtype=torch.bfloat16, device=dev)
        resid = torch.randn(T, H, device=dev).bfloat16()
        ss = torch.zeros(64 * max(T, 64), dtype=torch.float32, device=dev)
        counters = torch.zeros(4096, dtype=torch.int32, device=dev)
        twf = topw.float().contiguous()
        max_rows = T * k
        valid = sorted_rows.data_ptr()

        def w13(cfg, w):
            kn.moe_gemm_m64g_rows(x.data_ptr(), sorted_rows.data_ptr(), offs.data_ptr(), E, H, w.data_ptr(), 2 * F, P,
                                  0, act.data_ptr(), 1, 2, 2, cfg, max_rows, stream_ptr(), valid, T * k)

        res13 = []
        for cfg in range(7):
            try:
                us = graph_time([lambda w=w, cfg=cfg: w13(cfg, w) for w in w13s])
            except (RuntimeError, ValueError):
                continue
            res13.append((round(us, 2), cfg))
        res13.sort()
        print(json.dumps({"T": T, "w13_sweep": res13[:a.top], "shipped_cfg": MO.MOE_CFG_W13}), flush=True)

        res2 = []
        for nw in (1, 2):
            for cfg in range(7):
                cols = 16 * nw * MO.M64G_CFG_WAVES[cfg]
                if H % cols or H // cols > 64:
                    continue
                for S in (1, 2, 4, 8):
                    part = torch.empty(S, P, H, dtype=torch.float32, device=dev)

                    def w2(w, nw=nw, cfg=cfg, S=S, part=part):
                        kn.moe_gemm_m64g_resid(act.data_ptr(), 0, offs.data_ptr(), E, F, w.data_ptr(), H, P,
                                               part.data_ptr(), S, nw, cfg, max_rows, stream_ptr(), valid,
                                               dest.data_ptr(), twf.data_ptr(), resid.data_ptr(), ss.data_ptr(),
                                               counters.data_ptr(), T, k, T * k)
                    try:
                        us = graph_time([lambda w=w, f=w2: f(w) for w in w2s])
                    except (RuntimeError, ValueError):
                        continue
                    res2.append((round(us, 2), [nw, cfg, S]))
        res2.sort()
        print(json.dumps({"T": T, "w2_resid_sweep": res2[:a.top], "shipped": [2, MO.MOE_CFG_W2, "S by T*k"]}),
              flush=True)


if __name__ == "__main__":
    main()
