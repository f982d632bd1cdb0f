#!/usr/bin/env python3
"""Fused decode-layer GEMM forms vs their plain forms at small M, graph-timed with
cold weights (a ring of weight copies larger than the Infinity Cache):

  qkv / gate_up : m64_linear on a pre-normalised x   vs  m64_norm_linear (RMSNorm as
                  a row scale from per-tile statistics, ss_n of them)
  o / down      : m64_linear (partials)               vs  m64_resid_linear (GG_RESID:
                  residual add + next statistics in the launch)

Shapes: --model llama3-8b | llama3-70b with --tp (shard of one rank).

  python bench/fused_gemm_bench.py --model llama3-70b --tp 8 --M 1
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

DIMS = {"llama3-8b": (4096, 14336, 32, 8), "llama3-70b": (8192, 28672, 64, 8)}


def graph_time(fns, iters=40):
    """Device time per call of fns cycled (one graph of `iters` calls, replayed)."""
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
    ap.add_argument("--model", default="llama3-70b", choices=list(DIMS))
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--M", type=int, nargs="+", default=[1])
    ap.add_argument("--sweep", action="store_true",
                    help="every valid (nw, S, cfg) of the FUSED form (norm128 / resid), fastest first")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    kernels()
    H, F, Hq, Hkv = DIMS[a.model]
    D = H // Hq
    t = a.tp
    shapes = {"qkv": ((Hq + 2 * Hkv) * D // t, H, L.MODE_PARTIAL, "norm"),
              "gate_up": (2 * F // t, H, L.MODE_SILU, "norm"),
              "o": (H, Hq * D // t, L.MODE_PARTIAL, "resid"),
              "down": (H, F // t, L.MODE_PARTIAL, "resid")}
    dev = torch.device("cuda")
    for name, (N, K, mode, kind) in shapes.items():
        nbytes = N * K * 2
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(copies)]
        for M in a.M:
            x = torch.randn(M, K, device=dev).bfloat16()
            plan = L.m64_plan(M, N, K, mode)
            rows = {}
            if plan is None:
                print(json.dumps({"shape": name, "M": M, "skip": "no plan"}), flush=True)
                continue
            rows["plain"] = graph_time([lambda w=w: L.m64_linear(x, w, mode) for w in ws])
            if kind == "norm":
                for n_parts in (8, 64, 128):
                    if n_parts > 128 or (M > 16 and n_parts > 64):
                        continue
                    ss = torch.rand(n_parts, M, device=dev) * K / n_parts
                    st = L.RowStats(ss, n_parts, M)
                    rows[f"norm{n_parts}"] = graph_time([lambda w=w, st=st: L.m64_norm_linear(x, w, mode, st, 1e-5)
                                                         for w in ws])
            else:
                rw = L.ResidWorkspace(4, max(64, M), N, dev)
                resid = torch.randn(M, N, device=dev).bfloat16()
                rows["resid"] = graph_time([lambda w=w: L.m64_resid_linear(x, w, resid, rw, 1, 1e-5) for w in ws])
            if a.sweep:
                res = []
                for cfg, (wv, kc, _) in L.M64G_CFGS.items():
                    for nw in ((2,) if mode == L.MODE_SILU else (1, 2)):
                        for S in ((1, 2, 4) if mode == L.MODE_SILU else (1, 2, 3, 4, 6, 8)):
                            p = (nw, S, cfg)
                            if not L._m64_valid(N, K, mode, nw, S, cfg, M) or (mode == L.MODE_SILU and K % (S * kc)):
                                continue
                            try:
                                if kind == "norm":
                                    n_parts = 128 if M <= 16 else 64
                                    st = L.RowStats(torch.rand(n_parts, M, device=dev) * K / n_parts, n_parts, M)
                                    us = graph_time([lambda w=w, st=st, p=p: L.m64_norm_linear(x, w, mode, st, 1e-5,
                                                                                               plan=p) for w in ws])
                                else:
                                    us = graph_time([lambda w=w, p=p: L.m64_resid_linear(x, w, resid, rw, 1, 1e-5,
                                                                                         plan=p) for w in ws])
                            except (ValueError, RuntimeError):
                                continue
                            res.append((us, p))
                res.sort()
                print(json.dumps({"shape": name, "M": M, "fused_sweep": [[round(u, 2), list(p)] for u, p in res[:a.top]],
                                  "shipped": list(plan)}), flush=True)
            base = rows["plain"]
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "plan": plan,
                              **{k: round(v, 2) for k, v in rows.items()},
                              "TB/s_plain": round(nbytes / base / 1e6, 2)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
