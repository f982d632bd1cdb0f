#!/usr/bin/env python3
"""Prompt-sized expert GEMMs of a Mixtral 8x7B layer: the grouped gemm_m64g path vs
gemm_pf's grouped form (xgserve/ops/moe.py fused_moe), whole fused_moe calls timed
with events, random routing of T tokens (top-2 of 8). One JSON line per (T, path)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xgserve import ops  # noqa: E402
from xgserve.ops import moe as MOE  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[575, 1024])
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--H", type=int, default=4096)
    ap.add_argument("--F", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cfg", type=int, nargs="*", default=[], help="gemm_pf tiles to force (6 / 7 / 8)")
    a = ap.parse_args()
    dev = "cuda"
    E, H, F = a.E, a.H, a.F
    w13 = (torch.randn(E, 2 * F, H, device=dev) * 0.02).bfloat16()
    w2 = (torch.randn(E, H, F, device=dev) * 0.02).bfloat16()
    for T in a.T:
        x = torch.randn(T, H, device=dev).bfloat16()
        w, ids = ops.moe_topk_softmax(torch.randn(T, E, device=dev), 2)
        variants = [("m64g", False, None)] + [("pf", True, None)] + [(f"pf_c{c}", True, c) for c in a.cfg]
        for name, on, cfg in variants:
            MOE.MOE_PF = on
            keep = MOE._moe_pf_cfg
            if cfg is not None:
                MOE._moe_pf_cfg = lambda pairs, E_, c=cfg: c
            for _ in range(3):
                ops.fused_moe(x, w13, w2, w, ids)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ops.fused_moe(x, w13, w2, w, ids)
            e.record()
            torch.cuda.synchronize()
            MOE._moe_pf_cfg = keep
            us = s.elapsed_time(e) / a.iters * 1000
            print(json.dumps({"op": "fused_moe", "T": T, "path": name, "us": round(us, 1),
                              "expert_rows_max": int(torch.bincount(ids.flatten().long(), minlength=E).max())}),
                  flush=True)


if __name__ == "__main__":
    main()
