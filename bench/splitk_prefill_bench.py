#!/usr/bin/env python3
"""Prefill-sized projections (M ~ 512-2048) on one MI355X: the library GEMM
(F.linear -> hipBLASLt / rocBLAS, with the engine's shipped selection table) against
a split-K form -- one strided-batched GEMM over S slices of K with fp32 outputs
(torch.bmm out_dtype=float32), reduced later by the consumer kernel
(add_partials_rmsnorm) -- which gives N = 4096 projections S x the tiles. Prints
one JSON line per (shape, M, variant): us, TFLOP/s, rel err vs fp32."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve import tuning  # noqa: E402
from xgserve.ops import _native  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "o70": (8192, 8192), "down70": (8192, 28672)}


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def split_k(x, w, S):
    M, K = x.shape
    N = w.shape[0]
    a = x.view(M, S, K // S).permute(1, 0, 2)          # [S, M, K/S], row stride K
    b = w.view(N, S, K // S).permute(1, 2, 0)          # [S, K/S, N], column-major slices of W
    return torch.bmm(a, b, out_dtype=torch.float32)    # [S, M, N] fp32 partials


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[575, 1024, 2048])
    ap.add_argument("--shapes", nargs="+", default=["o", "down", "qkv"])
    ap.add_argument("--splits", type=int, nargs="+", default=[2, 4])
    a = ap.parse_args()
    _native.kernels()
    tuning.enable_gemm_table(torch.device("cuda"))
    for name in a.shapes:
        N, K = SHAPES[name]
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        for M in a.M:
            x = torch.randn(M, K, device="cuda").bfloat16()
            ref = x.float() @ w.float().t()
            fl = 2.0 * M * N * K
            rows = [("linear", timeit(lambda: F.linear(x, w)), F.linear(x, w).float())]
            for S in a.splits:
                if K % S:
                    continue
                try:
                    y = split_k(x, w, S).sum(0)
                except Exception as ex:  # noqa: BLE001
                    print(json.dumps({"shape": name, "M": M, "op": f"splitk{S}", "error": str(ex)[:200]}), flush=True)
                    continue
                rows.append((f"splitk{S}", timeit(lambda S=S: split_k(x, w, S)), y))
            for op, us, y in rows:
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "op": op, "us": round(us, 2),
                                  "TFLOP/s": round(fl / us / 1e6, 1),
                                  "rel_err": float((y - ref).norm() / ref.norm())}), flush=True)


if __name__ == "__main__":
    main()
