#!/usr/bin/env python3
"""Prefill-GEMM shoot-out on one MI355X: y = x . W^T at Llama-3 projection shapes
for prefill-sized M (mixed continuous-batching steps, long prompts). Compares
hipBLASLt and rocBLAS (torch F.linear with each preferred BLAS library) and the
hand-written MFMA kernel (xgserve.ops.gemm_mfma) when built; prints one JSON line
per (shape, M, backend) with us and TFLOP/s, and checks the kernel's numerics
against an fp32 reference."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "qkv70t8": (1280, 8192), "o70t8": (8192, 1024), "gate_up70t8": (7168, 8192), "down70t8": (8192, 3584),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=20, warm=3):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[128, 256, 575, 1024, 2048, 8192])
    ap.add_argument("--shapes", nargs="+", default=["qkv", "o", "gate_up", "down"])
    ap.add_argument("--backends", nargs="+", default=["hipblaslt", "hipblas", "ck", "mfma"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.shapes:
        N, K = SHAPES[name]
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        for M in a.M:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = None
            for be in a.backends:
                rec = {"shape": name, "N": N, "K": K, "M": M, "backend": be}
                if be in ("hipblaslt", "hipblas", "ck"):
                    torch.backends.cuda.preferred_blas_library(be)
                    fn = lambda: F.linear(x, w)  # noqa: E731
                else:
                    try:
                        from xgserve.ops.gemm_mfma import gemm_mfma, gemm_mfma_ok
                    except ImportError:
                        continue
                    if not gemm_mfma_ok(M, N, K):
                        continue
                    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                    fn = lambda: gemm_mfma(x, w, out=out)  # noqa: E731
                    if ref is None:
                        ref = (x.float() @ w.float().t())
                    y = fn().float()
                    rec["max_err"] = float((y - ref).abs().max())
                    rec["ref_absmax"] = float(ref.abs().max())
                us = timeit(fn)
                rec["us"] = round(us, 2)
                rec["tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
                print(json.dumps(rec), flush=True)
    torch.backends.cuda.preferred_blas_library("hipblaslt")


if __name__ == "__main__":
    main()
