#!/usr/bin/env python3
"""hipBLASLt (F.linear) throughput at prefill-chunk shapes (Llama-3-8B projections)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


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


def main():
    args = sys.argv[1:]
    tag = "hipblaslt"
    if args and args[0] == "--tunable":  # PyTorch TunableOp: benchmark rocBLAS + hipBLASLt solutions per shape
        args = args[1:]
        tag = "tunableop"
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_max_tuning_duration(200)
        torch.cuda.tunable.set_filename(os.environ.get("TUNABLE_FILE", "/tmp/tunableop.csv"))
    Ms = [int(m) for m in args] or [512, 575, 576, 640, 768, 1024, 2048, 4096]
    for name, (N, K) in SHAPES.items():
        w = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        for M in Ms:
            x = torch.randn(M, K, device="cuda").bfloat16()
            us = timeit(lambda: F.linear(x, w))
            print(json.dumps({"op": tag, "shape": name, "M": M, "us": round(us, 2), "TFLOP/s": round(2 * M * N * K / us / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
