"""Tiny driver for rocprofv3 --pmc passes over gemm_pf: the 8B gate_up at M = 575
(SiLU epilogue) with the given cfgs (default: the 288-row tile and its no-DMA probe)
and the library GEMM, a few launches each."""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=575)
ap.add_argument("--N", type=int, default=28672)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--cfgs", type=int, nargs="+", default=[5, 13])
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
kernels()
x = torch.randn(a.M, a.K, device="cuda").bfloat16()
w = (torch.randn(a.N, a.K, device="cuda") * 0.02).bfloat16()
for cfg in a.cfgs:
    for _ in range(a.iters):
        L.pf_linear(x, w, L.MODE_SILU, plan=(1, cfg))
for _ in range(a.iters):
    F.linear(x, w)
torch.cuda.synchronize()
print("done")
