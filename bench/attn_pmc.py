"""Tiny driver for rocprofv3 --pmc passes over the prefill attention kernel: one
Llama-3-8B-headed causal prompt of --L tokens, the default configuration (gh 0) and
any forced ones (--gh), a few launches each (bench/pf_pmc.sh DRIVER=bench/attn_pmc.py)."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xgserve import ops  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=8192)
ap.add_argument("--gh", type=int, nargs="+", default=[0])
ap.add_argument("--iters", type=int, default=3)
a = ap.parse_args()
kernels()
Hq, Hkv, D, bs, L = 32, 8, 128, 16, a.L
n_pages = (L + bs - 1) // bs
kc = (torch.randn(n_pages, Hkv, bs, D, device="cuda") * 0.5).bfloat16()
vc = torch.randn(n_pages, Hkv, bs, D, device="cuda").bfloat16()
bt = torch.randperm(n_pages, device="cuda", dtype=torch.int32)[None, :].contiguous()
q = torch.randn(L, Hq, D, device="cuda").bfloat16()
qsl = torch.tensor([0, L], dtype=torch.int32, device="cuda")
sl = torch.tensor([L], dtype=torch.int32, device="cuda")
out = torch.empty_like(q)
for gh in a.gh:
    for _ in range(a.iters):
        ops.prefill_attention(q, kc, vc, bt, qsl, sl, L, 1.0 / math.sqrt(D), out=out, gh=gh)
torch.cuda.synchronize()
print("done")
