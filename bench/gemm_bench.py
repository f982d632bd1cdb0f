#!/usr/bin/env python3
"""Decode-GEMM shoot-out on one MI355X: hipBLASLt (F.linear) vs the hand-written
kernels at the Llama-3-8B projection shapes, cold weights (a ring of weight
copies larger than the 256 MB Infinity Cache, as in a real decode step where
every layer's weights are touched once). Also checks numerics vs fp32."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fns, iters=30, warm=5):
    """fns: list of zero-arg callables cycled per iteration (distinct weight copies)."""
    for i in range(warm):
        fns[i % len(fns)]()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fns[i % len(fns)]()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--shapes", nargs="+", default=list(SHAPES))
    ap.add_argument("--variants", type=int, nargs="+", default=[2, 4])
    a = ap.parse_args()
    kernels()
    dev = "cuda"
    for name in a.shapes:
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(8, (1 << 30) // nbytes + 1))
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(copies)]
        for M in a.M:
            x = torch.randn(M, K, device=dev).bfloat16()
            ref = x.float() @ ws[0].float().t()
            rows = []
            us = timeit([lambda w=w: F.linear(x, w) for w in ws])
            rows.append(("hipblaslt", us, None))
            mode = L.MODE_SILU if name == "gate_up" else (L.MODE_BF16 if name == "lm_head" else L.MODE_PARTIAL)
            if M <= 16:
                for S in ((1,) if mode != L.MODE_PARTIAL else (1, 2, 4, 7, 8, 14, 16)):
                    if K % (S * 256) or (mode == L.MODE_PARTIAL and N % 64):
                        continue
                    fn = lambda w, S=S: L.skinny_linear(x, w, S, mode)  # noqa: E731
                    us3 = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                    rows.append((f"skinny(S={S},mode={mode})", us3, None))
            plan = L.m64_plan(M, N, K, mode)
            if plan is not None:
                for nw in ((1, 2) if mode == L.MODE_PARTIAL and N % 128 == 0 else (plan[0],)):
                    S = plan[1] if nw == plan[0] else L.m64_plan(M, N, K, mode)[1] * (2 if nw < plan[0] else 1)
                    if mode != L.MODE_PARTIAL:
                        S = 1
                    if K % (S * 256):
                        continue
                    for var in a.variants:
                        fn = lambda w, nw=nw, S=S, var=var: L.m64_linear(x, w, mode, S, nw, variant=var)  # noqa: E731
                        us2 = timeit([lambda w=w, fn=fn: fn(w) for w in ws])
                        y = fn(ws[0])
                        if mode == L.MODE_PARTIAL:
                            y = y.part.sum(0)
                            want = ref
                        elif mode == L.MODE_SILU:
                            g, u = L.deinterleave_gate_up(ws[0])
                            want = F.silu(x.float() @ g.float().t()) * (x.float() @ u.float().t())
                        else:
                            want = ref
                        err = float((y.float() - want).norm() / want.norm())
                        rows.append((f"gemm_m64(nw={nw},S={S},mode={mode},var={var})", us2, err))
            if M <= 16 or plan is None:
                pass
            for op, t, err in rows:
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "op": op, "us": round(t, 2),
                                  "TB/s": round(nbytes / t / 1e6, 3), "rel_err": err}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
