#!/usr/bin/env python3
"""gemm_pf (csrc/kernels/gemm_pf.hip) vs hipBLASLt at prompt-sized M on one MI355X.

Numerics against an fp32 torch reference, then interleaved timing rounds in ONE
process (cdna_hip_programming.md §5.4 rule 24): per (shape, M), every variant is
timed once per round for `--rounds` rounds on random bf16 operands; median and
min are reported as JSON lines. Weights rotate over enough copies to exceed the
256 MB Infinity Cache (cold, as in a real step)."""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve import ops  # noqa: E402
from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402

SHAPES = {"qkv": (6144, 4096, L.MODE_BF16), "o": (4096, 4096, L.MODE_BF16),
          "gate_up": (28672, 4096, L.MODE_SILU), "down": (4096, 14336, L.MODE_BF16),
          "qkv_p": (6144, 4096, L.MODE_PARTIAL), "o_p": (4096, 4096, L.MODE_PARTIAL),
          "down_p": (4096, 14336, L.MODE_PARTIAL), "gate_up_bf16": (28672, 4096, L.MODE_BF16),
          "sq4k": (4096, 4096, L.MODE_BF16), "sq8k": (8192, 8192, L.MODE_BF16)}


def ref(x, w, mode):
    y = x.float() @ w.float().t()
    if mode == L.MODE_SILU:
        g, u = L.deinterleave_gate_up(w)
        yg, yu = x.float() @ g.float().t(), x.float() @ u.float().t()
        return torch.nn.functional.silu(yg) * yu
    return y


def run_pf(x, w, mode, plan):
    r = L.pf_linear(x, w, mode, plan=plan)
    return r.part.sum(0) if mode == L.MODE_PARTIAL else r


def time_rounds(fns, rounds, iters):
    """fns: {name: callable(i)}; returns {name: [us per call per round]}"""
    out = {k: [] for k in fns}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f in fns.values():
        for i in range(3):
            f(i)
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            s.record()
            for i in range(iters):
                f(i)
            e.record()
            torch.cuda.synchronize()
            out[k].append(s.elapsed_time(e) / iters * 1000.0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="+", default=["gate_up", "down_p", "qkv_p", "o_p"])
    ap.add_argument("--M", type=int, nargs="+", default=[575, 1024, 2048])
    ap.add_argument("--cfgs", type=int, nargs="+", default=None, help="gemm_pf cfgs to time (default: the plan's)")
    ap.add_argument("--splits", type=int, nargs="+", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--probe", action="store_true", help="also time the no-DMA / no-MFMA anatomy builds")
    ap.add_argument("--krot", action="store_true", help="also time each variant with K-tile rotation on")
    a = ap.parse_args()
    if a.probe:  # the probe kernels live only in a probe build of _kernels.so
        from xgserve import _build
        _build.build_kernels(probes=True)
    kernels()
    torch.manual_seed(0)
    dev = "cuda"
    # the library baselines run with the shipped TunableOp table, as in the engine
    from xgserve.tuning import enable_gemm_table
    print(json.dumps({"gemm_table": enable_gemm_table(torch.device(dev))}), flush=True)
    for name in a.shapes:
        N, K, mode = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, min(6, (600 << 20) // nbytes + 1))
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(copies)]
        for M in a.M:
            x = torch.randn(M, K, device=dev).bfloat16()
            plan = L.pf_plan(M, N, K, mode)
            cfgs = a.cfgs if a.cfgs is not None else [plan[1]]
            splits = a.splits if (a.splits is not None and mode == L.MODE_PARTIAL) else [plan[0]]
            variants = {}
            for cfg in cfgs:
                for S in splits:
                    variants[f"pf_c{cfg}_s{S}"] = (S, cfg)
            probes = {}
            if a.probe:
                for k, (S, cfg) in list(variants.items()):
                    probes[k + "_nodma"] = (S, cfg % 16 + 16)
                    probes[k + "_nomfma"] = (S, cfg % 16 + 32)
            if not a.no_check:
                r = ref(x, ws[0], mode)
                for k, p in variants.items():
                    y = run_pf(x, ws[0], mode, p).float()
                    err = ((y - r).abs().max() / r.abs().max()).item()
                    print(json.dumps({"check": name, "M": M, "variant": k, "rel_err": round(err, 5)}), flush=True)
                    if not err < 2e-2:
                        raise SystemExit(f"numerics: {name} M={M} {k} rel err {err}")
            fns = {}
            if mode == L.MODE_SILU:
                fns["hipblaslt"] = lambda i: ops.silu_and_mul(F.linear(x, ws[i % copies]), interleave16=True)
                fns["hipblaslt_gemm"] = lambda i: F.linear(x, ws[i % copies])
            elif mode == L.MODE_PARTIAL and K >= 3 * N and M <= L.SPLITK_PREFILL_MAX_M:
                fns["hipblaslt_splitk4"] = lambda i: L.splitk_linear(x, ws[i % copies], 4)
                fns["hipblaslt"] = lambda i: F.linear(x, ws[i % copies])
            else:
                fns["hipblaslt"] = lambda i: F.linear(x, ws[i % copies])
            for k, p in list(variants.items()) + list(probes.items()):
                fns[k] = (lambda p: (lambda i: L.pf_linear(x, ws[i % copies], mode, plan=p)))(p)
            if a.krot:
                def with_krot(p):
                    def f(i):
                        kernels().set_pf_krot(1)
                        L.pf_linear(x, ws[i % copies], mode, plan=p)
                        kernels().set_pf_krot(0)
                    return f
                for k, p in variants.items():
                    fns[k + "_krot"] = with_krot(p)
            res = time_rounds(fns, a.rounds, a.iters)
            fl = 2.0 * M * N * K
            for k, v in res.items():
                med = statistics.median(v)
                print(json.dumps({"shape": name, "N": N, "K": K, "M": M, "variant": k, "us_med": round(med, 2),
                                  "us_min": round(min(v), 2), "tflops": round(fl / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
