#!/usr/bin/env python3
"""Probe: do decode-step weight streams (gemm_m64g at 64 rows, memory-bound, MFMA
mostly idle) and prompt-sized GEMMs (library GEMMs at 512+ rows, MFMA-bound) overlap
when they run on two streams of one MI355X at the same time?

Each side is captured as a HIP graph on its own stream:
  A = the 4 projections of `--layers` Llama-3-8B decode layers at 64 rows (gemm_m64g),
      replayed `--reps` times (cold weights: the layers together exceed the 256 MB
      Infinity Cache);
  B = the same projections at `--prompt` rows on hipBLASLt (the mixed step's GEMMs).
Prints one JSON line with A alone, B alone, A and B concurrently (wall of both, and
the time at which A's replays ended), and the overlap gain = (A + B) / both.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xgserve.ops import linear as L  # noqa: E402
from xgserve.ops._native import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--prompt", type=int, nargs="+", default=[512])
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--prio", action="store_true", help="stream A at high priority")
    a = ap.parse_args()
    kernels()
    dev = "cuda"
    H, Fi, Nqkv = 4096, 14336, 6144
    r = lambda *s: (torch.randn(*s, device=dev) * 0.02).bfloat16()  # noqa: E731
    layers = [dict(qkv=r(Nqkv, H), o=r(H, H), gu=r(2 * Fi, H), down=r(H, Fi)) for _ in range(a.layers)]
    x64, act64 = r(64, H), r(64, Fi)

    sA = torch.cuda.Stream(priority=-1 if a.prio else 0)
    sB = torch.cuda.Stream()

    def decode_pass():
        for l in layers:
            L.m64_linear(x64, l["qkv"], L.MODE_PARTIAL)
            L.m64_linear(x64, l["o"], L.MODE_PARTIAL)
            L.m64_linear(x64, l["gu"], L.MODE_SILU)
            L.m64_linear(act64, l["down"], L.MODE_PARTIAL)

    def capture(fn, stream):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(stream):
            fn()  # warm (workspaces, plans)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=stream):
                fn()
        torch.cuda.synchronize()
        return g

    gA = capture(decode_pass, sA)

    def timed(launch):
        ts = []
        for _ in range(a.iters):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            endA = launch()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[len(ts) // 2], endA

    def run_A():
        for _ in range(a.reps):
            gA.replay()

    for P in a.prompt:
        xP, actP = r(P, H), r(P, Fi)

        def prefill_pass():
            for l in layers:
                F.linear(xP, l["qkv"])
                F.linear(xP, l["o"])
                F.linear(xP, l["gu"])
                F.linear(actP, l["down"])

        gB = capture(prefill_pass, sB)
        with torch.cuda.stream(sA):
            tA, _ = timed(lambda: (run_A(), None)[1])
        with torch.cuda.stream(sB):
            tB, _ = timed(lambda: (gB.replay(), None)[1])
        evA = torch.cuda.Event(enable_timing=True)
        ev0 = torch.cuda.Event(enable_timing=True)

        def both():
            ev0.record(torch.cuda.current_stream())
            sA.wait_event(ev0)
            sB.wait_event(ev0)
            with torch.cuda.stream(sB):
                gB.replay()
            with torch.cuda.stream(sA):
                run_A()
                evA.record(sA)
            return None
        tAB, _ = timed(both)
        a_end = ev0.elapsed_time(evA)
        print(json.dumps({"layers": a.layers, "decode_reps": a.reps, "prompt_rows": P, "A_alone_ms": round(tA, 3),
                          "B_alone_ms": round(tB, 3), "both_ms": round(tAB, 3), "A_end_in_both_ms": round(a_end, 3),
                          "overlap_gain": round((tA + tB) / tAB, 3), "prio": a.prio}), flush=True)


if __name__ == "__main__":
    main()
