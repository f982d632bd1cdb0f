#!/usr/bin/env python3
"""Probe: spatial partitioning of one MI355X between the decode step (weight-streaming,
HBM-bound) and a prompt's prefill (MFMA-bound) with CU-masked HIP streams
(hipExtStreamCreateWithCUMask). Round 4 found two ordinary streams all but serialise
(profiles/r4_overlap_probe.md: the gemm_m64g workgroups fill every CU); with disjoint
CU sets both can run at once.

  A = the 4 projections of `--layers` Llama-3-8B decode layers at 64 rows (gemm_m64g),
      replayed `--reps` times (HIP graph);
  B = the same projections at `--prompt` rows (hipBLASLt, the prefill GEMMs; graph).
For each split (n CUs for A, the rest for B) and mask layout ("block": CU ids 0..n-1;
"stride": CU ids whose id % 8 is below n / 32) prints A alone on its mask, B alone on
its mask, both at once, and the full-chip serial time of A + B."""
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


def mask_words(ids, ncu):
    w = [0] * ((ncu + 31) // 32)
    for i in ids:
        w[i // 32] |= 1 << (i % 32)
    return w


def layout(kind, n, ncu):
    if kind == "block":
        a = list(range(n))
    else:  # stride: whole residues mod 8
        per = n * 8 // ncu
        a = [i for i in range(ncu) if i % 8 < per]
    b = [i for i in range(ncu) if i not in set(a)]
    return a, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--splits", type=int, nargs="+", default=[128, 160, 192])
    ap.add_argument("--layouts", nargs="+", default=["block", "stride"])
    ap.add_argument("--fit", action="store_true",
                    help="also time A with grids sized to its CU share (split-K so tiles x S <= A's CUs)")
    a = ap.parse_args()
    k = kernels()
    dev = "cuda"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    H, Fi, Nqkv = 4096, 14336, 6144
    r = lambda *s: (torch.randn(*s, device=dev) * 0.02).bfloat16()  # noqa: E731
    layers = [dict(qkv=r(Nqkv, H), o=r(H, H), gu=r(2 * Fi, H), down=r(H, Fi)) for _ in range(a.layers)]
    x64, act64 = r(64, H), r(64, Fi)
    xP, actP = r(a.prompt, H), r(a.prompt, Fi)

    def decode_pass(plans=None):
        def lin(x, w, mode, key):
            if plans is None:
                return L.m64_linear(x, w, mode)
            nw, S, cfg = plans[key]
            return L.m64_linear(x, w, mode, S, nw, cfg=cfg)
        for _ in range(a.reps):
            for l in layers:
                lin(x64, l["qkv"], L.MODE_PARTIAL, "qkv")
                lin(x64, l["o"], L.MODE_PARTIAL, "o")
                lin(x64, l["gu"], L.MODE_SILU, "gu")
                lin(act64, l["down"], L.MODE_PARTIAL, "down")

    def fit_plans(cus):
        """(nw, S, cfg) per projection with tiles x S <= cus: KC-128 4-wave tiles for
        the partial-sum GEMMs, the 256-column 8-wave tile for gate_up (S = 1)."""
        out = {}
        for key, (N, K) in {"qkv": (Nqkv, H), "o": (H, H), "down": (H, Fi)}.items():
            best = None
            for nw, cfg in ((2, 1), (1, 1), (2, 3), (1, 3)):
                wv, kc, _ = L.M64G_CFGS[cfg]
                tiles = N // (16 * nw * wv)
                S = max(1, min(cus // tiles, K // kc, 16))
                if tiles * S <= cus and (best is None or tiles * S > best[0]):
                    best = (tiles * S, (nw, S, cfg))
            out[key] = best[1]
        out["gu"] = (2, 1, 7) if (2 * Fi) // 256 <= cus else (2, 1, 1)
        return out

    def prefill_pass():
        for l in layers:
            F.linear(xP, l["qkv"])
            F.linear(xP, l["o"])
            F.linear(xP, l["gu"])
            F.linear(actP, l["down"])

    def capture(fn):
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                fn()
        torch.cuda.synchronize()
        return g

    gA, gB = capture(decode_pass), capture(prefill_pass)
    fitted = {}

    def timed(fn):
        ts = []
        for _ in range(a.iters):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[len(ts) // 2]

    full = torch.cuda.Stream()
    with torch.cuda.stream(full):
        tA_full = timed(gA.replay)
        tB_full = timed(gB.replay)
    print(json.dumps({"cus": ncu, "A_full_ms": round(tA_full, 3), "B_full_ms": round(tB_full, 3),
                      "serial_full_ms": round(tA_full + tB_full, 3)}), flush=True)
    for kind in a.layouts:
        for n in a.splits:
            ida, idb = layout(kind, n, ncu)
            pa = k.cu_mask_stream_create(mask_words(ida, ncu))
            pb = k.cu_mask_stream_create(mask_words(idb, ncu))
            sa, sb = torch.cuda.ExternalStream(pa), torch.cuda.ExternalStream(pb)
            with torch.cuda.stream(sa):
                tA = timed(gA.replay)
            with torch.cuda.stream(sb):
                tB = timed(gB.replay)
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

            def both():
                evs[0].record(torch.cuda.current_stream())
                sa.wait_event(evs[0])
                sb.wait_event(evs[0])
                with torch.cuda.stream(sb):
                    gB.replay()
                    evs[2].record(sb)
                with torch.cuda.stream(sa):
                    gA.replay()
                    evs[1].record(sa)
            tAB = timed(both)
            a_end, b_end = evs[0].elapsed_time(evs[1]), evs[0].elapsed_time(evs[2])
            if a.fit and kind == "block":
                plans = fit_plans(len(ida))
                gF = capture(lambda: decode_pass(plans))
                with torch.cuda.stream(full):
                    tF_full = timed(gF.replay)
                with torch.cuda.stream(sa):
                    tF = timed(gF.replay)

                def both_f():
                    evs[0].record(torch.cuda.current_stream())
                    sa.wait_event(evs[0])
                    sb.wait_event(evs[0])
                    with torch.cuda.stream(sb):
                        gB.replay()
                        evs[2].record(sb)
                    with torch.cuda.stream(sa):
                        gF.replay()
                        evs[1].record(sa)
                tFB = timed(both_f)
                print(json.dumps({"layout": kind, "A_cus": len(ida), "fit_plans": plans, "A_fit_full_ms": round(tF_full, 3),
                                  "A_fit_ms": round(tF, 3), "both_fit_ms": round(tFB, 3),
                                  "A_end_in_both_ms": round(evs[0].elapsed_time(evs[1]), 3),
                                  "B_end_in_both_ms": round(evs[0].elapsed_time(evs[2]), 3),
                                  "gain_vs_serial_full": round((tA_full + tB_full) / tFB, 3)}), flush=True)
            print(json.dumps({"layout": kind, "A_cus": len(ida), "B_cus": len(idb),
                              "mask_a": [hex(w) for w in k.cu_mask_stream_get(pa, (ncu + 31) // 32)],
                              "A_ms": round(tA, 3), "B_ms": round(tB, 3), "both_ms": round(tAB, 3),
                              "A_end_in_both_ms": round(a_end, 3), "B_end_in_both_ms": round(b_end, 3),
                              "gain_vs_serial_full": round((tA_full + tB_full) / tAB, 3)}), flush=True)
            torch.cuda.synchronize()
            k.stream_destroy(pa)
            k.stream_destroy(pb)


if __name__ == "__main__":
    main()
