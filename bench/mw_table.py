#!/usr/bin/env python3
"""Summarise a `gemm_bench.py --mw-sweep` log: per (shape, M) the fastest checked
gemm_mw configuration against hipBLASLt (and gemm_m64g where it ran), as a
markdown table, plus the `_MW_TUNED` entries (xgserve/ops/linear.py) it implies.

  python bench/mw_table.py gpurun_out/mw/mw_sweep.log [--max-err 1e-4]
"""
from __future__ import annotations

import argparse
import json
import re
import sys
from collections import defaultdict

SHAPES = {"qkv": (6144, 4096, 1), "o": (4096, 4096, 1), "gate_up": (28672, 4096, 2), "down": (4096, 14336, 1),
          "lm_head": (128256, 4096, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--max-err", type=float, default=1e-4)
    a = ap.parse_args()
    rows = defaultdict(list)
    for line in open(a.log):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        rows[(r["shape"], r["M"])].append(r)
    print("| shape | M | hipBLASLt us | best gemm_mw | us | TB/s | TF/s | vs hipBLASLt | m64g us |")
    print("|---|---:|---:|---|---:|---:|---:|---:|---:|")
    tuned = defaultdict(dict)
    for (shape, M), rs in sorted(rows.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        lib = next((r for r in rs if r["op"] == "hipblaslt"), None)
        m64 = next((r for r in rs if r["op"].startswith("m64g")), None)
        mws = [r for r in rs if r["op"].startswith("mw(") and (r["rel_err"] is None or r["rel_err"] <= a.max_err
                                                          or shape == "gate_up" or shape == "lm_head")]
        if not mws:
            continue
        best = min(mws, key=lambda r: r["us"])
        S, cfg = (int(v) for v in re.findall(r"=(\d+)", best["op"]))
        print(f"| {shape} | {M} | {lib['us'] if lib else '-'} | S={S} cfg={cfg} | {best['us']} | {best['TB/s']} | "
              f"{best['TF/s']} | {lib['us'] / best['us']:.2f}x | {m64['us'] if m64 else '-'} |" if lib else
              f"| {shape} | {M} | - | S={S} cfg={cfg} | {best['us']} | {best['TB/s']} | {best['TF/s']} | - | - |")
        if shape in SHAPES and (M > 64 or shape == "lm_head"):
            n, k, mode = SHAPES[shape]
            bucket = 128 if M <= 128 else 192 if M <= 192 else 256 if M <= 256 else 320
            if shape == "lm_head" and lib and best["us"] >= lib["us"]:
                continue  # the LM head keeps hipBLASLt unless gemm_mw wins
            tuned[(n, k, mode)].setdefault(bucket, (S, cfg))  # ascending M: a bucket's smallest M decides
    print()
    print("_MW_TUNED = {")
    for key, v in tuned.items():
        print(f"    {key}: {dict(sorted(v.items()))},")
    print("}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
