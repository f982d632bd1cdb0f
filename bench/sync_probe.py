#!/usr/bin/env python3
"""Which host call blocks on the GPU in the serving loop? Runs bench.py (same
arguments) with torch's host synchronisation points wrapped: Event.synchronize,
Stream.synchronize, torch.cuda.synchronize and Tensor.item / tolist / cpu. Every call
that blocks longer than --min-us is recorded with its Python call site; the summary
(calls, total / mean blocked time per site) goes to stderr after the run.

  python bench/sync_probe.py --min-us 30 -- --steps 200 --warmup 20
"""
import argparse
import collections
import os
import sys
import time
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REC = collections.defaultdict(lambda: [0, 0.0, 0.0])  # site -> [calls, total s, max s]


def _site() -> str:
    fs = [f for f in traceback.extract_stack()[:-3] if "sync_probe" not in f.filename]
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fs[-4:][::-1])


def _wrap(owner, name, min_s):
    orig = getattr(owner, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = orig(*a, **k)
        dt = time.perf_counter() - t0
        if dt >= min_s:
            e = REC[f"{owner.__name__}.{name} @ {_site()}"]
            e[0] += 1
            e[1] += dt
            e[2] = max(e[2], dt)
        return r

    setattr(owner, name, w)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-us", type=float, default=30.0)
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest[:1] == ["--"] else a.rest
    min_s = a.min_us * 1e-6
    _wrap(torch.cuda.Event, "synchronize", min_s)
    _wrap(torch.cuda.Stream, "synchronize", min_s)
    orig_sync = torch.cuda.synchronize

    def dev_sync(*aa, **kk):
        t0 = time.perf_counter()
        orig_sync(*aa, **kk)
        dt = time.perf_counter() - t0
        if dt >= min_s:
            e = REC[f"torch.cuda.synchronize @ {_site()}"]
            e[0] += 1
            e[1] += dt
            e[2] = max(e[2], dt)

    torch.cuda.synchronize = dev_sync
    for n in ("item", "tolist", "cpu"):
        _wrap(torch.Tensor, n, min_s)
    sys.argv = ["bench.py"] + rest
    import bench
    rc = bench.main()
    rows = sorted(REC.items(), key=lambda kv: -kv[1][1])
    print(f"\n# host calls blocking >= {a.min_us:.0f} us (whole run, incl. setup)\n", file=sys.stderr)
    print("| site | calls | total ms | mean us | max us |\n|---|---:|---:|---:|---:|", file=sys.stderr)
    for k, (c, tot, mx) in rows[:25]:
        print(f"| `{k}` | {c} | {tot * 1e3:.2f} | {tot / c * 1e6:.0f} | {mx * 1e6:.0f} |", file=sys.stderr)
    return rc


if __name__ == "__main__":
    sys.exit(main())
