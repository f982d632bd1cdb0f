#!/usr/bin/env python3
"""Explain the idle gaps between engine steps from a rocprofv3 trace taken with
``--kernel-trace --hip-trace --output-format csv``.

For every GPU idle gap longer than --min-us (in the last --window-ms), it splits the
gap into
  wake   = GPU went idle -> the host's blocking synchronize call returned
  host   = synchronize returned -> the next HIP call that enqueues GPU work starts
  submit = that call started -> the next kernel actually started on the GPU
and prints the means plus the most frequent HIP calls made on the host during gaps.

  python bench/gap_analysis.py gpurun_out/prof_gap/ --window-ms 300
"""
import argparse
import bisect
import collections
import csv
import glob
import os

SYNC = ("hipStreamSynchronize", "hipDeviceSynchronize", "hipEventSynchronize")
ENQ = ("hipMemcpyAsync", "hipMemcpyWithStream", "hipGraphLaunch", "hipLaunchKernel",
       "hipExtModuleLaunchKernel", "hipModuleLaunchKernel", "hipMemsetAsync", "hipExtLaunchKernel")


def _load(d, suffix):
    fs = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not fs:
        raise SystemExit(f"no *{suffix} under {d}")
    return list(csv.DictReader(open(fs[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window-ms", type=float, default=300.0)
    ap.add_argument("--min-us", type=float, default=50.0)
    a = ap.parse_args()
    ks = _load(a.dir, "kernel_trace.csv")
    hs = _load(a.dir, "hip_api_trace.csv")
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(ks[-1]["End_Timestamp"])
    lo = last - a.window_ms * 1e6
    ks = [r for r in ks if int(r["Start_Timestamp"]) > lo]
    hs = [r for r in hs if int(r["Start_Timestamp"]) > lo - 5e6]
    hs.sort(key=lambda r: int(r["Start_Timestamp"]))
    h_start = [int(r["Start_Timestamp"]) for r in hs]
    syncs = sorted(int(r["End_Timestamp"]) for r in hs if r["Function"] in SYNC)
    enq = sorted(int(r["Start_Timestamp"]) for r in hs if r["Function"] in ENQ)

    gaps = []
    prev = None
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None and s - prev > a.min_us * 1e3:
            gaps.append((prev, s))
        prev = e if prev is None else max(prev, e)
    span = (last - int(ks[0]["Start_Timestamp"])) / 1e6
    print(f"# Step-gap analysis (last {a.window_ms:.0f} ms, gaps > {a.min_us:.0f} us)\n")
    print(f"- window {span:.1f} ms, {len(gaps)} gaps, idle {sum(b - a_ for a_, b in gaps) / 1e6:.2f} ms")
    wake, host, sub, calls = [], [], [], collections.Counter()
    for g0, g1 in gaps:
        i = bisect.bisect_left(syncs, g0)
        if i >= len(syncs) or syncs[i] > g1:
            continue
        ts = syncs[i]
        j = bisect.bisect_left(enq, ts)
        if j >= len(enq) or enq[j] > g1:
            continue
        te = enq[j]
        wake.append(ts - g0)
        host.append(te - ts)
        sub.append(g1 - te)
        k0, k1 = bisect.bisect_left(h_start, ts), bisect.bisect_left(h_start, g1)
        for r in hs[k0:k1]:
            calls[r["Function"]] += 1
    n = max(1, len(wake))
    if wake:
        print(f"- attributed {len(wake)} gaps: mean wake {sum(wake) / n / 1e3:.0f} us, "
              f"host {sum(host) / n / 1e3:.0f} us, submit {sum(sub) / n / 1e3:.0f} us")
    print("\n| HIP call during gaps | per gap |\n|---|---:|")
    for f, c in calls.most_common(15):
        print(f"| {f} | {c / n:.1f} |")


if __name__ == "__main__":
    main()
