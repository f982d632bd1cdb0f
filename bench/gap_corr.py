#!/usr/bin/env python3
"""Who is late at a GPU idle gap: the host or the GPU? From a rocprofv3
``--kernel-trace --hip-trace --output-format csv`` directory, for every idle gap
longer than --min-us (last --window-ms) the kernel that ends the gap is matched to
the HIP call that enqueued it (Correlation_Id), and the gap is split into
  late_host = gap start -> that call started   (the host had not asked yet)
  in_flight = the call started -> the kernel started (runtime + queue latency)
grouped by the kernels on both sides of the gap.

  python bench/gap_corr.py <dir> --window-ms 600 --min-us 8
"""
import argparse
import bisect
import collections
import csv
import glob
import os


def _load(d, suffix):
    fs = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not fs:
        raise SystemExit(f"no *{suffix} under {d}")
    return list(csv.DictReader(open(fs[0])))


def _short(n):
    return n.split("(")[0].split("<")[0].replace("void ", "")[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window-ms", type=float, default=600.0)
    ap.add_argument("--min-us", type=float, default=8.0)
    ap.add_argument("--dump", type=int, default=0,
                    help="print the HIP call timeline around the first N gaps of the largest group")
    a = ap.parse_args()
    ks = _load(a.dir, "kernel_trace.csv")
    hs = _load(a.dir, "hip_api_trace.csv")
    try:
        mc = _load(a.dir, "memory_copy_trace.csv")
    except SystemExit:
        mc = []
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(ks[-1]["End_Timestamp"])
    ks = [r for r in ks if int(r["Start_Timestamp"]) > last - a.window_ms * 1e6]
    api = {r["Correlation_Id"]: r for r in hs}
    hs.sort(key=lambda r: int(r["Start_Timestamp"]))
    h_start = [int(r["Start_Timestamp"]) for r in hs]
    groups = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, collections.Counter()])
    where = collections.defaultdict(list)  # group -> [(gap start, gap end, enqueue start)]
    prev_e, prev_n = None, None
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = _short(r["Kernel_Name"])
        if prev_e is not None and s - prev_e > a.min_us * 1e3:
            c = api.get(r["Correlation_Id"])
            g = groups[(prev_n, n, c["Function"] if c else "?")]
            g[0] += 1
            g[1] += (s - prev_e) / 1e3
            if c is not None:
                cs = int(c["Start_Timestamp"])
                g[2] += max(0, cs - prev_e) / 1e3
                where[(prev_n, n, c["Function"])].append((prev_e, s, cs))
                g[3] += (s - max(cs, prev_e)) / 1e3
                # host calls made between the gap start and the enqueue
                for hr in hs[bisect.bisect_left(h_start, prev_e):bisect.bisect_left(h_start, cs)]:
                    g[4][hr["Function"]] += 1
        if prev_e is None or e >= prev_e:
            prev_e, prev_n = e, n
    tot = sum(g[1] for g in groups.values())
    print(f"# Idle gaps > {a.min_us:.0f} us, last {a.window_ms:.0f} ms: {sum(g[0] for g in groups.values())}, "
          f"{tot / 1e3:.2f} ms\n")
    print("| before | after | enqueued by | gaps | mean us | late host us | in flight us | host calls in the gap |")
    print("|---|---|---|---:|---:|---:|---:|---|")
    for (pn, nn, fn), g in sorted(groups.items(), key=lambda x: -x[1][1])[:25]:
        k = g[0]
        top = ", ".join(f"{f} {c / k:.1f}" for f, c in g[4].most_common(4))
        print(f"| `{pn}` | `{nn}` | {fn} | {k} | {g[1] / k:.0f} | {g[2] / k:.0f} | {g[3] / k:.0f} | {top} |")
    if a.dump and groups:
        key = max(groups, key=lambda x: groups[x][1])
        kst = [int(r["Start_Timestamp"]) for r in ks]
        for g0, g1, cs in where[key][:a.dump]:
            print(f"\n### gap {(g1 - g0) / 1e3:.0f} us ({key[0]} -> {key[1]}), times relative to the gap start\n")
            print("| t us | dur us | thread | call / kernel |\n|---:|---:|---|---|")
            ev = []
            for hr in hs[bisect.bisect_left(h_start, g0 - 400e3):bisect.bisect_left(h_start, max(cs, g1) + 5e3)]:
                ev.append((int(hr["Start_Timestamp"]), int(hr["End_Timestamp"]), hr.get("Thread_Id", "?"),
                           hr["Function"]))
            for r in ks[bisect.bisect_left(kst, g0 - 30e3):bisect.bisect_left(kst, g1 + 5e3) + 1]:
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU", _short(r["Kernel_Name"])))
            for r in mc:
                t0 = int(r["Start_Timestamp"])
                if g0 - 400e3 <= t0 <= g1 + 5e3:
                    ev.append((t0, int(r["End_Timestamp"]), "COPY", r.get("Direction", "?") + " " + r.get("Size", "")))
            for t0, t1, th, fn in sorted(ev):
                print(f"| {(t0 - g0) / 1e3:.1f} | {(t1 - t0) / 1e3:.1f} | {th} | {fn} |")


if __name__ == "__main__":
    main()
