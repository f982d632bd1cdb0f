#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel time in the steady-state
window (the last --window-ms of the trace), GPU busy share, and the host gaps.

  python bench/prof_summary.py gpurun_out/prof1/run_kernel_trace.csv --window-ms 600 > profiles/x.md
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=600.0)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--by-grid", action="store_true", help="one row per (kernel, grid size)")
    ap.add_argument("--gap-us", type=float, default=0.0,
                    help="also list idle gaps longer than this, grouped by the kernels around them")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = int(rows[-1]["End_Timestamp"])
    win = [r for r in rows if int(r["Start_Timestamp"]) > last - a.window_ms * 1e6]
    t0 = int(win[0]["Start_Timestamp"])
    span = (last - t0) / 1e6
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win) / 1e6
    agg = collections.defaultdict(lambda: [0, 0])
    durs = collections.defaultdict(list)
    for r in win:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        key = r["Kernel_Name"]
        if a.by_grid:
            key = key.split("(")[0] + f" [grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}]"
        agg[key][0] += d
        agg[key][1] += 1
        durs[key].append(d)
    gaps = []
    prev = None
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None and s - prev > 200e3:
            gaps.append((s - prev) / 1e3)
        prev = e if prev is None else max(prev, e)
    print(f"# Kernel profile (steady-state window: last {a.window_ms:.0f} ms of the trace)\n")
    print(f"- window span: {span:.1f} ms, GPU busy: {busy:.1f} ms ({100 * busy / span:.1f}%)")
    if gaps:
        print(f"- host gaps > 200 us: {len(gaps)}, mean {sum(gaps) / len(gaps):.0f} us, total {sum(gaps) / 1e3:.1f} ms")
    # median / max per call separate the steady decode launches from the (rarer,
    # larger) mixed prefill launches of the same kernel
    print("\n| kernel | calls | total ms | avg us | median us | max us | share |\n|---|---:|---:|---:|---:|---:|---:|")
    for n, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:a.top]:
        short = (n if a.by_grid else n.split("(")[0])[:110].replace("|", "/")
        v = sorted(durs[n])
        med, mx = v[len(v) // 2] / 1e3, v[-1] / 1e3
        print(f"| `{short}` | {c} | {d / 1e6:.2f} | {d / c / 1e3:.1f} | {med:.1f} | {mx:.1f} | {100 * d / 1e6 / busy:.1f}% |")
    if a.gap_us > 0:
        ctx = collections.defaultdict(list)
        prev_e, prev_n, small = None, None, 0.0
        for r in win:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")[:40]
            if prev_e is not None and s > prev_e:
                g = (s - prev_e) / 1e3
                if g > a.gap_us:
                    ctx[(prev_n, n)].append(g)
                else:
                    small += g
            if prev_e is None or e >= prev_e:
                prev_e, prev_n = e, n
        tot = sum(sum(v) for v in ctx.values())
        print(f"\n## Idle gaps > {a.gap_us:.0f} us: {sum(len(v) for v in ctx.values())}, {tot / 1e3:.2f} ms"
              f" (shorter gaps: {small / 1e3:.2f} ms)\n")
        print("| before | after | gaps | total ms | mean us | max us |\n|---|---|---:|---:|---:|---:|")
        for (pn, nn), v in sorted(ctx.items(), key=lambda x: -sum(x[1]))[:a.top]:
            print(f"| `{pn}` | `{nn}` | {len(v)} | {sum(v) / 1e3:.2f} | {sum(v) / len(v):.0f} | {max(v):.0f} |")


if __name__ == "__main__":
    main()
