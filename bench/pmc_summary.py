#!/usr/bin/env python3
"""Per-kernel sums of the counters of rocprofv3 --pmc pass directories (one
counter_collection.csv each): python bench/pmc_summary.py gpurun_out/pmc/p1 gpurun_out/pmc/p2"""
import collections
import csv
import glob
import os
import sys


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
                tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((d, r.get("Dispatch_Id", "")))
    for k, cs in tot.items():
        print(f"\n## `{k}` ({len(disp[k])} dispatch-passes)\n\n| counter | sum |\n|---|---:|")
        for c, v in sorted(cs.items()):
            print(f"| {c} | {v:,.0f} |")


if __name__ == "__main__":
    main()
