#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: mean per dispatch, per kernel, per counter."""
import collections
import csv
import glob
import sys


def load(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("Name")
            cn = r.get("Counter_Name") or r.get("Counter-Name")
            v = float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
            acc[name][cn].append((r.get("Dispatch_Id") or r.get("Dispatch-Id"), v))
    return acc


def main(root):
    acc = load(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True))
    for name, ctrs in sorted(acc.items()):
        if not any(s in name for s in ("sh::", "k_")):
            continue
        print(name[:90])
        for cn, vals in sorted(ctrs.items()):
            per = collections.defaultdict(float)
            for d, v in vals:
                per[d] += v
            xs = list(per.values())
            print(f"    {cn:28s} n={len(xs):3d} mean={sum(xs)/len(xs):.4g}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
