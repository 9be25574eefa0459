#!/usr/bin/env python3
"""Print per-kernel stats (calls, average/min/max us) and resources from a rocprofv3 output dir."""
import csv
import glob
import sys

d = sys.argv[1]
f = glob.glob(f"{d}/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])) if f else []:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} "
          f"min_us={float(r['MinNs'])/1e3:9.1f} max_us={float(r['MaxNs'])/1e3:9.1f}")
t = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)
seen = set()
for r in csv.DictReader(open(t[0])) if t else []:
    n = r["Kernel_Name"][:56]
    if n in seen:
        continue
    seen.add(n)
    print(f"{n:56s} vgpr={r.get('VGPR_Count')} sgpr={r.get('SGPR_Count')} lds={r.get('LDS_Block_Size')} "
          f"wg={r.get('Workgroup_Size')} grid={r.get('Grid_Size')}")
