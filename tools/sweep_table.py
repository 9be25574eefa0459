#!/usr/bin/env python3
"""Print the headline ops and the sweep of a bench.py JSON line (measurement aid):
    python tools/sweep_table.py gpurun_out/bench.log"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    print(d["value"], d["unit"], d["ops"])
    for s in d.get("sweep", []):
        print(f"{s['config']:12s} ({s['k']},{s['m']},{s['B']}) {s['path']:6s} G={s['groups']:6d} "
              f"enc {s.get('encode_ms') or 0:7.4f} ms {s.get('encode_frac') or 0:6.4f}  "
              f"dec {s['decode_ms']:7.4f} ms {s['decode_frac']:6.4f}  e={s['mean_e']}  "
              f"product rate enc {s.get('encode_product_rate', 0)} dec {s.get('decode_product_rate', 0)}")
