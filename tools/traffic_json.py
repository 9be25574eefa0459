#!/usr/bin/env python3
"""rocprofv3 FETCH_SIZE / WRITE_SIZE passes -> per-kernel HBM bytes per launch (JSON), plus the
SQ / GRBM pass when present (VALU instructions, wave and wait cycles, busy clock cycles).

FETCH_SIZE and WRITE_SIZE are in KiB. gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE
counts 64 B per 128-B request of a wide streaming read, so it is doubled; WRITE_SIZE is exact for
16-B/lane stores. The library hash ties the numbers to the build they were measured on; bench.py
quotes them (roofline.traffic and the VALU leg) only for that build."""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main(d):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for p in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name")
            cn = r.get("Counter_Name") or r.get("Counter-Name")
            did = (p, r.get("Dispatch_Id") or r.get("Dispatch-Id"))
            per[name][cn][did] = per[name][cn].get(did, 0.0) + float(r.get("Counter_Value") or r.get("Counter-Value"))
    lib = os.path.join(ROOT, "shorthair_amd", "libcauchy256.so")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ+GRBM (separate passes) over tools/run_ops.py --op both",
           "correction": "read = 2 x FETCH_SIZE (gfx950, 16-B/lane streaming reads); write = WRITE_SIZE",
           "workload": {"k": 200, "m": 32, "block_bytes": 1400, "groups": 8192, "erasures": 32},
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "kernels": {}}
    for name, ctrs in per.items():
        if "sh::" not in name or "fill_pcg" in name:
            continue
        f = list(ctrs.get("FETCH_SIZE", {}).values())
        w = list(ctrs.get("WRITE_SIZE", {}).values())
        if not f or not w:
            continue
        rd = 2 * 1024 * sum(f) / len(f)
        wr = 1024 * sum(w) / len(w)
        key = name.split("(")[0]
        out["kernels"][key] = {"read_bytes": round(rd), "write_bytes": round(wr), "hbm_bytes": round(rd + wr),
                               "launches": [len(f), len(w)]}
        sq = {}
        for cn in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                   "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES", "SQ_WAVES"):
            v = list(ctrs.get(cn, {}).values())
            if v:
                sq[cn] = sum(v) / len(v)
        if sq:
            out["kernels"][key]["sq"] = sq
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traffic")
