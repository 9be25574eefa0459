#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) of the codec kernels for library variants.
# usage: tools/gpu_traffic_ab.sh NAME[,NAME...]
set -u
mkdir -p gpurun_out/tab
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in $(echo $1 | tr , ' '); do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/tab/${v}_$ctr
    SH_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/tab/${v}_$ctr -o run --output-format csv -- python3 tools/run_ops.py --op both --iters 3 > gpurun_out/tab/${v}_$ctr.log 2>&1 || { echo "pmc $v $ctr failed"; tail -3 gpurun_out/tab/${v}_$ctr.log; exit 1; }
  done
  echo "== $v"
  python3 - "$v" <<'PY'
import sys, glob, csv, collections
v = sys.argv[1]
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(f"gpurun_out/tab/{v}_{ctr}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            acc[r["Kernel_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        if "k200_m32" in k or "stageb" in k:
            xs = list(d.values())
            print(f"  {ctr:10s} {k[:48]:48s} mean KB={sum(xs)/len(xs):.4g}")
PY
done
