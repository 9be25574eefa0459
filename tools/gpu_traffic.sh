#!/bin/bash
# HBM traffic per launch of the codec kernels at the bench workload, from rocprofv3 PMC
# (FETCH_SIZE and WRITE_SIZE in separate passes, --kernel-trace only beside --pmc), corrected as
# MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE x2 on gfx950 for 16-B/lane streaming reads;
# WRITE_SIZE as is for 16-B/lane stores. Output: gpurun_out/traffic/traffic.json (copy it to
# profiles/ for bench.py's roofline.traffic).
set -u
OUT=gpurun_out/traffic
mkdir -p $OUT
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/run_ops.py --op both --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $ctr failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $ctr ok"
done
python3 tools/traffic_json.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
