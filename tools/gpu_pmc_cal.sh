#!/bin/bash
# FETCH_SIZE / TCC calibration on the staging microbenchmark (known input bytes per dispatch).
set -u
mkdir -p gpurun_out/cal
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for ctr in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/cal/c$i -o run --output-format csv -- ./tools/stage_bench > gpurun_out/cal/c$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/cal/c$i.log; }
done
python3 tools/pmc_summary.py gpurun_out/cal > gpurun_out/cal.txt; cat gpurun_out/cal.txt
