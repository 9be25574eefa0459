#!/bin/bash
# Round-end rehearsal on one box: packet-group tests, smoke(), then the driver's bench command
# three times back to back (spread of the settled headline). Each GPU step has its own limit.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_groups.py > gpurun_out/final_groups.txt 2>&1 || { tail -30 gpurun_out/final_groups.txt; exit 1; }
tail -1 gpurun_out/final_groups.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1 || { tail -20 gpurun_out/final_smoke.txt; exit 1; }
tail -2 gpurun_out/final_smoke.txt
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_$i.json 2> gpurun_out/final_bench_$i.err || { tail -5 gpurun_out/final_bench_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/final_bench_$i.json').read().strip().splitlines()[-1])
print($i, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic_over_alg'), d['cpu_baseline']['value'], d['ops'].get('decode_setup_ms'))"
done
