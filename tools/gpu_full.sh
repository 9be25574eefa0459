#!/bin/bash
# Parity tests + smoke + PMC traffic passes + bench (with CPU baseline) + rocprof kernel trace of the same bench command.
# Stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
step traffic 400 bash tools/gpu_traffic.sh || exit $?
mkdir -p profiles/box && cp gpurun_out/traffic/traffic.json profiles/box/traffic.json
step bench 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 || exit $?
rm -rf gpurun_out/prof
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
PY
