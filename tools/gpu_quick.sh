#!/bin/bash
# Quick GPU iteration: parity tests, then a short bench + kernel trace (VGPR/LDS per kernel).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_prof.log 2>&1; r2=$?
echo "bench rc=$r2"; grep '^{' gpurun_out/bench_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ops', d['ops'])"
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
t = glob.glob('gpurun_out/prof/**/run_kernel_trace.csv', recursive=True)[0]
seen = set()
for r in csv.DictReader(open(t)):
    n = r['Kernel_Name'][:50]
    if n in seen or not n.startswith('sh::'): continue
    seen.add(n)
    print(f"{n:50s} vgpr={r.get('VGPR_Count')} agpr={r.get('Accum_VGPR_Count')} sgpr={r.get('SGPR_Count')} lds={r.get('LDS_Block_Size')} wg={r.get('Workgroup_Size')}")
PY
exit $rc
