#!/bin/bash
# Microbenchmarks + parity tests + rocprof kernel trace of a short bench run.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 ./tools/microbench > gpurun_out/microbench.log 2>&1; rc=$?; echo "microbench rc=$rc"; cat gpurun_out/microbench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1; r2=$?; echo "rocprof rc=$r2"; tail -2 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
