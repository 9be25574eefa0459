#!/bin/bash
# GPU-box check: parity tests, smoke, bench. Every GPU step has its own time limit; the script
# stops at the first crash/timeout (exit codes other than 0/1 from pytest).
set -u
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 || exit $?
exit $rc
