#!/bin/bash
# GPU-box check of the current tree: GPU tests, smoke, a short bench line, the step-event probe and
# a rocprofv3 kernel-stats pass of the bench (measurement workflow, round 6).
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-6}
  return $rc
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $? ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) TAILN=1 step bench 400 python bench.py --steps 20 --warmup 3 --no-cpu --host-calls 0 --no-sweep || exit $? ;;
    events) step step_events 300 python tools/step_events.py --steps 20 --rounds 3 || exit $? ;;
    prof)
      rm -rf gpurun_out/prof
      step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --host-calls 0 --no-sweep || exit $?
      python3 tools/kstats.py gpurun_out/prof | head -8 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
