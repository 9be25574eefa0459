#!/bin/bash
# GPU-box driver for iteration runs: tools/gpu_run.sh STEP [STEP ...]
# Steps: tests (pytest -m gpu), smoke, bench (short, no CPU leg), prof (rocprofv3 kernel stats of
# a short bench), ab:NAME[,NAME...] (per-op device time of library variants via run_ops.py).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -8 "gpurun_out/$name.log"
  return $rc
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $? ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) step bench 300 python bench.py --steps 20 --warmup 3 --no-cpu --host-calls 0 || exit $? ;;
    prof)
      rm -rf gpurun_out/prof
      step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --host-calls 0 || exit $?
      python3 tools/kstats.py gpurun_out/prof ;;
    ab:*)
      for v in $(echo ${s#ab:} | tr , ' '); do
        L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
        echo "== variant $v"
        SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
      done ;;
    env:*) bash tools/gpu_envab.sh "$(echo ${s#env:} | tr + " ")" || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
