#!/bin/bash
# A/B of library variants (run_ops.py per-op device time) + one SQ/GRBM counter pass per variant.
# usage: tools/gpu_ab_pmc.sh NAME[,NAME...]   (main = libcauchy256.so)
set -u
mkdir -p gpurun_out/abpmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in $(echo $1 | tr , ' '); do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  echo "== variant $v"
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in $(echo ${2:-} | tr , ' '); do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  rm -rf gpurun_out/abpmc/$v
  SH_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU --kernel-trace -d gpurun_out/abpmc/$v -o run --output-format csv -- python3 tools/run_ops.py --op both --iters 3 > gpurun_out/abpmc/$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/abpmc/$v.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/abpmc/$v 2>/dev/null | grep -A12 "kern_k200_m32\|stageb" | head -60
done
