#!/bin/bash
# Fixed-kernel per-wave stamps (vmcnt wait / barrier share of a wave's life) for library variants
# built with -DSH_EXPERIMENT_STAMPS (tools/build_variant.sh NAME SH_EXTRA_FLAGS=-DSH_EXPERIMENT_STAMPS).
set -u
for v in "$@"; do
  SH_DEBUG_STAMPS=1 SH_LIB_PATH=$PWD/shorthair_amd/libcauchy256_$v.so timeout -k 10 120 \
    python tools/run_ops.py --op both --iters 2 > gpurun_out/stamps_$v.log 2>&1 || exit 1
  echo "$v:"; grep 'stamps' gpurun_out/stamps_$v.log | tail -4
done
