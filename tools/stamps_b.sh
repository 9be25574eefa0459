#!/bin/bash
# Stage-B phase stamps for library variants built with -DSH_EXPERIMENT_STAMPS (tools/build_variant.sh).
set -u
for v in "$@"; do
  SH_DEBUG_STAMPS=1 SH_LIB_PATH=$PWD/shorthair_amd/libcauchy256_$v.so timeout -k 10 120 \
    python tools/run_ops.py --op decode --iters 2 > gpurun_out/stamps_$v.log 2>&1 || exit 1
  echo "$v: $(grep 'stamps stageB' gpurun_out/stamps_$v.log | tail -1)"
done
