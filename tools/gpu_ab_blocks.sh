#!/bin/bash
# Per-op device time of library variants at several block sizes (alignment / shape probes):
#   tools/gpu_ab_blocks.sh "main late" "1400 1408"
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in $1; do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  for B in $2; do
    echo "== variant $v B=$B"
    SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --block $B 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
