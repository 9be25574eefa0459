#!/bin/bash
# A/B the library variants given as arguments (names of shorthair_amd/libcauchy256_NAME.so; "main"
# = libcauchy256.so) on the headline shape: per-op device time from run_ops.py.
set -u
for v in "$@"; do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$v: /" || exit 1
done
