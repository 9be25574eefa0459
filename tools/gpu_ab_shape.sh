#!/bin/bash
# Per-op device times of library variants at one shape (measurement only):
#   tools/gpu_ab_shape.sh K M B GROUPS VARIANT [VARIANT ...]     (main = shorthair_amd/libcauchy256.so)
set -u
K=$1 M=$2 B=$3 G=$4; shift 4
E=$(( K < M ? K : M ))
for v in "$@"; do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  printf "%-8s (%d,%d,%d) " "$v" "$K" "$M" "$B"
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --k "$K" --m "$M" --block "$B" \
      --groups "$G" --erasures "$E" 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
