#!/bin/bash
# Same-box A/B of library variants at one shape and several batch sizes (measurement only):
#   tools/gpu_ab_shape.sh "NAME[,NAME...]" K M B E G[,G...]
set -u
VARS=$1 K=$2 M=$3 B=$4 E=$5 GS=$6
lib() { if [ "$1" = main ]; then echo "$PWD/shorthair_amd/libcauchy256.so"; else echo "$PWD/shorthair_amd/libcauchy256_$1.so"; fi; }
for round in 1 2; do
  for G in $(echo "$GS" | tr , ' '); do
    for v in $(echo "$VARS" | tr , ' '); do
      printf "%-8s G=%-6s " "$v" "$G"
      SH_LIB_PATH=$(lib "$v") timeout -k 10 120 python tools/run_ops.py --op both --iters 20 --k $K --m $M --block $B --groups $G --erasures $E 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
for v in $(echo "$VARS" | tr , ' '); do
  printf "%-8s " "$v"
  SH_LIB_PATH=$(lib "$v") timeout -k 10 120 python tools/run_ops.py --op both --iters 1 --digest --k $K --m $M --block $B --groups 4096 --erasures $E 2>&1 | grep digest
  [ "${PIPESTATUS[0]}" = 0 ] || exit 1
done
