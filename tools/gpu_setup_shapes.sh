#!/bin/bash
# Decode setup share at the m >= 7 sweep shapes (measurement only): per-op times of the
# product library, setup / stage A / stage B split.
set -u
for shape in "50 10 1000 30000 10" "112 16 256 52315 16" "224 32 256 26157 32" "64 16 1400 16741 16" "64 16 1400 4096 16" "112 16 1400 9566 16" "200 56 1352 5547 56" "150 40 1400 7142 40"; do
  set -- $shape
  printf "(%s,%s,%s) G=%s e=%s  " $1 $2 $3 $4 $5
  timeout -k 10 120 python tools/run_ops.py --op decode --iters 10 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
  [ "${PIPESTATUS[0]}" = 0 ] || exit 1
done
