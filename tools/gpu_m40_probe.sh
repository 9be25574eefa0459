#!/bin/bash
# (216,40) compile-time kernel serving k = 130..216 (measurement): digest check against the
# product library's tile path, then per-op times at (150,40) and (200,40), same box.
set -u
for v in main m40; do
  L=$PWD/shorthair_amd/libcauchy256.so; [ $v = m40 ] && L=$PWD/shorthair_amd/libcauchy256_m40.so
  printf "%-4s " $v
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 1 --digest --k 150 --m 40 --block 1400 --groups 2000 --erasures 40 2>&1 | grep digest
  [ "${PIPESTATUS[0]}" = 0 ] || exit 1
done
for round in 1 2; do
  for shape in "150 40 1400 7142 40" "200 40 1400 6000 40" "135 40 1400 7000 40"; do
    set -- $shape
    for v in main m40; do
      L=$PWD/shorthair_amd/libcauchy256.so; [ $v = m40 ] && L=$PWD/shorthair_amd/libcauchy256_m40.so
      printf "%-4s (%s,%s,%s) G=%s  " $v $1 $2 $3 $4
      SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
