#!/bin/bash
# Setup kernel choice at small group counts (measurement only): product library (multi-group
# setup for m <= 6 at any G) against the measurement build with the one-wave setup.
set -u
for round in 1 2; do
  for shape in "28 4 65536 817 4" "28 4 256 2048 4" "28 4 256 1 4" "250 6 1400 2000 6" "250 6 1400 1 6" "20 6 1400 64 6"; do
    set -- $shape
    for v in main wave; do
      if [ $v = main ]; then L=$PWD/shorthair_amd/libcauchy256.so; W=0; else L=$PWD/shorthair_amd/libcauchy256_meas.so; W=1; fi
      printf "%-5s (%s,%s,%s) G=%s e=%s  " $v $1 $2 $3 $4 $5
      SH_LIB_PATH=$L SH_SETUP_WAVE=$W timeout -k 10 120 python tools/run_ops.py --op decode --iters 20 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
