#!/bin/bash
# stageb_small2 (two word columns per lane, ds_read_b64 lookups) against stageb_small, same
# measurement library, same box (measurement only): decode tests with small2 forced on, then
# per-op times at the C4 B = 256 shapes.
set -u
mkdir -p gpurun_out
L=$PWD/shorthair_amd/libcauchy256_meas.so
SH_LIB_PATH=$L SH_SMALL2=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "decode or setup or malformed" > gpurun_out/small2_tests.txt 2>&1 || { tail -30 gpurun_out/small2_tests.txt; exit 1; }
tail -1 gpurun_out/small2_tests.txt
for round in 1 2; do
  for shape in "224 32 256 26157 32" "112 16 256 52315 16" "28 4 256 209263 4" "224 32 512 13078 32"; do
    set -- $shape
    for v in 0 1; do
      printf "small2=%s (%s,%s,%s) G=%s  " $v $1 $2 $3 $4
      SH_LIB_PATH=$L SH_SMALL2=$v timeout -k 10 120 python tools/run_ops.py --op decode --iters 20 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
