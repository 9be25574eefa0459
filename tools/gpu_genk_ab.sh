#!/bin/bash
# Compile-time kernels for k below their K (fixed_kernel_k) against the tile kernels those shapes
# ran on before (measurement only): the GPU tests, then per-op times of the product library and
# of the previous build (libcauchy256_old.so) at shapes k < K of a compiled (K, m), same box.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/genk_tests.txt 2>&1 || { tail -30 gpurun_out/genk_tests.txt; exit 1; }
tail -1 gpurun_out/genk_tests.txt
for round in 1 2; do
  for shape in "150 32 1400 6000 32" "135 32 1400 6000 32" "100 16 1400 6000 16" "70 16 1400 6000 16" "20 4 1400 30000 4" "150 56 1352 6000 56" "125 56 1352 6000 56" "120 66 1336 6000 66"; do
    set -- $shape
    for v in main old; do
      L=$PWD/shorthair_amd/libcauchy256.so; [ $v = old ] && L=$PWD/shorthair_amd/libcauchy256_old.so
      printf "%-4s (%s,%s,%s) G=%s  " $v $1 $2 $3 $4
      SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
