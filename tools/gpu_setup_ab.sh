#!/bin/bash
# Multi-group decode setup A/B (measurement only): the GPU tests (all, or the setup-related
# subset with "quick"), then decode times per shape with the product library against the
# measurement build forced onto the one-wave-per-group setup (SH_SETUP_WAVE=1).
#   tools/gpu_setup_ab.sh [all|quick|notests]
set -u
mkdir -p gpurun_out
case "${1:-all}" in
  all)   K="";;
  quick) K="searched_table or malformed or single_group_decode_random or decode_batch_roundtrip or no_erasures";;
esac
if [ "${1:-all}" != notests ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests ${K:+-k "$K"} \
    > gpurun_out/setup_tests.txt 2>&1 || { tail -30 gpurun_out/setup_tests.txt; exit 1; }
  tail -2 gpurun_out/setup_tests.txt
fi
for round in 1 2; do
  for shape in "28 4 256 209263 4" "40 6 256 65536 6" "112 16 256 52315 16" "224 32 256 26157 32" \
               "64 16 1400 16741 16" "64 16 1400 4096 16" "50 10 1000 30000 10" "200 32 1400 8192 32"; do
    set -- $shape
    for v in main wave; do
      if [ $v = main ]; then L=$PWD/shorthair_amd/libcauchy256.so; W=0; else L=$PWD/shorthair_amd/libcauchy256_meas.so; W=1; fi
      printf "%-5s (%s,%s,%s) G=%s e=%s  " $v $1 $2 $3 $4 $5
      SH_LIB_PATH=$L SH_SETUP_WAVE=$W timeout -k 10 120 python tools/run_ops.py --op decode --iters 10 --k $1 --m $2 --block $3 --groups $4 --erasures $5 2>&1 | grep -v amdgpu.ids | tail -1
      [ "${PIPESTATUS[0]}" = 0 ] || exit 1
    done
  done
done
