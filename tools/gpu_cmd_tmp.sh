#!/bin/bash
# scratch GPU command: stream-mode A/B for (28,4)
set -u
mkdir -p gpurun_out
{
bash tools/gpu_ab_shape.sh 28 4 256 209263 main st4 st6 st8 || exit 1
bash tools/gpu_ab_shape.sh 28 4 1400 38000 main st4 st6 st8 || exit 1
bash tools/gpu_ab_shape.sh 28 4 65536 800 main st4 st6 st8 || exit 1
SH_LIB_PATH=$PWD/shorthair_amd/libcauchy256_st8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "28" 2>&1 | tail -5 || exit 1
} > gpurun_out/stream_ab.txt 2>&1 || exit 1
bash tools/gpu_run.sh tests smoke > gpurun_out/final_tests.txt 2>&1
