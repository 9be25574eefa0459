#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S=$PWD/shorthair_amd/libcauchy256_split.so
M=$PWD/shorthair_amd/libcauchy256_base.so
for r in 1 2; do
  printf "main        "; SH_LIB_PATH=$M timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  for n in 0 128 256 512; do
    printf "split %-5s " $n; SH_SPLIT=$n SH_LIB_PATH=$S timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
for n in 0 256 512; do
  printf "split %-5s " $n; SH_SPLIT=$n SH_LIB_PATH=$S timeout -k 10 120 python tools/run_ops.py --op both --iters 2 --digest 2>&1 | grep digest || exit 1
done
printf "main        "; SH_LIB_PATH=$M timeout -k 10 120 python tools/run_ops.py --op both --iters 2 --digest 2>&1 | grep digest || exit 1
for G in 1000 4096 2048; do
  printf "G=%-5s main " $G; SH_LIB_PATH=$M timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --groups $G 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  printf "G=%-5s split " $G; SH_LIB_PATH=$S timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --groups $G --digest 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
done
