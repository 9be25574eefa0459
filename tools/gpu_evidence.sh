#!/bin/bash
# One build's evidence set on the GPU box: tools/gpu_evidence.sh TAG [tests]
#   1. tools/gpu_profile.sh TAG (PMC traffic + SQ/GRBM + ifetch passes, kernel stats of the
#      headline bench) -> gpurun_out/prof_TAG/, traffic JSON -> profiles/r06/traffic_TAG.json
#   2. the default `python bench.py` line (it quotes the hash-matched traffic JSON)
#   3. optionally the GPU test suite
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=${1:?tag}
mkdir -p gpurun_out
IFETCH="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES" PROFDIR=profiles/r06 \
  bash tools/gpu_profile.sh "$TAG" > "gpurun_out/prof_$TAG.out" 2>&1 || { tail -5 "gpurun_out/prof_$TAG.out"; exit 1; }
tail -3 "gpurun_out/prof_$TAG.out"
timeout -k 10 600 python bench.py > "gpurun_out/bench_full_$TAG.json" 2> "gpurun_out/bench_full_$TAG.err" || { tail -5 "gpurun_out/bench_full_$TAG.err"; exit 1; }
python tools/sweep_table.py "gpurun_out/bench_full_$TAG.json"
if [ "${2:-}" = tests ]; then bash tools/gpu_run.sh tests || exit $?; fi
