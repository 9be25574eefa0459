#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/snippet_probe > gpurun_out/snip.log 2>&1; echo "snippet_probe rc=$?"; cat gpurun_out/snip.log
timeout -k 10 200 ./tools/microbench > gpurun_out/microbench.log 2>&1; echo "microbench rc=$?"; grep -i "lds\|unal" gpurun_out/microbench.log
bash tools/gpu_full.sh
