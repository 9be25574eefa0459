#!/bin/bash
# Same-box A/B of library variants: per-op device times (two interleaved rounds), then per
# variant three PMC passes over an encode+decode run (instruction fetch, SQ waits / VALU, HBM
# fetch). Measurement only.
#   tools/gpu_ab_ifetch.sh NAME[,NAME...]      (main = shorthair_amd/libcauchy256.so)
#   PMC=0 tools/gpu_ab_ifetch.sh ...           (times only)
set -u
mkdir -p gpurun_out/abif
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
lib() { if [ "$1" = main ]; then echo "$PWD/shorthair_amd/libcauchy256.so"; else echo "$PWD/shorthair_amd/libcauchy256_$1.so"; fi; }
for round in 1 2; do
  for v in $(echo "$1" | tr , ' '); do
    printf "%-10s " "$v"
    SH_LIB_PATH=$(lib "$v") timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids | tail -1
    [ "${PIPESTATUS[0]}" = 0 ] || exit 1
  done
done
for v in $(echo "$1" | tr , ' '); do
  printf "%-10s " "$v"
  SH_LIB_PATH=$(lib "$v") timeout -k 10 120 python tools/run_ops.py --op both --iters 1 --digest 2>&1 | grep digest
  [ "${PIPESTATUS[0]}" = 0 ] || exit 1
done
[ "${PMC:-1}" = 0 ] && exit 0
i=0
for v in $(echo "$1" | tr , ' '); do
  for pass in "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" \
              "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU" \
              "FETCH_SIZE"; do
    i=$((i + 1))
    rm -rf gpurun_out/abif/p$i
    SH_LIB_PATH=$(lib "$v") timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/abif/p$i -o run \
        --output-format csv -- python3 tools/run_ops.py --op both --iters 2 > gpurun_out/abif/p$i.log 2>&1 \
        || { echo "pmc $v failed"; tail -3 gpurun_out/abif/p$i.log; exit 1; }
    echo "== $v: $pass"
    python3 tools/pmc_summary.py gpurun_out/abif/p$i 2>/dev/null | grep -A14 "kern_k200_m32" | grep -v "^--"
  done
done
