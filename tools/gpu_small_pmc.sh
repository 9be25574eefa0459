#!/bin/bash
# PMC passes over the small-block stage B (measurement only): tools/gpu_small_pmc.sh K M B G E
set -u
mkdir -p gpurun_out/small_pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
K=$1 M=$2 B=$3 G=$4 E=$5
L=$PWD/shorthair_amd/libcauchy256_meas.so
i=0
for v in 0 1; do
  for pass in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS" \
              "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"; do
    i=$((i + 1))
    rm -rf gpurun_out/small_pmc/p$i
    SH_LIB_PATH=$L SH_SMALL2=$v timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/small_pmc/p$i -o run --output-format csv -- \
        python3 tools/run_ops.py --op decode --iters 2 --k $K --m $M --block $B --groups $G --erasures $E > gpurun_out/small_pmc/p$i.log 2>&1 \
        || { echo "pass $i failed"; tail -3 gpurun_out/small_pmc/p$i.log; exit 1; }
    echo "== small2=$v"
    python3 tools/pmc_summary.py gpurun_out/small_pmc/p$i 2>/dev/null | grep -A10 "stageb_small"
  done
done
