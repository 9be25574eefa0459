#!/bin/bash
# rocprofv3 PMC passes over tools/run_ops.py (each pass its own run, --kernel-trace only beside
# --pmc, as required on this pool). Usage: tools/gpu_pmc.sh [op] [tag]; summary -> gpurun_out/pmc_<tag>.txt
set -u
OP=${1:-encode}
TAG=${2:-run}
mkdir -p gpurun_out/pmc_$TAG
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmc_$TAG/p$i -o run --output-format csv -- python3 tools/run_ops.py --op $OP --iters 2 > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG.txt; cat gpurun_out/pmc_$TAG.txt
