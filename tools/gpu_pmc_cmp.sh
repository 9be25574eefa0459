#!/bin/bash
# PMC passes over the codec encode (run_ops) and the staging microbenchmark, same counters.
set -u
mkdir -p gpurun_out/pmcc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH_LEVEL SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmcc/a$i -o run --output-format csv -- python3 tools/run_ops.py --op encode --iters 2 > gpurun_out/pmcc/a$i.log 2>&1 || { echo "pass a$i failed"; tail -5 gpurun_out/pmcc/a$i.log; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/pmcc/b$i -o run --output-format csv -- ./tools/stage_bench2 > gpurun_out/pmcc/b$i.log 2>&1 || { echo "pass b$i failed"; tail -5 gpurun_out/pmcc/b$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py gpurun_out/pmcc > gpurun_out/pmcc.txt; cat gpurun_out/pmcc.txt
