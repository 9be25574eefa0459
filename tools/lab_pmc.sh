#!/bin/bash
# PMC passes over a lab binary (measurement only): tools/lab_pmc.sh BIN TAG [--only VARIANTS]
set -u
BIN=$1; TAG=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
O=gpurun_out/labpmc_$TAG; rm -rf $O; mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_IFETCH" \
           "SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_MISSES SQC_ICACHE_REQ SQC_TC_STALL SQC_ICACHE_BUSY_CYCLES SQC_TC_INST_REQ"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $O/p$i -o run --output-format csv -- "$BIN" --iters 3 "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
