#!/bin/bash
# PMC passes over decode_setup at one shape (measurement only):
#   tools/gpu_setup_pmc.sh K M B GROUPS
set -u
mkdir -p gpurun_out/setup_pmc
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
K=$1 M=$2 B=$3 G=$4
E=$(( K < M ? K : M ))
i=0
for pass in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
            "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"; do
  i=$((i + 1))
  rm -rf gpurun_out/setup_pmc/p$i
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d gpurun_out/setup_pmc/p$i -o run --output-format csv -- \
      python3 tools/run_ops.py --op decode --iters 2 --k $K --m $M --block $B --groups $G --erasures $E > gpurun_out/setup_pmc/p$i.log 2>&1 \
      || { echo "pass $i failed"; tail -3 gpurun_out/setup_pmc/p$i.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/setup_pmc/p$i 2>/dev/null | grep -A10 "decode_setup"
done
timeout -k 10 120 python tools/run_ops.py --op decode --iters 10 --k $K --m $M --block $B --groups $G --erasures $E 2>&1 | grep -v amdgpu.ids | tail -1
