#!/bin/bash
# One rocprofv3 counter pass per argument over the headline batch ops (tools/run_ops.py):
#   tools/gpu_pmc.sh "SQ_A SQ_B ..." "SQC_X SQC_Y" ...   -> gpurun_out/pmc/pass<i>.txt
# Keep each pass within the per-block limits (8 SQ, 4 TCC, ...): an over-full pass hangs rocprofv3,
# so every pass runs under its own SIGKILL limit and the script stops at the first failure.
set -u
O=gpurun_out/pmc; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace -d $O/p$i -o run --output-format csv -- \
    python3 tools/run_ops.py --op both --iters 3 > $O/p$i.log 2>&1 || { echo "pass $i ($ctrs) failed"; tail -3 $O/p$i.log; exit 1; }
  python3 tools/pmc_summary.py $O/p$i > $O/pass$i.txt
  rm -rf $O/p$i
  echo "== pass $i: $ctrs"; grep -A12 "kern_k200_m32_enc\|stageb_fixed" $O/pass$i.txt | grep -v "^--"
done
