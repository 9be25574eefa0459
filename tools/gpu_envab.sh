#!/bin/bash
# Per-op device time of one library under several environment settings (host-side switches):
#   tools/gpu_envab.sh "SH_DEC_CHUNKS=1 SH_DEC_CHUNKS=4" [run_ops.py args...]
# Each setting is one `VAR=VAL[,VAR=VAL]` word; "-" = no extra environment.
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
sets=$1; shift
for e in $sets; do
  echo "== env $e"
  envs=""; [ "$e" != "-" ] && envs=$(echo "$e" | tr , ' ')
  env $envs timeout -k 10 120 python tools/run_ops.py --op both --iters 10 "$@" 2>&1 | grep -v amdgpu.ids || exit 1
done
