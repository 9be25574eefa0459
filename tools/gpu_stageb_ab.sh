#!/bin/bash
# Stage-B dispatch A/B (measurement only): per-op device times of tools/run_ops.py for the
# Tester / large-e shapes under the SH_V2_MAX / SH_V2_NW switches. Each run has its own limit.
set -u
mkdir -p gpurun_out
run() {  # run LABEL K M B [ENV=VAL ...]
  local lab=$1 k=$2 m=$3 b=$4; shift 4
  printf "%-28s (%d,%d,%d) " "$lab" "$k" "$m" "$b"
  env "$@" timeout -k 10 120 python tools/run_ops.py --op decode --iters 10 --k "$k" --m "$m" --block "$b" --groups ${G:-4096} \
      --erasures $(( k < m ? k : m )) 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
}
for shp in "200 56 1352" "190 66 1336" "120 136 1400" "200 32 1400"; do
  set -- $shp
  run default "$@" || exit 1
  run v2all "$@" SH_V2_MAX=128 || exit 1
  run v2all_nw4 "$@" SH_V2_MAX=128 SH_V2_NW=4 || exit 1
  run v2all_nw8 "$@" SH_V2_MAX=128 SH_V2_NW=8 || exit 1
done
