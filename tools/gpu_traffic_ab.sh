#!/bin/bash
# Per-op time + FETCH_SIZE / WRITE_SIZE per kernel for library variants (A/B of memory behaviour):
#   tools/gpu_traffic_ab.sh NAME[,NAME...]   (main = libcauchy256.so)   -> gpurun_out/tab/<name>/
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in $(echo $1 | tr , ' '); do
  L=$PWD/shorthair_amd/libcauchy256_$v.so; [ "$v" = main ] && L=$PWD/shorthair_amd/libcauchy256.so
  O=gpurun_out/tab/$v; rm -rf $O; mkdir -p $O
  echo "== variant $v"
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    SH_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/$c -o run --output-format csv -- \
      python3 tools/run_ops.py --op both --iters 3 > $O/$c.log 2>&1 || { echo "pmc $c failed"; tail -3 $O/$c.log; exit 1; }
  done
  python3 tools/traffic_json.py $O | python3 -c "import json,sys; d=json.load(sys.stdin)
for k,v in d['kernels'].items():
    print(f\"  {k[:40]:40s} read {v['read_bytes']/1e9:.3f} GB  write {v['write_bytes']/1e9:.3f} GB\")"
done
