set -u
L=$PWD/shorthair_amd/libcauchy256_cfg.so
for c in "200 16 8192" "200 32 8192" "64 16 25600" "112 16 14628" "224 32 7314"; do
  set -- $c
  SH_LIB_PATH=$L timeout -k 10 120 python tools/run_ops.py --op encode --iters 10 --k $1 --m $2 --groups $3 2>&1 | grep -v amdgpu.ids | sed "s/^/k=$1 m=$2 G=$3: /" || exit 1
done
