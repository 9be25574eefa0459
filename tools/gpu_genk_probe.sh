set -u
for round in 1 2; do
for shape in "224 32" "150 32" "200 32" "112 16" "100 16" "200 56" "150 56" "190 66" "120 66"; do
  set -- $shape
  printf "(%s,%s,1400) G=6000 " $1 $2
  timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --k $1 --m $2 --block 1400 --groups 6000 --erasures 8 2>&1 | grep -v amdgpu.ids | tail -1
  [ "${PIPESTATUS[0]}" = 0 ] || exit 1
done
done
