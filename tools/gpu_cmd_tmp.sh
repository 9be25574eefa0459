set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
SH_V2_MIN=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -2 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
for shp in "64 16 1400 16741" "28 4 1400 38265" "112 16 1400 9566" "64 16 256 60000"; do
  bash tools/gpu_ab_shape.sh $shp main || exit 1
  SH_V2_MIN=0 bash tools/gpu_ab_shape.sh $shp main || exit 1
done
