set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for shp in "28 4 256 209263" "112 16 256 52315" "224 32 256 26157" "28 4 1400 38265" "200 32 1400 8192"; do
  bash tools/gpu_ab_shape.sh $shp main || exit 1
done
