set -u
timeout -k 10 200 python -u -m pytest tests/test_shorthair_link.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/sl.log 2>&1; rc=$?; tail -2 gpurun_out/sl.log
timeout -k 10 60 oracle/_ref/shorthair_link --seconds 3 || exit 1
SH_V2_NW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden or decode" > gpurun_out/t.log 2>&1 || { tail -5 gpurun_out/t.log; exit 1; }; tail -1 gpurun_out/t.log
for shp in "200 32 1400 8192" "200 56 1352 5547"; do
  bash tools/gpu_ab_shape.sh $shp main || exit 1
  SH_V2_NW=2 bash tools/gpu_ab_shape.sh $shp main || exit 1
  bash tools/gpu_ab_shape.sh $shp main || exit 1
done
exit $rc
