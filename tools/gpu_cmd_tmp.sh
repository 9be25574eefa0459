set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for shp in "150 40 1400 7142" "180 76 1352 6163" "120 136 1400 8928" "90 49 1400 8192" "50 10 1000 30000"; do
  bash tools/gpu_ab_shape.sh $shp main || exit 1
  SH_COL_DEC=1 SH_COL_ENC=1 bash tools/gpu_ab_shape.sh $shp main || exit 1
done
