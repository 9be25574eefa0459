mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
IFETCH="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES" timeout -k 10 900 bash tools/gpu_profile.sh a > gpurun_out/prof_a.log 2>&1; rc=$?; tail -25 gpurun_out/prof_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err; rc=$?; tail -c 600 gpurun_out/bench_a.json; exit $rc
