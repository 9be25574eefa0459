mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py tests/test_groups.py tests/test_loopback.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t10.log 2>&1; rc=$?; tail -3 gpurun_out/t10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-sweep > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err; rc=$?; python -c "import json; d=json.load(open('gpurun_out/bench_h.json')); print(d['value'], d['host_path'])"; exit $rc
