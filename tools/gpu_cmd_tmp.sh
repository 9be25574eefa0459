mkdir -p gpurun_out
for b in 4 2 8 1; do timeout -k 10 60 tools/jump_probe $b 4000 || exit 1; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "decode or tile or golden" --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/run_ops.py --op decode --iters 5 --k 200 --m 56 --block 1352 --groups 5547 --erasures 56 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/run_ops.py --op decode --iters 5 --k 190 --m 66 --block 1336 --groups 5909 --erasures 66 2>&1 | grep -v amdgpu.ids || exit 1
