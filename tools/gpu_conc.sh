set -u
timeout -k 10 120 python tools/run_ops.py --op both --iters 10 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/run_ops.py --op both --iters 10 --concurrent 2>&1 | grep -v amdgpu.ids || exit 1
