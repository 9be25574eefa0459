set -u
mkdir -p gpurun_out
IFETCH="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES" PROFDIR=profiles/r03 bash tools/gpu_profile.sh e > gpurun_out/prof_e.out 2>&1 || { tail -5 gpurun_out/prof_e.out; exit 1; }
tail -3 gpurun_out/prof_e.out
timeout -k 10 600 python bench.py > gpurun_out/bench_full_e.json 2> gpurun_out/bench_full_e.err || { tail -5 gpurun_out/bench_full_e.err; exit 1; }
python tools/sweep_table.py gpurun_out/bench_full_e.json
bash tools/gpu_run.sh tests || exit $?
