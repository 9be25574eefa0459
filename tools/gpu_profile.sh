#!/bin/bash
# Evidence set for one build, all at the headline workload (k=200 m=32 B=1400, 8192 groups, e=32):
#   tools/gpu_profile.sh TAG      -> gpurun_out/prof_TAG/
#   1. traffic.json   rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace only)
#                     over tools/run_ops.py (batch ops only, no single-group host-path calls),
#                     corrected per MI355X_MICROARCH.md (tools/traffic_json.py); carries the
#                     library's SHA-256, which bench.py matches before using it.
#   2. sq.txt         one SQ/GRBM pass (VALU busy, wait / issue-stall cycles, SALU count).
#   3. ifetch.txt     with IFETCH="<SQC counters>": one instruction-fetch pass.
#   4. bench_kernel_stats.csv + bench.log: rocprofv3 --kernel-trace --stats of the headline bench
#                     (no sweep, no CPU leg) -- its per-kernel averages are what bench.py's
#                     roofline.launch_ms is checked against.
# Copy the directory to profiles/<round>/ to commit it. Every GPU step has its own time limit.
set -u
TAG=${1:-cur}
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
pmc() {  # pmc NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- \
    python3 tools/run_ops.py --op both --iters 3 > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$OUT/$name.log"; return 1; }
  echo "pass $name ok"
}
pmc fetch FETCH_SIZE || exit 1
pmc write WRITE_SIZE || exit 1
pmc sq GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU || exit 1
python3 tools/pmc_summary.py "$OUT/sq" > "$OUT/sq.txt"
python3 tools/traffic_json.py "$OUT" > "$OUT/traffic.json" || exit 1
# bench.py reads profiles/*/traffic*.json (matched by the library hash): the run below sees it
PROFDIR=${PROFDIR:-profiles/r06}; mkdir -p $PROFDIR && cp "$OUT/traffic.json" "$PROFDIR/traffic_$TAG.json"
if [ -n "${IFETCH:-}" ]; then  # e.g. IFETCH="SQC_ICACHE_REQ SQC_ICACHE_MISSES" (names from --list-avail)
  pmc ifetch $IFETCH || exit 1
  python3 tools/pmc_summary.py "$OUT/ifetch" > "$OUT/ifetch.txt"
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv -- \
  python3 bench.py --steps 40 --warmup 3 --no-cpu --host-calls 0 --no-sweep > "$OUT/bench.log" 2>&1 || { echo "stats run failed"; tail -5 "$OUT/bench.log"; exit 1; }
cp "$(find "$OUT/stats" -name run_kernel_stats.csv | head -1)" "$OUT/bench_kernel_stats.csv"
python3 tools/kstats.py "$OUT/stats" > "$OUT/kstats.txt"
rm -rf "$OUT/fetch" "$OUT/write" "$OUT/sq" "$OUT/ifetch" "$OUT/stats"
[ -n "${LIST:-}" ] && { timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1; grep -c . "$OUT/list_avail.txt"; }
cat "$OUT/traffic.json"; cat "$OUT/kstats.txt"; grep -v amdgpu.ids "$OUT/bench.log" | tail -1 | cut -c1-600
