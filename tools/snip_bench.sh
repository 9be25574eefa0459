set -u
for m in 0 1; do timeout -k 5 60 tools/snip_bench $m 8192 0 32 || exit 1; done
timeout -k 5 60 tools/snip_bench 3 16384 0 32 || exit 1
timeout -k 5 60 tools/snip_bench 0 8192 0 32 || exit 1
timeout -k 5 60 tools/snip_bench 3 16384 0 32 || exit 1
