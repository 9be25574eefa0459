set -u
for m in 0 4 0 4 1; do timeout -k 5 60 tools/snip_bench $m 8192 0 32 || exit 1; done
