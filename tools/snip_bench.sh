set -u
for m in 0 1 2; do for l in 0 49152; do timeout -k 5 60 tools/snip_bench $m 8192 $l 32 || exit 1; done; done
