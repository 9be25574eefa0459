set -u
for m in 0 1; do for l in 0 49152 81920; do timeout -k 5 60 tools/snip_bench $m 8192 $l 32 || exit 1; done; done
timeout -k 5 60 tools/snip_bench 0 1024 0 256 || exit 1
timeout -k 5 60 tools/snip_bench 1 1024 0 256 || exit 1
