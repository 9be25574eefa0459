#!/bin/bash
# Build the encode-kernel lab (tools/enc_lab.hip, measurement only) against freshly generated
# (200, 32) bodies: tools/enc_lab.sh TAG [ENV=VAL ...]  -> tools/lab_bin/enc_lab_TAG
# ENV overrides go to the generator (e.g. SH_RING=14) and LAB_R must match the ring it generates.
set -eu
TAG=$1; shift
cd "$(dirname "$0")/.."
GEN=shorthair_amd/csrc/gen_lab_$TAG
mkdir -p "$GEN" tools/lab_bin
env "$@" python - "$GEN" <<'EOF'
import importlib.util, sys
spec = importlib.util.spec_from_file_location("g", "tools/gen_fixed_kernels.py")
g = importlib.util.module_from_spec(spec); spec.loader.exec_module(g)
g.OUTDIR = sys.argv[1]
g.gen_config(200, 32)
EOF
R=$(grep -o 'FIXED_KERNEL(k200_m32, 200, 32, [0-9]*, [0-9]*, [0-9]*' "$GEN/fixed_k200_m32_enc.hip" | awk -F', ' '{print $NF}')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLAB_R=$R -I"$GEN" -Ishorthair_amd/csrc \
    ${LAB_FLAGS:-} tools/enc_lab.hip -o tools/lab_bin/enc_lab_$TAG
echo "built tools/lab_bin/enc_lab_$TAG (R=$R)"
