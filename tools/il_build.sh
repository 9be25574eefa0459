#!/bin/bash
# Measurement builds (round 5): code objects of the compile-time kernels of one (k, m), as
# compiled (hsaco_ref/) and with the parts' units interleaved by tools/il_reorder.py (hsaco_il/),
# for SH_HSACO_DIR A/B runs:   tools/il_build.sh K M [--group G]
set -eu
K=$1; M=$2; shift 2
cd "$(dirname "$0")/.."
GEN=shorthair_amd/csrc/gen_ilm
mkdir -p "$GEN" hsaco_ref hsaco_il
SH_IL_MARK=1 python - "$GEN" "$K" "$M" <<'PY'
import importlib.util, sys
spec = importlib.util.spec_from_file_location("g", "tools/gen_fixed_kernels.py")
g = importlib.util.module_from_spec(spec); spec.loader.exec_module(g)
g.OUTDIR = sys.argv[1]; g.load_sched_cache(); g.gen_config(int(sys.argv[2]), int(sys.argv[3]))
PY
LLVM=/opt/rocm/lib/llvm/bin
for mode in enc dec; do
  tag=k${K}_m${M}_$mode
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --cuda-device-only -S -I"$GEN" -Ishorthair_amd/csrc \
      "$GEN/fixed_${tag}.hip" -o "$GEN/$tag.s" &
done
wait
for mode in enc dec; do
  tag=k${K}_m${M}_$mode
  python tools/il_reorder.py "$GEN/$tag.s" "$GEN/${tag}_il.s" "$@"
  $LLVM/clang --target=amdgcn-amd-amdhsa -mcpu=gfx950 -c "$GEN/${tag}_il.s" -o "$GEN/${tag}_il.o"
  $LLVM/ld.lld -shared "$GEN/${tag}_il.o" -o "hsaco_il/$tag.hsaco"
  $LLVM/clang --target=amdgcn-amd-amdhsa -mcpu=gfx950 -c "$GEN/$tag.s" -o "$GEN/$tag.o"
  $LLVM/ld.lld -shared "$GEN/$tag.o" -o "hsaco_ref/$tag.hsaco"
done
ls -la hsaco_il hsaco_ref
