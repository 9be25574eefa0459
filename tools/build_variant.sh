#!/bin/bash
# Build an experimental library variant: tools/build_variant.sh NAME [ENV=VAL ...]
# -> shorthair_amd/libcauchy256_NAME.so (generator/compile env overrides, (200,32) only unless
# SH_CONFIGS is given). Used with SH_LIB_PATH=... for A/B runs on the GPU. Variants are measurement
# builds (-DSH_MEASUREMENT_BUILD, csrc/measure.hpp): only they read the A/B environment switches.
set -eu
NAME=$1; shift
cd "$(dirname "$0")/.."
env SH_CONFIGS="${SH_CONFIGS:-200,32}" "$@" SH_MEASUREMENT=1 SH_GEN_DIR=gen_$NAME SH_OBJ_DIR=build_obj_$NAME SH_LIB_NAME=libcauchy256_$NAME.so \
    python -c "
import importlib.util, sys
spec = importlib.util.spec_from_file_location('b', 'shorthair_amd/build.py'); b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
b.build(force=True, verbose=False)
print('built', b.LIB)"
