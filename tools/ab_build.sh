#!/bin/bash
# Build a variant of the product library for A/B timing (not shipped):
#   bash tools/ab_build.sh <name> "<extra hipcc flags>"
# -> build/ab/<name>/libquadiron_amd.so ; use with QI_LIB_PATH=... bench.py
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build/ab/$1
mkdir -p $D/obj
make -s -j8 -C $R/quadiron_amd/csrc OUT=$D/libquadiron_amd.so OBJDIR=$D/obj EXTRA="$2"
