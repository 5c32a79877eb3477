#!/bin/bash
# Build a variant of the product library for A/B timing (not shipped):
#   bash tools/ab_build.sh <name> "<extra hipcc flags>" [patch]
# -> build/ab/<name>/libquadiron_amd.so ; use with QI_LIB_PATH=... bench.py
# With a patch (unified diff against quadiron_amd/csrc, `git diff --relative`
# style paths), the sources are copied under build/ab/<name>/q and patched
# there: probe variants (results deliberately wrong) never touch the product
# source.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/build/ab/$1
mkdir -p $D/obj
if [ -n "$3" ]; then
  P=$(cd "$(dirname "$3")" && pwd)/$(basename "$3")
  rm -rf $D/q
  mkdir -p $D/q/quadiron_amd
  cp -r $R/quadiron_amd/csrc $D/q/quadiron_amd/csrc
  ln -s $R/include $D/q/include
  ln -s $R/tests $D/q/tests
  patch -s -d $D/q/quadiron_amd/csrc -p1 < "$P"
  make -s -j8 -C $D/q/quadiron_amd/csrc OUT=$D/libquadiron_amd.so OBJDIR=$D/obj EXTRA="$2" \
      $D/libquadiron_amd.so
else
  make -s -j8 -C $R/quadiron_amd/csrc OUT=$D/libquadiron_amd.so OBJDIR=$D/obj EXTRA="$2" \
      $D/libquadiron_amd.so
fi
