#!/bin/bash
# decode-context timing of build/ab/<variant> libraries (phase probes)
#   bash tools/ctx_probe.sh <tag> <variant>...
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
for v in "$@"; do
  QI_LIB_PATH=build/ab/$v/libquadiron_amd.so timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_$v.log 2>&1 || exit $?
done
