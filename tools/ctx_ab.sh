#!/bin/bash
# decode-context timing: product vs build/ab/<variant>, alternating twice
#   bash tools/ctx_ab.sh <tag> <variant>...
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_main_$i.log 2>&1 || exit $?
  for v in "$@"; do
    QI_LIB_PATH=build/ab/$v/libquadiron_amd.so timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_${v}_$i.log 2>&1 || exit $?
  done
done
