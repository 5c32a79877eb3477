#!/bin/bash
# context phase probes: tools/ctx_time.py per build/ab/skip* variant
set -o pipefail
O=gpurun_out/r3ctx
mkdir -p $O
for i in 1 2; do
for v in main skip1 skip2 skip4 skip8 skip16 skip32 skip63; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_${v}_$i.log 2>&1 || exit $?
done
done
