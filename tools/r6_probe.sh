#!/bin/bash
# Round-6 probes (GPU box):
#   bash tools/r6_probe.sh <tag>
# 1. race audit: the golden + route-table tests on
#    two probe builds of the context kernels with the route-table clears
#    delayed by s_sleep (tools/ab/race_sleep_*.patch, built beforehand by
#    tools/ab_build.sh race_fixed / race_r4):
#      race_fixed: the product protocol -> must pass
#      race_r4:    round 4's protocol (every thread clears, nothing orders the
#                  clears before the adds) -> the lost OOR restores show
# 2. the write ceiling (tools/writebw.hip, built as build/writebw)
set -o pipefail
T=${1:-r6p}
O=gpurun_out/$T
mkdir -p $O
SEL="golden or dense or route or cfg3_random or batch_vs_oracle"
for v in race_fixed race_r4; do
  QI_LIB_PATH=build/ab/$v/libquadiron_amd.so timeout -k 10 600 python3 -u -m pytest \
    tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread \
    -k "$SEL" > $O/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 $O/$v.log)"
  # a fault / abort / kill ends the script (rc 1 = test failures, expected for race_r4)
  case $rc in 0|1) ;; *) exit $rc;; esac
done
timeout -k 10 300 ./build/writebw > $O/writebw.txt 2>&1 || exit $?
cat $O/writebw.txt
