#!/bin/bash
# A/B of the pipelined MFMA super-tile loop (main: KS >= 2, pipe4: KS = 4,
# nopipe: never) on cfg3 and a k = 32 code, after the full GPU suite.
set -o pipefail
O=gpurun_out/ab_pipe
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for i in 1 2; do
  for v in main pipe4 nopipe; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --cfg cfg3 > $O/${v}_cfg3_$i.log 2>&1 &&
    QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --systematic > $O/${v}_sys_$i.log 2>&1 || exit 1
  done
done
