#!/bin/bash
set -o pipefail
O=gpurun_out/s12
mkdir -p $O
QI_LIB_PATH=build/ab/mf16/libquadiron_amd.so timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_mf16.log 2>&1 &&
for i in 1 2; do
for v in main mf16 nomfma; do
  L=build/ab/$v/libquadiron_amd.so; [ $v = main ] && L=quadiron_amd/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_cfg2_${v}_$i.log 2>&1 || exit $?
done
done
