#!/bin/bash
set -o pipefail
O=gpurun_out/s6
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
bash tools/ab_bench.sh mfc2 nomfma &&
for v in main mfc2 nomfma; do
  L=build/ab/$v/libquadiron_amd.so; [ $v = main ] && L=quadiron_amd/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --systematic > gpurun_out/ab_sys_$v.log 2>&1 || exit $?
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --cfg cfg3 > gpurun_out/ab_cfg3_$v.log 2>&1 || exit $?
done
