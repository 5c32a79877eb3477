#!/bin/bash
set -o pipefail
for i in 1 2; do
for v in main nomfma; do
  L=build/ab/$v/libquadiron_amd.so; [ $v = main ] && L=quadiron_amd/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/ab_cfg2_${v}_$i.log 2>&1 || exit $?
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --systematic > gpurun_out/ab_sys_${v}_$i.log 2>&1 || exit $?
  QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --cfg cfg3 > gpurun_out/ab_cfg3_${v}_$i.log 2>&1 || exit $?
done
done
