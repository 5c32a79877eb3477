#!/bin/bash
set -o pipefail
O=gpurun_out/r3ab1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for v in main nopk nopl; do
  L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
  QI_LIB_PATH=$L timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_$v.log 2>&1 || exit $?
done
bash tools/ab_run.sh r3ab1 "--cfg cfg3" "" base || exit $?
mv gpurun_out/abr_r3ab1 $O/cfg3
bash tools/ab_run.sh r3ab1 "" "" base || exit $?
mv gpurun_out/abr_r3ab1 $O/cfg2
