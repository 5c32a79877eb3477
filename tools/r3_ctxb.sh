#!/bin/bash
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
QI_LIB_PATH=build/ab/ts/libquadiron_amd.so timeout -k 10 120 python3 tools/ctxb_ts.py > $O/ts.log 2>&1 || exit $?
for c in k200 k256 k300 k384; do
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
done
