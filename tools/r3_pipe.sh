#!/bin/bash
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_time.log 2>&1 &&
QI_LIB_PATH=build/ab/ts/libquadiron_amd.so timeout -k 10 120 python3 tools/ctx_ts.py > $O/ts.log 2>&1 || exit $?
for i in 1 2; do
  for v in 1 0; do
    QI_PIPE=$v timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline --steps 20 > $O/cfg3_pipe${v}_$i.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_cfg2.log 2>&1
