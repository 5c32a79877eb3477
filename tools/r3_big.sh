#!/bin/bash
# GPU box: parity suite + k300 / k384 bench lines
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for c in k300 k200 k256; do
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
done
