#!/bin/bash
# matrix-path parity (incl. the matrix-encode knob) + cfg3/cfg2 encode A/B lines
set -o pipefail
T=${1:-ab4}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3_$i.log 2>&1 &&
  QI_ENC_MATRIX=1 timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_matcfg3_$i.log 2>&1 || exit 1
done &&
timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline > $O/bench_sys.log 2>&1 &&
QI_ENC_MATRIX=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_matcfg2.log 2>&1
