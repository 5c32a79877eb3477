#!/bin/bash
# cfg3 A/B lines: parity subset, then bench lines (codelet and matrix encode).
set -o pipefail
T=${1:-ab3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "64-960 or golden or dense or 33-31 or 32-32 or cfg4 or 16-48" > $O/pytest_ab.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 &&
QI_ENC_MATRIX=1 timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_matcfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_cfg2.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline > $O/bench_sys.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3b.log 2>&1
