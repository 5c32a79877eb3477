#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-s5}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --systematic > $O/bench_sys.log 2>&1
