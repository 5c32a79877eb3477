#!/bin/bash
# Quick GPU check: parity tests then headline/cfg3/sys bench lines (no CPU
# baseline).   bash tools/gpu_quick.sh <tag>
set -o pipefail
T=${1:-quick}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline > $O/bench_sys.log 2>&1
[ $? -eq 0 ] && QI_ENC_MATRIX=1 timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_matcfg3.log 2>&1 &&
QI_ENC_MATRIX=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_matcfg2.log 2>&1
