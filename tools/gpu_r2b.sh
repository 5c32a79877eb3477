#!/bin/bash
# Parity (general path subset + full), general-path lines, headline and cfg3
# lines.   bash tools/gpu_r2b.sh <tag>
set -o pipefail
T=${1:-r2b}
O=gpurun_out/$T
mkdir -p $O
bash tools/gpu_ntt.sh $T &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k200 --no-cpu-baseline --steps 5 > $O/bench_k200.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k256 --no-cpu-baseline --steps 5 > $O/bench_k256.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k200 --systematic --no-cpu-baseline --steps 5 > $O/bench_k200_sys.log 2>&1
