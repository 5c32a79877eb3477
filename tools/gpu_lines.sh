#!/bin/bash
# Extra bench lines (cfg3, systematic, cfg1) + host-inclusive rate on the GPU box.
set -o pipefail
O=gpurun_out/${1:-lines}
mkdir -p $O
timeout -k 10 300 python3 bench.py --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic > $O/bench_sys.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg1 > $O/bench_cfg1.log 2>&1 &&
timeout -k 10 300 python3 tools/host_rate.py > $O/host_rate.log 2>&1
