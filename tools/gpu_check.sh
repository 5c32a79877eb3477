#!/bin/bash
# One GPU-box session: parity tests, memory-pattern ceilings, bench lines.
# Every GPU step has its own time limit and the chain stops at the first
# failure.  Usage (from the repo root on the box): bash tools/gpu_check.sh
set -o pipefail
O=gpurun_out
mkdir -p $O
rm -f $O/pytest_gpu.log $O/membw2.log $O/bench*.log $O/host_rate.log
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 ./build/membw2 4096 > $O/membw2.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic > $O/bench_sys.log 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 300 python3 tools/host_rate.py > $O/host_rate.log 2>&1
