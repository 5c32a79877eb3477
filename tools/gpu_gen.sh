#!/bin/bash
# General-path bench lines + rocprof kernel stats.  bash tools/gpu_gen.sh <tag>
set -o pipefail
T=${1:-gen}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --cfg k200 --no-cpu-baseline --steps 5 > $O/bench_k200.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k256 --no-cpu-baseline --steps 5 > $O/bench_k256.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k200 --systematic --no-cpu-baseline --steps 5 > $O/bench_k200_sys.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k200 -- python3 bench.py --cfg k200 --no-cpu-baseline --steps 5 > $O/prof_k200.log 2>&1
