#!/bin/bash
# Parity tests + one bench line (GPU box).  Usage: bash tools/gpu_quick.sh <tag> [bench args]
set -o pipefail
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > $O/bench.log 2>&1
