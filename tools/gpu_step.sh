#!/bin/bash
# Parity on the product build, context timing, then A/B timing lines of
# build/ab/<variant> libraries at one config.
#   bash tools/gpu_step.sh <tag> "<bench args>" <variant>...
set -o pipefail
T=$1; ARGS=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_time.log 2>&1 &&
bash tools/ab_run.sh $T "$ARGS" "" "$@"
