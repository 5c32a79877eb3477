#!/bin/bash
# General-path (k > 64) GPU check: the new parity tests first, then the
# whole GPU suite.   bash tools/gpu_ntt.sh <tag>
set -o pipefail
T=${1:-ntt}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "general or golden or 65-63 or 100- or 200- or 256- or 130- or 1000- or dense or overflow" > $O/pytest_ntt.log 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
