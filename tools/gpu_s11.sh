#!/bin/bash
set -o pipefail
O=gpurun_out/s11
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 tools/host_rate.py > $O/host_rate.log 2>&1
