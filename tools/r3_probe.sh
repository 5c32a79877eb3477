#!/bin/bash
# GPU box: parity suite + matrix-kernel block timelines (probe build)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
QI_LIB_PATH=build/ab/ts/libquadiron_amd.so timeout -k 10 120 python3 tools/mm_ts.py cfg3 > $O/mm_cfg3.log 2>&1 &&
QI_LIB_PATH=build/ab/ts/libquadiron_amd.so timeout -k 10 120 python3 tools/mm_ts.py cfg2 > $O/mm_cfg2.log 2>&1
