#!/bin/bash
set -o pipefail
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 60 ./build/mfma_probe > $O/mfma_probe.log 2>&1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
QI_LIB_PATH=build/ab/nopair/libquadiron_amd.so timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_nopair_old.log 2>&1
