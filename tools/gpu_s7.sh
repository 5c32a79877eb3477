#!/bin/bash
set -o pipefail
O=gpurun_out/s7
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab_main_1.log 2>&1 &&
QI_LIB_PATH=build/ab/mst18/libquadiron_amd.so timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab_mst18_1.log 2>&1 &&
QI_LIB_PATH=build/ab/mfc2/libquadiron_amd.so timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab_mfc2_1.log 2>&1 &&
bash tools/prof.sh gpurun_out/s7/prof --steps 3 --no-cpu-baseline
