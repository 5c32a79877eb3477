#!/bin/bash
# Round-6 (session 2): operand-stationary kernel with the route list staged
# once per route tile and mark buffer (product) vs every tile (os_restage)
set -o pipefail
O=gpurun_out/r6v18
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; cp $O/pytest_gpu.log profiles/r6_fail_v18.log; exit 1; }
tail -1 $O/pytest_gpu.log
AB_WARMUP=50 bash tools/ab_quick.sh r6v18 "cfg3 cfg3p64 k128 k300" os_restage || exit 1
