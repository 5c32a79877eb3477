#!/bin/bash
# quick GPU check: parity suite, smoke, context timing, cfg2 + cfg3 bench lines
#   bash tools/r3_quick.sh <tag>
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 120 python3 tools/ctx_time.py > $O/ctx_time.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1
