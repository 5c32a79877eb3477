#!/bin/bash
# GPU box: parity suite, smoke, and the given bench lines
#   bash tools/r3_check.sh <tag> <cfg>...
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
done
