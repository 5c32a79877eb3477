#!/bin/bash
# GPU box: parity suite, then the NTT-engine bench line under rocprofv3
#   bash tools/r3_ntt.sh <tag> [cfg...]
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for c in "${@:-k1000}"; do
  bash tools/prof.sh $O/prof_$c --cfg $c --steps 5 --no-cpu-baseline || exit $?
done
