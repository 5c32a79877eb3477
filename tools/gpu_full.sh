#!/bin/bash
# Full measurement session (GPU box): headline bench with the CPU baseline,
# rocprofv3 kernel stats, PMC traffic passes, extra bench lines, host rate.
#   bash tools/gpu_full.sh <tag>
set -o pipefail
T=${1:-full}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 &&
bash tools/prof.sh $O/prof --steps 10 --no-cpu-baseline &&
bash tools/pmc.sh $O/pmc --steps 3 --warmup 1 &&
bash tools/gpu_lines.sh $T/lines
