#!/bin/bash
# k300 NTT-engine profile: rocprofv3 kernel stats + pipe-level PMC (GPU box)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
bash tools/prof.sh $O/prof --cfg k300 --steps 5 --no-cpu-baseline &&
BENCH_ARGS="--cfg k300" bash tools/pmc_pipe.sh $O/pipe --cfg k300
