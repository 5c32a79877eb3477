#!/bin/bash
# cfg3 parity subset + bench line + rocprof kernel stats.  bash tools/gpu_cfg3.sh <tag>
set -o pipefail
T=${1:-cfg3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "64-960 or golden or dense or 33-31 or cfg4" > $O/pytest_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline > $O/bench_cfg3.log 2>&1 &&
bash tools/prof.sh gpurun_out/$T/prof --cfg cfg3 --steps 10 --no-cpu-baseline &&
python3 tools/kstats.py gpurun_out/$T/prof > $O/prof_summary.txt 2>&1
