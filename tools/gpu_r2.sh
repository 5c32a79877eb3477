#!/bin/bash
# Round-2 GPU session: parity tests, smoke, headline + extra bench lines,
# rocprofv3 kernel stats of the headline.  Each GPU step has its own limit;
# the chain stops at the first failure.   bash tools/gpu_r2.sh <tag>
set -o pipefail
T=${1:-r2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic > $O/bench_sys.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg1 > $O/bench_cfg1.log 2>&1 &&
bash tools/prof.sh $O/prof --steps 10 --no-cpu-baseline
