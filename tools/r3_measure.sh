#!/bin/bash
# Round-3 measurement pass (GPU box): parity, smoke, the bench lines, PMC
# roofline records (cfg2, cfg3, systematic), rocprofv3 kernel stats.
#   bash tools/r3_measure.sh <tag> [quick]
set -o pipefail
T=${1:-r3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic > $O/bench_sys.log 2>&1 &&
bash tools/pmc_roofline.sh $O/pmc_cfg2 cfg2 4096 &&
bash tools/pmc_roofline.sh $O/pmc_cfg3 cfg3 1024 --cfg cfg3 &&
bash tools/pmc_roofline.sh $O/pmc_sys cfg2_sys 4096 --systematic &&
bash tools/prof.sh $O/prof --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_cfg3 --cfg cfg3 --steps 10 --no-cpu-baseline
