#!/bin/bash
# Round-3 measurement pass (GPU box): parity, smoke, every bench line, PMC
# roofline records, rocprofv3 kernel stats.
#   bash tools/r3_final.sh <tag>
set -o pipefail
T=${1:-r3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
for c in cfg3 k32 k128 k200 k256 k300 k384 k1000 cfg1 cfg3p64; do
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline > $O/bench_sys.log 2>&1 &&
bash tools/pmc_roofline.sh $O/pmc_cfg2 cfg2 4096 &&
bash tools/pmc_roofline.sh $O/pmc_cfg3 cfg3 1024 --cfg cfg3 &&
bash tools/pmc_roofline.sh $O/pmc_sys cfg2_sys 4096 --systematic &&
bash tools/pmc_roofline.sh $O/pmc_k200 k200 64 --cfg k200 &&
bash tools/pmc_roofline.sh $O/pmc_k256 k256 256 --cfg k256 &&
bash tools/prof.sh $O/prof_cfg2 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_cfg3 --cfg cfg3 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_k200 --cfg k200 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_k1000 --cfg k1000 --steps 5 --no-cpu-baseline &&
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1
