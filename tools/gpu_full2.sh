#!/bin/bash
# Round-2 measurement pass: parity, smoke, every bench line, rocprofv3 kernel
# stats at cfg2 / cfg3 / k128, PMC traffic at cfg2.  Each GPU step has its
# own limit; the chain stops at the first failure.   bash tools/gpu_full2.sh <tag>
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
timeout -k 10 300 python3 bench.py --cfg k128 --steps 10 > $O/bench_k128.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k200 --steps 5 > $O/bench_k200.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k256 --steps 5 > $O/bench_k256.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k300 --steps 3 > $O/bench_k300.log 2>&1 &&
bash tools/prof.sh $O/prof --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_cfg3 --cfg cfg3 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_k128 --cfg k128 --steps 5 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_k200 --cfg k200 --steps 5 --no-cpu-baseline &&
bash tools/prof.sh $O/prof_k256 --cfg k256 --steps 5 --no-cpu-baseline &&
bash tools/pmc.sh $O/pmc --steps 3 --warmup 1
