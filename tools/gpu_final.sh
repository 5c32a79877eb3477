#!/bin/bash
# Round measurement pass: full parity suite, smoke, every bench line (the
# headline with its CPU baseline), rocprofv3 kernel stats of cfg2 / cfg3 /
# general path.   bash tools/gpu_final.sh <tag>
set -o pipefail
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg3 > $O/bench_cfg3.log 2>&1 &&
timeout -k 10 300 python3 bench.py --systematic --no-cpu-baseline > $O/bench_sys.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg cfg1 > $O/bench_cfg1.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k200 --no-cpu-baseline --steps 5 > $O/bench_k200.log 2>&1 &&
timeout -k 10 300 python3 bench.py --cfg k256 --no-cpu-baseline --steps 5 > $O/bench_k256.log 2>&1 &&
bash tools/prof.sh gpurun_out/$T/prof_cfg2 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh gpurun_out/$T/prof_cfg3 --cfg cfg3 --steps 10 --no-cpu-baseline &&
bash tools/prof.sh gpurun_out/$T/prof_k200 --cfg k200 --steps 5 --no-cpu-baseline &&
python3 tools/kstats.py gpurun_out/$T > $O/kstats.txt 2>&1
