#!/bin/bash
# Round-6 check pass (GPU box): GPU parity suite, smoke, the default bench
# line (cfg2 + its cfg3 secondary + CPU baseline), extra bench lines and
# rocprofv3 kernel stats of the named configs.
#   bash tools/r6_check.sh <tag> [cfg...]      (default cfgs: cfg2 cfg3)
# Set R6_SKIP_TESTS=1 to skip the parity suite (A/B-only passes).
set -o pipefail
T=${1:-r6}; shift
CFGS=${*:-cfg2 cfg3}
O=gpurun_out/$T
mkdir -p $O
if [ -z "$R6_SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
fi
timeout -k 10 300 python3 bench.py > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
python3 tools/summ.py $O
for c in $CFGS; do
  [ $c = cfg2 ] && continue
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || { cat $O/bench_$c.log; exit 1; }
done
python3 tools/summ.py $O
for c in $CFGS; do
  bash tools/prof.sh $O/prof_$c --cfg $c --steps 10 --no-cpu-baseline --no-secondary || exit $?
done
python3 tools/kstats.py $O
