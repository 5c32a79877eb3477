#!/bin/bash
# Round-4 check pass (GPU box): GPU parity suite, smoke, bench lines and
# rocprofv3 kernel stats of the named configs.
#   bash tools/r4_check.sh <tag> [cfg...]      (default cfgs: cfg2 cfg3)
set -o pipefail
T=${1:-r4}; shift
CFGS=${*:-cfg2 cfg3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
for c in $CFGS; do
  timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline > $O/bench_$c.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1]); print('$c', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), d['roundtrip_ok'])"
done
for c in $CFGS; do
  bash tools/prof.sh $O/prof_$c --cfg $c --steps 10 --no-cpu-baseline || exit $?
done
