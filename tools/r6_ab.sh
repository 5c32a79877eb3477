#!/bin/bash
# Round-6 quick A/B pass (GPU box): bench lines of the named configs with 30+
# warmup steps (60 at cfg3, whose steps are ~1 ms), each twice, plus the PMC
# roofline record of the configs listed in PMC (e.g. PMC="k256 256").
#   bash tools/r6_ab.sh <tag> cfg...
set -o pipefail
T=${1:-r6ab}; shift
O=gpurun_out/$T
mkdir -p $O
wu() { case $1 in cfg3|cfg3p64|cfg1) echo 60;; *) echo 30;; esac; }
for rep in 1 2; do
  for c in "$@"; do
    timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup $(wu $c) > $O/bench_${c}_$rep.log 2>&1 || { cat $O/bench_${c}_$rep.log; exit 1; }
  done
done
python3 tools/summ.py $O
if [ -n "$PMC" ]; then
  set -- $PMC
  bash tools/pmc_roofline.sh $O/pmc_$1 $1 $2 --cfg $1 --no-secondary || exit $?
  python3 -c "import json; d=json.load(open('$O/pmc_$1/pmc_roofline.json')); print(json.dumps(d, indent=1)[:1500])"
fi
