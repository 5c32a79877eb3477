#!/bin/bash
# Alternate bench runs with different bench.py argument sets (GPU box):
#   bash tools/ab_args.sh "<args A>" "<args B>" ... ; gpurun_out/ab_argN_i.log
O=gpurun_out
mkdir -p $O
for i in 1 2; do
  n=0
  for a in "$@"; do
    n=$((n+1))
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $a > $O/ab_arg${n}_$i.log 2>&1 || exit $?
  done
done
