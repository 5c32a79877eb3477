#!/bin/bash
# Alternate bench runs of the product library and variants (GPU box):
#   bash tools/ab_bench.sh <variant>... ; results in gpurun_out/ab_<name>_<i>.log
# BENCH_ARGS (env) is passed to every run.
O=gpurun_out
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS > $O/ab_main_$i.log 2>&1 || exit $?
  for v in "$@"; do
    QI_LIB_PATH=build/ab/$v/libquadiron_amd.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS > $O/ab_${v}_$i.log 2>&1 || exit $?
  done
done
