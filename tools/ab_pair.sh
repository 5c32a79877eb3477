#!/bin/bash
# A/B on the GPU box: parity on the product build, then bench lines of the
# product build and each build/ab/<variant> alternating (2 rounds):
#   bash tools/ab_pair.sh <tag> "<variant>..." <cfg>...
set -o pipefail
T=$1; V=$2; shift 2
O=gpurun_out/ab_$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_main.log 2>&1 || exit $?
for i in 1 2; do
  for v in main $V; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    for c in "$@"; do
      QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --cfg $c > $O/${v}_${c}_$i.log 2>&1 || exit $?
    done
  done
done
