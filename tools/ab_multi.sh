#!/bin/bash
# A/B: product build vs several build/ab/<variant> libraries (GPU box).
#   bash tools/ab_multi.sh <tag> <variant>...
# Parity tests run on every variant (matrix encode forced), then the bench
# lines alternate over the builds twice.
set -o pipefail
T=$1; shift
O=gpurun_out/ab_$T
mkdir -p $O
for v in "$@"; do
  QI_ENC_MATRIX=1 QI_LIB_PATH=build/ab/$v/libquadiron_amd.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || exit $?
done
run() {  # name, lib, env, args
  env $3 QI_LIB_PATH=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $4 > $O/$1.log 2>&1
}
for i in 1 2; do
  for v in main "$@"; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    run ${v}_cfg2_$i $L "" "" &&
    run ${v}_sys_$i $L "" "--systematic" &&
    run ${v}_cfg3_$i $L "" "--cfg cfg3" &&
    run ${v}_matcfg3_$i $L "QI_ENC_MATRIX=1" "--cfg cfg3" || exit $?
  done
done
