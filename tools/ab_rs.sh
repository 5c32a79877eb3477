#!/bin/bash
# A/B: product build vs build/ab/<variant> on the encode-heavy configs;
# parity tests on the variant first (matrix encode forced and not).
set -o pipefail
V=${1:-rs}
O=gpurun_out/ab_$V
mkdir -p $O
VL=build/ab/$V/libquadiron_amd.so
QI_LIB_PATH=$VL timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
QI_ENC_MATRIX=1 QI_LIB_PATH=$VL timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_mat.log 2>&1 || exit $?
run() {  # name, lib, env, args
  env $3 QI_LIB_PATH=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $4 > $O/$1.log 2>&1
}
for i in 1 2; do
  for v in main $V; do
    L=quadiron_amd/libquadiron_amd.so; [ $v = $V ] && L=$VL
    run ${v}_cfg2_$i $L "" "" &&
    run ${v}_sys_$i $L "" "--systematic" &&
    run ${v}_cfg3_$i $L "" "--cfg cfg3" &&
    run ${v}_matcfg3_$i $L "QI_ENC_MATRIX=1" "--cfg cfg3" &&
    run ${v}_matcfg2_$i $L "QI_ENC_MATRIX=1" "" || exit $?
  done
done
