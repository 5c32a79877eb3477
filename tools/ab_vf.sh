#!/bin/bash
# A/B of the MFMA VGPR-form build (build/ab/vf) across configs and encode paths.
set -o pipefail
O=gpurun_out/abvf
mkdir -p $O
run() {  # name, lib, env, args
  env $3 QI_LIB_PATH=$2 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 $4 > $O/$1.log 2>&1
}
for i in 1 2; do
  for v in main vf; do
    L=quadiron_amd/libquadiron_amd.so; [ $v = vf ] && L=build/ab/vf/libquadiron_amd.so
    run ${v}_cfg2_$i $L "" "" &&
    run ${v}_sys_$i $L "" "--systematic" &&
    run ${v}_cfg3_$i $L "" "--cfg cfg3" &&
    run ${v}_matcfg3_$i $L "QI_ENC_MATRIX=1" "--cfg cfg3" &&
    run ${v}_matcfg2_$i $L "QI_ENC_MATRIX=1" "" || exit $?
  done
done
