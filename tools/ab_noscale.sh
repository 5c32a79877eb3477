#!/bin/bash
set -o pipefail
O=gpurun_out/ab_noscale
mkdir -p $O
for i in 1 2; do
  for v in main noscale; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    QI_ENC_MATRIX=1 QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --cfg cfg3 > $O/${v}_matcfg3_$i.log 2>&1 || true
  done
done
