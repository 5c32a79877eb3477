#!/bin/bash
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
  for v in 0 1 2; do
    QI_MATK=$v timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline --steps 20 > $O/cfg3_m${v}_$i.log 2>&1 || exit $?
  done
  QI_MATK=1 QI_LIB_PATH=build/ab/pw3/libquadiron_amd.so timeout -k 10 300 python3 bench.py --cfg cfg3 --no-cpu-baseline --steps 20 > $O/cfg3_pw3_$i.log 2>&1 || exit $?
  QI_MATK=2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --systematic > $O/sys_m2_$i.log 2>&1 || exit $?
  QI_MATK=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --systematic > $O/sys_m0_$i.log 2>&1 || exit $?
done
