#!/bin/bash
# A/B timing only (no parity): bench lines of build/ab/<variant> libraries
# against the product build, alternating twice.  Variants may compute wrong
# results on purpose (timing probes), so a failed round-trip check (exit 3)
# is recorded, not fatal; any other failure stops the run.
#   bash tools/ab_run.sh <tag> "<bench args>" <env> <variant>...
T=$1; ARGS=$2; ENVS=$3; shift 3
O=gpurun_out/abr_$T
mkdir -p $O
for i in 1 2; do
  for v in main "$@"; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    env $ENVS QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 10 $ARGS > $O/${v}_$i.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && [ $rc -ne 3 ] && exit $rc
  done
done
exit 0
