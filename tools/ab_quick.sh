#!/bin/bash
# Quick A/B on the GPU box: bench lines of the product build and of
# build/ab/<variant> libraries, alternating, for the given configs
# (<cfg>:sys = the systematic code).
#   bash tools/ab_quick.sh <tag> "<cfgs>" <variant>...
# AB_WARMUP=<n>: warmup steps (default bench.py's 3; short-step configs such
# as cfg3 need ~50 for the GPU clock to settle, tools/ramp.py)
set -o pipefail
T=$1; CFGS=$2; shift 2
O=gpurun_out/ab_$T
mkdir -p $O
for i in 1 2 3; do
  for v in main "$@"; do
    L=quadiron_amd/libquadiron_amd.so; [ $v != main ] && L=build/ab/$v/libquadiron_amd.so
    for c in $CFGS; do
      F="--cfg ${c%:sys}"; [ "${c%:sys}" != "$c" ] && F="$F --systematic"
      QI_LIB_PATH=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 ${AB_WARMUP:+--warmup $AB_WARMUP} $F $AB_ARGS > $O/${v}_${c}_$i.log 2>&1
      rc=$?
      # a probe variant (results deliberately wrong) exits 3 after its line;
      # anything else (no bench line, a fault, a time limit) ends the run
      grep -q '^{' $O/${v}_${c}_$i.log && { [ $rc -eq 0 ] || [ $rc -eq 3 ]; } || { cat $O/${v}_${c}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${c}_$i.log').read().strip().splitlines()[-1]); print('$v $c $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), d['roundtrip_ok'])"
    done
  done
done
