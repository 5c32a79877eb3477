#!/bin/bash
# Round 6: chunk rows written column-scaled (no multiplies in the packing pass) -- the
# GPU
# suite, then the steps vs ab_lib/prev.so.
set -o pipefail
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for lib in new prev; do
    for c in "k256" "k200" "k300" "k384" "k600" "k300 --systematic"; do
      L=""; [ $lib = prev ] && L=ab_lib/prev.so
      t=$(echo $c | tr -d ' -')
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 30 > $O/${t}_${lib}_$i.log 2>&1 || { cat $O/${t}_${lib}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${t}_${lib}_$i.log').read().strip().splitlines()[-1]); print('$t $lib $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
    done
  done
done
