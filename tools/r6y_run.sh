#!/bin/bash
# Round 6: KS = 40 launches sized for ~1024 blocks (k600: 16 column ranges,
# 1280 blocks = five full rounds) vs the product's ~512 (9 ranges, 720).
set -o pipefail
O=gpurun_out/r6y; mkdir -p $O
QI_LIB_PATH=build/ab/target40/libquadiron_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "batch_vs_oracle and (600-1400 or 385 or 640)" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in prod t40; do
    L=""; [ $v = t40 ] && L=build/ab/target40/libquadiron_amd.so
    for c in "k600" "k600 --systematic"; do
      t=$(echo $c | tr -d ' -')
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 30 > $O/${t}_${v}_$i.log 2>&1 || { cat $O/${t}_${v}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${t}_${v}_$i.log').read().strip().splitlines()[-1]); print('$t $v $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
    done
  done
done
