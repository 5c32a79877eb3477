#!/bin/bash
# Round 6: non-systematic 384 < k <= 640 encodes on the matrix cores
# (Vandermonde generator, KS = 40) vs the NTT engine: k500 (R = 800 rows,
# n = 1024) and k600 (R = 2000, n = 2048).  Variant: build/ab/gen640.
set -o pipefail
O=gpurun_out/r6z; mkdir -p $O
QI_LIB_PATH=build/ab/gen640/libquadiron_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "batch_vs_oracle and (600-1400 or 385 or 640 or 500)" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in prod gen; do
    L=""; [ $v = gen ] && L=build/ab/gen640/libquadiron_amd.so
    for c in k500 k600; do
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 30 > $O/${c}_${v}_$i.log 2>&1 || { cat $O/${c}_${v}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_${v}_$i.log').read().strip().splitlines()[-1]); print('$c $v $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'], d['roofline']['kernel'])"
    done
  done
done
