#!/bin/bash
# Round 6: systematic decodes at KS = 16 / 20 with two row blocks per wave
# (the one-load staging left the registers for it) vs ab_lib/prev.so.
set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "batch_vs_oracle or unaligned or cabi or golden" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for lib in new prev; do
    for c in "k200 --systematic" "k300 --systematic" "k256 --systematic" "k384 --systematic"; do
      L=""; [ $lib = prev ] && L=ab_lib/prev.so
      t=$(echo $c | tr -d ' -')
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 20 > $O/${t}_${lib}_$i.log 2>&1 || { cat $O/${t}_${lib}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${t}_${lib}_$i.log').read().strip().splitlines()[-1]); print('$t $lib $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'], d['decode_roofline']['kernels'])"
    done
  done
done
