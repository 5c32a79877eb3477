#!/bin/bash
# Round 6: systematic 384 < k <= 640 decodes on the matrix cores (KS = 40,
# two source regions) and the whole-tile systematic contexts in row chunks
# over several blocks per stripe -- parity, then the steps vs ab_lib/old.so
# (the library before the change: the NTT engine's decode at k > 384, one
# context block per systematic stripe).
set -o pipefail
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_kernel_names.py \
  -k "batch_vs_oracle and (385 or 500 or 600 or 640 or 300 or 320 or 384 or 200 or 129 or 130) or unaligned or reported_kernels or cabi or golden" \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2; do
  for lib in new old; do
    for c in "k600 --systematic" "k384 --systematic" "k300 --systematic" "k200 --systematic" "k600" "k300"; do
      L=""; [ $lib = old ] && L=ab_lib/old.so
      t=$(echo $c | tr -d ' -')
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 20 > $O/${t}_${lib}_$i.log 2>&1 || { cat $O/${t}_${lib}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${t}_${lib}_$i.log').read().strip().splitlines()[-1]); print('$t $lib $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
    done
  done
done
