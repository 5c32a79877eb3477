#!/bin/bash
# Round 6: operand-stationary image row pitch (64 x NST columns + 8 / 16 /
# 24 / 48 bytes; the product is + 16) -- parity of each variant, then the
# steps.  Variants: build/ab/pitch<P> (tools/ab/os_pitch<P>.patch).
set -o pipefail
O=gpurun_out/r6x; mkdir -p $O
for v in 8 24; do
  QI_LIB_PATH=build/ab/pitch$v/libquadiron_amd.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "batch_vs_oracle and (600-1400 or 300-212 or 64-960 or 200-56 or 385)" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
for i in 1 2; do
  for v in 16 8 24; do
    L=""; [ $v != 16 ] && L=build/ab/pitch$v/libquadiron_amd.so
    for c in k600 k300 k128 cfg3; do
      wu=30; [ $c = cfg3 ] && wu=60
      QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup $wu > $O/${c}_p${v}_$i.log 2>&1 || { cat $O/${c}_p${v}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_p${v}_$i.log').read().strip().splitlines()[-1]); print('$c p$v $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
    done
  done
done
