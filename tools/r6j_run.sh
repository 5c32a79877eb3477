#!/bin/bash
# Round 6: decode contexts from the ids on a low-priority second stream beside
# a high-priority encode (bench.py --ctx-stream 2) vs the serial step (0) and
# the round-5 equal-priority overlap (1).
set -o pipefail
O=gpurun_out/r6j; mkdir -p $O
for i in 1 2 3; do
  for cs in 0 2 1; do
    for c in cfg3 cfg2; do
      wu=30; [ $c = cfg3 ] && wu=60
      timeout -k 10 300 python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup $wu --ctx-stream $cs > $O/${c}_cs${cs}_$i.log 2>&1 || { cat $O/${c}_cs${cs}_$i.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/${c}_cs${cs}_$i.log').read().strip().splitlines()[-1]); print('$c cs$cs $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
    done
  done
done
