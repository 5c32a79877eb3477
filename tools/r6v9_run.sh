#!/bin/bash
# Round-6 (session 2): stage stamps of the product k <= 128 context; the Q
# chains one coefficient per step at 33 <= k <= 64 (ctx_q1step) vs the
# product's four
set -o pipefail
O=gpurun_out/r6v9
mkdir -p $O
for a in 64,960,1024,2048 64,960,64,32768 16,48,4096,32768 128,128,128,32768; do
  QI_LIB_PATH=build/ab/ctx_ts8/libquadiron_amd.so timeout -k 10 120 python3 tools/ctx_stages8.py $a 2>/dev/null || exit 1
done > $O/stages.txt
cat $O/stages.txt
AB_WARMUP=50 bash tools/ab_quick.sh r6v9 "cfg3 cfg3p64 cfg3:sys" ctx_q1step || exit 1
for f in gpurun_out/ab_r6v9/*.log; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], 'ctx', round(d['decode_ctx_ms'],4), 'dec', round(d['decode_ms'],4))"
done
