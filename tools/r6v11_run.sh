#!/bin/bash
# Round-6 (session 2): k > 128 contexts with the lean packing pass (product)
# vs the previous one (ctx_pack_r6a)
set -o pipefail
O=gpurun_out/r6v11
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; cp $O/pytest_gpu.log profiles/r6_fail_v11.log; exit 1; }
tail -1 $O/pytest_gpu.log
AB_WARMUP=30 bash tools/ab_quick.sh r6v11 "k256 k200 k300 k384 k600 k300:sys k600:sys" ctx_pack_r6a || exit 1
for f in gpurun_out/ab_r6v11/*.log; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], 'ctx', round(d['decode_ctx_ms'],4), 'dec', round(d['decode_ms'],4))"
done
