#!/bin/bash
# Round-6 (session 2): k <= 128 contexts with the wave roles rotated by the
# stripe (product) vs fixed (ctx_norot)
set -o pipefail
O=gpurun_out/r6v3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "golden or cabi or batch or ctx or ids" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; cp $O/pytest_gpu.log profiles/r6_fail_v3.log; exit 1; }
tail -1 $O/pytest_gpu.log
AB_WARMUP=50 bash tools/ab_quick.sh r6v3 "cfg3 cfg3p64 cfg3:sys k32 k128 cfg2" ctx_norot || exit 1
for f in gpurun_out/ab_r6v3/*.log; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], 'ctx', round(d['decode_ctx_ms'],4), 'dec', round(d['decode_ms'],4))"
done
