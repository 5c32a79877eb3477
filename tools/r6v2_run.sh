#!/bin/bash
# Round-6 (session 2): merged context row pass vs round-5's three passes.
set -o pipefail
O=gpurun_out/r6v2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; cp $O/pytest_gpu.log profiles/r6_fail_v2.log; exit 1; }
tail -1 $O/pytest_gpu.log
AB_WARMUP=50 bash tools/ab_quick.sh r6v2 "cfg3 cfg2 cfg3:sys k32 k128" ctx_r5passes || exit 1
for f in gpurun_out/ab_r6v2/*cfg3_*.log gpurun_out/ab_r6v2/*k128_*.log gpurun_out/ab_r6v2/*k32_*.log; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'ctx', round(d['decode_ctx_ms'],4))"
done
