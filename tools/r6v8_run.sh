#!/bin/bash
# Round-6 (session 2): k <= 128 contexts with lean row pass (product) vs the merged row pass of d607308 (ctx_rowpass_r6a)
# (product) vs the square-and-multiply chain (ctx_rowpass_r6a); stage stamps
set -o pipefail
O=gpurun_out/r6v8
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; cp $O/pytest_gpu.log profiles/r6_fail_v8.log; exit 1; }
tail -1 $O/pytest_gpu.log
for a in 64,960,1024,2048 64,960,64,32768 16,48,4096,32768 128,128,128,32768; do
  QI_LIB_PATH=build/ab/ctx_ts8/libquadiron_amd.so timeout -k 10 120 python3 tools/ctx_stages8.py $a 2>/dev/null || exit 1
done > $O/stages.txt
cat $O/stages.txt
AB_WARMUP=50 bash tools/ab_quick.sh r6v8 "cfg3 cfg3p64 cfg3:sys k32 k128 cfg2" ctx_rowpass_r6a || exit 1
for f in gpurun_out/ab_r6v8/*.log; do
  python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], 'ctx', round(d['decode_ctx_ms'],4), 'dec', round(d['decode_ms'],4))"
done
