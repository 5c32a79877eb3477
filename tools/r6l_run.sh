#!/bin/bash
# Round 6: where the two-region KS = 40 decode's time goes -- the product vs
# ab_lib/oneload.so (one load per row, every row read through the region-1
# descriptor: the same bytes, wrong output, timing only),
# and kernel stats of the k600 systematic and non-systematic steps.
set -o pipefail
O=gpurun_out/r6l; mkdir -p $O
for i in 1 2; do
  for lib in new oneload; do
    L=""; [ $lib = oneload ] && L=ab_lib/oneload.so
    QI_LIB_PATH=$L timeout -k 10 300 python3 bench.py --cfg k600 --systematic --no-cpu-baseline --no-secondary --warmup 20 > $O/k600s_${lib}_$i.log 2>&1
    rc=$?  # (oneload: the round trip fails by design, exit 1)
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && [ $lib = oneload ]; } || { cat $O/k600s_${lib}_$i.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/k600s_${lib}_$i.log').read().strip().splitlines()[-1]); print('k600s $lib $i', round(d['value'],1), 'enc', round(d['encode_kernel_ms'],4), 'dec', round(d['decode_ms'],4), 'ctx', round(d['decode_ctx_ms'],4), d['roundtrip_ok'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "k600 --systematic" "k600"; do
  t=$(echo $c | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$t -o run -- python3 bench.py --cfg $c --no-cpu-baseline --no-secondary --warmup 5 --steps 10 > $O/prof_$t.log 2>&1 || { tail -20 $O/prof_$t.log; exit 1; }
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:6]: print(x['Name'][:70], x['Calls'], round(float(x['AverageNs'])/1e3,1),'us')
"; done
