#!/bin/bash
# Round 6: SQ passes over the k600 bench (the KS = 40 decode), each its own
# rocprofv3 run: instruction mix / waits, then MFMA busy and LDS conflicts.
set -o pipefail
O=gpurun_out/${1:-r6g}
mkdir -p $O
bash tools/pmc_sq.sh $O/sq python3 bench.py --cfg k600 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary || exit $?
python3 tools/pmc_sq_summary.py $O/sq
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/mf -o mf \
  -- python3 $R/bench.py --cfg k600 --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > $R/$O/mf.log 2>&1 || exit $?
cd $R
python3 - $O/mf <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); calls = defaultdict(set)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][:60]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        calls[k].add(r.get('Dispatch_Id', ''))
for k, v in acc.items():
    if 'qi::' not in k: continue
    n = max(1, len(calls[k])); gui = v['GRBM_GUI_ACTIVE'] / 8 / n
    print(k, 'n', n, 'gui/8', round(gui), 'mfma_busy/(1024 SIMD x gui)', round(v['SQ_VALU_MFMA_BUSY_CYCLES'] / n / (1024 * gui), 3),
          'lds_conflict/lds_active', round(v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_LDS_IDX_ACTIVE']), 3),
          'wait_inst_lds/wave', round(v['SQ_WAIT_INST_LDS'] / max(1, v['SQ_WAVES'])))
PY
