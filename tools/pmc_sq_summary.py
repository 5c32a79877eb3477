#!/usr/bin/env python3
"""Summarise a tools/pmc_sq.sh pass per kernel (summed over its launches):
instructions per wave (VALU, SALU, LDS), wave-cycle fractions (waitcnt
parked, issue-stalled, VALU active) and the launches' mean duration from
GRBM_GUI_ACTIVE / 8 XCDs at the clock the pass ran.
    python3 tools/pmc_sq_summary.py <outdir> [name substring]"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][:70]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        calls[k].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
sub = sys.argv[2] if len(sys.argv) > 2 else ''
for k, v in sorted(acc.items()):
    if sub not in k or 'at::' in k:
        continue
    w = v['SQ_WAVES'] or 1
    wc = v['SQ_WAVE_CYCLES'] or 1
    n = max(1, len(calls[k]))
    print('%-70s n=%d valu/w %.0f salu/w %.0f lds/w %.0f | wait_any %.2f wait_inst %.2f '
          'valu_act %.2f | gui/8/call %.0f' % (
              k, n, v['SQ_INSTS_VALU'] / w, v['SQ_INSTS_SALU'] / w, v['SQ_INSTS_LDS'] / w,
              v['SQ_WAIT_ANY'] / wc, v['SQ_WAIT_INST_ANY'] / wc,
              v['SQ_ACTIVE_INST_VALU'] / wc, v['GRBM_GUI_ACTIVE'] / 8 / n))
