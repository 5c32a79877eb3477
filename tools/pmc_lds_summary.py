#!/usr/bin/env python3
"""Summarise a tools/pmc_lds.sh pass per kernel: wave-cycle fractions
(waitcnt, issue stalls, VALU active, LDS active) and LDS bank-conflict
cycles per LDS instruction.
    python3 tools/pmc_lds_summary.py <outdir>"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + '/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        acc[r['Kernel_Name'][:48]][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in sorted(acc.items()):
    if 'qi::' not in k:
        continue
    wc = v['SQ_WAVE_CYCLES'] or 1
    print('%-48s valu %.3g lds %.3g | wait_any %.2f wait_inst %.2f valu_active %.2f '
          'lds_active %.2f lds_conflict/inst %.2f' % (
              k, v['SQ_INSTS_VALU'], v['SQ_INSTS_LDS'], v['SQ_WAIT_ANY'] / wc,
              v['SQ_WAIT_INST_ANY'] / wc, v['SQ_ACTIVE_INST_VALU'] / wc,
              v['SQ_LDS_IDX_ACTIVE'] / wc,
              v['SQ_LDS_BANK_CONFLICT'] / max(1, v['SQ_INSTS_LDS'])))
