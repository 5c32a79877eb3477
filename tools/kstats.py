#!/usr/bin/env python3
"""Print the qi:: kernels of a rocprofv3 --stats csv (or every csv under a
directory): name, calls, average / min duration in microseconds."""
import csv
import glob
import os
import sys

paths = []
for a in sys.argv[1:]:
    paths += (sorted(glob.glob(os.path.join(a, "**", "*kernel_stats.csv"), recursive=True))
              if os.path.isdir(a) else [a])
for p in paths:
    print(p)
    for r in csv.DictReader(open(p)):
        n = r["Name"]
        if "qi::" not in n:
            continue
        print(f"  {n.split('(')[0][:60]:60s} {int(r['Calls']):6d} "
              f"avg {float(r['AverageNs']) / 1e3:9.2f} us  min {float(r['MinNs']) / 1e3:9.2f} us")
