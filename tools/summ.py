#!/usr/bin/env python3
"""Summarise bench JSON lines and the pytest tail of a gpurun_out/<tag> dir."""
import glob
import json
import os
import sys

d = sys.argv[1]
p = os.path.join(d, "pytest_gpu.log")
if os.path.exists(p):
    lines = open(p).read().strip().splitlines()
    print(lines[-1] if lines else "(empty pytest log)")
    for ln in lines:
        if "FAILED" in ln or "Error" in ln[:80]:
            print("  ", ln[:200])
for f in sorted(glob.glob(os.path.join(d, "bench*.log"))):
    js = [ln for ln in open(f) if ln.startswith("{")]
    if not js:
        print(os.path.basename(f), "NO JSON:", open(f).read()[-400:])
        continue
    j = json.loads(js[0])
    c = j.get("cpu_baseline") or {}
    print(f"{os.path.basename(f):18s} {j['value']:8.1f} GB/s  enc {j['encode_kernel_ms']:.3f} ms"
          f"  dec {j['decode_ms']:.3f} ms  frac {j['roofline']['frac']:.3f}"
          f"  ok {j['roundtrip_ok']}"
          + (f"  cpu {c['value']:.2f} (1c {c['one_core']['value']:.2f})" if c else ""))
