#!/usr/bin/env python3
"""Tabulate bench JSON lines of A/B runs: python3 tools/ab_lines.py <dir>..."""
import glob
import json
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(d + "/*.log")):
        try:
            j = json.loads(open(f).read().strip().splitlines()[-1])
            print(f"{f:40s} {j['value']:8.1f} GB/s enc {j['encode_kernel_ms']:.3f} "
                  f"dec {j['decode_ms']:.3f} ok {j['roundtrip_ok']}")
        except Exception:
            pass
