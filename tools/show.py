#!/usr/bin/env python3
"""Print the bench lines / logs of a gpurun_out/<tag> directory."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.log"))):
    lines = [x for x in open(f, errors="replace") if x.startswith("{")]
    if lines:
        o = json.loads(lines[-1])
        print(f"{os.path.basename(f):28s} {o['value']:8.1f} GB/s  enc {o['encode_kernel_ms']:.4f} ms"
              f"  dec {o['decode_ms']:.4f} ms  ok={o['roundtrip_ok']}")
    else:
        txt = [x.strip() for x in open(f, errors="replace") if x.strip() and "amdgpu.ids" not in x]
        print(f"{os.path.basename(f):28s} " + " | ".join(txt[-3:])[:300])
