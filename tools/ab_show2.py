#!/usr/bin/env python3
"""Table of bench logs in a directory: value, encode ms, decode ms."""
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print("%-22s %8.1f GB/s  enc %6.3f ms  dec %6.3f ms" % (
            os.path.basename(f)[:-4], d["value"], d["encode_kernel_ms"], d["decode_ms"]))
    except Exception as e:
        print(os.path.basename(f), "ERR", open(f).read()[-300:])
