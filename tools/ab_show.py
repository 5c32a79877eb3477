import glob, json, sys
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f"{f:34s} value {d['value']:8.1f} enc {d['encode_kernel_ms']:.3f} dec {d['decode_ms']:.3f} ok {d['roundtrip_ok']}")
    except Exception as e:
        print(f, "ERR", e)
