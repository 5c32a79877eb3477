#!/usr/bin/env python3
"""Index the rocprofv3 --stats averages of the bench configurations' kernels
for bench.py's `frac_rocprof` (profiles/rocprof_index.json).

    python tools/rocprof_index.py <out.json> <cfg>=<kernel_stats.csv>,<bench.log> ...

For each configuration: the bench line of the profiled run (its kernel names,
build id and stripe count) and the rocprofv3 kernel statistics of the same
run.  encode.avg_ms = the encode kernel's average duration; decode.avg_ms =
the sum of the averages of the decode's kernels (context builder, matrix or
NTT kernels, redo), i.e. the decode step's kernel time without launch gaps.
A role whose kernel also runs in the other role (the systematic code's
encode and decode share matrix_mfma_kernel<1, 16, 4, false>) is left out:
its average would mix the two."""
import csv
import json
import sys


def kernel_avgs(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        if "qi::" not in name:
            continue
        out[name.split("qi::", 1)[1].split("(")[0]] = float(r["AverageNs"]) / 1e6
    return out


def main():
    out_path = sys.argv[1]
    idx = {"configs": {}, "build": None,
           "note": "rocprofv3 --kernel-trace --stats averages (warmup calls "
                   "included) of the kernels each bench line names; "
                   "tools/rocprof_index.py"}
    for arg in sys.argv[2:]:
        cfg, files = arg.split("=", 1)
        stats, log = files.split(",")
        line = [ln for ln in open(log) if ln.startswith("{")][-1]
        b = json.loads(line)
        avgs = kernel_avgs(stats)
        enc, dec = b["roofline"]["kernel"], b["decode_roofline"]["kernels"]
        enc_names = [n.replace(" (tail)", "").strip() for n in enc.split(" + ")]
        dec_names = [n.replace(" (tail)", "").strip() for n in dec.split(" + ")]
        rec = {"stripes": b["config"]["stripes_per_gpu"], "source": stats,
               "build": b.get("build_id")}
        shared = set(enc_names) & set(dec_names)
        for role, names in (("encode", enc_names), ("decode", dec_names)):
            if shared or not all(n in avgs for n in names):
                continue
            rec[role] = {"kernels": names, "avg_ms": sum(avgs[n] for n in names)}
        idx["configs"][cfg] = rec
        idx["build"] = b.get("build_id") or idx["build"]
    with open(out_path, "w") as f:
        json.dump(idx, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
