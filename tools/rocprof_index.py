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
import os
import sys


def kernel_avgs(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        if "qi::" not in name:
            continue
        out[name.split("qi::", 1)[1].split("(")[0]] = float(r["AverageNs"]) / 1e6
    return out


def kname(name):
    return name.split("qi::", 1)[1].split("(")[0] if "qi::" in name else None


def timed_avgs(trace, enc_names, dec_names, steps):
    """Per-role kernel time of the last `steps` steps from the kernel trace:
    a step is one dispatch of the context builder (dec_names[0]); the qi
    dispatch right before it that names an encode kernel is that step's
    encode, the qi dispatches right after it that name decode kernels its
    decode.  (The warmup steps ramp the GPU clock; the stats average over
    every call mixes them in, and a kernel that serves both roles -- the
    operand-stationary kernel at k > 128 -- cannot be split by name.)"""
    rows = sorted((int(r["Dispatch_Id"]), kname(r["Kernel_Name"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                  for r in csv.DictReader(open(trace)))
    qi = [(n, d) for _, n, d in rows if n]
    ctx = dec_names[0]
    enc, dec = [], []
    for i, (n, _) in enumerate(qi):
        if n != ctx:
            continue
        e = qi[i - 1][1] if i > 0 and qi[i - 1][0] in enc_names else None
        d, j = 0.0, i + 1
        while j < len(qi) and qi[j][0] in dec_names[1:] and qi[j][0] != ctx:
            d += qi[j][1]
            j += 1
            if j - i - 1 >= len(dec_names) - 1:
                break
        enc.append(e)
        dec.append(qi[i][1] + d)
    enc, dec = enc[-steps:], dec[-steps:]
    out = {}
    if enc and all(e is not None for e in enc):
        out["encode"] = sum(enc) / len(enc)
    if dec:
        out["decode"] = sum(dec) / len(dec)
    return out


def main():
    out_path = sys.argv[1]
    idx = {"configs": {}, "build": None,
           "note": "rocprofv3 --kernel-trace durations of the kernels each "
                   "bench line names, averaged over the run's timed steps "
                   "(avg_ms; avg_ms_all_calls: the --stats average over every "
                   "call, warmup included); tools/rocprof_index.py"}
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
        trace = stats.replace("kernel_stats.csv", "kernel_trace.csv")
        timed = {}
        if os.path.exists(trace):
            timed = timed_avgs(trace, enc_names, dec_names, int(b["steps"]))
            rec["source_timed"] = trace
        shared = set(enc_names) & set(dec_names)
        for role, names in (("encode", enc_names), ("decode", dec_names)):
            r = {"kernels": names}
            if not shared and all(n in avgs for n in names):
                r["avg_ms_all_calls"] = sum(avgs[n] for n in names)
            if role in timed:
                r["avg_ms"] = timed[role]  # the timed steps only
            elif "avg_ms_all_calls" in r:
                r["avg_ms"] = r["avg_ms_all_calls"]
            if "avg_ms" in r:
                rec[role] = r
        idx["configs"][cfg] = rec
        idx["build"] = b.get("build_id") or idx["build"]
    with open(out_path, "w") as f:
        json.dump(idx, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
