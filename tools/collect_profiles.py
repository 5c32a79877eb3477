#!/usr/bin/env python3
"""Copy a measurement pass's results (gpurun_out/<tag>, tools/r5_final.sh)
into tracked profiles:
    python tools/collect_profiles.py <tag> <prefix> [main|pmc]
main: <prefix>_bench[_<cfg>].json (each bench line), <prefix>_<cfg>_kernel_
stats.csv / _kernel_trace.csv (qi dispatches only), the GPU suite and smoke
logs, host rates, and profiles/rocprof_index.json over those traces;
pmc: profiles/pmc_roofline.json from the pass's per-configuration records."""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")


def last_line(path):
    return [ln for ln in open(path) if ln.startswith("{")][-1]


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    part = sys.argv[3] if len(sys.argv) > 3 else "main"
    src = os.path.join(ROOT, "gpurun_out", tag)
    if part == "pmc":
        out = {"configs": {}}
        for f in sorted(glob.glob(os.path.join(src, "pmc_*", "pmc_roofline.json"))):
            d = json.load(open(f))
            out["configs"].update(d.get("configs", d))
        with open(os.path.join(P, "pmc_roofline.json"), "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
        print("pmc configs:", sorted(out["configs"]))
        return
    for f in sorted(glob.glob(os.path.join(src, "bench*.log"))):
        name = os.path.basename(f)[:-4].replace("bench", prefix + "_bench")
        with open(os.path.join(P, name + ".json"), "w") as o:
            o.write(last_line(f))
    for name in ("pytest_gpu.log", "smoke.log"):
        if os.path.exists(os.path.join(src, name)):
            shutil.copy(os.path.join(src, name),
                        os.path.join(P, f"{prefix}_{name[:-4]}.txt"))
    if os.path.exists(os.path.join(src, "host_rate.json")):
        shutil.copy(os.path.join(src, "host_rate.json"), os.path.join(P, f"{prefix}_host_rate.json"))
    args = []
    for d in sorted(glob.glob(os.path.join(src, "prof_*"))):
        cfg = os.path.basename(d)[5:]
        stats = os.path.join(P, f"{prefix}_{cfg}_kernel_stats.csv")
        trace = os.path.join(P, f"{prefix}_{cfg}_kernel_trace.csv")
        shutil.copy(os.path.join(d, "run_kernel_stats.csv"), stats)
        rows = list(csv.reader(open(os.path.join(d, "run_kernel_trace.csv"))))
        with open(trace, "w", newline="") as o:
            w = csv.writer(o, quoting=csv.QUOTE_ALL)
            w.writerow(rows[0])
            ki = rows[0].index("Kernel_Name")
            w.writerows(r for r in rows[1:] if "qi::" in r[ki])
        log = os.path.join(P, f"{prefix}_{cfg}_rocprof_bench.json")
        with open(log, "w") as o:
            o.write(last_line(os.path.join(d, "bench.log")))
        args.append(f"{cfg}={os.path.relpath(stats, ROOT)},{os.path.relpath(log, ROOT)}")
    if args:
        subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "rocprof_index.py"),
                               os.path.join(P, "rocprof_index.json")] + args, cwd=ROOT)


if __name__ == "__main__":
    main()
