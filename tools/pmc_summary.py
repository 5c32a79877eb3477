#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-kernel averages per dispatch."""
import collections
import csv
import os
import sys

d = sys.argv[1]
tot = collections.defaultdict(dict)
for f in ["sq", "sq2", "fetch", "write"]:
    p = os.path.join(d, f + "_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"].split("(")[0][:40]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
    for name, dd in agg.items():
        if "qi::" not in name:
            continue
        for k, v in dd.items():
            tot[name][k] = v / len(disp[name])
for name, dd in tot.items():
    w = dd.get("SQ_WAVES", 1)
    wc = dd.get("SQ_WAVE_CYCLES", 1)
    print(name)
    print("  per-wave: VALU %.0f SALU %.0f VMEM_RD %.1f VMEM_WR %.1f" % (
        dd.get("SQ_INSTS_VALU", 0) / w, dd.get("SQ_INSTS_SALU", 0) / w,
        dd.get("SQ_INSTS_VMEM_RD", 0) / w, dd.get("SQ_INSTS_VMEM_WR", 0) / w))
    print("  wave-cycle share: active %.2f wait_inst %.2f wait_any %.2f" % (
        dd.get("SQ_ACTIVE_INST_ANY", 0) / wc, dd.get("SQ_WAIT_INST_ANY", 0) / wc,
        dd.get("SQ_WAIT_ANY", 0) / wc))
    g = dd.get("GRBM_GUI_ACTIVE", 0) / 8
    if g:
        print("  cycles/XCD %.3g  VALU busy (4 cyc/instr) %.2f" % (
            g, dd.get("SQ_INSTS_VALU", 0) * 4 / (1024 * g)))
    if "FETCH_SIZE" in dd:
        print("  FETCH_SIZE x2 %.3g B  WRITE_SIZE %.3g B" % (
            dd["FETCH_SIZE"] * 1024 * 2, dd.get("WRITE_SIZE", 0) * 1024))

# machine-readable summary (bench.py reads profiles/pmc_traffic.json):
#   python tools/pmc_summary.py <dir> --json <out.json>
if "--json" in sys.argv:
    import json
    out = {"source": d, "correction": "FETCH_SIZE x2 (gfx950, "
           "MI355X_MICROARCH.md HBM section), WRITE_SIZE as reported; "
           "counters in KiB", "kernels": {}}
    for name, dd in tot.items():
        if "FETCH_SIZE" not in dd:
            continue
        rd = dd["FETCH_SIZE"] * 1024 * 2
        wr = dd.get("WRITE_SIZE", 0) * 1024
        out["kernels"][name] = {"read_bytes_per_launch": rd,
                                "write_bytes_per_launch": wr,
                                "hbm_bytes_per_launch": rd + wr}
        if "encode_fnt_kernel" in name:
            out["encode_bytes_per_launch"] = rd + wr
        if "matrix_kernel" in name:
            out["decode_bytes_per_launch"] = rd + wr
    with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
        json.dump(out, f, indent=1)
