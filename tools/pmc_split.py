#!/usr/bin/env python3
"""tools/pmc_pipe.sh output, per kernel *role*: dispatches of one kernel name
are split by their MFMA instructions per wave (the same instantiation runs
the encode generator and the decode matrices).  python3 tools/pmc_split.py <dir>"""
import collections
import csv
import sys

d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in ["p1", "p2", "p3"]:
    for r in csv.DictReader(open(f"{d}/{f}_counter_collection.csv")):
        if "qi::" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"].split("(")[0][5:50]
groups = collections.defaultdict(list)
for k, dd in per.items():
    sig = round(dd.get("SQ_INSTS_MFMA", 0) / max(1, dd.get("SQ_WAVES", 1)))
    groups[(names[k], sig)].append(dd)
for (name, sig), lst in sorted(groups.items()):
    dd = {c: sum(x.get(c, 0) for x in lst) / len(lst) for c in lst[0]}
    w = dd.get("SQ_WAVES", 1)
    wc = dd.get("SQ_WAVE_CYCLES", 1)
    g = dd.get("GRBM_GUI_ACTIVE", 0) / 8
    sc = g * 1024 if g else 1
    print(f"{name} [mfma/wave {sig}] x{len(lst)}")
    print("  per wave: VALU %.0f MFMA %.0f LDS %.0f SALU %.0f VMEM_WR %.0f" % (
        dd.get("SQ_INSTS_VALU", 0) / w, dd.get("SQ_INSTS_MFMA", 0) / w,
        dd.get("SQ_INSTS_LDS", 0) / w, dd.get("SQ_INSTS_SALU", 0) / w,
        dd.get("SQ_INSTS_VMEM_WR", 0) / w))
    print("  wave-cycle shares: active %.2f (valu %.2f lds %.2f vmem %.2f sca %.2f) "
          "wait_inst %.2f (lds %.2f) wait_any %.2f" % (
              dd.get("SQ_ACTIVE_INST_ANY", 0) / wc, dd.get("SQ_ACTIVE_INST_VALU", 0) / wc,
              dd.get("SQ_ACTIVE_INST_LDS", 0) / wc, dd.get("SQ_ACTIVE_INST_VMEM", 0) / wc,
              dd.get("SQ_ACTIVE_INST_SCA", 0) / wc, dd.get("SQ_WAIT_INST_ANY", 0) / wc,
              dd.get("SQ_WAIT_INST_LDS", 0) / wc, dd.get("SQ_WAIT_ANY", 0) / wc))
    print("  per SIMD: MFMA busy %.2f  MFMA||VALU %.2f  VALU instr/cyc %.3f  waves %.2f  "
          "LDS conflict cyc/instr %.2f  kernel %.3g cyc" % (
              dd.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / sc,
              dd.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / sc,
              dd.get("SQ_INSTS_VALU", 0) / sc, wc * 4 / sc,
              dd.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, dd.get("SQ_INSTS_LDS", 1)), g))
