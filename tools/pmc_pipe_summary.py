#!/usr/bin/env python3
"""Summarise tools/pmc_pipe.sh: per-kernel, per-dispatch pipe shares.
SQ_*CYCLES / WAIT / ACTIVE counters are per-wave quad-cycles summed over
waves (MI355X_MICROARCH.md constants table); GRBM_GUI_ACTIVE sums 8 XCDs."""
import collections
import csv
import os
import sys

d = sys.argv[1]
tot = collections.defaultdict(dict)
for f in ["p1", "p2", "p3"]:
    p = os.path.join(d, f + "_counter_collection.csv")
    if not os.path.exists(p):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"].split("(")[0][:44] + " grid=" + r["Grid_Size"]
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
    g = dd.get("GRBM_GUI_ACTIVE", 0) / 8  # cycles of the kernel (per XCD)
    simd_cyc = g * 1024 if g else 0
    print(name)
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
    if simd_cyc:
        print("  per SIMD over the kernel: MFMA busy %.2f  MFMA||VALU %.2f  VALU instr/cycle %.3f "
              " waves resident %.2f  LDS bank-conflict cyc/instr %.2f  kernel %.3g cyc" % (
                  dd.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cyc,
                  dd.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / simd_cyc,
                  dd.get("SQ_INSTS_VALU", 0) / simd_cyc,
                  wc * 4 / simd_cyc,
                  dd.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, dd.get("SQ_INSTS_LDS", 1)),
                  g))
