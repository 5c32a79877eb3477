#!/usr/bin/env python3
"""Summarise the PMC passes of tools/pmc_roofline.sh into the per-launch
record bench.py reads (profiles/pmc_roofline.json, one entry per bench
configuration).

    python tools/pmc_roofline.py <pmc dir> <key> <stripes> [json path]

Dispatches are grouped by bench step: a torch / runtime dispatch (the
counters' zero_ before each encode) starts a step; inside it the qi kernels
before the first *ctx_kernel are the encode call, the context kernel and
everything after it the decode.  (qi dispatches before the first torch
dispatch -- a systematic NTT plan's own context -- are not part of a step.)
Per role and step the counters are summed over the role's dispatches, then
averaged over the steps: per *call*, which is one launch for the encode at
every BASELINE config.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is doubled on
gfx950 (wide coalesced reads tallied at half their bytes); WRITE_SIZE is
taken as reported; both in KiB.  VALU busy = SQ_INSTS_VALU x 4 cycles (a
wave64 int32 VALU instruction occupies a 16-lane SIMD for 4 cycles) over
1024 SIMDs x the role's cycles (GRBM_GUI_ACTIVE / 8 XCDs).
"""
import collections
import csv
import json
import os
import sys


def dispatches(path):
    """[(dispatch id, kernel name, {counter: value})] in dispatch order."""
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        key = int(r["Dispatch_Id"])
        e = d.setdefault(key, [r["Kernel_Name"], collections.Counter()])
        e[1][r["Counter_Name"]] += float(r["Counter_Value"])
    return [(k, v[0], v[1]) for k, v in sorted(d.items())]


def roles(path):
    """{role: [per-step Counter]}, {role: set of kernel names}"""
    steps = {"encode": [], "decode": []}
    names = {"encode": set(), "decode": set()}
    cur, phase, started = None, None, False
    for _, name, ctr in dispatches(path):
        if "qi::" not in name:
            started = True
            if cur is not None:
                for role in steps:
                    if cur[role]:
                        steps[role].append(cur[role])
            cur, phase = {"encode": collections.Counter(),
                          "decode": collections.Counter()}, "encode"
            continue
        if not started:
            continue
        if "ctx_kernel" in name or "ctx_lds_kernel" in name:
            phase = "decode"
        cur[phase].update(ctr)
        cur[phase]["dispatches"] += 1
        names[phase].add(name.split("(")[0].replace("void ", ""))
    if cur is not None:
        for role in steps:
            if cur[role]:
                steps[role].append(cur[role])
    return steps, names


def mean(counters):
    out = collections.Counter()
    for c in counters:
        out.update(c)
    return {k: v / len(counters) for k, v in out.items()} if counters else {}


def main():
    d, key, stripes = sys.argv[1], sys.argv[2], int(sys.argv[3])
    jpath = sys.argv[4] if len(sys.argv) > 4 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
        "profiles", "pmc_roofline.json")
    rec = {"stripes": stripes, "source": f"tools/pmc_roofline.sh ({d})",
           "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as reported, KiB"}
    for role in ("encode", "decode"):
        agg = {}
        for f in ("sq", "fetch", "write"):
            p = os.path.join(d, f + "_counter_collection.csv")
            if os.path.exists(p):
                st, names = roles(p)
                agg.update(mean(st[role]))
                agg["kernels"] = sorted(names[role])
        if not agg:
            continue
        r = {"kernels": agg.get("kernels"),
             "dispatches_per_call": agg.get("dispatches")}
        if "FETCH_SIZE" in agg:
            rd = agg["FETCH_SIZE"] * 1024 * 2
            wr = agg.get("WRITE_SIZE", 0.0) * 1024
            r.update(read_bytes_per_launch=rd, write_bytes_per_launch=wr,
                     hbm_bytes_per_launch=rd + wr)
        if "SQ_INSTS_VALU" in agg:
            cyc = agg.get("GRBM_GUI_ACTIVE", 0.0) / 8
            r.update(valu_instr=agg["SQ_INSTS_VALU"],
                     valu_instr_per_wave=agg["SQ_INSTS_VALU"] / max(1.0, agg.get("SQ_WAVES", 1)),
                     salu_instr_per_wave=agg.get("SQ_INSTS_SALU", 0) / max(1.0, agg.get("SQ_WAVES", 1)),
                     cycles=cyc,
                     valu_busy=agg["SQ_INSTS_VALU"] * 4 / (1024 * cyc) if cyc else None,
                     wait_any=agg.get("SQ_WAIT_ANY", 0) / max(1.0, agg.get("SQ_WAVE_CYCLES", 1)))
        rec[role] = r
    try:
        with open(jpath) as f:
            allrec = json.load(f)
    except (OSError, ValueError):
        allrec = {"configs": {}}
    allrec["configs"][key] = rec
    with open(jpath, "w") as f:
        json.dump(allrec, f, indent=1, sort_keys=True)
    print(json.dumps({key: rec}, indent=1))


if __name__ == "__main__":
    main()
