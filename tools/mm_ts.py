#!/usr/bin/env python3
"""Block timeline of matrix_mfma_kernel from a QI_PROBE_TS build
(s_memrealtime stamps per block, 100 MHz: entry, row loads back, staging
barrier, exit; HW_ID / XCC_ID give the CU):
    bash tools/ab_build.sh ts -DQI_PROBE_TS
    QI_LIB_PATH=build/ab/ts/libquadiron_amd.so python3 tools/mm_ts.py [cfg3|cfg2]"""
import collections
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quadiron_amd as qa  # noqa: E402

torch.cuda.set_device(0)
lib = qa.lib()
lib.qi_probe_mm_read.argtypes = [C.c_void_p, C.c_size_t]
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
k, m, S, P = {"cfg3": (64, 960, 1024, 2048), "cfg2": (16, 48, 4096, 32768),
              "k128": (128, 128, 128, 32768)}[cfg]
plan = qa.Plan(k, m, False)
rng = np.random.default_rng(1)
data = torch.randint(-32768, 32767, (S, k, P), dtype=torch.int16, device="cuda")
out = torch.zeros((S, plan.n_outputs, P), dtype=torch.int16, device="cuda")
cap = 64
counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
entries = torch.zeros(S * plan.n_outputs * cap, dtype=torch.int32, device="cuda")
ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
di = torch.from_numpy(ids.astype(np.int16)).cuda()
ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
dec = torch.zeros_like(data)


def show(tag):
    torch.cuda.synchronize()
    ts = np.zeros((16384, 6), np.uint64)
    assert lib.qi_probe_mm_read(ts.ctypes.data, ts.nbytes) == 0
    t = ts[:, :4].astype(np.int64)
    live = t[:, 0] > 0
    t = t[live]
    hw = ts[live, 4].astype(np.int64)
    xcc = ts[live, 5].astype(np.int64) & 15
    n = len(t)
    t0 = t[:, 0].min()
    print(f"{tag}: {n} blocks, span {(t[:, 3].max() - t0) / 100:.1f} us")
    d = np.diff(t, axis=1) / 100.0
    for i, nm in enumerate(["row loads", "LDS+barrier", "compute+stores"]):
        print(f"   {nm:15s} median {np.median(d[:, i]):6.2f} us  p10 {np.percentile(d[:, i], 10):6.2f}"
              f"  p90 {np.percentile(d[:, i], 90):6.2f}  max {d[:, i].max():6.2f}")
    tot = (t[:, 3] - t[:, 0]) / 100.0
    print(f"   per-block total median {np.median(tot):.2f} us")
    cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
    per = collections.defaultdict(list)
    for i in range(n):
        per[cu[i]].append((t[i, 0], t[i, 1], t[i, 2], t[i, 3]))
    print(f"   CUs used {len(per)}; blocks per CU median {np.median([len(v) for v in per.values()]):.0f}")
    # residency over time (blocks live) and phase mix, sampled every 0.5 us
    grid = np.arange(t0, t[:, 3].max(), 50)
    live_n = [(np.sum((t[:, 0] <= g) & (t[:, 3] > g))) for g in grid]
    loading = [(np.sum((t[:, 0] <= g) & (t[:, 1] > g))) for g in grid]
    print("   time(us) live loading")
    for j in range(0, len(grid), max(1, len(grid) // 25)):
        print(f"   {(grid[j] - t0) / 100:7.1f} {live_n[j]:5d} {loading[j]:5d}")
    # gaps on one CU between a block's exit and the next entry
    gaps = []
    for v in per.values():
        v.sort()
        ends = sorted(x[3] for x in v)
        for x in v[2:]:
            prev = [e for e in ends if e <= x[0]]
            if prev:
                gaps.append((x[0] - prev[-1]) / 100.0)
    if gaps:
        print(f"   refill gap (exit -> next entry on the CU) median {np.median(gaps):.2f} us p90 {np.percentile(gaps, 90):.2f}")


for _ in range(2):
    plan.encode(data, out, counts, entries, cap)
show(f"{cfg} encode (matrix kernel at k > 32)" if k > 32 else f"{cfg} encode: not the matrix kernel")
plan.decode_ctx(di, ctx, P, counts, entries, cap)
for _ in range(2):
    plan.decode(ctx, di, out, dec, counts=counts, entries=entries, cap=cap)
show(f"{cfg} decode")
