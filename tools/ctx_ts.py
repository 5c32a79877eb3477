#!/usr/bin/env python3
"""Phase timeline of decode_ctx_lds_kernel from a QI_PROBE_TS build
(s_memrealtime stamps per workgroup, 100 MHz):
    QI_LIB_PATH=build/ab/ts/libquadiron_amd.so python3 tools/ctx_ts.py"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quadiron_amd as qa  # noqa: E402

torch.cuda.set_device(0)
lib = qa.lib()
lib.qi_probe_read.argtypes = [C.c_void_p, C.c_size_t]
names = ["ids", "A(x)+route", "Q+inv", "scale", "rows", "tiles+plain"]
for k, m, S, P in ((64, 960, 1024, 2048), (16, 48, 4096, 32768)):
    plan = qa.Plan(k, m, False)
    rng = np.random.default_rng(1)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
    di = torch.from_numpy(ids.astype(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * 8, dtype=torch.int32, device="cuda")
    for _ in range(3):
        plan.decode_ctx(di, ctx, P, counts, entries, 8)
    torch.cuda.synchronize()
    ts = np.zeros((8192, 8), np.uint64)
    assert lib.qi_probe_read(ts.ctypes.data, ts.nbytes) == 0
    n = min(S, 8192)
    t = ts[:n, :7].astype(np.int64)
    t0 = t[:, 0].min()
    print(f"k={k} S={S}: WG starts spread {(t[:, 0].max() - t0) / 100:.1f} us, "
          f"ends spread {(t[:, 6].min() - t0) / 100:.1f}..{(t[:, 6].max() - t0) / 100:.1f} us")
    d = np.diff(t, axis=1) / 100.0
    for i, nm in enumerate(names):
        print(f"   {nm:12s} median {np.median(d[:, i]):6.2f} us  p90 {np.percentile(d[:, i], 90):6.2f}"
              f"  max {d[:, i].max():6.2f}")
    tot = (t[:, 6] - t[:, 0]) / 100.0
    print(f"   per-WG total median {np.median(tot):.2f} us max {tot.max():.2f}")
