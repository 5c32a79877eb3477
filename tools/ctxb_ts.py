#!/usr/bin/env python3
"""Phase timeline of decode_ctx_kernel<1024, true> (k > 128) from a
QI_PROBE_TS build (s_memrealtime stamps per workgroup, 100 MHz):
    bash tools/ab_build.sh ts -DQI_PROBE_TS
    QI_LIB_PATH=build/ab/ts/libquadiron_amd.so python3 tools/ctxb_ts.py"""
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
names = ["ids/route", "A(x)", "Q_i, A'", "pack rows", "tiles"]
for k, m, S, P in ((200, 56, 64, 32768), (256, 768, 256, 2048), (300, 212, 32, 32768)):
    plan = qa.Plan(k, m, False)
    rng = np.random.default_rng(1)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
    di = torch.from_numpy(ids.astype(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * 8, dtype=torch.int32, device="cuda")
    for _ in range(3):
        plan.decode_ctx(di, ctx, P, counts, entries, 8)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    plan.decode_ctx(di, ctx, P, counts, entries, 8)
    b.record()
    torch.cuda.synchronize()
    ts = np.zeros((8192, 8), np.uint64)
    assert lib.qi_probe_read(ts.ctypes.data, ts.nbytes) == 0
    t = ts[:S, :6].astype(np.int64)
    t0 = t[:, 0].min()
    print(f"k={k} S={S}: launch {a.elapsed_time(b) * 1e3:.1f} us; WG starts spread "
          f"{(t[:, 0].max() - t0) / 100:.1f} us, ends {(t[:, 5].min() - t0) / 100:.1f}.."
          f"{(t[:, 5].max() - t0) / 100:.1f} us")
    d = np.diff(t, axis=1) / 100.0
    for i, nm in enumerate(names):
        print(f"   {nm:12s} median {np.median(d[:, i]):7.2f} us  max {d[:, i].max():7.2f}")
