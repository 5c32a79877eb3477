#!/usr/bin/env python3
"""Stage timeline of the k > 128 decode-context kernel (decode_ctx_kernel<1024,
true>) from a probe build with per-block s_memrealtime stamps
(tools/ab/probe_ctxbig_ts.patch, built by tools/ab_build.sh ctxbig_ts; QI_LIB_PATH
points at it): setup, route table, A(x) product tree, A'(x_i), the division
down to the block's first chunk, that chunk's rows and its packing, in
microseconds (per block; a stripe's chunks may be spread over blocks).
    QI_LIB_PATH=build/ab/ctxbig_ts/libquadiron_amd.so python3 tools/ctxbig_stages.py [k,m,S,P]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quadiron_amd as qa  # noqa: E402

torch.cuda.set_device(0)
for arg in (sys.argv[1:] or ["300,212,32,32768"]):
    k, m, S, P = (int(v) for v in arg.split(","))
    plan = qa.Plan(k, m, False)
    rng = np.random.default_rng(1)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
    di = torch.from_numpy(ids.astype(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * 8, dtype=torch.int32, device="cuda")
    for _ in range(50):
        plan.decode_ctx(di, ctx, P, counts, entries, 8)
    torch.cuda.synchronize()
    plan.decode_ctx(di, ctx, P, counts, entries, 8)
    torch.cuda.synchronize()
    lib = qa.lib()
    n = min(S, 8192)
    buf = np.zeros(n * 10, dtype=np.uint64)
    assert lib.qi_probe_ts(buf.ctypes.data_as(C.c_void_p), n) == 0
    ts = buf.reshape(n, 10).astype(np.float64) / 100.0  # 100 MHz -> us
    t0 = ts[:, 0].min()
    print(f"k={k} S={S}: block start skew {ts[:, 0].max() - t0:.2f} us; "
          f"last block end {ts[:, 9].max() - t0:.2f} us")
    # stamps: 0 start, 1 setup, 7 route table, 2 A(x) tree, 3 A'(x_i),
    # 4 division to the first chunk, 5 its rows, 6 its packing, 9 end
    names = {1: "setup", 7: "route", 2: "A(x) tree", 3: "A'(x_i)", 4: "division",
             5: "chunk rows", 6: "chunk pack", 9: "rest"}
    prev = ts[:, 0]
    for i, nm in names.items():
        if ts[:, i].min() <= 0:
            continue
        d = ts[:, i] - prev
        prev = ts[:, i]
        print(f"  {nm:10s} median {np.median(d):7.2f}  max {d.max():7.2f} us")
