#!/usr/bin/env python3
"""Time decode_ctx alone with HIP events; the library comes from QI_LIB_PATH
(A/B of context-kernel variants).  Shapes k,m,S,P from the arguments
(default: cfg3 and cfg2):  python tools/ctx_time.py 256,768,256,2048"""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quadiron_amd as qa

torch.cuda.set_device(0)
shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or \
    [(64, 960, 1024, 2048), (16, 48, 4096, 32768)]
for k, m, S, P in shapes:
    plan = qa.Plan(k, m, False)
    rng = np.random.default_rng(1)
    ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
    di = torch.from_numpy(ids.astype(np.int16)).cuda()
    ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
    entries = torch.zeros(S * plan.n_outputs * 8, dtype=torch.int32, device="cuda")

    # a long warmup: the GPU clock settles after a few tens of ms of load
    for _ in range(300):
        plan.decode_ctx(di, ctx, P, counts, entries, 8)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        plan.decode_ctx(di, ctx, P, counts, entries, 8)
    b.record()
    torch.cuda.synchronize()
    print("k=%d S=%d ctx %.1f us" % (k, S, a.elapsed_time(b) / 20 * 1e3))
