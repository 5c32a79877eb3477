#!/usr/bin/env python3
"""Stage timeline of the k <= 128 decode-context kernel from the probe build
tools/ab/probe_ctx_ts8.patch (per-block s_memrealtime stamps, 100 MHz; built
by `tools/ab_build.sh ctx_ts8 "" tools/ab/probe_ctx_ts8.patch`):
    QI_LIB_PATH=build/ab/ctx_ts8/libquadiron_amd.so python3 tools/ctx_stages8.py [k,m,S,P]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import quadiron_amd as qa  # noqa: E402

torch.cuda.set_device(0)
k, m, S, P = (tuple(int(v) for v in sys.argv[1].split(",")) if len(sys.argv) > 1
              else (64, 960, 1024, 2048))
plan = qa.Plan(k, m, False)
rng = np.random.default_rng(1)
ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
di = torch.from_numpy(ids.astype(np.int16)).cuda()
ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
counts = torch.zeros(S * plan.n_outputs, dtype=torch.int32, device="cuda")
entries = torch.zeros(S * plan.n_outputs * 8, dtype=torch.int32, device="cuda")
for _ in range(300):
    plan.decode_ctx(di, ctx, P, counts, entries, 8)
torch.cuda.synchronize()
plan.decode_ctx(di, ctx, P, counts, entries, 8)
torch.cuda.synchronize()
lib = qa.lib()
n = min(S, 8192)
buf = np.zeros(n * 8, dtype=np.uint64)
assert lib.qi_probe_ts(buf.ctypes.data_as(C.c_void_p), n) == 0
ts = buf.reshape(n, 8)[:, :7].astype(np.float64) / 100.0  # 100 MHz -> us
t0 = ts[:, 0].min()
start = ts[:, 0] - t0
end = ts[:, 6] - t0
d = np.diff(ts, axis=1)
print(f"k={k} S={S}: block start skew {start.min():.2f}..{start.max():.2f} us "
      f"(median {np.median(start):.2f}); last block end {end.max():.2f} us")
for i, nm in enumerate(["ids+order", "x_i (rpow)", "A(x) chain", "route wait", "Q chains",
                        "row pass"]):
    print(f"  {nm:12s} median {np.median(d[:, i]):6.2f}  p90 {np.percentile(d[:, i], 90):6.2f}"
          f"  max {d[:, i].max():6.2f} us")
