#!/usr/bin/env python3
"""Per-block timeline of the cfg3 decode's operand-stationary kernel from the
probe build tools/ab/probe_os_ts.patch (s_memrealtime at entry, after the
block's first tile is in LDS, at the end; built by `tools/ab_build.sh os_ts ""
tools/ab/probe_os_ts.patch`):
    QI_LIB_PATH=build/ab/os_ts/libquadiron_amd.so python3 tools/os_stages.py [k,m,S,P]"""
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
no = plan.n_outputs
g = torch.Generator(device="cuda").manual_seed(1)
data = torch.randint(-32768, 32767, (S, k, P), dtype=torch.int16, device="cuda", generator=g)
coded = torch.zeros((S, no, P), dtype=torch.int16, device="cuda")
cap = 64 + P // 512
counts = torch.zeros(S * no, dtype=torch.int32, device="cuda")
entries = torch.zeros(S * no * cap, dtype=torch.int32, device="cuda")
plan.encode(data, coded, counts, entries, cap)
rng = np.random.default_rng(1)
ids = np.stack([np.sort(rng.choice(k + m, k, replace=False)) for _ in range(S)])
di = torch.from_numpy(ids.astype(np.int16)).cuda()
ctx = torch.zeros(plan.ctx_bytes(S, P), dtype=torch.uint8, device="cuda")
out = torch.zeros((S, k, P), dtype=torch.int16, device="cuda")
plan.decode_ctx(di, ctx, P, counts, entries, cap)
for _ in range(100):
    plan.decode(ctx, di, coded, out, None, counts, entries, cap, check=False)
torch.cuda.synchronize()
plan.decode(ctx, di, coded, out, None, counts, entries, cap)
assert torch.equal(out, data), "round trip"
lib = qa.lib()
n = 16384
buf = np.zeros(n * 4, dtype=np.uint64)
assert lib.qi_probe_os_ts(buf.ctypes.data_as(C.c_void_p), n) == 0
ts = buf.reshape(n, 4)
nb = int((ts[:, 0] > 0).sum())
ts = ts[:nb, :3].astype(np.float64) / 100.0
t0 = ts[:, 0].min()
st, pro, run = ts[:, 0] - t0, ts[:, 1] - ts[:, 0], ts[:, 2] - ts[:, 1]
end = ts[:, 2] - t0
print(f"k={k} S={S} P={P}: {nb} blocks; span {end.max():.1f} us")
print(f"  prologue (entry -> first tile in LDS) median {np.median(pro):.2f} p90 {np.percentile(pro, 90):.2f} max {pro.max():.2f} us")
print(f"  streaming (first tile -> end)         median {np.median(run):.2f} p90 {np.percentile(run, 90):.2f} max {run.max():.2f} us")
print(f"  block life median {np.median(end - st):.2f} us; prologue share {pro.sum() / (end - st).sum():.3f}")
h, e = np.histogram(st, bins=12)
print("  block start histogram (us: count):", ", ".join(f"{e[i]:.0f}:{h[i]}" for i in range(len(h))))
h, e = np.histogram(end, bins=12)
print("  block end histogram   (us: count):", ", ".join(f"{e[i]:.0f}:{h[i]}" for i in range(len(h))))
