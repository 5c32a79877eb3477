#!/usr/bin/env python3
"""How the encode / decode kernel times of a bench configuration evolve over
a long run (GPU clock ramp under sustained load): runs bench.py's step for
`--seconds` and prints the HIP-event encode and decode-step times averaged
over consecutive windows of steps.
    python3 tools/ramp.py [--cfg cfg3] [--seconds 3] [--window 20]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import quadiron_amd as qa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="cfg3")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--window", type=int, default=20)
    args = ap.parse_args()
    k, m, pkt, S = bench.CONFIGS[args.cfg]
    P = pkt // 2
    dev = torch.device("cuda", 0)
    plan = qa.Plan(k, m, False)
    no, cap = plan.n_outputs, 64
    g = torch.Generator(device=dev)
    g.manual_seed(0x51D00001)
    data = torch.randint(-32768, 32768, (S, k, P), dtype=torch.int16, device=dev, generator=g)
    coded = torch.empty((S, no, P), dtype=torch.int16, device=dev)
    dec = torch.empty((S, k, P), dtype=torch.int16, device=dev)
    counts = torch.zeros(S * no, dtype=torch.int32, device=dev)
    entries = torch.zeros(S * no * cap, dtype=torch.int32, device=dev)
    perm = torch.rand((S, k + m), device=dev, generator=g).argsort(dim=1)
    ids = perm[:, :k].sort(dim=1).values.to(torch.int16).contiguous()
    ctx = torch.empty(plan.ctx_bytes(S, P), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    ev = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        for _ in range(args.window):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            counts.zero_()
            e0.record(st)
            plan.encode(data, coded, counts, entries, cap)
            e1.record(st)
            plan.decode_ctx(ids, ctx, P, counts, entries, cap)
            plan.decode(ctx, ids, coded, dec, data=data, counts=counts, entries=entries,
                        cap=cap, check=False)
            e2.record(st)
            ev.append((e0, e1, e2))
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(dec, data) and plan.take_error() == 0
    enc = np.array([a.elapsed_time(b) for a, b, _ in ev])
    dcs = np.array([b.elapsed_time(c) for _, b, c in ev])
    w = args.window
    print(f"{args.cfg}: {len(ev)} steps in {time.perf_counter() - t0:.2f} s; "
          f"per {w}-step window: encode ms, decode ms")
    for i in range(0, len(ev), w):
        print(f"  steps {i:5d}-{i + w - 1:5d}  enc {enc[i:i + w].mean():.4f}  "
              f"dec {dcs[i:i + w].mean():.4f}")


if __name__ == "__main__":
    main()
