#!/usr/bin/env python3
"""Benchmark: device-resident RS-FNT encode+decode GB/s per GPU
(BASELINE.json metric; configs[1]: k=16, n=64, pkt=64 KiB, batch 4096 stripes).

One *step* = encode the whole stripe batch (k=16 data rows -> n=64 coded rows,
OOR side channel recorded) + build the per-stripe decode contexts (a random
n-k erasure pattern per stripe) + decode every stripe back to its k data rows.
Inputs are resident in HBM before the timed region starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--stripes S]

For N > 1 launch one process per GPU (torch.distributed.run); stripes shard
across ranks with no data-path collective (weak scaling: S stripes per GPU).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import quadiron_amd as qa  # noqa: E402

K_DATA, M_PAR, PKT_BYTES = 16, 48, 65536
# BASELINE.json configs measurable on one GPU: (k, m, packet bytes, stripes).
# cfg2 is the headline metric (the default); the others are extra lines.
CONFIGS = {
    "cfg2": (16, 48, 65536, 4096),
    "cfg3": (64, 960, 4096, 1024),   # high fragmentation, n = 1024
    "cfg1": (4, 4, 1024, 100),       # the reference's CPU plumbing case
}
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)


def alg_bytes(k, m, P, systematic=False):
    """Algorithmic HBM bytes per stripe: encode (k + n) * 2P
    (systematic: (k + m) * 2P), decode (k + k) * 2P."""
    n = 1
    while n < k + m:
        n *= 2
    enc_rows = k + (m if systematic else n)
    return enc_rows * 2 * P, 2 * k * 2 * P


def cpu_baseline(k, m, P, threads, stripes_per_thread, systematic=False):
    """QuadIron's own AVX2 path (oracle/_ref/libqiref_avx2.so, compiled from
    the reference sources) timed on this host: `threads` independent replicas
    (the reference bench's -g model) each encoding + decoding
    `stripes_per_thread` stripes of k x 64 KiB, one fixed n-k erasure
    pattern.  Falls back to the plain-C oracle port when the reference build
    is absent."""
    import ctypes as C
    ref = os.path.join(ROOT, "oracle", "_ref", "libqiref_avx2.so")
    enc_b, dec_b = alg_bytes(k, m, P, systematic)
    if os.path.exists(ref):
        lib = C.CDLL(ref)
        lib.ref_bench.restype = C.c_double
        rng = np.random.default_rng(1)
        missing = np.zeros(k + m, np.int32)
        missing[rng.choice(k + m, m, replace=False)] = 1
        e = C.c_double()
        d = C.c_double()
        wall = lib.ref_bench(int(systematic), k, m, C.c_size_t(P), stripes_per_thread,
                             threads, missing.ctypes.data_as(C.c_void_p),
                             C.byref(e), C.byref(d))
        total = threads * stripes_per_thread * (enc_b + dec_b)
        return {"value": total / wall / 1e9, "unit": "GB/s", "cores": threads,
                "kind": "reference",
                "sample": f"{threads} threads x {stripes_per_thread} stripes "
                          f"of RS-FNT{'-sys' if systematic else ''} k={k} "
                          f"m={m} pkt={2 * P // 1024}KiB enc+dec "
                          f"(QuadIron AVX2 build, pkt_size {P} words), "
                          f"wall {wall:.2f}s"}
    return None


def shard(rank, world, stripes_per_gpu):
    """Global stripe range [lo, hi) of a rank: the batch partitions by stripe
    (independent codewords), weak scaling -- no data-path collective."""
    return rank * stripes_per_gpu, (rank + 1) * stripes_per_gpu


def reduce_over_ranks(dist, elapsed, ok, device):
    """MAX of the per-rank timed-region wall time and AND of the per-rank
    round-trip checks (the only collectives in the bench)."""
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([1 if ok else 0], device=device, dtype=torch.int32)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    return t.item(), bool(okt.item())


def aggregate_value(world, stripes_per_gpu, steps, k, m, P, elapsed,
                    systematic=False):
    """Whole-job GB/s: algorithmic bytes of every rank's stripes / max time."""
    enc_b, dec_b = alg_bytes(k, m, P, systematic)
    return world * stripes_per_gpu * steps * (enc_b + dec_b) / elapsed / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=None)
    ap.add_argument("--cfg", choices=sorted(CONFIGS), default="cfg2")
    ap.add_argument("--systematic", action="store_true")
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-stripes", type=int, default=200)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    k, m, pkt_bytes, S = CONFIGS[args.cfg]
    if args.stripes:
        S = args.stripes
    P = pkt_bytes // 2
    sys_ = bool(args.systematic)
    headline = args.cfg == "cfg2" and not sys_
    plan = qa.Plan(k, m, sys_)
    n_out = plan.n_outputs
    cap = 64
    g = torch.Generator(device=dev)
    lo, _ = shard(rank, world, S)
    g.manual_seed(0x51D00001 + lo)  # this rank's shard of the global batch
    data = torch.randint(-32768, 32768, (S, k, P), dtype=torch.int16,
                         device=dev, generator=g)
    coded = torch.empty((S, n_out, P), dtype=torch.int16, device=dev)
    dec = torch.empty((S, k, P), dtype=torch.int16, device=dev)
    counts = torch.zeros(S * n_out, dtype=torch.int32, device=dev)
    entries = torch.zeros(S * n_out * cap, dtype=torch.int32, device=dev)
    # per-stripe erasure pattern: keep a random k-subset of the n ids
    perm = torch.rand((S, k + m), device=dev, generator=g).argsort(dim=1)
    ids = perm[:, :k].sort(dim=1).values.to(torch.int16).contiguous()
    ctx = torch.empty(plan.ctx_bytes(S, P), dtype=torch.uint8, device=dev)
    # the batch is processed as `chunks` slices round-robin over `streams`
    # HIP streams, so one slice's encode (write-heavy) overlaps another's
    # decode (read-heavy); every slice is still encoded, erased and decoded
    # inside the timed step
    NC = max(1, args.chunks)
    assert S % NC == 0, "stripes must divide into chunks"
    C = S // NC
    streams = ([torch.cuda.current_stream()] if NC == 1 else
               [torch.cuda.Stream() for _ in range(max(1, args.streams))])
    cstride = plan.ctx_bytes(1, P)

    ev = []

    def step(timed):
        for j in range(NC):
            st = streams[j % len(streams)]
            a, b = j * C, (j + 1) * C
            with torch.cuda.stream(st):
                cnt = counts[a * n_out:b * n_out]
                ent = entries[a * n_out * cap:b * n_out * cap]
                cx = ctx[a * cstride:b * cstride]
                cnt.zero_()
                if timed:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e2 = torch.cuda.Event(enable_timing=True)
                    e0.record(st)
                plan.encode(data[a:b], coded[a:b], cnt, ent, cap,
                            stream=st.cuda_stream)
                if timed:
                    e1.record(st)
                plan.decode_ctx(ids[a:b], cx, P, cnt, ent, cap,
                                stream=st.cuda_stream)
                plan.decode(cx, ids[a:b], coded[a:b], dec[a:b], data=data[a:b],
                            counts=cnt, entries=ent, cap=cap,
                            stream=st.cuda_stream, check=False)
                if timed:
                    e2.record(st)
                    ev.append((e0, e1, e2))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    # correctness of the measured pipeline (outside the timed region)
    ok = bool(torch.equal(dec, data)) and plan.take_error() == 0
    oor_max = int(counts.max().item())
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ok = ok and plan.take_error() == 0
    if dist:
        elapsed, ok = reduce_over_ranks(dist, elapsed, ok, dev)

    enc_b, dec_b = alg_bytes(k, m, P, sys_)
    value = aggregate_value(world, S, args.steps, k, m, P, elapsed, sys_)
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    # per launch: C stripes (the whole batch unless chunked)
    enc_gbs = C * enc_b / (enc_ms * 1e-3) / 1e9
    dec_gbs = C * dec_b / (dec_ms * 1e-3) / 1e9

    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if headline and os.path.exists(pmc):
        try:
            with open(pmc) as f:
                traffic = json.load(f).get("encode_bytes_per_launch")
        except Exception:
            traffic = None

    K = 1
    while K < k:
        K *= 2
    name = (f"RS-FNT{'-sys' if sys_ else ''} k={k} n={plan.n} "
            f"pkt={pkt_bytes // 1024}KiB")
    metric = ("device-resident encode+decode GB/s per GPU, RS-FNT k=16 n=64 "
              "pkt=64KiB" if headline else
              f"device-resident encode+decode GB/s per GPU, {name}")
    # the matrix path runs on the matrix cores for k <= 64
    # (matrix_pack.h MatLayout::KS), on the dot2 kernel otherwise
    mat_kernel = "matrix_mfma_kernel<*>" if k <= 64 else "matrix_kernel<*>"
    enc_kernel = (f"encode_fnt_kernel<{K},*>" if not sys_ and K <= 64
                  else mat_kernel)
    out = {
        "metric": metric,
        "value": value,
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic",
        "config": {
            "workload": f"{name} encode+decode, batch={S} stripes per GPU",
            "k": k, "m": m, "n": plan.n, "pkt_bytes": pkt_bytes,
            "systematic": sys_,
            "stripes_per_gpu": S,
            "decode": "per-stripe random n-k erasures, contexts built "
                      "on-GPU inside the timed step",
            "parallelism": f"stripe-sharded x{world} (no collective)",
            "chunks": NC, "streams": len(streams),
        },
        "per_gpu_value": value / world,
        "hbm_fraction": value / world / HBM_PEAK_GBS,
        "encode_kernel_ms": enc_ms,
        "encode_GBps": enc_gbs,
        "decode_ms": dec_ms,
        "decode_GBps": dec_gbs,
        "roundtrip_ok": ok,
        "oor_max_per_bucket": oor_max,
        "roofline": {
            "bound": "hbm",
            "kernel": enc_kernel,
            "achieved": enc_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": enc_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "bytes_per_launch": C * enc_b,
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
        out["cpu_baseline"] = cpu_baseline(k, m, P, threads, args.cpu_stripes,
                                           sys_)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
