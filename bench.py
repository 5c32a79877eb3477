#!/usr/bin/env python3
"""Benchmark: device-resident RS-FNT encode+decode GB/s per GPU
(BASELINE.json metric; configs[1]: k=16, n=64, pkt=64 KiB, batch 4096 stripes).

One *step* = encode the whole stripe batch (k=16 data rows -> n=64 coded rows,
OOR side channel recorded) + build the per-stripe decode contexts (a random
n-k erasure pattern per stripe) + decode every stripe back to its k data rows.
Inputs are resident in HBM before the timed region starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--stripes S]

Multi-GPU: one process per GPU.  Stripes are independent codewords, so every
rank encodes/decodes its own batch of S stripes with no data-path collective
(weak scaling, the reference bench's per-thread replica model,
benchmark/benchmark.cpp:813-817).  Either launch the ranks yourself
(`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`) or
run `python bench.py --gpus N`: the process then starts torch.distributed.run
itself, as a child, before anything touches the GPU.  `--gpus` must match the
world size the ranks see; a mismatch is an error, never a silent 1-GPU run.
Rank 0 prints ONE JSON line; `n_gpus` is the process group's size.

`--dry-run` runs the same launch / shard / reduce / report logic on the CPU
(gloo, no HIP calls, no kernels): tests/test_distributed.py drives it.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import quadiron_amd as qa  # noqa: E402  (loads no library until used)

K_DATA, M_PAR, PKT_BYTES = 16, 48, 65536
# BASELINE.json configs measurable on one GPU: (k, m, packet bytes, stripes).
# cfg2 is the headline metric (the default); the others are extra lines.
CONFIGS = {
    "cfg2": (16, 48, 65536, 4096),
    "cfg3": (64, 960, 4096, 1024),   # high fragmentation, n = 1024
    "cfg1": (4, 4, 1024, 100),       # the reference's CPU plumbing case
    # larger codes: not BASELINE configs, extra lines.  64 < k <= 384 on
    # the matrix cores (whole 1024-column tiles above 256), larger k on the
    # NTT engine
    "k32": (32, 32, 65536, 1024),    # n = 64: the KS = 2 matrix decode
    "k128": (128, 128, 65536, 128),  # n = 256
    "k200": (200, 56, 65536, 64),    # n = 256
    "k256": (256, 768, 4096, 256),   # n = 1024
    "k300": (300, 212, 65536, 32),   # n = 512: the matrix cores at KS = 20
    "k384": (384, 128, 65536, 32),   # n = 512: the largest matrix-path k
    "k1000": (1000, 24, 65536, 16),  # n = 1024, len_2k = 2048: NTT engine
    # general decode at k > 384 with n - k > 64 (no erasure solve): the
    # reference's INTT_n -> NTT_2k -> x C -> INTT_2k pipeline on the engine
    "k600": (600, 1400, 65536, 16),  # n = 2048, len_2k = 2048
    # cfg3's code at 64 KiB packets (the same bytes per step as cfg3)
    "cfg3p64": (64, 960, 65536, 64),
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Host threads this process may use: the box's CPU share (OMP_NUM_THREADS
    is set to it on the GPU boxes), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_mhz():
    """Current clock of every CPU in this process's affinity mask, from
    /proc/cpuinfo ("cpu MHz" per processor), or [] where not readable."""
    try:
        mask = os.sched_getaffinity(0)
    except AttributeError:
        mask = None
    out, proc = [], None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("processor"):
                    proc = int(line.split(":", 1)[1])
                elif line.startswith("cpu MHz") and (mask is None or proc in mask):
                    out.append(float(line.split(":", 1)[1]))
    except (OSError, ValueError):
        pass
    return out


class _HostSampler:
    """Samples the host's clock and load while a CPU-baseline leg runs (the
    leg is one ctypes call, which releases the GIL): the spread of the same
    reference build across hosts (1-core legs from 0.2 to 3.3 GB/s) is read
    against these."""

    def __init__(self, period=0.25):
        import threading
        self.period, self.samples = period, []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            mhz = _cpu_mhz()
            if mhz:
                self.samples.append(mhz)
            self._stop.wait(self.period)

    def __enter__(self):
        self.load0 = os.getloadavg()
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()
        self.load1 = os.getloadavg()

    def summary(self, threads):
        allv = sorted(v for s in self.samples for v in s)
        busiest = sorted(v for s in self.samples for v in sorted(s)[-threads:])
        med = (lambda v: round(v[len(v) // 2], 1) if v else None)
        return {"cpu_mhz_median_all": med(allv),
                "cpu_mhz_median_busiest": med(busiest),
                "cpu_mhz_max": round(allv[-1], 1) if allv else None,
                "mhz_samples": len(self.samples),
                "loadavg_1m_before_after": [round(self.load0[0], 2),
                                            round(self.load1[0], 2)],
                "pinning": f"none: {threads} std::thread(s) float over the "
                           f"process's {len(_cpu_mhz()) or '?'} affinity CPUs"}


def _ref_leg(lib, k, m, P, threads, seconds, systematic, missing):
    import ctypes as C
    enc_b, dec_b = alg_bytes(k, m, P, systematic)
    stripes = C.c_longlong()
    enc_s, dec_s = C.c_double(), C.c_double()
    with _HostSampler() as hs:
        wall = lib.ref_bench(int(systematic), k, m, C.c_size_t(P), C.c_double(seconds),
                             threads, missing.ctypes.data_as(C.c_void_p),
                             C.byref(stripes), C.byref(enc_s), C.byref(dec_s))
    n = stripes.value
    # thread-time per stripe in each phase (the decode's share includes
    # building its DecodeContext, src/fec_base.h:1177-1321)
    enc_ms, dec_ms = enc_s.value / n * 1e3, dec_s.value / n * 1e3
    return {"value": n * (enc_b + dec_b) / wall / 1e9, "unit": "GB/s",
            "cores": threads, "stripes": n, "wall_s": round(wall, 3),
            "encode_ms_per_stripe": round(enc_ms, 4),
            "decode_ms_per_stripe": round(dec_ms, 4),
            "encode_GBps_per_thread": round(enc_b / enc_ms / 1e6, 3),
            "decode_GBps_per_thread": round(dec_b / dec_ms / 1e6, 3),
            "host": hs.summary(threads)}


def _port_leg(k, m, P, seconds, systematic, missing):
    """The plain-C oracle (a scalar restatement, one thread) when the
    reference build is absent."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from qi_testlib import oracle_decode_blocks, oracle_encode_blocks
    enc_b, dec_b = alg_bytes(k, m, P, systematic)
    rng = np.random.default_rng(1)
    data = rng.integers(0, 256, (k, 2 * P), dtype=np.uint8)
    n, te, td, t0 = 0, 0.0, 0.0, time.perf_counter()
    while True:
        a = time.perf_counter()
        outs, oor, cnt = oracle_encode_blocks(k, m, systematic, data)
        b = time.perf_counter()
        oracle_decode_blocks(k, m, systematic, outs, oor, cnt, missing, data)
        c = time.perf_counter()
        te, td, n = te + b - a, td + c - b, n + 1
        wall = c - t0
        if wall >= seconds:
            break
    return {"value": n * (enc_b + dec_b) / wall / 1e9, "unit": "GB/s",
            "cores": 1, "stripes": n, "wall_s": round(wall, 3),
            "encode_ms_per_stripe": round(te / n * 1e3, 4),
            "decode_ms_per_stripe": round(td / n * 1e3, 4)}


def cpu_baseline(k, m, P, systematic=False, seconds=1.0, threads=None):
    """QuadIron's own AVX2 path (oracle/_ref/libqiref_avx2.so, compiled from
    the reference sources; ref_driver.cpp ref_bench) timed on this host on
    the same stripes: independent per-thread replicas (benchmark.cpp:813-817)
    each encoding + decoding one stripe at a time from one fixed n-k erasure
    pattern for >= `seconds` of wall time, on 1 thread and on every thread of
    this process's CPU share.  Falls back to the plain-C oracle (1 thread,
    kind "port") when the reference build is absent."""
    import ctypes as C
    rng = np.random.default_rng(1)
    missing = np.zeros(k + m, np.int32)
    missing[rng.choice(k + m, m, replace=False)] = 1
    threads = threads or cpu_share()
    ref = os.path.join(ROOT, "oracle", "_ref", "libqiref_avx2.so")
    name = (f"RS-FNT{'-sys' if systematic else ''} k={k} m={m} "
            f"pkt={2 * P // 1024}KiB")
    if os.path.exists(ref):
        lib = C.CDLL(ref)
        lib.ref_bench.restype = C.c_double
        lib.ref_bench.argtypes = [C.c_int, C.c_int, C.c_int, C.c_size_t,
                                  C.c_double, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p]
        one = _ref_leg(lib, k, m, P, 1, seconds, systematic, missing)
        allc = _ref_leg(lib, k, m, P, threads, seconds, systematic, missing)
        kind = "reference"
        what = f"QuadIron AVX2 build (oracle/_ref), pkt_size {P} words"
    else:
        one = _port_leg(k, m, P, seconds, systematic, missing)
        allc = dict(one)
        kind = "port"
        what = "plain-C oracle restatement, scalar, 1 thread"
    return {"value": allc["value"], "unit": "GB/s", "cores": allc["cores"],
            "kind": kind,
            "sample": f"{name} enc+dec one stripe at a time per thread, "
                      f"fixed n-k erasure pattern, >= {seconds:g} s per leg: "
                      f"{allc['stripes']} stripes on {allc['cores']} threads "
                      f"in {allc['wall_s']} s, {one['stripes']} stripes on 1 "
                      f"thread in {one['wall_s']} s ({what}); per stripe on "
                      f"1 thread: encode {one['encode_ms_per_stripe']} ms, "
                      f"decode (context + apply) {one['decode_ms_per_stripe']} ms",
            "all_cores": allc, "one_core": one,
            "cpu": cpu_model(), "host_cpus": os.cpu_count()}


def pmc_record(key, stripes):
    """profiles/pmc_roofline.json entry for a bench configuration (measured
    at the same stripe count), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_roofline.json")
    try:
        with open(path) as f:
            rec = json.load(f)["configs"].get(key)
    except (OSError, ValueError, KeyError):
        return None
    if not rec or rec.get("stripes") != stripes:
        return None
    return dict(rec, source=rec.get("source"))


def valu_summary(k):
    """VALU issue of a kernel from its PMC record: SQ_INSTS_VALU per wave,
    and the busy fraction = SQ_INSTS_VALU x 4 cycles (a wave64 int32 VALU
    instruction issues over 4 cycles on a 16-lane SIMD) / (1024 SIMDs x the
    launch's cycles, GRBM_GUI_ACTIVE / 8 XCDs)."""
    if not k or not k.get("valu_instr"):
        return None
    return {"instr_per_wave": k.get("valu_instr_per_wave"),
            "busy": k.get("valu_busy"), "unit": "fraction of VALU issue cycles"}


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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Start `n` ranks of this script under torch.distributed.run as a child
    process and return its exit code.  The caller has not initialised HIP
    (nothing here touches the GPU), so no process is replaced."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--stripes", type=int, default=None)
    ap.add_argument("--cfg", choices=sorted(CONFIGS), default="cfg2")
    ap.add_argument("--systematic", action="store_true")
    ap.add_argument("--chunks", type=int, default=1)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--timed-events", action="store_true",
                    help="record the per-kernel HIP events on the timed steps "
                         "(default: on the last warmup steps)")
    ap.add_argument("--ctx-stream", type=int, default=None, choices=(0, 1, 2),
                    help="build the decode contexts from the ids alone on a "
                         "second stream beside the encode (default: off, "
                         "see CTX_STREAM); 2: that stream at the low and the "
                         "encode / decode stream at the high priority, so the "
                         "context blocks fill the encode's last round")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the cfg3 line the default (cfg2) run appends")
    ap.add_argument("--cpu-seconds", type=float, default=1.0)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch/shard/reduce/report on the CPU (gloo), no "
                         "HIP calls: tests the multi-rank path without GPUs")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, argv))
        world_env = 1
    else:
        world_env = int(env_world)
        if world_env != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}: "
                     "launch one process per GPU with matching sizes")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_run

    dist = None
    if world_env > 1:
        import torch.distributed as dist
        if dry:
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl",
                                    device_id=torch.device("cuda", local))
        world = dist.get_world_size()
        rank = dist.get_rank()
    else:
        world = 1
    if dry:
        dev = torch.device("cpu")
    else:
        if world == 1:
            torch.cuda.set_device(0)
        dev = torch.device("cuda", torch.cuda.current_device())

    res = run_config(args.cfg, args.stripes, bool(args.systematic), args.steps,
                     args.warmup, NC=max(1, args.chunks), n_streams=args.streams,
                     dist=dist, dev=dev, dry=dry, rank=rank, world=world,
                     ctx_stream=args.ctx_stream, timed_events=args.timed_events)
    out = report(res, args.cfg, world, args.steps, args.warmup, dry)
    ok = res["ok"]
    # BASELINE.json configs[2] (k=64 n=1024 pkt=4KiB, 1024 stripes) in the
    # same process, after the headline's timed region and in a timed region
    # of its own: a driver-observed line for the high-fragmentation code
    if (args.cfg == "cfg2" and not args.systematic and not args.no_secondary
            and args.chunks == 1):
        # (50 warmup steps, ~60 ms: a cfg3 step is 1.1 ms, and the GPU's
        # clock takes a few tens of ms of load to settle, tools/ramp.py)
        w3 = 50
        r3 = run_config("cfg3", None, False, max(5, min(args.steps, 20)), w3,
                        dist=dist, dev=dev, dry=dry, rank=rank, world=world)
        o3 = report(r3, "cfg3", world, r3["steps"], w3, dry)
        out["secondary"] = {"cfg3": {
            key: o3[key] for key in (
                "metric", "value", "ms_per_step", "steps", "warmup", "config",
                "hbm_fraction", "encode_kernel_ms", "encode_GBps", "decode_ms",
                "decode_ctx_ms", "decode_GBps", "roundtrip_ok", "roofline",
                "decode_roofline")}}
        ok = ok and r3["ok"]
    # the CPU baseline runs on rank 0 after the timed regions and their final
    # barriers (every rank's kernels are done), at every world size, so a
    # multi-GPU line carries the same-run CPU number as the 1-GPU one
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(res["k"], res["m"], res["P"],
                                           res["sys"], args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()  # the other ranks wait for rank 0's CPU baseline
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# configurations whose step builds the decode contexts on a second stream,
# from the ids alone, while the encode runs (init_context_dec before the
# fragments exist; the decode then reads the OOR marks from the buckets).
# None by default: measured slower everywhere (cfg3 4.45-4.58 vs 4.79-4.84
# TB/s: the encode 0.95-0.98 vs 0.91 ms beside the context blocks, the
# bucket-scanning decode 0.141-0.146 vs 0.134 ms; cfg2 6.04 vs 6.23;
# gpurun_out/ab_r5i_*, profiles/r5_ab_notes.txt)
CTX_STREAM = set()


def run_config(cfg, stripes, sys_, steps, warmup, NC=1, n_streams=2, dist=None,
               dev=None, dry=False, rank=0, world=1, ctx_stream=None, timed_events=False):
    """Build one configuration's synthetic batch in HBM, run `warmup`
    untimed steps, check the round trip, then time exactly `steps` steps
    between barriers + device synchronisations (max over ranks).  One step =
    encode every stripe (OOR recorded) + build the per-stripe decode
    contexts (a random n-k erasure pattern per stripe) + decode every
    stripe back to its k data rows."""
    k, m, pkt_bytes, S = CONFIGS[cfg]
    if stripes:
        S = stripes
    P = pkt_bytes // 2
    n = 1
    while n < k + m:
        n *= 2
    lo, _ = shard(rank, world, S)
    assert S % NC == 0, "stripes must divide into chunks"
    C = S // NC
    ev = []
    overlap = (cfg in CTX_STREAM) if ctx_stream is None else bool(ctx_stream)
    overlap = overlap and NC == 1 and not dry
    prio = overlap and ctx_stream == 2

    if dry:
        # the same loop structure on a small CPU stand-in per step
        data = torch.zeros((NC, 1024), dtype=torch.int64)
        data += lo

        def step(timed):
            for j in range(NC):
                data[j] = (data[j] * 3 + 1) % 65537

        def check():
            return True
        streams = [None]
        plan = None
    else:
        plan = qa.Plan(k, m, sys_)
        n_out = plan.n_outputs
        cap = 64
        g = torch.Generator(device=dev)
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
        # the batch is processed as `chunks` slices round-robin over
        # `streams` HIP streams, so one slice's encode (write-heavy) overlaps
        # another's decode (read-heavy); every slice is still encoded,
        # erased and decoded inside the timed step
        lo_p, hi_p = torch.cuda.Stream.priority_range() if prio else (0, 0)
        streams = ([torch.cuda.Stream(priority=hi_p)] if prio else
                   [torch.cuda.current_stream()] if NC == 1 else
                   [torch.cuda.Stream() for _ in range(max(1, n_streams))])
        cstride = plan.ctx_bytes(1, P)
        cst = torch.cuda.Stream(priority=lo_p) if overlap else None

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
                        # HIP events on the launch stream itself
                        e0, e1, ec, e2 = (torch.cuda.Event(enable_timing=True)
                                          for _ in range(4))
                    if overlap:
                        # the contexts from the ids alone on their own
                        # stream, beside the encode (after the previous
                        # step's decode, their last reader)
                        cst.wait_stream(st)
                        with torch.cuda.stream(cst):
                            if timed:
                                c0, c1 = (torch.cuda.Event(enable_timing=True)
                                          for _ in range(2))
                                c0.record(cst)
                            plan.decode_ctx(ids[a:b], cx, P, stream=cst.cuda_stream)
                            if timed:
                                c1.record(cst)
                    if timed:
                        e0.record(st)
                    plan.encode(data[a:b], coded[a:b], cnt, ent, cap,
                                stream=st.cuda_stream)
                    if timed:
                        e1.record(st)
                    if overlap:
                        st.wait_stream(cst)
                    else:
                        plan.decode_ctx(ids[a:b], cx, P, cnt, ent, cap,
                                        stream=st.cuda_stream)
                    if timed:
                        ec.record(st)
                    plan.decode(cx, ids[a:b], coded[a:b], dec[a:b],
                                data=data[a:b], counts=cnt, entries=ent,
                                cap=cap, stream=st.cuda_stream, check=False)
                    if timed:
                        e2.record(st)
                        ev.append((e0, e1, ec, e2, (c0, c1) if overlap else None))

        def check():
            # every stripe decoded back to its data, no OOR bucket overflowed
            # (a count above cap would also raise the plan's sticky error)
            return (bool(torch.equal(dec, data)) and plan.take_error() == 0
                    and int(counts.max().item()) <= cap)

    def sync():
        if not dry:
            torch.cuda.synchronize()

    # the round trip is checked after the FIRST warmup step (and again after
    # the timed steps), so the remaining warmup steps run back to back up to
    # the timed region: a host-synchronous check right before it left the GPU
    # idle for a few ms, and the timed steps then started at a lower clock
    # (cfg3 encode 1.03-1.05 ms over 20 steps vs 0.925 steady,
    # tools/ramp.py)
    # the kernel times come from HIP events on the last n_ev warmup steps,
    # which run back to back into the timed region: event markers between
    # the kernels of a timed step added launch bubbles to the wall time.
    # With few warmup steps those would follow the host-side check too
    # closely (the clock drops while the GPU idles: cfg2 encode 3.94 vs
    # 3.45 ms on warmup steps 1-2), so then the events go on the last
    # n_tev timed steps instead (--timed-events: on every timed step)
    n_ev = 0 if timed_events or warmup < 12 else min(8, warmup - 4)
    n_tev = steps if timed_events else (0 if n_ev else min(5, steps))
    ok = True
    for w in range(warmup):
        step(w >= warmup - n_ev)
        if w == 0:
            sync()
            ok = check()  # the measured pipeline, outside the timed region
    if warmup == 0:
        ok = check()
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i >= steps - n_tev)
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # and again after the timed steps (their last decode), outside the timer
    ok = ok and check()
    if dist:
        elapsed, ok = reduce_over_ranks(dist, elapsed, ok, dev)
    enc_ms = dec_ms = ctx_ms = None  # dry run: no kernels
    if ev:
        enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _, _, _ in ev]))
        # overlapped: the context kernel's own time on its stream (not on
        # the step's critical path); the decode time runs from the encode's
        # end to the decode's end either way
        ctx_ms = float(np.mean([c[0].elapsed_time(c[1]) if c else b.elapsed_time(cc)
                                for _, b, cc, _, c in ev]))
        dec_ms = float(np.mean([b.elapsed_time(d) for _, b, _, d, _ in ev]))
    # the kernels this plan launches (the library's own dispatch,
    # qi_gpu_kernels); the dry run names the cfg2 kernels it stands in for
    if dry:
        kernels = "encode=encode_fnt_kernel<16,2>; decode=(dry run: none)"
    else:
        kernels = plan.kernels(P)
    return {"ctx_overlap": overlap, "events_on": (
                f"warmup steps {warmup - n_ev}..{warmup - 1} (back to back into "
                f"the timed region, which runs without event markers)" if n_ev else
                "every timed step" if n_tev == steps else
                f"the last {n_tev} of the {steps} timed steps"),
            "k": k, "m": m, "n": n, "P": P, "pkt_bytes": pkt_bytes, "S": S,
            "C": C, "NC": NC, "sys": sys_, "steps": steps, "elapsed": elapsed,
            "ok": ok, "enc_ms": enc_ms, "dec_ms": dec_ms, "ctx_ms": ctx_ms,
            "kernels": kernels, "streams": len(streams)}


def rocprof_record(key):
    """profiles/rocprof_index.json entry for a bench configuration: the
    rocprofv3 --stats average durations of its encode and decode kernels
    (tools/rocprof_index.py, from the tracked *_kernel_stats.csv), with the
    build they were measured on."""
    path = os.path.join(ROOT, "profiles", "rocprof_index.json")
    try:
        with open(path) as f:
            idx = json.load(f)
    except (OSError, ValueError):
        return None
    rec = (idx.get("configs") or {}).get(key)
    if not rec:
        return None
    rec = dict(rec)
    rec.setdefault("build", idx.get("build"))
    return rec


def report(res, cfg, world, steps, warmup, dry):
    """The bench line of one run_config result."""
    k, m, n, P, S, C = (res[x] for x in ("k", "m", "n", "P", "S", "C"))
    sys_, pkt_bytes = res["sys"], res["pkt_bytes"]
    headline = cfg == "cfg2" and not sys_
    enc_b, dec_b = alg_bytes(k, m, P, sys_)
    elapsed = res["elapsed"]
    value = aggregate_value(world, S, steps, k, m, P, elapsed, sys_)
    enc_ms, dec_ms, ctx_ms = res["enc_ms"], res["dec_ms"], res["ctx_ms"]
    enc_gbs = dec_gbs = None
    if enc_ms:
        # per launch: C stripes (the whole batch unless chunked)
        enc_gbs = C * enc_b / (enc_ms * 1e-3) / 1e9
        dec_gbs = C * dec_b / (dec_ms * 1e-3) / 1e9

    # PMC record of this configuration (tools/pmc_roofline.sh: separate
    # rocprofv3 --pmc passes over a bench run of the same shape, FETCH_SIZE
    # doubled per MI355X_MICROARCH.md's gfx950 HBM note): HBM bytes and
    # VALU issue per launch of the encode kernel and of the decode kernels
    key = cfg + ("_sys" if sys_ else "")
    pmc = pmc_record(key, S)
    # rocprofv3 average durations of the same kernels (tracked profiles),
    # for a frac beside the event-timed one
    rp = rocprof_record(key) if not dry else None
    if rp and rp.get("stripes") != C:
        rp = None
    build = None if dry else qa.build_id()
    name = (f"RS-FNT{'-sys' if sys_ else ''} k={k} n={n} "
            f"pkt={pkt_bytes // 1024}KiB")
    metric = ("device-resident encode+decode GB/s per GPU, RS-FNT k=16 n=64 "
              "pkt=64KiB" if headline else
              f"device-resident encode+decode GB/s per GPU, {name}")
    enc_kernel, dec_kernels = (x.split("=", 1)[1]
                               for x in res["kernels"].split("; "))
    penc = (pmc or {}).get("encode") or {}
    pdec = (pmc or {}).get("decode") or {}

    def rocprof_frac(role, nbytes):
        r = (rp or {}).get(role)
        if not r or not r.get("avg_ms"):
            return {}
        same = bool(build and rp.get("build") and
                    build.split("+src:")[-1] == rp["build"].split("+src:")[-1])
        # frac_rocprof: the kernel trace over the profiled run's timed steps;
        # frac_stats: the --stats summary average over every call (warmup
        # steps at a ramping clock included), the lowest of the three
        allc = r.get("avg_ms_all_calls")
        return {"frac_rocprof": nbytes / (r["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "rocprof_ms": r["avg_ms"],
                "frac_stats": (nbytes / (allc * 1e-3) / 1e9 / HBM_PEAK_GBS
                               if allc else None),
                "stats_ms": allc,
                "rocprof_source": rp.get("source"),
                "rocprof_same_build": same}

    out = {
        "metric": metric,
        "value": value,
        "unit": "GB/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic",
        "config": {
            "workload": f"{name} encode+decode, batch={S} stripes per GPU",
            "k": k, "m": m, "n": n, "pkt_bytes": pkt_bytes,
            "systematic": sys_,
            "stripes_per_gpu": S,
            "decode": "per-stripe random n-k erasures, contexts built "
                      "on-GPU inside the timed step" +
                      (" (from the ids on a second stream, beside the encode; "
                       "the decode reads the OOR marks from the buckets)"
                       if res.get("ctx_overlap") else ""),
            "parallelism": f"stripe-sharded x{world} (no collective)",
            "chunks": res["NC"], "streams": res["streams"],
        },
        "per_gpu_value": value / world,
        "hbm_fraction": value / world / HBM_PEAK_GBS,
        "encode_kernel_ms": enc_ms,
        "encode_GBps": enc_gbs,
        "decode_ms": dec_ms,
        "decode_ctx_ms": ctx_ms,
        "kernel_times_from": res.get("events_on"),
        "decode_GBps": dec_gbs,
        "roundtrip_ok": res["ok"],
        # the dominant kernel: the encode (one launch per encode call at
        # every BASELINE config: whole 1024-column tiles, no tail kernel),
        # timed by HIP events on its launch stream
        "roofline": dict({
            "bound": "hbm",
            "kernel": enc_kernel,
            "timed_by": "hip_events",  # around the one encode launch, on its stream
            "achieved": enc_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": enc_gbs / HBM_PEAK_GBS if enc_gbs else None,
            "traffic": penc.get("hbm_bytes_per_launch"),
            "bytes_per_launch": C * enc_b,
            "traffic_ratio": (penc["hbm_bytes_per_launch"] / (C * enc_b)
                              if penc.get("hbm_bytes_per_launch") else None),
            "valu": valu_summary(penc),
        }, **rocprof_frac("encode", C * enc_b)),
        # the decode step (context build + matrix kernels) against the same
        # roofline: algorithmic bytes 2k * 2P per stripe
        "decode_roofline": dict({
            "kernels": dec_kernels,
            "timed_by": "hip_events",  # context build + decode kernels, on their stream
            "achieved": dec_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": dec_gbs / HBM_PEAK_GBS if dec_gbs else None,
            "traffic": pdec.get("hbm_bytes_per_launch"),
            "bytes_per_launch": C * dec_b,
            "traffic_ratio": (pdec["hbm_bytes_per_launch"] / (C * dec_b)
                              if pdec.get("hbm_bytes_per_launch") else None),
            "valu": valu_summary(pdec),
        }, **rocprof_frac("decode", C * dec_b)),
        "pmc_source": (pmc or {}).get("source"),
        "cpu_baseline": None,
        "build_id": build,
    }
    if dry:
        out["dry_run"] = True
    return out


if __name__ == "__main__":
    main()
