"""Multi-GPU path on CPU: bench.py's stripe sharding and its only
collectives (MAX of the timed region, AND of the round-trip checks), run as
2 gloo ranks, and bench.py's own rank launcher (`--gpus N` -> N processes)
in its device-free dry-run mode.  The GPU bench uses the same code over
RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = bench.shard(rank, world, 4096)
        el, ok = bench.reduce_over_ranks(dist, 1.0 + rank, True, "cpu")
        el2, ok2 = bench.reduce_over_ranks(dist, 0.5, rank == 0, "cpu")
        v = bench.aggregate_value(world, 4096, 10, 16, 48, 32768, el)
        q.put((rank, lo, hi, el, ok, el2, ok2, v))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_bench_reductions(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [(lo, hi) for _, lo, hi, *_ in res]
    # disjoint, contiguous shards covering world * 4096 stripes
    assert ranges == [(r * 4096, (r + 1) * 4096) for r in range(world)]
    for _, _, _, el, ok, el2, ok2, v in res:
        assert el == float(world)         # MAX over ranks
        assert ok is True
        assert el2 == 0.5 and ok2 is False  # one failing rank fails all
        per_stripe = (16 + 64) * 2 * 32768 + 2 * 16 * 2 * 32768
        assert v == pytest.approx(world * 4096 * 10 * per_stripe / el / 1e9)


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, env=env,
                          timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [1, 2])
def test_bench_launches_n_ranks(n):
    """`bench.py --gpus N` (no launcher around it) starts N ranks itself
    before anything touches HIP, and rank 0 reports the process group's
    size -- the dry run takes the same launch/shard/reduce path on gloo."""
    r = _bench(["--gpus", str(n), "--dry-run", "--steps", "2", "--warmup", "1",
                "--cpu-seconds", "0.2"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["dry_run"] is True and out["roundtrip_ok"] is True
    assert out["scaling"] == "weak"
    assert out["config"]["parallelism"] == f"stripe-sharded x{n} (no collective)"
    per = (16 + 64) * 2 * 32768 + 2 * 16 * 2 * 32768
    assert out["value"] == pytest.approx(
        n * 4096 * 2 * per / (out["ms_per_step"] * 2e-3) / 1e9, rel=1e-6)
    # the same-run CPU baseline rides on every world size (rank 0, after the
    # timed region and the final barrier)
    cb = out["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["kind"] in ("reference", "port")


def test_bench_world_mismatch_fails():
    """--gpus N under a launcher whose world size differs is an error, not a
    silent run on fewer GPUs."""
    r = _bench(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"],
               {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr
