"""Multi-GPU path on CPU: bench.py's stripe sharding and its only
collectives (MAX of the timed region, AND of the round-trip checks), run as
2 gloo ranks.  The GPU bench uses the same functions over RCCL."""
import os
import socket
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
