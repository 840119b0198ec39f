"""Multi-rank path on CPU: byte-balanced contiguous sharding, and a world_size-2 gloo run where
each rank seals only its shard (no data-path collective) and the union equals the single-rank
result.  The per-rank crypto here is the CPU oracle -- this tests the distribution logic, the GPU
kernels are covered by the -m gpu suite."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ephemeralnet_amd.shard import shard_ranges
from util import splitmix_bytes


def test_shard_ranges_cover_and_balance():
    rng = np.random.default_rng(5)
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), 5000)).astype(int).tolist()
    for world in (1, 2, 3, 8):
        rs = shard_ranges(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        tot = sum(lens)
        loads = [sum(lens[a:b]) for a, b in rs]
        assert max(loads) - min(loads) <= 2 * max(lens)
        assert sum(loads) == tot
    assert shard_ranges([], 4) == [(0, 0)] * 4
    assert shard_ranges([10], 3) in ([(0, 0), (0, 1), (1, 1)], [(0, 1), (1, 1), (1, 1)],
                                     [(0, 0), (0, 0), (0, 1)])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, lens, q):
    import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_ranges(lens, world)[rank]
    out = []
    for i in range(lo, hi):
        pt = splitmix_bytes(1000 + i, lens[i])
        ct, tag = oracle.aead_seal(splitmix_bytes(2000 + i, 32), splitmix_bytes(3000 + i, 12), pt)
        out.append((i, ct, tag))
    gathered = [None] * world
    dist.all_gather_object(gathered, out)  # test-only gather to compare
    if rank == 0:
        q.put([x for part in gathered for x in part])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_union_equals_single_rank():
    import oracle
    lens = [int(x) % 3000 for x in np.frombuffer(splitmix_bytes(9, 4 * 40), "<u4")]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, lens, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g[0] for g in got] == list(range(len(lens)))
    for i, ct, tag in got:
        pt = splitmix_bytes(1000 + i, lens[i])
        c, t = oracle.aead_seal(splitmix_bytes(2000 + i, 32), splitmix_bytes(3000 + i, 12), pt)
        assert ct == c and tag == t


def _report_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # rank r moved (r + 1) GiB in 0.5 s; rank 1 reports a failed round trip
    ranks = bench.rank_report(world, torch.device("cpu"), (rank + 1) << 30, 0.5, rank != 1)
    q.put((rank, ranks, dist.get_backend(), dist.get_world_size()))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_rank_report_two_rank_gloo():
    """bench.py's N > 1 reporting: every rank all-gathers each rank's own
    rate and round-trip verdict, so rank 0's line shows both ranks and a failure on rank 1."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_report_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ranks, backend, ws in res:
        assert backend == "gloo" and ws == 2
        assert [r["rank"] for r in ranks] == [0, 1]
        assert [r["gibs"] for r in ranks] == [2.0, 4.0]
        assert [r["ok"] for r in ranks] == [True, False]
    import bench
    assert bench.rank_report(1, None, 1, 1.0, True) is None
