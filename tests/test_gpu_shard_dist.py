"""Multi-rank path through the HIP kernels: two ranks in separate processes (gloo
for the rendezvous, as bench.py's ENET_BENCH_BACKEND=gloo rehearsal), both on the one GPU of the
test box.  Each rank takes its byte-balanced contiguous shard (ephemeralnet_amd.shard.shard_ranges)
of a C5-shaped mixed batch, seals it with AEAD + HMAC-SHA256 (duplex kernel) and opens it again on
the device; no collective touches the data, a test-only all_gather brings the per-rank results to
rank 0, which checks the union record by record against the CPU oracle."""
import os
import socket

import numpy as np
import pytest

from util import splitmix_bytes

pytestmark = pytest.mark.gpu

N_REC = 96


def _lens():
    rng = np.random.default_rng(77)
    return np.exp(rng.uniform(np.log(512), np.log(16384), N_REC)).astype(int).tolist()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import ephemeralnet_amd as E
    from ephemeralnet_amd.shard import shard_ranges

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens = _lens()
    lo, hi = shard_ranges(lens, world)[rank]
    res = []
    if hi > lo:
        idx = list(range(lo, hi))
        items = [splitmix_bytes(5000 + i, lens[i]) for i in idx]
        keys = [splitmix_bytes(6000 + i, 32) for i in idx]
        nonces = [splitmix_bytes(7000 + i, 12) for i in idx]
        b = E.make_batch(items, keys, nonces)
        n = hi - lo
        ct = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
        E.aead_hmac_seal(b, ct, tags, macs)
        b2 = E.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                     max_len_hint=b.max_len_hint)
        back = torch.zeros_like(ct)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        E.aead_hmac_open(b2, back, tags, macs, ok)
        torch.cuda.synchronize()
        offs = b.offsets.cpu().tolist()
        cth = ct.cpu().numpy().tobytes()
        th, mh = tags.cpu().numpy().tobytes(), macs.cpu().numpy().tobytes()
        roundtrip = bool(torch.equal(back, b.arena)) and int(ok.sum()) == n
        for k, i in enumerate(idx):
            res.append((i, cth[offs[k]:offs[k + 1]], th[16 * k:16 * k + 16], mh[32 * k:32 * k + 32],
                        roundtrip))
    gathered = [None] * world
    dist.all_gather_object(gathered, (rank, lo, hi, res))  # test-only gather to compare
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_one_gpu_shards_match_oracle():
    import torch.multiprocessing as mp

    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    lens = _lens()
    # the two shards are contiguous, cover every record once, and balance bytes
    (r0, lo0, hi0, _), (r1, lo1, hi1, _) = sorted(gathered)[:2]
    assert (lo0, hi1) == (0, N_REC) and hi0 == lo1 and 0 < hi0 < N_REC
    assert abs(sum(lens[lo0:hi0]) - sum(lens[lo1:hi1])) <= 2 * max(lens)
    got = sorted(x for g in gathered for x in g[3])
    assert [g[0] for g in got] == list(range(N_REC))
    for i, ct, tag, mac, roundtrip in got:
        pt = splitmix_bytes(5000 + i, lens[i])
        key, nonce = splitmix_bytes(6000 + i, 32), splitmix_bytes(7000 + i, 12)
        c, t = oracle.aead_seal(key, nonce, pt)
        assert ct == c and tag == t, i
        assert mac == oracle.hmac_sha256(key, pt), i
        assert roundtrip, i
