"""GPU parity of the host-resident pipeline (include/enet_crypto.h "host pipeline"): batches in
host memory, cut into chunks and pipelined H2D -> kernels -> D2H over several streams, must give
the same bytes as the CPU oracle (which restates src/crypto and RFC 8439).  Chunk sizes are made
small so every batch spans many chunks, slots are reused and grown, and one record is larger
than a chunk."""
import numpy as np
import pytest

import oracle
from util import splitmix_bytes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enet():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import ephemeralnet_amd as E
    E.lib()
    yield E


def host_batch(E, items, keys, nonces, pinned, key_stride=32):
    import torch
    offs = np.concatenate([[0], np.cumsum([len(x) for x in items])]).astype(np.int64)
    total = int(offs[-1])
    arena = torch.frombuffer(bytearray(b"".join(items) or b"\0"), dtype=torch.uint8)[:total]
    k = torch.frombuffer(bytearray(b"".join(keys)), dtype=torch.uint8)
    nn = torch.frombuffer(bytearray(b"".join(nonces)), dtype=torch.uint8)
    o = torch.from_numpy(offs)
    if pinned:
        arena, k, nn, o = arena.pin_memory(), k.pin_memory(), nn.pin_memory(), o.pin_memory()
    return E.Batch(arena, o, k, nn, key_stride=key_stride, total_bytes_hint=total,
                   max_len_hint=max((len(x) for x in items), default=0))


def empty_like(t, pinned):
    import torch
    x = torch.zeros_like(t)
    return x.pin_memory() if pinned else x


def records(t, offs):
    b = t.numpy().tobytes()
    o = offs.tolist()
    return [b[o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.mark.parametrize("pinned,uniform,streams,chunk", [(True, True, 3, 40000),
                                                          (True, False, 4, 100000),
                                                          (False, False, 2, 70000),
                                                          (True, True, 1, 1 << 30)])
def test_pipeline_aead_roundtrip_vs_oracle(enet, pinned, uniform, streams, chunk):
    import torch
    n = 257
    if uniform:
        lens = [4096] * n
    else:
        raw = np.frombuffer(splitmix_bytes(5 + streams, 4 * n), dtype="<u4")
        lens = [int(x % 9000) for x in raw]
        lens[17] = 150000  # a record larger than a chunk
        lens[3] = 0
    items = [splitmix_bytes(1000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(2000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(3000 + i, 12) for i in range(n)]
    b = host_batch(enet, items, keys, nonces, pinned)
    ct = empty_like(b.arena, pinned)
    tags = empty_like(torch.zeros(16 * n, dtype=torch.uint8), pinned)
    with enet.Pipeline(0, chunk, streams) as pipe:
        pipe.aead_seal(b, ct, tags)
        got, th = records(ct, b.offsets), tags.numpy().tobytes()
        for i in range(n):
            c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
            assert got[i] == c and th[16 * i:16 * i + 16] == t, i
        # open (and reject one tampered record, whose plaintext comes back zeroed)
        if lens[40] > 1:
            ct[int(b.offsets[40]) + 1] ^= 0x80
        b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                        max_len_hint=b.max_len_hint)
        back = empty_like(b.arena, pinned)
        back.fill_(0x33)
        ok = empty_like(torch.zeros(n, dtype=torch.uint8), pinned)
        pipe.aead_open(b2, back, tags, ok)
        okh = ok.tolist()
        bk = records(back, b.offsets)
        for i in range(n):
            if i == 40 and lens[40] > 1:
                assert okh[i] == 0 and bk[i] == bytes(lens[i])
            else:
                assert okh[i] == 1 and bk[i] == items[i], i


def test_pipeline_hmac_and_xor_vs_oracle(enet):
    import torch
    n = 90
    raw = np.frombuffer(splitmix_bytes(77, 4 * n), dtype="<u4")
    lens = [512 + int(x % 20000) for x in raw]
    items = [splitmix_bytes(4000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(5000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(6000 + i, 12) for i in range(n)]
    b = host_batch(enet, items, keys, nonces, True)
    ct = empty_like(b.arena, True)
    tags = torch.zeros(16 * n, dtype=torch.uint8).pin_memory()
    macs = torch.zeros(32 * n, dtype=torch.uint8).pin_memory()
    with enet.Pipeline(0, 150000, 3) as pipe:
        pipe.aead_hmac_seal(b, ct, tags, macs)
        got, th, mh = records(ct, b.offsets), tags.numpy().tobytes(), macs.numpy().tobytes()
        for i in range(n):
            c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
            assert got[i] == c and th[16 * i:16 * i + 16] == t, i
            assert mh[32 * i:32 * i + 32] == oracle.hmac_sha256(keys[i], items[i]), i
        macs[32 * 7 + 3] ^= 1  # HMAC must reject record 7
        b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                        max_len_hint=b.max_len_hint)
        back = empty_like(b.arena, True)
        ok = torch.zeros(n, dtype=torch.uint8).pin_memory()
        pipe.aead_hmac_open(b2, back, tags, macs, ok)
        okh, bk = ok.tolist(), records(back, b.offsets)
        for i in range(n):
            assert (okh[i], bk[i]) == ((0, bytes(lens[i])) if i == 7 else (1, items[i])), i
        # reference ChaCha20::apply with per-record start counters (u32 wrap)
        ctr = np.frombuffer(splitmix_bytes(99, 4 * n), dtype="<u4").copy()
        ctr[0] = 0xFFFFFFFF
        xo = empty_like(b.arena, True)
        pipe.chacha20_xor(b, xo, torch.from_numpy(ctr.view(np.int32)).pin_memory())
        xg = records(xo, b.offsets)
        for i in range(n):
            assert xg[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctr[i])), i


def test_pipeline_shared_key_and_errors(enet):
    import torch
    n = 64
    key = splitmix_bytes(8, 32)
    items = [splitmix_bytes(7000 + i, 1500) for i in range(n)]
    nonces = [splitmix_bytes(8000 + i, 12) for i in range(n)]
    b = host_batch(enet, items, [key], nonces, True, key_stride=0)
    ct = empty_like(b.arena, True)
    tags = torch.zeros(16 * n, dtype=torch.uint8).pin_memory()
    with enet.Pipeline(0, 20000, 2) as pipe:
        pipe.aead_seal(b, ct, tags)
        got = records(ct, b.offsets)
        for i in range(0, n, 5):
            assert got[i] == oracle.aead_seal(key, nonces[i], items[i])[0]
        bad = enet.Batch(b.arena, b.offsets, b.keys, b.nonces, key_stride=0,
                         order=torch.zeros(n, dtype=torch.int32))
        with pytest.raises(enet.EnetError):
            pipe.aead_seal(bad, ct, tags)


@pytest.mark.parametrize("devices", [[0, 0, 0], [0], None])
def test_pipeline_group_vs_single(enet, devices):
    """enet_pipeline_group_*: a mixed 512 B - 64 KiB batch (C5 shape) cut into byte-balanced
    ranges over several pipelines (here three on device 0, so the split, the per-range offsets and
    the concurrent host threads are exercised on a one-GPU box) gives exactly the bytes, tags, MACs
    and verdicts of the single-device pipeline and of the oracle; a tampered tag and a tampered MAC
    in different ranges are both rejected."""
    import torch
    n = 211
    rng = np.random.default_rng(5)
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), n)).astype(int).tolist()
    items = [splitmix_bytes(9000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(9500 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(9800 + i, 12) for i in range(n)]
    b = host_batch(enet, items, keys, nonces, True)
    outs = []
    for mk in (lambda: enet.PipelineGroup(devices, 1 << 20, 2), lambda: enet.Pipeline(0, 1 << 20, 2)):
        ct = empty_like(b.arena, True)
        tags = torch.zeros(16 * n, dtype=torch.uint8).pin_memory()
        macs = torch.zeros(32 * n, dtype=torch.uint8).pin_memory()
        with mk() as pipe:
            if isinstance(pipe, enet.PipelineGroup):
                assert pipe.size == (len(devices) if devices else torch.cuda.device_count())
            pipe.aead_hmac_seal(b, ct, tags, macs)
            tg, mg = tags.clone(), macs.clone()
            tg[16 * 3] ^= 1          # first range
            mg[32 * (n - 2) + 5] ^= 1  # last range
            b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                            max_len_hint=b.max_len_hint)
            back = empty_like(b.arena, True)
            ok = torch.zeros(n, dtype=torch.uint8).pin_memory()
            pipe.aead_hmac_open(b2, back, tg, mg, ok)
        outs.append((ct.numpy().tobytes(), tags.numpy().tobytes(), macs.numpy().tobytes(),
                     back.numpy().tobytes(), ok.tolist()))
    assert outs[0] == outs[1]
    ctb, th, mh, bk, okh = outs[0]
    got, back = records(torch.frombuffer(bytearray(ctb), dtype=torch.uint8), b.offsets), \
        records(torch.frombuffer(bytearray(bk), dtype=torch.uint8), b.offsets)
    for i in list(range(0, n, 13)) + [3, n - 2, n - 1]:
        c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == c and th[16 * i:16 * i + 16] == t, i
        assert mh[32 * i:32 * i + 32] == oracle.hmac_sha256(keys[i], items[i]), i
    for i in range(n):
        assert (okh[i], back[i]) == ((0, bytes(lens[i])) if i in (3, n - 2) else (1, items[i])), i
