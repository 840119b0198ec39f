"""GPU parity of chunk store / fetch on the reference's real chunk sizes: a stored file is ONE chunk of
up to 32 MiB (include/ephemeralnet/Config.hpp:62, src/main.cpp:4467), hashed whole for its id and
manifest hash (src/core/Node.cpp:1414-1417, StoreProof.cpp:75-78) and checked whole on fetch
(Node.cpp:1644-1655).  Long chunks take the host-hash route (capi.cpp chunk_*_host_hash,
chunk_hybrid.cpp): their SHA-256 chain runs on host threads while the device runs their ChaCha20
on the sequence-parallel tiles; shorter chunks in the same batch stay on the one-pass duplex
kernel.  Expected bytes from the CPU oracle (ChaCha20 from LE32(chunk_id), CryptoManager.cpp:8-13,
with the u32 counter wrap of ChaCha20.cpp:110) and hashlib; every comparison is bit-exact."""
import hashlib

import numpy as np
import pytest

import oracle
from util import splitmix_bytes

pytestmark = pytest.mark.gpu

MiB = 1 << 20
NEVER = (1 << 63) - 1


@pytest.fixture(scope="module")
def enet():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import ephemeralnet_amd as E
    E.lib()
    yield E
    E.set_host_hash_min(-1)
    E.set_seg_min(-1)


def host(t) -> bytes:
    return t.cpu().numpy().tobytes()


def dev(b: bytes):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


def shapes():
    small = [int(x) % 5000 for x in np.frombuffer(splitmix_bytes(11, 4 * 300), "<u4")]
    return {
        "1x32MiB": [32 * MiB],
        "8x1MiB": [MiB] * 8,
        "mixed_with_32MiB": small[:150] + [32 * MiB] + small[150:] + [300 << 10, (256 << 10) + 17],
    }


def ids_for(n, seed):
    """Chunk ids; every third one starts its counter just below 2^32 so the keystream wraps inside
    a long chunk (ChaCha20.cpp:110)."""
    out = []
    for i in range(n):
        c = bytearray(splitmix_bytes(seed + i, 32))
        if i % 3 == 0:
            c[0:4] = (0xFFFFFFF0 - i).to_bytes(4, "little")
        out.append(bytes(c))
    return out


def make(enet, lens, seed, base=0):
    items = [splitmix_bytes(seed + i, L) for i, L in enumerate(lens)]
    n = len(lens)
    keys = [splitmix_bytes(seed + 10_000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(seed + 20_000 + i, 12) for i in range(n)]
    return enet.make_batch(items, keys, nonces, base_offset=base), items, keys, nonces


def store(enet, b, ids):
    import torch
    n = b.offsets.numel() - 1
    hashes = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    out = torch.full_like(b.arena, 0x55)
    enet.chunk_store(b, out, hashes, chunk_ids=dev(b"".join(ids)) if ids is not None else None)
    torch.cuda.synchronize()
    return out, host(hashes)


def fetch(enet, b, ct, ids, hashes):
    import dataclasses
    import torch
    n = b.offsets.numel() - 1
    bf = dataclasses.replace(b, arena=ct)
    back = torch.full_like(ct, 0xAA)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.chunk_fetch(bf, back, dev(b"".join(ids)), dev(hashes), ok)
    torch.cuda.synchronize()
    return back, ok.cpu().tolist()


@pytest.mark.parametrize("name", list(shapes()))
@pytest.mark.parametrize("given_ids", [True, False])
def test_long_chunks_store_fetch_vs_oracle(enet, name, given_ids):
    lens = shapes()[name]
    n = len(lens)
    b, items, keys, nonces = make(enet, lens, 4000 + len(name), base=3 if name == "mixed_with_32MiB" else 0)
    ids = ids_for(n, 777) if given_ids else None
    before = enet.host_hash_batches()
    ct, hh = store(enet, b, ids)
    assert enet.host_hash_batches() == before + 1, "long chunks did not take the host-hash route"
    offs = b.offsets.cpu().tolist()
    cth = host(ct)
    want_hash = [hashlib.sha256(it).digest() for it in items]
    for i in range(n):
        assert hh[32 * i:32 * i + 32] == want_hash[i], f"chunk hash {i} (len {lens[i]})"
        cid = ids[i] if given_ids else want_hash[i]  # content-derived id = the digest
        want = oracle.chacha20_xor(keys[i], nonces[i], items[i], oracle.derive_counter(cid))
        assert cth[offs[i]:offs[i + 1]] == want, f"ciphertext {i} (len {lens[i]})"
    assert cth[:offs[0]] == b"\x55" * offs[0], "bytes before the first record were written"
    fid = ids if given_ids else want_hash
    before = enet.host_hash_batches()
    back, ok = fetch(enet, b, ct, fid, hh)
    assert enet.host_hash_batches() == before + 1
    assert ok == [1] * n
    bh = host(back)
    for i in range(n):
        assert bh[offs[i]:offs[i + 1]] == items[i], f"plaintext {i} (len {lens[i]})"


def test_long_chunk_fetch_rejects_and_zeroes(enet):
    """A flipped ciphertext byte deep inside the 32 MiB chunk and a wrong manifest hash on a short
    chunk of the same batch: both fail, their plaintext is zeroed, every other chunk opens."""
    import torch
    lens = shapes()["mixed_with_32MiB"]
    n = len(lens)
    b, items, keys, nonces = make(enet, lens, 9100)
    ids = ids_for(n, 31)
    ct, hh = store(enet, b, ids)
    offs = b.offsets.cpu().tolist()
    big = lens.index(32 * MiB)
    small = next(i for i, L in enumerate(lens) if 0 < L < 4096)
    ct[offs[big] + 20 * MiB + 5] ^= 0x01
    bad = bytearray(hh)
    bad[32 * small] ^= 0x80
    back, ok = fetch(enet, b, ct, ids, bytes(bad))
    bh = host(back)
    for i in range(n):
        if i in (big, small):
            assert ok[i] == 0, i
            assert bh[offs[i]:offs[i + 1]] == b"\0" * lens[i], f"failed chunk {i} not zeroed"
        else:
            assert ok[i] == 1, i
            assert bh[offs[i]:offs[i + 1]] == items[i], i
    del torch


def test_long_chunks_same_bytes_on_gpu_lanes(enet):
    """enet_set_host_hash_min(INT64_MAX) keeps every hash chain on the GPU (one lane per chunk):
    8 x 1 MiB gives the same hashes and ciphertext as the host-hash route."""
    b, items, keys, nonces = make(enet, [MiB] * 8, 5200)
    ids = ids_for(8, 99)
    ct1, hh1 = store(enet, b, ids)
    enet.set_host_hash_min(NEVER)
    try:
        before = enet.host_hash_batches()
        ct2, hh2 = store(enet, b, ids)
        assert enet.host_hash_batches() == before
    finally:
        enet.set_host_hash_min(-1)
    assert hh1 == hh2 and host(ct1) == host(ct2)


def test_forced_threshold_small_chunks(enet):
    """enet_set_host_hash_min(1000): chunks of >= 1000 bytes hash on the host even when short (the
    record engine ciphers them, below the tiles' threshold), the rest on the duplex kernel; empty
    and one-byte chunks included."""
    lens = [0, 1, 999, 1000, 1001, 4096, 65536 + 7, 3, 70000]
    n = len(lens)
    b, items, keys, nonces = make(enet, lens, 6600, base=5)
    ids = ids_for(n, 5)
    enet.set_host_hash_min(1000)
    try:
        before = enet.host_hash_batches()
        ct, hh = store(enet, b, ids)
        back, ok = fetch(enet, b, ct, ids, hh)
        assert enet.host_hash_batches() == before + 2
    finally:
        enet.set_host_hash_min(-1)
    offs = b.offsets.cpu().tolist()
    cth, bh = host(ct), host(back)
    for i in range(n):
        assert hh[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest(), i
        assert cth[offs[i]:offs[i + 1]] == oracle.chacha20_xor(keys[i], nonces[i], items[i],
                                                              oracle.derive_counter(ids[i])), i
        assert bh[offs[i]:offs[i + 1]] == items[i], i
    assert ok == [1] * n


def test_long_chunks_in_host_mapped_memory(enet):
    """Arenas in pinned host memory the device maps (what the host-batch runtime's zero-copy mode
    and enet_host_alloc callers hand the C ABI): the host threads hash the long chunks where they
    lie -- on fetch only after the decrypt kernel has finished writing them -- and the bytes match
    the device-memory run."""
    import torch
    lens = [3 * MiB + 5, 700, (256 << 10) + 64]
    n = len(lens)
    b, items, keys, nonces = make(enet, lens, 7300)
    ids = ids_for(n, 17)
    ct_dev, hh_dev = store(enet, b, ids)
    pin_in = b.arena.cpu().pin_memory()
    pin_ct = torch.full_like(pin_in, 0x55).pin_memory()
    hashes = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    import dataclasses
    bh = dataclasses.replace(b, arena=pin_in)
    before = enet.host_hash_batches()
    enet.chunk_store(bh, pin_ct, hashes, chunk_ids=dev(b"".join(ids)))
    torch.cuda.synchronize()
    assert enet.host_hash_batches() == before + 1
    assert host(hashes) == hh_dev and pin_ct.numpy().tobytes() == host(ct_dev)
    back = torch.full_like(pin_in, 0xAA).pin_memory()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.chunk_fetch(dataclasses.replace(b, arena=pin_ct), back, dev(b"".join(ids)), dev(hh_dev), ok)
    torch.cuda.synchronize()
    assert ok.cpu().tolist() == [1] * n
    offs = b.offsets.cpu().tolist()
    bb = back.numpy().tobytes()
    for i in range(n):
        assert bb[offs[i]:offs[i + 1]] == items[i], i
