"""GPU parity of the one-pass chunk store / fetch path (duplex.hip, DK_CHUNK) against the CPU
oracle and hashlib on uniform batches with caller-given chunk ids (content-derived ids stay
two-pass: the counter needs the digest first); staging variant 0 forces the two-pass path
(sha_kernel + records_kernel), so both must give the same bytes.  Reference: Node::store_chunk (src/core/Node.cpp:1414-1417:
chunk_hash = Sha256::digest(data), encrypt_with_key(chunk_key, chunk_id, data)) and
Node::fetch_chunk (:1644-1655: decrypt_with_key, then the hash check); ChaCha20 start counter
LE32(chunk_id[0..3]) (src/crypto/CryptoManager.cpp:8-13).  Bit-exact comparisons throughout."""
import hashlib

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
    E.set_staging(-1)


def host(t) -> bytes:
    return t.cpu().numpy().tobytes()


def dev(b: bytes):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


def records_of(arena_bytes: bytes, offs):
    return [arena_bytes[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def chunk_ids_for(n, seed, wrap_every=5):
    """Random 32-byte chunk ids; every wrap_every-th one starts its counter just below 2^32 so the
    u32 wrap (ChaCha20.cpp:110) happens inside the record."""
    ids = []
    for i in range(n):
        c = bytearray(splitmix_bytes(seed + i, 32))
        if i % wrap_every == 0:
            c[0:4] = (0xFFFFFFF0 - (i & 7)).to_bytes(4, "little")
        ids.append(bytes(c))
    return ids


def store(enet, items, keys, nonces, ids, base, key_stride=32, inplace=False):
    import torch
    n = len(items)
    b = enet.make_batch(items, keys, nonces, base_offset=base, key_stride=key_stride)
    hashes = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    out = b.arena if inplace else torch.full_like(b.arena, 0x55)
    enet.chunk_store(b, out, hashes, chunk_ids=dev(b"".join(ids)))
    return b, records_of(host(out), b.offsets.cpu().tolist()), host(hashes)


def fetch(enet, b, cts, ids, hashes):
    import torch
    import dataclasses
    n = len(cts)
    offs = b.offsets.cpu().tolist()
    arena = bytearray(host(b.arena))
    for i, c in enumerate(cts):
        arena[offs[i]:offs[i + 1]] = c
    bf = dataclasses.replace(b, arena=dev(bytes(arena)))
    back = torch.full_like(bf.arena, 0xAA)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.chunk_fetch(bf, back, dev(b"".join(ids)), dev(hashes), ok)
    return records_of(host(back), offs), ok.cpu().tolist()


@pytest.mark.parametrize("L,n,base", [(4096, 512, 0), (128, 256, 0), (256, 300, 5), (1536, 600, 3),
                                      (4096, 257, 16), (65536, 256, 0)])
def test_fused_chunks_vs_oracle(enet, L, n, base):
    """Store: ciphertexts match the oracle's ChaCha20 from LE32(chunk_id) (u32 wrap included) and
    the hashes are SHA-256 of the plaintexts; fetch returns every chunk with ok = 1; both agree
    with the two-pass path (staging 0); unaligned arenas included."""
    items = [splitmix_bytes(11000 + 7 * L + i, L) for i in range(n)]
    keys = [splitmix_bytes(12000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(13000 + i, 12) for i in range(n)]
    ids = chunk_ids_for(n, 14000)
    enet.set_staging(-1)
    b, cts, hh = store(enet, items, keys, nonces, ids, base)
    idx = range(n) if n * L <= 1 << 21 else list(range(0, n, 9)) + [n - 1]
    for i in idx:
        assert hh[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest(), i
        ctr = int.from_bytes(ids[i][:4], "little")
        assert cts[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], ctr), i
    got, ok = fetch(enet, b, cts, ids, hh)
    assert ok == [1] * n and got == items
    enet.set_staging(0)
    try:
        b2, cts2, hh2 = store(enet, items, keys, nonces, ids, base)
        assert cts2 == cts and hh2 == hh
        assert fetch(enet, b2, cts, ids, hh) == (got, ok)
    finally:
        enet.set_staging(-1)


def test_fused_chunks_reject_tampered(enet):
    """A flipped ciphertext byte (first, middle, last workgroup), a wrong manifest hash and a wrong
    chunk id (different counter) fail with ok = 0 and a zeroed chunk; neighbours are untouched."""
    n, L = 768, 1024
    items = [splitmix_bytes(600 + i, L) for i in range(n)]
    keys = [splitmix_bytes(700 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(800 + i, 12) for i in range(n)]
    ids = chunk_ids_for(n, 900)
    b, cts, hh = store(enet, items, keys, nonces, ids, 0)
    cts = list(cts)
    hb = bytearray(hh)
    bad_ids = list(ids)

    def flip(i, pos):
        c = bytearray(cts[i])
        c[pos] ^= 0x04
        cts[i] = bytes(c)

    flip(0, 0)
    flip(300, 517)
    flip(767, L - 1)
    hb[32 * 400 + 31] ^= 0x01
    bad_ids[555] = bytes([ids[555][0] ^ 1]) + ids[555][1:]
    tampered = {0, 300, 767, 400, 555}
    got, ok = fetch(enet, b, cts, bad_ids, bytes(hb))
    for i in range(n):
        if i in tampered:
            assert ok[i] == 0 and got[i] == bytes(L), i
        else:
            assert ok[i] == 1 and got[i] == items[i], i


def test_fused_chunks_shared_key_inplace(enet):
    """key_stride 0 (one key for the batch) and in-place store (out = in)."""
    n, L = 512, 2048
    items = [splitmix_bytes(1100 + i, L) for i in range(n)]
    key = splitmix_bytes(1101, 32)
    nonces = [splitmix_bytes(1200 + i, 12) for i in range(n)]
    ids = chunk_ids_for(n, 1300)
    b, cts, hh = store(enet, items, [key], nonces, ids, 0, key_stride=0, inplace=True)
    for i in (0, 1, 255, 256, 511):
        assert cts[i] == oracle.chacha20_xor(key, nonces[i], items[i],
                                             int.from_bytes(ids[i][:4], "little")), i
        assert hh[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest(), i
    got, ok = fetch(enet, b, cts, ids, hh)
    assert ok == [1] * n and got == items
