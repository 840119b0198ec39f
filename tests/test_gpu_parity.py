"""GPU parity: the HIP kernels (through the C ABI) against the golden vectors (compiled reference
src/crypto; OpenSSL + RFC 8439 for the AEAD) and the CPU oracle on seeded random batches.
Integer/byte work: every comparison is bit-exact."""
import hashlib

import numpy as np
import pytest

import oracle
from util import splitmix_bytes

pytestmark = pytest.mark.gpu

LANES = [1, 2, 4, 8, 16]


@pytest.fixture(scope="module")
def enet():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import ephemeralnet_amd as E
    E.lib()
    yield E
    E.set_lanes_per_record(0)


def dev(b: bytes):
    import torch
    return torch.frombuffer(bytearray(b if b else b"\0"), dtype=torch.uint8)[: len(b)].cuda()


def host(t) -> bytes:
    return t.cpu().numpy().tobytes()


def expect(rep, got: bytes):
    if "hex" in rep:
        assert got.hex() == rep["hex"]
    else:
        assert hashlib.sha256(got).hexdigest() == rep["sha256"]


def records_of(arena_bytes: bytes, offs):
    return [arena_bytes[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def out_like(b):
    import torch
    return torch.zeros_like(b.arena)


def rand_lengths(seed, n, hi):
    raw = np.frombuffer(splitmix_bytes(seed, 4 * n), dtype="<u4")
    return [int(x % (hi + 1)) for x in raw]


# ------------------------------------------------------------------------------ ChaCha20
@pytest.mark.parametrize("lanes", LANES)
def test_chacha20_golden(enet, golden, lanes):
    import torch
    enet.set_lanes_per_record(lanes)
    cs = golden["chacha20"]
    items = [splitmix_bytes(c["pt_seed"], c["len"]) for c in cs]
    b = enet.make_batch(items, [bytes.fromhex(c["key"]) for c in cs],
                        [bytes.fromhex(c["nonce"]) for c in cs])
    ctr = torch.tensor(np.array([c["counter"] for c in cs], dtype=np.uint32).view(np.int32)).cuda()
    out = out_like(b)
    enet.chacha20_xor(b, out, counters=ctr)
    torch.cuda.synchronize()
    offs = b.offsets.cpu().tolist()
    got = records_of(host(out), offs)
    for c, g in zip(cs, got):
        expect(c["ct"], g)


def test_chacha20_rfc8439(enet, golden):
    import torch
    v = golden["rfc8439_2_4_2"]
    b = enet.make_batch([bytes.fromhex(v["pt"])], [bytes.fromhex(v["key"])], [bytes.fromhex(v["nonce"])])
    out = out_like(b)
    ctr = torch.tensor([1], dtype=torch.int32).cuda()
    enet.chacha20_xor(b, out, counters=ctr)
    assert host(out).hex() == v["ct"]


@pytest.mark.parametrize("lanes", LANES)
@pytest.mark.parametrize("base", [0, 3])
def test_chacha20_random_vs_oracle(enet, lanes, base):
    import torch
    enet.set_lanes_per_record(lanes)
    n = 300
    lens = rand_lengths(11 + lanes, n, 5000)
    lens[:6] = [0, 1, 63, 64, 65, 4096]
    items = [splitmix_bytes(100 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(10000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(20000 + i, 12) for i in range(n)]
    ctrs = np.frombuffer(splitmix_bytes(7, 4 * n), dtype="<u4").copy()
    ctrs[:4] = [0xFFFFFFFF, 0xFFFFFFFE, 0xFFFFFFC0, 0]
    b = enet.make_batch(items, keys, nonces, base_offset=base)
    out = out_like(b)
    enet.chacha20_xor(b, out, counters=torch.tensor(ctrs.view(np.int32)).cuda())
    got = records_of(host(out), b.offsets.cpu().tolist())
    for i in range(n):
        assert got[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctrs[i])), i


def test_chacha20_in_place_shared_key(enet):
    import torch
    enet.set_lanes_per_record(0)
    n = 64
    items = [splitmix_bytes(300 + i, 4096) for i in range(n)]
    key = splitmix_bytes(1, 32)
    nonces = [splitmix_bytes(400 + i, 12) for i in range(n)]
    b = enet.make_batch(items, [key], nonces, key_stride=0)
    enet.chacha20_xor(b, b.arena)  # in place, counter 0 (SessionManager.cpp:374)
    got = records_of(host(b.arena), b.offsets.cpu().tolist())
    for i in range(n):
        assert got[i] == oracle.chacha20_xor(key, nonces[i], items[i], 0)


def test_cryptomanager_golden(enet, golden):
    import torch
    cs = golden["cryptomanager"]
    items = [splitmix_bytes(c["pt_seed"], c["len"]) for c in cs]
    b = enet.make_batch(items, [bytes.fromhex(c["key"]) for c in cs], [bytes.fromhex(c["nonce"]) for c in cs])
    ctr = np.array([enet.chunk_counter(bytes.fromhex(c["chunk_id"])) for c in cs], dtype=np.uint32)
    out = out_like(b)
    enet.chacha20_xor(b, out, counters=torch.tensor(ctr.view(np.int32)).cuda())
    for c, g in zip(cs, records_of(host(out), b.offsets.cpu().tolist())):
        expect(c["ct"], g)


# ------------------------------------------------------------------------------ chunk pipeline
def test_chunk_store_golden(enet, golden):
    """Store pipeline with caller-given chunk ids reproduces the reference's encrypt_with_key
    ciphertexts, and the chunk hashes are SHA-256 of the plaintexts."""
    import torch
    cs = golden["cryptomanager"]
    items = [splitmix_bytes(c["pt_seed"], c["len"]) for c in cs]
    b = enet.make_batch(items, [bytes.fromhex(c["key"]) for c in cs], [bytes.fromhex(c["nonce"]) for c in cs])
    ids = dev(b"".join(bytes.fromhex(c["chunk_id"]) for c in cs))
    hashes = torch.zeros(32 * len(cs), dtype=torch.uint8, device="cuda")
    out = out_like(b)
    enet.chunk_store(b, out, hashes, chunk_ids=ids)
    hh = host(hashes)
    for i, (c, g) in enumerate(zip(cs, records_of(host(out), b.offsets.cpu().tolist()))):
        expect(c["ct"], g)
        assert hh[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest()


@pytest.mark.parametrize("lanes", [1, 4])
def test_chunk_store_fetch_vs_oracle(enet, lanes):
    """Content-derived ids (daemon store path): counter = LE32(SHA-256(chunk)[0..3]); the fetch
    side decrypts and keeps only chunks whose hash matches the manifest."""
    import torch
    enet.set_lanes_per_record(lanes)
    n = 160
    lens = rand_lengths(91, n, 9000)
    lens[:6] = [0, 1, 63, 64, 4096, 65536]
    items = [splitmix_bytes(3000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(4000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(5000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces, base_offset=2)
    hashes = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ct = out_like(b)
    enet.chunk_store(b, ct, hashes)
    hh = host(hashes)
    offs = b.offsets.cpu().tolist()
    cts = records_of(host(ct), offs)
    for i in range(n):
        h = hashlib.sha256(items[i]).digest()
        assert hh[32 * i:32 * i + 32] == h, i
        ctr = int.from_bytes(h[:4], "little")
        assert cts[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], ctr), i
    # fetch: tamper one ciphertext byte and one manifest hash
    ctb = bytearray(host(ct))
    ctb[offs[10] + 3] ^= 0x01
    bad_hashes = bytearray(hh)
    bad_hashes[32 * 11] ^= 0x80
    bf = enet.Batch(torch.frombuffer(ctb, dtype=torch.uint8).cuda(), b.offsets, b.keys, b.nonces,
                    total_bytes_hint=b.total_bytes_hint, max_len_hint=b.max_len_hint)
    back = torch.full_like(ct, 0x55)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.chunk_fetch(bf, back, hashes.clone(), dev(bytes(bad_hashes)), ok)
    okh = ok.cpu().tolist()
    got = records_of(host(back), offs)
    for i in range(n):
        if i in (10, 11):
            assert okh[i] == 0 and got[i] == bytes(len(got[i])), i
        else:
            assert okh[i] == 1 and got[i] == items[i], i


# ------------------------------------------------------------------------------ AEAD
def aead_batch(enet, cases, base=0):
    import torch
    items = [splitmix_bytes(c["pt_seed"], c["len"]) for c in cases]
    aads = [splitmix_bytes(c["aad_seed"], c["aad_len"]) for c in cases]
    b = enet.make_batch(items, [bytes.fromhex(c["key"]) for c in cases],
                        [bytes.fromhex(c["nonce"]) for c in cases], base_offset=base)
    aoff = np.concatenate([[0], np.cumsum([len(a) for a in aads])]).astype(np.int64)
    aad = dev(b"".join(aads) or b"\0")
    return items, aads, b, aad, torch.tensor(aoff).cuda()


@pytest.mark.parametrize("lanes", LANES)
def test_aead_golden(enet, golden, lanes):
    import torch
    enet.set_lanes_per_record(lanes)
    cs = golden["aead"]
    items, aads, b, aad, aoff = aead_batch(enet, cs)
    out = out_like(b)
    tags = torch.zeros(16 * len(cs), dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags, aad, aoff)
    offs = b.offsets.cpu().tolist()
    got = records_of(host(out), offs)
    th = host(tags)
    for i, c in enumerate(cs):
        expect(c["ct"], got[i])
        assert th[16 * i:16 * i + 16].hex() == c["tag"], (i, c["len"], c["aad_len"])
    # open the ciphertext back, one tampered record and one tampered tag
    ct = out.clone()
    tags2 = tags.clone()
    tamper_rec = next(i for i, c in enumerate(cs) if c["len"] >= 64)
    ct[offs[tamper_rec] + 5] ^= 1
    tags2[16 * 2] ^= 0x40
    b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                    max_len_hint=b.max_len_hint)
    pt = torch.full_like(ct, 0xAA)
    ok = torch.zeros(len(cs), dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, pt, tags2, ok, aad, aoff)
    okh = ok.cpu().tolist()
    back = records_of(host(pt), offs)
    for i in range(len(cs)):
        if i in (tamper_rec, 2):
            assert okh[i] == 0
            assert back[i] == bytes(len(back[i]))  # plaintext not released
        else:
            assert okh[i] == 1, i
            assert back[i] == items[i]


def test_aead_rfc8439(enet, golden):
    import torch
    v = golden["rfc8439_2_8_2"]
    b = enet.make_batch([bytes.fromhex(v["pt"])], [bytes.fromhex(v["key"])], [bytes.fromhex(v["nonce"])])
    aad = dev(bytes.fromhex(v["aad"]))
    aoff = torch.tensor([0, 12], dtype=torch.int64).cuda()
    out = out_like(b)
    tags = torch.zeros(16, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags, aad, aoff)
    assert host(out).hex() == v["ct"]
    assert host(tags).hex() == v["tag"] == "1ae10b594f09e26a7e902ecbd0600691"


@pytest.mark.parametrize("lanes", LANES)
@pytest.mark.parametrize("base", [0, 5])
def test_aead_random_vs_oracle(enet, lanes, base):
    import torch
    enet.set_lanes_per_record(lanes)
    n = 257
    lens = rand_lengths(50 + lanes, n, 3000)
    lens[:8] = [0, 1, 15, 16, 17, 64, 1500, 4096]
    items = [splitmix_bytes(600 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(30000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(40000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces, base_offset=base)
    out = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    got = records_of(host(out), b.offsets.cpu().tolist())
    th = host(tags)
    for i in range(n):
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct, i
        assert th[16 * i:16 * i + 16] == tag, (i, lens[i])


def test_aead_roundtrip_headline_size(enet):
    """C2 shape at full size (65 536 x 4 KiB, per-record keys): size-independent properties --
    open(seal(x)) == x with every tag verified, one flipped bit rejected, and a 512-record
    sample checked bit-exact against the oracle."""
    import torch
    enet.set_lanes_per_record(0)
    n, L = 65536, 4096
    g = torch.Generator(device="cuda").manual_seed(2)
    pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device="cuda", generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device="cuda", generator=g)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda")
    b = enet.Batch(pt, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    ct = torch.empty_like(pt)
    tags = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, ct, tags)
    back = torch.empty_like(pt)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    b2 = enet.Batch(ct, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    ct[12345 * L + 77] ^= 4
    enet.aead_open(b2, back, tags, ok)
    okh = ok.cpu()
    assert int(okh.sum()) == n - 1 and int(okh[12345]) == 0
    assert torch.equal(back.view(n, L)[:12345], pt.view(n, L)[:12345])
    assert torch.equal(back.view(n, L)[12346:], pt.view(n, L)[12346:])
    ct[12345 * L + 77] ^= 4
    idx = np.linspace(0, n - 1, 512).astype(int)
    pth, cth, kh, nh, th = (t.cpu().numpy() for t in (pt, ct, keys, nonces, tags))
    for i in idx:
        c, t = oracle.aead_seal(kh[32 * i:32 * i + 32].tobytes(), nh[12 * i:12 * i + 12].tobytes(),
                                pth[i * L:(i + 1) * L].tobytes())
        assert cth[i * L:(i + 1) * L].tobytes() == c
        assert th[16 * i:16 * i + 16].tobytes() == t


# ------------------------------------------------------------------------------ SHA / HMAC
def test_sha256_golden(enet, golden):
    import torch
    cs = golden["sha256"]
    items = [b"abc" if c["abc"] else splitmix_bytes(c["seed"], c["len"]) for c in cs]
    offs = np.concatenate([[0], np.cumsum([len(x) for x in items])]).astype(np.int64)
    arena = dev(b"".join(items))
    dig = torch.zeros(32 * len(cs), dtype=torch.uint8, device="cuda")
    enet.sha256(arena, torch.tensor(offs).cuda(), dig)
    dh = host(dig)
    for i, c in enumerate(cs):
        assert dh[32 * i:32 * i + 32].hex() == c["digest"], c["len"]


def test_hmac_golden(enet, golden):
    import torch
    cs = golden["hmac"]
    items = [splitmix_bytes(c["seed"], c["len"]) for c in cs]
    keys = [bytes.fromhex(c["key"]) for c in cs]
    offs = np.concatenate([[0], np.cumsum([len(x) for x in items])]).astype(np.int64)
    koffs = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.int64)
    arena, karena = dev(b"".join(items)), dev(b"".join(keys) or b"\0")
    macs = torch.zeros(32 * len(cs), dtype=torch.uint8, device="cuda")
    to, tk = torch.tensor(offs).cuda(), torch.tensor(koffs).cuda()
    enet.hmac_sha256(karena, arena, to, macs, key_offsets=tk)
    mh = host(macs)
    for i, c in enumerate(cs):
        assert mh[32 * i:32 * i + 32].hex() == c["mac"], (len(keys[i]), c["len"])
    # verify: all good, then one corrupted
    ok = torch.zeros(len(cs), dtype=torch.uint8, device="cuda")
    macs[32 * 3] ^= 1
    enet.hmac_sha256_verify(karena, arena, to, macs, ok, key_offsets=tk)
    okh = ok.cpu().tolist()
    assert okh[3] == 0 and sum(okh) == len(cs) - 1


# ------------------------------------------------------------------------------ frames
@pytest.mark.parametrize("lanes", [1, 4])
def test_frames_golden(enet, golden, lanes):
    import torch
    enet.set_lanes_per_record(lanes)
    fs = golden["frames"]
    msgs = [bytes.fromhex(f["signed"])[:-32] for f in fs]
    keys = [bytes.fromhex(f["key"]) for f in fs]
    nonces = [bytes.fromhex(f["nonce"]) for f in fs]
    b = enet.make_batch(msgs, keys, nonces)
    ooffs = np.concatenate([[0], np.cumsum([len(m) + 32 for m in msgs])]).astype(np.int64)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    to = torch.tensor(ooffs).cuda()
    enet.frame_seal(b, out, to)
    bodies = records_of(host(out), ooffs.tolist())
    for f, body in zip(fs, bodies):
        assert body.hex() == f["body"]
    # open: good frames, one tampered, one too short
    bodies[1] = bytes([bodies[1][0] ^ 1]) + bodies[1][1:]
    bodies.append(b"\x01" * 20)
    keys.append(keys[0])
    nonces.append(nonces[0])
    bo = enet.make_batch(bodies, keys, nonces)
    poffs = np.concatenate([[0], np.cumsum([max(len(x) - 32, 0) for x in bodies])]).astype(np.int64)
    pt = torch.full((max(int(poffs[-1]), 1),), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * len(bodies), dtype=torch.uint8, device="cuda")
    ok = torch.zeros(len(bodies), dtype=torch.uint8, device="cuda")
    enet.frame_open(bo, pt, torch.tensor(poffs).cuda(), macs, ok)
    okh = ok.cpu().tolist()
    got = records_of(host(pt), poffs.tolist())
    for i in range(len(bodies)):
        if i in (1, len(bodies) - 1):
            assert okh[i] == 0
            assert got[i] == bytes(len(got[i]))
        else:
            assert okh[i] == 1 and got[i] == msgs[i]


@pytest.mark.parametrize("lanes", [1, 2, 16])
def test_frames_random_vs_oracle(enet, lanes):
    import torch
    enet.set_lanes_per_record(lanes)
    n = 200
    lens = rand_lengths(77, n, 2100)
    msgs = [splitmix_bytes(900 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(50000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(60000 + i, 12) for i in range(n)]
    b = enet.make_batch(msgs, keys, nonces, base_offset=1)
    ooffs = np.concatenate([[0], np.cumsum([L + 32 for L in lens])]).astype(np.int64)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    enet.frame_seal(b, out, torch.tensor(ooffs).cuda())
    bodies = records_of(host(out), ooffs.tolist())
    for i in range(n):
        assert bodies[i] == oracle.frame_seal(keys[i], nonces[i], msgs[i]), i


# ------------------------------------------------------------------------------ wire frames
def wire_of(nonce: bytes, body: bytes) -> bytes:
    """SessionManager::send framing (SessionManager.cpp:376-387): nonce || BE32(len) || body."""
    return nonce + len(body).to_bytes(4, "big") + body


def wire_open_batch(enet, frames, keys):
    import dataclasses

    import torch
    bo = dataclasses.replace(enet.make_batch(frames, keys, [b"\0" * 12] * len(frames),
                                             base_offset=3), nonces=None)
    poffs = np.concatenate([[0], np.cumsum([max(len(x) - 48, 0) for x in frames])]).astype(np.int64)
    pt = torch.full((max(int(poffs[-1]), 1),), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * len(frames), dtype=torch.uint8, device="cuda")
    ok = torch.zeros(len(frames), dtype=torch.uint8, device="cuda")
    enet.wire_open(bo, pt, torch.tensor(poffs).cuda(), macs, ok)
    return records_of(host(pt), poffs.tolist()), ok.cpu().tolist()


@pytest.mark.parametrize("lanes", [1, 4])
def test_wire_frames_golden(enet, golden, lanes):
    """Whole wire frames against the reference's encode_signed bodies plus its framing; the
    receive side rejects tampered bodies, wrong length fields, a tampered nonce and short frames."""
    import torch
    enet.set_lanes_per_record(lanes)
    fs = golden["frames"]
    msgs = [bytes.fromhex(f["signed"])[:-32] for f in fs]
    keys = [bytes.fromhex(f["key"]) for f in fs]
    nonces = [bytes.fromhex(f["nonce"]) for f in fs]
    b = enet.make_batch(msgs, keys, nonces, base_offset=1)
    ooffs = np.concatenate([[0], np.cumsum([len(m) + 48 for m in msgs])]).astype(np.int64)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    enet.wire_seal(b, out, torch.tensor(ooffs).cuda())
    frames = records_of(host(out), ooffs.tolist())
    for f, n, fr in zip(fs, nonces, frames):
        assert fr == wire_of(n, bytes.fromhex(f["body"]))
    good = len(frames)
    bad = [
        frames[0][:20] + bytes([frames[0][20] ^ 0x40]) + frames[0][21:],  # body bit flip
        frames[0][:12] + (len(frames[0]) - 15).to_bytes(4, "big") + frames[0][16:],  # length
        bytes([frames[0][0] ^ 1]) + frames[0][1:],  # nonce
        frames[0][:47],  # shorter than header + MAC
        frames[0][:10],  # shorter than the header
    ]
    got, okh = wire_open_batch(enet, frames + bad, keys + [keys[0]] * len(bad))
    for i in range(good):
        assert okh[i] == 1 and got[i] == msgs[i]
    for i in range(good, good + len(bad)):
        assert okh[i] == 0 and got[i] == bytes(len(got[i])), i


@pytest.mark.parametrize("lanes", [1, 2, 16])
def test_wire_frames_random_vs_oracle(enet, lanes):
    import torch
    enet.set_lanes_per_record(lanes)
    n = 300
    lens = rand_lengths(78, n, 3000)
    lens[:4] = [0, 1, 16, 1 << 14]
    msgs = [splitmix_bytes(1900 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(51000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(61000 + i, 12) for i in range(n)]
    b = enet.make_batch(msgs, keys, nonces, base_offset=5)
    ooffs = np.concatenate([[7], 7 + np.cumsum([L + 48 for L in lens])]).astype(np.int64)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    enet.wire_seal(b, out, torch.tensor(ooffs).cuda())
    frames = records_of(host(out), ooffs.tolist())
    for i in range(n):
        assert frames[i] == wire_of(nonces[i], oracle.frame_seal(keys[i], nonces[i], msgs[i])), i
    got, okh = wire_open_batch(enet, frames, keys)
    assert okh == [1] * n and got == msgs


# ------------------------------------------------------------------------------ uniform (COOP)
@pytest.mark.parametrize("staging", [1, 0, 4, 5])
@pytest.mark.parametrize("L,n,lanes", [(1500, 1000, 1), (1500, 517, 2), (4096, 300, 2),
                                       (4096, 129, 4), (65536, 40, 8), (65536, 33, 16),
                                       (640, 700, 1), (127, 300, 1), (64, 260, 1), (0, 10, 1),
                                       (1504, 300, 1), (1472, 300, 1), (1400, 300, 1),
                                       (200, 300, 1), (100, 260, 1), (80, 300, 1), (31, 300, 1),
                                       (17, 300, 1), (16, 300, 1), (15, 300, 1), (143, 300, 1),
                                       (132, 600, 1), (196, 600, 1), (192, 520, 1), (1000, 600, 1),
                                       (4100, 520, 1)])
def test_aead_uniform_batches_vs_oracle(enet, L, n, lanes, staging):
    """Uniform-length batches take the cooperative LDS-staged path (whole workgroups; staging
    variant 1 = default, 4 = run staging only, 5 = lockstep run staging) plus the per-lane path for the partial
    workgroup; 1500-byte records start unaligned and end in a partial block.  With one lane per
    record, staging 1 also moves the ragged end (odd block + partial block, >= 16 bytes)
    through LDS."""
    import torch
    enet.set_lanes_per_record(lanes)
    enet.set_staging(staging)
    items = [splitmix_bytes(70000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(80000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(90000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces)
    assert b.total_bytes_hint == n * L and b.max_len_hint == L
    out = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    got = records_of(host(out), b.offsets.cpu().tolist())
    th = host(tags)
    idx = range(n) if n * max(L, 1) <= 4 << 20 else np.linspace(0, n - 1, 64).astype(int)
    for i in idx:
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct, (i, L)
        assert th[16 * i:16 * i + 16] == tag, (i, L)
    # in place (out == in) gives the same ciphertext and tags
    inp = b.arena.clone()
    tags_ip = torch.zeros_like(tags)
    bi = enet.Batch(inp, b.offsets, b.keys, b.nonces, total_bytes_hint=n * L, max_len_hint=L)
    enet.aead_seal(bi, inp, tags_ip)
    assert torch.equal(inp, out) and torch.equal(tags_ip, tags)
    b2 = enet.Batch(out, b.offsets, b.keys, b.nonces, total_bytes_hint=n * L, max_len_hint=L)
    back = torch.zeros_like(out)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, back, tags, ok)
    assert int(ok.sum()) == n
    assert torch.equal(back, b.arena)
    if L and n > 6:  # a tampered record is rejected and zeroed, its neighbours are untouched
        bad = out.clone()
        o5 = int(b.offsets[5])
        bad[o5 + L - 1] ^= 1
        b3 = enet.Batch(bad, b.offsets, b.keys, b.nonces, total_bytes_hint=n * L, max_len_hint=L)
        back.fill_(0xAA)
        enet.aead_open(b3, back, tags, ok)
        okh = ok.cpu().tolist()
        assert okh[5] == 0 and sum(okh) == n - 1
        bh = records_of(host(back), b.offsets.cpu().tolist())
        assert bh[5] == bytes(L) and bh[4] == items[4] and bh[6] == items[6]
    # xor mode (reference ChaCha20::apply with per-record counters) on the same shape
    ctr = np.frombuffer(splitmix_bytes(L + n, 4 * n), dtype="<u4").copy()
    xo = out_like(b)
    enet.chacha20_xor(b, xo, counters=torch.tensor(ctr.view(np.int32)).cuda())
    xg = records_of(host(xo), b.offsets.cpu().tolist())
    for i in list(idx)[:64]:
        assert xg[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctr[i]))
    enet.set_staging(-1)


# ------------------------------------------------------------------------------ AEAD + HMAC (C5)
@pytest.mark.parametrize("lanes", [0, 1, 4])
def test_aead_hmac_mixed_vs_oracle(enet, lanes):
    """Mixed 512 B - 64 KiB records (log-uniform, C5 shape, small n): Poly1305 tag and
    HMAC-SHA256(key, plaintext) bit-exact; open verifies both and rejects either tampering."""
    import torch
    enet.set_lanes_per_record(lanes)
    n = 64
    rng = np.random.default_rng(123)
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), n)).astype(int).tolist()
    items = [splitmix_bytes(110000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(120000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(130000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces)
    out = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    enet.aead_hmac_seal(b, out, tags, macs)
    offs = b.offsets.cpu().tolist()
    got, th, mh = records_of(host(out), offs), host(tags), host(macs)
    for i in range(n):
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct and th[16 * i:16 * i + 16] == tag, i
        assert mh[32 * i:32 * i + 32] == oracle.hmac_sha256(keys[i], items[i]), i
    ct2 = out.clone()
    macs2 = macs.clone()
    ct2[offs[5] + 3] ^= 1        # poly1305 must reject record 5
    macs2[32 * 9 + 7] ^= 2       # hmac must reject record 9
    b2 = enet.Batch(ct2, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                    max_len_hint=b.max_len_hint)
    back = torch.full_like(out, 0x55)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_hmac_open(b2, back, tags, macs2, ok)
    okh = ok.cpu().tolist()
    bk = records_of(host(back), offs)
    for i in range(n):
        if i in (5, 9):
            assert okh[i] == 0 and bk[i] == bytes(len(bk[i]))
        else:
            assert okh[i] == 1 and bk[i] == items[i], i


def test_c1_single_key_gpu_cpu_roundtrips(enet):
    """1024 x 4 KiB, one session key (key_stride 0), per-record nonces.  GPU seal ->
    CPU (oracle) open, CPU seal -> GPU open, and the reference-mode ChaCha20 both ways."""
    import torch
    enet.set_lanes_per_record(0)
    n, L = 1024, 4096
    key = splitmix_bytes(1, 32)
    items = [splitmix_bytes(140000 + i, L) for i in range(n)]
    nonces = [splitmix_bytes(150000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, [key], nonces, key_stride=0)
    ct = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, ct, tags)
    cth, th = records_of(host(ct), b.offsets.cpu().tolist()), host(tags)
    for i in range(0, n, 7):
        ok, pt = oracle.aead_open(key, nonces[i], cth[i], th[16 * i:16 * i + 16])
        assert ok and pt == items[i]
    # CPU seal -> GPU open
    sealed = [oracle.aead_seal(key, nonces[i], items[i]) for i in range(n)]
    bo = enet.make_batch([s[0] for s in sealed], [key], nonces, key_stride=0)
    t2 = dev(b"".join(s[1] for s in sealed))
    back = out_like(bo)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(bo, back, t2, ok)
    assert int(ok.sum()) == n and torch.equal(back, b.arena)


# ------------------------------------------------------------------------------ uniform + AAD
@pytest.mark.parametrize("staging", [1, 4, 5])
@pytest.mark.parametrize("L,n,lanes", [(4096, 600, 2), (4096, 300, 1), (1500, 600, 1),
                                       (65536, 40, 16), (2048, 700, 4), (640, 600, 1)])
def test_aead_uniform_aad_vs_oracle(enet, L, n, lanes, staging):
    """Per-record AAD of assorted lengths on the staged / streaming paths: lane 0 absorbs the AAD
    before its run, the other lanes scale by r^e with e counting the AAD blocks.  Tags bit-exact
    against the oracle; a tampered AAD byte is rejected and that record zeroed."""
    import torch
    enet.set_lanes_per_record(lanes)
    enet.set_staging(staging)
    alens = [[0, 1, 12, 16, 17, 100][i % 6] for i in range(n)]
    items = [splitmix_bytes(71000 + i, L) for i in range(n)]
    aads = [splitmix_bytes(72000 + i, a) for i, a in enumerate(alens)]
    keys = [splitmix_bytes(73000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(74000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces)
    aoff = torch.tensor(np.concatenate([[0], np.cumsum(alens)]).astype(np.int64)).cuda()
    aad = dev(b"".join(aads))
    out = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags, aad, aoff)
    got = records_of(host(out), b.offsets.cpu().tolist())
    th = host(tags)
    idx = range(n) if n * L <= 4 << 20 else np.linspace(0, n - 1, 96).astype(int)
    for i in idx:
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i], aads[i])
        assert got[i] == ct, (i, L)
        assert th[16 * i:16 * i + 16] == tag, (i, L, alens[i])
    b2 = enet.Batch(out, b.offsets, b.keys, b.nonces, total_bytes_hint=n * L, max_len_hint=L)
    back = torch.zeros_like(out)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, back, tags, ok, aad, aoff)
    assert int(ok.sum()) == n and torch.equal(back, b.arena)
    bad_aad = aad.clone()
    k = 5 if alens[5] else 4
    bad_aad[int(aoff[k])] ^= 0x10
    back.fill_(0xAA)
    enet.aead_open(b2, back, tags, ok, bad_aad, aoff)
    okh = ok.cpu().tolist()
    assert okh[k] == 0 and sum(okh) == n - 1
    bh = records_of(host(back), b.offsets.cpu().tolist())
    assert bh[k] == bytes(L) and bh[k + 1] == items[k + 1]
    enet.set_staging(-1)


# ------------------------------------------------------------------------------ lying hints
@pytest.mark.parametrize("staging", [1, 4, 5])
@pytest.mark.parametrize("L,lanes", [(4096, 2), (4096, 1), (1500, 1), (65536, 16), (2048, 4)])
def test_lying_hints_give_correct_bytes(enet, L, lanes, staging):
    """The hints say uniform (total == n * max_len_hint) but two records are 64 bytes shorter /
    longer than max_len_hint: the staged and streaming paths address records at in_off[0] + g L,
    so the workgroups holding them must notice and take the per-lane path.  Every record stays
    bit-exact (seal, open, ChaCha20 xor)."""
    import torch
    enet.set_lanes_per_record(lanes)
    enet.set_staging(staging)
    n = max(600, (4 << 20) // L) if L < 65536 else 72
    lens = [L] * n
    lens[n // 3] -= 64
    lens[n // 3 + 7] += 64           # total still n * L; the true maximum is L + 64
    items = [splitmix_bytes(75000 + i, x) for i, x in enumerate(lens)]
    keys = [splitmix_bytes(76000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(77000 + i, 12) for i in range(n)]
    b0 = enet.make_batch(items, keys, nonces)
    b = enet.Batch(b0.arena, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    out = out_like(b)
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    offs = b.offsets.cpu().tolist()
    got = records_of(host(out), offs)
    th = host(tags)
    idx = sorted(set(list(range(0, n, max(1, n // 64))) + [n // 3 - 1, n // 3, n // 3 + 1,
                                                            n // 3 + 7, n // 3 + 8, n - 1]))
    for i in idx:
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct, (i, lens[i])
        assert th[16 * i:16 * i + 16] == tag, (i, lens[i])
    b2 = enet.Batch(out, b.offsets, b.keys, b.nonces, total_bytes_hint=n * L, max_len_hint=L)
    back = torch.zeros_like(out)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, back, tags, ok)
    assert int(ok.sum()) == n and torch.equal(back, b.arena)
    xo = out_like(b)
    enet.chacha20_xor(b, xo)
    xg = records_of(host(xo), offs)
    for i in idx:
        assert xg[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], 0), i
    enet.set_staging(-1)


# ------------------------------------------------------------------------------ full-size shapes
@pytest.mark.parametrize("n,L", [(1048576, 1500), (32768, 65536)])
def test_aead_roundtrip_full_size(enet, n, L):
    """C3 (1 M x 1500 B: the line-staging path's 32-bit line offsets reach 1.57 GB) and the C4
    per-GPU share (32 768 x 64 KiB, 2 GiB: the streaming kernel's 32-bit offsets) at full size:
    open(seal(x)) == x with every tag verified, one flipped bit rejected with its record zeroed,
    and a 512-record oracle sample bit-exact."""
    import torch
    enet.set_lanes_per_record(0)
    enet.set_staging(-1)
    g = torch.Generator(device="cuda").manual_seed(3)
    pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device="cuda", generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device="cuda", generator=g)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device="cuda")
    b = enet.Batch(pt, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    ct = torch.empty_like(pt)
    tags = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, ct, tags)
    idx = np.linspace(0, n - 1, 512).astype(int)
    rows = torch.tensor(idx, device="cuda")
    pth = pt.view(n, L)[rows].cpu().numpy()
    cth = ct.view(n, L)[rows].cpu().numpy()
    kh = keys.view(n, 32)[rows].cpu().numpy()
    nh = nonces.view(n, 12)[rows].cpu().numpy()
    th = tags.view(n, 16)[rows].cpu().numpy()
    for r in range(len(idx)):
        c, t = oracle.aead_seal(kh[r].tobytes(), nh[r].tobytes(), pth[r].tobytes())
        assert cth[r].tobytes() == c, idx[r]
        assert th[r].tobytes() == t, idx[r]
    victim = n - 5
    ct[victim * L + L // 2] ^= 0x80
    back = torch.empty_like(pt)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    b2 = enet.Batch(ct, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    enet.aead_open(b2, back, tags, ok)
    okh = ok.cpu()
    assert int(okh.sum()) == n - 1 and int(okh[victim]) == 0
    bv, pv = back.view(n, L), pt.view(n, L)
    assert torch.equal(bv[:victim], pv[:victim]) and torch.equal(bv[victim + 1:], pv[victim + 1:])
    assert int(bv[victim].count_nonzero()) == 0


@pytest.mark.parametrize("shift", [4, 64, 100])
def test_aead_uniform_out_arena_phase(enet, shift):
    """1500-byte uniform records whose output arena starts at another 128-byte phase than the input
    arena: the line-staging path cannot be used and the workgroups take the per-lane path (which
    must still derive the one-time Poly1305 key)."""
    import torch
    enet.set_lanes_per_record(1)
    enet.set_staging(-1)
    n, L = 1024, 1500
    items = [splitmix_bytes(78000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(79000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(79500 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces)
    big = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    out = big[shift:shift + n * L]
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    got = records_of(host(out), b.offsets.cpu().tolist())
    th = host(tags)
    for i in range(0, n, 7):
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct and th[16 * i:16 * i + 16] == tag, i


@pytest.mark.parametrize("ishift,oshift", [(4, 4), (8, 100), (0, 12), (64, 0)])
def test_stream_kernel_unaligned_arenas(enet, ishift, oshift):
    """The headline streaming kernel (C2 shape: 4 KiB records, two lanes each, whole 512-lane
    workgroups) with input / output arenas that start off 16-byte alignment: its LDS DMAs and
    whole-run stores then take unaligned 16-byte pieces.  Bit-exact against the oracle (seal and
    the reference-mode ChaCha20), open(seal(x)) == x, and a tampered record rejected and zeroed."""
    import torch
    enet.set_lanes_per_record(2)
    enet.set_staging(-1)
    n, L = 768, 4096
    items = [splitmix_bytes(91000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(92000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(93000 + i, 12) for i in range(n)]
    b0 = enet.make_batch(items, keys, nonces)
    ibig = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    ibig[ishift:ishift + n * L] = b0.arena
    src = ibig[ishift:ishift + n * L]
    b = enet.Batch(src, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    obig = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    out = obig[oshift:oshift + n * L]
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    offs = b0.offsets.cpu().tolist()
    got, th = records_of(host(out), offs), host(tags)
    for i in list(range(0, n, 37)) + [n - 1]:
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct and th[16 * i:16 * i + 16] == tag, i
    assert int(obig[:oshift].count_nonzero()) == 0 and int(obig[oshift + n * L:].count_nonzero()) == 0
    b2 = enet.Batch(out, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    bbig = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    back = bbig[ishift:ishift + n * L]
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, back, tags, ok)
    assert int(ok.sum()) == n and torch.equal(back, src)
    bad = out.clone()
    bad[offs[300] + 2049] ^= 4
    b3 = enet.Batch(bad, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    enet.aead_open(b3, back, tags, ok)
    okh = ok.cpu().tolist()
    assert okh[300] == 0 and sum(okh) == n - 1
    bh = records_of(host(back), offs)
    assert bh[300] == bytes(L) and bh[299] == items[299] and bh[301] == items[301]
    xo = obig[oshift:oshift + n * L]
    enet.chacha20_xor(b, xo)
    xg = records_of(host(xo), offs)
    for i in range(0, n, 97):
        assert xg[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], 0), i
    enet.set_lanes_per_record(0)


@pytest.mark.parametrize("L", [1500, 1436, 1284, 260, 132, 196, 4100, 1504, 1496, 136, 4092])
@pytest.mark.parametrize("ishift,oshift", [(0, 0), (4, 4), (8, 100), (0, 12), (64, 0), (2, 0), (0, 1)])
def test_uniform_one_lane_shapes(enet, L, ishift, oshift):
    """Uniform one-lane batches whose length is not a multiple of 128 (C3 class: line staging over
    whole workgroups, the rest per lane): record starts at every 4-byte phase of a line (L mod 16 =
    12, 4, 0, 8), two to 33 stages, tails of 4 to 124 bytes, arenas off alignment (in / out phases
    that differ, or a 2- or 1-byte shift, take the per-lane path).  Seal bit-exact against the oracle
    at every record of the first workgroup's edges and a sample, nothing written outside the
    output arena, open(seal(x)) == x, a tampered record (first, middle and last unit) rejected
    and zeroed with its neighbours intact, and reference-mode ChaCha20 with counters at the
    u32 wrap."""
    import torch
    enet.set_lanes_per_record(1)
    enet.set_staging(-1)
    n = 1100
    items = [splitmix_bytes(94000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(95000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(96000 + i, 12) for i in range(n)]
    b0 = enet.make_batch(items, keys, nonces)
    ibig = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    ibig[ishift:ishift + n * L] = b0.arena
    src = ibig[ishift:ishift + n * L]
    b = enet.Batch(src, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    obig = torch.full((n * L + 256,), 0x5A, dtype=torch.uint8, device="cuda")
    out = obig[oshift:oshift + n * L]
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    enet.aead_seal(b, out, tags)
    offs = b0.offsets.cpu().tolist()
    got, th = records_of(host(out), offs), host(tags)
    idx = sorted(set(list(range(0, 70)) + list(range(440, 580)) + list(range(1000, n)) +
                     list(range(0, n, 13))))
    for i in idx:
        ct, tag = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert got[i] == ct, (i, L)
        assert th[16 * i:16 * i + 16] == tag, (i, L)
    ob = host(obig)
    assert ob[:oshift] == b"\x5a" * oshift and ob[oshift + n * L:] == b"\x5a" * (256 - oshift)
    b2 = enet.Batch(out, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    bbig = torch.zeros(n * L + 256, dtype=torch.uint8, device="cuda")
    back = bbig[ishift:ishift + n * L]
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(b2, back, tags, ok)
    assert int(ok.sum()) == n and torch.equal(back, src)
    bad = out.clone()
    for v, pos in ((3, 0), (300, L // 2), (511, L - 1), (513, 5)):
        bad[offs[v] + pos] ^= 4
    b3 = enet.Batch(bad, b0.offsets, b0.keys, b0.nonces, total_bytes_hint=n * L, max_len_hint=L)
    back.fill_(0xAA)
    enet.aead_open(b3, back, tags, ok)
    okh = ok.cpu().tolist()
    assert [i for i in range(n) if okh[i] == 0] == [3, 300, 511, 513]
    bh = records_of(host(back), offs)
    for v in (3, 300, 511, 513):
        assert bh[v] == bytes(L) and bh[v - 1] == items[v - 1] and bh[v + 1] == items[v + 1], v
    ctr = np.full(n, 0xFFFFFFF0, dtype=np.uint32)
    ctr[::3] = np.arange(0, n, 3, dtype=np.uint32)
    xo = obig[oshift:oshift + n * L]
    enet.chacha20_xor(b, xo, counters=torch.tensor(ctr.view(np.int32)).cuda())
    xg = records_of(host(xo), offs)
    for i in idx[::3]:
        assert xg[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctr[i])), i
    enet.set_lanes_per_record(0)
