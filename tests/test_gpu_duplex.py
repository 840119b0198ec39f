"""GPU parity of the one-pass duplex kernel (duplex.hip) against the CPU oracle, for the shapes
the round-1 fused kernel could not take: ragged lengths (MTU frames of 1500 / 1452 / 100 B),
mixed lengths in one batch, any record alignment, a caller `order`, records of invalid geometry,
and the AEAD + HMAC-SHA256 path of BASELINE config 5.  Every case is also run through the
two-pass path (staging variant 0) and must give the same bytes.  Reference: SessionManager::send
/ receive (src/network/SessionManager.cpp:362-387, :760-822), encode_signed / decode_signed
(src/protocol/Message.cpp:305-328), Node::store_chunk / fetch_chunk (src/core/Node.cpp:1414-1417,
1644-1655), HmacSha256.cpp:11-54.  Bit-exact comparisons throughout."""
import dataclasses

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


def records_of(arena_bytes: bytes, offs):
    return [arena_bytes[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]


def wire_of(nonce: bytes, body: bytes) -> bytes:
    return nonce + len(body).to_bytes(4, "big") + body


def offsets_for(lens, base):
    return np.concatenate([[base], base + np.cumsum(lens)]).astype(np.int64)


def seal_frames(enet, msgs, keys, nonces, hdr, base, order=None, key_stride=32):
    import torch
    b = enet.make_batch(msgs, keys, nonces, base_offset=base, key_stride=key_stride)
    if order is not None:
        b = dataclasses.replace(b, order=torch.tensor(order, dtype=torch.int32, device="cuda"))
    ooffs = offsets_for([len(m) + 32 + hdr for m in msgs], base + 1)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    (enet.wire_seal if hdr else enet.frame_seal)(b, out, torch.tensor(ooffs).cuda())
    return records_of(host(out), ooffs.tolist())


def open_frames(enet, frames, keys, nonces, hdr, base, order=None, key_stride=32, out_lens=None):
    import torch
    b = enet.make_batch(frames, keys, nonces, base_offset=base, key_stride=key_stride)
    if hdr:
        b = dataclasses.replace(b, nonces=None)
    if order is not None:
        b = dataclasses.replace(b, order=torch.tensor(order, dtype=torch.int32, device="cuda"))
    lens = out_lens if out_lens is not None else [max(len(f) - 32 - hdr, 0) for f in frames]
    poffs = offsets_for(lens, 2)
    pt = torch.full((int(poffs[-1]) + 1,), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * len(frames), dtype=torch.uint8, device="cuda")
    ok = torch.zeros(len(frames), dtype=torch.uint8, device="cuda")
    (enet.wire_open if hdr else enet.frame_open)(b, pt, torch.tensor(poffs).cuda(), macs, ok)
    return records_of(host(pt), poffs.tolist()), ok.cpu().tolist(), host(macs)


def both_paths(enet, fn):
    """fn() through the duplex kernel, then through the two-pass path (staging 0)."""
    enet.set_staging(-1)
    a = fn()
    enet.set_staging(0)
    try:
        b = fn()
    finally:
        enet.set_staging(-1)
    return a, b


# ------------------------------------------------------------------------------ frames
@pytest.mark.parametrize("hdr", [16, 0])
@pytest.mark.parametrize("L,n,base", [(1500, 600, 0), (1452, 300, 3), (100, 513, 1), (1, 260, 0),
                                      (0, 257, 2), (127, 256, 0), (129, 300, 7), (1535, 260, 0),
                                      (1408, 256, 5), (4096, 300, 0), (96, 300, 0), (97, 256, 0)])
def test_ragged_frames_vs_oracle(enet, hdr, L, n, base):
    """Uniform batches whose length is not a multiple of 128 B (the MTU case):
    seal = oracle, open round-trips with ok = 1 and the decrypted MACs, two-pass agrees."""
    msgs = [splitmix_bytes(17000 + 7 * L + i, L) for i in range(n)]
    keys = [splitmix_bytes(18000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(19000 + i, 12) for i in range(n)]
    frames, frames2 = both_paths(enet, lambda: seal_frames(enet, msgs, keys, nonces, hdr, base))
    assert frames == frames2
    for i in range(n):
        body = oracle.frame_seal(keys[i], nonces[i], msgs[i])
        assert frames[i] == (wire_of(nonces[i], body) if hdr else body), i
    res, res2 = both_paths(enet, lambda: open_frames(enet, frames, keys, nonces, hdr, base))
    got, ok, macs = res
    assert ok == [1] * n and got == msgs
    assert res2 == res
    for i in range(0, n, 37):
        dec = oracle.chacha20_xor(keys[i], nonces[i], frames[i][hdr:], 0)
        assert macs[32 * i:32 * i + 32] == dec[L:], i


@pytest.mark.parametrize("hdr", [16, 0])
def test_mixed_frames_with_order_vs_oracle(enet, hdr):
    """One batch of mixed lengths 0..5000 (plus a 64 KiB and a 1 MiB frame, SessionManager's
    kMaxPayloadSize), processed in a caller-given order (length-sorted), unaligned arena."""
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 5000, 700).tolist() + [65536, (1 << 20) - 32 - hdr, 0, 1, 127, 128, 129]
    n = len(lens)
    msgs = [splitmix_bytes(21000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(22000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(23000 + i, 12) for i in range(n)]
    order = np.argsort(np.array(lens), kind="stable")[::-1].astype(np.int32).copy()
    frames, frames2 = both_paths(enet, lambda: seal_frames(enet, msgs, keys, nonces, hdr, 3, order))
    assert frames == frames2
    for i in range(n):
        body = oracle.frame_seal(keys[i], nonces[i], msgs[i])
        assert frames[i] == (wire_of(nonces[i], body) if hdr else body), i
    got, ok, _ = open_frames(enet, frames, keys, nonces, hdr, 1, order)
    assert ok == [1] * n and got == msgs
    # no order: same bytes
    got2, ok2, _ = open_frames(enet, frames, keys, nonces, hdr, 0)
    assert ok2 == [1] * n and got2 == msgs


@pytest.mark.parametrize("hdr", [16, 0])
def test_ragged_frames_reject_tampered(enet, hdr):
    """Flips in the ragged end (last message byte, every MAC byte position), the first stage and
    (wire) the header fail with ok = 0 and a zeroed message; neighbours are untouched; frames
    shorter than [hdr] + MAC fail too."""
    n, L = 300, 1500
    msgs = [splitmix_bytes(31000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(32000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(33000 + i, 12) for i in range(n)]
    frames = seal_frames(enet, msgs, keys, nonces, hdr, 0)
    bad = list(frames)

    def flip(i, pos):
        f = bytearray(bad[i])
        f[pos] ^= 0x04
        bad[i] = bytes(f)

    tampered = set()
    for k, pos in enumerate([hdr + L - 1, hdr + 1408, hdr + 0] + [hdr + L + j for j in range(32)]):
        flip(3 + 2 * k, pos)
        tampered.add(3 + 2 * k)
    if hdr:
        flip(200, 14)
        flip(201, 5)
        tampered |= {200, 201}
    got, ok, _ = open_frames(enet, bad, keys, nonces, hdr, 0)
    for i in range(n):
        if i in tampered:
            assert ok[i] == 0 and got[i] == bytes(L), i
        else:
            assert ok[i] == 1 and got[i] == msgs[i], i
    short = [frames[0][:hdr + 31], frames[1][:hdr], frames[2]]
    got, ok, _ = open_frames(enet, short, keys[:3], nonces[:3], hdr, 0)
    assert ok == [0, 0, 1] and got[2] == msgs[2] and got[0] == b"" and got[1] == b""


def test_frames_invalid_geometry(enet):
    """An output range of the wrong size (not |in| + 32 + hdr on seal, not |in| - 32 - hdr on
    open) is not processed: it is zeroed, and open reports ok = 0; the other records are fine."""
    import torch
    n, L = 260, 700
    msgs = [splitmix_bytes(41000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(42000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(43000 + i, 12) for i in range(n)]
    b = enet.make_batch(msgs, keys, nonces)
    lens = [L + 32] * n
    lens[7] = L + 31
    lens[8] = L + 40
    ooffs = offsets_for(lens, 0)
    out = torch.full((int(ooffs[-1]),), 0x5A, dtype=torch.uint8, device="cuda")
    enet.frame_seal(b, out, torch.tensor(ooffs).cuda())
    bodies = records_of(host(out), ooffs.tolist())
    for i in range(n):
        if i in (7, 8):
            assert bodies[i] == bytes(lens[i]), i
        else:
            assert bodies[i] == oracle.frame_seal(keys[i], nonces[i], msgs[i]), i
    good = [oracle.frame_seal(keys[i], nonces[i], msgs[i]) for i in range(n)]
    out_lens = [L] * n
    out_lens[9] = L - 1
    got, ok, _ = open_frames(enet, good, keys, nonces, 0, 0, out_lens=out_lens)
    for i in range(n):
        assert (ok[i], got[i]) == ((0, bytes(L - 1)) if i == 9 else (1, msgs[i])), i


def test_frames_decreasing_offsets(enet):
    """Output offsets that DECREASE (out_off[k+1] < out_off[k]) must not wrap the record length:
    record k is skipped (nothing written for it), the records whose range is merely the wrong
    size are zeroed as usual, and everything else -- including the guard bytes past the arena --
    is untouched (Lo was never bounds-checked)."""
    import torch
    n, L = 300, 500
    msgs = [splitmix_bytes(44000 + i, L) for i in range(n)]
    keys = [splitmix_bytes(45000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(46000 + i, 12) for i in range(n)]
    b = enet.make_batch(msgs, keys, nonces)
    ooffs = offsets_for([L + 32] * n, 0)
    ooffs[11] = ooffs[10] - 5          # record 10: end < start; record 11: too long
    total = int(ooffs[-1])
    out = torch.full((total + 4096,), 0x5A, dtype=torch.uint8, device="cuda")
    enet.frame_seal(b, out, torch.tensor(ooffs).cuda())
    ob = host(out)
    assert ob[total:] == b"\x5a" * 4096
    for i in range(n):
        if i in (10, 11):
            continue
        want = oracle.frame_seal(keys[i], nonces[i], msgs[i])
        if i == 9:  # record 11's zeroed range starts 5 bytes inside record 9
            assert ob[ooffs[9]:ooffs[10] - 5] == want[:-5]
            continue
        assert ob[ooffs[i]:ooffs[i + 1]] == want, i
    # (its first 5 bytes are also record 9's last 5: either writer may land last)
    assert ob[ooffs[11] + 5:ooffs[12]] == bytes(int(ooffs[12] - ooffs[11] - 5))
    # open with a decreasing pair: ok = 0 for the disordered record, nothing written past the arena
    good = [oracle.frame_seal(keys[i], nonces[i], msgs[i]) for i in range(n)]
    bw = enet.make_batch(good, keys, nonces)
    poffs = offsets_for([L] * n, 0)
    poffs[21] = poffs[20] - 3
    pt = torch.full((int(poffs[-1]) + 4096,), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ok = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    enet.frame_open(bw, pt, torch.tensor(poffs).cuda(), macs, ok)
    okl = ok.cpu().tolist()
    pb = host(pt)
    assert pb[int(poffs[-1]):] == b"\xaa" * 4096
    for i in range(n):
        if i in (20, 21):
            assert okl[i] == 0, i
        elif i == 19:  # record 21's zeroed range starts 3 bytes inside record 19
            assert okl[i] == 1 and pb[poffs[19]:poffs[20] - 3] == msgs[19][:-3]
        else:
            assert okl[i] == 1 and pb[poffs[i]:poffs[i + 1]] == msgs[i], i


@pytest.mark.parametrize("n,L", [(1 << 20, 1500)])
def test_wire_frames_full_c3_roundtrip(enet, n, L):
    """C3 at full size (1 M x 1500 B MTU frames -> 1548-byte wire frames): open(seal(m)) == m with
    every MAC verified, a flipped bit rejected, and a 512-frame oracle sample."""
    import torch
    g = torch.Generator(device="cuda").manual_seed(11)
    pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device="cuda", generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device="cuda", generator=g)
    ioff = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    F = L + 48
    foff = torch.arange(n + 1, dtype=torch.int64, device="cuda") * F
    b = enet.Batch(pt, ioff, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    wire = torch.zeros(n * F, dtype=torch.uint8, device="cuda")
    enet.wire_seal(b, wire, foff)
    bw = enet.Batch(wire, foff, keys, None, total_bytes_hint=n * F, max_len_hint=F)
    back = torch.zeros_like(pt)
    macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.wire_open(bw, back, ioff, macs, ok)
    assert int(ok.sum()) == n and torch.equal(back, pt)
    idx = np.linspace(0, n - 1, 512).astype(int)
    ph, wh, kh, nh = (t.cpu().numpy().tobytes() for t in (pt, wire, keys, nonces))
    for i in idx:
        m, k, nn = ph[i * L:(i + 1) * L], kh[32 * i:32 * i + 32], nh[12 * i:12 * i + 12]
        assert wh[i * F:(i + 1) * F] == wire_of(nn, oracle.frame_seal(k, nn, m)), i
    wire[(n - 3) * F + 16 + L + 5] ^= 1
    enet.wire_open(bw, back, ioff, macs, ok)
    assert int(ok.sum()) == n - 1 and int(ok[n - 3]) == 0
    assert torch.count_nonzero(back[(n - 3) * L:(n - 2) * L]).item() == 0


@pytest.fixture(params=[-1, 0, 1], ids=["split-auto", "split-off", "split-on"])
def split(enet, request):
    """Chunk and AEAD+HMAC duplex paths with each record split over cipher / schedule / rounds
    waves (duplex_split.hip) forced on, off, or automatic (longest record >= 16 KiB)."""
    enet.set_duplex_split(request.param)
    yield request.param
    enet.set_duplex_split(-1)


# ------------------------------------------------------------------------------ chunks
@pytest.mark.parametrize("L,n,base", [(4000, 300, 0), (100, 260, 3), (65536, 40, 0), (4096, 300, 1)])
def test_ragged_chunks_vs_oracle(enet, split, L, n, base):
    """Chunk store / fetch with given ids at ragged and 64 KiB lengths: ciphertext from counter
    LE32(id), digests = SHA-256(pt), fetch verifies and zeroes a tampered chunk; two-pass agrees."""
    import torch
    items = [splitmix_bytes(51000 + 3 * L + i, L) for i in range(n)]
    keys = [splitmix_bytes(52000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(53000 + i, 12) for i in range(n)]
    ids = [splitmix_bytes(54000 + i, 32) for i in range(n)]
    b = enet.make_batch(items, keys, nonces, base_offset=base)
    idt = torch.frombuffer(bytearray(b"".join(ids)), dtype=torch.uint8).cuda()

    def store():
        out = torch.zeros_like(b.arena)
        hashes = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
        enet.chunk_store(b, out, hashes, chunk_ids=idt)
        return host(out), host(hashes)

    (ct, hs), (ct2, hs2) = both_paths(enet, store)
    assert ct == ct2 and hs == hs2
    offs = b.offsets.cpu().tolist()
    cts = records_of(ct, offs)
    import hashlib
    for i in range(n):
        ctr = int.from_bytes(ids[i][:4], "little")
        assert cts[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], ctr), i
        assert hs[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest(), i
    cta = torch.frombuffer(bytearray(ct), dtype=torch.uint8).cuda()
    cta[offs[4] + max(L - 1, 0)] ^= 1
    bf = enet.Batch(cta, b.offsets, b.keys, b.nonces)
    hst = torch.frombuffer(bytearray(hs), dtype=torch.uint8).cuda()

    def fetch():
        back = torch.full_like(b.arena, 0x33)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        enet.chunk_fetch(bf, back, idt, hst, ok)
        return host(back), ok.cpu().tolist()

    (pb, ok), (pb2, ok2) = both_paths(enet, fetch)
    assert ok == ok2 and ok == [0 if i == 4 else 1 for i in range(n)]
    got = records_of(pb, offs)
    for i in range(n):
        assert got[i] == (bytes(L) if i == 4 else items[i]), i


# ------------------------------------------------------------------------------ AEAD + HMAC (C5)
@pytest.mark.parametrize("sort", [False, True])
def test_aead_hmac_c5_mixed_vs_oracle(enet, split, sort):
    """C5 shape (log-uniform 512 B - 64 KiB) in one pass, optionally length-sorted through
    `order`: tags and HMACs bit-exact, open verifies both, either tampering zeroes the record;
    the two-pass path agrees."""
    import torch
    n = 300
    rng = np.random.default_rng(99)
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), n)).astype(int).tolist()
    lens[:3] = [512, 65536, 1000]
    items = [splitmix_bytes(61000 + i, L) for i, L in enumerate(lens)]
    keys = [splitmix_bytes(62000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(63000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces, base_offset=1)
    if sort:
        order = np.argsort(np.array(lens), kind="stable")[::-1].astype(np.int32).copy()
        b = dataclasses.replace(b, order=torch.tensor(order, device="cuda"))

    def seal():
        out = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
        enet.aead_hmac_seal(b, out, tags, macs)
        return host(out), host(tags), host(macs)

    (ct, th, mh), second = both_paths(enet, seal)
    assert (ct, th, mh) == second
    offs = b.offsets.cpu().tolist()
    cts = records_of(ct, offs)
    for i in range(n):
        c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
        assert cts[i] == c and th[16 * i:16 * i + 16] == t, i
        assert mh[32 * i:32 * i + 32] == oracle.hmac_sha256(keys[i], items[i]), i
    cta = torch.frombuffer(bytearray(ct), dtype=torch.uint8).cuda()
    tt = torch.frombuffer(bytearray(th), dtype=torch.uint8).cuda()
    mt = torch.frombuffer(bytearray(mh), dtype=torch.uint8).cuda()
    cta[offs[5] + lens[5] - 1] ^= 1   # Poly1305 rejects 5 (last byte: the ragged end)
    mt[32 * 9 + 31] ^= 2              # HMAC rejects 9
    tt[16 * 11] ^= 1                  # tag rejects 11
    b2 = dataclasses.replace(b, arena=cta)

    def open_():
        back = torch.full_like(b.arena, 0x55)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        enet.aead_hmac_open(b2, back, tt, mt, ok)
        return host(back), ok.cpu().tolist()

    (pb, ok), second = both_paths(enet, open_)
    assert (pb, ok) == second
    got = records_of(pb, offs)
    for i in range(n):
        if i in (5, 9, 11):
            assert ok[i] == 0 and got[i] == bytes(lens[i]), i
        else:
            assert ok[i] == 1 and got[i] == items[i], i


# every ragged-end shape of the split kernel: tail 0..127 bytes (1, 2 or 3 final SHA-256 blocks:
# r + 9 <= 64, <= 128, > 128), whole stages, empty records, a record of the wrong output size
EDGE_LENS = [0, 1, 15, 16, 55, 56, 63, 64, 65, 119, 120, 127, 128, 129, 183, 184, 191, 192, 255, 256,
             257, 383, 1000, 1500, 4095, 4096, 16384, 20000 + 37, 65536]


@pytest.mark.parametrize("kind", ["chunk", "aeadh"])
@pytest.mark.parametrize("base", [0, 3])
def test_split_kernel_edge_lengths_vs_oracle(enet, kind, base):
    """duplex_split.hip forced on: bit-exact ciphertext, SHA-256 / HMAC and Poly1305 tags for
    every tail shape, in-order and reversed (caller order); open verifies and rejects a flipped
    last byte per record shape; a record whose output range is the wrong size is zeroed (ok 0)."""
    import hashlib
    import torch
    enet.set_duplex_split(1)
    try:
        lens = EDGE_LENS * 3
        n = len(lens)
        items = [splitmix_bytes(71000 + i, L) for i, L in enumerate(lens)]
        keys = [splitmix_bytes(72000 + i, 32) for i in range(n)]
        nonces = [splitmix_bytes(73000 + i, 12) for i in range(n)]
        ids = [splitmix_bytes(74000 + i, 32) for i in range(n)]
        b = enet.make_batch(items, keys, nonces, base_offset=base)
        order = torch.tensor(list(range(n))[::-1], dtype=torch.int32, device="cuda")
        b = dataclasses.replace(b, order=order)
        idt = torch.frombuffer(bytearray(b"".join(ids)), dtype=torch.uint8).cuda()
        offs = b.offsets.cpu().tolist()
        out = torch.zeros_like(b.arena)
        d1 = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        d2 = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
        if kind == "chunk":
            enet.chunk_store(b, out, d2, chunk_ids=idt)
        else:
            enet.aead_hmac_seal(b, out, d1, d2)
        cts = records_of(host(out), offs)
        h1, h2 = host(d1), host(d2)
        for i in range(n):
            if kind == "chunk":
                ctr = int.from_bytes(ids[i][:4], "little")
                assert cts[i] == oracle.chacha20_xor(keys[i], nonces[i], items[i], ctr), (i, lens[i])
                assert h2[32 * i:32 * i + 32] == hashlib.sha256(items[i]).digest(), (i, lens[i])
            else:
                c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
                assert cts[i] == c and h1[16 * i:16 * i + 16] == t, (i, lens[i])
                assert h2[32 * i:32 * i + 32] == oracle.hmac_sha256(keys[i], items[i]), (i, lens[i])
        # open: flip the last byte of every third non-empty record
        cta = torch.frombuffer(bytearray(host(out)), dtype=torch.uint8).cuda()
        bad = {i for i in range(0, n, 3) if lens[i] > 0}
        for i in bad:
            cta[offs[i] + lens[i] - 1] ^= 0x40
        b2 = dataclasses.replace(b, arena=cta)
        back = torch.full_like(b.arena, 0x77)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        if kind == "chunk":
            enet.chunk_fetch(b2, back, idt, d2, ok)
        else:
            enet.aead_hmac_open(b2, back, d1, d2, ok)
        got = records_of(host(back), offs)
        okl = ok.cpu().tolist()
        for i in range(n):
            if i in bad:
                assert okl[i] == 0 and got[i] == bytes(lens[i]), (i, lens[i])
            else:
                assert okl[i] == 1 and got[i] == items[i], (i, lens[i])
        # wrong output size (AEAD + HMAC seal): record 7's output range one byte short -> zeroed
        ooffs = np.array(offs, dtype=np.int64)
        ooffs[8:] -= 1
        o2 = torch.full((int(ooffs[-1]) + 64,), 0x5A, dtype=torch.uint8, device="cuda")
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
        r = dataclasses.replace(b, order=None).records(o2, torch.tensor(ooffs).cuda())
        import ctypes as C
        if kind == "aeadh":
            assert enet.lib().enet_aead_hmac_seal_batch(C.byref(r), enet._ptr(tags), enet._ptr(macs),
                                                        enet._stream(None)) == 0
            ob = host(o2)
            seg = records_of(ob, ooffs.tolist())
            assert seg[7] == bytes(len(seg[7]))
            for i in (6, 9, 20):
                c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
                assert seg[i] == c, i
    finally:
        enet.set_duplex_split(-1)


def test_wire_frames_sessions_vs_per_frame_keys(enet):
    """Session-keyed wire frames (enet_wire_seal/open_batch_sessions): a table
    of 37 session keys, frames filed under sessions at random, the sessions' HMAC midstates
    computed once (enet_hmac_midstates) instead of the two key-block compressions per frame.
    Bit-exact with the per-frame-key path (keys[i] = table[session[i]]) and with the oracle's
    SessionManager::send restatement; opening accepts every frame, rejects a tampered body, a
    frame filed under another session and session indices past the table (seal: the whole frame
    slot zeroed, open: ok = 0 -- never a read past the table), and zeroes their plaintext."""
    import torch
    rng = np.random.default_rng(9)
    S, n = 37, 700
    table = [splitmix_bytes(97000 + s, 32) for s in range(S)]
    sess = rng.integers(0, S, n).astype(np.uint32)
    lens = [int(x) for x in rng.integers(0, 3000, n)]
    lens[:6] = [0, 1, 63, 128, 1500, 16384]
    msgs = [splitmix_bytes(98000 + i, L) for i, L in enumerate(lens)]
    nonces = [splitmix_bytes(99000 + i, 12) for i in range(n)]
    keys_per = [table[s] for s in sess]
    ref = seal_frames(enet, msgs, keys_per, nonces, 16, 3)
    tbl = torch.tensor(np.frombuffer(b"".join(table), np.uint8).copy()).cuda()
    mid = torch.zeros(16 * S, dtype=torch.int32, device="cuda")
    enet.hmac_midstates(tbl, S, mid)
    sess_seal = sess.copy()
    sess_seal[11] = S + 5  # past the table: the frame slot comes out all zeros
    st = torch.tensor(sess_seal.view(np.int32)).cuda()
    b = dataclasses.replace(enet.make_batch(msgs, keys_per, nonces, base_offset=3), keys=tbl)
    ooffs = offsets_for([L + 48 for L in lens], 4)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    enet.wire_seal_sessions(b, out, torch.tensor(ooffs).cuda(), st, S, mid)
    got = records_of(host(out), ooffs.tolist())
    assert got[:11] == ref[:11] and got[12:] == ref[12:]
    # fail closed: nothing of frame 11 is encrypted under another session's key
    assert got[11] == bytes(len(ref[11]))
    for i in list(range(0, n, 23)) + [0, 1, 5]:
        assert got[i] == wire_of(nonces[i], oracle.frame_seal(keys_per[i], nonces[i], msgs[i])), i
    frames = list(got)
    frames[5] = frames[5][:20] + bytes([frames[5][20] ^ 0x10]) + frames[5][21:]
    sess2 = sess.copy()
    sess2[7] = (sess2[7] + 1) % S
    sess2[9] = 0xFFFFFFF0  # past the table on open
    bo = dataclasses.replace(enet.make_batch(frames, keys_per, nonces, base_offset=2), keys=tbl, nonces=None)
    poffs = offsets_for(lens, 1)
    pt = torch.full((int(poffs[-1]) + 1,), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.wire_open_sessions(bo, pt, torch.tensor(poffs).cuda(), torch.tensor(sess2.view(np.int32)).cuda(),
                            S, mid, macs, ok)
    okh = ok.cpu().tolist()
    back = records_of(host(pt), poffs.tolist())
    assert [i for i in range(n) if okh[i] == 0] == [5, 7, 9, 11]
    for i in range(n):
        assert back[i] == (bytes(lens[i]) if i in (5, 7, 9, 11) else msgs[i]), i
