"""GPU parity of the sequence-parallel path (segments.hip): records of the reference's real sizes
-- a stored file is ONE chunk of up to 32 MiB (Config.hpp:62, Node.cpp:1414-1417, 1644-1655),
session payloads up to 1 MiB (SessionManager.cpp:87) -- cut into 64 KiB tiles across the chip,
against the CPU oracle (ChaCha20::apply semantics incl. the u32 counter wrap, ChaCha20.cpp:110;
RFC 8439 AEAD, tag pinned by OpenSSL / RFC vectors through the oracle's golden checks).
Byte work: every comparison is bit-exact."""
import numpy as np
import pytest

import oracle
from util import splitmix_bytes

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(scope="module")
def enet():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import ephemeralnet_amd as E
    E.lib()
    yield E
    E.set_seg_min(-1)
    E.set_lanes_per_record(0)


def host(t) -> bytes:
    return t.cpu().numpy().tobytes()


def shapes():
    # name -> (lengths, seg_min setting); -1 = the automatic rule
    small = [int(x) % 5000 for x in np.frombuffer(splitmix_bytes(7, 4 * 300), "<u4")]
    return {
        "1x32MiB": ([32 * MiB], -1),
        "8x1MiB": ([MiB] * 8, -1),
        "mixed_with_32MiB": (small[:150] + [32 * MiB] + small[150:] + [300 << 10, (256 << 10) + 17], -1),
        "ragged_tiles_forced": ([0, 1, 63, 64, 65, 4095, 65535, 65536, 65537, (2 << 16) + 17, 3 * 65536 - 1,
                                 (256 << 10) + 100], 0),
    }


def make(enet, lens, seed, base=0, shared_key=False):
    items = [splitmix_bytes(seed + i, L) for i, L in enumerate(lens)]
    n = len(lens)
    keys = [splitmix_bytes(seed + 10_000 + i, 32) for i in range(1 if shared_key else n)]
    nonces = [splitmix_bytes(seed + 20_000 + i, 12) for i in range(n)]
    b = enet.make_batch(items, keys, nonces, key_stride=0 if shared_key else 32, base_offset=base)
    return b, items, [keys[0]] * n if shared_key else keys, nonces


@pytest.mark.parametrize("name", list(shapes()))
@pytest.mark.parametrize("base", [0, 3])
def test_seg_chacha20_vs_oracle(enet, name, base):
    import torch
    lens, seg = shapes()[name]
    if base and name == "1x32MiB":
        pytest.skip("unaligned start covered by the other shapes")
    enet.set_seg_min(seg)
    try:
        b, items, keys, nonces = make(enet, lens, 1000 + base)
        n = len(lens)
        # start counters near the u32 wrap: the keystream wraps inside the long records
        ctr = np.array([0xFFFFFFFF - (i * 977) % 4096 for i in range(n)], dtype=np.uint32)
        out = torch.zeros_like(b.arena)
        before = enet.seg_batches()
        enet.chacha20_xor(b, out, counters=torch.tensor(ctr.view(np.int32)).cuda())
        torch.cuda.synchronize()
        assert enet.seg_batches() == before + 1, "the batch did not take the sequence-parallel path"
        oh = host(out)
        offs = b.offsets.cpu().tolist()
        for i in range(n):
            want = oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctr[i]))
            assert oh[offs[i]:offs[i + 1]] == want, f"record {i} (len {lens[i]})"
    finally:
        enet.set_seg_min(-1)


@pytest.mark.parametrize("name", list(shapes()))
def test_seg_aead_vs_oracle_and_tamper(enet, name):
    import torch
    lens, seg = shapes()[name]
    enet.set_seg_min(seg)
    try:
        b, items, keys, nonces = make(enet, lens, 3000)
        n = len(lens)
        ct = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        before = enet.seg_batches()
        enet.aead_seal(b, ct, tags)
        torch.cuda.synchronize()
        assert enet.seg_batches() == before + 1
        cth, th = host(ct), host(tags)
        offs = b.offsets.cpu().tolist()
        for i in range(n):
            c, t = oracle.aead_seal(keys[i], nonces[i], items[i])
            assert cth[offs[i]:offs[i + 1]] == c, f"ciphertext {i} (len {lens[i]})"
            assert th[16 * i:16 * i + 16] == t, f"tag {i} (len {lens[i]})"
        # open: every record verifies and round-trips
        b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                        max_len_hint=b.max_len_hint)
        back = torch.zeros_like(ct)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        enet.aead_open(b2, back, tags, ok)
        torch.cuda.synchronize()
        assert int(ok.sum()) == n and torch.equal(back, b.arena)
        # tamper: the longest record's tag, and one ciphertext byte in the middle of another long one
        big = int(np.argmax(lens))
        bad_tags = tags.clone()
        bad_tags[16 * big] ^= 1
        ct2 = ct.clone()
        others = [i for i in range(n) if lens[i] >= 65536 and i != big]
        if others:
            o = others[-1]
            ct2[offs[o] + lens[o] // 2] ^= 0x80
        b3 = enet.Batch(ct2, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                        max_len_hint=b.max_len_hint)
        back.fill_(0xAA)
        ok.zero_()
        enet.aead_open(b3, back, bad_tags, ok)
        torch.cuda.synchronize()
        okh = ok.cpu().tolist()
        bh = host(back)
        for i in range(n):
            seg_ = bh[offs[i]:offs[i + 1]]
            if i == big or (others and i == others[-1]):
                assert okh[i] == 0, f"tampered record {i} verified"
                assert seg_ == bytes(lens[i]), f"tampered record {i} released plaintext"
            else:
                assert okh[i] == 1 and seg_ == items[i], f"record {i}"
    finally:
        enet.set_seg_min(-1)


def test_seg_aead_with_aad_forced(enet):
    """AAD prefixes (RFC 8439 2.8: aad || pad || ct || pad || lengths) on records cut into tiles."""
    import torch
    lens = [0, 17, 65536, 65536 * 3 + 5, 200_000]
    enet.set_seg_min(0)
    try:
        b, items, keys, nonces = make(enet, lens, 5000, base=5)
        n = len(lens)
        aads = [splitmix_bytes(9000 + i, (i * 13) % 40) for i in range(n)]
        aoff = [0]
        for a in aads:
            aoff.append(aoff[-1] + len(a))
        aad = torch.frombuffer(bytearray(b"".join(aads) or b"\0"), dtype=torch.uint8).cuda()
        aad_off = torch.tensor(aoff, dtype=torch.int64).cuda()
        ct = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        enet.aead_seal(b, ct, tags, aad=aad, aad_offsets=aad_off)
        torch.cuda.synchronize()
        cth, th = host(ct), host(tags)
        offs = b.offsets.cpu().tolist()
        for i in range(n):
            c, t = oracle.aead_seal(keys[i], nonces[i], items[i], aads[i])
            assert cth[offs[i]:offs[i + 1]] == c and th[16 * i:16 * i + 16] == t, f"record {i}"
        b2 = enet.Batch(ct, b.offsets, b.keys, b.nonces, total_bytes_hint=b.total_bytes_hint,
                        max_len_hint=b.max_len_hint)
        back = torch.zeros_like(ct)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        enet.aead_open(b2, back, tags, ok, aad=aad, aad_offsets=aad_off)
        torch.cuda.synchronize()
        assert int(ok.sum()) == n and torch.equal(back, b.arena)
    finally:
        enet.set_seg_min(-1)


def test_seg_shared_key_in_place_lying_hints(enet):
    """One shared key, out == in, and hints that understate the batch (the plan's capacities come
    from the hints: records past them stay with the record engine -- slower, same bytes)."""
    import torch
    lens = [MiB, 3 * MiB + 7, 5000, 2 * MiB]
    b, items, keys, nonces = make(enet, lens, 7000, shared_key=True)
    b.total_bytes_hint = MiB          # a lie: 6 MiB really
    b.max_len_hint = 300 << 10        # a lie: 3 MiB really
    n = len(lens)
    arena = b.arena.clone()
    tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
    bi = enet.Batch(arena, b.offsets, b.keys, b.nonces, key_stride=0,
                    total_bytes_hint=b.total_bytes_hint, max_len_hint=b.max_len_hint)
    enet.aead_seal(bi, arena, tags)
    torch.cuda.synchronize()
    offs = b.offsets.cpu().tolist()
    ah, th = host(arena), host(tags)
    for i in range(n):
        c, t = oracle.aead_seal(keys[0], nonces[i], items[i])
        assert ah[offs[i]:offs[i + 1]] == c and th[16 * i:16 * i + 16] == t, f"record {i}"


def test_seg_never_and_auto_agree(enet):
    """The record engine alone (seg never) and the tiles give the same bytes for a 2 MiB record."""
    import torch
    lens = [2 * MiB, 100, 700_000]
    b, items, keys, nonces = make(enet, lens, 8000)
    n = len(lens)
    outs = []
    for seg in (enet.SEG_NEVER, -1):
        enet.set_seg_min(seg)
        ct = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        enet.aead_seal(b, ct, tags)
        torch.cuda.synchronize()
        outs.append((host(ct), host(tags)))
    enet.set_seg_min(-1)
    assert outs[0] == outs[1]


@pytest.mark.parametrize("lens", [[300 << 10] * 4, [300 << 10, 100, (600 << 10) + 7, 0, 300 << 10, 65536 + 1]])
def test_seg_uniform_xor_one_launch_and_lying_hints(enet, lens):
    """ChaCha20 over a batch the hints call uniform (n x 300 KiB): one launch of tile workgroups,
    no plan, no record-engine pass.  The second shape lies -- records of 100 B, 600 KiB + 7, 0 and
    64 KiB + 1 under a 300 KiB hint -- and each such record is run whole by its tile-0 workgroup:
    the bytes are the oracle's either way.  Counters near the u32 wrap; in place too."""
    import torch
    n = len(lens)
    b, items, keys, nonces = make(enet, lens, 9300 + len(lens))
    hinted = enet.Batch(b.arena, b.offsets, b.keys, b.nonces, total_bytes_hint=n * (300 << 10),
                        max_len_hint=300 << 10)
    ctr = np.array([0xFFFFFFFF - 37 * i for i in range(n)], dtype=np.uint32)
    counters = torch.tensor(ctr.view(np.int32)).cuda()
    offs = b.offsets.cpu().tolist()
    for inplace in (False, True):
        out = b.arena.clone() if inplace else torch.zeros_like(b.arena)
        src = enet.Batch(out, b.offsets, b.keys, b.nonces, total_bytes_hint=n * (300 << 10),
                         max_len_hint=300 << 10) if inplace else hinted
        before = enet.seg_batches()
        enet.chacha20_xor(src, out, counters=counters)
        torch.cuda.synchronize()
        assert enet.seg_batches() == before + 1
        oh = host(out)
        for i in range(n):
            want = oracle.chacha20_xor(keys[i], nonces[i], items[i], int(ctr[i]))
            assert oh[offs[i]:offs[i + 1]] == want, f"record {i} (len {lens[i]}, in place {inplace})"


H53 = 52 * 65536 + 100  # 53 tiles, the last one ragged


@pytest.mark.parametrize("with_aad", [False, True])
@pytest.mark.parametrize("lens", [
    [300 << 10] * 5,
    [300 << 10, 100, (600 << 10) + 7, 0, 300 << 10, 65536 + 1, 4095],
    # > 256 tiles: two tiles per workgroup, an odd tile count (the last workgroup holds one)
    [H53] * 6,
    [H53, 100, H53, 0, H53 - 1, H53, H53, H53 + 70000],
], ids=["5x300K", "300K_lying", "6x53tiles", "53tiles_lying"])
def test_seg_uniform_aead_one_launch_lying_hints_tamper(enet, lens, with_aad):
    """RFC 8439 seal / open over a batch the hints call uniform (n x 300 KiB): one launch -- each
    record's last tile to arrive combines the partials and, on open, zeroes a failed record itself
    (write-through plaintext).  The second shape lies: records of 100 B, 600 KiB + 7, 0, 64 KiB + 1
    and 4 095 B under the 300 KiB hint are run whole by their tile-0 workgroups.  Bit-exact vs the
    oracle (tags pinned by RFC 8439 / OpenSSL through the oracle's golden checks), every record
    opens; then a flipped tag on an as-hinted record, a flipped ciphertext byte in another and in
    a fallback record: those three fail and are zeroed, the rest open.  Runs twice: the per-stream
    arrival counters must be back at zero for the second launch.  The last two shapes have more
    tiles than the chip has CUs (two tiles per workgroup) and 53 tiles per record."""
    import torch
    n = len(lens)
    H = max(set(lens), key=lens.count)  # the hinted length
    b, items, keys, nonces = make(enet, lens, 9600 + len(lens) + (7 if with_aad else 0))
    hint = dict(total_bytes_hint=n * H, max_len_hint=H)
    aads = [splitmix_bytes(9900 + i, (i * 37) % 90) for i in range(n)] if with_aad else None
    aad = aad_off = None
    if with_aad:
        ao = [0]
        for a_ in aads:
            ao.append(ao[-1] + len(a_))
        aad = torch.frombuffer(bytearray(b"".join(aads) or b"\0"), dtype=torch.uint8).cuda()
        aad_off = torch.tensor(ao, dtype=torch.int64, device="cuda")
    offs = b.offsets.cpu().tolist()
    sb = enet.Batch(b.arena, b.offsets, b.keys, b.nonces, **hint)
    for rep in range(2):
        ct = torch.zeros_like(b.arena)
        tags = torch.zeros(16 * n, dtype=torch.uint8, device="cuda")
        before = enet.seg_batches()
        enet.aead_seal(sb, ct, tags, aad=aad, aad_offsets=aad_off)
        torch.cuda.synchronize()
        assert enet.seg_batches() == before + 1
        cth, th = host(ct), host(tags)
        for i in range(n):
            c, t = oracle.aead_seal(keys[i], nonces[i], items[i], aads[i] if with_aad else b"")
            assert cth[offs[i]:offs[i + 1]] == c, f"ciphertext {i} (len {lens[i]}, rep {rep})"
            assert th[16 * i:16 * i + 16] == t, f"tag {i} (len {lens[i]}, rep {rep})"
        ob = enet.Batch(ct, b.offsets, b.keys, b.nonces, **hint)
        back = torch.full_like(ct, 0xAA)
        ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
        enet.aead_open(ob, back, tags, ok, aad=aad, aad_offsets=aad_off)
        torch.cuda.synchronize()
        assert ok.cpu().tolist() == [1] * n, rep
        bh = host(back)
        for i in range(n):
            assert bh[offs[i]:offs[i + 1]] == items[i], f"plaintext {i} (rep {rep})"
    # tamper
    hinted = [i for i in range(n) if lens[i] == H]
    fallback = [i for i in range(n) if lens[i] != H and lens[i] > 0]
    bad_tags = tags.clone()
    bad_tags[16 * hinted[0] + 3] ^= 0x40
    ct2 = ct.clone()
    victims = {hinted[0]}
    if len(hinted) > 1:
        ct2[offs[hinted[1]] + 150_000] ^= 0x01
        victims.add(hinted[1])
    if fallback:
        f = fallback[-1]
        ct2[offs[f] + lens[f] // 2] ^= 0x02
        victims.add(f)
    ob2 = enet.Batch(ct2, b.offsets, b.keys, b.nonces, **hint)
    back = torch.full_like(ct, 0xAA)
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    enet.aead_open(ob2, back, bad_tags, ok, aad=aad, aad_offsets=aad_off)
    torch.cuda.synchronize()
    okh, bh = ok.cpu().tolist(), host(back)
    for i in range(n):
        if i in victims:
            assert okh[i] == 0, f"tampered record {i} verified"
            assert bh[offs[i]:offs[i + 1]] == bytes(lens[i]), f"tampered record {i} released plaintext"
        else:
            assert okh[i] == 1 and bh[offs[i]:offs[i + 1]] == items[i], f"record {i}"
