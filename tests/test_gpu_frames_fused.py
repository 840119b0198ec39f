"""GPU parity of the one-pass HMAC-SHA256 + ChaCha20 frame path (duplex.hip, DK_FRAME) against
the CPU oracle on uniform batches (round 1's fused-kernel shapes: multiples of 128 B, whole and
partial workgroups, unaligned arenas); staging variant 0 forces the two-pass path (sha_kernel +
records_kernel), so both must give the same bytes.  Ragged and mixed shapes: test_gpu_duplex.py.
Reference: SessionManager::send / receive_loop framing (src/network/SessionManager.cpp:362-387,
:760-822), encode_signed / decode_signed (src/protocol/Message.cpp:305-328).  Bit-exact."""
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


def uniform_offsets(n, size, base):
    return (base + size * np.arange(n + 1)).astype(np.int64)


def seal(enet, msgs, keys, nonces, hdr, base, key_stride=32):
    import torch
    n, L = len(msgs), len(msgs[0])
    b = enet.make_batch(msgs, keys, nonces, base_offset=base, key_stride=key_stride)
    ooffs = uniform_offsets(n, L + 32 + hdr, base)
    out = torch.zeros(int(ooffs[-1]), dtype=torch.uint8, device="cuda")
    (enet.wire_seal if hdr else enet.frame_seal)(b, out, torch.tensor(ooffs).cuda())
    return records_of(host(out), ooffs.tolist())


def open_(enet, frames, keys, nonces, hdr, base, key_stride=32):
    import torch
    n, F = len(frames), len(frames[0])
    b = enet.make_batch(frames, keys, nonces, base_offset=base, key_stride=key_stride)
    if hdr:
        b = dataclasses.replace(b, nonces=None)
    poffs = uniform_offsets(n, F - 32 - hdr, base)
    pt = torch.full((int(poffs[-1]),), 0xAA, dtype=torch.uint8, device="cuda")
    macs = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    (enet.wire_open if hdr else enet.frame_open)(b, pt, torch.tensor(poffs).cuda(), macs, ok)
    return records_of(host(pt), poffs.tolist()), ok.cpu().tolist(), host(macs)


@pytest.mark.parametrize("hdr", [16, 0])
@pytest.mark.parametrize("L,n,base", [(4096, 512, 0), (128, 256, 0), (256, 300, 5), (1536, 600, 3),
                                      (384, 255, 0), (4096, 257, 16)])
def test_fused_frames_vs_oracle(enet, hdr, L, n, base):
    """Seal matches the oracle byte for byte (header, encrypted body, encrypted MAC); open
    returns every message with ok = 1 and the decrypted MACs; both agree with the two-pass path
    (staging 0); unaligned arenas (base 3, 5) included."""
    msgs = [splitmix_bytes(7000 + 13 * L + i, L) for i in range(n)]
    keys = [splitmix_bytes(8000 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(9000 + i, 12) for i in range(n)]
    enet.set_staging(-1)
    frames = seal(enet, msgs, keys, nonces, hdr, base)
    idx = range(n) if n * L <= 1 << 20 else list(range(0, n, 7)) + [n - 1]
    for i in idx:
        body = oracle.frame_seal(keys[i], nonces[i], msgs[i])
        assert frames[i] == (wire_of(nonces[i], body) if hdr else body), i
    got, ok, macs = open_(enet, frames, keys, nonces, hdr, base)
    assert ok == [1] * n and got == msgs
    for i in idx:
        dec = oracle.chacha20_xor(keys[i], nonces[i], frames[i][hdr:], 0)
        assert macs[32 * i:32 * i + 32] == dec[L:], i
        assert oracle.frame_open(keys[i], nonces[i], frames[i][hdr:]) == (True, msgs[i])
    enet.set_staging(0)
    try:
        assert seal(enet, msgs, keys, nonces, hdr, base) == frames
        assert open_(enet, frames, keys, nonces, hdr, base) == (got, ok, macs)
    finally:
        enet.set_staging(-1)


@pytest.mark.parametrize("hdr", [16, 0])
def test_fused_frames_reject_tampered(enet, hdr):
    """Tampered body byte, tampered MAC byte and (wire) a wrong length field or nonce fail with
    ok = 0 and a zeroed message; their neighbours are untouched."""
    n, L = 512, 1024
    msgs = [splitmix_bytes(100 + i, L) for i in range(n)]
    keys = [splitmix_bytes(200 + i, 32) for i in range(n)]
    nonces = [splitmix_bytes(300 + i, 12) for i in range(n)]
    frames = seal(enet, msgs, keys, nonces, hdr, 0)
    bad = list(frames)

    def flip(i, pos):
        f = bytearray(bad[i])
        f[pos] ^= 0x10
        bad[i] = bytes(f)

    flip(5, hdr + 100)             # body byte
    flip(300, hdr + L + 7)         # encrypted MAC byte
    flip(511, hdr + L - 1)         # last message byte, last workgroup
    tampered = {5, 300, 511}
    if hdr:
        flip(77, 13)               # length field
        flip(260, 2)               # nonce
        tampered |= {77, 260}
    got, ok, _ = open_(enet, bad, keys, nonces, hdr, 0)
    for i in range(n):
        if i in tampered:
            assert ok[i] == 0 and got[i] == bytes(L), i
        else:
            assert ok[i] == 1 and got[i] == msgs[i], i


def test_fused_frames_shared_key(enet):
    """key_stride 0: one session key for the whole batch."""
    n, L = 256, 512
    msgs = [splitmix_bytes(400 + i, L) for i in range(n)]
    key = splitmix_bytes(401, 32)
    nonces = [splitmix_bytes(500 + i, 12) for i in range(n)]
    frames = seal(enet, msgs, [key], nonces, 16, 0, key_stride=0)
    for i in (0, 1, 128, 255):
        assert frames[i] == wire_of(nonces[i], oracle.frame_seal(key, nonces[i], msgs[i]))
    got, ok, _ = open_(enet, frames, [key], nonces, 16, 0, key_stride=0)
    assert ok == [1] * n and got == msgs
