"""Pin the CPU oracle (oracle/enet_oracle.c) to the golden vectors generated from the compiled
reference src/crypto (and OpenSSL / RFC 8439 for the AEAD).  CPU only."""
import hashlib
import os

import pytest

import oracle
from util import splitmix_bytes


def expect(rep, got: bytes):
    if "hex" in rep:
        assert got.hex() == rep["hex"]
    else:
        assert hashlib.sha256(got).hexdigest() == rep["sha256"]


def test_splitmix_c_matches_numpy():
    for seed, n in [(0, 0), (1, 1), (7, 9), (123456789, 1000)]:
        assert oracle.splitmix_bytes(seed, n) == splitmix_bytes(seed, n)


def test_rfc8439_chacha20(golden):
    v = golden["rfc8439_2_4_2"]
    ct = oracle.chacha20_xor(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["pt"]), 1)
    assert ct.hex() == v["ct"]
    assert ct[:8].hex() == "6e2e359a2568f980"  # RFC 8439 2.4.2


def test_chacha20_golden(golden):
    for c in golden["chacha20"]:
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        ct = oracle.chacha20_xor(bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), pt, c["counter"])
        expect(c["ct"], ct)


def test_chacha20_counter_wrap():
    k, n = bytes(32), bytes(12)
    # block at counter 0xFFFFFFFF followed by block 0 (ChaCha20.cpp:110, u32 wrap)
    ks = oracle.chacha20_xor(k, n, bytes(128), 0xFFFFFFFF)
    assert ks[64:] == oracle.chacha20_block(k, n, 0)


def test_sha256_golden(golden):
    for c in golden["sha256"]:
        data = b"abc" if c["abc"] else splitmix_bytes(c["seed"], c["len"])
        assert oracle.sha256(data).hex() == c["digest"]
        assert hashlib.sha256(data).hexdigest() == c["digest"]


def test_hmac_golden(golden):
    for c in golden["hmac"]:
        d = splitmix_bytes(c["seed"], c["len"])
        assert oracle.hmac_sha256(bytes.fromhex(c["key"]), d).hex() == c["mac"]
    v = golden["rfc4231_tc2"]
    assert oracle.hmac_sha256(bytes.fromhex(v["key"]), bytes.fromhex(v["data"])).hex() == v["mac"]
    for c in golden["hmac_verify"]:
        d = splitmix_bytes(c["seed"], c["len"])
        assert oracle.hmac_sha256_verify(bytes.fromhex(c["key"]), d, bytes.fromhex(c["mac"])) == c["ok"]


def test_cryptomanager_golden(golden):
    for c in golden["cryptomanager"]:
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        cid = bytes.fromhex(c["chunk_id"])
        ctr = oracle.derive_counter(cid)
        ct = oracle.chacha20_xor(bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), pt, ctr)
        expect(c["ct"], ct)


def test_frames_golden(golden):
    for f in golden["frames"]:
        key, nonce, signed = bytes.fromhex(f["key"]), bytes.fromhex(f["nonce"]), bytes.fromhex(f["signed"])
        body = oracle.frame_seal(key, nonce, signed[:-32])
        assert body.hex() == f["body"]
        ok, m = oracle.frame_open(key, nonce, body)
        assert ok and m == signed[:-32]
        bad = bytearray(body)
        bad[min(5, len(bad) - 1)] ^= 1
        assert not oracle.frame_open(key, nonce, bytes(bad))[0]
    assert not oracle.frame_open(bytes(32), bytes(12), bytes(31))[0]  # Message.cpp:315


def test_poly1305_golden(golden):
    for c in golden["poly1305"]:
        assert oracle.poly1305(bytes.fromhex(c["key"]), bytes.fromhex(c["msg"])).hex() == c["tag"]


def test_aead_golden(golden):
    v = golden["rfc8439_2_8_2"]
    ct, tag = oracle.aead_seal(bytes.fromhex(v["key"]), bytes.fromhex(v["nonce"]), bytes.fromhex(v["pt"]),
                               bytes.fromhex(v["aad"]))
    assert ct.hex() == v["ct"] and tag.hex() == v["tag"] == "1ae10b594f09e26a7e902ecbd0600691"
    for c in golden["aead"]:
        k, n = bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"])
        aad = splitmix_bytes(c["aad_seed"], c["aad_len"])
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        ct, tag = oracle.aead_seal(k, n, pt, aad)
        expect(c["ct"], ct)
        assert tag.hex() == c["tag"]
        ok, back = oracle.aead_open(k, n, ct, tag, aad)
        assert ok and back == pt
        if c["len"]:
            bad = bytearray(ct)
            bad[-1] ^= 0x80
            assert not oracle.aead_open(k, n, bytes(bad), tag, aad)[0]


@pytest.mark.skipif(not os.path.exists(oracle.REF_PATH), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_vs_reference_random():
    """Where the compiled reference is present (build container), cross-check random cases."""
    import ctypes as C
    ref = C.CDLL(oracle.REF_PATH)
    for i in range(50):
        L = int.from_bytes(splitmix_bytes(90000 + i, 2), "little") % 3000
        k = splitmix_bytes(91000 + i, 32)
        n = splitmix_bytes(92000 + i, 12)
        ctr = int.from_bytes(splitmix_bytes(93000 + i, 4), "little")
        pt = splitmix_bytes(94000 + i, L)
        o = (C.c_uint8 * max(L, 1))()
        ref.ref_chacha20_apply(k, n, pt, C.c_size_t(L), o, C.c_uint32(ctr))
        assert bytes(o)[:L] == oracle.chacha20_xor(k, n, pt, ctr)
        m = (C.c_uint8 * 32)()
        ref.ref_hmac(k, C.c_size_t(32), pt, C.c_size_t(L), m)
        assert bytes(m) == oracle.hmac_sha256(k, pt)
