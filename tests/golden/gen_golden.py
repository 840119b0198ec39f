#!/usr/bin/env python3
"""Generate tests/golden/golden.json -- run ONLY in the survey/build container.

Sources of truth (never shipped to the GPU box; only the resulting JSON is committed):
  * the reference src/crypto + src/protocol/Message.cpp, compiled from /root/reference by
    `make -C oracle ref` into oracle/_ref/libenet_ref.so (ChaCha20, SHA-256, HMAC-SHA256,
    CryptoManager, encode_signed / decode_signed);
  * OpenSSL 3.0.2 libcrypto.so.3 (EVP chacha20-poly1305 and EVP_MAC POLY1305) for the
    RFC 8439 AEAD, which the reference does not implement -- "parity
    unpinned by the reference", pinned by OpenSSL and the RFC 8439 vectors instead.

Inputs are regenerated from seeds with tests/util.py:splitmix_bytes, so the fixture stores
seeds + lengths + expected outputs (full hex up to 1500 B, SHA-256 of the output above).
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from util import splitmix_bytes  # noqa: E402

REF = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libenet_ref.so"))
SSL = C.CDLL("libcrypto.so.3")

FULL_HEX_MAX = 1500
LENS = [0, 1, 15, 16, 17, 63, 64, 65, 127, 128, 1500, 4095, 4096, 4097, 65536]


def ub(n):
    return (C.c_uint8 * max(n, 1))()


def out_repr(b: bytes) -> dict:
    if len(b) <= FULL_HEX_MAX:
        return {"hex": b.hex()}
    return {"sha256": hashlib.sha256(b).hexdigest()}


def ref_chacha(key, nonce, data, counter):
    o = ub(len(data))
    REF.ref_chacha20_apply(key, nonce, data, C.c_size_t(len(data)), o, C.c_uint32(counter))
    return bytes(o)[: len(data)]


def ref_sha(data):
    o = ub(32)
    REF.ref_sha256(data, C.c_size_t(len(data)), o)
    return bytes(o)


def ref_sha_pieces(data, piece):
    o = ub(32)
    REF.ref_sha256_pieces(data, C.c_size_t(len(data)), C.c_size_t(piece), o)
    return bytes(o)


def ref_hmac(key, data):
    o = ub(32)
    REF.ref_hmac(key, C.c_size_t(len(key)), data, C.c_size_t(len(data)), o)
    return bytes(o)


def ref_hmac_verify(key, data, mac):
    return bool(REF.ref_hmac_verify(key, C.c_size_t(len(key)), data, C.c_size_t(len(data)), mac,
                                    C.c_size_t(len(mac))))


# ---- OpenSSL EVP (AEAD) -----------------------------------------------------------------
SSL.EVP_CIPHER_CTX_new.restype = C.c_void_p
SSL.EVP_chacha20_poly1305.restype = C.c_void_p
SSL.EVP_EncryptInit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p]
SSL.EVP_EncryptUpdate.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.c_char_p, C.c_int]
SSL.EVP_EncryptFinal_ex.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
SSL.EVP_CIPHER_CTX_ctrl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
SSL.EVP_CIPHER_CTX_free.argtypes = [C.c_void_p]
SSL.EVP_MAC_fetch.restype = C.c_void_p
SSL.EVP_MAC_fetch.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
SSL.EVP_MAC_CTX_new.restype = C.c_void_p
SSL.EVP_MAC_CTX_new.argtypes = [C.c_void_p]
SSL.EVP_MAC_init.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_void_p]
SSL.EVP_MAC_update.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
SSL.EVP_MAC_final.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t), C.c_size_t]
SSL.EVP_MAC_CTX_free.argtypes = [C.c_void_p]
EVP_CTRL_AEAD_GET_TAG = 0x10


def ssl_aead_seal(key, nonce, aad, pt):
    ctx = SSL.EVP_CIPHER_CTX_new()
    assert SSL.EVP_EncryptInit_ex(ctx, SSL.EVP_chacha20_poly1305(), None, key, nonce) == 1
    outl = C.c_int(0)
    if aad:
        assert SSL.EVP_EncryptUpdate(ctx, None, C.byref(outl), aad, len(aad)) == 1
    ct = ub(len(pt) + 16)
    if pt:
        assert SSL.EVP_EncryptUpdate(ctx, ct, C.byref(outl), pt, len(pt)) == 1
        assert outl.value == len(pt)
    fin = C.c_int(0)
    assert SSL.EVP_EncryptFinal_ex(ctx, ub(16), C.byref(fin)) == 1
    tag = ub(16)
    assert SSL.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_AEAD_GET_TAG, 16, tag) == 1
    SSL.EVP_CIPHER_CTX_free(ctx)
    return bytes(ct)[: len(pt)], bytes(tag)


def ssl_poly1305(key, msg):
    mac = SSL.EVP_MAC_fetch(None, b"POLY1305", None)
    assert mac
    ctx = SSL.EVP_MAC_CTX_new(mac)
    assert SSL.EVP_MAC_init(ctx, key, 32, None) == 1
    if msg:
        assert SSL.EVP_MAC_update(ctx, msg, len(msg)) == 1
    out = ub(16)
    ol = C.c_size_t(0)
    assert SSL.EVP_MAC_final(ctx, out, C.byref(ol), 16) == 1
    SSL.EVP_MAC_CTX_free(ctx)
    return bytes(out)


def main():
    g = {
        "_about": "Golden vectors. chacha20/sha256/hmac/cryptomanager/frame: reference src/crypto "
                  "(oracle/_ref). aead/poly1305: OpenSSL 3.0.2 + RFC 8439. Inputs: "
                  "tests/util.py splitmix_bytes(seed, len). Generator: tests/golden/gen_golden.py.",
        "full_hex_max": FULL_HEX_MAX,
    }

    # -- RFC 8439 2.4.2 through the reference ChaCha20::apply (counter 1)
    key = bytes(range(32))
    nonce = bytes.fromhex("000000000000004a00000000")
    sunscreen = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for "
                 b"the future, sunscreen would be it.")
    g["rfc8439_2_4_2"] = {"key": key.hex(), "nonce": nonce.hex(), "counter": 1,
                          "pt": sunscreen.hex(), "ct": ref_chacha(key, nonce, sunscreen, 1).hex()}

    # -- ChaCha20::apply: lengths x counters (incl. the u32 wrap, ChaCha20.cpp:110)
    cases = []
    seed = 1000
    for L in LENS:
        for ctr_kind in ("zero", "one", "wrap", "wrap16", "chunk_id"):
            seed += 1
            k = splitmix_bytes(seed * 3 + 0, 32)
            n = splitmix_bytes(seed * 3 + 1, 12)
            if ctr_kind == "zero":
                ctr = 0
            elif ctr_kind == "one":
                ctr = 1
            elif ctr_kind == "wrap":
                ctr = 0xFFFFFFFF
            elif ctr_kind == "wrap16":
                ctr = 0xFFFFFFF0
            else:
                cid = splitmix_bytes(seed * 7 + 5, 32)
                ctr = int.from_bytes(cid[:4], "little")  # CryptoManager.cpp:8-13
            pt_seed = seed * 3 + 2
            ct = ref_chacha(k, n, splitmix_bytes(pt_seed, L), ctr)
            cases.append({"len": L, "key": k.hex(), "nonce": n.hex(), "counter": ctr,
                          "pt_seed": pt_seed, "ct": out_repr(ct)})
    g["chacha20"] = cases

    # -- SHA-256 digest + streaming pieces
    sh = []
    for i, L in enumerate([0, 1, 3, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 1000, 1500, 4096,
                           65536]):
        data = b"abc" if L == 3 else splitmix_bytes(2000 + i, L)
        sh.append({"len": L, "seed": None if L == 3 else 2000 + i, "abc": L == 3,
                   "digest": ref_sha(data).hex(),
                   "digest_pieces_7": ref_sha_pieces(data, 7).hex() if L else None})
    g["sha256"] = sh

    # -- HMAC-SHA256 (keys over 64 B hashed first, HmacSha256.cpp:15-17)
    hm = []
    seed = 3000
    for kl in (0, 16, 32, 64, 65, 100):
        for L in (0, 1, 64, 66, 1500, 4096):
            seed += 2
            k = splitmix_bytes(seed, kl)
            d = splitmix_bytes(seed + 1, L)
            hm.append({"key": k.hex(), "len": L, "seed": seed + 1, "mac": ref_hmac(k, d).hex()})
    g["hmac"] = hm
    # RFC 4231 test case 2 through the reference
    g["rfc4231_tc2"] = {"key": b"Jefe".hex(), "data": b"what do ya want for nothing?".hex(),
                        "mac": ref_hmac(b"Jefe", b"what do ya want for nothing?").hex()}
    # verify() rejects wrong-length MACs (HmacSha256.cpp:44)
    k = splitmix_bytes(3999, 32)
    d = splitmix_bytes(3998, 100)
    m = ref_hmac(k, d)
    g["hmac_verify"] = [
        {"key": k.hex(), "seed": 3998, "len": 100, "mac": m.hex(), "ok": ref_hmac_verify(k, d, m)},
        {"key": k.hex(), "seed": 3998, "len": 100, "mac": m[:31].hex(),
         "ok": ref_hmac_verify(k, d, m[:31])},
        {"key": k.hex(), "seed": 3998, "len": 100, "mac": (bytes([m[0] ^ 1]) + m[1:]).hex(),
         "ok": ref_hmac_verify(k, d, bytes([m[0] ^ 1]) + m[1:])},
    ]

    # -- CryptoManager::encrypt_with_key (random nonce drawn by the reference, recorded)
    cm = []
    for i, L in enumerate([0, 1, 100, 4096, 65536, 70000]):
        k = splitmix_bytes(4000 + 3 * i, 32)
        cid = splitmix_bytes(4001 + 3 * i, 32)
        pt = splitmix_bytes(4002 + 3 * i, L)
        ct = ub(L)
        nn = ub(12)
        REF.ref_cm_encrypt_with_key(k, cid, pt, C.c_size_t(L), ct, nn)
        ctb = bytes(ct)[:L]
        back = ub(L)
        REF.ref_cm_decrypt_with_key(k, cid, ctb, C.c_size_t(L), bytes(nn), back)
        assert bytes(back)[:L] == pt
        cm.append({"len": L, "key": k.hex(), "chunk_id": cid.hex(), "pt_seed": 4002 + 3 * i,
                   "nonce": bytes(nn).hex(), "ct": out_repr(ctb)})
    g["cryptomanager"] = cm

    # -- session frames: encode_signed(Request / Chunk) then ChaCha20(ctr 0) with a fixed nonce
    fr = []
    for i, (kind, L) in enumerate([("request", 0), ("chunk", 0), ("chunk", 1), ("chunk", 1400),
                                   ("chunk", 4096)]):
        key = splitmix_bytes(5000 + 5 * i, 32)
        cid = splitmix_bytes(5001 + 5 * i, 32)
        nn = splitmix_bytes(5003 + 5 * i, 12)
        buf = ub(1 << 17)
        if kind == "request":
            peer = splitmix_bytes(5002 + 5 * i, 32)
            sz = REF.ref_encode_signed_request(cid, peer, key, C.c_size_t(32), buf, C.c_size_t(1 << 17))
        else:
            data = splitmix_bytes(5002 + 5 * i, L)
            sz = REF.ref_encode_signed_chunk(cid, data, C.c_size_t(L), C.c_int64(3600), key,
                                             C.c_size_t(32), buf, C.c_size_t(1 << 17))
        signed = bytes(buf)[:sz]
        assert REF.ref_decode_signed_ok(signed, C.c_size_t(sz), key, C.c_size_t(32)) == 1
        tampered = bytearray(signed)
        tampered[min(5, sz - 1)] ^= 1
        body = ref_chacha(key, nn, signed, 0)
        fr.append({"kind": kind, "key": key.hex(), "nonce": nn.hex(), "signed": signed.hex(),
                   "body": body.hex(), "tamper_rejected": REF.ref_decode_signed_ok(
                       bytes(tampered), C.c_size_t(sz), key, C.c_size_t(32)) == 0})
    g["frames"] = fr

    # -- RFC 8439 AEAD via OpenSSL (reference has none)
    ae = []
    seed = 6000
    for L in LENS:
        for al in (0, 12, 17):
            seed += 4
            k = splitmix_bytes(seed, 32)
            nn = splitmix_bytes(seed + 1, 12)
            aad = splitmix_bytes(seed + 2, al)
            pt = splitmix_bytes(seed + 3, L)
            ct, tag = ssl_aead_seal(k, nn, aad, pt)
            ae.append({"len": L, "aad_len": al, "key": k.hex(), "nonce": nn.hex(),
                       "aad_seed": seed + 2, "pt_seed": seed + 3, "ct": out_repr(ct),
                       "tag": tag.hex()})
    g["aead"] = ae
    # RFC 8439 2.8.2
    k = bytes(range(0x80, 0xA0))
    nn = bytes.fromhex("070000004041424344454647")
    aad = bytes.fromhex("50515253c0c1c2c3c4c5c6c7")
    ct, tag = ssl_aead_seal(k, nn, aad, sunscreen)
    assert tag.hex() == "1ae10b594f09e26a7e902ecbd0600691"
    g["rfc8439_2_8_2"] = {"key": k.hex(), "nonce": nn.hex(), "aad": aad.hex(), "pt": sunscreen.hex(),
                          "ct": ct.hex(), "tag": tag.hex()}
    # Poly1305 one-shot (RFC 8439 2.5.2 + random)
    pk = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    msg = b"Cryptographic Forum Research Group"
    assert ssl_poly1305(pk, msg).hex() == "a8061dc1305136c6c22b8baf0c0127a9"
    po = [{"key": pk.hex(), "msg": msg.hex(), "tag": ssl_poly1305(pk, msg).hex()}]
    for i, L in enumerate([0, 1, 15, 16, 17, 33, 64, 1000]):
        k = splitmix_bytes(7000 + 2 * i, 32)
        mm = splitmix_bytes(7001 + 2 * i, L)
        po.append({"key": k.hex(), "msg": mm.hex(), "tag": ssl_poly1305(k, mm).hex()})
    # edge: r and s all-ones-ish (exercise final reduction)
    k = b"\xff" * 32
    mm = b"\xff" * 64
    po.append({"key": k.hex(), "msg": mm.hex(), "tag": ssl_poly1305(k, mm).hex()})
    g["poly1305"] = po

    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
