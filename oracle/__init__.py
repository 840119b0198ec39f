"""oracle -- TEST INFRASTRUCTURE ONLY: ctypes view of the CPU restatement (liboracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
package ephemeralnet_amd never imports this module (tests/test_boundary.py checks that)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libenet_ref.so")

_lib = None


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        sz = C.c_size_t
        p = C.c_char_p
        _lib.orc_splitmix_bytes.argtypes = [C.c_uint64, C.c_void_p, sz]
        _lib.orc_chacha20_xor.argtypes = [p, p, C.c_uint32, p, C.c_void_p, sz]
        _lib.orc_chacha20_block.argtypes = [p, p, C.c_uint32, C.c_void_p]
        _lib.orc_sha256.argtypes = [p, sz, C.c_void_p]
        _lib.orc_hmac_sha256.argtypes = [p, sz, p, sz, C.c_void_p]
        _lib.orc_hmac_sha256_verify.argtypes = [p, sz, p, sz, p, sz]
        _lib.orc_poly1305.argtypes = [p, p, sz, C.c_void_p]
        _lib.orc_aead_seal.argtypes = [p, p, p, sz, p, sz, C.c_void_p, C.c_void_p]
        _lib.orc_aead_open.argtypes = [p, p, p, sz, p, sz, p, C.c_void_p]
        _lib.orc_frame_seal.argtypes = [p, p, p, sz, C.c_void_p]
        _lib.orc_frame_open.argtypes = [p, p, p, sz, C.c_void_p]
        _lib.orc_derive_counter.argtypes = [p]
        _lib.orc_derive_counter.restype = C.c_uint32
        _lib.orc_bench_aead.argtypes = [C.c_void_p] * 6 + [sz, sz, C.c_int, C.c_void_p]
    return _lib


def _buf(n: int):
    return (C.c_uint8 * max(n, 1))()


def splitmix_bytes(seed: int, n: int) -> bytes:
    b = _buf(n)
    lib().orc_splitmix_bytes(seed & 0xFFFFFFFFFFFFFFFF, b, n)
    return bytes(b)[:n]


def chacha20_xor(key: bytes, nonce: bytes, data: bytes, counter: int = 0) -> bytes:
    o = _buf(len(data))
    lib().orc_chacha20_xor(key, nonce, counter & 0xFFFFFFFF, data, o, len(data))
    return bytes(o)[: len(data)]


def chacha20_block(key: bytes, nonce: bytes, counter: int) -> bytes:
    o = _buf(64)
    lib().orc_chacha20_block(key, nonce, counter & 0xFFFFFFFF, o)
    return bytes(o)


def sha256(data: bytes) -> bytes:
    o = _buf(32)
    lib().orc_sha256(data, len(data), o)
    return bytes(o)


def hmac_sha256(key: bytes, data: bytes) -> bytes:
    o = _buf(32)
    lib().orc_hmac_sha256(key, len(key), data, len(data), o)
    return bytes(o)


def hmac_sha256_verify(key: bytes, data: bytes, mac: bytes) -> bool:
    return bool(lib().orc_hmac_sha256_verify(key, len(key), data, len(data), mac, len(mac)))


def poly1305(key: bytes, msg: bytes) -> bytes:
    o = _buf(16)
    lib().orc_poly1305(key, msg, len(msg), o)
    return bytes(o)


def aead_seal(key: bytes, nonce: bytes, pt: bytes, aad: bytes = b"") -> tuple[bytes, bytes]:
    ct = _buf(len(pt))
    tag = _buf(16)
    lib().orc_aead_seal(key, nonce, aad, len(aad), pt, len(pt), ct, tag)
    return bytes(ct)[: len(pt)], bytes(tag)


def aead_open(key: bytes, nonce: bytes, ct: bytes, tag: bytes, aad: bytes = b""):
    pt = _buf(len(ct))
    ok = lib().orc_aead_open(key, nonce, aad, len(aad), ct, len(ct), tag, pt)
    return bool(ok), bytes(pt)[: len(ct)]


def frame_seal(key: bytes, nonce: bytes, m: bytes) -> bytes:
    o = _buf(len(m) + 32)
    lib().orc_frame_seal(key, nonce, m, len(m), o)
    return bytes(o)[: len(m) + 32]


def frame_open(key: bytes, nonce: bytes, body: bytes):
    o = _buf(len(body))
    ok = lib().orc_frame_open(key, nonce, body, len(body), o)
    return bool(ok), bytes(o)[: max(len(body) - 32, 0)]


def derive_counter(chunk_id: bytes) -> int:
    return int(lib().orc_derive_counter(chunk_id))
