#!/usr/bin/env python3
"""Generate tests/golden/pow.json -- run ONLY in the survey/build container (needs oracle/_ref).

Sources of truth (only the resulting JSON is committed):
  * store PoW: the reference security::compute_store_pow / store_pow_valid themselves
    (src/security/StoreProof.cpp, compiled by `make -C oracle ref`);
  * announce / handshake PoW: those functions live in an anonymous namespace of
    src/core/Node.cpp (not linkable), so their serialisation (Node.cpp:149-171, 233-245) is
    restated here, hashed by the reference crypto::Sha256 (ref_sha256_concat), with the seed ->
    start step taken from libstdc++'s std::mt19937_64 + uniform_int_distribution exactly as
    Node.cpp:203-220 / 258-282 call them (ref_mt64_uniform_first), and the search loop run here;
  * std::mt19937_64 output streams (ref_mt64);
  * session keys: network::KeyManager (src/network/KeyManager.cpp) register_session_with_material
    and rotate_if_needed.
Inputs come from tests/util.py splitmix_bytes(seed, len).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from util import splitmix_bytes  # noqa: E402

REF = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libenet_ref.so"))
REF.ref_compute_store_pow.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_size_t, C.c_uint8,
                                      C.c_uint64, C.POINTER(C.c_uint64)]
REF.ref_store_pow_valid.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_size_t, C.c_uint64,
                                    C.c_uint8]
REF.ref_mt64.argtypes = [C.c_uint64, C.c_size_t, C.c_void_p]
REF.ref_mt64_uniform_first.argtypes = [C.c_uint64]
REF.ref_mt64_uniform_first.restype = C.c_uint64
REF.ref_sha256_concat.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
REF.ref_keymanager_material_key.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t, C.c_void_p]
REF.ref_keymanager_rotate.argtypes = [C.c_char_p, C.c_int64, C.c_void_p]
REF.ref_keymanager_rotate.restype = C.c_int64
REF.ref_sanitize_filename_hint.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p, C.c_size_t]
REF.ref_sanitize_filename_hint.restype = C.c_long


def be64(v: int) -> bytes:
    return (v & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "big")


def ref_sha_concat(pieces) -> bytes:
    bufs = [C.create_string_buffer(p, max(len(p), 1)) for p in pieces]
    arr = (C.c_void_p * len(pieces))(*[C.cast(b, C.c_void_p) for b in bufs])
    lens = (C.c_size_t * len(pieces))(*[len(p) for p in pieces])
    out = (C.c_uint8 * 32)()
    REF.ref_sha256_concat(arr, lens, len(pieces), out)
    return bytes(out)


def lz(d: bytes) -> int:
    total = 0
    for b in d:
        if b == 0:
            total += 8
            continue
        return total + (8 - b.bit_length())
    return total


def lp64(data: bytes):  # update_length_prefixed, Node.cpp:149-153
    return [be64(len(data)), data]


def node_search(pieces, difficulty: int, max_attempts: int):
    """compute_announce_pow / compute_handshake_pow (Node.cpp:200-230, 257-292)."""
    if difficulty == 0:
        return True, 0, 0
    d0 = ref_sha_concat(pieces + [be64(0)])
    seed = int.from_bytes(d0[:8], "big")
    start = REF.ref_mt64_uniform_first(seed)
    for a in range(max_attempts):
        cand = (start + a) & 0xFFFFFFFFFFFFFFFF
        if lz(ref_sha_concat(pieces + [be64(cand)])) >= difficulty:
            return True, cand, a
    return False, 0, max_attempts


def main():
    g = {"_about": "PoW + session-key golden vectors; generator tests/golden/gen_pow_golden.py "
                   "(reference StoreProof.cpp / KeyManager.cpp compiled from /root/reference; "
                   "Node.cpp PoW serialisation restated, hashed by the reference Sha256, seeded by "
                   "libstdc++ std::mt19937_64). Inputs: tests/util.py splitmix_bytes."}

    # -- std::mt19937_64 streams
    mts = []
    for seed in (0, 1, 5489, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF):
        out = (C.c_uint64 * 700)()
        REF.ref_mt64(seed, 700, out)
        mts.append({"seed": seed, "first": list(out[:5]), "at_311_315": list(out[311:316]),
                    "at_623_627": list(out[623:628]), "uniform_first": REF.ref_mt64_uniform_first(seed)})
    g["mt19937_64"] = mts

    # -- store PoW through the reference (hints of every length class: tail 0..63 mod 64)
    sp = []
    seed = 20000
    hints = [b"", b"a", b"file.txt", b"x" * 3, b"y" * 7, b"report-2025.pdf", b"z" * 19, b"h" * 20,
             b"q" * 23, b"w" * 24, b"e" * 40, b"r" * 60, b"t" * 63, b"u" * 64, b"i" * 100, b"o" * 255]
    for hint in hints:
        for diff, maxa in ((0, 500000), (1, 500000), (6, 500000), (8, 500000), (12, 500000),
                           (16, 500000), (20, 3000), (30, 0), (30, 100)):
            seed += 1
            cid = splitmix_bytes(seed, 32)
            size = int.from_bytes(splitmix_bytes(seed + 100000, 8), "little") >> (seed % 40)
            nonce = C.c_uint64()
            if diff == 30 and maxa == 0:  # clamp to 24 + default attempts: too slow, skip search
                continue
            if diff == 16 and len(hint) not in (0, 8, 24, 100):
                continue
            f = REF.ref_compute_store_pow(cid, size, hint, len(hint), diff, maxa, C.byref(nonce))
            case = {"chunk_id": cid.hex(), "payload_size": size, "hint": hint.hex(),
                    "difficulty": diff, "max_attempts": maxa, "found": bool(f),
                    "nonce": nonce.value if f else None}
            if f:
                case["valid"] = REF.ref_store_pow_valid(cid, size, hint, len(hint), nonce.value, diff) == 1
                case["valid_next"] = REF.ref_store_pow_valid(cid, size, hint, len(hint),
                                                             (nonce.value + 1) & (2**64 - 1), diff) == 1
            sp.append(case)
    g["store_pow"] = sp

    # -- handshake PoW (Node.cpp:233-292)
    hs = []
    for i in range(12):
        s = 21000 + 10 * i
        init, resp = splitmix_bytes(s, 32), splitmix_bytes(s + 1, 32)
        pub = int.from_bytes(splitmix_bytes(s + 2, 4), "little")
        diff = [0, 1, 4, 4, 6, 8, 8, 10, 11, 12, 12, 13][i]
        pieces = lp64(init) + lp64(resp) + [be64(pub)]
        f, nonce, att = node_search(pieces, diff, 500000)
        hs.append({"initiator": init.hex(), "responder": resp.hex(), "public": pub,
                   "difficulty": diff, "found": f, "nonce": nonce, "attempt": att})
    g["handshake_pow"] = hs

    # -- announce PoW (Node.cpp:155-230): strings of several lengths move the nonce through every
    # position of the final block (one- and two-block tails)
    an = []
    for i in range(24):
        s = 22000 + 10 * i
        cid, peer = splitmix_bytes(s, 32), splitmix_bytes(s + 1, 32)
        ep = (b"10.0.%d.%d:45000" % (i, 7 * i))[: 4 + (i * 5) % 17]
        uri = b"eph://" + splitmix_bytes(s + 2, (i * 13) % 61).hex().encode()[: (i * 13) % 61]
        shards = splitmix_bytes(s + 3, (i * 3) % 11)
        ttl = int.from_bytes(splitmix_bytes(s + 4, 3), "little")
        diff = [4, 6, 8, 10][i % 4]
        pieces = (lp64(cid) + lp64(peer) + lp64(ep) + lp64(uri) + lp64(shards) + [be64(ttl)])
        f, nonce, att = node_search(pieces, diff, 500000)
        an.append({"chunk_id": cid.hex(), "peer_id": peer.hex(), "endpoint": ep.hex(),
                   "manifest_uri": uri.hex(), "assigned_shards": shards.hex(), "ttl": ttl,
                   "difficulty": diff, "found": f, "nonce": nonce, "attempt": att,
                   "prefix_len": sum(len(p) for p in pieces)})
    g["announce_pow"] = an

    # -- KeyManager (KeyManager.cpp:15-46, 56-92)
    ks = []
    for i in range(8):
        secret = splitmix_bytes(23000 + i, 32)
        material = splitmix_bytes(23100 + i, 16)
        o = (C.c_uint8 * 32)()
        REF.ref_keymanager_material_key(secret, material, 16, o)
        now = int.from_bytes(splitmix_bytes(23200 + i, 7), "little") + 2_000_000_000
        o2 = (C.c_uint8 * 32)()
        assert REF.ref_keymanager_rotate(secret, now, o2) == now
        ks.append({"secret": secret.hex(), "material": material.hex(), "material_key": bytes(o).hex(),
                   "rotate_ticks": now, "rotate_counter": 1, "rotated_key": bytes(o2).hex()})
    g["session_keys"] = ks

    # -- sanitize_filename_hint (StoreProof.cpp:91-107)
    sn = []
    for raw in [b"", b".", b"..", b"a.txt", b"/tmp/x/report.pdf", b"dir/", b"C:/data/f.bin", b"./..",
                b"/abs/" + b"n" * 300, b"rel/path/with space.txt", b"/", b"x/.", b"x/.."]:
        out = (C.c_char * 512)()
        n = REF.ref_sanitize_filename_hint(raw, len(raw), out, 512)
        sn.append({"raw": raw.hex(), "result": None if n < 0 else bytes(out)[:n].hex()})
    g["sanitize_filename_hint"] = sn

    path = os.path.join(HERE, "pow.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
