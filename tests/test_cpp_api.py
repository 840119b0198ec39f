"""The C++ drop-in API (include/ephemeralnet/crypto/*.hpp, reference signatures) compiled the way a
reference caller would be, linked against libenet_crypto.so.  CPU: it compiles and links.
GPU: every reference entry point reproduces the golden vectors of the compiled reference."""
import hashlib
import os
import subprocess

import pytest

import oracle

from util import splitmix_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "api_test.cpp")


@pytest.fixture(scope="module")
def api_bin(tmp_path_factory):
    from ephemeralnet_amd import build as B
    lib = B.build(verbose=False)
    out = str(tmp_path_factory.mktemp("cpp") / "api_test")
    subprocess.run(["g++", "-std=c++20", "-O1", "-I", os.path.join(ROOT, "include"), SRC, "-o", out,
                    "-L", os.path.dirname(lib), "-lenet_crypto", "-Wl,-rpath," + os.path.dirname(lib)],
                   check=True)
    return out


def h(b: bytes) -> str:
    return b.hex() if b else "-"


def test_cpp_api_compiles_and_links(api_bin):
    assert os.access(api_bin, os.X_OK)


@pytest.mark.gpu
def test_cpp_api_matches_reference_golden(api_bin, golden):
    ops, expect = [], []
    for c in golden["chacha20"]:
        if c["len"] > 4097:
            continue
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        ops.append(f"chacha {c['key']} {c['nonce']} {c['counter']} {h(pt)}")
        expect.append(("hex", c["ct"]))
    for c in golden["sha256"]:
        data = b"abc" if c["abc"] else splitmix_bytes(c["seed"], c["len"])
        ops.append(f"sha {h(data)}")
        expect.append(("eq", c["digest"]))
        if c["digest_pieces_7"]:
            ops.append(f"sha_pieces 7 {h(data)}")
            expect.append(("eq", c["digest_pieces_7"]))
    for c in golden["hmac"]:
        ops.append(f"hmac {c['key'] or '-'} {h(splitmix_bytes(c['seed'], c['len']))}")
        expect.append(("eq", c["mac"]))
    for c in golden["hmac_verify"]:
        ops.append(f"hverify {c['key']} {h(splitmix_bytes(c['seed'], c['len']))} {c['mac']}")
        expect.append(("eq", "1" if c["ok"] else "0"))
    for c in golden["cryptomanager"]:
        if c["len"] > 4097:
            continue
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        import oracle
        ct = oracle.chacha20_xor(bytes.fromhex(c["key"]), bytes.fromhex(c["nonce"]), pt,
                                 oracle.derive_counter(bytes.fromhex(c["chunk_id"])))
        assert ("hex" not in c["ct"]) or ct.hex() == c["ct"]["hex"]
        ops.append(f"cm_dec {c['key']} {c['chunk_id']} {c['nonce']} {h(ct)}")
        expect.append(("eq", h(pt)))
        ops.append(f"cm_roundtrip {c['chunk_id']} {h(pt)}")
        expect.append(("eq", "1"))
    for f in golden["frames"]:
        m = bytes.fromhex(f["signed"])[:-32]
        ops.append(f"frame_seal {f['key']} {f['nonce']} {h(m)}")
        expect.append(("eq", f"{f['body']} 1"))
    for f in golden["frames"]:
        m = bytes.fromhex(f["signed"])[:-32]
        ops.append(f"wire_queue {f['key']} {h(m)}")
        expect.append(("wire", (bytes.fromhex(f["key"]), m)))
    for L in (0, 1, 64, 1500, 4096):
        pt = splitmix_bytes(777 + L, L)
        ops.append(f"chunk_pipe {h(pt)}")
        expect.append(("eq", f"{hashlib.sha256(pt).hexdigest()} 1"))
    for c in golden["aead"]:
        if c["aad_len"] or c["len"] > 1500:
            continue
        pt = splitmix_bytes(c["pt_seed"], c["len"])
        ops.append(f"aead_seal {c['key']} {c['nonce']} {h(pt)}")
        expect.append(("eq", f"{c['ct']['hex'] or '-'} {c['tag']}"))
    res = subprocess.run([api_bin], input="\n".join(ops) + "\n", capture_output=True, text=True,
                         check=True, timeout=300).stdout.splitlines()
    assert len(res) == len(ops)
    for op, (kind, e), got in zip(ops, expect, res):
        if kind == "hex":
            if "hex" in e:
                assert got == (e["hex"] or "-"), op[:60]
            else:
                assert hashlib.sha256(bytes.fromhex(got)).hexdigest() == e["sha256"]
        elif kind == "wire":  # random nonce: check the frame against the oracle with its nonce
            key, m = e
            fr, flag = got.split()
            fr = bytes.fromhex(fr)
            nonce, body = fr[:12], fr[16:]
            assert flag == "1" and int.from_bytes(fr[12:16], "big") == len(body) == len(m) + 32
            assert body == oracle.frame_seal(key, nonce, m)
        else:
            assert got == e, op[:60]


@pytest.mark.gpu
def test_cpp_pow_and_keys_match_reference_golden(api_bin):
    """security::StoreProof, crypto::batch PoW (Node.cpp announce / handshake) and
    network::KeyManager through the reference C++ signatures against tests/golden/pow.json."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "pow.json")) as f:
        pg = json.load(f)
    ops, expect = [], []
    for c in pg["store_pow"]:
        if c["max_attempts"] == 0:
            continue
        ops.append(f"store_pow {c['chunk_id']} {c['payload_size']} {c['hint'] or '-'} {c['difficulty']} "
                   f"{c['max_attempts']}")
        expect.append(f"{c['nonce']} {int(c['valid'])} {int(c['valid_next'])}" if c["found"] else "none")
    for c in pg["handshake_pow"]:
        ops.append(f"handshake_pow {c['initiator']} {c['responder']} {c['public']} {c['difficulty']}")
        dn = c["nonce"] if c["found"] else 2**64 - 1  # Node.cpp drop-in: nonce_out untouched if not found
        expect.append(f"{int(c['found'])} {c['nonce']} {c['attempt']} 1 {int(c['found'])} {dn}")
    for c in pg["announce_pow"]:
        ops.append("announce_pow " + " ".join(c[k] or "-" for k in ("chunk_id", "peer_id", "endpoint",
                                                                   "manifest_uri", "assigned_shards"))
                   + f" {c['ttl']} {c['difficulty']}")
        dn = c["nonce"] if c["found"] else 2**64 - 1
        expect.append(f"{int(c['found'])} {c['nonce']} {c['attempt']} {int(c['found'])} {dn}")
    for c in pg["session_keys"]:
        ops.append(f"keymgr {c['secret']} {c['material']} {c['rotate_ticks']}")
        expect.append(f"{c['material_key']} {c['rotated_key']} 1")
    for c in pg["sanitize_filename_hint"]:
        ops.append(f"sanitize {c['raw'] or '-'}")
        expect.append(c["result"] if c["result"] is not None else "none")
    for L in (0, 1, 4096):
        d = splitmix_bytes(40000 + L, L)
        ops.append(f"chunk_id {h(d)}")
        expect.append(hashlib.sha256(d).hexdigest())
    res = subprocess.run([api_bin], input="\n".join(ops) + "\n", capture_output=True, text=True,
                         check=True, timeout=300).stdout.splitlines()
    assert len(res) == len(ops)
    for op, e, got in zip(ops, expect, res):
        assert got == e, op[:80]
