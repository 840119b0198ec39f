"""Pin the oracle's proof-of-work and session-key restatement (oracle/enet_oracle.c) to
tests/golden/pow.json: the reference StoreProof.cpp / KeyManager.cpp themselves, Node.cpp's PoW
searches over the reference Sha256 and libstdc++ std::mt19937_64.  CPU only."""
import json
import os

import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def pg():
    with open(os.path.join(HERE, "golden", "pow.json")) as f:
        return json.load(f)


def test_mt19937_64(pg):
    for c in pg["mt19937_64"]:
        s = oracle.mt19937_64(c["seed"], 700)
        assert s[:5] == c["first"]
        assert s[311:316] == c["at_311_315"]  # first twist boundary
        assert s[623:628] == c["at_623_627"]
        assert s[0] == c["uniform_first"]    # uniform_int_distribution(0, max) == raw draw


def test_store_pow(pg):
    for c in pg["store_pow"]:
        pre = oracle.store_pow_prefix(bytes.fromhex(c["chunk_id"]), c["payload_size"],
                                      bytes.fromhex(c["hint"]))
        d = min(c["difficulty"], 24)  # StoreProof.cpp:128-130
        f, nonce, _ = oracle.pow_search(pre, d, 1, c["max_attempts"])
        assert f == c["found"], c
        if f:
            assert nonce == c["nonce"]
            assert oracle.pow_check(pre, nonce, d) == c["valid"]
            assert oracle.pow_check(pre, (nonce + 1) % 2**64, d) == c["valid_next"]


def test_handshake_pow(pg):
    for c in pg["handshake_pow"]:
        pre = oracle.handshake_pow_prefix(bytes.fromhex(c["initiator"]), bytes.fromhex(c["responder"]),
                                          c["public"])
        assert len(pre) == 88
        f, nonce, att = oracle.pow_search(pre, c["difficulty"], 0, 500000)
        assert (f, nonce, att) == (c["found"], c["nonce"], c["attempt"])


def test_announce_pow(pg):
    for c in pg["announce_pow"]:
        pre = oracle.announce_pow_prefix(*(bytes.fromhex(c[k]) for k in
                                           ("chunk_id", "peer_id", "endpoint", "manifest_uri",
                                            "assigned_shards")), c["ttl"])
        assert len(pre) == c["prefix_len"]
        f, nonce, att = oracle.pow_search(pre, c["difficulty"], 0, 500000)
        assert (f, nonce, att) == (c["found"], c["nonce"], c["attempt"])


def test_leading_zero_bits():
    assert oracle.leading_zero_bits(bytes(32)) == 256
    assert oracle.leading_zero_bits(bytes([0, 0x10]) + bytes(30)) == 11
    assert oracle.leading_zero_bits(bytes([0x80]) + bytes(31)) == 0


def test_session_keys(pg):
    for c in pg["session_keys"]:
        secret = bytes.fromhex(c["secret"])
        # register_session: material = BE64(0) || BE64(ticks) (KeyManager.cpp:15-30)
        m = bytes.fromhex(c["material"])
        assert oracle.hmac_sha256(secret, m).hex() == c["material_key"]
        assert oracle.session_key(secret, c["rotate_counter"], c["rotate_ticks"]).hex() == c["rotated_key"]
