"""GPU parity of the proof-of-work search / check and the session-key derivation (SURVEY.md 8f
rows 3-4) through the C ABI: against tests/golden/pow.json (reference StoreProof.cpp /
KeyManager.cpp; Node.cpp searches over the reference Sha256 + libstdc++ mt19937_64) and against
the CPU oracle on seeded random jobs.  Bit-exact: same found flag, nonce and attempt index."""
import json
import os

import numpy as np
import pytest

import oracle
from util import splitmix_bytes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def enet():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import ephemeralnet_amd as E
    E.lib()
    return E


@pytest.fixture(scope="module")
def pg():
    with open(os.path.join(HERE, "golden", "pow.json")) as f:
        return json.load(f)


def dev_arena(items):
    import torch
    offs = np.zeros(len(items) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in items])
    buf = np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8).copy()
    return torch.from_numpy(buf).cuda(), torch.from_numpy(offs).cuda()


def gpu_search(E, prefixes, diffs, schedule, max_attempts):
    import torch
    arena, offs = dev_arena(prefixes)
    n = len(prefixes)
    d = torch.tensor(diffs, dtype=torch.uint8).cuda()
    nonces = torch.full((n,), -1, dtype=torch.int64).cuda()
    atts = torch.full((n,), -1, dtype=torch.int64).cuda()
    found = torch.full((n,), 7, dtype=torch.uint8).cuda()
    E.pow_search(arena, offs, d, schedule, max_attempts, nonces, found, atts)
    torch.cuda.synchronize()
    u = lambda t: [int(x) & 0xFFFFFFFFFFFFFFFF for x in t.cpu().tolist()]
    return [bool(x) for x in found.cpu().tolist()], u(nonces), u(atts)


def gpu_check(E, prefixes, nonces, diffs):
    import torch
    arena, offs = dev_arena(prefixes)
    nn = torch.tensor(np.array(nonces, dtype=np.uint64).view(np.int64)).cuda()
    d = torch.tensor(diffs, dtype=torch.uint8).cuda()
    ok = torch.full((len(prefixes),), 7, dtype=torch.uint8).cuda()
    E.pow_check(arena, offs, nn, d, ok)
    torch.cuda.synchronize()
    return [bool(x) for x in ok.cpu().tolist()]


def test_store_pow_golden(enet, pg):
    by_max = {}
    for c in pg["store_pow"]:
        by_max.setdefault(c["max_attempts"], []).append(c)
    for maxa, cs in by_max.items():
        pre = [oracle.store_pow_prefix(bytes.fromhex(c["chunk_id"]), c["payload_size"],
                                       bytes.fromhex(c["hint"])) for c in cs]
        f, nonce, _ = gpu_search(enet, pre, [min(c["difficulty"], 24) for c in cs], enet.POW_STORE, maxa)
        for c, fi, ni in zip(cs, f, nonce):
            assert fi == c["found"], c
            if fi:
                assert ni == c["nonce"], c
        found = [(p, n, min(c["difficulty"], 24)) for p, n, c, fi in zip(pre, nonce, cs, f) if fi]
        if found:
            ok = gpu_check(enet, [x[0] for x in found], [x[1] for x in found], [x[2] for x in found])
            assert all(ok)
            ok2 = gpu_check(enet, [x[0] for x in found], [(x[1] + 1) % 2**64 for x in found],
                            [x[2] for x in found])
            want = [c["valid_next"] for c, fi in zip(cs, f) if fi]
            assert ok2 == want


def test_node_pow_golden(enet, pg):
    pre, diffs, want = [], [], []
    for c in pg["handshake_pow"]:
        pre.append(oracle.handshake_pow_prefix(bytes.fromhex(c["initiator"]),
                                               bytes.fromhex(c["responder"]), c["public"]))
        diffs.append(c["difficulty"])
        want.append((c["found"], c["nonce"], c["attempt"]))
    for c in pg["announce_pow"]:
        pre.append(oracle.announce_pow_prefix(*(bytes.fromhex(c[k]) for k in
                                                ("chunk_id", "peer_id", "endpoint", "manifest_uri",
                                                 "assigned_shards")), c["ttl"]))
        diffs.append(c["difficulty"])
        want.append((c["found"], c["nonce"], c["attempt"]))
    f, nonce, att = gpu_search(enet, pre, diffs, enet.POW_NODE, 500000)
    for w, g in zip(want, zip(f, nonce, att)):
        assert g == w
    # one job at a time (16 waves per workgroup) gives the same answers
    for i in (0, 5, len(pre) - 1):
        g = gpu_search(enet, [pre[i]], [diffs[i]], enet.POW_NODE, 500000)
        assert (g[0][0], g[1][0], g[2][0]) == want[i]


def random_jobs(seed, n, max_len):
    lens = np.frombuffer(splitmix_bytes(seed, 4 * n), dtype="<u4") % (max_len + 1)
    pre = [splitmix_bytes(seed + 1 + i, int(L)) for i, L in enumerate(lens)]
    diffs = [int(x) % 13 for x in np.frombuffer(splitmix_bytes(seed + 7, n), dtype=np.uint8)]
    return pre, diffs


@pytest.mark.parametrize("schedule", [0, 1])
@pytest.mark.parametrize("n,maxa", [(1, 5000), (7, 3000), (300, 700), (4500, 64), (200, 1)])
def test_random_vs_oracle(enet, schedule, n, maxa):
    pre, diffs = random_jobs(31000 + 17 * n + schedule, n, 200)
    f, nonce, att = gpu_search(enet, pre, diffs, schedule, maxa)
    idx = range(n) if n <= 300 else range(0, n, 9)
    for i in idx:
        of, on, oa = oracle.pow_search(pre[i], diffs[i], schedule, maxa)
        assert (f[i], att[i]) == (of, oa if of else maxa), (i, len(pre[i]), diffs[i])
        if of:
            assert nonce[i] == on, (i, len(pre[i]), diffs[i])


def test_every_tail_length(enet):
    """Prefix lengths 0..130: the nonce at every byte offset of a one- or two-block tail."""
    pre = [splitmix_bytes(32000 + L, L) for L in range(131)]
    for schedule in (0, 1):
        f, nonce, att = gpu_search(enet, pre, [7] * len(pre), schedule, 4000)
        for i, p in enumerate(pre):
            of, on, oa = oracle.pow_search(p, 7, schedule, 4000)
            assert f[i] == of and att[i] == (oa if of else 4000), i
            if of:
                assert nonce[i] == on, i


def test_check_random(enet):
    pre, _ = random_jobs(33000, 500, 150)
    nonces = [int.from_bytes(splitmix_bytes(34000 + i, 8), "little") for i in range(500)]
    diffs = [i % 4 for i in range(500)]  # 0..3: a good share of random nonces pass
    ok = gpu_check(enet, pre, nonces, diffs)
    assert ok == [oracle.pow_check(p, n, d) for p, n, d in zip(pre, nonces, diffs)]
    assert 0 < sum(ok) < 500


def test_edge_cases(enet):
    import torch
    # difficulty 0 -> nonce 0 at attempt 0 (StoreProof.cpp:127, Node.cpp:213-216)
    f, nonce, att = gpu_search(enet, [b"abc", b""], [0, 0], 1, 500000)
    assert f == [True, True] and nonce == [0, 0] and att == [0, 0]
    # max_attempts 0: nothing searched
    f, nonce, att = gpu_search(enet, [b"abc"], [3], 0, 0)
    assert f == [False] and att == [0]
    # unreachable difficulty: not found after exactly max_attempts
    f, _, att = gpu_search(enet, [b"x" * 50], [200], 1, 2000)
    assert f == [False] and att == [2000]
    # empty batch is a no-op
    e = torch.zeros(1, dtype=torch.uint8).cuda()
    o = torch.zeros(1, dtype=torch.int64).cuda()
    enet.pow_search(e, o, e, 0, 10, o, e)


def test_full_size_batch_properties(enet):
    """65 536 store jobs at the reference default difficulty (Config.hpp store_pow_difficulty 6):
    every nonce found passes the GPU check, the attempt index is consistent with the found flag,
    and a sample agrees with the oracle."""
    n = 65536
    pre = [oracle.store_pow_prefix(splitmix_bytes(35000 + i, 32), 4096, b"") for i in range(n)]
    f, nonce, att = gpu_search(enet, pre, [6] * n, 1, 500000)
    assert all(f)
    assert all(gpu_check(enet, pre, nonce, [6] * n))
    for i in range(0, n, 4099):
        assert oracle.pow_search(pre[i], 6, 1, 500000) == (True, nonce[i], att[i])


def test_session_keys_golden_and_random(enet, pg):
    import torch
    cs = pg["session_keys"]
    secrets = b"".join(bytes.fromhex(c["secret"]) for c in cs)
    # register_session material BE64(0) || BE64(ticks) is the counter-0 form of derive_key
    ctr = [c["rotate_counter"] for c in cs] + [int.from_bytes(bytes.fromhex(c["material"])[:8], "big")
                                              for c in cs]
    ticks = [c["rotate_ticks"] for c in cs] + [int.from_bytes(bytes.fromhex(c["material"])[8:], "big", signed=True)
                                              for c in cs]
    sec = torch.frombuffer(bytearray(secrets * 2), dtype=torch.uint8).cuda()
    out = torch.zeros(32 * len(ctr), dtype=torch.uint8).cuda()
    enet.session_keys(sec, torch.tensor(np.array(ctr, dtype=np.uint64).view(np.int64)).cuda(),
                      torch.tensor(ticks, dtype=torch.int64).cuda(), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    want = [c["rotated_key"] for c in cs] + [c["material_key"] for c in cs]
    assert [got[32 * i:32 * i + 32].hex() for i in range(len(want))] == want
    # random batch vs the oracle
    n = 5000
    sec = splitmix_bytes(36000, 32 * n)
    ctr = np.frombuffer(splitmix_bytes(36001, 8 * n), dtype=np.uint64)
    tk = np.frombuffer(splitmix_bytes(36002, 8 * n), dtype=np.int64)
    out = torch.zeros(32 * n, dtype=torch.uint8).cuda()
    enet.session_keys(torch.frombuffer(bytearray(sec), dtype=torch.uint8).cuda(),
                      torch.from_numpy(ctr.view(np.int64).copy()).cuda(),
                      torch.from_numpy(tk.copy()).cuda(), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().tobytes()
    for i in range(0, n, 97):
        assert got[32 * i:32 * i + 32] == oracle.session_key(sec[32 * i:32 * i + 32], int(ctr[i]), int(tk[i]))
