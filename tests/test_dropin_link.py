"""Drop-in boundary, checked with the reference's own callers.

CPU (needs /root/reference, so it is skipped on the GPU box): every reference translation unit
that includes a crypto header -- Message.cpp, SessionManager.cpp, KeyExchange.cpp, Node.cpp,
RelayClient.cpp, ControlServer.cpp, TokenChallenge.cpp, Manifest.cpp, main.cpp -- compiles
unmodified with include/ placed before the reference's include/, and every crypto / StoreProof /
KeyManager symbol those objects leave undefined is exported, with the identical mangled name, by
libenet_crypto.so.  Message.cpp & co. link into an executable (oracle/_ref/dropin_caller).

GPU: that executable -- the reference's encode_signed / decode_signed (Message.cpp:305-328) and
KeyExchange::derive_shared_secret (KeyExchange.cpp:34-47) running on the GPU library -- produces
HMAC-SHA256 / SHA-256 results equal to the CPU oracle's.  The binary was built in this
container; /root/reference is not read on the box.
"""
import hashlib
import hmac
import os
import subprocess

import pytest

from util import splitmix_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
DROPIN = os.path.join(ROOT, "oracle", "_ref", "dropin")
CALLER = os.path.join(ROOT, "oracle", "_ref", "dropin_caller")
LIB = os.path.join(ROOT, "ephemeralnet_amd", "libenet_crypto.so")
# namespaces this repo replaces (the rest -- Shamir, protocol, storage -- stays reference code)
REPLACED = ("ephemeralnet::crypto::ChaCha20", "ephemeralnet::crypto::Sha256",
            "ephemeralnet::crypto::HmacSha256", "ephemeralnet::crypto::CryptoManager",
            "ephemeralnet::security::", "ephemeralnet::network::KeyManager")

needs_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")),
                               reason="reference sources absent (GPU box)")


@pytest.fixture(scope="module")
def built():
    from ephemeralnet_amd import build as B
    B.build(verbose=False)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "dropin"], check=True)
    return DROPIN


@needs_ref
def test_reference_callers_compile_against_dropin_headers(built):
    objs = sorted(os.listdir(built))
    want = {"protocol_Message.o", "network_SessionManager.o", "network_KeyExchange.o", "core_Node.o",
            "network_RelayClient.o", "daemon_ControlServer.o", "bootstrap_TokenChallenge.o",
            "protocol_Manifest.o", "main.o"}
    assert want <= set(objs)


@needs_ref
def test_reference_callers_crypto_symbols_exported(built):
    exported = set()
    for ln in subprocess.run(["nm", "-D", "-C", "--defined-only", LIB], check=True, capture_output=True,
                             text=True).stdout.splitlines():
        exported.add(ln.split(" ", 2)[2])
    need = set()
    for o in os.listdir(built):
        for ln in subprocess.run(["nm", "-C", "-u", os.path.join(built, o)], check=True,
                                 capture_output=True, text=True).stdout.splitlines():
            sym = ln.strip()[2:].strip()
            if sym.startswith(REPLACED):
                need.add(sym)
    # the reference callers reach at least these entry points
    for s in ("ephemeralnet::crypto::HmacSha256::compute", "ephemeralnet::crypto::HmacSha256::verify",
              "ephemeralnet::crypto::ChaCha20::apply", "ephemeralnet::crypto::Sha256::digest",
              "ephemeralnet::crypto::CryptoManager::encrypt_with_key",
              "ephemeralnet::security::compute_store_pow", "ephemeralnet::network::KeyManager::current_key"):
        assert any(n.startswith(s + "(") for n in need), s
    missing = sorted(need - exported)
    assert not missing, missing


@needs_ref
def test_reference_callers_link(built):
    assert os.access(CALLER, os.X_OK)
    # every crypto symbol of the executable resolves into libenet_crypto.so, none into a copy
    out = subprocess.run(["ldd", CALLER], check=True, capture_output=True, text=True).stdout
    assert "libenet_crypto.so" in out
    defined = subprocess.run(["nm", "-C", "--defined-only", CALLER], check=True, capture_output=True,
                             text=True).stdout
    assert "crypto::HmacSha256::compute" not in defined and "crypto::Sha256::digest" not in defined


def _modexp(b, e, m):
    return pow(b, e, m)


@pytest.mark.gpu
def test_reference_callers_run_on_gpu_library():
    if not os.access(CALLER, os.X_OK):
        pytest.skip("oracle/_ref/dropin_caller not built (needs /root/reference at build time)")
    ops, cases = [], []
    for i, L in enumerate([0, 1, 31, 64, 98, 1000, 1500, 4096, 65536]):
        key = splitmix_bytes(9000 + i, 32 if i % 3 else 17)
        data = splitmix_bytes(9100 + i, L)
        ops.append(f"signed {key.hex()} {data.hex() or '-'} {60 + i}")
        cases.append(("signed", key, data))
    for a, b in [(3, 7), (123456789, 987654321), (2147483646, 2)]:
        ops.append(f"kex {a} {b}")
        cases.append(("kex", a, b))
    res = subprocess.run([CALLER], input="\n".join(ops) + "\n", capture_output=True, text=True,
                         check=True, timeout=300).stdout.splitlines()
    assert len(res) == len(ops)
    p = 2147483647
    for (kind, x, y), got in zip(cases, res):
        f = got.split()
        if kind == "signed":
            body, sig = bytes.fromhex(f[0]), bytes.fromhex(f[1])
            assert y in body
            assert sig == body + hmac.new(x, body, hashlib.sha256).digest()
            assert f[2:] == ["1", "1", "1"]
        else:
            shared = _modexp(pow(5, y, p) % p, x, p)
            assert f[0] == hashlib.sha256(shared.to_bytes(4, "big")).hexdigest() and f[1] == "1"
