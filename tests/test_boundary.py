"""CPU tests of the drop-in boundary: the C-ABI library builds and loads, exports exactly what
include/*.h declares (C and C++ API), the product package never reaches into oracle/, and the
Python host fails loudly (no CPU fallback) when the HIP library is absent."""
import ast
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ephemeralnet_amd")
LIB = os.path.join(PKG, "libenet_crypto.so")


@pytest.fixture(scope="module")
def built():
    from ephemeralnet_amd import build as B
    B.build(verbose=False)
    assert os.path.exists(LIB)
    return LIB


def header_c_functions():
    src = open(os.path.join(ROOT, "include", "enet_crypto.h")).read()
    return sorted(set(re.findall(r"ENET_API\s+[\w\s\*]+?\b(enet_\w+)\s*\(", src)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_header_declares_functions():
    fns = header_c_functions()
    assert "enet_aead_seal_batch" in fns and "enet_chacha20_xor_batch" in fns
    assert len(fns) >= 13


def test_c_abi_exports_every_declared_symbol(built):
    syms = exported(built)
    missing = [f for f in header_c_functions() if f not in syms]
    assert not missing, missing
    # nothing else with C linkage leaks out
    extra = [s for s in syms if s.startswith("enet_") and s not in header_c_functions()]
    assert not extra, extra


def test_cpp_api_exports_reference_signatures(built):
    out = subprocess.run(["nm", "-DC", "--defined-only", built], capture_output=True, text=True,
                         check=True).stdout
    for sig in [
        "ephemeralnet::crypto::ChaCha20::apply(ephemeralnet::crypto::Key const&, "
        "ephemeralnet::crypto::Nonce const&, std::span<unsigned char const",
        "ephemeralnet::crypto::Sha256::digest(std::span<unsigned char const",
        "ephemeralnet::crypto::Sha256::update(std::span<unsigned char const",
        "ephemeralnet::crypto::Sha256::finalize()",
        "ephemeralnet::crypto::HmacSha256::compute(std::span<unsigned char const",
        "ephemeralnet::crypto::HmacSha256::verify(std::span<unsigned char const",
        "ephemeralnet::crypto::CryptoManager::encrypt_with_key(",
        "ephemeralnet::crypto::CryptoManager::decrypt_with_key(",
        "ephemeralnet::crypto::CryptoManager::generate_key()",
        "ephemeralnet::security::compute_store_pow(ephemeralnet::security::StoreWorkInput const&, "
        "unsigned char, unsigned long)",
        "ephemeralnet::security::store_pow_valid(ephemeralnet::security::StoreWorkInput const&, "
        "unsigned long, unsigned char)",
        "ephemeralnet::security::derive_chunk_id(std::span<unsigned char const",
        "ephemeralnet::security::sanitize_filename_hint",
        "ephemeralnet::network::KeyManager::rotate_if_needed(",
        "ephemeralnet::network::KeyManager::register_session_with_material(",
        "ephemeralnet::network::KeyManager::current_key(",
        "ephemeralnet::crypto::batch::pow_search(",
    ]:
        assert sig in out, sig


def test_library_loads_and_host_helpers(built):
    import ephemeralnet_amd as E
    L = E.lib()
    assert L.enet_abi_version() >> 16 == 1
    # CryptoManager.cpp:8-13 derive_counter
    assert E.chunk_counter(bytes([1, 2, 3, 4]) + bytes(28)) == 0x04030201
    # scheduler: many records -> 1 lane, few large records -> more lanes, capped by blocks
    assert E.lanes_per_record(1 << 20, (1 << 20) * 1500, 1500) == 1
    assert E.lanes_per_record(65536, 65536 * 4096, 4096) == 2        # C2
    assert E.lanes_per_record(1 << 20, (1 << 20) * 1500, 1500) == 1  # C3
    assert E.lanes_per_record(32768, 32768 * 65536, 65536) == 4      # C4 per GPU
    assert E.lanes_per_record(64, 64 * 65536, 65536) == 16
    assert E.lanes_per_record(64, 64 * 64, 64) == 1
    assert E.lanes_per_record(100000, 100000 * 512, 512) == 1        # >= 8 blocks per lane
    with pytest.raises(E.EnetError):
        E.set_lanes_per_record(3)
    E.set_lanes_per_record(0)
    with pytest.raises(E.EnetError):
        E.set_staging(2)
    with pytest.raises(E.EnetError):
        E.set_staging(3)  # the LDS-DMA variant, retired in round 6
    E.set_staging(4)
    E.set_staging(5)
    E.set_staging(-1)
    # host-memory runtime modes 0, 3, 4 and -1 = auto (enet_host_set_mode); the retired 1 / 2
    # and anything else are refused with the mode kept
    prev = E.host_mode()
    for m in E.HOST_MODES + (-1,):
        E.set_host_mode(m)
        assert E.host_mode() == m
    E.set_host_mode(4)
    for bad in (1, 2, 5, -2):
        with pytest.raises(E.EnetError):
            E.set_host_mode(bad)
        assert E.host_mode() == 4
    E.set_host_mode(prev)


def test_invalid_arguments_rejected_without_gpu(built):
    import ctypes as C
    import ephemeralnet_amd as E
    L = E.lib()
    r = E._Records()
    r.count = 5  # null arenas
    assert L.enet_aead_seal_batch(C.byref(r), None, None, None, None) == -1
    assert b"NULL" in L.enet_last_error()
    assert L.enet_chacha20_xor_batch(None, None, None) == -1
    r.count = 0  # empty batch is a no-op
    assert L.enet_chacha20_xor_batch(C.byref(r), None, None) == 0
    # proof of work / session keys: NULL buffers and unknown schedules are rejected on the host
    assert L.enet_pow_search_batch(3, None, None, None, 0, 10, None, None, None, None) == -1
    buf = (C.c_uint8 * 64)()
    assert L.enet_pow_search_batch(3, buf, buf, buf, 7, 10, buf, None, buf, None) == -1
    assert b"schedule" in L.enet_last_error()
    assert L.enet_pow_check_batch(3, buf, None, buf, buf, buf, None) == -1
    assert L.enet_session_key_batch(3, None, buf, buf, buf, None) == -1
    assert L.enet_pow_search_batch(0, None, None, None, 0, 10, None, None, None, None) == 0
    # multi-device pipeline group: NULL group / descriptor rejected, size of NULL is 0
    assert L.enet_pipeline_group_size(None) == 0
    assert L.enet_pipeline_group_aead_seal(None, C.byref(r), buf) == -1
    g_bad = (C.c_int * 1)(-1)
    assert L.enet_pipeline_group_create(g_bad, 1, 0, 0) is None  # no such device
    assert b"enet_pipeline_group_create" in L.enet_last_error()


def test_product_never_imports_oracle():
    for dp, _, fs in os.walk(PKG):
        for f in fs:
            p = os.path.join(dp, f)
            if f.endswith(".py"):
                tree = ast.parse(open(p).read())
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        assert not any(a.name.split(".")[0] == "oracle" for a in node.names), p
                    if isinstance(node, ast.ImportFrom):
                        assert (node.module or "").split(".")[0] != "oracle", p
            if f.endswith((".cpp", ".hip", ".hpp", ".h")):
                assert "enet_oracle" not in open(p).read(), p


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    import ephemeralnet_amd as E
    monkeypatch.setattr(E, "_lib", None)
    monkeypatch.setattr(E, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(E.EnetError):
        E.lib()
