"""ephemeralnet_amd -- MI355X bulk crypto engine for EphemeralNet's data path.

Python view of libenet_crypto.so's C ABI (include/enet_crypto.h) over torch device tensors
(torch is plumbing here: device memory and streams).  The product path is the HIP library:
there is no CPU fallback, and importing the package without the built library raises.

Operations mirror the reference src/crypto API, batched (ShardianLabs/EphemeralNet):
  chacha20_xor   ChaCha20::apply            src/crypto/ChaCha20.cpp:98-121
  aead_seal/open RFC 8439 (README.md:49 promise; no reference implementation)
  sha256         Sha256::digest             src/crypto/Sha256.cpp:128-132
  hmac_sha256    HmacSha256::compute/verify src/crypto/HmacSha256.cpp:11-54
  frame_seal/open encode_signed + SessionManager frame body
                  src/protocol/Message.cpp:305-328, src/network/SessionManager.cpp:362-374,815-822
  pow_search/check compute_store_pow / compute_{announce,handshake}_pow and the *_valid checks
                  src/security/StoreProof.cpp:109-146, src/core/Node.cpp:193-292
  session_keys   KeyManager::derive_key     src/network/KeyManager.cpp:74-92
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
# ENET_LIB_PATH: a differently-built copy of the library (tuning builds under tools/)
LIB_PATH = os.environ.get("ENET_LIB_PATH") or os.path.join(PKG, "libenet_crypto.so")

ENET_OK = 0


class EnetError(RuntimeError):
    pass


class _Records(C.Structure):
    _fields_ = [
        ("count", C.c_uint32),
        ("in_offsets", C.c_void_p),
        ("out_offsets", C.c_void_p),
        ("in_", C.c_void_p),
        ("out", C.c_void_p),
        ("keys", C.c_void_p),
        ("key_stride", C.c_uint32),
        ("nonces", C.c_void_p),
        ("order", C.c_void_p),
        ("total_bytes_hint", C.c_uint64),
        ("max_len_hint", C.c_uint32),
    ]


EXPORTS = [
    "enet_chacha20_xor_batch", "enet_aead_seal_batch", "enet_aead_open_batch",
    "enet_sha256_batch", "enet_hmac_sha256_batch", "enet_hmac_sha256_verify_batch",
    "enet_frame_seal_batch", "enet_frame_open_batch", "enet_wire_seal_batch",
    "enet_wire_open_batch", "enet_hmac_midstates", "enet_wire_seal_batch_sessions",
    "enet_wire_open_batch_sessions", "enet_chunk_store_batch", "enet_chunk_fetch_batch",
    "enet_aead_hmac_seal_batch",
    "enet_aead_hmac_open_batch", "enet_chunk_counter",
    "enet_lanes_per_record", "enet_set_lanes_per_record", "enet_set_staging", "enet_set_duplex_split",
    "enet_set_seg_min", "enet_seg_batches", "enet_set_host_hash_min", "enet_host_hash_batches", "enet_last_error",
    "enet_abi_version", "enet_pipeline_create", "enet_pipeline_destroy",
    "enet_pipeline_chacha20_xor", "enet_pipeline_aead_seal", "enet_pipeline_aead_open",
    "enet_pipeline_aead_hmac_seal", "enet_pipeline_aead_hmac_open", "enet_pipeline_wire_seal",
    "enet_pipeline_wire_open", "enet_host_set_mode", "enet_host_mode", "enet_host_alloc",
    "enet_host_free", "enet_pipeline_group_create", "enet_pipeline_group_destroy",
    "enet_pipeline_group_size", "enet_pipeline_group_chacha20_xor", "enet_pipeline_group_aead_seal",
    "enet_pipeline_group_aead_open", "enet_pipeline_group_aead_hmac_seal",
    "enet_pipeline_group_aead_hmac_open", "enet_pow_search_batch", "enet_pow_check_batch", "enet_session_key_batch",
    "enet_host_mode_probe", "enet_host_mode_auto", "enet_host_mode_for", "enet_pipeline_stats", "enet_device_numa_node",
    "enet_host_cpu_budget", "enet_host_pinned_bytes", "enet_host_plan", "enet_host_register",
    "enet_host_unregister",
]


class HostStats(C.Structure):
    """enet_host_stats (include/enet_crypto.h): a pipeline's counters and where its host side runs."""
    _fields_ = [(k, C.c_uint64) for k in ("jobs", "chunks", "records", "in_bytes", "out_bytes",
                                          "gathered_bytes", "scattered_bytes", "direct_in_chunks",
                                          "direct_out_chunks", "pinned_bytes")] + [
        ("device_node", C.c_int32), ("target_node", C.c_int32), ("staging_node", C.c_int32),
        ("workers", C.c_uint32), ("cpu_budget", C.c_uint32), ("spin", C.c_int32), ("mode", C.c_int32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class HostProbe(C.Structure):
    """enet_host_probe: a device's auto host-mode state (best GiB/s per mode, jobs sampled, decision)."""
    _fields_ = [("splitk_gibs", C.c_double), ("zcout_gibs", C.c_double), ("samples_splitk", C.c_int32),
                ("samples_zcout", C.c_int32), ("mode", C.c_int32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class HostPlan(C.Structure):
    """enet_host_plan_t: the host worker plan for given CPU / NUMA facts."""
    _fields_ = [("budget", C.c_uint32), ("workers", C.c_uint32), ("spin", C.c_int32), ("ncpus", C.c_uint32),
                ("cpus", C.c_char * 256)]

POW_NODE = 0   # candidates start + attempt (Node.cpp announce / handshake)
POW_STORE = 1  # candidates = successive mt19937_64 outputs (StoreProof.cpp)

_lib: Optional[C.CDLL] = None


def check_stamp() -> dict:
    """The in-tree library must have been built from the sources beside it: its stamp
    (libenet_crypto.so.stamp.json, written by build.py) carries the SHA-256 of the compiler
    flags, csrc/ and include/.  A stale or unstamped library raises instead of silently running
    old kernels (ENET_ALLOW_STALE_LIB=1 overrides, e.g. for tools' own builds)."""
    from . import build as B
    if os.path.abspath(LIB_PATH) != os.path.abspath(B.LIB) or os.environ.get("ENET_ALLOW_STALE_LIB") == "1":
        return {}
    st = B.read_stamp(B.LIB)
    want = B.source_digest()
    if st is None or st.get("sources_sha256") != want:
        raise EnetError(f"{LIB_PATH} was not built from these sources (stamp "
                        f"{None if st is None else st.get('sources_sha256', '?')[:12]}, sources "
                        f"{want[:12]}): rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    return st


def lib() -> C.CDLL:
    """Load the in-tree HIP library (fails loudly when it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EnetError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                            "g.build()'` (hipcc --offload-arch=gfx950)")
        check_stamp()
        L = C.CDLL(LIB_PATH)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        rp = C.POINTER(_Records)
        L.enet_chacha20_xor_batch.argtypes = [rp, vp, vp]
        L.enet_aead_seal_batch.argtypes = [rp, vp, vp, vp, vp]
        L.enet_aead_open_batch.argtypes = [rp, vp, vp, vp, vp, vp]
        L.enet_sha256_batch.argtypes = [u32, vp, vp, vp, vp]
        L.enet_hmac_sha256_batch.argtypes = [u32, vp, vp, u32, vp, vp, vp, vp]
        L.enet_hmac_sha256_verify_batch.argtypes = [u32, vp, vp, u32, vp, vp, vp, vp, vp]
        L.enet_frame_seal_batch.argtypes = [rp, vp]
        L.enet_frame_open_batch.argtypes = [rp, vp, vp, vp]
        L.enet_wire_seal_batch.argtypes = [rp, vp]
        L.enet_wire_open_batch.argtypes = [rp, vp, vp, vp]
        L.enet_hmac_midstates.argtypes = [vp, u32, vp, vp]
        L.enet_wire_seal_batch_sessions.argtypes = [rp, vp, u32, vp, vp]
        L.enet_wire_open_batch_sessions.argtypes = [rp, vp, u32, vp, vp, vp, vp]
        L.enet_chunk_store_batch.argtypes = [rp, vp, vp, vp]
        L.enet_chunk_fetch_batch.argtypes = [rp, vp, vp, vp, vp]
        L.enet_aead_hmac_seal_batch.argtypes = [rp, vp, vp, vp]
        L.enet_aead_hmac_open_batch.argtypes = [rp, vp, vp, vp, vp]
        L.enet_chunk_counter.argtypes = [C.c_char_p]
        L.enet_chunk_counter.restype = u32
        L.enet_lanes_per_record.argtypes = [u32, u64, u32]
        L.enet_lanes_per_record.restype = u32
        L.enet_set_lanes_per_record.argtypes = [u32]
        L.enet_set_staging.argtypes = [C.c_int]
        L.enet_set_duplex_split.argtypes = [C.c_int]
        L.enet_set_seg_min.argtypes = [C.c_int64]
        L.enet_seg_batches.restype = C.c_uint64
        L.enet_set_host_hash_min.argtypes = [C.c_int64]
        L.enet_host_hash_batches.restype = C.c_uint64
        L.enet_last_error.restype = C.c_char_p
        L.enet_pipeline_create.argtypes = [C.c_int, u64, u32]
        L.enet_pipeline_create.restype = vp
        L.enet_pipeline_destroy.argtypes = [vp]
        L.enet_pipeline_chacha20_xor.argtypes = [vp, rp, vp]
        L.enet_pipeline_aead_seal.argtypes = [vp, rp, vp]
        L.enet_pipeline_aead_open.argtypes = [vp, rp, vp, vp]
        L.enet_pipeline_aead_hmac_seal.argtypes = [vp, rp, vp, vp]
        L.enet_pipeline_aead_hmac_open.argtypes = [vp, rp, vp, vp, vp]
        L.enet_pipeline_wire_seal.argtypes = [vp, rp]
        L.enet_pipeline_wire_open.argtypes = [vp, rp, vp]
        L.enet_host_set_mode.argtypes = [C.c_int]
        L.enet_pipeline_group_create.argtypes = [vp, u32, u64, u32]
        L.enet_pipeline_group_create.restype = vp
        L.enet_pipeline_group_destroy.argtypes = [vp]
        L.enet_pipeline_group_size.argtypes = [vp]
        L.enet_pipeline_group_size.restype = u32
        L.enet_pipeline_group_chacha20_xor.argtypes = [vp, rp, vp]
        L.enet_pipeline_group_aead_seal.argtypes = [vp, rp, vp]
        L.enet_pipeline_group_aead_open.argtypes = [vp, rp, vp, vp]
        L.enet_pipeline_group_aead_hmac_seal.argtypes = [vp, rp, vp, vp]
        L.enet_pipeline_group_aead_hmac_open.argtypes = [vp, rp, vp, vp, vp]
        L.enet_host_alloc.argtypes = [u64]
        L.enet_host_alloc.restype = vp
        L.enet_host_free.argtypes = [vp]
        L.enet_abi_version.restype = u32
        L.enet_pow_search_batch.argtypes = [u32, vp, vp, vp, C.c_int, u64, vp, vp, vp, vp]
        L.enet_pow_check_batch.argtypes = [u32, vp, vp, vp, vp, vp, vp]
        L.enet_session_key_batch.argtypes = [u32, vp, vp, vp, vp, vp]
        L.enet_host_mode_probe.argtypes = [C.c_int, C.POINTER(HostProbe)]
        L.enet_host_mode_auto.argtypes = [C.c_int, C.POINTER(HostProbe)]
        L.enet_host_mode_for.argtypes = [C.POINTER(HostProbe)]
        L.enet_pipeline_stats.argtypes = [vp, C.POINTER(HostStats)]
        L.enet_device_numa_node.argtypes = [C.c_int]
        L.enet_host_cpu_budget.restype = u32
        L.enet_host_pinned_bytes.restype = u64
        L.enet_host_plan.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, u32, u32, C.POINTER(HostPlan)]
        L.enet_host_register.argtypes = [vp, u64]
        L.enet_host_unregister.argtypes = [vp]
        for name in EXPORTS:
            getattr(L, name)
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != ENET_OK:
        msg = lib().enet_last_error().decode(errors="replace")
        raise EnetError(f"{what} failed ({rc}): {msg}")


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _stream(stream) -> Optional[int]:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


@dataclass
class Batch:
    """Device-resident SoA record batch (all torch tensors on the GPU).

    arena: uint8 [total]; offsets: int64 [n+1]; keys: uint8 [n,32] (or [1,32] with
    key_stride=0); nonces: uint8 [n,12].  `out`/`out_offsets` default to a same-shape arena.
    """
    arena: "object"
    offsets: "object"
    keys: "object"
    nonces: "object"
    key_stride: int = 32
    order: "object" = None
    total_bytes_hint: int = 0
    max_len_hint: int = 0

    @property
    def n(self) -> int:
        return int(self.offsets.numel()) - 1

    def records(self, out, out_offsets) -> _Records:
        r = _Records()
        r.count = self.n
        r.in_offsets = _ptr(self.offsets)
        r.out_offsets = _ptr(out_offsets)
        r.in_ = _ptr(self.arena)
        r.out = _ptr(out)
        r.keys = _ptr(self.keys)
        r.key_stride = self.key_stride
        r.nonces = _ptr(self.nonces)
        r.order = _ptr(self.order)
        r.total_bytes_hint = self.total_bytes_hint
        r.max_len_hint = self.max_len_hint
        return r


def set_seg_min(nbytes: int) -> None:
    """enet_set_seg_min: -1 automatic; >= 0 every record of at least nbytes takes the
    sequence-parallel tiles (segments.hip); 2**63-1 never."""
    _check(lib().enet_set_seg_min(int(nbytes)), "enet_set_seg_min")


def seg_batches() -> int:
    return int(lib().enet_seg_batches())


SEG_MIN = 256 << 10
SEG_NEVER = (1 << 63) - 1


def set_host_hash_min(nbytes: int) -> None:
    """enet_set_host_hash_min: chunk store / fetch records of at least nbytes hash on host
    threads while the device ciphers them (-1 automatic; 2**63-1 never: every chain on the GPU)."""
    _check(lib().enet_set_host_hash_min(int(nbytes)), "enet_set_host_hash_min")


def host_hash_batches() -> int:
    return int(lib().enet_host_hash_batches())


HOST_HASH_MIN = 256 << 10


def chacha20_xor(b: Batch, out, counters=None, out_offsets=None, stream=None) -> None:
    r = b.records(out, b.offsets if out_offsets is None else out_offsets)
    _check(lib().enet_chacha20_xor_batch(C.byref(r), _ptr(counters), _stream(stream)),
           "enet_chacha20_xor_batch")


def aead_seal(b: Batch, out, tags, aad=None, aad_offsets=None, stream=None) -> None:
    r = b.records(out, b.offsets)
    _check(lib().enet_aead_seal_batch(C.byref(r), _ptr(aad), _ptr(aad_offsets), _ptr(tags),
                                      _stream(stream)), "enet_aead_seal_batch")


def aead_open(b: Batch, out, tags, ok, aad=None, aad_offsets=None, stream=None) -> None:
    r = b.records(out, b.offsets)
    _check(lib().enet_aead_open_batch(C.byref(r), _ptr(aad), _ptr(aad_offsets), _ptr(tags),
                                      _ptr(ok), _stream(stream)), "enet_aead_open_batch")


def aead_hmac_seal(b: Batch, out, tags, macs, stream=None) -> None:
    """AEAD seal + HMAC-SHA256(key_i, plaintext_i)."""
    r = b.records(out, b.offsets)
    _check(lib().enet_aead_hmac_seal_batch(C.byref(r), _ptr(tags), _ptr(macs), _stream(stream)),
           "enet_aead_hmac_seal_batch")


def aead_hmac_open(b: Batch, out, tags, macs, ok, stream=None) -> None:
    r = b.records(out, b.offsets)
    _check(lib().enet_aead_hmac_open_batch(C.byref(r), _ptr(tags), _ptr(macs), _ptr(ok),
                                           _stream(stream)), "enet_aead_hmac_open_batch")


def sha256(arena, offsets, digests, stream=None) -> None:
    n = int(offsets.numel()) - 1
    _check(lib().enet_sha256_batch(n, _ptr(arena), _ptr(offsets), _ptr(digests), _stream(stream)),
           "enet_sha256_batch")


def hmac_sha256(keys, arena, offsets, macs, key_offsets=None, key_stride=32, stream=None) -> None:
    n = int(offsets.numel()) - 1
    _check(lib().enet_hmac_sha256_batch(n, _ptr(keys), _ptr(key_offsets), key_stride, _ptr(arena),
                                        _ptr(offsets), _ptr(macs), _stream(stream)),
           "enet_hmac_sha256_batch")


def hmac_sha256_verify(keys, arena, offsets, macs, ok, key_offsets=None, key_stride=32,
                       stream=None) -> None:
    n = int(offsets.numel()) - 1
    _check(lib().enet_hmac_sha256_verify_batch(n, _ptr(keys), _ptr(key_offsets), key_stride,
                                               _ptr(arena), _ptr(offsets), _ptr(macs), _ptr(ok),
                                               _stream(stream)), "enet_hmac_sha256_verify_batch")


def frame_seal(b: Batch, out, out_offsets, stream=None) -> None:
    r = b.records(out, out_offsets)
    _check(lib().enet_frame_seal_batch(C.byref(r), _stream(stream)), "enet_frame_seal_batch")


def frame_open(b: Batch, out, out_offsets, macs, ok, stream=None) -> None:
    r = b.records(out, out_offsets)
    _check(lib().enet_frame_open_batch(C.byref(r), _ptr(macs), _ptr(ok), _stream(stream)),
           "enet_frame_open_batch")


def wire_seal(b: Batch, out, out_offsets, stream=None) -> None:
    """Whole wire frames nonce || BE32 len || ChaCha20(m || HMAC(m)) (SessionManager.cpp:362-387)."""
    r = b.records(out, out_offsets)
    _check(lib().enet_wire_seal_batch(C.byref(r), _stream(stream)), "enet_wire_seal_batch")


def wire_open(b: Batch, out, out_offsets, macs, ok, stream=None) -> None:
    """b.arena holds received wire frames; nonces come from the frames (b.nonces may be None)."""
    r = b.records(out, out_offsets)
    _check(lib().enet_wire_open_batch(C.byref(r), _ptr(macs), _ptr(ok), _stream(stream)),
           "enet_wire_open_batch")


def hmac_midstates(keys, n: int, mid, stream=None) -> None:
    """mid[16 i .. 16 i + 16) = HMAC-SHA256 ipad / opad midstates of the 32-byte key i."""
    _check(lib().enet_hmac_midstates(_ptr(keys), n, _ptr(mid), _stream(stream)), "enet_hmac_midstates")


def wire_seal_sessions(b: Batch, out, out_offsets, session, sessions: int, mid, stream=None) -> None:
    """wire_seal with b.keys a table of `sessions` keys, session[i] (int32) the session of frame i
    and mid the table's hmac_midstates (same bytes as wire_seal with per-frame keys
    table[session[i]]; an index >= sessions zeroes that frame's whole output slot)."""
    r = b.records(out, out_offsets)
    _check(lib().enet_wire_seal_batch_sessions(C.byref(r), _ptr(session), sessions, _ptr(mid),
                                               _stream(stream)), "enet_wire_seal_batch_sessions")


def wire_open_sessions(b: Batch, out, out_offsets, session, sessions: int, mid, macs, ok, stream=None) -> None:
    """wire_open under a session-key table (see wire_seal_sessions); ok[i] = 0 for an index >= sessions."""
    r = b.records(out, out_offsets)
    _check(lib().enet_wire_open_batch_sessions(C.byref(r), _ptr(session), sessions, _ptr(mid), _ptr(macs),
                                               _ptr(ok), _stream(stream)), "enet_wire_open_batch_sessions")


def chunk_store(b: Batch, out, chunk_hashes, chunk_ids=None, stream=None) -> None:
    """chunk_hashes = SHA-256(pt); out = ChaCha20 from LE32(chunk_id) (ids default to the hashes)."""
    r = b.records(out, b.offsets)
    _check(lib().enet_chunk_store_batch(C.byref(r), _ptr(chunk_ids), _ptr(chunk_hashes),
                                        _stream(stream)), "enet_chunk_store_batch")


def chunk_fetch(b: Batch, out, chunk_ids, chunk_hashes, ok, stream=None) -> None:
    """out = decrypt; ok = SHA-256(out) == chunk_hashes (zeroed on mismatch)."""
    r = b.records(out, b.offsets)
    _check(lib().enet_chunk_fetch_batch(C.byref(r), _ptr(chunk_ids), _ptr(chunk_hashes), _ptr(ok),
                                        _stream(stream)), "enet_chunk_fetch_batch")


def pow_search(prefixes, offsets, difficulty, schedule: int, max_attempts: int, nonces, found,
               attempts=None, stream=None) -> None:
    """First nonce (attempt order) with >= difficulty leading zero bits of
    SHA-256(prefix || BE64(nonce)); schedule POW_NODE or POW_STORE.  Device tensors: prefixes
    uint8 arena, offsets int64 [n+1], difficulty uint8 [n], nonces/attempts int64 [n], found
    uint8 [n]."""
    n = int(offsets.numel()) - 1
    _check(lib().enet_pow_search_batch(n, _ptr(prefixes), _ptr(offsets), _ptr(difficulty), schedule,
                                       max_attempts, _ptr(nonces), _ptr(attempts), _ptr(found),
                                       _stream(stream)), "enet_pow_search_batch")


def pow_check(prefixes, offsets, nonces, difficulty, ok, stream=None) -> None:
    n = int(offsets.numel()) - 1
    _check(lib().enet_pow_check_batch(n, _ptr(prefixes), _ptr(offsets), _ptr(nonces),
                                      _ptr(difficulty), _ptr(ok), _stream(stream)),
           "enet_pow_check_batch")


def session_keys(secrets, counters, ticks, out, stream=None) -> None:
    """KeyManager::derive_key for n sessions: out[i] = HMAC(secrets[i], BE64(counters[i]) ||
    BE64(ticks[i])).  secrets uint8 [n*32], counters/ticks int64 [n], out uint8 [n*32]."""
    n = int(counters.numel())
    _check(lib().enet_session_key_batch(n, _ptr(secrets), _ptr(counters), _ptr(ticks), _ptr(out),
                                        _stream(stream)), "enet_session_key_batch")


def chunk_counter(chunk_id: bytes) -> int:
    """LE32(chunk_id[0..3]) -- CryptoManager.cpp:8-13."""
    return int(lib().enet_chunk_counter(chunk_id))


def lanes_per_record(count: int, total_bytes: int = 0, max_len: int = 0) -> int:
    return int(lib().enet_lanes_per_record(count, total_bytes, max_len))


def set_lanes_per_record(lanes: int) -> None:
    """Force lanes per record (1/2/4/8/16); 0 restores the scheduler."""
    _check(lib().enet_set_lanes_per_record(lanes), "enet_set_lanes_per_record")


def set_staging(variant: int) -> None:
    """Uniform-batch staging variant: 1 register prefetch (default), 4 without line staging,
    5 lockstep run staging only, 0 per-lane path only, -1 restores the default (results are
    identical)."""
    _check(lib().enet_set_staging(variant), "enet_set_staging")


HOST_MODES = (0, 3, 4)  # 1 and 2 retired in round 5


def set_host_mode(mode: int) -> None:
    """Host-resident batches (enet_host_set_mode): 0 = zero-copy kernels on pinned host memory,
    3 = SDMA by direction with the kernels on their own streams, 4 = SDMA in, kernels writing host
    memory (no D2H copies), -1 = auto (mode 3; for output the device writes in place, the faster
    of 3 and 4 as the device's first large jobs measure it).  Default: ENET_HOST_MODE, else auto."""
    _check(lib().enet_host_set_mode(mode), "enet_host_set_mode")


def host_mode() -> int:
    """The fixed host mode, or -1 (auto)."""
    return int(lib().enet_host_mode())


def host_mode_auto(device: int = 0) -> dict:
    """The device's auto state: best GiB/s seen in mode 3 (splitk_gibs) and mode 4 (zcout_gibs),
    jobs sampled in each, and the decision (mode: 3 / 4, -1 while sampling)."""
    p = HostProbe()
    lib().enet_host_mode_auto(device, C.byref(p))
    return p.as_dict()


def host_mode_probe(device: int = 0) -> dict:
    """Decide up front (enet_host_mode_probe): 256 MiB of pinned AEAD seals per mode, best of
    three; the decision becomes the device's auto decision."""
    p = HostProbe()
    m = int(lib().enet_host_mode_probe(device, C.byref(p)))
    if m < 0:
        _check(m, "enet_host_mode_probe")
    return p.as_dict()


def host_mode_for(splitk_gibs: float, zcout_gibs: float) -> int:
    p = HostProbe(splitk_gibs, zcout_gibs, 0, 0, 0)
    return int(lib().enet_host_mode_for(C.byref(p)))


def host_plan(node_cpus: str, allowed_cpus: str, cpu_max: str = "", env_cpus: int = 0, engines: int = 1) -> dict:
    """enet_host_plan: budget / workers / spin / CPU list for synthetic topology facts."""
    p = HostPlan()
    _check(lib().enet_host_plan(node_cpus.encode(), allowed_cpus.encode(), cpu_max.encode(), env_cpus, engines,
                                C.byref(p)), "enet_host_plan")
    return {"budget": p.budget, "workers": p.workers, "spin": bool(p.spin), "ncpus": p.ncpus,
            "cpus": p.cpus.decode()}


def device_numa_node(device: int = 0) -> int:
    return int(lib().enet_device_numa_node(device))


def host_cpu_budget() -> int:
    return int(lib().enet_host_cpu_budget())


def host_pinned_bytes() -> int:
    return int(lib().enet_host_pinned_bytes())


def host_register(addr: int, nbytes: int) -> None:
    """enet_host_register: pin + device-map an existing host range (e.g. a buffer pool)."""
    _check(lib().enet_host_register(addr, nbytes), "enet_host_register")


def host_unregister(addr: int) -> None:
    _check(lib().enet_host_unregister(addr), "enet_host_unregister")


def set_duplex_split(mode: int) -> None:
    """Chunk / AEAD+HMAC duplex paths: 1 = split each record over cipher, schedule and rounds
    waves, 0 = one cipher + one hash lane, -1 = automatic (longest record >= 16 KiB in a uniform
    or caller-ordered batch)."""
    _check(lib().enet_set_duplex_split(mode), "enet_set_duplex_split")


def make_batch(items: Sequence[bytes], keys: Sequence[bytes], nonces: Sequence[bytes],
               device="cuda", key_stride: int = 32, base_offset: int = 0) -> Batch:
    """Pack host byte strings into a device Batch.  `base_offset` shifts every record start
    (e.g. 3 -> unaligned starts) by leaving a gap at the front of the arena."""
    import numpy as np
    import torch
    offs = [base_offset]
    for it in items:
        offs.append(offs[-1] + len(it))
    total = offs[-1]
    buf = np.zeros(max(total, 1), dtype=np.uint8)
    for i, it in enumerate(items):
        if it:
            buf[offs[i]:offs[i] + len(it)] = np.frombuffer(it, dtype=np.uint8)
    kb = b"".join(keys)
    nb = b"".join(nonces)
    return Batch(
        arena=torch.from_numpy(buf).to(device),
        offsets=torch.tensor(offs, dtype=torch.int64, device=device),
        keys=torch.frombuffer(bytearray(kb), dtype=torch.uint8).to(device),
        nonces=torch.frombuffer(bytearray(nb), dtype=torch.uint8).to(device),
        key_stride=key_stride,
        total_bytes_hint=total - base_offset,
        max_len_hint=max((len(i) for i in items), default=0),
    )


class Pipeline:
    """Host-resident batches (include/enet_crypto.h "host pipeline"): every tensor of the Batch
    and every output lives in HOST memory (pinned, e.g. tensor.pin_memory(), for asynchronous
    DMA); the library cuts the batch into chunks and overlaps H2D, kernels and D2H over several
    HIP streams.  Calls block until the outputs are in host memory."""
    _prefix = "enet_pipeline_"

    def __init__(self, device: int = 0, chunk_bytes: int = 0, streams: int = 0):
        self._p = lib().enet_pipeline_create(device, chunk_bytes, streams)
        if not self._p:
            raise EnetError("enet_pipeline_create failed: "
                            + lib().enet_last_error().decode(errors="replace"))

    def _fn(self, op: str):
        return getattr(lib(), self._prefix + op), self._prefix + op

    def close(self) -> None:
        if self._p:
            getattr(lib(), self._prefix + "destroy")(self._p)
            self._p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> dict:
        """enet_pipeline_stats (single pipelines): counters, NUMA placement, worker plan, mode."""
        st = HostStats()
        _check(lib().enet_pipeline_stats(self._p, C.byref(st)), "enet_pipeline_stats")
        return st.as_dict()

    def _run(self, op: str, b: Batch, out, *ptrs) -> None:
        r = b.records(out, b.offsets)
        fn, name = self._fn(op)
        _check(fn(self._p, C.byref(r), *[_ptr(p) for p in ptrs]), name)

    def chacha20_xor(self, b: Batch, out, counters=None) -> None:
        self._run("chacha20_xor", b, out, counters)

    def aead_seal(self, b: Batch, out, tags) -> None:
        self._run("aead_seal", b, out, tags)

    def aead_open(self, b: Batch, out, tags, ok) -> None:
        self._run("aead_open", b, out, tags, ok)

    def aead_hmac_seal(self, b: Batch, out, tags, macs) -> None:
        self._run("aead_hmac_seal", b, out, tags, macs)

    def aead_hmac_open(self, b: Batch, out, tags, macs, ok) -> None:
        self._run("aead_hmac_open", b, out, tags, macs, ok)

    def _run_out(self, op: str, b: Batch, out, out_offsets, *ptrs) -> None:
        r = b.records(out, out_offsets)
        fn, name = self._fn(op)
        _check(fn(self._p, C.byref(r), *[_ptr(p) for p in ptrs]), name)

    def wire_seal(self, b: Batch, frames, frame_offsets) -> None:
        """Wire frames nonce || BE32 || ChaCha20(m || HMAC(m)) of b's messages (frame_offsets:
        |m_i| + 48 each), host memory in and out."""
        self._run_out("wire_seal", b, frames, frame_offsets)

    def wire_open(self, b: Batch, out, out_offsets, ok) -> None:
        """b.arena holds wire frames; out gets the messages (out_offsets: |f_i| - 48 each)."""
        self._run_out("wire_open", b, out, out_offsets, ok)


class PipelineGroup(Pipeline):
    """Host-resident batches over several devices of one node (enet_pipeline_group_*): the batch
    is cut into contiguous record ranges balanced by input bytes, one pipeline and host thread
    per device, no collective.  devices=None: every visible device; a device may repeat."""
    _prefix = "enet_pipeline_group_"

    def __init__(self, devices=None, chunk_bytes: int = 0, streams: int = 0):
        devs = list(devices or [])
        arr = (C.c_int * max(len(devs), 1))(*devs)
        self._p = lib().enet_pipeline_group_create(arr if devs else None, len(devs), chunk_bytes,
                                                   streams)
        if not self._p:
            raise EnetError("enet_pipeline_group_create failed: "
                            + lib().enet_last_error().decode(errors="replace"))

    @property
    def size(self) -> int:
        return int(lib().enet_pipeline_group_size(self._p))
