/*
 * enet_crypto.h -- C ABI of the MI355X bulk crypto engine for EphemeralNet.
 *
 * The reference crypto (ShardianLabs/EphemeralNet src/crypto) is a set of static C++20 member
 * functions taking one record per call.  This ABI is the batched, device-side
 * form of exactly those operations: every entry point below names the reference interface it
 * replaces (file:line).  The C++ API in include/ephemeralnet/crypto/ keeps the reference
 * signatures and is implemented on top of these calls (libenet_crypto.so exports both).
 *
 * Conventions
 *   - All buffer pointers are DEVICE pointers (hipMalloc'd, or any device-accessible memory)
 *     unless a comment says otherwise.  `stream` is a hipStream_t (NULL = legacy default).
 *   - Calls are asynchronous on `stream`; nothing is synchronised inside them (safe to capture in
 *     a hipGraph).  The caller keeps ownership of every buffer.  The one allocation: batches
 *     holding records of >= 256 KiB (ENET_SEG_MIN; enet_set_seg_min) take the sequence-parallel
 *     path, whose small scratch (a header, one entry per long record, one byte per record, 32 B
 *     per 64 KiB tile) is stream-ordered memory from a library-private pool
 *     (hipMallocFromPoolAsync / hipFreeAsync on `stream`).
 *   - Records are described SoA: a byte arena plus uint64 offsets[n+1]; record i is
 *     arena[offsets[i] .. offsets[i+1]).  Input and output arenas have their own offsets so
 *     length-changing ops (frames: +32-byte MAC) and in-place ops (out == in) both work.
 *   - keys / nonces / counters / tags / ok arrays must be 4-byte aligned.  Arena offsets may
 *     be arbitrary; 16-byte-aligned record starts run fastest.
 *   - Return 0 on success, a negative ENET_E* code otherwise.  Nothing throws across the ABI.
 *   - Thread-safe: calls on different streams may run concurrently from any host thread.
 */
#ifndef ENET_CRYPTO_H
#define ENET_CRYPTO_H

#include <stddef.h>
#include <stdint.h>

#ifndef ENET_API
#define ENET_API __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define ENET_OK 0
#define ENET_EINVAL (-1)   /* bad argument (null pointer, misalignment, n too large) */
#define ENET_EHIP (-2)     /* a HIP runtime call or kernel launch failed */
#define ENET_ENODEV (-3)   /* no usable gfx950 device */
#define ENET_ENOMEM (-4)   /* allocation failed (host-side helpers only) */

/* A batch of independent records (SoA, device pointers). */
typedef struct enet_records {
    uint32_t count;             /* n records */
    const uint64_t* in_offsets; /* [n+1] byte offsets into `in` */
    const uint64_t* out_offsets;/* [n+1] byte offsets into `out` (may be == in_offsets) */
    const uint8_t* in;          /* input arena */
    uint8_t* out;               /* output arena (may be == in for in-place operation) */
    const uint8_t* keys;        /* [n][32] ChaCha20 keys, or [1][32] when key_stride == 0 */
    uint32_t key_stride;        /* 32 = per-record key (per-peer sessions), 0 = one shared key */
    const uint8_t* nonces;      /* [n][12] 96-bit nonces */
    const uint32_t* order;      /* optional [count] record indices to process, in this order
                                   (e.g. longest first, or one length class of a larger batch);
                                   NULL = 0..count-1.  Indices address offsets/keys/nonces/tags/ok
                                   of the full batch, so results stay position-indexed. */
    uint64_t total_bytes_hint;  /* host-known sum of input lengths, 0 = unknown (scheduling) */
    uint32_t max_len_hint;      /* host-known max record length, 0 = unknown (scheduling) */
    /* The hints only choose kernels and launch shapes.  total == count * max declares a uniform
       batch (record i at in_offsets[0] + i * max); every workgroup of the uniform paths checks
       its records' real offsets against that layout and takes the per-lane path over the real
       offsets on any mismatch, so wrong hints cost speed, never bytes
       (tests/test_gpu_parity.py::test_lying_hints_give_correct_bytes). */
} enet_records;

/* ---- ChaCha20 (reference: ChaCha20::apply, src/crypto/ChaCha20.cpp:98-121,
 *      include/ephemeralnet/crypto/ChaCha20.hpp:20-24)
 * out_i = in_i XOR keystream(key_i, nonce_i, counters[i], counters[i]+1, ...) with the
 * reference's uint32 counter wrap (ChaCha20.cpp:110).  counters == NULL means all zero
 * (SessionManager.cpp:374/822 frames); CryptoManager passes LE32(chunk_id)
 * (CryptoManager.cpp:8-13, see enet_chunk_counter). */
ENET_API int enet_chacha20_xor_batch(const enet_records* r, const uint32_t* counters, void* stream);

/* ---- RFC 8439 AEAD_CHACHA20_POLY1305 (promised by the reference README.md:49, not
 *      implemented there -- SURVEY.md 0.1).  Keystream = ChaCha20::apply(counter = 1), one-time
 *      Poly1305 key = block(counter = 0).  aad/aad_offsets may be NULL (no AAD).
 * seal: out_i = ciphertext, tags[i] = 16-byte tag.
 * open: out_i = plaintext, ok[i] = 1 if the tag verified, else 0 and out_i is zeroed. */
ENET_API int enet_aead_seal_batch(const enet_records* r, const uint8_t* aad, const uint64_t* aad_offsets,
                         uint8_t* tags, void* stream);
ENET_API int enet_aead_open_batch(const enet_records* r, const uint8_t* aad, const uint64_t* aad_offsets,
                         const uint8_t* tags, uint8_t* ok, void* stream);

/* ---- SHA-256 (reference: Sha256::digest, src/crypto/Sha256.cpp:128-132)
 * digests[i] = SHA-256(in[offsets[i]..offsets[i+1])).  Used for chunk ids / manifest hashes
 * (StoreProof.cpp:75-78, Node.cpp:1414, Node.cpp:1652). */
ENET_API int enet_sha256_batch(uint32_t n, const uint8_t* in, const uint64_t* offsets, uint8_t* digests,
                      void* stream);

/* ---- HMAC-SHA256 (reference: HmacSha256::compute / verify, src/crypto/HmacSha256.cpp:11-54)
 * Key of record i = keys[key_offsets[i] .. key_offsets[i+1]) (keys over 64 B are hashed first,
 * HmacSha256.cpp:15-17); key_offsets == NULL means fixed 32-byte keys at keys + 32*i, or one
 * shared 32-byte key when key_stride == 0.
 * compute: macs[i] = HMAC(key_i, msg_i).
 * verify : ok[i] = (HMAC(key_i, msg_i) == macs[i]) (constant-time OR-accumulate, :47-53). */
ENET_API int enet_hmac_sha256_batch(uint32_t n, const uint8_t* keys, const uint64_t* key_offsets,
                           uint32_t key_stride, const uint8_t* in, const uint64_t* offsets,
                           uint8_t* macs, void* stream);
ENET_API int enet_hmac_sha256_verify_batch(uint32_t n, const uint8_t* keys, const uint64_t* key_offsets,
                                  uint32_t key_stride, const uint8_t* in,
                                  const uint64_t* offsets, const uint8_t* macs, uint8_t* ok,
                                  void* stream);

/* ---- Session frame body (reference: protocol::encode_signed, src/protocol/Message.cpp:305-311
 *      followed by SessionManager::send, src/network/SessionManager.cpp:362-374; CLI twin
 *      send_protocol_message, src/main.cpp:1141-1147).
 * seal: out_i = ChaCha20_{key_i, nonce_i, ctr 0}(in_i || HMAC-SHA256_{key_i}(in_i)),
 *       |out_i| = |in_i| + 32 (out_offsets must say so).  Keys are the 32-byte session keys.
 * open (SessionManager.cpp:815-822 then Message.cpp:313-328): out_i = first |in_i|-32 bytes of
 *       the decryption (out_offsets must say |in_i|-32, or 0 when |in_i| < 32), macs[i] = the
 *       decrypted 32-byte MAC ([n][32] device buffer), ok[i] = MAC verified (records shorter
 *       than 32 bytes fail, Message.cpp:315); on failure out_i is zeroed.  The 16-byte wire
 *       header nonce || BE32(len) (SessionManager.cpp:376-387) is host framing. */
/* One pass over HBM for any lengths / alignment / order (duplex kernel).  A record whose output
 * length is not as stated is not processed: its output range is zeroed (and ok[i] = 0). */
ENET_API int enet_frame_seal_batch(const enet_records* r, void* stream);
ENET_API int enet_frame_open_batch(const enet_records* r, uint8_t* macs, uint8_t* ok, void* stream);

/* ---- Whole wire frames (the batched session-frame codec): the frame body
 *      above plus the 16-byte header, in one pass -- what SessionManager::send puts on the socket
 *      (src/network/SessionManager.cpp:362-387) and what receive_loop takes off it (:760-822).
 * seal: in_i = encoded message m_i, out_i = nonce_i(12) || BE32(|m_i|+32) || ChaCha20_{key_i,
 *       nonce_i, 0}(m_i || HMAC_{key_i}(m_i)); out_offsets must give |out_i| = |m_i| + 48.
 * open: in_i = a received frame; the nonce comes from the frame (r->nonces is ignored, may be
 *       NULL); out_i = m_i (out_offsets must give |in_i| - 48), macs/ok as frame_open.  ok[i] = 0
 *       also when the frame is shorter than 48 bytes or its length field differs from its body
 *       length; failed messages are zeroed. */
ENET_API int enet_wire_seal_batch(const enet_records* r, void* stream);
ENET_API int enet_wire_open_batch(const enet_records* r, uint8_t* macs, uint8_t* ok, void* stream);
/* Session-keyed frame batches (a relay's frames come from fewer sessions than
 * frames).  keys = the sessions' 32-byte keys as a table ([sessions][32], key_stride ignored),
 * session[i] = the session of frame i, mid = the table's HMAC midstates from
 * enet_hmac_midstates ([sessions][16] uint32).  Same bytes as enet_wire_seal_batch /
 * enet_wire_open_batch with keys[i] = table[session[i]]; every frame skips the two key-block
 * compressions of its HMAC (2 of 27 for a 1 500-byte message).  A session[i] >= sessions
 * (device-resident, so not checked on the host) never reads past the table and fails closed:
 * seal zeroes that frame's whole output slot (nothing is encrypted under another session's key),
 * open reports ok[i] = 0 and zeroes the message.  enet_hmac_midstates: for each of
 * n keys the SHA-256 states after (key || 0^32) ^ ipad and ^ opad (HmacSha256.cpp:11-39). */
ENET_API int enet_hmac_midstates(const uint8_t* keys, uint32_t n, uint32_t* mid, void* stream);
ENET_API int enet_wire_seal_batch_sessions(const enet_records* r, const uint32_t* session,
                                           uint32_t sessions, const uint32_t* mid, void* stream);
ENET_API int enet_wire_open_batch_sessions(const enet_records* r, const uint32_t* session,
                                           uint32_t sessions, const uint32_t* mid, uint8_t* macs,
                                           uint8_t* ok, void* stream);

/* ---- AEAD with a fused HMAC-SHA256 integrity tag ("AEAD plus fused
 *      HMAC-SHA256 tag and verify"): ONE pass over HBM per direction (duplex kernel: Poly1305
 *      in the cipher lanes, HMAC in the hash lanes on the same SIMDs).  in/out offsets
 *      equal-length; mixed lengths are balanced best with `order` = longest first.  The HMAC covers the plaintext under the record's 32-byte
 *      key, exactly what the reference signs before encrypting (encode_signed,
 *      src/protocol/Message.cpp:305-311, HmacSha256.cpp:11-39).
 * seal: out_i = ChaCha20-Poly1305 ciphertext, tags[i] = Poly1305 tag, macs[i] = HMAC_K(pt_i).
 * open: out_i = plaintext, ok[i] = Poly1305 tag verified AND HMAC verified (HmacSha256.cpp:41-54);
 *       on failure out_i is zeroed. */
ENET_API int enet_aead_hmac_seal_batch(const enet_records* r, uint8_t* tags, uint8_t* macs,
                                       void* stream);
ENET_API int enet_aead_hmac_open_batch(const enet_records* r, const uint8_t* tags,
                                       const uint8_t* macs, uint8_t* ok, void* stream);

/* ---- Chunk store / fetch pipeline (Node::store_chunk, src/core/Node.cpp:1414-1417,
 *      Node::fetch_chunk's decrypt + hash check, :1641-1655).  in/out offsets equal-length.
 * store: chunk_hashes[i] (device [n][32], 4-byte aligned) = SHA-256(in_i) -- the manifest
 *        chunk_hash, and derive_chunk_id (src/security/StoreProof.cpp:75-78);
 *        out_i = ChaCha20(key_i, nonce_i, LE32(chunk_id_i[0..3]), in_i) (encrypt_with_key,
 *        CryptoManager.cpp:38-46) where chunk_id_i = chunk_ids[i], or the fresh chunk_hashes[i]
 *        when chunk_ids == NULL (the daemon derives ids from content, ControlServer.cpp:1101).
 * fetch: out_i = ChaCha20(key_i, nonce_i, LE32(chunk_ids[i][0..3]), in_i); ok[i] =
 *        SHA-256(out_i) == chunk_hashes[i]; on mismatch out_i is zeroed (no plaintext).
 * With chunk_ids given: one pass over HBM (hash and cipher together) for any lengths;
 * content-derived ids need the digest first (two passes).  Long chunks (a stored file is one chunk
 * of up to 32 MiB, Config.hpp:62) hash on host threads while the device ciphers them across every
 * CU: see enet_set_host_hash_min -- such a call is synchronous. */
ENET_API int enet_chunk_store_batch(const enet_records* r, const uint8_t* chunk_ids,
                                    uint8_t* chunk_hashes, void* stream);
ENET_API int enet_chunk_fetch_batch(const enet_records* r, const uint8_t* chunk_ids,
                                    const uint8_t* chunk_hashes, uint8_t* ok, void* stream);

/* ---- proof of work
 * Every PoW in the reference hashes SHA-256(prefix || BE64(candidate)) and accepts the FIRST
 * candidate, in attempt order, whose digest has >= difficulty leading zero bits:
 *   ENET_POW_NODE  (0): compute_announce_pow / compute_handshake_pow (src/core/Node.cpp:212-230,
 *                       269-292): candidate(a) = start + a, start = first std::mt19937_64 output
 *                       seeded with BE64(SHA-256(prefix || BE64(0))[0..8]) (:200-209, :247-256);
 *   ENET_POW_STORE (1): security::compute_store_pow (src/security/StoreProof.cpp:124-146):
 *                       candidate(a) = a-th std::mt19937_64 output seeded with
 *                       LE64(SHA-256(prefix || BE64(0))[0..8]).
 * Prefix serialisations: StoreProof.cpp:39-52 (chunk_id || BE64 size || BE32 len || hint) and
 * Node.cpp:155-171 / 233-245 (BE64-length-prefixed fields); see crypto::batch::*_pow_prefix.
 * prefixes/prefix_offsets: arena + [n+1] offsets; difficulty: [n] bits (0 -> nonce 0, found;
 * callers clamp as the reference does, StoreProof.cpp:128-130).  Outputs: nonces [n],
 * attempts [n] (nullable: index of the nonce in attempt order, or max_attempts), found [n]. */
#define ENET_POW_NODE 0
#define ENET_POW_STORE 1
ENET_API int enet_pow_search_batch(uint32_t n, const uint8_t* prefixes,
                                   const uint64_t* prefix_offsets, const uint8_t* difficulty,
                                   int schedule, uint64_t max_attempts, uint64_t* nonces,
                                   uint64_t* attempts, uint8_t* found, void* stream);
/* store_pow_valid / announce_pow_valid / handshake_pow_valid (StoreProof.cpp:109-121,
 * Node.cpp:193-198, 247-255) without the clamp: ok[i] = lzb(SHA-256(prefix_i || BE64(nonces[i])))
 * >= difficulty[i] (difficulty 0 -> 1). */
ENET_API int enet_pow_check_batch(uint32_t n, const uint8_t* prefixes,
                                  const uint64_t* prefix_offsets, const uint64_t* nonces,
                                  const uint8_t* difficulty, uint8_t* ok, void* stream);

/* ---- session key derivation
 * network::KeyManager::derive_key (src/network/KeyManager.cpp:74-92) for n sessions:
 * keys_out[i] = HMAC-SHA256(secrets[i], BE64(counters[i]) || BE64(ticks[i])), ticks = the
 * rotation time in ns since the steady_clock epoch (register_session uses counter 0, :15-30). */
ENET_API int enet_session_key_batch(uint32_t n, const uint8_t* secrets, const uint64_t* counters,
                                    const int64_t* ticks, uint8_t* keys_out, void* stream);

/* ---- host-resident pipeline
 * The reference's crypto path starts and ends in host memory (socket / relay buffers,
 * SessionManager.cpp:362-387 and 815-822; chunk files, Node.cpp:1414-1417 and 1641-1655).  These
 * calls take an enet_records batch whose arenas, offsets, keys, nonces, counters, tags, MACs and
 * ok flags are all HOST pointers, cut it into chunks of about `chunk_bytes` on record boundaries
 * and run each chunk through one of `streams` slots (a HIP stream plus pinned, device-mapped
 * staging), chunks overlapped; inside a chunk of mixed lengths records are run longest first.
 * Arenas the device can address (enet_host_alloc, hipHostMalloc, registered memory) are worked
 * on in place; pageable arenas are gathered into / scattered out of the pinned staging by the
 * runtime's host worker threads (enet_host_stats).  See enet_host_set_mode for how the
 * kernels reach host memory.  `order` must be NULL.  Every call blocks until all outputs are in
 * host memory.  A pipeline owns its streams and staging (grown on demand) and serves one host
 * thread at a time. */
typedef struct enet_pipeline enet_pipeline;
/* device: HIP ordinal; chunk_bytes: 0 = 16 MiB (mixed-length batches with HMAC want larger
 * chunks: one lane hashes a whole record, so a chunk takes at least its longest record's
 * serial SHA-256 time); streams: 0 = 3 (max 16).  NULL on failure.  The defaults saturate
 * PCIe Gen5 on MI355X for uniform batches (~64 GB/s both directions together). */
ENET_API enet_pipeline* enet_pipeline_create(int device, uint64_t chunk_bytes, uint32_t streams);
ENET_API void enet_pipeline_destroy(enet_pipeline* pipe);
/* ChaCha20::apply per record (CryptoManager chunk mode with counters = LE32(chunk_id)) */
ENET_API int enet_pipeline_chacha20_xor(enet_pipeline* pipe, const enet_records* host_records,
                                        const uint32_t* counters);
/* RFC 8439 AEAD seal / open (no AAD): tags [n][16]; ok [n] (failed records come back zeroed) */
ENET_API int enet_pipeline_aead_seal(enet_pipeline* pipe, const enet_records* host_records,
                                     uint8_t* tags);
ENET_API int enet_pipeline_aead_open(enet_pipeline* pipe, const enet_records* host_records,
                                     const uint8_t* tags, uint8_t* ok);
/* AEAD + HMAC-SHA256(key, plaintext) (enet_aead_hmac_*_batch): macs [n][32] */
ENET_API int enet_pipeline_aead_hmac_seal(enet_pipeline* pipe, const enet_records* host_records,
                                          uint8_t* tags, uint8_t* macs);
ENET_API int enet_pipeline_aead_hmac_open(enet_pipeline* pipe, const enet_records* host_records,
                                          const uint8_t* tags, const uint8_t* macs, uint8_t* ok);
/* Whole wire frames (enet_wire_seal_batch / enet_wire_open_batch) from and to host memory:
 * seal out_offsets give |m_i| + 48, open out_offsets give max(0, |f_i| - 48); ok [n]. */
ENET_API int enet_pipeline_wire_seal(enet_pipeline* pipe, const enet_records* host_records);
ENET_API int enet_pipeline_wire_open(enet_pipeline* pipe, const enet_records* host_records, uint8_t* ok);
/* How host-resident batches reach the kernels (pipelines and crypto::batch::*), process-wide:
 * 0 = zero-copy -- the kernels read and write pinned host memory directly over PCIe;
 * 3 = SDMA with H2D on one stream, the kernels on their own stream(s) (two for hash-chain-bound
 * jobs) and D2H on another; 4 = SDMA for the H2D copies as 3, the kernels writing their outputs
 * straight into pinned host memory (no D2H copies).  Values 1 and 2 were retired (EINVAL).
 * Default: ENET_HOST_MODE=zc|splitk|zcout if set, else AUTO (-1): mode 3, except for jobs whose
 * output arena the device can write in place (caller-pinned: enet_host_alloc / registered) --
 * there the faster of 3 and 4 depends on the HIP runtime the process loaded (the system ROCm 7.2
 * runtime: 3, 39.7 vs 36.6 GiB/s per direction for C2; PyTorch's bundled runtime, loaded first in
 * a Python process: 4, 35.6 vs 29.5), so each device's first two such jobs of >= 64 MiB per mode
 * alternate 3 and 4 and the better rate is kept (mode 4 only when > 3 % faster).
 * enet_host_set_mode(-1) returns to auto and forgets the decisions; enet_host_mode() is the fixed
 * mode or -1.  Results are identical in every mode. */
#define ENET_HOST_MODE_AUTO (-1)
ENET_API int enet_host_set_mode(int mode);
ENET_API int enet_host_mode(void);
/* The auto state of a device: best job rate (GiB/s of input) seen in mode 3 and mode 4, jobs
 * sampled in each, and the decision (3 / 4, or -1 while sampling). */
typedef struct enet_host_probe {
    double splitk_gibs, zcout_gibs;
    int32_t samples_splitk, samples_zcout;
    int32_t mode;
} enet_host_probe;
/* Returns the device's decision (or -1) and fills *out (nullable). */
ENET_API int enet_host_mode_auto(int device, enet_host_probe* out);
/* Decides up front instead of from the first jobs: 256 MiB of 4 KiB AEAD seals from and to
 * pinned host memory (512 MiB pinned for the call, ~0.2 s), modes 3 and 4 alternating, best of
 * three each; the decision becomes the device's auto decision.  Returns 3 / 4 or ENET_EHIP /
 * ENET_ENOMEM. */
ENET_API int enet_host_mode_probe(int device, enet_host_probe* out);
/* The decision rule: 4 when zcout_gibs > 1.03 x splitk_gibs, else 3; -1 while either is 0. */
ENET_API int enet_host_mode_for(const enet_host_probe* rates);
/* Where a pipeline's host side runs (host_topo.hpp).  Pinned staging (and enet_host_alloc blocks)
 * go on the device's NUMA node: an anonymous mapping bound MPOL_PREFERRED to the node, faulted in
 * and hipHostRegister'ed (ENET_HOST_NUMA=auto (default) | hip (hipHostMalloc places it) | <node>).
 * Host worker threads run on that node's CPUs within the process's affinity mask; their number
 * comes from the CPU budget -- min(affinity mask, cgroup cpu.max quota), or ENET_HOST_CPUS --
 * shared by the engines alive in the process (at most 8 workers each), and they spin between task
 * sets only while every pool thread has a CPU of its own. */
typedef struct enet_host_stats {
    uint64_t jobs, chunks, records, in_bytes, out_bytes;
    uint64_t gathered_bytes, scattered_bytes;      /* copied by the host worker threads */
    uint64_t direct_in_chunks, direct_out_chunks;  /* chunks whose arena the device used in place */
    uint64_t pinned_bytes;                         /* staging the pipeline holds */
    int32_t device_node;   /* NUMA node of the device (-1 unknown) */
    int32_t target_node;   /* node the staging is placed on (-1: hipHostMalloc decides) */
    int32_t staging_node;  /* node its first staging page is on (-1 none yet / unknown) */
    uint32_t workers;      /* host worker threads (0 before the first gather / scatter) */
    uint32_t cpu_budget;   /* CPUs the plan had */
    int32_t spin;          /* workers spin between task sets */
    int32_t mode;          /* host mode of the last job */
} enet_host_stats;
ENET_API int enet_pipeline_stats(const enet_pipeline* pipe, enet_host_stats* out);
/* NUMA node of a device (from its PCI function; -1 unknown) */
ENET_API int enet_device_numa_node(int device);
/* the CPU budget of this process (affinity mask, cgroup quota, ENET_HOST_CPUS) */
ENET_API uint32_t enet_host_cpu_budget(void);
/* pinned host bytes held by the library (staging + enet_host_alloc) */
ENET_API uint64_t enet_host_pinned_bytes(void);
/* The thread plan for given facts (CPU-testable): node_cpulist / allowed_cpulist in sysfs list
 * form ("0-7,16"), cpu_max as cgroup v2 cpu.max ("1600000 100000", "max 100000"; NULL / "" =
 * unlimited), env_cpus as ENET_HOST_CPUS (0 = unset), engines sharing the budget. */
typedef struct enet_host_plan_t {
    uint32_t budget;    /* CPUs of the process */
    uint32_t workers;   /* worker threads per engine */
    int32_t spin;
    uint32_t ncpus;     /* CPUs the workers may run on */
    char cpus[256];     /* ... as a list (truncated if longer) */
} enet_host_plan_t;
ENET_API int enet_host_plan(const char* node_cpulist, const char* allowed_cpulist, const char* cpu_max,
                            uint32_t env_cpus, uint32_t engines, enet_host_plan_t* out);
/* ---- several devices of one node (no reference counterpart -- the reference
 *      runs src/crypto on one core per call): one pipeline, host thread and stream set per device,
 *      each call cuts the batch into contiguous record ranges balanced by input bytes and runs
 *      them concurrently, no collective.  devices == NULL or ndev == 0: every visible device (a
 *      device may be listed twice: two pipelines on it).  Same arguments and results as the
 *      single-device calls above; the first failing range's status is returned. */
typedef struct enet_pipeline_group enet_pipeline_group;
ENET_API enet_pipeline_group* enet_pipeline_group_create(const int* devices, uint32_t ndev,
                                                         uint64_t chunk_bytes, uint32_t streams);
ENET_API void enet_pipeline_group_destroy(enet_pipeline_group* group);
ENET_API uint32_t enet_pipeline_group_size(const enet_pipeline_group* group);
ENET_API int enet_pipeline_group_chacha20_xor(enet_pipeline_group* group,
                                              const enet_records* host_records,
                                              const uint32_t* counters);
ENET_API int enet_pipeline_group_aead_seal(enet_pipeline_group* group,
                                           const enet_records* host_records, uint8_t* tags);
ENET_API int enet_pipeline_group_aead_open(enet_pipeline_group* group,
                                           const enet_records* host_records, const uint8_t* tags,
                                           uint8_t* ok);
ENET_API int enet_pipeline_group_aead_hmac_seal(enet_pipeline_group* group,
                                                const enet_records* host_records, uint8_t* tags,
                                                uint8_t* macs);
ENET_API int enet_pipeline_group_aead_hmac_open(enet_pipeline_group* group,
                                                const enet_records* host_records,
                                                const uint8_t* tags, const uint8_t* macs,
                                                uint8_t* ok);
/* Pinned, device-mapped host memory for socket / relay buffer pools, on the NUMA node of the
 * calling thread's current device (see enet_pipeline_stats); NULL on failure. */
ENET_API void* enet_host_alloc(uint64_t bytes);
ENET_API void enet_host_free(void* p);
/* Register an existing host buffer pool (hipHostRegister, device-mapped) so pipelines work on it
 * in place; unregister before freeing it.  An arena is used in place only when it lies wholly in
 * ONE allocation or registered range -- otherwise it is gathered through the staging. */
ENET_API int enet_host_register(void* p, uint64_t bytes);
ENET_API int enet_host_unregister(void* p);

/* ---- helpers (host) */
/* LE32(chunk_id[0..3]) -- CryptoManager.cpp:8-13 derive_counter. */
ENET_API uint32_t enet_chunk_counter(const uint8_t chunk_id[32]);
/* Lanes the scheduler gives each record for a batch of this shape (for tests / tuning). */
ENET_API uint32_t enet_lanes_per_record(uint32_t count, uint64_t total_bytes, uint32_t max_len);
/* Force lanes per record (1, 2, 4, 8 or 16) for all later calls in this process; 0 restores the
 * scheduler.  Returns ENET_EINVAL for other values.  Tuning / test knob. */
ENET_API int enet_set_lanes_per_record(uint32_t lanes);
/* Sequence-parallel path (segments.hip) for enet_chacha20_xor_batch / enet_aead_seal_batch /
 * enet_aead_open_batch: a record of >= ENET_SEG_MIN bytes is cut into 64 KiB tiles spread over
 * every CU, the tiles' Poly1305 partials combined on the device (a lone 32 MiB record otherwise
 * gets 16 lanes).  Automatic (-1, default) when max_len_hint >= ENET_SEG_MIN, unless the batch is
 * uniform with count * 16 >= 131072 lanes (the record kernels fill the chip then); a value >= 0
 * sends every record of at least that many bytes to the tiles whatever the hints (0: every
 * record; INT64_MAX: never).  Results are identical; tuning / test knob. */
#define ENET_SEG_MIN (256u << 10)
ENET_API int enet_set_seg_min(int64_t bytes);
/* Chunk store / fetch: records of at least this many bytes (default ENET_HOST_HASH_MIN, and only
 * while the host threads' chains finish before one GPU lane's would: sum(long) < ~60 x CPU budget x
 * longest) have their SHA-256 computed on host threads (SHA-NI) while the device runs their
 * ChaCha20 on the tiles -- SHA-256 of one message is one serial chain (~34 MB/s on a GPU lane,
 * ~2.1 GB/s on a host core).  Taken only when the batch's max_len_hint is at least the threshold;
 * such a call synchronises the stream: it reads the offsets first and returns when the batch is
 * done.  -1 = auto; 0 .. INT64_MAX forces the threshold (INT64_MAX: never,
 * every chain on the GPU).  Results are identical; tuning / test knob. */
#define ENET_HOST_HASH_MIN (256u << 10)
ENET_API int enet_set_host_hash_min(int64_t bytes);
/* Chunk store / fetch batches that took the host-hash route in this process (tests / tuning). */
ENET_API uint64_t enet_host_hash_batches(void);
/* Batches that have taken the sequence-parallel path in this process (tests / tuning). */
ENET_API uint64_t enet_seg_batches(void);
/* Staging of uniform-length batches (all records the same length): 1 = register prefetch + LDS
 * transposition (default; records that are not 128-byte aligned and get one lane each are staged
 * as whole aligned 128-byte lines; the rest in lockstep 512-thread workgroups), 4 = 1 without the
 * line staging, 5 = lockstep run staging only, 0 = per-lane path only, -1 restores the default.
 * (3, the LDS-DMA variant, was retired: it is refused.)
 * Results are identical; tuning / test knob. */
ENET_API int enet_set_staging(int variant);
/* ---- scalar C++ drop-in routing (include/ephemeralnet/crypto/{ChaCha20,Sha256,HmacSha256,
 *      CryptoManager}.hpp, security/StoreProof.hpp, network/KeyManager.hpp)
 * The reference signatures take ONE record per call from many session threads
 * (SessionManager.cpp:332,703) and never throw.  A GPU round trip costs >= ~18 us,
 * and SHA-256 of one message is one serial chain, so the drop-in routes each call by size:
 *   ENET_SCALAR_AUTO (default)  SHA-256 / HMAC / single PoW checks, and ChaCha20 records below
 *                               the crossover, run on the calling thread's host engine (SHA-NI,
 *                               AVX-512 / AVX2; csrc/host_engine.cpp); ChaCha20 records at or
 *                               above it go to the MI355X, concurrent callers coalesced into one
 *                               launch through a pinned arena; PoW searches and
 *                               KeyManager::rotate_all_due run on the MI355X.  The default
 *                               crossover is UINT64_MAX (never): measured on the box, the host
 *                               engine's keystream (~10 GB/s per thread) is as fast as the memcpy
 *                               a pageable caller buffer needs to reach the device at all.
 *   ENET_SCALAR_DEVICE          every call that has a device kernel runs on the MI355X (round-2
 *                               behaviour; the streaming Sha256 class stays on the host).
 *   ENET_SCALAR_HOST            everything on the host engine.
 * crossover_bytes = 0 keeps the current value.  A failed device call of the
 * scalar API is finished on the host engine (bit-exact), counted in device_failures and reported
 * once on stderr -- or, after enet_scalar_set_on_device_error(1), abort()s.  No exception ever
 * leaves a reference signature except std::bad_alloc.  The batch entry points (this header's
 * *_batch / pipeline calls and C++ crypto::batch::*) never use the host engine. */
#define ENET_SCALAR_AUTO 0
#define ENET_SCALAR_DEVICE 1
#define ENET_SCALAR_HOST 2
ENET_API int enet_scalar_set_policy(int policy, uint64_t crossover_bytes);
ENET_API int enet_scalar_policy(void);
/* 0 = finish a failed device call on the host engine (default), 1 = abort() */
ENET_API int enet_scalar_set_on_device_error(int mode);
typedef struct enet_scalar_stats {
    uint64_t host_calls;         /* scalar calls served by the host engine */
    uint64_t device_calls;       /* scalar calls served by the MI355X */
    uint64_t device_failures;    /* device calls that failed and were finished on the host */
    uint64_t coalesced_launches; /* device launches of the ChaCha20::apply coalescer */
    uint64_t coalesced_records;  /* records they carried (>= launches: calls merged across threads) */
} enet_scalar_stats;
ENET_API void enet_scalar_get_stats(enet_scalar_stats* out);
ENET_API void enet_scalar_reset_stats(void);
/* Test hook: the next n device calls of the scalar API fail as if the device had. */
ENET_API void enet_scalar_inject_device_failures(uint32_t n);
/* The host engine's instruction sets on this CPU ("sha-ni+avx2", ..., "portable"). */
ENET_API const char* enet_host_isa(void);
/* The host engine itself, one record (host pointers): ChaCha20::apply, Sha256::digest,
 * HmacSha256::compute semantics.  For callers that want the scalar path without the C++ API. */
ENET_API void enet_host_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                                     const uint8_t* in, uint8_t* out, uint64_t n);
ENET_API void enet_host_sha256(const uint8_t* in, uint64_t n, uint8_t digest[32]);
ENET_API void enet_host_hmac_sha256(const uint8_t* key, uint64_t key_len, const uint8_t* in, uint64_t n,
                                    uint8_t mac[32]);
/* One session frame's body on the host engine (SessionManager::send, SessionManager.cpp:374-385):
 * out[0..n+32) = ChaCha20(key, nonce, counter 0) XOR (m || HMAC-SHA256(key, m)); the wire frame is
 * nonce || BE32(n + 32) || out.  On AMD CPUs with SHA-NI + AVX-512 the HMAC is stitched into the
 * keystream's rounds in one pass over m.  out may overlap m. */
ENET_API void enet_host_seal_body(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* m, uint64_t n,
                                  uint8_t* out);
/* The receiving side (SessionManager::receive_loop, SessionManager.cpp:815-822, then
 * decode_signed's MAC check, Message.cpp:313-328): m[0..bl-32) = the decrypted body; returns 1 when
 * the decrypted MAC verifies, else 0 with m zeroed (0 for bl < 32).  Stitched like seal (the hash
 * one keystream step behind).  m may overlap body. */
ENET_API int enet_host_open_body(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* body, uint64_t bl,
                                 uint8_t* m);
/* Tuning / test knob for the stitched pass of enet_host_seal_body / enet_host_open_body: -1 = on AMD
 * CPUs for bodies over 64 bytes (default), 0 = never, 1 = at every size whenever the CPU has
 * SHA-NI + AVX-512.  Results are identical.  Returns the previous mode. */
ENET_API int enet_host_set_seal_stitch(int mode);

/* Duplex paths with a hash beside the cipher (chunk store / fetch with ids, AEAD + HMAC): long
 * records run with each record's work split over a cipher, a SHA-256 schedule and a SHA-256
 * rounds wave (a ~1.4x shorter serial chain, duplex_split.hip).  -1 = automatic (when
 * max_len_hint >= 16 KiB and the batch is uniform or has an `order`, e.g. length-sorted; the
 * default), 0 = never, 1 = always.  Results are identical; tuning / test knob. */
ENET_API int enet_set_duplex_split(int mode);
/* Human-readable text of the last error on this host thread ("" if none). */
ENET_API const char* enet_last_error(void);
/* ABI version: (major << 16) | minor. */
ENET_API uint32_t enet_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ENET_CRYPTO_H */
