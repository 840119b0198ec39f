/*
 * enet_oracle.h -- CPU restatement of the EphemeralNet crypto hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ephemeralnet_amd/, the
 * C-ABI library, the C++ API) links, loads or calls this code.  It is imported
 * only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
 * always as the checker / CPU baseline, never as the thing measured.
 *
 * Parity is pinned against the JSON fixtures in tests/golden/, which were generated from the
 * reference src/crypto compiled in the survey container (oracle/_ref, see
 * oracle/Makefile) and, for Poly1305 / AEAD (absent from the reference), from
 * OpenSSL 3.0.2 plus the RFC 8439 vectors (tests/golden/gen_golden.py).
 *
 * Each function cites the reference file:line it restates.  Paths are relative
 * to the reference tree (ShardianLabs/EphemeralNet @ 2025-11-28).
 */
#ifndef ENET_ORACLE_H
#define ENET_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* splitmix64 byte generator shared by fixtures, tests and bench:
 * byte stream = concat_i LE64(mix(seed + (i+1) * 0x9E3779B97F4A7C15)). */
void orc_splitmix_bytes(uint64_t seed, uint8_t* out, size_t n);

/* src/crypto/ChaCha20.cpp:56-94 (chacha20_block) */
void orc_chacha20_block(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                        uint8_t out[64]);
/* src/crypto/ChaCha20.cpp:98-121 (ChaCha20::apply): byte-wise XOR, u32 counter wrap */
void orc_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                      const uint8_t* in, uint8_t* out, size_t n);

/* src/crypto/Sha256.cpp:66-176 (Sha256::digest) */
void orc_sha256(const uint8_t* data, size_t n, uint8_t out[32]);
/* src/crypto/HmacSha256.cpp:11-39 (HmacSha256::compute) */
void orc_hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* data, size_t n,
                     uint8_t out[32]);
/* src/crypto/HmacSha256.cpp:41-54 (HmacSha256::verify) */
int orc_hmac_sha256_verify(const uint8_t* key, size_t klen, const uint8_t* data, size_t n,
                           const uint8_t* mac, size_t maclen);

/* RFC 8439 section 2.5 Poly1305 (no reference implementation exists) */
void orc_poly1305(const uint8_t key[32], const uint8_t* msg, size_t n, uint8_t tag[16]);
/* RFC 8439 section 2.8 AEAD_CHACHA20_POLY1305 */
void orc_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                   size_t aad_len, const uint8_t* pt, size_t n, uint8_t* ct, uint8_t tag[16]);
int orc_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                  size_t aad_len, const uint8_t* ct, size_t n, const uint8_t tag[16],
                  uint8_t* pt);

/* src/crypto/CryptoManager.cpp:8-13 (derive_counter): LE32(chunk_id[0..3]) */
uint32_t orc_derive_counter(const uint8_t chunk_id[32]);

/* Session frame body, src/protocol/Message.cpp:305-311 + src/network/SessionManager.cpp:362-374:
 *   body = ChaCha20_{K,N,ctr=0}(m || HMAC-SHA256_K(m)),  |body| = n + 32.
 * The wire frame is nonce(12) || BE32(n+32) || body (SessionManager.cpp:376-387). */
void orc_frame_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* m, size_t n,
                    uint8_t* body);
/* Inverse: SessionManager.cpp:815-822 then Message.cpp:313-328.  body_len >= 32 or fails. */
int orc_frame_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* body,
                   size_t body_len, uint8_t* m_out);

/* ------------------------------------------------------------ proof of work
 * All three searches in the reference hash  SHA-256(prefix || BE64(candidate))  and accept the
 * first candidate, in attempt order, whose digest has >= difficulty leading zero bits.
 *   store     src/security/StoreProof.cpp:39-52 (pow_digest), :124-146 (compute_store_pow):
 *             seed = LE64(digest(nonce 0)[0..8]), candidates = successive std::mt19937_64(seed)
 *             outputs; difficulty clamped to 24; max_attempts 0 -> 500 000.
 *   announce  src/core/Node.cpp:155-171, 200-230;  handshake  Node.cpp:233-292:
 *             seed = BE64(digest(nonce 0)[0..8]), start = first std::mt19937_64(seed) output
 *             (uniform_int_distribution over the full u64 range returns it unchanged),
 *             candidates = start + attempt (mod 2^64), 500 000 attempts. */
typedef struct { uint64_t mt[312]; int mti; } orc_mt64;
void orc_mt64_seed(orc_mt64* g, uint64_t seed);           /* std::mt19937_64(seed) */
uint64_t orc_mt64_next(orc_mt64* g);                      /* operator() */
/* Node.cpp:174-190 == StoreProof.cpp:61-80 */
unsigned orc_leading_zero_bits(const uint8_t digest[32]);
void orc_pow_digest(const uint8_t* prefix, size_t plen, uint64_t nonce, uint8_t out[32]);
/* chunk_id(32) || BE64(payload_size) || BE32(|hint|) || hint  (StoreProof.cpp:25-52) */
size_t orc_store_pow_prefix(const uint8_t chunk_id[32], uint64_t payload_size, const uint8_t* hint,
                            size_t hint_len, uint8_t* out);
/* BE64(32)||chunk_id || BE64(32)||peer_id || BE64(|e|)||endpoint || BE64(|u|)||manifest_uri ||
 * BE64(|s|)||assigned_shards || BE64(ttl)   (Node.cpp:149-171) */
size_t orc_announce_pow_prefix(const uint8_t chunk_id[32], const uint8_t peer_id[32],
                               const uint8_t* endpoint, size_t elen, const uint8_t* uri,
                               size_t ulen, const uint8_t* shards, size_t slen, int64_t ttl,
                               uint8_t* out);
/* BE64(32)||initiator || BE64(32)||responder || BE64(initiator_public)  (Node.cpp:233-245) */
size_t orc_handshake_pow_prefix(const uint8_t initiator[32], const uint8_t responder[32],
                                uint32_t initiator_public, uint8_t* out);
/* schedule 0 = announce/handshake, 1 = store.  Returns 1 and the nonce (+ attempt index) when
 * found within max_attempts; difficulty 0 -> nonce 0.  No clamping here (callers clamp). */
int orc_pow_search(const uint8_t* prefix, size_t plen, unsigned difficulty, int schedule,
                   uint64_t max_attempts, uint64_t* nonce, uint64_t* attempt);
/* store_pow_valid / announce_pow_valid without the clamp: difficulty 0 -> 1 */
int orc_pow_check(const uint8_t* prefix, size_t plen, uint64_t nonce, unsigned difficulty);

/* ------------------------------------------------ session key derivation
 * KeyManager::derive_key (src/network/KeyManager.cpp:74-92) and register_session
 * (:15-30): HMAC-SHA256(shared_secret, BE64(counter) || BE64(ticks_ns)). */
void orc_session_key(const uint8_t secret[32], uint64_t counter, int64_t ticks, uint8_t out[32]);

/* CPU baseline: AEAD seal then open over n records of len bytes (record i uses key
 * keys+32*i, nonce nonces+12*i), split over `threads` std::threads-equivalent pthreads.
 * Returns seconds for seal (out[0]) and open (out[1]); returns number of failed opens. */
int orc_bench_aead(const uint8_t* pt, uint8_t* ct, uint8_t* back, const uint8_t* keys,
                   const uint8_t* nonces, uint8_t* tags, size_t n, size_t len, int threads,
                   double out_seconds[2]);

/* CPU baseline: orc_pow_search over `jobs` prefixes (arena + offsets) at `difficulty` with
 * schedule 0, `threads` pthreads; returns seconds, *hashes = candidates hashed. */
double orc_bench_pow(const uint8_t* prefixes, const uint64_t* offsets, size_t jobs,
                     unsigned difficulty, uint64_t max_attempts, int threads, uint64_t* hashes);

#ifdef __cplusplus
}
#endif
#endif
