// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A C-linkage veneer over the *reference* src/crypto and src/protocol/Message.cpp, compiled
// from the sources where they lie under /root/reference (see oracle/Makefile; output goes to
// oracle/_ref/, which is git-ignored).  It exists so tests/golden/gen_golden.py can generate
// golden vectors from the reference itself, and so the restatement in enet_oracle.c can be
// validated against it.  No reference source is copied into this repository.
#include "ephemeralnet/crypto/ChaCha20.hpp"
#include "ephemeralnet/crypto/CryptoManager.hpp"
#include "ephemeralnet/crypto/HmacSha256.hpp"
#include "ephemeralnet/crypto/Sha256.hpp"
#include "ephemeralnet/network/KeyManager.hpp"
#include "ephemeralnet/protocol/Message.hpp"
#include "ephemeralnet/security/StoreProof.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstring>
#include <limits>
#include <random>
#include <string_view>

using namespace ephemeralnet;

extern "C" {

// ChaCha20::apply (src/crypto/ChaCha20.cpp:98-121)
void ref_chacha20_apply(const uint8_t* key, const uint8_t* nonce, const uint8_t* in, size_t n,
                        uint8_t* out, uint32_t counter) {
    crypto::Key k{};
    crypto::Nonce nn{};
    std::memcpy(k.bytes.data(), key, 32);
    std::memcpy(nn.bytes.data(), nonce, 12);
    std::vector<uint8_t> o;
    crypto::ChaCha20::apply(k, nn, std::span<const uint8_t>(in, n), o, counter);
    if (n) std::memcpy(out, o.data(), n);
}

// Sha256::digest (src/crypto/Sha256.cpp:128-132)
void ref_sha256(const uint8_t* data, size_t n, uint8_t* out) {
    auto d = crypto::Sha256::digest(std::span<const uint8_t>(data, n));
    std::memcpy(out, d.data(), 32);
}

// Sha256 streaming update()/finalize() with a fixed piece size (Sha256.cpp:72-126)
void ref_sha256_pieces(const uint8_t* data, size_t n, size_t piece, uint8_t* out) {
    crypto::Sha256 h;
    for (size_t o = 0; o < n; o += piece) h.update(std::span<const uint8_t>(data + o, std::min(piece, n - o)));
    auto d = h.finalize();
    std::memcpy(out, d.data(), 32);
}

// HmacSha256::compute / verify (src/crypto/HmacSha256.cpp:11-54)
void ref_hmac(const uint8_t* key, size_t klen, const uint8_t* data, size_t n, uint8_t* out) {
    auto d = crypto::HmacSha256::compute(std::span<const uint8_t>(key, klen), std::span<const uint8_t>(data, n));
    std::memcpy(out, d.data(), 32);
}
int ref_hmac_verify(const uint8_t* key, size_t klen, const uint8_t* data, size_t n, const uint8_t* mac,
                    size_t maclen) {
    return crypto::HmacSha256::verify(std::span<const uint8_t>(key, klen), std::span<const uint8_t>(data, n),
                                      std::span<const uint8_t>(mac, maclen))
               ? 1
               : 0;
}

// CryptoManager::encrypt_with_key / decrypt_with_key (src/crypto/CryptoManager.cpp:77-90).
// The nonce is drawn by the reference's own mt19937_64; it is returned so callers can check.
void ref_cm_encrypt_with_key(const uint8_t* key, const uint8_t* chunk_id, const uint8_t* pt, size_t n,
                             uint8_t* ct, uint8_t* nonce_out) {
    crypto::Key k{};
    std::memcpy(k.bytes.data(), key, 32);
    ChunkId id{};
    std::memcpy(id.data(), chunk_id, 32);
    ChunkData p(pt, pt + n);
    auto c = crypto::CryptoManager::encrypt_with_key(k, id, p);
    if (n) std::memcpy(ct, c.data.data(), n);
    std::memcpy(nonce_out, c.nonce.bytes.data(), 12);
}
void ref_cm_decrypt_with_key(const uint8_t* key, const uint8_t* chunk_id, const uint8_t* ct, size_t n,
                             const uint8_t* nonce, uint8_t* pt) {
    crypto::Key k{};
    std::memcpy(k.bytes.data(), key, 32);
    ChunkId id{};
    std::memcpy(id.data(), chunk_id, 32);
    crypto::Nonce nn{};
    std::memcpy(nn.bytes.data(), nonce, 12);
    auto p = crypto::CryptoManager::decrypt_with_key(k, id, std::span<const uint8_t>(ct, n), nn);
    if (n) std::memcpy(pt, p->data(), n);
}

// protocol::encode_signed (src/protocol/Message.cpp:305-311) for a Request and a Chunk message.
size_t ref_encode_signed_request(const uint8_t* chunk_id, const uint8_t* requester, const uint8_t* key,
                                 size_t klen, uint8_t* out, size_t cap) {
    protocol::Message m{};
    m.type = protocol::MessageType::Request;
    protocol::RequestPayload p{};
    std::memcpy(p.chunk_id.data(), chunk_id, 32);
    std::memcpy(p.requester.data(), requester, 32);
    m.payload = p;
    auto v = protocol::encode_signed(m, std::span<const uint8_t>(key, klen));
    if (v.size() <= cap) std::memcpy(out, v.data(), v.size());
    return v.size();
}
size_t ref_encode_signed_chunk(const uint8_t* chunk_id, const uint8_t* data, size_t n, int64_t ttl,
                               const uint8_t* key, size_t klen, uint8_t* out, size_t cap) {
    protocol::Message m{};
    m.type = protocol::MessageType::Chunk;
    protocol::ChunkPayload p{};
    std::memcpy(p.chunk_id.data(), chunk_id, 32);
    p.data.assign(data, data + n);
    p.ttl = std::chrono::seconds(ttl);
    m.payload = p;
    auto v = protocol::encode_signed(m, std::span<const uint8_t>(key, klen));
    if (v.size() <= cap) std::memcpy(out, v.data(), v.size());
    return v.size();
}
// protocol::decode_signed (Message.cpp:313-328): 1 when it yields a message.
int ref_decode_signed_ok(const uint8_t* buf, size_t n, const uint8_t* key, size_t klen) {
    return protocol::decode_signed(std::span<const uint8_t>(buf, n), std::span<const uint8_t>(key, klen)).has_value()
               ? 1
               : 0;
}

// security::compute_store_pow / store_pow_valid / derive_chunk_id (src/security/StoreProof.cpp)
int ref_compute_store_pow(const uint8_t* chunk_id, uint64_t payload_size, const char* hint, size_t hlen,
                          uint8_t difficulty, uint64_t max_attempts, uint64_t* nonce) {
    security::StoreWorkInput in{};
    std::memcpy(in.chunk_id.data(), chunk_id, 32);
    in.payload_size = payload_size;
    in.filename_hint = std::string_view(hint, hlen);
    auto r = security::compute_store_pow(in, difficulty, max_attempts);
    if (!r) return 0;
    *nonce = *r;
    return 1;
}
int ref_store_pow_valid(const uint8_t* chunk_id, uint64_t payload_size, const char* hint, size_t hlen,
                        uint64_t nonce, uint8_t difficulty) {
    security::StoreWorkInput in{};
    std::memcpy(in.chunk_id.data(), chunk_id, 32);
    in.payload_size = payload_size;
    in.filename_hint = std::string_view(hint, hlen);
    return security::store_pow_valid(in, nonce, difficulty) ? 1 : 0;
}

// security::sanitize_filename_hint (StoreProof.cpp:91-107): length, or -1 for nullopt
long ref_sanitize_filename_hint(const char* p, size_t n, char* out, size_t cap) {
    auto r = security::sanitize_filename_hint(std::string_view(p, n));
    if (!r) return -1;
    if (r->size() <= cap) std::memcpy(out, r->data(), r->size());
    return (long)r->size();
}

// std::mt19937_64 and the full-range uniform_int_distribution draw Node.cpp:217-220 / 279-282 use
void ref_mt64(uint64_t seed, size_t n, uint64_t* out) {
    std::mt19937_64 g(seed);
    for (size_t i = 0; i < n; ++i) out[i] = g();
}
uint64_t ref_mt64_uniform_first(uint64_t seed) {
    std::mt19937_64 g(seed);
    std::uniform_int_distribution<std::uint64_t> d(0, std::numeric_limits<std::uint64_t>::max());
    return d(g);
}

// Sha256 over arbitrary pieces (used to restate Node.cpp's anonymous-namespace PoW digests with
// the reference hasher: update_length_prefixed = BE64(len) || data, Node.cpp:149-153)
void ref_sha256_concat(const uint8_t* const* pieces, const size_t* lens, size_t count, uint8_t* out) {
    crypto::Sha256 h;
    for (size_t i = 0; i < count; ++i)
        if (lens[i]) h.update(std::span<const uint8_t>(pieces[i], lens[i]));
    auto d = h.finalize();
    std::memcpy(out, d.data(), 32);
}

// network::KeyManager (src/network/KeyManager.cpp:33-46): current_key after
// register_session_with_material = HMAC(shared_secret, material)
void ref_keymanager_material_key(const uint8_t* secret, const uint8_t* material, size_t mlen, uint8_t* out) {
    network::KeyManager km;
    PeerId peer{};
    peer[0] = 1;
    crypto::Key k{};
    std::memcpy(k.bytes.data(), secret, 32);
    km.register_session_with_material(peer, k, std::span<const uint8_t>(material, mlen),
                                      std::chrono::steady_clock::time_point{});
    auto key = km.current_key(peer);
    std::memcpy(out, key->data(), 32);
}
// KeyManager::rotate_if_needed (:56-72) after one interval: derive_key(secret, 1, now) (:74-92).
// Returns the ticks (ns since the steady_clock epoch) the reference used.
int64_t ref_keymanager_rotate(const uint8_t* secret, int64_t now_ns, uint8_t* out) {
    network::KeyManager km(std::chrono::seconds(1));
    PeerId peer{};
    peer[0] = 2;
    crypto::Key k{};
    std::memcpy(k.bytes.data(), secret, 32);
    uint8_t material[16] = {};
    km.register_session_with_material(peer, k, std::span<const uint8_t>(material, 16),
                                      std::chrono::steady_clock::time_point{});
    const auto now = std::chrono::steady_clock::time_point{} + std::chrono::nanoseconds(now_ns);
    auto key = km.rotate_if_needed(peer, now);
    if (!key) return -1;
    std::memcpy(out, key->data(), 32);
    return now_ns;
}

// CPU baseline with the reference itself (bench.py): the reference's frame construction over n
// records of len bytes -- seal = HmacSha256::compute(key, m) + ChaCha20::apply(key, nonce, m || mac)
// (Message.cpp:305-311 + SessionManager.cpp:362-374), open = apply + HmacSha256::verify
// (SessionManager.cpp:815-822 + Message.cpp:313-328) -- on `threads` std::threads.  Seconds of
// seal and open in secs[0..1]; returns the number of failed opens.
int ref_bench_frames(const uint8_t* pt, const uint8_t* keys, const uint8_t* nonces, size_t n, size_t len,
                     int threads, double* secs) {
    if (threads < 1) threads = 1;
    std::vector<std::vector<uint8_t>> bodies(n);
    std::atomic<int> fails{0};
    for (int phase = 0; phase < 2; ++phase) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) {
            th.emplace_back([&, t] {
                for (size_t i = n * t / threads; i < n * (t + 1) / threads; ++i) {
                    crypto::Key k{};
                    crypto::Nonce nn{};
                    std::memcpy(k.bytes.data(), keys + 32 * i, 32);
                    std::memcpy(nn.bytes.data(), nonces + 12 * i, 12);
                    const std::span<const uint8_t> key(k.bytes);
                    if (phase == 0) {
                        std::vector<uint8_t> signed_msg(pt + len * i, pt + len * (i + 1));
                        const auto mac = crypto::HmacSha256::compute(key, signed_msg);
                        signed_msg.insert(signed_msg.end(), mac.begin(), mac.end());
                        crypto::ChaCha20::apply(k, nn, signed_msg, bodies[i], 0);
                    } else {
                        std::vector<uint8_t> plain;
                        crypto::ChaCha20::apply(k, nn, bodies[i], plain, 0);
                        const std::span<const uint8_t> all(plain);
                        if (!crypto::HmacSha256::verify(key, all.first(len), all.subspan(len))) ++fails;
                    }
                }
            });
        }
        for (auto& x : th) x.join();
        secs[phase] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return fails.load();
}

// security::compute_store_pow on `threads` std::threads over n inputs (chunk ids [n][32], payload
// size, no hint) at `difficulty` with max_attempts each; returns seconds, *found = jobs that found.
double ref_bench_store_pow(const uint8_t* chunk_ids, size_t n, uint64_t payload_size, uint8_t difficulty,
                           uint64_t max_attempts, int threads, uint64_t* found) {
    if (threads < 1) threads = 1;
    std::atomic<uint64_t> f{0};
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        th.emplace_back([&, t] {
            for (size_t i = n * t / threads; i < n * (t + 1) / threads; ++i) {
                security::StoreWorkInput in{};
                std::memcpy(in.chunk_id.data(), chunk_ids + 32 * i, 32);
                in.payload_size = payload_size;
                if (security::compute_store_pow(in, difficulty, max_attempts)) ++f;
            }
        });
    }
    for (auto& x : th) x.join();
    *found = f.load();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // extern "C"
