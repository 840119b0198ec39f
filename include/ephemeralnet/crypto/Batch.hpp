// Batch.hpp -- crypto::batch: the many-records-per-call form of the reference API, for callers
// that collect work across sessions / chunks (batched session-frame codec, store
// pipeline).  Host vectors in, host vectors out; one H2D, one kernel sequence and one D2H per
// call.  Device-resident callers use the C ABI (enet_crypto.h) directly.
#pragma once

#include <array>
#include <cstdint>
#include <span>
#include <vector>

#include "ephemeralnet/Types.hpp"
#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::crypto::batch {

struct Sealed {
    std::vector<std::uint8_t> data;
    std::array<std::uint8_t, 16> tag{};
};

// ChaCha20::apply for many records (counters[i] = start counter; empty span = all 0).
ENET_CXX_API std::vector<std::vector<std::uint8_t>> chacha20_apply(
    std::span<const Key> keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> inputs, std::span<const std::uint32_t> counters);

// RFC 8439 ChaCha20-Poly1305 (no AAD) for many records.
ENET_CXX_API std::vector<Sealed> aead_seal(std::span<const Key> keys,
                                           std::span<const Nonce> nonces,
                                           std::span<const std::span<const std::uint8_t>> plaintexts);
// Returns one entry per record; an empty optional-like flag vector `ok` says which verified.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> aead_open(
    std::span<const Key> keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> ciphertexts,
    std::span<const std::array<std::uint8_t, 16>> tags, std::vector<std::uint8_t>& ok);

// SHA-256 digests of many messages (Sha256::digest).
ENET_CXX_API std::vector<std::array<std::uint8_t, 32>> sha256(
    std::span<const std::span<const std::uint8_t>> messages);

// Session frame bodies: ChaCha20_{K,N,0}(m || HMAC_K(m)) (Message.cpp:305-311 +
// SessionManager.cpp:362-374) and the inverse with MAC verification.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> frame_seal(
    std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> messages);
ENET_CXX_API std::vector<std::vector<std::uint8_t>> frame_open(
    std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> bodies, std::vector<std::uint8_t>& ok);

}  // namespace ephemeralnet::crypto::batch
