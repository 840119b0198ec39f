// StoreProof.hpp -- drop-in for the reference include/ephemeralnet/security/StoreProof.hpp:11-39
// (same names, argument meaning and results), with the SHA-256 work on the MI355X through the
// C ABI (enet_sha256_batch, enet_pow_search_batch, enet_pow_check_batch), plus batch forms.
#pragma once

#include <cstdint>
#include <optional>
#include <span>
#include <string>
#include <string_view>
#include <vector>

#include "ephemeralnet/crypto/CryptoTypes.hpp"
#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::security {

struct StoreWorkInput {
    ChunkId chunk_id{};
    std::uint64_t payload_size{0};
    std::string_view filename_hint{};
};

constexpr std::uint8_t kMaxStorePowDifficulty = 24;
constexpr std::uint64_t kDefaultStorePowMaxAttempts = 500'000;

// StoreProof.cpp:84-89: SHA-256 of the chunk bytes
ENET_CXX_API ChunkId derive_chunk_id(std::span<const std::uint8_t> data);

// StoreProof.cpp:91-107: the file name part of a path, at most 255 bytes; nullopt for "", ".", ".."
ENET_CXX_API std::optional<std::string> sanitize_filename_hint(std::string_view raw_path);

// StoreProof.cpp:109-121: difficulty 0 -> true; clamped to kMaxStorePowDifficulty
ENET_CXX_API bool store_pow_valid(const StoreWorkInput& input, std::uint64_t nonce,
                                  std::uint8_t difficulty_bits);

// StoreProof.cpp:123-146: the first of max_attempts successive std::mt19937_64 outputs (seeded
// with LE64(SHA-256 of the input with nonce 0)) that is valid; difficulty 0 -> 0;
// max_attempts 0 -> kDefaultStorePowMaxAttempts
ENET_CXX_API std::optional<std::uint64_t> compute_store_pow(
    const StoreWorkInput& input, std::uint8_t difficulty_bits,
    std::uint64_t max_attempts = kDefaultStorePowMaxAttempts);

// The hashed prefix: chunk_id || BE64(payload_size) || BE32(|hint|) || hint (StoreProof.cpp:39-52)
ENET_CXX_API std::vector<std::uint8_t> store_pow_prefix(const StoreWorkInput& input);

namespace batch {
// compute_store_pow for many inputs in one device pass (e.g. a client uploading many chunks)
ENET_CXX_API std::vector<std::optional<std::uint64_t>> compute_store_pow(
    std::span<const StoreWorkInput> inputs, std::uint8_t difficulty_bits,
    std::uint64_t max_attempts = kDefaultStorePowMaxAttempts);
// store_pow_valid for many (input, nonce) pairs (e.g. a node admitting many stores); 1 = valid
ENET_CXX_API std::vector<std::uint8_t> store_pow_valid(std::span<const StoreWorkInput> inputs,
                                                       std::span<const std::uint64_t> nonces,
                                                       std::uint8_t difficulty_bits);
}  // namespace batch

}  // namespace ephemeralnet::security
