// Sha256.hpp -- drop-in for the reference include/ephemeralnet/crypto/Sha256.hpp:10-26.
// Public interface AND private layout identical to the reference (a 64-byte buffer and the
// running state: update() streams, memory stays O(1) for any message).  The compression runs on
// the calling thread's host engine (SHA-NI when available): SHA-256 of one message is a serial
// chain, which one GPU lane runs ~16x slower than a core.  Bulk hashing of many
// messages is crypto::batch::sha256 / enet_sha256_batch on the MI355X.
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <span>

#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::crypto {

class ENET_CXX_API Sha256 {
public:
    Sha256();

    void update(std::span<const std::uint8_t> data);
    std::array<std::uint8_t, 32> finalize();

    static std::array<std::uint8_t, 32> digest(std::span<const std::uint8_t> data);

private:
    void transform(const std::uint8_t block[64]);

    std::array<std::uint32_t, 8> state_{};
    std::array<std::uint8_t, 64> buffer_{};
    std::size_t buffer_size_{0};
    std::uint64_t bit_len_{0};
};

}  // namespace ephemeralnet::crypto
