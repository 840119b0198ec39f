// HmacSha256.hpp -- drop-in for the reference include/ephemeralnet/crypto/HmacSha256.hpp:9-20.
#pragma once

#include <array>
#include <cstdint>
#include <span>

#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::crypto {

class ENET_CXX_API HmacSha256 {
public:
    static constexpr std::size_t kBlockSize = 64;
    static constexpr std::size_t kDigestSize = 32;

    // HmacSha256.cpp:11-39 (keys over 64 bytes are hashed first)
    static std::array<std::uint8_t, kDigestSize> compute(std::span<const std::uint8_t> key,
                                                         std::span<const std::uint8_t> data);

    // HmacSha256.cpp:41-54 (false when mac.size() != 32)
    static bool verify(std::span<const std::uint8_t> key,
                       std::span<const std::uint8_t> data,
                       std::span<const std::uint8_t> mac);
};

}  // namespace ephemeralnet::crypto
