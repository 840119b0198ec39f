// ChaCha20.hpp -- drop-in for the reference include/ephemeralnet/crypto/ChaCha20.hpp:10-24.
// Same types and signature; the keystream runs on the MI355X (libenet_crypto.so).
#pragma once

#include <array>
#include <cstdint>
#include <span>
#include <vector>

#define ENET_CXX_API __attribute__((visibility("default")))

namespace ephemeralnet::crypto {

struct Key {
    std::array<std::uint8_t, 32> bytes{};
};

struct Nonce {
    std::array<std::uint8_t, 12> bytes{};
};

class ENET_CXX_API ChaCha20 {
public:
    // ChaCha20.cpp:98-121: output.resize(input.size()); output = input XOR keystream starting at
    // `counter` (uint32, wraps mod 2^32).  Throws std::runtime_error if the GPU path fails.
    static void apply(const Key& key,
                      const Nonce& nonce,
                      std::span<const std::uint8_t> input,
                      std::vector<std::uint8_t>& output,
                      std::uint32_t counter = 0);
};

}  // namespace ephemeralnet::crypto
