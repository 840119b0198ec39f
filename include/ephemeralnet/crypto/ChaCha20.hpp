// ChaCha20.hpp -- drop-in for the reference include/ephemeralnet/crypto/ChaCha20.hpp:10-24.
// Same types and signature.  Records below the scalar crossover run on the host engine, larger
// ones on the MI355X, concurrent callers coalesced into one launch (enet_crypto.h "scalar").
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
    // `counter` (uint32, wraps mod 2^32).  Never throws (except std::bad_alloc), like the reference.
    static void apply(const Key& key,
                      const Nonce& nonce,
                      std::span<const std::uint8_t> input,
                      std::vector<std::uint8_t>& output,
                      std::uint32_t counter = 0);
};

}  // namespace ephemeralnet::crypto
