// Sha256.hpp -- drop-in for the reference include/ephemeralnet/crypto/Sha256.hpp:10-26.
// Public interface identical; update() buffers on the host and finalize()/digest() hash on the
// MI355X (libenet_crypto.so).  Private members differ from the reference (API, not ABI, drop-in:
// the reference links ephemeralnet_core statically, CMakeLists.txt:38-67).
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <span>
#include <vector>

#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::crypto {

class ENET_CXX_API Sha256 {
public:
    Sha256();

    void update(std::span<const std::uint8_t> data);
    std::array<std::uint8_t, 32> finalize();

    static std::array<std::uint8_t, 32> digest(std::span<const std::uint8_t> data);

private:
    std::vector<std::uint8_t> pending_;
};

}  // namespace ephemeralnet::crypto
