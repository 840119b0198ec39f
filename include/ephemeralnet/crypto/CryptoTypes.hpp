// CryptoTypes.hpp -- the three aliases of the reference include/ephemeralnet/Types.hpp:11-13 the
// crypto API needs (ChunkId / PeerId / ChunkData).  Deliberately NOT named Types.hpp: a reference
// build puts this include/ first and must keep seeing its own Types.hpp (which also declares
// chunk_id_to_string & co.); an alias-declaration may be repeated for the identical type, so both
// headers coexist in one TU (tests/test_dropin_link.py compiles the reference callers that way).
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace ephemeralnet {
using ChunkId = std::array<std::uint8_t, 32>;
using PeerId = std::array<std::uint8_t, 32>;
using ChunkData = std::vector<std::uint8_t>;
}  // namespace ephemeralnet
