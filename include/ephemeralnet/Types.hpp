// Types.hpp -- the subset of the reference include/ephemeralnet/Types.hpp:10-12 the crypto API
// needs (ChunkId / PeerId / ChunkData aliases).  A reference build keeps its own Types.hpp; these
// aliases are identical so either header works.
#pragma once

#include <array>
#include <cstdint>
#include <vector>

namespace ephemeralnet {
using ChunkId = std::array<std::uint8_t, 32>;
using PeerId = std::array<std::uint8_t, 32>;
using ChunkData = std::vector<std::uint8_t>;
}  // namespace ephemeralnet
