// KeyManager.hpp -- drop-in for the reference include/ephemeralnet/network/KeyManager.hpp:15-47
// (same public interface and results).  Key derivation (HMAC-SHA256 of the shared secret over
// BE64(counter) || BE64(ticks), KeyManager.cpp:74-92) runs on the MI355X through the C ABI
// (enet_session_key_batch); rotate_all_due() rotates every due session in one device pass.
#pragma once

#include <array>
#include <chrono>
#include <cstdint>
#include <map>
#include <optional>
#include <span>
#include <utility>
#include <vector>

#include "ephemeralnet/crypto/CryptoTypes.hpp"
#include "ephemeralnet/crypto/CryptoManager.hpp"

namespace ephemeralnet::network {

struct SessionKeyContext {
    crypto::Key shared_secret{};
    std::array<std::uint8_t, 32> current_key{};
    std::uint64_t counter{0};
    std::chrono::steady_clock::time_point last_rotation{};
};

class ENET_CXX_API KeyManager {
public:
    explicit KeyManager(std::chrono::seconds rotation_interval = std::chrono::minutes(15));

    void register_session(const PeerId& peer_id, const crypto::Key& shared_secret);
    void register_session_with_material(const PeerId& peer_id,
                                        const crypto::Key& shared_secret,
                                        std::span<const std::uint8_t> material,
                                        std::chrono::steady_clock::time_point reference_time);
    std::optional<std::array<std::uint8_t, 32>> current_key(const PeerId& peer_id) const;
    std::optional<std::array<std::uint8_t, 32>> rotate_if_needed(
        const PeerId& peer_id,
        std::chrono::steady_clock::time_point now = std::chrono::steady_clock::now());
    std::vector<PeerId> known_peers() const;

    // Batch form of rotate_if_needed over every registered session: each session whose interval
    // has elapsed gets counter + 1 and a key derived at `now` (one device launch for all of them).
    // Returns the rotated (peer, new key) pairs in peer order.
    std::vector<std::pair<PeerId, std::array<std::uint8_t, 32>>> rotate_all_due(
        std::chrono::steady_clock::time_point now = std::chrono::steady_clock::now());

private:
    std::chrono::seconds rotation_interval_;
    std::map<PeerId, SessionKeyContext> contexts_;
};

}  // namespace ephemeralnet::network
