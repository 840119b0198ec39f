// CryptoManager.hpp -- drop-in for the reference include/ephemeralnet/crypto/CryptoManager.hpp:12-44.
#pragma once

#include "ephemeralnet/crypto/CryptoTypes.hpp"
#include "ephemeralnet/crypto/ChaCha20.hpp"

#include <optional>
#include <random>
#include <span>

namespace ephemeralnet::crypto {

struct CipherText {
    ChunkData data;
    Nonce nonce;
    bool encrypted{true};
};

class ENET_CXX_API CryptoManager {
public:
    CryptoManager();
    explicit CryptoManager(Key key);

    // CryptoManager.cpp:38-47: random nonce (mt19937_64), start counter LE32(chunk_id[0..3])
    CipherText encrypt(const ChunkId& chunk_id, const ChunkData& plaintext);
    // CryptoManager.cpp:49-58: always returns a value
    std::optional<ChunkData> decrypt(const ChunkId& chunk_id,
                                     std::span<const std::uint8_t> ciphertext,
                                     const Nonce& nonce) const;

    static Key generate_key();
    static void random_bytes(std::span<std::uint8_t> buffer);
    static CipherText encrypt_with_key(const Key& key,
                                       const ChunkId& chunk_id,
                                       const ChunkData& plaintext);
    static std::optional<ChunkData> decrypt_with_key(const Key& key,
                                                     const ChunkId& chunk_id,
                                                     std::span<const std::uint8_t> ciphertext,
                                                     const Nonce& nonce);

    const Key& key() const noexcept { return key_; }

private:
    Key key_{};
    mutable std::mt19937_64 prng_;

    void fill_random(std::span<std::uint8_t> buffer) const;
};

}  // namespace ephemeralnet::crypto
