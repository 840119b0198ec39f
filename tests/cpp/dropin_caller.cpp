// dropin_caller.cpp -- TEST DRIVER for the drop-in boundary.
//
// Linked with the reference's OWN caller translation units, compiled where they lie under
// /root/reference with this repo's include/ first (oracle/Makefile target `dropin`):
// protocol/Message.cpp (encode_signed / decode_signed, Message.cpp:305-328 -> HmacSha256),
// network/KeyExchange.cpp (derive_shared_secret, KeyExchange.cpp:34-47 -> Sha256),
// network/SessionManager.cpp (ChaCha20::apply at :374/:617/:686/:822), bootstrap/TokenChallenge.cpp,
// protocol/Manifest.cpp, crypto/Shamir.cpp, core/Types.cpp -- and against libenet_crypto.so for
// every crypto symbol.  So the reference's code runs unmodified on top of the GPU library.
//
// stdin, one op per line; stdout, one line per op:
//   signed <key_hex> <data_hex|-> <ttl>   -> <encode hex> <encode_signed hex> <decode_signed ok>
//                                           <tampered rejected> <decoded data == data>
//   kex <priv_a> <priv_b>                 -> <key hex of a's view> <a's view == b's view>
#include "ephemeralnet/crypto/HmacSha256.hpp"
#include "ephemeralnet/network/KeyExchange.hpp"
#include "ephemeralnet/protocol/Message.hpp"

#include <cstdint>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace {

std::vector<std::uint8_t> unhex(const std::string& s) {
    std::vector<std::uint8_t> v;
    if (s == "-") return v;
    for (std::size_t i = 0; i + 1 < s.size(); i += 2) v.push_back(std::stoi(s.substr(i, 2), nullptr, 16));
    return v;
}

template <class C>
std::string hex(const C& c) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (std::uint8_t b : c) { s += d[b >> 4]; s += d[b & 15]; }
    return s.empty() ? "-" : s;
}

}  // namespace

int main() {
    using namespace ephemeralnet;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string op;
        in >> op;
        if (op == "signed") {
            std::string k, d;
            long ttl = 0;
            in >> k >> d >> ttl;
            const auto key = unhex(k);
            protocol::ChunkPayload p;
            p.data = unhex(d);
            for (std::size_t i = 0; i < p.chunk_id.size(); ++i) p.chunk_id[i] = static_cast<std::uint8_t>(i * 7 + 1);
            p.ttl = std::chrono::seconds(ttl);
            protocol::Message m;
            m.type = protocol::MessageType::Chunk;
            m.payload = p;
            const auto body = protocol::encode(m);
            auto sig = protocol::encode_signed(m, key);
            const auto back = protocol::decode_signed(sig, key);
            bool same = back && std::get<protocol::ChunkPayload>(back->payload).data == p.data;
            auto bad = sig;
            bad[bad.size() / 2] ^= 0x01;
            const bool rejected = !protocol::decode_signed(bad, key).has_value();
            std::cout << hex(body) << ' ' << hex(sig) << ' ' << int(back.has_value()) << ' '
                      << int(rejected) << ' ' << int(same) << '\n';
        } else if (op == "kex") {
            std::uint32_t a = 0, b = 0;
            in >> a >> b;
            using network::KeyExchange;
            const auto ka = KeyExchange::derive_shared_secret(a, KeyExchange::compute_public(b));
            const auto kb = KeyExchange::derive_shared_secret(b, KeyExchange::compute_public(a));
            std::cout << hex(ka.bytes) << ' ' << int(ka.bytes == kb.bytes) << '\n';
        } else {
            std::cout << "?\n";
        }
    }
    return 0;
}
