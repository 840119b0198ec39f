// crypto_api.cpp -- the reference C++ API (namespace ephemeralnet::crypto) implemented on the
// MI355X through the C ABI.  Every call ships its record(s) to the device, runs the batch
// kernels and copies the result back; there is no CPU crypto path in the product (a failing
// GPU path throws std::runtime_error instead of silently computing on the host).
//
// Reference: src/crypto/{ChaCha20,Sha256,HmacSha256,CryptoManager}.cpp, src/security/StoreProof.cpp,
// src/network/KeyManager.cpp and the PoW searches of src/core/Node.cpp (ShardianLabs/EphemeralNet).
#include "ephemeralnet/crypto/Batch.hpp"
#include "ephemeralnet/crypto/ChaCha20.hpp"
#include "ephemeralnet/crypto/CryptoManager.hpp"
#include "ephemeralnet/crypto/HmacSha256.hpp"
#include "ephemeralnet/crypto/Sha256.hpp"
#include "ephemeralnet/network/KeyManager.hpp"
#include "ephemeralnet/security/StoreProof.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <filesystem>
#include <limits>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "enet_crypto.h"

namespace {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("enet: ") + what + ": " + hipGetErrorString(e));
}

void enet_check(int rc, const char* what) {
    if (rc != ENET_OK) throw std::runtime_error(std::string("enet: ") + what + ": " + enet_last_error());
}

// Staging buffers + one stream per host thread: the reference functions are reentrant and
// called from many session threads (SessionManager.cpp:332,703).  A scalar call is a GPU round
// trip, so its fixed cost is what matters: buffers of up to kZeroCopyMax bytes
// come from one pinned, device-mapped, coherent host blob -- "uploading" is a host memcpy into
// it, the kernel reads its operands over PCIe and writes its results straight back, and
// "downloading" is a memcpy after the stream sync -- so a small call costs one launch and one
// sync instead of up to six pageable copies.  Larger buffers keep grow-only device slots and
// async copies.  The blob is bump-allocated and rewound at every sync (every API call ends
// with one), so no region is rewritten while a kernel of the same call may still read it.
struct Staging {
    static constexpr int kSlots = 10;
    static constexpr size_t kHostBlob = 8u << 20;
    static constexpr size_t kZeroCopyMax = 8u << 10;  // a serial SHA lane pays PCIe latency per block
    void* dev[kSlots] = {};
    size_t cap[kSlots] = {};
    hipStream_t stream = nullptr;
    uint8_t* host = nullptr;
    bool host_failed = false;
    size_t used = 0;
    struct Pending {
        void* dst;
        const void* src;
        size_t n;
    };
    std::vector<Pending> pend;

    ~Staging() {
        for (int i = 0; i < kSlots; ++i)
            if (dev[i]) (void)hipFree(dev[i]);
        if (host) (void)hipHostFree(host);
        if (stream) (void)hipStreamDestroy(stream);
    }
    bool in_host(const void* p) const {
        return host && p >= host && static_cast<const uint8_t*>(p) < host + kHostBlob;
    }
    void* get(int slot, size_t bytes) {
        bytes = std::max<size_t>(bytes, 64);
        if (bytes <= kZeroCopyMax && !host_failed) {
            if (!host && hipHostMalloc(reinterpret_cast<void**>(&host), kHostBlob,
                                       hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
                host = nullptr;
                host_failed = true;
            }
            const size_t off = (used + 255) & ~size_t(255);
            if (host && off + bytes <= kHostBlob) {
                used = off + bytes;
                return host + off;
            }
        }
        if (cap[slot] < bytes) {
            if (dev[slot]) hip_check(hipFree(dev[slot]), "hipFree");
            size_t c = std::max(bytes, cap[slot] * 2);
            hip_check(hipMalloc(&dev[slot], c), "hipMalloc");
            cap[slot] = c;
        }
        return dev[slot];
    }
    hipStream_t s() {
        if (!stream) hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
        return stream;
    }
    void h2d(void* d, const void* h, size_t n) {
        if (!n) return;
        if (in_host(d)) std::memcpy(d, h, n);
        else hip_check(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s()), "H2D");
    }
    void d2h(void* h, const void* d, size_t n) {
        if (!n) return;
        if (in_host(d)) pend.push_back({h, d, n});
        else hip_check(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s()), "D2H");
    }
    void sync() {
        hip_check(hipStreamSynchronize(s()), "hipStreamSynchronize");
        for (const Pending& q : pend) std::memcpy(q.dst, q.src, q.n);
        pend.clear();
        used = 0;
    }
};

Staging& staging() {
    thread_local Staging st;
    return st;
}

enum Slot { S_IN = 0, S_OUT, S_INOFF, S_OUTOFF, S_KEYS, S_NONCES, S_CTR, S_TAGS, S_OK, S_AUX };

// Host-side packing of a list of byte spans into one arena + offsets.
struct Packed {
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off;
};

Packed pack(std::span<const std::span<const uint8_t>> items, size_t extra_per_item = 0) {
    Packed p;
    p.off.resize(items.size() + 1);
    uint64_t total = 0;
    for (size_t i = 0; i < items.size(); ++i) {
        p.off[i] = total;
        total += items[i].size() + extra_per_item;
    }
    p.off[items.size()] = total;
    p.arena.resize(total);
    for (size_t i = 0; i < items.size(); ++i)
        if (!items[i].empty()) std::memcpy(p.arena.data() + p.off[i], items[i].data(), items[i].size());
    return p;
}

std::vector<uint64_t> offsets_of(std::span<const std::span<const uint8_t>> items, int64_t delta) {
    std::vector<uint64_t> off(items.size() + 1);
    uint64_t total = 0;
    for (size_t i = 0; i < items.size(); ++i) {
        off[i] = total;
        int64_t len = (int64_t)items[i].size() + delta;
        total += (uint64_t)std::max<int64_t>(len, 0);
    }
    off[items.size()] = total;
    return off;
}

struct DevRecords {
    enet_records r{};
    uint8_t* out = nullptr;
    uint64_t out_total = 0;
};

// Upload arenas, offsets, keys and nonces; returns the descriptor pointing at device copies.
DevRecords upload(Staging& st, const Packed& in, const std::vector<uint64_t>& out_off,
                  const uint8_t* keys, size_t key_bytes, uint32_t key_stride, const uint8_t* nonces,
                  size_t n) {
    DevRecords d;
    auto* din = (uint8_t*)st.get(S_IN, in.arena.size());
    d.out_total = out_off.back();
    d.out = (uint8_t*)st.get(S_OUT, d.out_total);
    auto* dinoff = (uint64_t*)st.get(S_INOFF, in.off.size() * 8);
    auto* doutoff = (uint64_t*)st.get(S_OUTOFF, out_off.size() * 8);
    auto* dkeys = (uint8_t*)st.get(S_KEYS, key_bytes);
    auto* dnon = (uint8_t*)st.get(S_NONCES, 12 * n);
    st.h2d(din, in.arena.data(), in.arena.size());
    st.h2d(dinoff, in.off.data(), in.off.size() * 8);
    st.h2d(doutoff, out_off.data(), out_off.size() * 8);
    st.h2d(dkeys, keys, key_bytes);
    st.h2d(dnon, nonces, 12 * n);
    d.r.count = (uint32_t)n;
    d.r.in_offsets = dinoff;
    d.r.out_offsets = doutoff;
    d.r.in = din;
    d.r.out = d.out;
    d.r.keys = dkeys;
    d.r.key_stride = key_stride;
    d.r.nonces = dnon;
    d.r.total_bytes_hint = in.arena.size();
    uint64_t mx = 0;
    for (size_t i = 0; i < n; ++i) mx = std::max(mx, in.off[i + 1] - in.off[i]);
    d.r.max_len_hint = (uint32_t)std::min<uint64_t>(mx, 0xffffffffu);
    return d;
}

std::vector<std::vector<uint8_t>> download(Staging& st, const DevRecords& d,
                                           const std::vector<uint64_t>& out_off) {
    std::vector<uint8_t> all(d.out_total);
    st.d2h(all.data(), d.out, d.out_total);
    st.sync();
    std::vector<std::vector<uint8_t>> res(out_off.size() - 1);
    for (size_t i = 0; i + 1 < out_off.size(); ++i)
        res[i].assign(all.begin() + (ptrdiff_t)out_off[i], all.begin() + (ptrdiff_t)out_off[i + 1]);
    return res;
}

std::vector<uint8_t> flat_keys(std::span<const ephemeralnet::crypto::Key> keys) {
    std::vector<uint8_t> v(32 * keys.size());
    for (size_t i = 0; i < keys.size(); ++i) std::memcpy(v.data() + 32 * i, keys[i].bytes.data(), 32);
    return v;
}

std::vector<uint8_t> flat_nonces(std::span<const ephemeralnet::crypto::Nonce> nonces) {
    std::vector<uint8_t> v(12 * nonces.size());
    for (size_t i = 0; i < nonces.size(); ++i) std::memcpy(v.data() + 12 * i, nonces[i].bytes.data(), 12);
    return v;
}

std::array<uint8_t, 32> one_sha(std::span<const uint8_t> data) {
    Staging& st = staging();
    std::span<const uint8_t> items[1] = {data};
    Packed p = pack(items);
    auto* din = (uint8_t*)st.get(S_IN, p.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 16);
    auto* dout = (uint8_t*)st.get(S_OUT, 32);
    st.h2d(din, p.arena.data(), p.arena.size());
    st.h2d(doff, p.off.data(), 16);
    enet_check(enet_sha256_batch(1, din, doff, dout, st.s()), "sha256");
    std::array<uint8_t, 32> d{};
    st.d2h(d.data(), dout, 32);
    st.sync();
    return d;
}

}  // namespace

namespace ephemeralnet::crypto {

// ------------------------------------------------------------------------------ ChaCha20
void ChaCha20::apply(const Key& key, const Nonce& nonce, std::span<const std::uint8_t> input,
                     std::vector<std::uint8_t>& output, std::uint32_t counter) {
    if (input.empty()) {  // ChaCha20.cpp:103-108: resize(0), no block generated
        output.clear();
        return;
    }
    std::span<const uint8_t> items[1] = {input};
    const std::span<const Key> ks(&key, 1);
    const std::span<const Nonce> ns(&nonce, 1);
    const std::uint32_t ctr[1] = {counter};
    auto res = batch::chacha20_apply(ks, ns, items, ctr);
    output = std::move(res[0]);
}

// ------------------------------------------------------------------------------ SHA-256
Sha256::Sha256() = default;

void Sha256::update(std::span<const std::uint8_t> data) {
    pending_.insert(pending_.end(), data.begin(), data.end());
}

std::array<std::uint8_t, 32> Sha256::finalize() {
    auto d = one_sha(pending_);
    std::fill(pending_.begin(), pending_.end(), 0);  // finalize resets (Sha256.cpp:122-124)
    pending_.clear();
    return d;
}

std::array<std::uint8_t, 32> Sha256::digest(std::span<const std::uint8_t> data) { return one_sha(data); }

// ------------------------------------------------------------------------------ HMAC
std::array<std::uint8_t, HmacSha256::kDigestSize> HmacSha256::compute(std::span<const std::uint8_t> key,
                                                                      std::span<const std::uint8_t> data) {
    Staging& st = staging();
    std::span<const uint8_t> items[1] = {data};
    std::span<const uint8_t> kitems[1] = {key};
    Packed p = pack(items);
    Packed k = pack(kitems);
    auto* din = (uint8_t*)st.get(S_IN, p.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 16);
    auto* dk = (uint8_t*)st.get(S_KEYS, k.arena.size());
    auto* dkoff = (uint64_t*)st.get(S_OUTOFF, 16);
    auto* dout = (uint8_t*)st.get(S_OUT, 32);
    st.h2d(din, p.arena.data(), p.arena.size());
    st.h2d(doff, p.off.data(), 16);
    st.h2d(dk, k.arena.data(), k.arena.size());
    st.h2d(dkoff, k.off.data(), 16);
    enet_check(enet_hmac_sha256_batch(1, dk, dkoff, 0, din, doff, dout, st.s()), "hmac");
    std::array<uint8_t, 32> m{};
    st.d2h(m.data(), dout, 32);
    st.sync();
    return m;
}

bool HmacSha256::verify(std::span<const std::uint8_t> key, std::span<const std::uint8_t> data,
                        std::span<const std::uint8_t> mac) {
    if (mac.size() != kDigestSize) return false;  // HmacSha256.cpp:44
    Staging& st = staging();
    std::span<const uint8_t> items[1] = {data};
    std::span<const uint8_t> kitems[1] = {key};
    Packed p = pack(items);
    Packed k = pack(kitems);
    auto* din = (uint8_t*)st.get(S_IN, p.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 16);
    auto* dk = (uint8_t*)st.get(S_KEYS, k.arena.size());
    auto* dkoff = (uint64_t*)st.get(S_OUTOFF, 16);
    auto* dmac = (uint8_t*)st.get(S_TAGS, 32);
    auto* dok = (uint8_t*)st.get(S_OK, 4);
    st.h2d(din, p.arena.data(), p.arena.size());
    st.h2d(doff, p.off.data(), 16);
    st.h2d(dk, k.arena.data(), k.arena.size());
    st.h2d(dkoff, k.off.data(), 16);
    st.h2d(dmac, mac.data(), 32);
    enet_check(enet_hmac_sha256_verify_batch(1, dk, dkoff, 0, din, doff, dmac, dok, st.s()), "hmac verify");
    uint8_t ok = 0;
    st.d2h(&ok, dok, 1);
    st.sync();
    return ok == 1;
}

// ------------------------------------------------------------------------------ CryptoManager
namespace {
std::uint32_t derive_counter(const ChunkId& id) { return enet_chunk_counter(id.data()); }

void fill_random_bytes(std::span<std::uint8_t> buffer) {  // CryptoManager.cpp:17-24
    std::random_device rd;
    for (auto& b : buffer) b = static_cast<std::uint8_t>(rd());
}
}  // namespace

CryptoManager::CryptoManager() : CryptoManager(Key{}) {}

CryptoManager::CryptoManager(Key key) : key_(key), prng_(std::random_device{}()) {
    if (std::all_of(key_.bytes.begin(), key_.bytes.end(), [](auto v) { return v == 0U; }))
        fill_random(key_.bytes);
}

CipherText CryptoManager::encrypt(const ChunkId& chunk_id, const ChunkData& plaintext) {
    CipherText out{};
    fill_random(out.nonce.bytes);
    ChaCha20::apply(key_, out.nonce, plaintext, out.data, derive_counter(chunk_id));
    return out;
}

std::optional<ChunkData> CryptoManager::decrypt(const ChunkId& chunk_id,
                                                std::span<const std::uint8_t> ciphertext,
                                                const Nonce& nonce) const {
    ChunkData pt;
    ChaCha20::apply(key_, nonce, ciphertext, pt, derive_counter(chunk_id));
    return pt;
}

void CryptoManager::fill_random(std::span<std::uint8_t> buffer) const {  // CryptoManager.cpp:60-65
    std::uniform_int_distribution<std::uint32_t> dist(0, 0xFF);
    for (auto& b : buffer) b = static_cast<std::uint8_t>(dist(prng_));
}

Key CryptoManager::generate_key() {
    Key k{};
    fill_random_bytes(k.bytes);
    return k;
}

void CryptoManager::random_bytes(std::span<std::uint8_t> buffer) { fill_random_bytes(buffer); }

CipherText CryptoManager::encrypt_with_key(const Key& key, const ChunkId& chunk_id, const ChunkData& plaintext) {
    CryptoManager m{key};
    return m.encrypt(chunk_id, plaintext);
}

std::optional<ChunkData> CryptoManager::decrypt_with_key(const Key& key, const ChunkId& chunk_id,
                                                         std::span<const std::uint8_t> ciphertext,
                                                         const Nonce& nonce) {
    CryptoManager m{key};
    return m.decrypt(chunk_id, ciphertext, nonce);
}

// ------------------------------------------------------------------------------ batch
namespace batch {

std::vector<std::vector<std::uint8_t>> chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                                                      std::span<const std::span<const std::uint8_t>> inputs,
                                                      std::span<const std::uint32_t> counters) {
    const size_t n = inputs.size();
    if (keys.size() != n || nonces.size() != n || (!counters.empty() && counters.size() != n))
        throw std::invalid_argument("enet batch::chacha20_apply: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(inputs);
    auto kf = flat_keys(keys);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, in.off, kf.data(), kf.size(), 32, nf.data(), n);
    const uint32_t* dctr = nullptr;
    if (!counters.empty()) {
        auto* c = (uint32_t*)st.get(S_CTR, 4 * n);
        st.h2d(c, counters.data(), 4 * n);
        dctr = c;
    }
    enet_check(enet_chacha20_xor_batch(&d.r, dctr, st.s()), "chacha20");
    return download(st, d, in.off);
}

std::vector<Sealed> aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
                              std::span<const std::span<const std::uint8_t>> plaintexts) {
    const size_t n = plaintexts.size();
    if (keys.size() != n || nonces.size() != n) throw std::invalid_argument("enet batch::aead_seal: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(plaintexts);
    auto kf = flat_keys(keys);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, in.off, kf.data(), kf.size(), 32, nf.data(), n);
    auto* tags = (uint8_t*)st.get(S_TAGS, 16 * n);
    enet_check(enet_aead_seal_batch(&d.r, nullptr, nullptr, tags, st.s()), "aead_seal");
    std::vector<uint8_t> th(16 * n);
    st.d2h(th.data(), tags, 16 * n);
    auto data = download(st, d, in.off);
    std::vector<Sealed> res(n);
    for (size_t i = 0; i < n; ++i) {
        res[i].data = std::move(data[i]);
        std::memcpy(res[i].tag.data(), th.data() + 16 * i, 16);
    }
    return res;
}

std::vector<std::vector<std::uint8_t>> aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
                                                 std::span<const std::span<const std::uint8_t>> ciphertexts,
                                                 std::span<const std::array<std::uint8_t, 16>> tags,
                                                 std::vector<std::uint8_t>& ok) {
    const size_t n = ciphertexts.size();
    if (keys.size() != n || nonces.size() != n || tags.size() != n)
        throw std::invalid_argument("enet batch::aead_open: size mismatch");
    ok.assign(n, 0);
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(ciphertexts);
    auto kf = flat_keys(keys);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, in.off, kf.data(), kf.size(), 32, nf.data(), n);
    auto* dt = (uint8_t*)st.get(S_TAGS, 16 * n);
    auto* dok = (uint8_t*)st.get(S_OK, n);
    st.h2d(dt, tags.data(), 16 * n);
    enet_check(enet_aead_open_batch(&d.r, nullptr, nullptr, dt, dok, st.s()), "aead_open");
    st.d2h(ok.data(), dok, n);
    return download(st, d, in.off);
}

std::vector<std::array<std::uint8_t, 32>> sha256(std::span<const std::span<const std::uint8_t>> messages) {
    const size_t n = messages.size();
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(messages);
    auto* din = (uint8_t*)st.get(S_IN, in.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 8 * (n + 1));
    auto* dout = (uint8_t*)st.get(S_OUT, 32 * n);
    st.h2d(din, in.arena.data(), in.arena.size());
    st.h2d(doff, in.off.data(), 8 * (n + 1));
    enet_check(enet_sha256_batch((uint32_t)n, din, doff, dout, st.s()), "sha256");
    std::vector<std::array<std::uint8_t, 32>> res(n);
    st.d2h(res.data(), dout, 32 * n);
    st.sync();
    return res;
}

std::vector<std::vector<std::uint8_t>> frame_seal(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                  std::span<const Nonce> nonces,
                                                  std::span<const std::span<const std::uint8_t>> messages) {
    const size_t n = messages.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::frame_seal: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(messages);
    auto out_off = offsets_of(messages, 32);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, out_off, session_keys.data()->data(), 32 * n, 32, nf.data(), n);
    enet_check(enet_frame_seal_batch(&d.r, st.s()), "frame_seal");
    return download(st, d, out_off);
}

std::vector<std::vector<std::uint8_t>> frame_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                  std::span<const Nonce> nonces,
                                                  std::span<const std::span<const std::uint8_t>> bodies,
                                                  std::vector<std::uint8_t>& ok) {
    const size_t n = bodies.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::frame_open: size mismatch");
    ok.assign(n, 0);
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(bodies);
    auto out_off = offsets_of(bodies, -32);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, out_off, session_keys.data()->data(), 32 * n, 32, nf.data(), n);
    auto* macs = (uint8_t*)st.get(S_TAGS, 32 * n);
    auto* dok = (uint8_t*)st.get(S_OK, n);
    enet_check(enet_frame_open_batch(&d.r, macs, dok, st.s()), "frame_open");
    st.d2h(ok.data(), dok, n);
    return download(st, d, out_off);
}

std::vector<StoredChunk> chunk_store(std::span<const Key> keys, std::span<const Nonce> nonces,
                                     std::span<const std::span<const std::uint8_t>> chunks,
                                     std::span<const ChunkId> chunk_ids) {
    const size_t n = chunks.size();
    if (keys.size() != n || nonces.size() != n || (!chunk_ids.empty() && chunk_ids.size() != n))
        throw std::invalid_argument("enet batch::chunk_store: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(chunks);
    auto kf = flat_keys(keys);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, in.off, kf.data(), kf.size(), 32, nf.data(), n);
    auto* hashes = (uint8_t*)st.get(S_TAGS, 32 * n);
    uint8_t* ids = nullptr;
    if (!chunk_ids.empty()) {
        ids = (uint8_t*)st.get(S_AUX, 32 * n);
        st.h2d(ids, chunk_ids.data(), 32 * n);
    }
    enet_check(enet_chunk_store_batch(&d.r, ids, hashes, st.s()), "chunk_store");
    std::vector<uint8_t> hh(32 * n);
    st.d2h(hh.data(), hashes, 32 * n);
    auto data = download(st, d, in.off);
    std::vector<StoredChunk> res(n);
    for (size_t i = 0; i < n; ++i) {
        res[i].data = std::move(data[i]);
        std::memcpy(res[i].chunk_hash.data(), hh.data() + 32 * i, 32);
    }
    return res;
}

std::vector<std::vector<std::uint8_t>> chunk_fetch(std::span<const Key> keys, std::span<const Nonce> nonces,
                                                   std::span<const ChunkId> chunk_ids,
                                                   std::span<const std::span<const std::uint8_t>> ciphertexts,
                                                   std::span<const std::array<std::uint8_t, 32>> chunk_hashes,
                                                   std::vector<std::uint8_t>& ok) {
    const size_t n = ciphertexts.size();
    if (keys.size() != n || nonces.size() != n || chunk_ids.size() != n || chunk_hashes.size() != n)
        throw std::invalid_argument("enet batch::chunk_fetch: size mismatch");
    ok.assign(n, 0);
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(ciphertexts);
    auto kf = flat_keys(keys);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, in.off, kf.data(), kf.size(), 32, nf.data(), n);
    auto* ids = (uint8_t*)st.get(S_AUX, 32 * n);
    auto* hashes = (uint8_t*)st.get(S_TAGS, 32 * n);
    auto* dok = (uint8_t*)st.get(S_OK, n);
    st.h2d(ids, chunk_ids.data(), 32 * n);
    st.h2d(hashes, chunk_hashes.data(), 32 * n);
    enet_check(enet_chunk_fetch_batch(&d.r, ids, hashes, dok, st.s()), "chunk_fetch");
    st.d2h(ok.data(), dok, n);
    return download(st, d, in.off);
}

std::vector<std::vector<std::uint8_t>> wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                 std::span<const Nonce> nonces,
                                                 std::span<const std::span<const std::uint8_t>> messages) {
    const size_t n = messages.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::wire_seal: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(messages);
    auto out_off = offsets_of(messages, 16 + 32);
    auto nf = flat_nonces(nonces);
    DevRecords d = upload(st, in, out_off, session_keys.data()->data(), 32 * n, 32, nf.data(), n);
    enet_check(enet_wire_seal_batch(&d.r, st.s()), "wire_seal");
    return download(st, d, out_off);
}

std::vector<std::vector<std::uint8_t>> wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                 std::span<const std::span<const std::uint8_t>> frames,
                                                 std::vector<std::uint8_t>& ok) {
    const size_t n = frames.size();
    if (session_keys.size() != n) throw std::invalid_argument("enet batch::wire_open: size mismatch");
    ok.assign(n, 0);
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(frames);
    auto out_off = offsets_of(frames, -(16 + 32));
    std::vector<uint8_t> no_nonces(12 * n, 0);  // unused: the nonce travels in the frame
    DevRecords d = upload(st, in, out_off, session_keys.data()->data(), 32 * n, 32, no_nonces.data(), n);
    auto* macs = (uint8_t*)st.get(S_TAGS, 32 * n);
    auto* dok = (uint8_t*)st.get(S_OK, n);
    enet_check(enet_wire_open_batch(&d.r, macs, dok, st.s()), "wire_open");
    st.d2h(ok.data(), dok, n);
    return download(st, d, out_off);
}

bool FrameQueue::push(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> message) {
    if (message.size() + 32 > kMaxPayloadSize) return false;
    Nonce nonce{};
    std::random_device rd;
    for (auto& byte : nonce.bytes) byte = static_cast<std::uint8_t>(rd());
    keys_.push_back(session_key);
    nonces_.push_back(nonce);
    messages_.emplace_back(message.begin(), message.end());
    return true;
}

std::vector<std::vector<std::uint8_t>> FrameQueue::flush() {
    std::vector<std::span<const std::uint8_t>> views(messages_.begin(), messages_.end());
    auto frames = wire_seal(keys_, nonces_, views);
    keys_.clear();
    nonces_.clear();
    messages_.clear();
    return frames;
}

// ------------------------------------------------------------------------------ proof of work
namespace {
void put_be64(std::vector<std::uint8_t>& v, std::uint64_t x) {
    for (int i = 0; i < 8; ++i) v.push_back(static_cast<std::uint8_t>(x >> (56 - 8 * i)));
}
void put_lp64(std::vector<std::uint8_t>& v, const std::uint8_t* p, std::size_t n) {  // Node.cpp:149-153
    put_be64(v, n);
    v.insert(v.end(), p, p + n);
}
}  // namespace

std::vector<PowResult> pow_search(std::span<const std::span<const std::uint8_t>> prefixes,
                                  std::span<const std::uint8_t> difficulty, PowSchedule schedule,
                                  std::uint64_t max_attempts) {
    const size_t n = prefixes.size();
    if (difficulty.size() != n) throw std::invalid_argument("enet batch::pow_search: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(prefixes);
    auto* din = (uint8_t*)st.get(S_IN, in.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 8 * (n + 1));
    auto* dd = (uint8_t*)st.get(S_AUX, n);
    auto* dnonce = (uint64_t*)st.get(S_OUT, 8 * n);
    auto* datt = (uint64_t*)st.get(S_TAGS, 8 * n);
    auto* dfound = (uint8_t*)st.get(S_OK, n);
    st.h2d(din, in.arena.data(), in.arena.size());
    st.h2d(doff, in.off.data(), 8 * (n + 1));
    st.h2d(dd, difficulty.data(), n);
    enet_check(enet_pow_search_batch((uint32_t)n, din, doff, dd, static_cast<int>(schedule), max_attempts,
                                     dnonce, datt, dfound, st.s()),
               "pow_search");
    std::vector<std::uint64_t> nonce(n), att(n);
    std::vector<std::uint8_t> found(n);
    st.d2h(nonce.data(), dnonce, 8 * n);
    st.d2h(att.data(), datt, 8 * n);
    st.d2h(found.data(), dfound, n);
    st.sync();
    std::vector<PowResult> res(n);
    for (size_t i = 0; i < n; ++i) res[i] = PowResult{found[i] != 0, nonce[i], att[i]};
    return res;
}

std::vector<std::uint8_t> pow_check(std::span<const std::span<const std::uint8_t>> prefixes,
                                    std::span<const std::uint64_t> nonces,
                                    std::span<const std::uint8_t> difficulty) {
    const size_t n = prefixes.size();
    if (difficulty.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::pow_check: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    Packed in = pack(prefixes);
    auto* din = (uint8_t*)st.get(S_IN, in.arena.size());
    auto* doff = (uint64_t*)st.get(S_INOFF, 8 * (n + 1));
    auto* dd = (uint8_t*)st.get(S_AUX, n);
    auto* dnonce = (uint64_t*)st.get(S_CTR, 8 * n);
    auto* dok = (uint8_t*)st.get(S_OK, n);
    st.h2d(din, in.arena.data(), in.arena.size());
    st.h2d(doff, in.off.data(), 8 * (n + 1));
    st.h2d(dd, difficulty.data(), n);
    st.h2d(dnonce, nonces.data(), 8 * n);
    enet_check(enet_pow_check_batch((uint32_t)n, din, doff, dnonce, dd, dok, st.s()), "pow_check");
    std::vector<std::uint8_t> ok(n);
    st.d2h(ok.data(), dok, n);
    st.sync();
    return ok;
}

std::vector<std::uint8_t> announce_pow_prefix(const ChunkId& chunk_id, const PeerId& peer_id,
                                              std::string_view endpoint, std::string_view manifest_uri,
                                              std::span<const std::uint8_t> assigned_shards,
                                              std::int64_t ttl_seconds) {
    std::vector<std::uint8_t> v;
    v.reserve(120 + endpoint.size() + manifest_uri.size() + assigned_shards.size());
    put_lp64(v, chunk_id.data(), chunk_id.size());
    put_lp64(v, peer_id.data(), peer_id.size());
    put_lp64(v, reinterpret_cast<const std::uint8_t*>(endpoint.data()), endpoint.size());
    put_lp64(v, reinterpret_cast<const std::uint8_t*>(manifest_uri.data()), manifest_uri.size());
    put_lp64(v, assigned_shards.data(), assigned_shards.size());
    put_be64(v, static_cast<std::uint64_t>(ttl_seconds));  // Node.cpp:165-166
    return v;
}

std::vector<std::uint8_t> handshake_pow_prefix(const PeerId& initiator, const PeerId& responder,
                                               std::uint32_t initiator_public) {
    std::vector<std::uint8_t> v;
    v.reserve(88);
    put_lp64(v, initiator.data(), initiator.size());
    put_lp64(v, responder.data(), responder.size());
    put_be64(v, static_cast<std::uint64_t>(initiator_public));  // Node.cpp:241-242
    return v;
}

namespace {
bool node_pow_one(const std::vector<std::uint8_t>& prefix, std::uint8_t difficulty, std::uint64_t& nonce_out) {
    if (difficulty == 0) {  // Node.cpp:213-216 / 274-277
        nonce_out = 0;
        return true;
    }
    const std::span<const std::uint8_t> ps[1] = {prefix};
    const std::uint8_t d[1] = {difficulty};
    const auto r = pow_search(ps, d, PowSchedule::Node, kNodePowAttempts);
    if (!r[0].found) return false;
    nonce_out = r[0].nonce;
    return true;
}
}  // namespace

bool compute_announce_pow(const ChunkId& chunk_id, const PeerId& peer_id, std::string_view endpoint,
                          std::string_view manifest_uri, std::span<const std::uint8_t> assigned_shards,
                          std::int64_t ttl_seconds, std::uint8_t difficulty, std::uint64_t& nonce_out) {
    return node_pow_one(announce_pow_prefix(chunk_id, peer_id, endpoint, manifest_uri, assigned_shards, ttl_seconds),
                        difficulty, nonce_out);
}

bool compute_handshake_pow(const PeerId& initiator, const PeerId& responder, std::uint32_t initiator_public,
                           std::uint8_t difficulty, std::uint64_t& nonce_out) {
    return node_pow_one(handshake_pow_prefix(initiator, responder, initiator_public), difficulty, nonce_out);
}

std::vector<std::array<std::uint8_t, 32>> session_keys(std::span<const Key> secrets,
                                                       std::span<const std::uint64_t> counters,
                                                       std::span<const std::int64_t> ticks) {
    const size_t n = secrets.size();
    if (counters.size() != n || ticks.size() != n)
        throw std::invalid_argument("enet batch::session_keys: size mismatch");
    if (n == 0) return {};
    Staging& st = staging();
    auto kf = flat_keys(secrets);
    auto* dk = (uint8_t*)st.get(S_KEYS, 32 * n);
    auto* dc = (uint64_t*)st.get(S_CTR, 8 * n);
    auto* dt = (int64_t*)st.get(S_NONCES, 8 * n);
    auto* dout = (uint8_t*)st.get(S_OUT, 32 * n);
    st.h2d(dk, kf.data(), 32 * n);
    st.h2d(dc, counters.data(), 8 * n);
    st.h2d(dt, ticks.data(), 8 * n);
    enet_check(enet_session_key_batch((uint32_t)n, dk, dc, dt, dout, st.s()), "session_keys");
    std::vector<std::array<std::uint8_t, 32>> res(n);
    st.d2h(res.data(), dout, 32 * n);
    st.sync();
    return res;
}

}  // namespace batch
}  // namespace ephemeralnet::crypto

// ------------------------------------------------------------------------------ security::StoreProof
namespace ephemeralnet::security {

ChunkId derive_chunk_id(std::span<const std::uint8_t> data) { return one_sha(data); }

std::optional<std::string> sanitize_filename_hint(std::string_view raw_path) {
    if (raw_path.empty()) return std::nullopt;
    const std::filesystem::path provided(raw_path);
    const auto base = provided.filename().string();
    if (base.empty() || base == "." || base == "..") return std::nullopt;
    constexpr std::size_t kMaxFilenameLength = 255;  // StoreProof.cpp:100
    if (base.size() <= kMaxFilenameLength) return base;
    return base.substr(0, kMaxFilenameLength);
}

std::vector<std::uint8_t> store_pow_prefix(const StoreWorkInput& input) {
    std::vector<std::uint8_t> v(input.chunk_id.begin(), input.chunk_id.end());
    for (int i = 0; i < 8; ++i) v.push_back(static_cast<std::uint8_t>(input.payload_size >> (56 - 8 * i)));
    const auto len = static_cast<std::uint32_t>(
        std::min<std::size_t>(input.filename_hint.size(), std::numeric_limits<std::uint32_t>::max()));
    for (int i = 0; i < 4; ++i) v.push_back(static_cast<std::uint8_t>(len >> (24 - 8 * i)));
    v.insert(v.end(), input.filename_hint.begin(), input.filename_hint.end());
    return v;
}

namespace {
std::uint8_t clamp_store_difficulty(std::uint8_t d) {  // StoreProof.cpp:114-116, 128-130
    return d > kMaxStorePowDifficulty ? kMaxStorePowDifficulty : d;
}
}  // namespace

namespace batch {
std::vector<std::optional<std::uint64_t>> compute_store_pow(std::span<const StoreWorkInput> inputs,
                                                            std::uint8_t difficulty_bits,
                                                            std::uint64_t max_attempts) {
    std::vector<std::optional<std::uint64_t>> res(inputs.size());
    if (inputs.empty()) return res;
    if (difficulty_bits == 0) {  // StoreProof.cpp:125-127
        for (auto& r : res) r = std::uint64_t{0};
        return res;
    }
    const std::uint8_t d = clamp_store_difficulty(difficulty_bits);
    if (max_attempts == 0) max_attempts = kDefaultStorePowMaxAttempts;  // :131-133
    std::vector<std::vector<std::uint8_t>> pre;
    pre.reserve(inputs.size());
    for (const auto& in : inputs) pre.push_back(store_pow_prefix(in));
    std::vector<std::span<const std::uint8_t>> views(pre.begin(), pre.end());
    std::vector<std::uint8_t> diffs(inputs.size(), d);
    auto r = crypto::batch::pow_search(views, diffs, crypto::batch::PowSchedule::Store, max_attempts);
    for (size_t i = 0; i < r.size(); ++i)
        if (r[i].found) res[i] = r[i].nonce;
    return res;
}

std::vector<std::uint8_t> store_pow_valid(std::span<const StoreWorkInput> inputs,
                                          std::span<const std::uint64_t> nonces,
                                          std::uint8_t difficulty_bits) {
    if (nonces.size() != inputs.size()) throw std::invalid_argument("enet store_pow_valid: size mismatch");
    if (difficulty_bits == 0) return std::vector<std::uint8_t>(inputs.size(), 1);  // :112-113
    std::vector<std::vector<std::uint8_t>> pre;
    pre.reserve(inputs.size());
    for (const auto& in : inputs) pre.push_back(store_pow_prefix(in));
    std::vector<std::span<const std::uint8_t>> views(pre.begin(), pre.end());
    std::vector<std::uint8_t> diffs(inputs.size(), clamp_store_difficulty(difficulty_bits));
    return crypto::batch::pow_check(views, nonces, diffs);
}
}  // namespace batch

bool store_pow_valid(const StoreWorkInput& input, std::uint64_t nonce, std::uint8_t difficulty_bits) {
    return batch::store_pow_valid(std::span(&input, 1), std::span(&nonce, 1), difficulty_bits)[0] == 1;
}

std::optional<std::uint64_t> compute_store_pow(const StoreWorkInput& input, std::uint8_t difficulty_bits,
                                               std::uint64_t max_attempts) {
    return batch::compute_store_pow(std::span(&input, 1), difficulty_bits, max_attempts)[0];
}

}  // namespace ephemeralnet::security

// ------------------------------------------------------------------------------ network::KeyManager
namespace ephemeralnet::network {

namespace {
std::int64_t ticks_of(std::chrono::steady_clock::time_point t) {  // KeyManager.cpp:24, 83
    return std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
}
}  // namespace

KeyManager::KeyManager(std::chrono::seconds rotation_interval) : rotation_interval_(rotation_interval) {}

void KeyManager::register_session(const PeerId& peer_id, const crypto::Key& shared_secret) {
    const auto now = std::chrono::steady_clock::now();
    std::array<std::uint8_t, 16> material{};  // BE64(counter 0) || BE64(ticks), KeyManager.cpp:15-30
    const std::uint64_t ticks = static_cast<std::uint64_t>(ticks_of(now));
    for (int i = 0; i < 8; ++i) material[8 + i] = static_cast<std::uint8_t>(ticks >> (56 - 8 * i));
    register_session_with_material(peer_id, shared_secret, material, now);
}

void KeyManager::register_session_with_material(const PeerId& peer_id, const crypto::Key& shared_secret,
                                                std::span<const std::uint8_t> material,
                                                std::chrono::steady_clock::time_point reference_time) {
    SessionKeyContext context{};
    context.shared_secret = shared_secret;
    context.last_rotation = reference_time;
    context.counter = 0;
    context.current_key = crypto::HmacSha256::compute(shared_secret.bytes, material);  // :42-43
    contexts_[peer_id] = context;
}

std::optional<std::array<std::uint8_t, 32>> KeyManager::current_key(const PeerId& peer_id) const {
    const auto it = contexts_.find(peer_id);
    if (it == contexts_.end()) return std::nullopt;
    return it->second.current_key;
}

std::optional<std::array<std::uint8_t, 32>> KeyManager::rotate_if_needed(
    const PeerId& peer_id, std::chrono::steady_clock::time_point now) {
    auto it = contexts_.find(peer_id);
    if (it == contexts_.end()) return std::nullopt;
    auto& context = it->second;
    if (now - context.last_rotation < rotation_interval_) return std::nullopt;  // :63-65
    context.counter += 1;
    context.last_rotation = now;
    const std::uint64_t ctr[1] = {context.counter};
    const std::int64_t tk[1] = {ticks_of(now)};
    context.current_key = crypto::batch::session_keys(std::span(&context.shared_secret, 1), ctr, tk)[0];
    return context.current_key;
}

std::vector<PeerId> KeyManager::known_peers() const {
    std::vector<PeerId> peers;
    peers.reserve(contexts_.size());
    for (const auto& [peer, context] : contexts_) {
        (void)context;
        peers.push_back(peer);
    }
    return peers;
}

std::vector<std::pair<PeerId, std::array<std::uint8_t, 32>>> KeyManager::rotate_all_due(
    std::chrono::steady_clock::time_point now) {
    std::vector<SessionKeyContext*> due;
    std::vector<PeerId> peers;
    std::vector<crypto::Key> secrets;
    std::vector<std::uint64_t> counters;
    std::vector<std::int64_t> ticks;
    for (auto& [peer, context] : contexts_) {
        if (now - context.last_rotation < rotation_interval_) continue;
        due.push_back(&context);
        peers.push_back(peer);
        secrets.push_back(context.shared_secret);
        counters.push_back(context.counter + 1);
        ticks.push_back(ticks_of(now));
    }
    std::vector<std::pair<PeerId, std::array<std::uint8_t, 32>>> out;
    if (due.empty()) return out;
    auto keys = crypto::batch::session_keys(secrets, counters, ticks);
    out.reserve(due.size());
    for (size_t i = 0; i < due.size(); ++i) {
        due[i]->counter = counters[i];
        due[i]->last_rotation = now;
        due[i]->current_key = keys[i];
        out.emplace_back(peers[i], keys[i]);
    }
    return out;
}

}  // namespace ephemeralnet::network
