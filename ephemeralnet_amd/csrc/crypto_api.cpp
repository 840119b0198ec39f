// crypto_api.cpp -- the reference C++ API (namespace ephemeralnet::crypto, security, network)
// implemented over the C ABI and the scalar host engine.
//
// Two kinds of entry points live here:
//   * the reference's own signatures (ChaCha20::apply, Sha256, HmacSha256, CryptoManager,
//     security::*, network::KeyManager): one record per call, from many session threads, never
//     throwing.  They are routed by size (enet_crypto.h "scalar"): serial and
//     small work on the calling thread's host engine (host_engine.cpp), large ChaCha20 records
//     on the MI355X with concurrent callers coalesced into one launch, PoW searches on the
//     MI355X.  A device failure finishes the call on the host engine (bit-exact) instead of
//     throwing into a caller that never catches (SessionManager::receive_loop runs on a detached
//     thread, SessionManager.cpp:703-854).
//   * crypto::batch::* (Batch.hpp): many records per call, always on the MI355X; they throw
//     std::invalid_argument / std::runtime_error (not reference signatures).
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
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <limits>
#include <mutex>
#include <new>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "enet_crypto.h"
#include "host_batch.hpp"
#include "host_engine.hpp"
#include "scalar.hpp"

// ------------------------------------------------------------------------------ scalar routing
namespace enet::scalar {
// The initial policy: ENET_SCALAR_POLICY=auto|device|host, so an unmodified binary built against
// the reference headers (the reference's own test programs, tests/test_reference_programs.py) can
// run on either engine; enet_scalar_set_policy changes it at run time.
int initial_policy() {
    const char* e = std::getenv("ENET_SCALAR_POLICY");
    if (!e) return ENET_SCALAR_AUTO;
    if (std::strcmp(e, "device") == 0) return ENET_SCALAR_DEVICE;
    if (std::strcmp(e, "host") == 0) return ENET_SCALAR_HOST;
    return ENET_SCALAR_AUTO;
}
std::atomic<int> g_policy{initial_policy()};
// ChaCha20 records from this size go to the MI355X under ENET_SCALAR_AUTO.  Default: never.
// Measured on the box: the host engine's AVX-512 keystream runs ~10 GB/s per
// thread, i.e. as fast as the memcpy that moves a pageable caller buffer into pinned memory, so
// for a caller's std::vector the device round trip never wins; a deployment whose cores are the
// bottleneck opts in with enet_scalar_set_policy(ENET_SCALAR_AUTO, bytes).
std::atomic<uint64_t> g_crossover{UINT64_MAX};
std::atomic<int> g_on_error{0};
std::atomic<uint64_t> g_failures{0}, g_launches{0}, g_records{0};
// Per-call counters are sharded over cache lines: one shared atomic incremented by every session
// thread on every 0.25 us HMAC capped 16 threads at 7 M calls/s (the reference does 11.6 M).
struct alignas(64) CallShard {
    std::atomic<uint64_t> host{0}, device{0};
};
CallShard g_shards[64];
CallShard& shard() {
    static std::atomic<unsigned> next{0};
    thread_local CallShard& s = g_shards[next.fetch_add(1, std::memory_order_relaxed) & 63u];
    return s;
}
std::atomic<uint32_t> g_inject{0};
std::atomic<bool> g_reported{false};

// does a call with a device kernel and `bytes` of payload go to the MI355X?
bool device_for(uint64_t bytes, bool has_crossover) {
    const int p = g_policy.load(std::memory_order_relaxed);
    if (p == ENET_SCALAR_HOST) return false;
    if (p == ENET_SCALAR_DEVICE) return true;
    return has_crossover && bytes >= g_crossover.load(std::memory_order_relaxed);
}

void host_call() { shard().host.fetch_add(1, std::memory_order_relaxed); }
void device_call() { shard().device.fetch_add(1, std::memory_order_relaxed); }

// throws like a failed HIP call when a test injected failures
void maybe_inject() {
    uint32_t n = g_inject.load(std::memory_order_relaxed);
    while (n > 0 && !g_inject.compare_exchange_weak(n, n - 1, std::memory_order_relaxed)) {
    }
    if (n > 0) throw std::runtime_error("enet: injected device failure (enet_scalar_inject_device_failures)");
}

// a device call of the scalar API failed: count it, say so once, finish on the host (or abort)
void device_failed(const char* what, const char* why) noexcept {
    g_failures.fetch_add(1, std::memory_order_relaxed);
    if (g_on_error.load(std::memory_order_relaxed) == 1) {
        std::fprintf(stderr, "enet: device path of %s failed (%s); aborting as configured\n", what, why);
        std::abort();
    }
    if (!g_reported.exchange(true))
        std::fprintf(stderr,
                     "enet: device path of %s failed (%s); this and later failed scalar calls are "
                     "finished on the host engine (enet_scalar_get_stats counts them)\n",
                     what, why);
}

}  // namespace enet::scalar

namespace {
namespace scalar = enet::scalar;

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("enet: ") + what + ": " + hipGetErrorString(e));
}

void enet_check(int rc, const char* what) {
    if (rc != ENET_OK) throw std::runtime_error(std::string("enet: ") + what + ": " + enet_last_error());
}


// Staging buffers + one stream per host thread, for the batch API and the scalar API's device
// path under ENET_SCALAR_DEVICE.  Buffers of up to kZeroCopyMax bytes come from one pinned,
// device-mapped, coherent host blob -- "uploading" is a host memcpy into it, the kernel reads
// its operands over PCIe and writes its results straight back, and "downloading" is a memcpy
// after the stream sync -- so a small call costs one launch and one sync instead of up to six
// pageable copies.  The blob is 256 KiB (every small call fits: ~10 slots of <= 8 KiB; ADVICE r02:
// 8 MiB per session thread pinned too much), allocated on the first small call of a thread.
// Larger buffers keep grow-only device slots and async copies.  The blob is bump-allocated and
// rewound at every sync (every API call ends with one), so no region is rewritten while a kernel
// of the same call may still read it.
struct Staging {
    static constexpr int kSlots = 10;
    static constexpr size_t kHostBlob = 256u << 10;
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
            if (dev[slot]) {
                (void)hipFree(dev[slot]);
                dev[slot] = nullptr;
                cap[slot] = 0;
            }
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
    // Wait for the call's work, then run the deferred zero-copy downloads.  The pending list and
    // the blob are released BEFORE the status check: a failed sync must not leave pointers into
    // the caller's (about to be destroyed) vectors for the next call to write through.
    void sync() {
        std::vector<Pending> todo;
        todo.swap(pend);
        used = 0;
        hip_check(hipStreamSynchronize(s()), "hipStreamSynchronize");
        for (const Pending& q : todo) std::memcpy(q.dst, q.src, q.n);
    }
    // drop queued downloads and rewind after a failed call
    void reset() noexcept {
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

std::vector<uint8_t> flat_keys(std::span<const ephemeralnet::crypto::Key> keys) {
    std::vector<uint8_t> v(32 * keys.size());
    for (size_t i = 0; i < keys.size(); ++i) std::memcpy(v.data() + 32 * i, keys[i].bytes.data(), 32);
    return v;
}

// A throwing device call inside a Staging sequence: rewind the thread's staging before the
// exception leaves, so the next call starts clean.
template <class F>
auto staged(F&& f) -> decltype(f(staging())) {
    Staging& st = staging();
    st.reset();
    try {
        return f(st);
    } catch (...) {
        st.reset();
        throw;
    }
}

std::array<uint8_t, 32> device_sha(std::span<const uint8_t> data) {
    return staged([&](Staging& st) {
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
    });
}

std::array<uint8_t, 32> device_hmac(std::span<const uint8_t> key, std::span<const uint8_t> data) {
    return staged([&](Staging& st) {
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
    });
}

// ------------------------------------------------------------------------------ coalescer
// ChaCha20::apply records routed to the MI355X.  Each caller queues its request; whichever caller
// finds no launch in flight becomes the leader, takes EVERY pending request, and runs them as one
// enet_chacha20_xor_batch; requests arriving meanwhile wait for the next leader.  No artificial
// delay: a lone caller launches at once, and under load the batch grows by itself while the
// previous one runs.  The callers' vectors are pageable, and pageable hipMemcpy crawls on the
// box (~0.8 GB/s round trip: a 64 KiB call took 167 us), so the leader copies
// the records into a pinned, device-mapped arena and the kernel works on it in place over PCIe
// (zero-copy: one launch, no DMA), then copies the results out.  One arena, grow-only up to
// kArenaMax; records that do not fit are finished on the host engine.
struct ChachaReq {
    const uint8_t* key;
    const uint8_t* nonce;
    uint32_t counter;
    const uint8_t* in;
    uint8_t* out;
    size_t n;
    bool done = false;
    bool ok = false;
};

class Coalescer {
public:
    static constexpr size_t kArenaMax = 256u << 20;
    static Coalescer& get() {
        static Coalescer* c = new Coalescer();  // never destroyed: no HIP calls during exit
        return *c;
    }
    bool submit(ChachaReq& r) {
        std::unique_lock<std::mutex> lk(mu_);
        pending_.push_back(&r);
        while (!r.done) {
            if (busy_) {
                cv_.wait(lk);
                continue;
            }
            busy_ = true;
            std::vector<ChachaReq*> batch;
            batch.swap(pending_);
            lk.unlock();
            // Whatever leaves the leader section (bad_alloc included), every request it took is
            // marked done -- ok stays false for the ones not run, so their callers finish on the
            // host engine -- and the next leader can start (a throw here used to
            // leave busy_ set and every later device-routed caller waiting forever).
            struct Release {
                Coalescer& c;
                std::unique_lock<std::mutex>& lk;
                std::vector<ChachaReq*>& batch;
                ~Release() {
                    if (!lk.owns_lock()) lk.lock();
                    for (ChachaReq* q : batch) q->done = true;
                    c.busy_ = false;
                    c.cv_.notify_all();
                }
            } release{*this, lk, batch};
            // groups that fit the arena; a record larger than the arena alone stays !ok (host)
            size_t i = 0;
            while (i < batch.size()) {
                size_t j = i, bytes = 0;
                while (j < batch.size() && (j == i || bytes + batch[j]->n <= kArenaMax)) bytes += batch[j++]->n;
                bool ok = false;
                if (bytes <= kArenaMax) {
                    try {
                        scalar::maybe_inject();
                        run(batch, i, j);
                        ok = true;
                    } catch (const std::exception& e) {
                        scalar::device_failed("ChaCha20::apply", e.what());
                    } catch (...) {
                        scalar::device_failed("ChaCha20::apply", "unknown error");
                    }
                }
                for (size_t q = i; q < j; ++q) batch[q]->ok = ok;
                i = j;
            }
        }
        return r.ok;
    }

private:
    // Records longer than kSeg are cut into kSeg-byte segments, each its own record with start
    // counter counter + kSeg/64 * k (mod 2^32, as ChaCha20.cpp:110 wraps): one record gets at most
    // 16 lanes, so a lone 1 MiB record ran on 16 lanes at ~0.5 GB/s.
    static constexpr size_t kSeg = 16u << 10;

    void run(const std::vector<ChachaReq*>& all, size_t first, size_t last) {
        const std::span<ChachaReq* const> batch(all.data() + first, last - first);
        size_t nseg = 0;
        uint64_t rec = 0;
        for (const ChachaReq* q : batch) {
            nseg += (q->n + kSeg - 1) / kSeg;
            rec += q->n;
        }
        // arena: records back to back | offsets [nseg+1] | keys [nseg][32] | nonces [nseg][12] | counters [nseg]
        const size_t off_at = (rec + 255) & ~size_t(255), keys_at = off_at + 8 * (nseg + 1),
                     non_at = keys_at + 32 * nseg, ctr_at = (non_at + 12 * nseg + 3) & ~size_t(3),
                     total = ctr_at + 4 * nseg;
        if (total > cap_) {
            if (arena_) (void)hipHostFree(arena_);
            arena_ = nullptr;
            const size_t c = std::max(total, std::min(kArenaMax + (64u << 10), std::max<size_t>(2 * cap_, 4u << 20)));
            cap_ = 0;
            hip_check(hipHostMalloc(reinterpret_cast<void**>(&arena_), c, hipHostMallocMapped), "hipHostMalloc");
            cap_ = c;
            void* dp = nullptr;
            hip_check(hipHostGetDevicePointer(&dp, arena_, 0), "hipHostGetDevicePointer");
            dev_ = static_cast<uint8_t*>(dp);
        }
        uint64_t* offs = reinterpret_cast<uint64_t*>(arena_ + off_at);
        uint64_t o = 0;
        size_t k = 0;
        for (const ChachaReq* q : batch) {
            std::memcpy(arena_ + o, q->in, q->n);
            for (size_t at = 0; at < q->n; at += kSeg, ++k) {
                offs[k] = o + at;
                std::memcpy(arena_ + keys_at + 32 * k, q->key, 32);
                std::memcpy(arena_ + non_at + 12 * k, q->nonce, 12);
                const uint32_t c = q->counter + (uint32_t)(at / 64);  // u32 wrap
                std::memcpy(arena_ + ctr_at + 4 * k, &c, 4);
            }
            o += q->n;
        }
        offs[nseg] = o;
        enet_records r{};
        r.count = (uint32_t)nseg;
        r.in_offsets = reinterpret_cast<const uint64_t*>(dev_ + off_at);
        r.out_offsets = r.in_offsets;
        r.in = dev_;
        r.out = dev_;  // in place
        r.keys = dev_ + keys_at;
        r.key_stride = 32;
        r.nonces = dev_ + non_at;
        r.total_bytes_hint = rec;
        r.max_len_hint = (uint32_t)std::min<uint64_t>(rec, kSeg);
        enet_check(enet_chacha20_xor_batch(&r, reinterpret_cast<const uint32_t*>(dev_ + ctr_at), st_.s()),
                   "chacha20 (coalesced)");
        hip_check(hipStreamSynchronize(st_.s()), "hipStreamSynchronize");
        o = 0;
        for (const ChachaReq* q : batch) {
            std::memcpy(q->out, arena_ + o, q->n);
            o += q->n;
        }
        scalar::g_launches.fetch_add(1, std::memory_order_relaxed);
        scalar::g_records.fetch_add(batch.size(), std::memory_order_relaxed);
    }

    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<ChachaReq*> pending_;
    bool busy_ = false;
    uint8_t* arena_ = nullptr;  // pinned, device-mapped
    uint8_t* dev_ = nullptr;    // its device address
    size_t cap_ = 0;
    Staging st_;
};

}  // namespace

// ------------------------------------------------------------------------------ scalar C ABI
extern "C" {

int enet_scalar_set_policy(int policy, uint64_t crossover_bytes) {
    if (policy != ENET_SCALAR_AUTO && policy != ENET_SCALAR_DEVICE && policy != ENET_SCALAR_HOST)
        return ENET_EINVAL;
    scalar::g_policy.store(policy, std::memory_order_relaxed);
    if (crossover_bytes) scalar::g_crossover.store(crossover_bytes, std::memory_order_relaxed);
    return ENET_OK;
}

int enet_scalar_policy(void) { return scalar::g_policy.load(std::memory_order_relaxed); }

int enet_scalar_set_on_device_error(int mode) {
    if (mode != 0 && mode != 1) return ENET_EINVAL;
    scalar::g_on_error.store(mode, std::memory_order_relaxed);
    return ENET_OK;
}

void enet_scalar_get_stats(enet_scalar_stats* out) {
    if (!out) return;
    out->host_calls = 0;
    out->device_calls = 0;
    for (const auto& sh : scalar::g_shards) {
        out->host_calls += sh.host.load();
        out->device_calls += sh.device.load();
    }
    out->device_failures = scalar::g_failures.load();
    out->coalesced_launches = scalar::g_launches.load();
    out->coalesced_records = scalar::g_records.load();
}

void enet_scalar_reset_stats(void) {
    for (auto& sh : scalar::g_shards) {
        sh.host = 0;
        sh.device = 0;
    }
    scalar::g_failures = 0;
    scalar::g_launches = 0;
    scalar::g_records = 0;
}

void enet_scalar_inject_device_failures(uint32_t n) { scalar::g_inject.store(n); }

const char* enet_host_isa(void) { return enet::host::isa(); }

void enet_host_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                            const uint8_t* in, uint8_t* out, uint64_t n) {
    enet::host::chacha20_xor(key, nonce, counter, in, out, n);
}

void enet_host_sha256(const uint8_t* in, uint64_t n, uint8_t digest[32]) {
    const auto d = enet::host::sha256(in, n);
    std::memcpy(digest, d.data(), 32);
}

void enet_host_hmac_sha256(const uint8_t* key, uint64_t key_len, const uint8_t* in, uint64_t n,
                           uint8_t mac[32]) {
    const auto m = enet::host::hmac_sha256(key, key_len, in, n);
    std::memcpy(mac, m.data(), 32);
}

void enet_host_seal_body(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* m, uint64_t n,
                         uint8_t* out) {
    enet::host::seal_body(key, nonce, m, n, out);
}

int enet_host_open_body(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* body, uint64_t bl,
                        uint8_t* m) {
    return enet::host::open_body(key, nonce, body, bl, m) ? 1 : 0;
}

int enet_host_set_seal_stitch(int mode) { return enet::host::set_seal_stitch(mode); }

}  // extern "C"

namespace ephemeralnet::crypto {

// ------------------------------------------------------------------------------ ChaCha20
void ChaCha20::apply(const Key& key, const Nonce& nonce, std::span<const std::uint8_t> input,
                     std::vector<std::uint8_t>& output, std::uint32_t counter) {
    if (input.empty()) {  // ChaCha20.cpp:103-108: resize(0), no block generated
        output.clear();
        return;
    }
    const size_t n = input.size();
    // the input may alias the output vector (in-place use): copy it before resizing moves it
    std::vector<uint8_t> keep;
    const uint8_t* in = input.data();
    if (!output.empty() && in >= output.data() && in < output.data() + output.size() && n > output.size()) {
        keep.assign(input.begin(), input.end());
        in = keep.data();
    }
    output.resize(n);
    if (scalar::device_for(n, true)) {
        ChachaReq r{key.bytes.data(), nonce.bytes.data(), counter, in, output.data(), n};
        bool ok = false;
        try {
            ok = Coalescer::get().submit(r);
        } catch (const std::bad_alloc&) {
            throw;
        } catch (...) {
            scalar::device_failed("ChaCha20::apply", "coalescer error");
        }
        if (ok) {
            scalar::device_call();
            return;
        }
    }
    scalar::host_call();
    enet::host::chacha20_xor(key.bytes.data(), nonce.bytes.data(), counter, in, output.data(), n);
}

// ------------------------------------------------------------------------------ SHA-256
// Streaming over the reference's own member layout (Sha256.hpp): 64-byte buffer, running state.
Sha256::Sha256() {
    std::memcpy(state_.data(), enet::host::kIV, sizeof(enet::host::kIV));
}

void Sha256::transform(const std::uint8_t block[64]) { enet::host::sha256_blocks(state_.data(), block, 1); }

void Sha256::update(std::span<const std::uint8_t> data) {  // Sha256.cpp:72-92
    const uint8_t* p = data.data();
    size_t n = data.size();
    if (!n) return;
    bit_len_ += (std::uint64_t)n * 8u;
    if (buffer_size_) {
        const size_t m = std::min(n, 64 - buffer_size_);
        std::memcpy(buffer_.data() + buffer_size_, p, m);
        buffer_size_ += m;
        p += m;
        n -= m;
        if (buffer_size_ < 64) return;
        transform(buffer_.data());
        buffer_size_ = 0;
    }
    const size_t whole = n / 64;
    enet::host::sha256_blocks(state_.data(), p, whole);
    p += 64 * whole;
    n -= 64 * whole;
    if (n) std::memcpy(buffer_.data(), p, n);
    buffer_size_ = n;
}

std::array<std::uint8_t, 32> Sha256::finalize() {  // Sha256.cpp:94-126 (resets the hasher)
    enet::host::Sha256State s;
    std::memcpy(s.h, state_.data(), 32);
    std::memcpy(s.buf, buffer_.data(), 64);
    s.fill = buffer_size_;
    s.bits = bit_len_;
    const auto d = enet::host::sha256_final(s);
    std::memcpy(state_.data(), enet::host::kIV, sizeof(enet::host::kIV));
    buffer_.fill(0);
    buffer_size_ = 0;
    bit_len_ = 0;
    scalar::host_call();
    return d;
}

std::array<std::uint8_t, 32> Sha256::digest(std::span<const std::uint8_t> data) {
    // one message = one serial chain: the host engine unless the caller forced the device
    if (scalar::device_for(data.size(), false)) {
        std::array<std::uint8_t, 32> d{};
        if (scalar::try_device("Sha256::digest", [&] { d = device_sha(data); })) return d;
    }
    scalar::host_call();
    return enet::host::sha256(data.data(), data.size());
}

// ------------------------------------------------------------------------------ HMAC
std::array<std::uint8_t, HmacSha256::kDigestSize> HmacSha256::compute(std::span<const std::uint8_t> key,
                                                                      std::span<const std::uint8_t> data) {
    if (scalar::device_for(data.size(), false)) {
        std::array<std::uint8_t, 32> m{};
        if (scalar::try_device("HmacSha256::compute", [&] { m = device_hmac(key, data); })) return m;
    }
    scalar::host_call();
    return enet::host::hmac_sha256(key.data(), key.size(), data.data(), data.size());
}

bool HmacSha256::verify(std::span<const std::uint8_t> key, std::span<const std::uint8_t> data,
                        std::span<const std::uint8_t> mac) {
    if (mac.size() != kDigestSize) return false;  // HmacSha256.cpp:44
    const auto expect = compute(key, data);
    std::uint8_t diff = 0;  // OR-accumulate, no early exit (HmacSha256.cpp:48-53)
    for (size_t i = 0; i < kDigestSize; ++i) diff |= static_cast<std::uint8_t>(expect[i] ^ mac[i]);
    return diff == 0;
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

namespace {
static_assert(sizeof(Key) == 32 && sizeof(Nonce) == 12 && sizeof(ChunkId) == 32,
              "crypto::Key / Nonce / ChunkId are passed to the device as packed arrays");
const std::uint8_t* key_bytes(std::span<const Key> k) { return reinterpret_cast<const std::uint8_t*>(k.data()); }
const std::uint8_t* nonce_bytes(std::span<const Nonce> n) { return reinterpret_cast<const std::uint8_t*>(n.data()); }

// One batch call through the host-memory runtime of the calling thread's device (host_batch.hpp):
// pinned, device-mapped staging, host worker threads gathering / scattering, chunks overlapped.
void run_host_batch(const enet::hb::Job& j) {
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    enet::hb::run_shared(dev, j);
}

enet::hb::Job job_of(enet::hb::Op op, std::span<const std::span<const std::uint8_t>> in) {
    enet::hb::Job j;
    j.op = op;
    j.n = in.size();
    j.in_spans = in;
    return j;
}

// contiguous output of a batch call: record i at offsets[i], the prefix sums of the op's lengths
std::vector<std::uint64_t> out_offsets_for(std::span<const std::span<const std::uint8_t>> in, std::int64_t delta,
                                           std::size_t out_size, const char* what) {
    auto off = offsets_of(in, delta);
    if (off.back() > out_size)
        throw std::invalid_argument(std::string("enet batch::") + what + ": output span too small");
    return off;
}
}  // namespace

std::vector<std::uint64_t> packed_offsets(std::span<const std::span<const std::uint8_t>> records,
                                          std::int64_t delta) {
    return offsets_of(records, delta);
}

void chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                    std::span<const std::span<const std::uint8_t>> inputs, std::span<const std::uint32_t> counters,
                    std::vector<std::vector<std::uint8_t>>& out) {
    const size_t n = inputs.size();
    if (keys.size() != n || nonces.size() != n || (!counters.empty() && counters.size() != n))
        throw std::invalid_argument("enet batch::chacha20_apply: size mismatch");
    out.resize(n);
    if (n == 0) return;
    auto j = job_of(enet::hb::Op::Xor, inputs);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.counters = counters.empty() ? nullptr : counters.data();
    j.out_vecs = &out;
    run_host_batch(j);
}

std::vector<std::vector<std::uint8_t>> chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                                                      std::span<const std::span<const std::uint8_t>> inputs,
                                                      std::span<const std::uint32_t> counters) {
    std::vector<std::vector<std::uint8_t>> res;
    chacha20_apply(keys, nonces, inputs, counters, res);
    return res;
}

void chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                    std::span<const std::span<const std::uint8_t>> inputs, std::span<const std::uint32_t> counters,
                    std::span<std::uint8_t> out) {
    const size_t n = inputs.size();
    if (keys.size() != n || nonces.size() != n || (!counters.empty() && counters.size() != n))
        throw std::invalid_argument("enet batch::chacha20_apply: size mismatch");
    if (n == 0) return;
    const auto off = out_offsets_for(inputs, 0, out.size(), "chacha20_apply");
    auto j = job_of(enet::hb::Op::Xor, inputs);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.counters = counters.empty() ? nullptr : counters.data();
    j.out_base = out.data();
    j.out_off = off.data();
    run_host_batch(j);
}

void aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> plaintexts, std::vector<Sealed>& out) {
    const size_t n = plaintexts.size();
    if (keys.size() != n || nonces.size() != n) throw std::invalid_argument("enet batch::aead_seal: size mismatch");
    out.resize(n);
    if (n == 0) return;
    std::vector<std::vector<std::uint8_t>*> each(n);
    for (size_t i = 0; i < n; ++i) each[i] = &out[i].data;
    std::vector<std::uint8_t> th(16 * n);
    auto j = job_of(enet::hb::Op::AeadSeal, plaintexts);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.out_each = each;
    j.tags_out = th.data();
    run_host_batch(j);
    for (size_t i = 0; i < n; ++i) std::memcpy(out[i].tag.data(), th.data() + 16 * i, 16);
}

std::vector<Sealed> aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
                              std::span<const std::span<const std::uint8_t>> plaintexts) {
    std::vector<Sealed> res;
    aead_seal(keys, nonces, plaintexts, res);
    return res;
}

void aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> plaintexts, std::span<std::uint8_t> out,
               std::span<std::array<std::uint8_t, 16>> tags) {
    const size_t n = plaintexts.size();
    if (keys.size() != n || nonces.size() != n || tags.size() != n)
        throw std::invalid_argument("enet batch::aead_seal: size mismatch");
    if (n == 0) return;
    const auto off = out_offsets_for(plaintexts, 0, out.size(), "aead_seal");
    auto j = job_of(enet::hb::Op::AeadSeal, plaintexts);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.out_base = out.data();
    j.out_off = off.data();
    j.tags_out = tags.data()->data();
    run_host_batch(j);
}

void aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> ciphertexts,
               std::span<const std::array<std::uint8_t, 16>> tags, std::vector<std::vector<std::uint8_t>>& out,
               std::vector<std::uint8_t>& ok) {
    const size_t n = ciphertexts.size();
    if (keys.size() != n || nonces.size() != n || tags.size() != n)
        throw std::invalid_argument("enet batch::aead_open: size mismatch");
    ok.assign(n, 0);
    out.resize(n);
    if (n == 0) return;
    auto j = job_of(enet::hb::Op::AeadOpen, ciphertexts);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.tags_in = tags.data()->data();
    j.ok_out = ok.data();
    j.out_vecs = &out;
    run_host_batch(j);
}

std::vector<std::vector<std::uint8_t>> aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
                                                 std::span<const std::span<const std::uint8_t>> ciphertexts,
                                                 std::span<const std::array<std::uint8_t, 16>> tags,
                                                 std::vector<std::uint8_t>& ok) {
    std::vector<std::vector<std::uint8_t>> res;
    aead_open(keys, nonces, ciphertexts, tags, res, ok);
    return res;
}

void aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> ciphertexts,
               std::span<const std::array<std::uint8_t, 16>> tags, std::span<std::uint8_t> out,
               std::span<std::uint8_t> ok) {
    const size_t n = ciphertexts.size();
    if (keys.size() != n || nonces.size() != n || tags.size() != n || ok.size() != n)
        throw std::invalid_argument("enet batch::aead_open: size mismatch");
    if (n == 0) return;
    const auto off = out_offsets_for(ciphertexts, 0, out.size(), "aead_open");
    auto j = job_of(enet::hb::Op::AeadOpen, ciphertexts);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.tags_in = tags.data()->data();
    j.ok_out = ok.data();
    j.out_base = out.data();
    j.out_off = off.data();
    run_host_batch(j);
}

std::vector<std::array<std::uint8_t, 32>> sha256(std::span<const std::span<const std::uint8_t>> messages) {
    const size_t n = messages.size();
    if (n == 0) return {};
    Staging& st = staging();
    st.reset();  // a previous call that threw may have left queued downloads
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
    std::vector<std::vector<std::uint8_t>> res;
    if (n == 0) return res;
    auto j = job_of(enet::hb::Op::FrameSeal, messages);
    j.keys = session_keys.data()->data();
    j.nonces = nonce_bytes(nonces);
    j.out_vecs = &res;
    run_host_batch(j);
    return res;
}

std::vector<std::vector<std::uint8_t>> frame_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                  std::span<const Nonce> nonces,
                                                  std::span<const std::span<const std::uint8_t>> bodies,
                                                  std::vector<std::uint8_t>& ok) {
    const size_t n = bodies.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::frame_open: size mismatch");
    ok.assign(n, 0);
    std::vector<std::vector<std::uint8_t>> res;
    if (n == 0) return res;
    auto j = job_of(enet::hb::Op::FrameOpen, bodies);
    j.keys = session_keys.data()->data();
    j.nonces = nonce_bytes(nonces);
    j.ok_out = ok.data();
    j.out_vecs = &res;
    run_host_batch(j);
    return res;
}

std::vector<StoredChunk> chunk_store(std::span<const Key> keys, std::span<const Nonce> nonces,
                                     std::span<const std::span<const std::uint8_t>> chunks,
                                     std::span<const ChunkId> chunk_ids) {
    const size_t n = chunks.size();
    if (keys.size() != n || nonces.size() != n || (!chunk_ids.empty() && chunk_ids.size() != n))
        throw std::invalid_argument("enet batch::chunk_store: size mismatch");
    if (n == 0) return {};
    std::vector<std::vector<std::uint8_t>> data;
    std::vector<std::uint8_t> hh(32 * n);
    auto j = job_of(enet::hb::Op::ChunkStore, chunks);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.ids = chunk_ids.empty() ? nullptr : chunk_ids.data()->data();
    j.macs_out = hh.data();
    j.out_vecs = &data;
    run_host_batch(j);
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
    std::vector<std::vector<std::uint8_t>> res;
    if (n == 0) return res;
    auto j = job_of(enet::hb::Op::ChunkFetch, ciphertexts);
    j.keys = key_bytes(keys);
    j.nonces = nonce_bytes(nonces);
    j.ids = chunk_ids.data()->data();
    j.macs_in = chunk_hashes.data()->data();
    j.ok_out = ok.data();
    j.out_vecs = &res;
    run_host_batch(j);
    return res;
}

void wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> messages, std::vector<std::vector<std::uint8_t>>& frames) {
    const size_t n = messages.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::wire_seal: size mismatch");
    frames.resize(n);
    if (n == 0) return;
    auto j = job_of(enet::hb::Op::WireSeal, messages);
    j.keys = session_keys.data()->data();
    j.nonces = nonce_bytes(nonces);
    j.out_vecs = &frames;
    run_host_batch(j);
}

std::vector<std::vector<std::uint8_t>> wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                 std::span<const Nonce> nonces,
                                                 std::span<const std::span<const std::uint8_t>> messages) {
    std::vector<std::vector<std::uint8_t>> res;
    wire_seal(session_keys, nonces, messages, res);
    return res;
}

void wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
               std::span<const std::span<const std::uint8_t>> messages, std::span<std::uint8_t> frames) {
    const size_t n = messages.size();
    if (session_keys.size() != n || nonces.size() != n)
        throw std::invalid_argument("enet batch::wire_seal: size mismatch");
    if (n == 0) return;
    const auto off = out_offsets_for(messages, 48, frames.size(), "wire_seal");
    auto j = job_of(enet::hb::Op::WireSeal, messages);
    j.keys = session_keys.data()->data();
    j.nonces = nonce_bytes(nonces);
    j.out_base = frames.data();
    j.out_off = off.data();
    run_host_batch(j);
}

void wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
               std::span<const std::span<const std::uint8_t>> frames, std::vector<std::vector<std::uint8_t>>& messages,
               std::vector<std::uint8_t>& ok) {
    const size_t n = frames.size();
    if (session_keys.size() != n) throw std::invalid_argument("enet batch::wire_open: size mismatch");
    ok.assign(n, 0);
    messages.resize(n);
    if (n == 0) return;
    auto j = job_of(enet::hb::Op::WireOpen, frames);
    j.keys = session_keys.data()->data();
    j.ok_out = ok.data();
    j.out_vecs = &messages;
    run_host_batch(j);
}

std::vector<std::vector<std::uint8_t>> wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                                                 std::span<const std::span<const std::uint8_t>> frames,
                                                 std::vector<std::uint8_t>& ok) {
    std::vector<std::vector<std::uint8_t>> res;
    wire_open(session_keys, frames, res, ok);
    return res;
}

void wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
               std::span<const std::span<const std::uint8_t>> frames, std::span<std::uint8_t> messages,
               std::span<std::uint8_t> ok) {
    const size_t n = frames.size();
    if (session_keys.size() != n || ok.size() != n) throw std::invalid_argument("enet batch::wire_open: size mismatch");
    if (n == 0) return;
    const auto off = out_offsets_for(frames, -48, messages.size(), "wire_open");
    auto j = job_of(enet::hb::Op::WireOpen, frames);
    j.keys = session_keys.data()->data();
    j.ok_out = ok.data();
    j.out_base = messages.data();
    j.out_off = off.data();
    run_host_batch(j);
}

namespace {
void check_sessions(std::span<const std::uint32_t> session, size_t K, const char* what) {
    for (std::uint32_t s : session)
        if (s >= K) throw std::invalid_argument(std::string("enet batch::") + what + ": session index outside the table");
}
}  // namespace

std::vector<std::vector<std::uint8_t>> wire_seal_sessions(std::span<const std::array<std::uint8_t, 32>> session_table,
                                                          std::span<const std::uint32_t> session,
                                                          std::span<const Nonce> nonces,
                                                          std::span<const std::span<const std::uint8_t>> messages) {
    const size_t n = messages.size(), K = session_table.size();
    if (session.size() != n || nonces.size() != n || K > 0xffffffffu)
        throw std::invalid_argument("enet batch::wire_seal_sessions: size mismatch");
    std::vector<std::vector<std::uint8_t>> res;
    if (n == 0) return res;
    check_sessions(session, K, "wire_seal_sessions");
    auto j = job_of(enet::hb::Op::WireSeal, messages);
    j.keys = session_table.data()->data();
    j.session = session.data();
    j.n_sessions = (std::uint32_t)K;
    j.nonces = nonce_bytes(nonces);
    j.out_vecs = &res;
    run_host_batch(j);
    return res;
}

std::vector<std::vector<std::uint8_t>> wire_open_sessions(std::span<const std::array<std::uint8_t, 32>> session_table,
                                                          std::span<const std::uint32_t> session,
                                                          std::span<const std::span<const std::uint8_t>> frames,
                                                          std::vector<std::uint8_t>& ok) {
    const size_t n = frames.size(), K = session_table.size();
    if (session.size() != n || K > 0xffffffffu)
        throw std::invalid_argument("enet batch::wire_open_sessions: size mismatch");
    ok.assign(n, 0);
    std::vector<std::vector<std::uint8_t>> res;
    if (n == 0) return res;
    check_sessions(session, K, "wire_open_sessions");
    auto j = job_of(enet::hb::Op::WireOpen, frames);
    j.keys = session_table.data()->data();
    j.session = session.data();
    j.n_sessions = (std::uint32_t)K;
    j.ok_out = ok.data();
    j.out_vecs = &res;
    run_host_batch(j);
    return res;
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
    st.reset();  // a previous call that threw may have left queued downloads
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
    st.reset();  // a previous call that threw may have left queued downloads
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
// Node.cpp:212-230 / 269-292 on the host engine: start = first mt19937_64 draw seeded by the
// big-endian first 8 digest bytes of nonce 0, candidates start + attempt
bool host_node_pow(const std::vector<std::uint8_t>& prefix, std::uint8_t difficulty, std::uint64_t max_attempts,
                   std::uint64_t& nonce_out) {
    enet::host::PowPrefix pp;
    enet::host::pow_prefix(pp, prefix.data(), prefix.size());
    const auto d0 = enet::host::pow_digest(pp, 0);
    std::uint64_t seed = 0;
    for (int i = 0; i < 8; ++i) seed = (seed << 8) | d0[i];
    std::mt19937_64 gen(seed);
    std::uniform_int_distribution<std::uint64_t> dist(0, std::numeric_limits<std::uint64_t>::max());
    const std::uint64_t start = dist(gen);
    for (std::uint64_t a = 0; a < max_attempts; ++a) {
        if (enet::host::leading_zero_bits(enet::host::pow_digest(pp, start + a)) >= difficulty) {
            nonce_out = start + a;
            return true;
        }
    }
    return false;
}

bool node_pow_one(const std::vector<std::uint8_t>& prefix, std::uint8_t difficulty, std::uint64_t& nonce_out) {
    if (difficulty == 0) {  // Node.cpp:213-216 / 274-277
        nonce_out = 0;
        return true;
    }
    // a search: the MI355X unless the caller chose the host (never throws: a reference drop-in)
    if (scalar::device_for(0, false) || scalar::g_policy.load() == ENET_SCALAR_AUTO) {
        PowResult r{};
        if (scalar::try_device("compute_*_pow", [&] {
                const std::span<const std::uint8_t> ps[1] = {prefix};
                const std::uint8_t d[1] = {difficulty};
                r = pow_search(ps, d, PowSchedule::Node, kNodePowAttempts)[0];
            })) {
            if (!r.found) return false;
            nonce_out = r.nonce;
            return true;
        }
    }
    scalar::host_call();
    return host_node_pow(prefix, difficulty, kNodePowAttempts, nonce_out);
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
    st.reset();  // a previous call that threw may have left queued downloads
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

ChunkId derive_chunk_id(std::span<const std::uint8_t> data) {  // StoreProof.cpp:75-78
    return crypto::Sha256::digest(data);
}

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

namespace {
// StoreProof.cpp:47-69 on the host engine
bool host_store_pow_valid(const StoreWorkInput& input, std::uint64_t nonce, std::uint8_t d) {
    const auto pre = store_pow_prefix(input);
    enet::host::PowPrefix pp;
    enet::host::pow_prefix(pp, pre.data(), pre.size());
    return enet::host::leading_zero_bits(enet::host::pow_digest(pp, nonce)) >= d;
}

// StoreProof.cpp:123-146 on the host engine: successive mt19937_64 outputs seeded by the
// native-endian (x86: little-endian) first 8 digest bytes of nonce 0
std::optional<std::uint64_t> host_store_pow(const StoreWorkInput& input, std::uint8_t d, std::uint64_t max_attempts) {
    const auto pre = store_pow_prefix(input);
    enet::host::PowPrefix pp;
    enet::host::pow_prefix(pp, pre.data(), pre.size());
    const auto d0 = enet::host::pow_digest(pp, 0);
    std::uint64_t seed = 0;
    std::memcpy(&seed, d0.data(), sizeof(seed));
    std::mt19937_64 rng(seed);
    for (std::uint64_t a = 0; a < max_attempts; ++a) {
        const std::uint64_t c = rng();
        if (enet::host::leading_zero_bits(enet::host::pow_digest(pp, c)) >= d) return c;
    }
    return std::nullopt;
}
}  // namespace

bool store_pow_valid(const StoreWorkInput& input, std::uint64_t nonce, std::uint8_t difficulty_bits) {
    if (difficulty_bits == 0) return true;  // StoreProof.cpp:112-113
    const std::uint8_t d = clamp_store_difficulty(difficulty_bits);
    if (scalar::device_for(0, false)) {  // one hash: the host engine unless forced
        std::uint8_t ok = 0;
        if (scalar::try_device("store_pow_valid", [&] {
                ok = batch::store_pow_valid(std::span(&input, 1), std::span(&nonce, 1), difficulty_bits)[0];
            }))
            return ok == 1;
    }
    scalar::host_call();
    return host_store_pow_valid(input, nonce, d);
}

std::optional<std::uint64_t> compute_store_pow(const StoreWorkInput& input, std::uint8_t difficulty_bits,
                                               std::uint64_t max_attempts) {
    if (difficulty_bits == 0) return std::uint64_t{0};  // StoreProof.cpp:125-127
    const std::uint8_t d = clamp_store_difficulty(difficulty_bits);
    if (max_attempts == 0) max_attempts = kDefaultStorePowMaxAttempts;  // :131-133
    if (scalar::g_policy.load() != ENET_SCALAR_HOST) {  // a search: the MI355X
        std::optional<std::uint64_t> r;
        if (scalar::try_device("compute_store_pow", [&] {
                r = batch::compute_store_pow(std::span(&input, 1), difficulty_bits, max_attempts)[0];
            }))
            return r;
    }
    scalar::host_call();
    return host_store_pow(input, d, max_attempts);
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
    // derive_key (KeyManager.cpp:74-92): HMAC(secret, BE64(counter) || BE64(ticks)) -- one HMAC,
    // so the host engine unless the caller forced the device (HmacSha256::compute routes it)
    std::array<std::uint8_t, 16> material{};
    const std::uint64_t ticks = static_cast<std::uint64_t>(ticks_of(now));
    for (int i = 0; i < 8; ++i) {
        material[i] = static_cast<std::uint8_t>(context.counter >> (56 - 8 * i));
        material[8 + i] = static_cast<std::uint8_t>(ticks >> (56 - 8 * i));
    }
    context.current_key = crypto::HmacSha256::compute(context.shared_secret.bytes, material);
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
    // many sessions: one device batch; a failed device call is finished on the host engine
    std::vector<std::array<std::uint8_t, 32>> keys;
    if (!(scalar::g_policy.load() != ENET_SCALAR_HOST &&
          scalar::try_device("KeyManager::rotate_all_due",
                             [&] { keys = crypto::batch::session_keys(secrets, counters, ticks); }))) {
        scalar::host_call();
        keys.resize(due.size());
        for (size_t i = 0; i < due.size(); ++i) {
            std::array<std::uint8_t, 16> m{};
            for (int b = 0; b < 8; ++b) {
                m[b] = static_cast<std::uint8_t>(counters[i] >> (56 - 8 * b));
                m[8 + b] = static_cast<std::uint8_t>(static_cast<std::uint64_t>(ticks[i]) >> (56 - 8 * b));
            }
            keys[i] = enet::host::hmac_sha256(secrets[i].bytes.data(), 32, m.data(), m.size());
        }
    }
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
