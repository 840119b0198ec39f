// chunk_hybrid.cpp -- SHA-256 of long chunks on host threads while the MI355X does their cipher.
//
// A stored file is ONE chunk of up to 32 MiB (include/ephemeralnet/Config.hpp:62, src/main.cpp:4467);
// the node hashes it whole (chunk id, src/core/Node.cpp:1414; StoreProof.cpp:75-78) and checks the
// hash of the decrypted chunk on fetch (Node.cpp:1644-1655).  SHA-256 of one message is one serial
// chain: on a GPU lane it runs at ~34 MB/s (the 64 KiB duplex chain: 1.90 ms), so one 32 MiB chunk
// held the whole batch for ~1 s, while one SHA-NI core hashes it in ~16 ms (2.1 GB/s,
// INTEGRATION.md scalar table: 490 us per MiB).  The cipher of a long chunk is sequence-parallel
// (segments.hip tiles over every CU), so the split is: device = ChaCha20, host = the hash chain.
//
// host_hash_records() hashes a subset of a batch's records.  Records in device memory are copied
// down in pieces through a per-worker pinned double buffer on the worker's own stream (piece k+1
// in flight while piece k is hashed); records in host memory the device maps (hipHostMalloc'ed /
// registered: the host-batch runtime's staging) are hashed in place.  One worker thread per record
// up to the process's CPU budget; the calling thread is worker 0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "host_engine.hpp"

namespace enet {

namespace {

constexpr size_t kPiece = 4u << 20;  // D2H piece: large enough for full-rate SDMA, two per worker

struct Worker {
    int dev = -1;
    hipStream_t s = nullptr;
    uint8_t* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
};

std::mutex g_mu;
std::vector<Worker*> g_free;  // idle workers (any device; matched on checkout)

Worker* checkout(int dev, std::string& err) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (size_t i = 0; i < g_free.size(); ++i) {
            if (g_free[i]->dev == dev) {
                Worker* w = g_free[i];
                g_free.erase(g_free.begin() + (long)i);
                return w;
            }
        }
    }
    auto* w = new Worker;
    w->dev = dev;
    if (hipStreamCreateWithFlags(&w->s, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&w->buf[0]), kPiece, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&w->buf[1]), kPiece, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&w->ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->ev[1], hipEventDisableTiming) != hipSuccess) {
        err = "host hash worker: stream / pinned buffer / event creation failed";
        return nullptr;  // the partial worker leaks: a failing HIP runtime is not recovered here
    }
    return w;
}

void checkin(Worker* w) {
    std::lock_guard<std::mutex> lk(g_mu);
    g_free.push_back(w);
}

// SHA-256 of [p, p + n) in device memory through the worker's double buffer
bool hash_device(Worker* w, const uint8_t* p, uint64_t n, uint8_t out[32]) {
    host::Sha256State st;
    host::sha256_init(st);
    const uint64_t pieces = (n + kPiece - 1) / kPiece;
    auto issue = [&](uint64_t k) {
        const uint64_t len = std::min<uint64_t>(kPiece, n - k * kPiece);
        return hipMemcpyAsync(w->buf[k & 1], p + k * kPiece, len, hipMemcpyDeviceToHost, w->s) == hipSuccess &&
               hipEventRecord(w->ev[k & 1], w->s) == hipSuccess;
    };
    if (pieces && !issue(0)) return false;
    for (uint64_t k = 0; k < pieces; ++k) {
        if (k + 1 < pieces && !issue(k + 1)) return false;  // flies while piece k is hashed
        if (hipEventSynchronize(w->ev[k & 1]) != hipSuccess) return false;
        host::sha256_update(st, w->buf[k & 1], std::min<uint64_t>(kPiece, n - k * kPiece));
        // slot k & 1 is reused by piece k + 2, issued after this update returns
    }
    const auto d = host::sha256_final(st);
    std::memcpy(out, d.data(), 32);
    return true;
}

}  // namespace

// digests[32 k ..] = SHA-256(base[off[list[k]] .. off[list[k] + 1])) for k < m.  `off` is a host
// copy of the batch's offsets.  `ready` (nullable) is an event on the producing stream the copies
// wait for.  threads = the most host threads to use (>= 1).
int host_hash_records(const uint8_t* base, const uint64_t* off, const uint32_t* list, uint32_t m,
                      hipEvent_t ready, uint32_t threads, uint8_t* digests, std::string& err) {
    if (m == 0) return 0;
    // host memory the device maps (the host-batch runtime's staging, enet_host_alloc, registered
    // ranges): hash it where it is
    const uint8_t* host_base = nullptr;
    {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, base) == hipSuccess && a.type == hipMemoryTypeHost && a.hostPointer)
            host_base = static_cast<const uint8_t*>(a.hostPointer) +
                        (base - static_cast<const uint8_t*>(a.devicePointer ? a.devicePointer : a.hostPointer));
        (void)hipGetLastError();  // an unregistered pointer leaves an error behind
    }
    // host memory is read by the CPU directly: the producing stream's work must be done first
    if (host_base && ready && hipEventSynchronize(ready) != hipSuccess) {
        err = "host hash: hipEventSynchronize failed";
        return -1;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        err = "host hash: hipGetDevice failed";
        return -1;
    }
    const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(threads, m));
    std::atomic<uint32_t> next{0};
    std::atomic<bool> failed{false};
    std::vector<std::string> errs(T);
    auto run = [&](uint32_t t) {
        Worker* w = nullptr;
        if (!host_base) {
            if (hipSetDevice(dev) != hipSuccess || !(w = checkout(dev, errs[t]))) {
                failed = true;
                return;
            }
            if (ready && hipStreamWaitEvent(w->s, ready, 0) != hipSuccess) {
                errs[t] = "host hash: hipStreamWaitEvent failed";
                failed = true;
            }
        }
        for (uint32_t k; !failed && (k = next.fetch_add(1)) < m;) {
            const uint32_t rec = list[k];
            const uint64_t a = off[rec], n = off[rec + 1] - a;
            if (host_base) {
                const auto d = host::sha256(host_base + a, n);
                std::memcpy(digests + 32ull * k, d.data(), 32);
            } else if (!hash_device(w, base + a, n, digests + 32ull * k)) {
                errs[t] = "host hash: device-to-host copy failed";
                failed = true;
            }
        }
        if (w) checkin(w);
    };
    std::vector<std::thread> pool;
    pool.reserve(T - 1);
    for (uint32_t t = 1; t < T; ++t) {
        try {
            pool.emplace_back(run, t);
        } catch (const std::system_error&) {
            break;  // fewer threads: the started ones and this one take the rest of the list
        }
    }
    run(0);
    for (auto& th : pool) th.join();
    if (failed) {
        for (auto& e : errs)
            if (!e.empty()) {
                err = e;
                break;
            }
        if (err.empty()) err = "host hash failed";
        return -1;
    }
    return 0;
}

}  // namespace enet
