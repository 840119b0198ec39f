// scalar_latency.cpp -- per-call latency of the reference's scalar crypto API.
//
// One source, two builds (oracle/Makefile target `latency`):
//   oracle/_ref/scalar_latency_gpu : include/ + libenet_crypto.so (every call is a GPU round trip)
//   oracle/_ref/scalar_latency_ref : /root/reference/include + oracle/_ref/libenet_ref.so (the
//                                    reference's own CPU code, compiled from its sources)
// The call shapes are the reference's hot scalar call sites: Message.cpp:305-328 HMAC over a
// small signed message (98 B is an Acknowledge frame), SessionManager.cpp:374 ChaCha20::apply on
// a 1500 B frame, KeyExchange.cpp:44 Sha256::digest of 4 B, CryptoManager encrypt of a 4 KiB and
// 64 KiB chunk, and the Node.cpp:269-292 handshake PoW written as the reference writes it (one
// Sha256 per attempt).  With ENET_BATCH the drop-in crypto::batch::compute_handshake_pow (one device
// search) is timed beside it.  Output: one JSON line per case, median and mean microseconds.
//
// usage: scalar_latency [reps] [policy auto|device|host (drop-in build only)] [threads] [qthreads]
// After the single-thread latencies, `threads` threads call the same API concurrently for ~1 s
// per case (the reference's per-session reader threads, SessionManager.cpp:332,703) and the
// aggregate calls/s and GB/s are printed ("mt_*" cases).
#include "ephemeralnet/crypto/ChaCha20.hpp"
#include "ephemeralnet/crypto/CryptoManager.hpp"
#include "ephemeralnet/crypto/HmacSha256.hpp"
#include "ephemeralnet/crypto/Sha256.hpp"
#ifdef ENET_BATCH
#include "ephemeralnet/crypto/Batch.hpp"
#include "enet_crypto.h"
#endif

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <span>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;
std::uint64_t g_sink = 0;  // printed to stderr at exit so no call is elided

void run(const char* name, std::size_t bytes, int reps, const std::function<void()>& f) {
    for (int i = 0; i < std::max(3, reps / 10); ++i) f();
    std::vector<double> us(reps);
    for (int i = 0; i < reps; ++i) {
        const auto t0 = Clock::now();
        f();
        us[i] = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
    }
    double sum = 0;
    for (double u : us) sum += u;
    std::sort(us.begin(), us.end());
    std::printf("{\"case\": \"%s\", \"bytes\": %zu, \"reps\": %d, \"median_us\": %.2f, \"mean_us\": %.2f, "
                "\"p10_us\": %.2f, \"p90_us\": %.2f}\n",
                name, bytes, reps, us[reps / 2], sum / reps, us[reps / 10], us[(reps * 9) / 10]);
    std::fflush(stdout);
}

// `threads` threads call f(thread) back to back for ~secs; aggregate rate
void run_mt(const char* name, std::size_t bytes, int threads, double secs,
            const std::function<void(int, std::vector<std::uint8_t>&)>& f) {
    std::atomic<bool> go{false}, stop{false};
    std::vector<std::uint64_t> calls(threads, 0);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
            std::vector<std::uint8_t> out;
            while (!go.load()) std::this_thread::yield();
            std::uint64_t c = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                f(t, out);
                ++c;
            }
            calls[t] = c;
        });
    const auto t0 = Clock::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    stop = true;
    for (auto& th : ts) th.join();
    const double el = std::chrono::duration<double>(Clock::now() - t0).count();
    std::uint64_t total = 0;
    for (auto c : calls) total += c;
    std::printf("{\"case\": \"mt_%s\", \"bytes\": %zu, \"threads\": %d, \"calls_per_s\": %.0f, "
                "\"GB_per_s\": %.4f}\n",
                name, bytes, threads, total / el, total * (double)bytes / el / 1e9);
    std::fflush(stdout);
}

std::vector<std::uint8_t> pattern(std::size_t n, std::uint8_t s) {
    std::vector<std::uint8_t> v(n);
    for (std::size_t i = 0; i < n; ++i) v[i] = static_cast<std::uint8_t>(s + 31 * i + (i >> 7));
    return v;
}

// Node.cpp:232-245 / 269-292, as written there: a fresh Sha256 per attempt
std::array<std::uint8_t, 8> be64(std::uint64_t x) {
    std::array<std::uint8_t, 8> b{};
    for (int i = 0; i < 8; ++i) b[i] = static_cast<std::uint8_t>(x >> (56 - 8 * i));
    return b;
}
int lz_bits(const std::array<std::uint8_t, 32>& d) {
    int t = 0;
    for (auto b : d) {
        if (b == 0) { t += 8; continue; }
        for (int k = 7; k >= 0; --k) { if ((b >> k) & 1) return t; ++t; }
    }
    return t;
}
std::uint64_t host_loop_pow(const std::array<std::uint8_t, 32>& a, const std::array<std::uint8_t, 32>& b,
                            std::uint32_t pub, int difficulty, std::uint64_t start, std::uint64_t* attempts) {
    for (std::uint64_t at = 0; at < 500000; ++at) {
        ephemeralnet::crypto::Sha256 h;
        h.update(be64(32));
        h.update(a);
        h.update(be64(32));
        h.update(b);
        h.update(be64(pub));
        h.update(be64(start + at));
        if (lz_bits(h.finalize()) >= difficulty) {
            *attempts = at + 1;
            return start + at;
        }
    }
    *attempts = 500000;
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    using namespace ephemeralnet::crypto;
    const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
    const std::string policy = argc > 2 ? argv[2] : "auto";
    const int threads = argc > 3 ? std::atoi(argv[3]) : 16;
#ifdef ENET_BATCH
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    std::printf("{\"case\": \"config\", \"build\": \"dropin\", \"policy\": \"%s\", \"host_isa\": \"%s\"}\n",
                policy.c_str(), enet_host_isa());
#else
    std::printf("{\"case\": \"config\", \"build\": \"reference\"}\n");
#endif
    Key key{};
    for (int i = 0; i < 32; ++i) key.bytes[i] = static_cast<std::uint8_t>(i * 5 + 1);
    Nonce nonce{};
    for (int i = 0; i < 12; ++i) nonce.bytes[i] = static_cast<std::uint8_t>(i + 9);
    const auto m98 = pattern(98, 1), f1500 = pattern(1500, 2), c4k = pattern(4096, 3), c64k = pattern(65536, 4);
    const auto mac = HmacSha256::compute(key.bytes, m98);
    std::vector<std::uint8_t> out;
    std::array<std::uint8_t, 32> cid{};
    cid[0] = 7;

    run("hmac_compute", 98, reps, [&] { g_sink += HmacSha256::compute(key.bytes, m98)[0]; });
    run("hmac_verify", 98, reps, [&] { g_sink += HmacSha256::verify(key.bytes, m98, mac); });
    run("chacha20_apply", 1500, reps, [&] { ChaCha20::apply(key, nonce, f1500, out, 0); g_sink += out[0]; });
    run("chacha20_apply", 65536, reps, [&] { ChaCha20::apply(key, nonce, c64k, out, 0); g_sink += out[0]; });
    const std::array<std::uint8_t, 4> four{1, 2, 3, 4};
    run("sha256_digest", 4, reps, [&] { g_sink += Sha256::digest(four)[0]; });
    run("sha256_digest", 65536, reps, [&] { g_sink += Sha256::digest(c64k)[0]; });
    run("cm_encrypt_with_key", 4096, reps,
        [&] { g_sink += CryptoManager::encrypt_with_key(key, cid, c4k).data.size(); });
    run("cm_encrypt_with_key", 65536, reps,
        [&] { g_sink += CryptoManager::encrypt_with_key(key, cid, c64k).data.size(); });
    const auto c1m = pattern(1u << 20, 5), c8m = pattern(8u << 20, 6);
    // the size sweep that places the AUTO crossover (host engine vs coalesced device path)
    for (std::size_t sz : {std::size_t(128) << 10, std::size_t(256) << 10, std::size_t(512) << 10,
                           std::size_t(1) << 20, std::size_t(2) << 20, std::size_t(4) << 20,
                           std::size_t(8) << 20, std::size_t(32) << 20}) {
        const std::vector<std::uint8_t> buf(c8m.begin(), c8m.begin() + std::min(sz, c8m.size()));
        const auto big = sz > c8m.size() ? pattern(sz, 7) : buf;
        run("chacha20_apply", sz, sz >= (8u << 20) ? 5 : std::max(10, reps / 10),
            [&] { ChaCha20::apply(key, nonce, big, out, 0); g_sink += out[0]; });
    }
    run("sha256_digest", 1u << 20, std::max(10, reps / 10), [&] { g_sink += Sha256::digest(c1m)[0]; });

    // many session threads at once
    if (threads > 0) {
        run_mt("hmac_compute", 98, threads, 1.0, [&](int, std::vector<std::uint8_t>&) {
            g_sink += HmacSha256::compute(key.bytes, m98)[0]; });
        run_mt("chacha20_apply", 1500, threads, 1.0, [&](int, std::vector<std::uint8_t>& o) {
            ChaCha20::apply(key, nonce, f1500, o, 0); g_sink += o[0]; });
        run_mt("chacha20_apply", 65536, threads, 1.0, [&](int, std::vector<std::uint8_t>& o) {
            ChaCha20::apply(key, nonce, c64k, o, 0); g_sink += o[0]; });
        run_mt("chacha20_apply", 1u << 20, threads, 1.5, [&](int, std::vector<std::uint8_t>& o) {
            ChaCha20::apply(key, nonce, c1m, o, 0); g_sink += o[0]; });
        run_mt("sha256_digest", 65536, threads, 1.0, [&](int, std::vector<std::uint8_t>&) {
            g_sink += Sha256::digest(c64k)[0]; });
    }

    // Session frames: SessionManager::send seals a 1500-byte message on the
    // caller's thread as HMAC + ChaCha20 over message || MAC (SessionManager.cpp:362-374,
    // Message.cpp:305-311), and receive_loop opens it with ChaCha20 + HmacSha256::verify
    // (:815-822, Message.cpp:313-328); one key per session thread.  Per-call: those reference
    // calls on every thread (the drop-in build serves them on its host engine).  Queue (drop-in
    // build): every thread hands its frame to one shared FrameQueue / FrameReceiveQueue, which
    // seals / opens a whole flush in one MI355X pass (policy device / auto) or on the host engine
    // (policy host).  `qthreads` session threads (argv[4], default 256: a relay serves hundreds).
    const int qthreads = argc > 4 ? std::atoi(argv[4]) : 256;
    for (int nt : {threads, qthreads}) {
        if (nt <= 0) continue;
        std::vector<Key> keys(nt);
        for (int t = 0; t < nt; ++t)
            for (int i = 0; i < 32; ++i) keys[t].bytes[i] = static_cast<std::uint8_t>(i * 7 + t);
        // as SessionManager::send is written: a fresh std::random_device per frame, one draw per
        // nonce byte (:365-371), then HMAC and ChaCha20 over message || MAC
        run_mt("frame_seal_percall", 1500, nt, 1.0, [&](int t, std::vector<std::uint8_t>& o) {
            Nonce fn{};
            {
                std::random_device rd;
                for (auto& b : fn.bytes) b = static_cast<std::uint8_t>(rd());
            }
            g_sink += fn.bytes[0];
            const auto m = HmacSha256::compute(keys[t].bytes, f1500);
            std::vector<std::uint8_t> sig(f1500);
            sig.insert(sig.end(), m.begin(), m.end());
            ChaCha20::apply(keys[t], fn, sig, o, 0);
            g_sink += o[0]; });
        std::vector<std::vector<std::uint8_t>> bodies(nt);
        for (int t = 0; t < nt; ++t) {
            const auto m = HmacSha256::compute(keys[t].bytes, f1500);
            std::vector<std::uint8_t> sig(f1500);
            sig.insert(sig.end(), m.begin(), m.end());
            ChaCha20::apply(keys[t], nonce, sig, bodies[t], 0);
        }
        run_mt("frame_open_percall", 1500, nt, 1.0, [&](int t, std::vector<std::uint8_t>& o) {
            ChaCha20::apply(keys[t], nonce, bodies[t], o, 0);
            const std::span<const std::uint8_t> msg(o.data(), o.size() - 32), tag(o.data() + o.size() - 32, 32);
            g_sink += HmacSha256::verify(keys[t].bytes, msg, tag); });
#ifdef ENET_BATCH
        batch::FrameQueue tx;
        batch::FrameReceiveQueue rx;
        std::vector<std::array<std::uint8_t, 32>> sk(nt);
        for (int t = 0; t < nt; ++t) std::copy(keys[t].bytes.begin(), keys[t].bytes.end(), sk[t].begin());
        run_mt("frame_queue_seal", 1500, nt, 1.5, [&](int t, std::vector<std::uint8_t>&) {
            g_sink += tx.seal(sk[t], f1500)->size(); });
        std::vector<std::vector<std::uint8_t>> wire(nt);
        for (int t = 0; t < nt; ++t) wire[t] = *tx.seal(sk[t], f1500);
        run_mt("frame_queue_open", 1500, nt, 1.5, [&](int t, std::vector<std::uint8_t>&) {
            g_sink += rx.open(sk[t], wire[t])->size(); });
        const auto ts = tx.stats(), rs = rx.stats();
        std::printf("{\"case\": \"frame_queue_stats\", \"threads\": %d, \"tx_frames\": %llu, \"tx_flushes\": %llu, "
                    "\"tx_host_flushes\": %llu, \"rx_frames\": %llu, \"rx_flushes\": %llu, \"rx_host_flushes\": %llu}\n",
                    nt, (unsigned long long)ts.frames, (unsigned long long)ts.flushes,
                    (unsigned long long)ts.host_flushes, (unsigned long long)rs.frames,
                    (unsigned long long)rs.flushes, (unsigned long long)rs.host_flushes);
        std::fflush(stdout);
#endif
    }

    // handshake PoW at difficulty 8 (about 256 attempts expected), 5 different peers
    std::array<std::uint8_t, 32> pa{}, pb{};
    for (int d : {8, 12}) {
        for (int i = 0; i < 3; ++i) {
            pa[0] = static_cast<std::uint8_t>(i + 1);
            pb[1] = static_cast<std::uint8_t>(d);
            std::uint64_t att = 0;
            const auto t0 = Clock::now();
            const auto n = host_loop_pow(pa, pb, 77u + i, d, 1000003u * i, &att);
            const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
            std::printf("{\"case\": \"handshake_pow_host_loop\", \"difficulty\": %d, \"attempts\": %llu, "
                        "\"us\": %.1f, \"us_per_attempt\": %.3f, \"nonce\": %llu}\n",
                        d, (unsigned long long)att, us, us / att, (unsigned long long)n);
#ifdef ENET_BATCH
            std::uint64_t dn = 0;
            const auto t1 = Clock::now();
            const bool ok = batch::compute_handshake_pow(pa, pb, 77u + i, static_cast<std::uint8_t>(d), dn);
            const double us1 = std::chrono::duration<double, std::micro>(Clock::now() - t1).count();
            std::printf("{\"case\": \"handshake_pow_batch_dropin\", \"difficulty\": %d, \"found\": %d, "
                        "\"us\": %.1f}\n", d, ok ? 1 : 0, us1);
#endif
            std::fflush(stdout);
        }
    }
    std::fprintf(stderr, "sink %llu\n", (unsigned long long)g_sink);
    return 0;
}
