// queue_stress.cpp -- many session threads through the cross-session frame queues at once
// (crypto::batch::FrameQueue / FrameReceiveQueue).
//
// usage: queue_stress <policy auto|device|host> <threads> <frames per thread> <seed>
//        queue_stress nonces <policy> <threads> <frames per thread>: every thread seals that many
//        empty messages under ONE shared key; prints how many of the nonces were distinct
// Phase 1: every thread seals its own session's messages (lengths 0..3000, some 64 KiB, one
// frame of the 1 MiB maximum payload per run) through ONE shared FrameQueue.  Phase 2: every
// thread opens its own frames through ONE shared FrameReceiveQueue, with every 7th frame
// tampered (nonce, length field, body or MAC byte) and every 11th opened under the NEXT thread's
// session key.  Each thread checks that exactly the untouched frames come back, byte-equal to its
// own messages.  Prints a sample of (key, message, frame) lines for the oracle check in
// tests/test_frame_queue.py and a summary line.
#include <algorithm>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <string>
#include <span>
#include <thread>
#include <vector>

#include "enet_crypto.h"
#include "ephemeralnet/crypto/Batch.hpp"

using namespace ephemeralnet::crypto;
using namespace ephemeralnet::crypto::batch;

namespace {

std::uint64_t splitmix(std::uint64_t& s) {
    std::uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

std::string hex(const std::vector<std::uint8_t>& v) {
    static const char* d = "0123456789abcdef";
    std::string s;
    for (auto b : v) {
        s += d[b >> 4];
        s += d[b & 15];
    }
    return s.empty() ? "-" : s;
}

// Every sealed frame against the host engine's bytes for the same key, message and nonce (the
// nonce from the frame's header): header nonce(12) || BE32(|m| + 32), body = the host engine's
// seal_body (SessionManager.cpp:362-387, Message.cpp:305-311).  The host engine is itself pinned
// to the oracle (tests/test_host_engine.py).  Returns true when the frame differs.
bool frame_mismatch(const std::array<std::uint8_t, 32>& key, const std::vector<std::uint8_t>& m,
                    const std::vector<std::uint8_t>& f) {
    if (f.size() != m.size() + 48) return true;
    std::vector<std::uint8_t> body(m.size() + 32);
    enet_host_seal_body(key.data(), f.data(), m.data(), m.size(), body.data());
    const std::uint32_t len = (std::uint32_t)f[12] << 24 | (std::uint32_t)f[13] << 16 | (std::uint32_t)f[14] << 8 | f[15];
    return len != m.size() + 32 || !std::equal(body.begin(), body.end(), f.begin() + 16);
}

}  // namespace

int nonce_uniqueness(const std::string& policy, int T, int F) {
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    FrameQueue tx;
    std::array<std::uint8_t, 32> key{};
    key[0] = 1;
    std::vector<std::vector<std::array<std::uint8_t, 12>>> got(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            got[t].reserve(F);
            for (int i = 0; i < F; ++i) {
                const auto f = tx.seal(key, {});
                std::array<std::uint8_t, 12> n{};
                std::copy(f->begin(), f->begin() + 12, n.begin());
                got[t].push_back(n);
            }
        });
    for (auto& x : th) x.join();
    std::vector<std::array<std::uint8_t, 12>> all;
    for (auto& g : got) all.insert(all.end(), g.begin(), g.end());
    std::sort(all.begin(), all.end());
    const auto distinct = std::unique(all.begin(), all.end()) - all.begin();
    std::printf("nonces total=%zu distinct=%td\n", all.size(), distinct);
    return distinct == (std::ptrdiff_t)all.size() ? 0 : 1;
}

// async <policy> <threads> <frames>: every thread submits ALL its frames with seal_async before
// waiting for any (then the same with open_async, every 5th frame tampered), so a device pass can
// carry frames of many threads and many frames of one thread.  Prints a summary line.
int async_mode(const std::string& policy, int T, int F) {
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    FrameQueue tx;
    FrameReceiveQueue rx;
    std::atomic<int> bad{0}, opened{0}, rejected{0}, mismatch{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::uint64_t s = 77 + (std::uint64_t)t;
            std::array<std::uint8_t, 32> key{};
            for (auto& b : key) b = (std::uint8_t)splitmix(s);
            std::vector<std::vector<std::uint8_t>> msgs(F);
            for (auto& m : msgs) {
                m.resize(splitmix(s) % 2049);
                for (auto& b : m) b = (std::uint8_t)splitmix(s);
            }
            std::vector<std::future<std::optional<std::vector<std::uint8_t>>>> fs;
            for (auto& m : msgs) fs.push_back(tx.seal_async(key, m));
            std::vector<std::vector<std::uint8_t>> frames(F);
            for (int i = 0; i < F; ++i) {
                auto f = fs[i].get();
                if (!f || f->size() != msgs[i].size() + 48) { ++bad; continue; }
                if (frame_mismatch(key, msgs[i], *f)) ++mismatch;
                frames[i] = std::move(*f);
            }
            fs.clear();
            for (int i = 0; i < F; ++i) {
                auto f = frames[i];
                if (i % 5 == 2 && f.size() > 20) f[20] ^= 0x08;  // body byte
                fs.push_back(rx.open_async(key, std::move(f)));
            }
            for (int i = 0; i < F; ++i) {
                auto m = fs[i].get();
                const bool expect = !(i % 5 == 2 && frames[i].size() > 20);
                if (m) ++opened;
                else ++rejected;
                if ((bool)m != expect || (m && *m != msgs[i])) ++bad;
            }
        });
    for (auto& x : th) x.join();
    const auto st = tx.stats(), sr = rx.stats();
    std::printf("summary bad=%d mismatch=%d opened=%d rejected=%d tx_frames=%llu tx_flushes=%llu tx_host_flushes=%llu "
                "rx_frames=%llu rx_flushes=%llu rx_host_flushes=%llu\n",
                bad.load(), mismatch.load(), opened.load(), rejected.load(), (unsigned long long)st.frames,
                (unsigned long long)st.flushes, (unsigned long long)st.host_flushes, (unsigned long long)sr.frames,
                (unsigned long long)sr.flushes, (unsigned long long)sr.host_flushes);
    return (bad || mismatch) ? 1 : 0;
}

// window <policy> <threads> <window> <frames>: every thread keeps `window` frames in flight with
// submit() / FrameTicket::get(), get(out) or view() (a relay draining its socket buffers), MTU-sized and ragged
// messages, then opens them the same way (every 9th frame tampered, every 13th under the next
// thread's key).  Every sealed frame is checked independently on the host engine (the nonce from
// its header, body = ChaCha20_{K,N,0}(m || HMAC_K(m)); SessionManager.cpp:362-387).  The summary
// carries frames per pass, the batching the device queue reaches at this load.
int window_mode(const std::string& policy, int T, int W, int F) {
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    // QUEUE_STRESS_MAX_FRAMES: small passes that fill (and overflow) at once
    FrameQueueOptions opt;
    if (const char* e = std::getenv("QUEUE_STRESS_MAX_FRAMES")) opt.max_frames = (std::size_t)std::atoll(e);
    FrameQueue tx(opt);
    FrameReceiveQueue rx(opt);
    std::vector<std::array<std::uint8_t, 32>> keys(T);
    for (int t = 0; t < T; ++t) {
        std::uint64_t s = 1234 + (std::uint64_t)t;
        for (auto& b : keys[t]) b = (std::uint8_t)splitmix(s);
    }
    std::atomic<int> bad{0}, opened{0}, rejected{0}, mismatch{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::uint64_t s = 991 + (std::uint64_t)t;
            std::vector<std::vector<std::uint8_t>> msgs(F), frames(F);
            for (int i = 0; i < F; ++i) {
                msgs[i].resize(i % 3 ? 1500 : splitmix(s) % 1700);
                for (auto& b : msgs[i]) b = (std::uint8_t)splitmix(s);
            }
            std::deque<std::pair<int, FrameTicket>> q;
            // frames collected three ways: get(), get(out) into one reused vector (its capacity
            // kept), and a zero-copy view() of the result read in place, then release()
            std::vector<std::uint8_t> reuse;
            auto collect = [&](int i, FrameTicket& tk) -> std::optional<std::vector<std::uint8_t>> {
                if (i % 3 == 0) return tk.get();
                if (i % 3 == 2) {
                    std::span<const std::uint8_t> v;
                    const bool ok = tk.view(v);
                    std::optional<std::vector<std::uint8_t>> r;
                    if (ok) r.emplace(v.begin(), v.end());
                    else if (!v.empty()) ++bad;
                    tk.release();
                    if (tk.valid()) ++bad;
                    return r;
                }
                if (!tk.get(reuse)) {
                    if (!reuse.empty()) ++bad;
                    return std::nullopt;
                }
                return reuse;
            };
            auto seal_one = [&](int i, std::optional<std::vector<std::uint8_t>> f) {
                const auto& m = msgs[i];
                if (!f || f->size() != m.size() + 48) {
                    ++bad;
                    return;
                }
                std::vector<std::uint8_t> body(f->begin() + 16, f->end());
                enet_host_chacha20_xor(keys[t].data(), f->data(), 0, body.data(), body.data(), body.size());
                std::uint8_t mac[32];
                enet_host_hmac_sha256(keys[t].data(), 32, m.data(), m.size(), mac);
                const std::uint32_t len = (std::uint32_t)(*f)[12] << 24 | (std::uint32_t)(*f)[13] << 16 |
                                          (std::uint32_t)(*f)[14] << 8 | (*f)[15];
                if (len != m.size() + 32 || !std::equal(m.begin(), m.end(), body.begin()) ||
                    !std::equal(mac, mac + 32, body.begin() + (std::ptrdiff_t)m.size()))
                    ++bad;
                if (frame_mismatch(keys[t], m, *f)) ++mismatch;
                frames[i] = std::move(*f);
            };
            for (int i = 0; i < F; ++i) {
                q.emplace_back(i, tx.submit(keys[t], msgs[i]));
                if ((int)q.size() >= W) {
                    seal_one(q.front().first, collect(q.front().first, q.front().second));
                    q.pop_front();
                }
            }
            for (; !q.empty(); q.pop_front()) seal_one(q.front().first, collect(q.front().first, q.front().second));
            auto open_one = [&](int i, std::optional<std::vector<std::uint8_t>> m) {
                const bool expect = !(i % 9 == 4) && !(i % 13 == 6 && T > 1);
                if (m) ++opened;
                else ++rejected;
                if ((bool)m != expect || (m && *m != msgs[i])) ++bad;
            };
            for (int i = 0; i < F; ++i) {
                auto f = frames[i];
                if (f.empty()) continue;
                auto key = keys[t];
                if (i % 9 == 4) f[16 + (i % (f.size() - 16))] ^= 0x01;  // body or MAC byte
                else if (i % 13 == 6) key = keys[(t + 1) % T];
                q.emplace_back(i, rx.submit(key, f));
                if ((int)q.size() >= W) {
                    open_one(q.front().first, collect(q.front().first, q.front().second));
                    q.pop_front();
                }
            }
            for (; !q.empty(); q.pop_front()) open_one(q.front().first, collect(q.front().first, q.front().second));
        });
    for (auto& x : th) x.join();
    const auto st = tx.stats(), sr = rx.stats();
    enet_scalar_stats ss{};
    enet_scalar_get_stats(&ss);
    std::printf("summary bad=%d mismatch=%d opened=%d rejected=%d tx_frames=%llu tx_flushes=%llu tx_host_flushes=%llu "
                "rx_frames=%llu rx_flushes=%llu rx_host_flushes=%llu evicted=%llu device_failures=%llu overflows=%llu\n",
                bad.load(), mismatch.load(), opened.load(), rejected.load(), (unsigned long long)st.frames,
                (unsigned long long)st.flushes, (unsigned long long)st.host_flushes, (unsigned long long)sr.frames,
                (unsigned long long)sr.flushes, (unsigned long long)sr.host_flushes,
                (unsigned long long)(st.evicted + sr.evicted), (unsigned long long)ss.device_failures,
                (unsigned long long)(st.cas_retries + sr.cas_retries));
    return (bad || mismatch) ? 1 : 0;
}

// split <policy> <frames> <window>: ONE reader thread submits (FrameQueue::submit) and ONE writer
// thread collects (FrameTicket::get), the relay split of SessionManager (a socket reader hands
// frames to a sender), at most `window` frames between them.  Every frame is checked against the
// host engine's bytes.  AUTO must count each frame against the submitting thread only while it is
// uncollected, wherever it is collected: a trickle stays on the host engine.
int split_mode(const std::string& policy, int F, int W) {
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    FrameQueue tx;
    std::array<std::uint8_t, 32> key{};
    std::uint64_t seed = 4242;
    for (auto& b : key) b = (std::uint8_t)splitmix(seed);
    std::vector<std::vector<std::uint8_t>> msgs(F);
    for (auto& m : msgs) {
        m.resize(splitmix(seed) % 1600);
        for (auto& b : m) b = (std::uint8_t)splitmix(seed);
    }
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<int, FrameTicket>> q;
    int in_flight = 0;
    std::atomic<int> bad{0}, mismatch{0};
    std::thread reader([&] {
        for (int i = 0; i < F; ++i) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return in_flight < W; });
            }
            FrameTicket t = tx.submit(key, msgs[i]);
            std::lock_guard<std::mutex> lk(mu);
            q.emplace_back(i, std::move(t));
            ++in_flight;
            cv.notify_all();
        }
    });
    std::thread writer([&] {
        for (int done = 0; done < F; ++done) {
            std::pair<int, FrameTicket> it;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !q.empty(); });
                it = std::move(q.front());
                q.pop_front();
            }
            auto f = it.second.get();
            if (!f) ++bad;
            else if (frame_mismatch(key, msgs[it.first], *f)) ++mismatch;
            std::lock_guard<std::mutex> lk(mu);
            --in_flight;
            cv.notify_all();
        }
    });
    reader.join();
    writer.join();
    const auto st = tx.stats();
    std::printf("summary bad=%d mismatch=%d tx_frames=%llu tx_flushes=%llu tx_host_flushes=%llu\n", bad.load(),
                mismatch.load(), (unsigned long long)st.frames, (unsigned long long)st.flushes,
                (unsigned long long)st.host_flushes);
    return (bad || mismatch) ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "window")
        return window_mode(argc > 2 ? argv[2] : "device", argc > 3 ? std::atoi(argv[3]) : 16,
                           argc > 4 ? std::atoi(argv[4]) : 256, argc > 5 ? std::atoi(argv[5]) : 4000);
    if (argc > 1 && std::string(argv[1]) == "split")
        return split_mode(argc > 2 ? argv[2] : "auto", argc > 3 ? std::atoi(argv[3]) : 2000,
                          argc > 4 ? std::atoi(argv[4]) : 8);
    if (argc > 1 && std::string(argv[1]) == "async")
        return async_mode(argc > 2 ? argv[2] : "device", argc > 3 ? std::atoi(argv[3]) : 8,
                          argc > 4 ? std::atoi(argv[4]) : 500);
    if (argc > 1 && std::string(argv[1]) == "nonces")
        return nonce_uniqueness(argc > 2 ? argv[2] : "auto", argc > 3 ? std::atoi(argv[3]) : 8,
                                argc > 4 ? std::atoi(argv[4]) : 10000);
    const std::string policy = argc > 1 ? argv[1] : "auto";
    const int T = argc > 2 ? std::atoi(argv[2]) : 16;
    const int F = argc > 3 ? std::atoi(argv[3]) : 200;
    const std::uint64_t seed = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 1;
    enet_scalar_set_policy(policy == "device" ? ENET_SCALAR_DEVICE : policy == "host" ? ENET_SCALAR_HOST
                                                                                      : ENET_SCALAR_AUTO, 0);
    std::vector<std::array<std::uint8_t, 32>> keys(T);
    std::vector<std::vector<std::vector<std::uint8_t>>> msgs(T), frames(T);
    for (int t = 0; t < T; ++t) {
        std::uint64_t s = seed * 1000003u + (std::uint64_t)t;
        for (auto& b : keys[t]) b = (std::uint8_t)splitmix(s);
        msgs[t].resize(F);
        for (int i = 0; i < F; ++i) {
            std::size_t L = splitmix(s) % 3001;
            if (i % 53 == 5) L = 65536;
            if (t == 0 && i == 1) L = FrameQueue::kMaxPayloadSize - 32;  // largest signed payload
            msgs[t][i].resize(L);
            for (auto& b : msgs[t][i]) b = (std::uint8_t)splitmix(s);
        }
    }
    FrameQueueOptions opt;
    opt.max_frames = 512;
    opt.max_delay = std::chrono::microseconds(200);
    FrameQueue tx(opt);
    FrameReceiveQueue rx(opt);
    std::atomic<int> bad{0}, oversize_ok{0}, mismatch{0};
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                frames[t].resize(F);
                for (int i = 0; i < F; ++i) {
                    auto f = tx.seal(keys[t], msgs[t][i]);
                    if (!f || f->size() != msgs[t][i].size() + 48) {
                        ++bad;
                        continue;
                    }
                    if (frame_mismatch(keys[t], msgs[t][i], *f)) ++mismatch;
                    frames[t][i] = std::move(*f);
                }
                // too large: refused like SessionManager::send, nothing queued
                std::vector<std::uint8_t> huge(FrameQueue::kMaxPayloadSize - 31);
                if (!tx.seal(keys[t], huge)) ++oversize_ok;
            });
        for (auto& x : th) x.join();
    }
    std::atomic<int> opened{0}, rejected{0}, wrong{0};
    {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                for (int i = 0; i < F; ++i) {
                    std::vector<std::uint8_t> f = frames[t][i];
                    if (f.empty()) continue;
                    bool expect_ok = true;
                    auto key = keys[t];
                    if (i % 7 == 3) {  // tamper: nonce, length field, body or MAC byte
                        const std::size_t pos[4] = {5, 13, 16 + msgs[t][i].size() / 2, f.size() - 1};
                        f[pos[(i / 7) % 4]] ^= 0x10;
                        expect_ok = false;
                    } else if (i % 11 == 4) {  // another session's key
                        key = keys[(t + 1) % T];
                        expect_ok = T == 1;
                    }
                    auto m = rx.open(key, f);
                    if (m) ++opened;
                    else ++rejected;
                    if ((bool)m != expect_ok || (m && *m != msgs[t][i])) ++wrong;
                }
            });
        for (auto& x : th) x.join();
    }
    // sample for the oracle: the first 3 frames of every thread with a message <= 4 KiB
    for (int t = 0; t < T; ++t) {
        int shown = 0;
        for (int i = 0; i < F && shown < 3; ++i) {
            if (msgs[t][i].size() > 4096 || frames[t][i].empty()) continue;
            std::printf("frame %s %s %s\n", hex(std::vector<std::uint8_t>(keys[t].begin(), keys[t].end())).c_str(),
                        hex(msgs[t][i]).c_str(), hex(frames[t][i]).c_str());
            ++shown;
        }
    }
    const auto st = tx.stats(), sr = rx.stats();
    enet_scalar_stats ss{};
    enet_scalar_get_stats(&ss);
    std::printf("summary bad=%d mismatch=%d oversize_refused=%d opened=%d rejected=%d wrong=%d tx_frames=%llu tx_flushes=%llu "
                "tx_host_flushes=%llu rx_frames=%llu rx_flushes=%llu rx_host_flushes=%llu device_failures=%llu\n",
                bad.load(), mismatch.load(), oversize_ok.load(), opened.load(), rejected.load(), wrong.load(),
                (unsigned long long)st.frames, (unsigned long long)st.flushes, (unsigned long long)st.host_flushes,
                (unsigned long long)sr.frames, (unsigned long long)sr.flushes, (unsigned long long)sr.host_flushes,
                (unsigned long long)ss.device_failures);
    return (bad || wrong || mismatch || oversize_ok != T) ? 1 : 0;
}
