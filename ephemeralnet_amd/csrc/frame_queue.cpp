// frame_queue.cpp -- the cross-session frame queues of Batch.hpp.
//
// Reference: SessionManager::send (src/network/SessionManager.cpp:337-388), receive_loop
// (:703-854) and protocol::encode_signed / decode_signed (src/protocol/Message.cpp:305-328): one
// frame per call on the session's own thread.
//
// Design (round 5).  A queue direction owns a few PASSES: blocks of pinned, device-mapped host
// memory laid out as one wire-frame batch (offsets, keys, nonces, ok / MAC arrays, input arena,
// output arena).  A submitting thread
//   1. reserves the next slot of its shard's open pass with ONE atomic add on a packed word
//      (closed bit | slot count | input bytes used) -- the output offset follows from the slot
//      index (frames are +48 / -48 bytes), so nothing else is shared;
//   2. copies its message / frame into the pass arena and its key, nonce, offset and length
//      into the slot's own 128-byte record (no cache line shared with a neighbouring slot), then
//      sets the record's state;
//   3. gets a FrameTicket (a small heap State shared with the pass).
// A worker thread takes an open pass once it reaches a quarter of the size limits, when no frame
// has arrived for 30 us, or 250 us after its first frame; closes it (the same word: no slot can be
// reserved after), waits for the slots' states, packs the records into the offsets / keys /
// nonces arrays, and runs enet_wire_seal_batch / _open_batch on the pass in place (its own HIP
// stream; the kernel reads a small pass over PCIe, a large one from a device copy of its input
// side, and writes the results into the pass).  Each ticket copies its own result out of the pass on its
// owner's thread.  A pass is reused once every ticket of it has collected or dropped its result;
// when every pass is referenced, the oldest finished one is evicted (its uncollected results
// copied into their tickets).  Round 4's queue built every pass in its worker (a gather of every
// request through the batch runtime's pool, a scatter into per-request vectors, a promise per
// frame): ~300 us and ~100 frames per pass at 4 096 frames in flight, 1.29 M frames/s sealed.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <future>
#include <memory>
#include <mutex>
#include <new>
#include <pthread.h>
#include <sched.h>
#include <unistd.h>
#include <sys/prctl.h>
#include <time.h>
#include <random>
#include <stdexcept>
#include <system_error>
#include <thread>
#include <vector>

#include <immintrin.h>

#include <hip/hip_runtime.h>

#include "enet_crypto.h"
#include "ephemeralnet/crypto/Batch.hpp"
#include "host_batch.hpp"
#include "host_engine.hpp"
#include "host_topo.hpp"
#include "scalar.hpp"

namespace ephemeralnet::crypto::batch {

namespace {

#ifdef ENET_TOOLS_BUILD
// ENET_QUEUE_FAKE_US=<us> (tools build only): a stand-in for the device on a CPU-only host -- a
// pass "runs" for that long and computes nothing (outputs are garbage, opens report ok), so the
// submitting threads' CPU per frame can be measured without a GPU (tools/queue_bench); with
// ENET_QUEUE_FAKE_COMPUTE=1 the worker computes it on the host engine first (real bytes, so
// tests/cpp/queue_stress checks device-style passes, evictions included, on a CPU-only host)
double fake_us() {
    static const double v = [] {
        const char* e = std::getenv("ENET_QUEUE_FAKE_US");
        return e ? std::atof(e) : 0.0;
    }();
    return v;
}
// ENET_QUEUE_PROF=1 (tools build only): TSC cycles per phase of submit() / get(), summed over
// threads, printed at exit
constexpr int kProfPhases = 16;
const char* const kProfName[kProfPhases] = {"submit: ticket state", "submit: reserve (atomic add)",
                                            "submit: fill slot", "submit: notify", "get: claim",
                                            "get: wait (pass not done)", "get: copy result", "get: release",
                                            "submit: open a pass", "submit: pass full / closed",
                                            "open_pass: lock mu_", "open_pass: reuse a released pass",
                                            "open_pass: allocate a pass", "open_pass: wait for a pass",
                                            "open_pass: another opened it", "get: release store"};
std::atomic<std::uint64_t> g_prof_c[kProfPhases], g_prof_n[kProfPhases];
bool prof_on() {
    static const bool v = std::getenv("ENET_QUEUE_PROF") != nullptr;
    return v;
}
struct ProfThread {
    std::uint64_t c[kProfPhases] = {}, n[kProfPhases] = {};
    ~ProfThread() {
        for (int i = 0; i < kProfPhases; ++i) {
            g_prof_c[i] += c[i];
            g_prof_n[i] += n[i];
        }
    }
};
thread_local ProfThread t_prof;
struct ProfReport {
    ~ProfReport() {
        if (!prof_on()) return;
        const auto w0 = std::chrono::steady_clock::now();
        const std::uint64_t c0 = __rdtsc();
        while (std::chrono::steady_clock::now() - w0 < std::chrono::milliseconds(20)) {
        }
        const double ghz = (double)(__rdtsc() - c0) / 2e7;
        for (int i = 0; i < kProfPhases; ++i)
            std::fprintf(stderr, "[enet queue prof] %-26s %12llu calls %8.1f ns/call %8.3f s\n", kProfName[i],
                         (unsigned long long)g_prof_n[i].load(),
                         (double)g_prof_c[i].load() / ghz / std::max<double>(1, (double)g_prof_n[i].load()),
                         (double)g_prof_c[i].load() / ghz * 1e-9);
    }
} g_prof_report;
inline std::uint64_t prof_t() { return prof_on() ? __rdtsc() : 0; }
inline void prof_add(int i, std::uint64_t& t0) {
    if (!prof_on()) return;
    const std::uint64_t t = __rdtsc();
    t_prof.c[i] += t - t0;
    t_prof.n[i] += 1;
    t0 = t;
}
// ENET_QUEUE_STALL_OVERFLOW_US=<us> (tools build only): a submitter whose reservation found its
// pass full sleeps that long before closing it -- the preemption window of ADVICE r05's stale
// close, made wide for tests/cpp/queue_stress
void stall_overflow() {
    static const int us = std::getenv("ENET_QUEUE_STALL_OVERFLOW_US") ? std::atoi(std::getenv("ENET_QUEUE_STALL_OVERFLOW_US")) : 0;
    if (us > 0) std::this_thread::sleep_for(std::chrono::microseconds(us));
}
#else
inline void stall_overflow() {}
constexpr double fake_us() { return 0.0; }
inline std::uint64_t prof_t() { return 0; }
inline void prof_add(int, std::uint64_t&) {}
#endif

// A large device pass is staged: its input side goes to device memory by one SDMA copy and the
// kernel reads HBM; smaller passes run zero-copy (the kernel reads the pinned pass over PCIe).
// Box, 16 threads, sealed / opened M frames/s, staged vs zero-copy forced (tools/stage_ab.sh):
// with 4 passes in flight (profiles/r05_queue_stage_ab.jsonl) x 1 024 in flight 15.7-15.8 /
// 16.8-17.0 vs 14.0 / 13.7-13.8, x 128 6.3-6.9 / 7.2-7.5 vs 7.4 / 7.4-8.2; with the default 8
// (profiles/r05_queue_stage_ab_w8.jsonl) x 256 (passes of 580-640 frames) 10.6-10.8 / 12.2 vs
// 11.6-11.7 / 11.5-11.6, x 384 (670-770) 13.9-14.1 / 15.6-16.1 vs 13.2-13.4 / 13.7-13.8, x 512
// (870-910) 15.3-16.7 / 18.3-18.8 vs 14.5 / 14.2-14.5.  A sealing pass pays for the copy from
// ~640 frames, an opening pass from ~512 (below, the copy only adds latency to a kernel bound by
// its per-frame chain).  Tools build: ENET_QUEUE_STAGE=0 / 1 forces either.
bool stage_pass(std::uint32_t n, bool open_dir) {
#ifdef ENET_TOOLS_BUILD
    static const int v = std::getenv("ENET_QUEUE_STAGE") ? std::atoi(std::getenv("ENET_QUEUE_STAGE")) : -1;
    if (v >= 0) return v != 0;
#endif
    return n >= (open_dir ? 512u : 640u);
}

constexpr std::size_t kHeader = 16;  // nonce(12) || BE32(|body|), SessionManager.cpp:376-385
constexpr std::size_t kMac = 32;
constexpr std::size_t kWire = kHeader + kMac;  // |frame| - |message|

void put_be32(std::uint8_t* p, std::uint32_t v) {
    p[0] = (std::uint8_t)(v >> 24);
    p[1] = (std::uint8_t)(v >> 16);
    p[2] = (std::uint8_t)(v >> 8);
    p[3] = (std::uint8_t)v;
}

// host engine: SessionManager::send for one frame, into `f` (|m| + 48 bytes)
void host_wire_seal_into(const std::uint8_t key[32], const std::uint8_t nonce[12], std::span<const std::uint8_t> m,
                         std::uint8_t* f) {
    enet::host::seal_body(key, nonce, m.data(), m.size(), f + kHeader);
    std::memcpy(f, nonce, 12);
    put_be32(f + 12, (std::uint32_t)(m.size() + kMac));
}

std::vector<std::uint8_t> host_wire_seal(const std::uint8_t key[32], const std::uint8_t nonce[12],
                                         std::span<const std::uint8_t> m) {
    std::vector<std::uint8_t> f(kWire + m.size());
    host_wire_seal_into(key, nonce, m, f.data());
    return f;
}

// the length checks of receive_loop (:760-796) and decode_signed (Message.cpp:315)
bool frame_shape_ok(std::span<const std::uint8_t> f) {
    if (f.size() < kWire) return false;
    const std::uint32_t len = (std::uint32_t)f[12] << 24 | (std::uint32_t)f[13] << 16 |
                              (std::uint32_t)f[14] << 8 | f[15];
    return (std::uint64_t)len == f.size() - kHeader && len <= FrameQueue::kMaxPayloadSize;
}

// host engine: receive_loop decrypt + decode_signed verify for one frame (shape already checked);
// the message goes to `m` (|f| - 48 bytes; zeroed when the MAC does not verify)
bool host_wire_open_into(const std::uint8_t key[32], std::span<const std::uint8_t> f, std::uint8_t* m) {
    return enet::host::open_body(key, f.data(), f.data() + kHeader, f.size() - kHeader, m);
}

bool host_wire_open(const std::uint8_t key[32], std::span<const std::uint8_t> f, std::vector<std::uint8_t>& m) {
    std::vector<std::uint8_t> out(f.size() - kWire);
    if (!host_wire_open_into(key, f, out.data())) return false;
    m = std::move(out);
    return true;
}

// Frame nonces.  SessionManager::send draws each nonce from a fresh std::random_device
// (SessionManager.cpp:365-371); on the box that source serves ~0.4 M nonces/s for the whole
// machine however many threads ask, which capped every sender.  Each thread here keeps a
// ChaCha20 keystream generator keyed with 256 bits from std::random_device and re-keyed every
// 2^20 nonces (the arc4random construction): 12 unpredictable bytes per frame, never reused under
// one session key.  fork() copies a thread's generator into the child, so parent and child would
// hand out the same nonces; a pthread_atfork child handler bumps a generation
// counter, and a generator whose generation is stale re-keys from std::random_device before its
// next nonce.
std::atomic<std::uint32_t> g_fork_generation{0};
[[maybe_unused]] const int g_atfork_registered = pthread_atfork(nullptr, nullptr, [] {
    g_fork_generation.fetch_add(1, std::memory_order_relaxed);
});

class NonceSource {
public:
    void draw(std::uint8_t* n) {
        const std::uint32_t gen = g_fork_generation.load(std::memory_order_relaxed);
        if (gen != gen_) {  // first use, or a forked child: new key, discard buffered keystream
            gen_ = gen;
            left_ = 0;
            pos_ = sizeof(buf_);
        }
        if (pos_ + 12 > sizeof(buf_)) refill();
        std::memcpy(n, buf_ + pos_, 12);
        std::memset(buf_ + pos_, 0, 12);
        pos_ += 12;
    }

private:
    void refill() {
        if (left_ == 0) {
            std::random_device rd;
            for (int i = 0; i < 32; i += 4) {
                const std::uint32_t v = rd();
                std::memcpy(key_ + i, &v, 4);
            }
            for (int i = 0; i < 12; i += 4) {
                const std::uint32_t v = rd();
                std::memcpy(iv_ + i, &v, 4);
            }
            ctr_ = 0;
            left_ = 1u << 20;
        }
        // whole keystream blocks only: the next refill starts at the next unused block, so no
        // keystream byte (and no nonce) is ever handed out twice
        std::memset(buf_, 0, sizeof(buf_));
        enet::host::chacha20_xor(key_, iv_, ctr_, buf_, buf_, sizeof(buf_));
        ctr_ += kBlocks;
        pos_ = 0;
        left_ = left_ > kPerFill ? left_ - kPerFill : 0;
    }
    static constexpr std::uint32_t kBlocks = 16;                      // keystream blocks per fill
    static constexpr std::uint32_t kPerFill = kBlocks * 64 / 12;     // 85 nonces per fill
    std::uint8_t key_[32] = {}, iv_[12] = {};
    std::uint32_t ctr_ = 0, left_ = 0, gen_ = 0;
    std::uint8_t buf_[kBlocks * 64] = {};
    std::size_t pos_ = sizeof(buf_);
};

NonceSource& nonce_source() {
    thread_local NonceSource src;
    return src;
}

double thread_cpu_s() {
    timespec ts{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool trace_on() {
    static const bool v = [] {
        const char* e = std::getenv("ENET_HOST_TRACE");
        return e && e[0] == '1';
    }();
    return v;
}

struct Pass;

// A slot's ticket word (SlotRec::tk) = pass generation << 3 | one of these.  The generation
// makes a reused slot's word differ from every earlier use of it, so a ticket can never act on
// a slot that has moved on to another frame.
enum : std::uint64_t {
    kPending = 1,   // in the pass, not collected
    kClaimed = 2,   // its ticket is reading the pass (get / ready)
    kReleased = 3,  // collected or dropped: the pass may be reused
    kEvicting = 4,  // the queue is copying the result into the ticket's State
    kEvicted = 5,   // ... done: the pass may be reused
    kViewing = 6,   // its ticket holds a zero-copy view of the result (FrameTicket::view)
};
// FrameTicket::State::st
enum : int { kInPass = 0, kHasResult = 1 };

}  // namespace

// A ticket's state: owned, allocated and freed by the ticket (the submitting thread, normally),
// never by the queue.  The queue writes it only while evicting (between winning the slot's
// kPending -> kEvicting and setting st = kHasResult), and the ticket does not free it before it
// sees kHasResult in that case.
struct FrameTicket::State {
    std::atomic<int> st{kHasResult};
    Pass* pass = nullptr;
    std::uint32_t idx = 0;
    std::uint64_t gen = 0;
    bool viewing = false;  // the slot is kViewing: this ticket holds a view into the pass
    // AUTO's routing signals this ticket is counted in until it is collected or dropped (on
    // whatever thread): its submitting thread's backlog, and its shard of the process-wide count
    std::shared_ptr<std::atomic<std::int32_t>> backlog;
    std::atomic<std::int64_t>* inflight = nullptr;
    std::optional<std::vector<std::uint8_t>> result;
};

namespace {

enum : int { kOpen = 0, kClosed = 1, kDone = 2 };
constexpr std::uint64_t kClosedBit = 1ull << 63;
constexpr int kSlotShift = 40;  // res = closed | slots << 40 | input bytes used (< 2^40)
constexpr std::uint64_t kBytesMask = (1ull << kSlotShift) - 1;
constexpr std::uint64_t kSlotMask = (1ull << 23) - 1;
// A slot's fill word (SlotRec::fill) = pass generation << 2 | one of these; an older generation
// reads as empty
enum : std::uint64_t { kFilled = 1, kOverflow = 2 };

std::uint64_t up256(std::uint64_t x) { return (x + 255) & ~std::uint64_t(255); }

// the slot's fill state in generation gen, once its submitter has written it
std::uint64_t spin_until(const std::atomic<std::uint64_t>& f, std::uint64_t gen) {
    for (int i = 0;; ++i) {
        const std::uint64_t v = f.load(std::memory_order_acquire);
        if ((v >> 2) == gen) return v & 3;
        if (i < 1024) _mm_pause();
        else std::this_thread::yield();  // its submitter was preempted mid-copy
    }
}

struct alignas(128) SlotRec {
    std::atomic<std::uint64_t> fill{0};  // gen << 2 | kFilled / kOverflow
    std::atomic<std::uint64_t> tk{0};    // gen << 3 | kPending .. kEvicted
    std::uint64_t in_at = 0;             // input offset in the pass arena
    std::uint64_t len = 0;               // input bytes
    FrameTicket::State* ticket = nullptr;
    std::uint8_t key[32];
    std::uint8_t nonce[12];
};

// One device pass: pinned, device-mapped staging laid out as a wire-frame batch.
struct Pass {
    bool open_dir = false;  // FrameReceiveQueue (frames in, messages out)
    std::uint8_t* h = nullptr;  // host view of the block
    std::uint8_t* d = nullptr;  // device view (nullptr: plain heap memory, host engine only)
    bool pinned = false;        // h from topo::alloc_pinned
    std::size_t bytes = 0;
    std::uint32_t cap_frames = 0;
    std::uint64_t cap_in = 0;
    std::uint64_t o_inoff = 0, o_outoff = 0, o_keys = 0, o_nonces = 0, o_ok = 0, o_macs = 0, o_in = 0, o_out = 0;
    // [cap_frames] what each submitter writes about its slot, one 128-byte record per slot: the
    // offsets / keys / nonces arrays the kernel reads pack 2-10 slots per cache line, and filling
    // them from the submitting threads shared every such line between neighbouring slots; the
    // worker packs them from these records when the pass runs
    std::unique_ptr<SlotRec[]> recs;
    alignas(64) std::atomic<std::uint64_t> res{kClosedBit};
    alignas(64) std::atomic<std::int64_t> first_us{0};
    std::atomic<int> state{kDone};
    // generation: +1 each time the pass is reopened (under the queue's mu_; read without it by a
    // submitter, before its reservation, to tie a later close_full to that generation)
    std::atomic<std::uint64_t> gen{0};
    std::uint32_t reserved = 0;  // reservations made before the close (some may be overflows)
    std::uint32_t n = 0;         // final slot count (set when the pass runs)
    std::uint32_t rel_scan = 0;  // released(): slots [0, rel_scan) are known released (under mu_)
    std::uint64_t in_used = 0;   // final input bytes
    double closed_at = 0;
    std::mutex mu;
    std::condition_variable cv;  // waiters for kDone

    std::uint64_t* in_off() const { return reinterpret_cast<std::uint64_t*>(h + o_inoff); }
    std::uint64_t* out_off() const { return reinterpret_cast<std::uint64_t*>(h + o_outoff); }
    // output bytes of a frame with `in` input bytes, and the output offset of slot idx
    std::uint64_t out_len(std::uint64_t in) const { return open_dir ? in - kWire : in + kWire; }
    std::uint64_t out_at(std::uint64_t in_at, std::uint32_t idx) const {
        return open_dir ? in_at - kWire * idx : in_at + kWire * idx;
    }
    void wait_done() {
        for (int i = 0; i < 64; ++i) {  // a pass takes ~100 us: only a short spin, then sleep
            if (state.load(std::memory_order_acquire) == kDone) return;
            _mm_pause();
        }
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return state.load(std::memory_order_acquire) == kDone; });
    }
    // the slot's result (pass done)
    std::optional<std::vector<std::uint8_t>> result_of(std::uint32_t i) const {
        const std::uint64_t a = in_off()[i], b = in_off()[i + 1];
        if (open_dir && h[o_ok + i] != 1) return std::nullopt;
        const std::uint8_t* p = h + o_out + out_at(a, i);
        return std::vector<std::uint8_t>(p, p + out_len(b - a));
    }
    bool result_view(std::uint32_t i, std::span<const std::uint8_t>& out) const {
        const std::uint64_t a = in_off()[i], b = in_off()[i + 1];
        if (open_dir && h[o_ok + i] != 1) {
            out = {};
            return false;
        }
        out = std::span<const std::uint8_t>(h + o_out + out_at(a, i), out_len(b - a));
        return true;
    }
    bool result_into(std::uint32_t i, std::vector<std::uint8_t>& out) const {
        const std::uint64_t a = in_off()[i], b = in_off()[i + 1];
        if (open_dir && h[o_ok + i] != 1) {
            out.clear();
            return false;
        }
        const std::uint8_t* p = h + o_out + out_at(a, i);
        out.assign(p, p + out_len(b - a));
        return true;
    }
    ~Pass() {
        if (pinned) enet::topo::free_pinned(h);
        else delete[] h;
    }
};

// Ticket states come from a per-thread cache: the ticket that frees a state is normally on the
// thread that allocated it (the submitter collects its own frames), so a state goes back to the
// cache it came from; a malloc / free pair per frame measured ~100 ns on the box (r05g profile).
struct StateCache {
    std::vector<FrameTicket::State*> v;
    ~StateCache();
};
// The AUTO policy's signals (use_queue_async), counted for every non-blocking submission whatever
// its route and uncounted when its ticket is collected or dropped, on any thread:
//  * the submitting thread's backlog -- a counter the thread shares with its tickets, so a ticket
//    collected by another thread (a reader thread submits, a writer thread collects) or after the
//    submitter exited decrements the right one (a thread-local count only grew on the
//    submitting side of such a split, sending trickle loads to the device);
//  * the process-wide count per direction (many session threads, each with a
//    few frames in flight), sharded over cache lines by thread so submitters do not share one.
struct ThreadBacklog {
    std::shared_ptr<std::atomic<std::int32_t>> c = std::make_shared<std::atomic<std::int32_t>>(0);
};
thread_local ThreadBacklog t_backlog;
struct alignas(64) PaddedCount {
    std::atomic<std::int64_t> v{0};
};
constexpr unsigned kCountShards = 16;
PaddedCount g_inflight[2][kCountShards];
std::atomic<unsigned> g_next_count_shard{0};
std::atomic<std::int64_t>* inflight_slot(bool open_dir) {
    thread_local const unsigned sh = g_next_count_shard.fetch_add(1, std::memory_order_relaxed) % kCountShards;
    return &g_inflight[open_dir ? 1 : 0][sh].v;
}
void count_submission(FrameTicket::State* s, bool open_dir) {
    s->backlog = t_backlog.c;
    s->backlog->fetch_add(1, std::memory_order_relaxed);
    s->inflight = inflight_slot(open_dir);
    s->inflight->fetch_add(1, std::memory_order_relaxed);
}
thread_local int t_cache_state = 0;  // 0 untouched, 1 live, 2 destroyed (trivially destructible)
thread_local StateCache t_cache;
StateCache::~StateCache() {
    t_cache_state = 2;
    for (auto* x : v) delete x;
    v.clear();
}
FrameTicket::State* new_state() {
    if (t_cache_state == 0) {
        t_cache.v.reserve(1024);
        t_cache_state = 1;
    }
    if (t_cache_state != 1 || t_cache.v.empty()) return new FrameTicket::State();
    FrameTicket::State* x = t_cache.v.back();
    t_cache.v.pop_back();
    return x;
}
void free_state(FrameTicket::State* x) {
    if (x->backlog) {
        x->backlog->fetch_sub(1, std::memory_order_relaxed);
        x->backlog.reset();
    }
    if (x->inflight) {
        x->inflight->fetch_sub(1, std::memory_order_relaxed);
        x->inflight = nullptr;
    }
    x->result.reset();
    x->viewing = false;
    x->st.store(kHasResult, std::memory_order_relaxed);
    if (t_cache_state == 1 && t_cache.v.size() < 8192) t_cache.v.push_back(x);
    else delete x;
}

// The ticket word of a ticket's slot
std::atomic<std::uint64_t>& tk_of(const FrameTicket::State* s) { return s->pass->recs[s->idx].tk; }

// Claim a pending slot's result for reading (kPending -> kClaimed); false once it is being or
// has been evicted
bool claim(FrameTicket::State* s) {
    std::uint64_t e = s->gen << 3 | kPending;
    return tk_of(s).compare_exchange_strong(e, s->gen << 3 | kClaimed, std::memory_order_acq_rel);
}
void set_tk(FrameTicket::State* s, std::uint64_t st) { tk_of(s).store(s->gen << 3 | st, std::memory_order_release); }
// an evicted ticket's result is in its State once st says so
void await_evicted(const FrameTicket::State* s) {
    while (s->st.load(std::memory_order_acquire) != kHasResult) _mm_pause();
}
// Does the ticket read its result from the pass (it holds the slot: claimed now, or under its own
// view)?  false: the result is in the State (a ready ticket, or evicted -- awaited here)
bool hold(FrameTicket::State* s) {
    if (s->viewing) return true;
    if (s->st.load(std::memory_order_acquire) != kHasResult && claim(s)) return true;
    await_evicted(s);
    return false;
}

// Submitting threads are spread over a few open passes (shards), each with its own reservation
// word: one shared word measured 3.6-4.7 failed compare-and-swaps per frame at 16 threads
// (profiles/r05b_queue_bench_cas.jsonl), and every attempt moves the cache line, across sockets too.
// Which shard a submitting thread uses: the L3 domain (CCD) of the CPU it runs on, modulo 8
// shards, so the threads sharing a reservation word and a pass's lines mostly share a cache (an
// atomic add or a slot write on a line another CCD owns is a cross-die transfer).  On the box,
// 16 threads x 256 frames in flight: 11.2-12.1 M frames/s at 0.45-0.49 us of CPU per frame vs
// 9.5-9.7 M at 0.53-0.60 with 4 shards by thread order (profiles/r05i_queue_shards.jsonl).
// Without L3 information in sysfs: the thread's arrival order.  Tools build: ENET_QUEUE_SHARDS =
// 1..8, ENET_QUEUE_SHARD_BY = l3 | thread.
constexpr unsigned kMaxShards = 8;
struct ShardPlan {
    unsigned n = 8;
    bool by_l3 = true;
};
ShardPlan shard_plan() {
    ShardPlan p;
#ifdef ENET_TOOLS_BUILD
    if (const char* e = std::getenv("ENET_QUEUE_SHARDS"))
        p.n = std::min<unsigned>(kMaxShards, std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("ENET_QUEUE_SHARD_BY")) p.by_l3 = std::strcmp(e, "l3") == 0;
#endif
    return p;
}
// dense L3-domain index of every CPU (-1 unknown), from sysfs
const std::vector<int>& l3_of_cpu() {
    static const std::vector<int> v = [] {
        std::vector<int> out;
        std::vector<int> ids;
        const long ncpu = sysconf(_SC_NPROCESSORS_CONF);
        for (long c = 0; c < ncpu && c < 4096; ++c) {
            int dense = -1;
            for (int idx = 0; idx < 6 && dense < 0; ++idx) {
                char path[128];
                std::snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%ld/cache/index%d/level", c, idx);
                FILE* f = std::fopen(path, "r");
                if (!f) break;
                int level = 0;
                const bool got = std::fscanf(f, "%d", &level) == 1;
                std::fclose(f);
                if (!got || level != 3) continue;
                std::snprintf(path, sizeof path, "/sys/devices/system/cpu/cpu%ld/cache/index%d/id", c, idx);
                f = std::fopen(path, "r");
                if (!f) break;
                int id = -1;
                if (std::fscanf(f, "%d", &id) == 1 && id >= 0) {
                    auto it = std::find(ids.begin(), ids.end(), id);
                    dense = (int)(it - ids.begin());
                    if (it == ids.end()) ids.push_back(id);
                }
                std::fclose(f);
            }
            out.push_back(dense);
        }
        return out;
    }();
    return v;
}
std::atomic<unsigned> g_next_shard{0};
unsigned my_shard(const ShardPlan& plan) {
    if (plan.by_l3) {
        const int c = sched_getcpu();
        const auto& m = l3_of_cpu();
        if (c >= 0 && (std::size_t)c < m.size() && m[(std::size_t)c] >= 0) return (unsigned)m[(std::size_t)c] % plan.n;
    }
    thread_local const unsigned s = g_next_shard.fetch_add(1, std::memory_order_relaxed);
    return s % plan.n;
}

class Core {
public:
    Core(const FrameQueueOptions& o, bool open_dir) : opt_(o), open_dir_(open_dir) {
        opt_.max_frames = std::min<std::size_t>(std::max<std::size_t>(1, opt_.max_frames), 1u << 20);
        opt_.max_bytes = std::max<std::size_t>(opt_.max_bytes, 4096);
        opt_.max_inflight = std::min<std::size_t>(std::max<std::size_t>(1, opt_.max_inflight), 16);
        // passes: in flight + one open per shard + those still referenced by uncollected tickets
        // (16 threads x 256 frames in flight reference up to ~28 passes when a slow consumer keeps
        // them at ~150 frames); allocated on demand, each sized to the close target below (a
        // quarter of max_frames / max_bytes, at least one maximum frame) -- a pass closes when
        // full anyway, and small passes waste less of the pinned memory they hold
        max_passes_ = 8 * opt_.max_inflight + 2 * plan_.n;
        int count = 0;
        has_device_ = hipGetDeviceCount(&count) == hipSuccess && opt_.device >= 0 && opt_.device < count;
        if (!has_device_) (void)hipGetLastError();
        if (fake_us() > 0) has_device_ = true;
        const bool delay = opt_.max_delay.count() > 0;
        target_frames_ = std::max<std::size_t>(1, delay ? opt_.max_frames : opt_.max_frames / 4);
        target_bytes_ = delay ? opt_.max_bytes : std::max<std::size_t>(opt_.max_bytes / 4, 4096);
    }
    ~Core() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        work_cv_.notify_all();
        for (auto& w : workers_)
            if (w.joinable()) w.join();
        // the workers ran every closed pass and every non-empty open one; a slot reserved while
        // the queue was being destroyed is finished here.  Tickets may outlive the queue: copy
        // out whatever is uncollected, then free.
        for (auto& p : passes_) {
            if (p->state.load() != kDone && close_pass(*p)) {
                double ema = 0;
                std::uint8_t* none = nullptr;
                if (p->reserved) run_pass(*p, false, nullptr, nullptr, ema, none);
                else p->state.store(kDone, std::memory_order_release);
            }
            bool complete = true;
            evict(*p, &complete);
            // a ticket still viewing this pass (FrameTicket::view not yet released): leave the
            // pass's memory to it rather than free it under the view
            if (!complete) (void)p.release();
        }
        if (trace_on() && st_.flushes)
            std::fprintf(stderr, "[enet queue] %s: %llu frames in %llu passes (%.1f per pass), %llu host passes, "
                         "%llu evicted, %zu passes allocated; device pass %.1f us = fill wait %.1f + kernel %.1f "
                         "+ queueing\n",
                         open_dir_ ? "open" : "seal", (unsigned long long)st_.frames,
                         (unsigned long long)st_.flushes, (double)st_.frames / (double)st_.flushes,
                         (unsigned long long)st_.host_flushes, (unsigned long long)st_.evicted, passes_.size(),
                         sum_pass_us_ / std::max<double>(1, dev_passes_), sum_fill_us_ / std::max<double>(1, dev_passes_),
                         sum_kernel_us_ / std::max<double>(1, dev_passes_));
    }

    bool has_device() const { return has_device_; }

    // Reserve a slot of this thread's shard's open pass for `in` (one atomic add), fill it,
    // return its ticket
    FrameTicket submit(const std::uint8_t key[32], std::span<const std::uint8_t> in) {
        const std::uint64_t len = in.size();
        Shard& sh = shards_[my_shard(plan_)];
        std::uint64_t pt = prof_t();
        // the nonce is drawn before any slot is reserved: NonceSource::refill may throw
        // (std::random_device), and a reserved slot never filled would stall its pass's worker
        // in spin_until forever
        std::uint8_t nonce[12];
        if (!open_dir_) nonce_source().draw(nonce);
        auto* ts = new_state();
        ts->st.store(kInPass, std::memory_order_relaxed);
        count_submission(ts, open_dir_);
        prof_add(0, pt);
        for (;;) {
            Pass* p = sh.open.load(std::memory_order_acquire);
            if (!p) {
                prof_add(1, pt);
                open_pass(sh);
                prof_add(8, pt);
                continue;
            }
            // the generation this reservation lands in, or an older one (then close_full below
            // leaves the pass alone; the retry reads the current one)
            const std::uint64_t g0 = p->gen.load(std::memory_order_acquire);
            const std::uint64_t v = p->res.fetch_add((1ull << kSlotShift) | len, std::memory_order_acq_rel);
            if (v & kClosedBit) {  // taken by a worker: the shard's next open pass
                prof_add(1, pt);
                if (sh.open.load(std::memory_order_acquire) == p) std::this_thread::yield();
                prof_add(9, pt);
                continue;
            }
            const std::uint32_t idx = (std::uint32_t)((v >> kSlotShift) & kSlotMask);
            const std::uint64_t used = v & kBytesMask;
            if (idx >= p->cap_frames || used + len > p->cap_in) {
                // full: this and every later reservation of the pass is past its end; the first
                // one marks the cut (a slot index below capacity), whoever closes it runs it
                if (idx < p->cap_frames)  // the pass cannot run before this mark: its generation is still ours
                    p->recs[idx].fill.store(p->gen.load(std::memory_order_relaxed) << 2 | kOverflow, std::memory_order_release);
                overflows_.fetch_add(1, std::memory_order_relaxed);
                prof_add(1, pt);
                stall_overflow();
                close_full(p, g0);
                prof_add(9, pt);
                continue;
            }
            if (idx == 0) p->first_us.store((std::int64_t)now_us(), std::memory_order_relaxed);
            prof_add(1, pt);
            fill_slot(*p, idx, used, key, nonce, in, ts);
            prof_add(2, pt);
            if (idx == 0 || idx + 1 == target_frames_ || (used < target_bytes_ && used + len >= target_bytes_)) {
                std::lock_guard<std::mutex> lk(mu_);  // no lost wake-up: workers check under mu_
                work_cv_.notify_one();
                prof_add(3, pt);
            }
            return FrameTicket(ts);
        }
    }

    FrameQueueStats stats() {
        std::lock_guard<std::mutex> lk(mu_);
        FrameQueueStats s = st_;
        const std::uint64_t d = direct_.load(std::memory_order_relaxed);
        s.frames += d;
        s.flushes += d;
        s.host_flushes += d;
        s.pass_us = dev_passes_ ? sum_pass_us_ / dev_passes_ : 0;
        s.kernel_us = dev_passes_ ? sum_kernel_us_ / dev_passes_ : 0;
        s.cas_retries = overflows_.load(std::memory_order_relaxed);
        return s;
    }
    // a frame served on its caller's thread (host engine): one frame, one host pass
    void count_direct() { direct_.fetch_add(1, std::memory_order_relaxed); }

private:
    struct Shard {
        alignas(64) std::atomic<Pass*> open{nullptr};  // read by every submit
        // takeable(): the open pass's slot count when last looked at (under mu_; its own line)
        alignas(64) const Pass* seen_pass = nullptr;
        std::uint64_t seen_n = 0;
        double seen_us = 0;
    };

    void fill_slot(Pass& p, std::uint32_t idx, std::uint64_t at, const std::uint8_t key[32],
                   const std::uint8_t nonce[12], std::span<const std::uint8_t> in, FrameTicket::State* ts) {
        SlotRec& r = p.recs[idx];  // this slot's own cache lines
        const std::uint64_t gen = p.gen.load(std::memory_order_relaxed);  // stable: the pass cannot run before this slot is filled
        r.in_at = at;
        r.len = in.size();
        r.ticket = ts;
        std::memcpy(r.key, key, 32);
        if (!open_dir_) std::memcpy(r.nonce, nonce, 12);
        if (!in.empty()) enet::hb::copy_streaming(p.h + p.o_in + at, in.data(), in.size());
        _mm_sfence();  // the streamed lines are visible before the fill word says so
        ts->pass = &p;
        ts->idx = idx;
        ts->gen = gen;
        r.tk.store(gen << 3 | kPending, std::memory_order_relaxed);
        r.fill.store(gen << 2 | kFilled, std::memory_order_release);
    }

    // A pass for target_frames_ frames and max(target_bytes_, one maximum frame) input bytes
    std::unique_ptr<Pass> make_pass() {
        auto p = std::make_unique<Pass>();
        p->open_dir = open_dir_;
        const std::uint32_t F = (std::uint32_t)target_frames_;
        const std::uint64_t cap_in = std::max<std::uint64_t>(target_bytes_, FrameQueue::kMaxPayloadSize + 256);
        const std::uint64_t cap_out = cap_in + kWire * (std::uint64_t)F;
        std::uint64_t at = 0;
        auto take = [&](std::uint64_t& where, std::uint64_t b) {
            where = at;
            at = up256(at + b);
        };
        take(p->o_inoff, 8ull * (F + 1));
        take(p->o_outoff, 8ull * (F + 1));
        take(p->o_keys, 32ull * F);
        take(p->o_nonces, 12ull * F);
        take(p->o_ok, F);
        take(p->o_macs, 32ull * F);
        take(p->o_in, cap_in);
        take(p->o_out, cap_out);
        p->bytes = at;
        p->cap_frames = F;
        p->cap_in = cap_in;
        if (has_device_ && fake_us() > 0) {
            p->h = new std::uint8_t[at];
            p->d = p->h;
        } else if (has_device_) {
            try {
                void* dp = nullptr;
                p->h = static_cast<std::uint8_t*>(enet::topo::alloc_pinned(at, enet::topo::target_node(opt_.device), &dp));
                p->d = static_cast<std::uint8_t*>(dp);
                p->pinned = true;
            } catch (const std::bad_alloc&) {
                throw;
            } catch (const std::exception& e) {
                enet::scalar::device_failed("FrameQueue pass staging", e.what());
                p->h = nullptr;
                p->d = nullptr;
            }
        }
        if (!p->h) p->h = new std::uint8_t[at];
        p->recs = std::make_unique<SlotRec[]>(F);
        return p;
    }

    // is a finished pass free (every ticket of it collected or dropped)?  Under mu_.  A release is
    // final until the pass is reopened, so the scan resumes where the last one stopped: each slot
    // is looked at about once per pass (rescanning from slot 0 on every open_pass held mu_ for
    // tens of microseconds with many partly collected passes)
    static bool released(Pass& p) {
        if (p.state.load(std::memory_order_acquire) != kDone) return false;
        for (; p.rel_scan < p.n; ++p.rel_scan) {
            const std::uint64_t v = p.recs[p.rel_scan].tk.load(std::memory_order_acquire);
            const std::uint64_t g = p.gen.load(std::memory_order_relaxed);
            if (v != (g << 3 | kReleased) && v != (g << 3 | kEvicted)) return false;
        }
        return true;
    }

    // Copy every uncollected result of a finished pass into its ticket; afterwards no ticket reads
    // the pass -- unless one holds a view (kViewing): *complete is then false and the pass must not
    // be reused until that ticket releases it
    std::uint64_t evict(Pass& p, bool* complete = nullptr) {
        std::uint64_t moved = 0;
        const std::uint64_t g = p.gen.load(std::memory_order_relaxed) << 3;
        if (complete) *complete = true;
        for (std::uint32_t i = 0; i < p.n; ++i) {
            SlotRec& r = p.recs[i];
            for (;;) {
                std::uint64_t e = g | kPending;
                if (r.tk.compare_exchange_strong(e, g | kEvicting, std::memory_order_acq_rel)) {
                    FrameTicket::State* s = r.ticket;
                    s->result = p.result_of(i);
                    s->st.store(kHasResult, std::memory_order_release);  // the ticket may free s now
                    r.tk.store(g | kEvicted, std::memory_order_release);
                    ++moved;
                    break;
                }
                if (e == (g | kViewing)) {  // held by a view: cannot be moved
                    if (complete) *complete = false;
                    break;
                }
                if (e != (g | kClaimed)) break;  // collected or dropped
                _mm_pause();                     // a get() / ready() mid-read
            }
        }
        return moved;
    }

    // Make p the shard's open pass (its old tickets all released or evicted)
    // O(1): the new generation retires every slot word of the old one
    void reopen(Shard& sh, Pass& p) {
        p.gen.store(p.gen.load(std::memory_order_relaxed) + 1, std::memory_order_release);
        p.n = 0;
        p.rel_scan = 0;
        p.reserved = 0;
        p.in_used = 0;
        p.first_us.store(0, std::memory_order_relaxed);
        p.state.store(kOpen, std::memory_order_relaxed);
        p.res.store(0, std::memory_order_release);
        sh.open.store(&p, std::memory_order_release);
    }

    static bool is_open(const Pass* p) { return p && !(p->res.load(std::memory_order_acquire) & kClosedBit); }

    // A new open pass for the shard: a released finished one, a new one, or (all referenced) the
    // oldest finished one evicted; waits while every pass is in flight
    void open_pass(Shard& sh) {
        std::uint64_t pt = prof_t();
        std::size_t evict_tries = 0;  // finished passes found held by a view this call
        std::unique_lock<std::mutex> lk(mu_);
        prof_add(10, pt);
        start_workers();
        for (;;) {
            if (is_open(sh.open.load(std::memory_order_acquire))) {
                prof_add(14, pt);
                return;
            }
            for (auto it = done_.begin(); it != done_.end(); ++it)
                if (released(**it)) {
                    Pass* p = *it;
                    done_.erase(it);
                    reopen(sh, *p);
                    prof_add(11, pt);
                    return;
                }
            if (passes_.size() + allocating_ < max_passes_) {
                prof_add(11, pt);
                ++allocating_;
                lk.unlock();
                std::unique_ptr<Pass> np;
                try {
                    np = make_pass();
                } catch (...) {
                    lk.lock();
                    --allocating_;
                    throw;
                }
                lk.lock();
                --allocating_;
                passes_.push_back(std::move(np));
                Pass* p = passes_.back().get();
                if (is_open(sh.open.load(std::memory_order_acquire))) {
                    done_.push_front(p);  // another submitter opened one meanwhile: keep it spare
                    free_cv_.notify_all();
                    return;
                }
                reopen(sh, *p);
                free_cv_.notify_all();  // submitters waiting for a pass
                prof_add(12, pt);
                return;
            }
            if (!done_.empty() && evict_tries < done_.size()) {
                Pass* p = done_.front();
                done_.pop_front();
                lk.unlock();
                bool complete = true;
                const std::uint64_t moved = evict(*p, &complete);
                lk.lock();
                st_.evicted += moved;
                if (!complete) {  // a ticket holds a view into it: try the next one
                    done_.push_back(p);
                    ++evict_tries;
                    continue;
                }
                if (is_open(sh.open.load(std::memory_order_acquire))) {
                    done_.push_front(p);
                    free_cv_.notify_all();
                    return;
                }
                reopen(sh, *p);
                free_cv_.notify_all();
                return;
            }
            if (evict_tries) {  // every finished pass is held by a view: look again shortly
                evict_tries = 0;
                free_cv_.wait_for(lk, std::chrono::microseconds(100));
                continue;
            }
            prof_add(11, pt);
            free_cv_.wait(lk);  // every pass in flight: wait for one to finish
            prof_add(13, pt);
        }
    }

    // Set p's closed bit; true when this call closed it (no reservation succeeds after it)
    static bool close_pass(Pass& p) {
        const std::uint64_t v = p.res.fetch_or(kClosedBit, std::memory_order_acq_rel);
        if (v & kClosedBit) return false;
        p.reserved = (std::uint32_t)std::min<std::uint64_t>((v >> kSlotShift) & kSlotMask, 0xFFFFFFFFu);
        p.state.store(kClosed, std::memory_order_release);
        p.closed_at = now_us();
        return true;
    }

    // Close a pass a reservation found full.  Only the generation that reservation was made in:
    // a submitter delayed between its reservation and this call may find the pass closed, run,
    // released and reopened -- for another shard, too -- and closing that generation would leave
    // the new owner's open pointer on a closed pass that no worker takes and no submitter
    // reopens.  Once closed, no shard keeps it as its open pass.
    void close_full(Pass* p, std::uint64_t gen) {
        std::lock_guard<std::mutex> lk(mu_);  // reopen() runs under mu_: gen is stable here
        if (p->gen.load(std::memory_order_relaxed) != gen) return;
        if (close_pass(*p)) {
            for (auto& s : shards_)
                if (s.open.load(std::memory_order_relaxed) == p) s.open.store(nullptr, std::memory_order_release);
            closed_.push_back(p);
            work_cv_.notify_one();
        }
    }

    // under mu_
    void start_workers() {
        if (!workers_.empty()) return;
        try {
            for (std::size_t w = 0; w < opt_.max_inflight; ++w) workers_.emplace_back([this] { work(); });
        } catch (const std::system_error&) {
            if (workers_.empty()) throw;
        }
    }

    // When a shard's open pass closes (max_delay 0): at a quarter of the size limits, when no
    // frame has arrived for kGapUs (a lone caller or a burst that ended: not held back), or at
    // kMaxLingerUs after its first frame.  A pass costs the device about the same for 100 frames
    // or 1 000 (one lane's serial HMAC chain per frame), so a steady stream is worth collecting.
    // Closing whenever the device idled gave ~170-frame passes at 16 threads x 256 frames in
    // flight, and ~24 passes referenced by uncollected tickets, so most results were evicted
    // (round 5, first box run).  With max_delay > 0: the size limits or max_delay.
    static constexpr double kGapUs = 30.0, kMaxLingerUs = 250.0;
    // under mu_: should a free worker take the shard's open pass now?
    bool takeable(Shard& sh, const Pass& p) {
        const std::uint64_t r = p.res.load(std::memory_order_acquire);
        if (r & kClosedBit) return false;
        const std::uint64_t n = (r >> kSlotShift) & kSlotMask, b = r & kBytesMask;
        if (n == 0) return false;
        if (stop_ || n >= target_frames_ || b >= target_bytes_) return true;
        const double now = now_us();
        const double age = now - (double)p.first_us.load(std::memory_order_relaxed);
        if (opt_.max_delay.count() > 0) return age >= (double)opt_.max_delay.count();
        if (age >= kMaxLingerUs) return true;
        if (&p != sh.seen_pass || n != sh.seen_n) {  // still arriving: note it, look again later
            sh.seen_pass = &p;
            sh.seen_n = n;
            sh.seen_us = now;
            return false;
        }
        return now - sh.seen_us >= kGapUs;
    }

    void work() {
        const bool fake = fake_us() > 0;
        bool dev_ok = has_device_ && (fake || hipSetDevice(opt_.device) == hipSuccess);
        hipStream_t stream = nullptr;
        hipEvent_t ev = nullptr;
        if (dev_ok && !fake) {
            dev_ok = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) == hipSuccess &&
                     hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
            if (!dev_ok) (void)hipGetLastError();
        }
        (void)prctl(PR_SET_TIMERSLACK, 1000ul, 0, 0, 0);  // fine-grained sleeps in run_pass
        double cpu_seen = thread_cpu_s();
        double kern_ema_us = 0;  // this worker's recent device-pass kernel time
        std::uint8_t* dstage = nullptr;  // device copy of a pass's input side (staged passes)
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            Pass* p = nullptr;
            for (;;) {
                if (!closed_.empty()) {
                    p = closed_.front();
                    closed_.pop_front();
                    break;
                }
                bool frames = false;
                for (unsigned si = 0; si < plan_.n; ++si) {
                    Shard& sh = shards_[si];
                    Pass* o = sh.open.load(std::memory_order_acquire);
                    if (!o) continue;
                    if (takeable(sh, *o)) {
                        if (close_pass(*o)) {
                            sh.open.store(nullptr, std::memory_order_release);
                            p = o;
                            break;
                        }
                        continue;
                    }
                    frames = frames || ((o->res.load(std::memory_order_acquire) >> kSlotShift) & kSlotMask) > 0;
                }
                if (p) break;
                if (stop_) {
                    if (dstage) (void)hipFree(dstage);
                    if (ev) (void)hipEventDestroy(ev);
                    if (stream) (void)hipStreamDestroy(stream);
                    return;
                }
                if (frames && !watching_) {  // one worker watches the open passes' arrivals
                    watching_ = true;
                    const double step = opt_.max_delay.count() > 0
                                            ? std::max<double>(1.0, (double)opt_.max_delay.count() / 4)
                                            : kGapUs / 2;
                    work_cv_.wait_for(lk, std::chrono::microseconds((std::int64_t)step + 1));
                    watching_ = false;
                } else {
                    work_cv_.wait(lk);
                }
            }
            ++inflight_;
            lk.unlock();
            const bool host = run_pass(*p, dev_ok, stream, ev, kern_ema_us, dstage);
            const double cpu = thread_cpu_s();
            lk.lock();
            st_.worker_cpu_s += cpu - cpu_seen;
            cpu_seen = cpu;
            --inflight_;
            st_.frames += p->n;
            st_.flushes += 1;
            st_.host_flushes += host ? 1 : 0;
            done_.push_back(p);
            free_cv_.notify_all();
            work_cv_.notify_one();  // a peer may take an open pass now
        }
    }

    // the pass on the host engine, in place (same layout as the kernel's)
    void host_run(Pass& p) {
        for (std::uint32_t i = 0; i < p.n; ++i) {
            const std::uint64_t a = p.in_off()[i], b = p.in_off()[i + 1];
            std::span<const std::uint8_t> in(p.h + p.o_in + a, b - a);
            std::uint8_t* out = p.h + p.o_out + p.out_at(a, i);
            const std::uint8_t* key = p.h + p.o_keys + 32ull * i;
            if (open_dir_) p.h[p.o_ok + i] = host_wire_open_into(key, in, out) ? 1 : 0;
            else host_wire_seal_into(key, p.h + p.o_nonces + 12ull * i, in, out);
        }
    }

    // Run one closed pass: the device (the kernel on the pinned pass, its input side staged in
    // device memory for large passes) or the host engine (same layout); true when the host
    // engine served it
    bool run_pass(Pass& p, bool dev_ok, hipStream_t stream, hipEvent_t ev, double& kern_ema_us,
                  std::uint8_t*& dstage) {
        const double t0 = now_us();
        // the filled prefix: every reservation before the close writes its slot (filled, or the
        // overflow mark where the pass ran full -- every later reservation is past the end too)
        const std::uint32_t lim = std::min(p.reserved, p.cap_frames);
        std::uint32_t n = lim;
        for (std::uint32_t i = 0; i < lim; ++i)
            if (spin_until(p.recs[i].fill, p.gen.load(std::memory_order_relaxed)) == kOverflow) {
                n = i;
                break;
            }
        // pack the slots' records into the arrays the kernel reads
        std::uint64_t* io = p.in_off();
        std::uint64_t* oo = p.out_off();
        std::uint64_t mx = 0;
        for (std::uint32_t i = 0; i < n; ++i) {
            const SlotRec& r = p.recs[i];
            io[i] = r.in_at;
            oo[i] = p.out_at(r.in_at, i);
            std::memcpy(p.h + p.o_keys + 32ull * i, r.key, 32);
            if (!open_dir_) std::memcpy(p.h + p.o_nonces + 12ull * i, r.nonce, 12);
            mx = std::max(mx, r.len);
        }
        p.n = n;
        p.in_used = n ? p.recs[n - 1].in_at + p.recs[n - 1].len : 0;
        io[n] = p.in_used;
        oo[n] = p.out_at(p.in_used, n);
        const double t1 = now_us();
        bool host = true;
        const bool want_dev = enet::scalar::g_policy.load() != ENET_SCALAR_HOST;
        if (p.n && want_dev && !(dev_ok && p.d))  // counted like a failed launch (enet_scalar_get_stats)
            enet::scalar::device_failed(open_dir_ ? "FrameReceiveQueue pass" : "FrameQueue pass",
                                        "no usable device or pinned staging");
        if (p.n && dev_ok && p.d && want_dev && fake_us() > 0) {
            host = false;
            if (std::getenv("ENET_QUEUE_FAKE_COMPUTE")) host_run(p);  // real bytes, for checks
            else if (open_dir_) std::memset(p.h + p.o_ok, 1, p.n);
            while (now_us() < t1 + fake_us()) std::this_thread::sleep_for(std::chrono::microseconds(20));
        } else if (p.n && dev_ok && p.d && want_dev) {
            host = !enet::scalar::try_device(open_dir_ ? "FrameReceiveQueue pass" : "FrameQueue pass", [&] {
                // staged: the pass's input side (offsets, keys, nonces, messages: one contiguous
                // prefix of the layout) goes to device memory by one SDMA copy and the kernel
                // reads HBM; the results are still written straight into the pinned pass
                const std::uint8_t* din = p.d;
                if (stage_pass(p.n, open_dir_)) {
                    if (!dstage && hipMalloc(reinterpret_cast<void**>(&dstage), p.o_out) != hipSuccess) {
                        dstage = nullptr;
                        const hipError_t e = hipGetLastError();
                        throw std::runtime_error(hipGetErrorString(e));
                    }
                    if (hipMemcpyAsync(dstage, p.h, p.o_in + p.in_used, hipMemcpyHostToDevice, stream) != hipSuccess) {
                        const hipError_t e = hipGetLastError();
                        throw std::runtime_error(hipGetErrorString(e));
                    }
                    din = dstage;
                }
                enet_records r{};
                r.count = p.n;
                r.in_offsets = reinterpret_cast<const std::uint64_t*>(din + p.o_inoff);
                r.out_offsets = reinterpret_cast<const std::uint64_t*>(din + p.o_outoff);
                r.in = din + p.o_in;
                r.out = p.d + p.o_out;
                r.keys = din + p.o_keys;
                r.key_stride = 32;
                r.nonces = open_dir_ ? nullptr : din + p.o_nonces;
                r.total_bytes_hint = p.in_used;
                r.max_len_hint = (std::uint32_t)std::min<std::uint64_t>(mx, 0xFFFFFFFFu);
                const int rc = open_dir_ ? enet_wire_open_batch(&r, p.d + p.o_macs, p.d + p.o_ok, stream)
                                         : enet_wire_seal_batch(&r, stream);
                if (rc != ENET_OK) throw std::runtime_error(enet_last_error());
                if (hipEventRecord(ev, stream) != hipSuccess) {
                    const hipError_t e = hipGetLastError();
                    throw std::runtime_error(hipGetErrorString(e));
                }
                // Poll with ~20 us sleeps: a pass takes ~150-300 us, and a blocking-sync event
                // cost the worker 0.21-0.23 us of CPU per frame against 0.05-0.06 polling, for the
                // same throughput (profiles/r05c_queue_bench.jsonl).  The first sleep covers most of
                // this worker's recent kernel time (a decaying average), so a pass costs a couple of
                // wake-ups instead of ~10.
                const double first = 0.7 * kern_ema_us - 20.0;
                if (first > 0) std::this_thread::sleep_for(std::chrono::microseconds((std::int64_t)first));
                hipError_t q;
                while ((q = hipEventQuery(ev)) == hipErrorNotReady)
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                if (q != hipSuccess) throw std::runtime_error(hipGetErrorString(q));
            });
        }
        if (host && p.n) {  // no device, HOST policy, or a failed launch: the host engine, same layout
            enet::scalar::host_call();
            host_run(p);
        }
        const double t2 = now_us();
        {
            std::lock_guard<std::mutex> lk(p.mu);
            p.state.store(kDone, std::memory_order_release);
        }
        p.cv.notify_all();
        if (!host) {
            kern_ema_us = kern_ema_us > 0 ? 0.8 * kern_ema_us + 0.2 * (t2 - t1) : t2 - t1;
            std::lock_guard<std::mutex> lk(mu_);
            dev_passes_ += 1;
            sum_pass_us_ += t2 - p.closed_at;
            sum_kernel_us_ += t2 - t1;
            sum_fill_us_ += t1 - t0;
        }
        return host;
    }

    FrameQueueOptions opt_;
    bool open_dir_;
    bool has_device_ = false;
    std::size_t max_passes_ = 24;
    std::uint64_t target_frames_ = 1024, target_bytes_ = 2u << 20;
    std::mutex mu_;
    std::condition_variable work_cv_, free_cv_;
    const ShardPlan plan_ = shard_plan();
    Shard shards_[kMaxShards];
    std::vector<std::unique_ptr<Pass>> passes_;
    std::deque<Pass*> closed_, done_;
    std::size_t inflight_ = 0;
    std::size_t allocating_ = 0;  // passes being allocated (outside mu_)
    bool watching_ = false;       // a worker polls the open passes' arrivals
    bool stop_ = false;
    std::vector<std::thread> workers_;
    FrameQueueStats st_{};
    std::atomic<std::uint64_t> direct_{0};
    std::atomic<std::uint64_t> overflows_{0};  // reservations that found their pass full
    double dev_passes_ = 0, sum_pass_us_ = 0, sum_kernel_us_ = 0, sum_fill_us_ = 0;
};

// a ticket whose result is known on the caller's thread (counted like a queued one: AUTO's signals
// see every non-blocking submission, whichever route served it)
FrameTicket ready_ticket(std::optional<std::vector<std::uint8_t>> r, bool open_dir, bool counted = true) {
    auto* s = new_state();
    s->result = std::move(r);
    if (counted) count_submission(s, open_dir);
    return FrameTicket(s);
}

// Non-blocking submissions: the queue under DEVICE; under AUTO when the device is there and either
//  * the submitting thread holds >= 320 uncollected frames -- where the device queue overtakes the
//    host engine in frames/s for a few deep submitters (box, 1 500-byte frames, 16 threads, sealed /
//    opened M frames/s device vs the stitched host engine: x 256 in flight 10.9-11.0 / 11.7-11.8 vs
//    13.2-13.3 / 11.9-12.6, x 384 12.6-12.8 / 13.0 vs 13.2 / 11.9-12.8, x 512 13.4-14.0 / 13.5-13.7
//    vs 11.9-13.1 / 12.8; profiles/r05_seal_crossover_hi.jsonl; below ~64 per thread the device is
//    5-100x slower, profiles/r05s_crossover.jsonl), or
//  * the process holds >= 320 uncollected frames per CPU of its budget in this direction -- many
//    session threads with a few frames each: the host engine's rate is bounded by the CPUs
//    (~0.8 M frames/s each), the device queue's by the frames in flight (profiles/
//    r06_sessions_async.jsonl).
// Blocking seal() / open() never take the queue under AUTO: one frame per blocked session thread
// costs a thread wake-up per frame (7-11 us of CPU), and 64-768 blocked threads moved 0.2-2.2 M
// frames/s through the device queue against 7-10 M on the host engine
// (profiles/r06_sessions_blocking.jsonl).  The device costs a third of the CPU per frame once it
// is fed (0.35-0.44 vs 1.2-1.35 us): ENET_SCALAR_DEVICE is the choice for a relay whose cores have
// other work.  Tools build: ENET_QUEUE_AUTO_BACKLOG overrides the 320.
std::int32_t auto_backlog() {
    static const std::int32_t v = [] {
        std::int32_t b = 320;
#ifdef ENET_TOOLS_BUILD
        if (const char* e = std::getenv("ENET_QUEUE_AUTO_BACKLOG")) b = std::atoi(e);
#endif
        return b;
    }();
    return v;
}
std::int64_t cpu_budget() {
    static const std::int64_t v = [] {
        std::int64_t b = (std::int64_t)enet::topo::allowed_cpus().size();
        if (const std::uint32_t q = enet::topo::cgroup_quota_cpus()) b = std::min<std::int64_t>(b, q);
        if (const std::uint32_t e = enet::topo::env_cpus()) b = std::min<std::int64_t>(b, e);
        return std::max<std::int64_t>(1, b);
    }();
    return v;
}
// the process-wide count of one direction, re-summed every 16th call on a thread (the shards sit on
// lines other threads write; one sum is 16 cache-line reads)
std::int64_t inflight_estimate(bool open_dir) {
    thread_local std::int64_t cached[2] = {0, 0};
    thread_local std::uint32_t calls[2] = {0, 0};
    const int d = open_dir ? 1 : 0;
    if ((calls[d]++ & 15u) == 0) {
        std::int64_t sum = 0;
        for (auto& c : g_inflight[d]) sum += c.v.load(std::memory_order_relaxed);
        cached[d] = sum;
    }
    return cached[d];
}
bool use_queue_async(const Core& c, bool open_dir) {
    const int pol = enet::scalar::g_policy.load();
    if (pol == ENET_SCALAR_DEVICE) return true;
    if (pol != ENET_SCALAR_AUTO || !c.has_device()) return false;
    return t_backlog.c->load(std::memory_order_relaxed) >= auto_backlog() ||
           inflight_estimate(open_dir) >= (std::int64_t)auto_backlog() * cpu_budget();
}

}  // namespace

// ------------------------------------------------------------------------------ FrameTicket
FrameTicket& FrameTicket::operator=(FrameTicket&& o) noexcept {
    if (this != &o) {
        release();
        s_ = o.s_;
        o.s_ = nullptr;
    }
    return *this;
}

FrameTicket::~FrameTicket() { release(); }

// drops the ticket's claim on its slot (or view), frees its state; the ticket is empty after
void FrameTicket::release() noexcept {
    if (!s_) return;
    if (s_->viewing) {
        set_tk(s_, kReleased);
    } else if (s_->st.load(std::memory_order_acquire) != kHasResult) {
        std::uint64_t e = s_->gen << 3 | kPending;
        if (!tk_of(s_).compare_exchange_strong(e, s_->gen << 3 | kReleased, std::memory_order_acq_rel))
            await_evicted(s_);  // the queue is evicting it into s_
    }
    free_state(s_);
    s_ = nullptr;
}

bool FrameTicket::ready() const noexcept {
    if (!s_) return false;
    if (s_->viewing || s_->st.load(std::memory_order_acquire) == kHasResult) return true;
    if (!claim(s_)) return s_->st.load(std::memory_order_acquire) == kHasResult;
    const bool r = s_->pass->state.load(std::memory_order_acquire) == kDone;
    set_tk(s_, kPending);
    return r;
}

std::optional<std::vector<std::uint8_t>> FrameTicket::get() {
    if (!s_) return std::nullopt;
    std::optional<std::vector<std::uint8_t>> r;
    std::uint64_t pt = prof_t();
    if (hold(s_)) {
        prof_add(4, pt);
        if (s_->pass->state.load(std::memory_order_acquire) != kDone) {
            s_->pass->wait_done();
            prof_add(5, pt);
        }
        r = s_->pass->result_of(s_->idx);
        prof_add(6, pt);
        set_tk(s_, kReleased);
        prof_add(15, pt);
    } else {
        r = std::move(s_->result);  // a ready ticket, or evicted
    }
    free_state(s_);
    prof_add(7, pt);
    s_ = nullptr;
    return r;
}

bool FrameTicket::get(std::vector<std::uint8_t>& out) {
    if (!s_) {
        out.clear();
        return false;
    }
    bool ok = false;
    std::uint64_t pt = prof_t();
    if (hold(s_)) {
        prof_add(4, pt);
        if (s_->pass->state.load(std::memory_order_acquire) != kDone) {
            s_->pass->wait_done();
            prof_add(5, pt);
        }
        ok = s_->pass->result_into(s_->idx, out);
        prof_add(6, pt);
        set_tk(s_, kReleased);
        prof_add(15, pt);
    } else {
        ok = s_->result.has_value();
        if (ok) out.assign(s_->result->begin(), s_->result->end());
        else out.clear();
    }
    free_state(s_);
    prof_add(7, pt);
    s_ = nullptr;
    return ok;
}

bool FrameTicket::view(std::span<const std::uint8_t>& out) {
    out = {};
    if (!s_) return false;
    if (!s_->viewing && s_->st.load(std::memory_order_acquire) != kHasResult) {
        std::uint64_t e = s_->gen << 3 | kPending;
        if (tk_of(s_).compare_exchange_strong(e, s_->gen << 3 | kViewing, std::memory_order_acq_rel)) {
            s_->viewing = true;
            if (s_->pass->state.load(std::memory_order_acquire) != kDone) s_->pass->wait_done();
        } else {
            await_evicted(s_);
        }
    }
    if (s_->viewing) return s_->pass->result_view(s_->idx, out);
    if (!s_->result) return false;
    out = std::span<const std::uint8_t>(*s_->result);
    return true;
}

// ------------------------------------------------------------------------------ send
struct FrameQueue::Impl {
    explicit Impl(const FrameQueueOptions& o) : core(o, false) {}
    Core core;
    // push / flush
    mutable std::mutex manual_mu;
    std::vector<std::array<std::uint8_t, 32>> keys;
    std::vector<std::vector<std::uint8_t>> messages;
};

FrameQueue::FrameQueue() : FrameQueue(FrameQueueOptions{}) {}
FrameQueue::FrameQueue(FrameQueueOptions options) : impl_(new Impl(options)) {}
FrameQueue::~FrameQueue() { delete impl_; }

std::optional<std::vector<std::uint8_t>> FrameQueue::seal(const std::array<std::uint8_t, 32>& session_key,
                                                          std::span<const std::uint8_t> message) {
    if (message.size() + kMac > kMaxPayloadSize) return std::nullopt;  // SessionManager.cpp:358-360
    if (enet::scalar::g_policy.load() != ENET_SCALAR_DEVICE) {
        // host engine (policies auto and host): a blocked session thread seals its own frame --
        // one MTU frame costs a core ~1 us, while a device pass cannot return before one lane's
        // serial HMAC over the frame (~70 us), and blocked callers bring one frame each
        std::uint8_t nonce[12];
        nonce_source().draw(nonce);
        enet::scalar::host_call();
        impl_->core.count_direct();
        return host_wire_seal(session_key.data(), nonce, message);
    }
    return impl_->core.submit(session_key.data(), message).get();
}

FrameTicket FrameQueue::submit(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> message) {
    if (message.size() + kMac > kMaxPayloadSize) return ready_ticket(std::nullopt, false, false);
    if (!use_queue_async(impl_->core, false)) {
        std::uint8_t nonce[12];
        nonce_source().draw(nonce);
        enet::scalar::host_call();
        impl_->core.count_direct();
        return ready_ticket(host_wire_seal(session_key.data(), nonce, message), false);
    }
    return impl_->core.submit(session_key.data(), message);
}

std::future<std::optional<std::vector<std::uint8_t>>> FrameQueue::seal_async(
    const std::array<std::uint8_t, 32>& session_key, std::vector<std::uint8_t> message) {
    auto t = submit(session_key, message);  // the message is in the pass already
    return std::async(std::launch::deferred, [t = std::move(t)]() mutable { return t.get(); });
}

bool FrameQueue::push(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> message) {
    if (message.size() + kMac > kMaxPayloadSize) return false;
    std::lock_guard<std::mutex> lk(impl_->manual_mu);
    impl_->keys.push_back(session_key);
    impl_->messages.emplace_back(message.begin(), message.end());
    return true;
}

std::size_t FrameQueue::size() const {
    std::lock_guard<std::mutex> lk(impl_->manual_mu);
    return impl_->messages.size();
}

std::vector<std::vector<std::uint8_t>> FrameQueue::flush() {
    std::vector<std::array<std::uint8_t, 32>> keys;
    std::vector<std::vector<std::uint8_t>> messages;
    {
        std::lock_guard<std::mutex> lk(impl_->manual_mu);
        keys.swap(impl_->keys);
        messages.swap(impl_->messages);
    }
    const std::size_t n = messages.size();
    std::vector<std::vector<std::uint8_t>> frames;
    if (n == 0) return frames;
    std::vector<Nonce> nonces(n);
    for (auto& x : nonces) nonce_source().draw(x.bytes.data());
    std::vector<std::span<const std::uint8_t>> ms(messages.begin(), messages.end());
    // one batch call (the host-memory runtime, crypto::batch::wire_seal); a failed device call is
    // finished on the host engine
    if (enet::scalar::g_policy.load() != ENET_SCALAR_HOST &&
        enet::scalar::try_device("FrameQueue::flush", [&] { frames = wire_seal(keys, nonces, ms); }))
        return frames;
    enet::scalar::host_call();
    frames.assign(n, {});
    for (std::size_t i = 0; i < n; ++i) frames[i] = host_wire_seal(keys[i].data(), nonces[i].bytes.data(), ms[i]);
    return frames;
}

FrameQueueStats FrameQueue::stats() const { return impl_->core.stats(); }

// ------------------------------------------------------------------------------ receive
struct FrameReceiveQueue::Impl {
    explicit Impl(const FrameQueueOptions& o) : core(o, true) {}
    Core core;
};

FrameReceiveQueue::FrameReceiveQueue() : FrameReceiveQueue(FrameQueueOptions{}) {}
FrameReceiveQueue::FrameReceiveQueue(FrameQueueOptions options) : impl_(new Impl(options)) {}
FrameReceiveQueue::~FrameReceiveQueue() { delete impl_; }

std::optional<std::vector<std::uint8_t>> FrameReceiveQueue::open(const std::array<std::uint8_t, 32>& session_key,
                                                                 std::span<const std::uint8_t> frame) {
    if (!frame_shape_ok(frame)) return std::nullopt;  // never reaches a pass
    if (enet::scalar::g_policy.load() != ENET_SCALAR_DEVICE) {  // the caller's thread, no queue
        enet::scalar::host_call();
        impl_->core.count_direct();
        std::vector<std::uint8_t> m;
        if (!host_wire_open(session_key.data(), frame, m)) return std::nullopt;
        return m;
    }
    return impl_->core.submit(session_key.data(), frame).get();
}

FrameTicket FrameReceiveQueue::submit(const std::array<std::uint8_t, 32>& session_key,
                                      std::span<const std::uint8_t> frame) {
    if (!frame_shape_ok(frame)) return ready_ticket(std::nullopt, true, false);
    if (!use_queue_async(impl_->core, true)) {
        enet::scalar::host_call();
        impl_->core.count_direct();
        std::vector<std::uint8_t> m;
        if (!host_wire_open(session_key.data(), frame, m)) return ready_ticket(std::nullopt, true);
        return ready_ticket(std::move(m), true);
    }
    return impl_->core.submit(session_key.data(), frame);
}

std::future<std::optional<std::vector<std::uint8_t>>> FrameReceiveQueue::open_async(
    const std::array<std::uint8_t, 32>& session_key, std::vector<std::uint8_t> frame) {
    auto t = submit(session_key, frame);
    return std::async(std::launch::deferred, [t = std::move(t)]() mutable { return t.get(); });
}

FrameQueueStats FrameReceiveQueue::stats() const { return impl_->core.stats(); }

}  // namespace ephemeralnet::crypto::batch
