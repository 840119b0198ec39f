// host_batch.cpp -- the host-memory batch runtime (host_batch.hpp): gather -> device -> scatter
// over S slots of pinned, device-mapped staging, consecutive chunks overlapped.
//
// Reference: the reference seals and opens frames and chunks in host std::vectors
// (SessionManager.cpp:337-388, 703-854; Message.cpp:305-328; Node.cpp:1414-1417, 1641-1655).
// crypto::batch::* (Batch.hpp), the FrameQueue flushes and the enet_pipeline_* C ABI all run here.
#include "host_batch.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "enet_crypto.h"

namespace enet::hb {

namespace {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("enet host batch: ") + what + ": " + hipGetErrorString(e));
}

void enet_check(int rc, const char* what) {
    if (rc != ENET_OK)
        throw std::runtime_error(std::string("enet host batch: ") + what + ": " + enet_last_error());
}

// ------------------------------------------------------------------------------ worker pool
// parallel(parts, fn): fn(0..parts-1) on the pool's threads and the caller, returns when all ran.
class Pool {
public:
    explicit Pool(unsigned workers) {
        for (unsigned i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            pub_stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void parallel(size_t parts, const std::function<void(size_t)>& fn) {
        if (parts == 0) return;
        if (parts == 1 || th_.empty()) {
            for (size_t i = 0; i < parts; ++i) fn(i);
            return;
        }
        Task t;
        t.fn = &fn;
        t.parts = parts;
        {
            std::lock_guard<std::mutex> lk(mu_);
            task_ = &t;
            ++gen_;
            pub_gen_.store(gen_, std::memory_order_release);
        }
        cv_.notify_all();
        work(t);
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return t.refs == 0 && t.done.load() == t.parts; });
        task_ = nullptr;
        lk.unlock();
        if (t.err) std::rethrow_exception(t.err);
    }

private:
    struct Task {
        const std::function<void(size_t)>* fn = nullptr;
        size_t parts = 0;
        std::atomic<size_t> next{0}, done{0};
        int refs = 0;  // workers inside work() (under mu_)
        std::exception_ptr err;
        std::mutex emu;
    };
    void work(Task& t) {
        for (;;) {
            const size_t i = t.next.fetch_add(1);
            if (i >= t.parts) break;
            try {
                (*t.fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> lk(t.emu);
                if (!t.err) t.err = std::current_exception();
            }
            t.done.fetch_add(1);
        }
    }
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            if (!stop_ && !(task_ && gen_ != seen)) {
                // a pipeline hands out a task set every few hundred microseconds: spin ~20 us for
                // the next one before sleeping (a futex wake-up per worker per set cost ~1.5 ms per
                // 256 MiB job)
                lk.unlock();
                for (int i = 0; i < 4000 && pub_gen_.load(std::memory_order_acquire) == seen && !pub_stop_.load(); ++i)
                    _mm_pause();
                lk.lock();
            }
            cv_.wait(lk, [&] { return stop_ || (task_ && gen_ != seen); });
            if (stop_) return;
            seen = gen_;
            Task* t = task_;
            ++t->refs;
            lk.unlock();
            work(*t);
            lk.lock();
            if (--t->refs == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    Task* task_ = nullptr;
    uint64_t gen_ = 0;
    bool stop_ = false;
    std::atomic<uint64_t> pub_gen_{0};  // gen_ for the spinning workers
    std::atomic<bool> pub_stop_{false};
};

// ------------------------------------------------------------------------------ streaming copy
// Gather / scatter copies move every record once between the caller's memory and the pinned
// staging, while the copy engines read / write that staging too.  Non-temporal (streaming)
// stores skip the read-for-ownership of the destination lines and keep the copies out of the
// caches the session threads use; ENET_HOST_NT=0 selects plain memcpy.  The caller issues a store
// fence before the staging is handed to the device (fence_stores).
__attribute__((target("avx512f"))) void copy_nt512(uint8_t* d, const uint8_t* s, size_t n) {
    const size_t head = std::min<size_t>(n, (64 - (reinterpret_cast<uintptr_t>(d) & 63)) & 63);
    std::memcpy(d, s, head);
    d += head;
    s += head;
    n -= head;
    for (; n >= 256; n -= 256, d += 256, s += 256) {
        const __m512i a = _mm512_loadu_si512(s), b = _mm512_loadu_si512(s + 64), c = _mm512_loadu_si512(s + 128),
                      e = _mm512_loadu_si512(s + 192);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(d), a);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(d + 64), b);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(d + 128), c);
        _mm512_stream_si512(reinterpret_cast<__m512i*>(d + 192), e);
    }
    for (; n >= 64; n -= 64, d += 64, s += 64) _mm512_stream_si512(reinterpret_cast<__m512i*>(d), _mm512_loadu_si512(s));
    std::memcpy(d, s, n);
}

bool use_nt() {
    static const bool v = [] {
        const char* e = std::getenv("ENET_HOST_NT");
        return !(e && e[0] == '0') && __builtin_cpu_supports("avx512f");
    }();
    return v;
}

void copy_out(uint8_t* d, const uint8_t* s, size_t n) {
    if (n >= 512 && use_nt()) copy_nt512(d, s, n);
    else if (n) std::memcpy(d, s, n);
}

void fence_stores() { _mm_sfence(); }

// ------------------------------------------------------------------------------ buffers
struct Pinned {  // pinned, device-mapped host memory, grow-only
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap) return;
        release();
        const size_t c = std::max<size_t>(n + (n >> 3), 64u << 10);
        hip_check(hipHostMalloc(reinterpret_cast<void**>(&h), c, hipHostMallocMapped), "hipHostMalloc");
        void* dp = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&dp, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            h = nullptr;
            hip_check(e, "hipHostGetDevicePointer");
        }
        d = static_cast<uint8_t*>(dp);
        cap = c;
    }
    void release() {
        if (h) (void)hipHostFree(h);
        h = d = nullptr;
        cap = 0;
    }
    ~Pinned() { release(); }
};

struct DevBuf {  // device memory, grow-only
    uint8_t* p = nullptr;
    size_t cap = 0;
    void ensure(size_t n) {
        if (n <= cap) return;
        release();
        const size_t c = std::max<size_t>(n + (n >> 3), 64u << 10);
        hip_check(hipMalloc(reinterpret_cast<void**>(&p), c), "hipMalloc");
        cap = c;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    ~DevBuf() { release(); }
};

// device address of [p, p + n) when the whole range is device-accessible host memory (pinned by
// hipHostMalloc / registered) or device memory; nullptr for pageable memory
uint8_t* device_view(const uint8_t* p, uint64_t n) {
    if (!p || n == 0) return nullptr;
    auto view = [](const uint8_t* q) -> uint8_t* {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();  // pageable: clear the sticky "invalid value"
            return nullptr;
        }
        if (a.type != hipMemoryTypeHost && a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged)
            return nullptr;
        return static_cast<uint8_t*>(a.devicePointer);
    };
    uint8_t* a = view(p);
    uint8_t* b = view(p + (n - 1));
    if (!a || !b || b - a != (ptrdiff_t)(n - 1)) return nullptr;
    return a;
}

int64_t delta_of(Op op) {
    switch (op) {
        case Op::FrameSeal: return 32;
        case Op::FrameOpen: return -32;
        case Op::WireSeal: return 48;
        case Op::WireOpen: return -48;
        default: return 0;
    }
}

bool is_open(Op op) {
    return op == Op::AeadOpen || op == Op::AeadHmacOpen || op == Op::FrameOpen || op == Op::WireOpen ||
           op == Op::ChunkFetch;
}

// Small per-record arrays of one chunk, one pinned block: inputs first, outputs last (so SDMA
// mode moves each half with one copy).
struct Layout {
    uint64_t in_off = 0, out_off = 0, keys = 0, nonces = 0, ctr = 0, tags_in = 0, macs_in = 0, ids = 0,
             session = 0, order = 0, in_end = 0;
    uint64_t tags_out = 0, macs_out = 0, ok = 0, total = 0;
    uint64_t key_bytes = 0;
};

uint64_t up256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

Layout layout(const Job& j, uint32_t m) {
    Layout l;
    uint64_t at = 0;
    auto take = [&](uint64_t& where, uint64_t bytes) {
        where = at;
        at = up256(at + bytes);
    };
    take(l.in_off, 8ull * (m + 1));
    take(l.out_off, 8ull * (m + 1));
    l.key_bytes = j.session ? 0 : (j.key_stride ? 32ull * m : 32ull);
    take(l.keys, std::max<uint64_t>(l.key_bytes, 32));
    take(l.nonces, 12ull * m);
    if (j.counters) take(l.ctr, 4ull * m);
    if (j.tags_in) take(l.tags_in, 16ull * m);
    if (j.macs_in) take(l.macs_in, 32ull * m);
    if (j.ids) take(l.ids, 32ull * m);
    if (j.session) take(l.session, 4ull * m);
    take(l.order, 4ull * m);
    l.in_end = at;
    take(l.tags_out, 16ull * m);
    take(l.macs_out, 32ull * m);
    take(l.ok, m);
    l.total = at;
    return l;
}

std::atomic<int> g_mode{-1};

std::vector<uint8_t>& vec_of(const Job& j, size_t i) { return j.out_vecs ? (*j.out_vecs)[i] : *j.out_each[i]; }

}  // namespace

int64_t out_delta(Op op) { return delta_of(op); }

Mode default_mode() {
    int m = g_mode.load(std::memory_order_relaxed);
    if (m < 0) {
        const char* e = std::getenv("ENET_HOST_MODE");
        // default: copies split by direction, kernels on their own streams -- measured best on
        // the HIP runtime the library is built against, for uniform (C2 e2e 19.0-19.4 GiB/s) and
        // mixed HMAC batches (C5 share 18.7) alike; kernels writing host memory (mode 4) reach
        // 15.8-18.0 / 15.3-15.7 there.  On any other HIP runtime (in practice PyTorch's bundled
        // one, when torch is imported before the library) every D2H hipMemcpyAsync runs as a blit
        // kernel (profiles/r04_torch_runtime_host_c2_*_stats.csv): there mode 4, with no D2H
        // copies, measured 17.9 against 14.0-14.3 (profiles/r04_host_mode4.jsonl)
        int v = 0;
        const bool own_runtime = hipRuntimeGetVersion(&v) == hipSuccess && v / 10000000 == HIP_VERSION_MAJOR &&
                                 (v / 100000) % 100 == HIP_VERSION_MINOR;
        m = (e && std::strcmp(e, "sdma") == 0)    ? (int)Mode::Sdma
            : (e && std::strcmp(e, "split") == 0) ? (int)Mode::SdmaSplit
            : (e && std::strcmp(e, "zc") == 0)    ? (int)Mode::ZeroCopy
            : (e && std::strcmp(e, "zcout") == 0) ? (int)Mode::SdmaInZcOut
            : (e && std::strcmp(e, "splitk") == 0) ? (int)Mode::SdmaSplitK
            : own_runtime                          ? (int)Mode::SdmaSplitK
                                                   : (int)Mode::SdmaInZcOut;
        g_mode.store(m, std::memory_order_relaxed);
    }
    return (Mode)m;
}

void set_default_mode(Mode m) { g_mode.store((int)m, std::memory_order_relaxed); }

uint32_t worker_threads() {
    static const uint32_t n = [] {
        if (const char* e = std::getenv("ENET_HOST_THREADS")) return (uint32_t)std::max(0l, std::strtol(e, nullptr, 10));
        const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
        return std::min<uint32_t>(8, std::max<uint32_t>(1, hc / 2));
    }();
    return n;
}

// ------------------------------------------------------------------------------ engine
bool via_copies(Mode m) { return m != Mode::ZeroCopy; }

// ENET_HOST_TRACE=1: one stderr line per job with where its wall time went (tuning)
bool trace_on() {
    static const bool v = [] {
        const char* e = std::getenv("ENET_HOST_TRACE");
        return e && e[0] == '1';
    }();
    return v;
}
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool split_dirs(Mode m) { return m == Mode::SdmaSplit || m == Mode::SdmaSplitK || m == Mode::SdmaInZcOut; }
bool kern_streams(Mode m) { return m == Mode::SdmaSplitK || m == Mode::SdmaInZcOut; }
bool zc_out(Mode m) { return m == Mode::SdmaInZcOut; }  // kernels write host memory, no D2H

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    hipEvent_t kdone = nullptr;   // SdmaSplit*: the chunk's kernel has run (-> down stream)
    hipEvent_t indone = nullptr;  // SdmaSplitK: the chunk's H2D copies are done (-> slot stream)
    Pinned in, out, small;
    DevBuf d_in, d_out, d_small;
    // the chunk in flight
    bool busy = false;
    uint64_t seq = 0;  // chunk number within the job
    size_t c0 = 0, c1 = 0;
    uint64_t out_b = 0;
    bool direct_out = false;
    Layout lay{};
};

class Engine {
public:
    Engine(int dev, const Config& cfg) : dev_(dev), cfg_(cfg) {}
    ~Engine() {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev_);
        for (auto& sp : slots_) {
            Slot& s = *sp;
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.kdone) (void)hipEventDestroy(s.kdone);
            if (s.indone) (void)hipEventDestroy(s.indone);
            if (s.stream) (void)hipStreamDestroy(s.stream);
        }
        slots_.clear();
        for (hipStream_t x : {up_, kern_[0], kern_[1], down_})
            if (x) {
                (void)hipStreamSynchronize(x);
                (void)hipStreamDestroy(x);
            }
        table_.release();
        mid_.release();
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    void run(const Job& j);
    EngineStats stats() const {
        std::lock_guard<std::mutex> lk(mu_);
        return st_;
    }

private:
    Mode mode() const { return cfg_.mode >= 0 ? (Mode)cfg_.mode : default_mode(); }
    // Streams are created only when a job needs them: the box maps every stream of the process
    // (torch's included, when the library runs on torch's HIP runtime) onto GPU_MAX_HW_QUEUES = 4
    // hardware queues, and streams that share a queue serialise.  Eight streams (4 slot streams
    // that split modes never use + up, 2 kernel, down) put the H2D and D2H streams behind each
    // other: C2 e2e 12.4 GiB/s in bench.py (torch's runtime) against 18.5 with the library's own
    // runtime, same box (profiles/r04_e2e_variants_bench_process.txt, r04d_host_oneshots.jsonl).
    // Split modes: up + down (+ one kernel stream, + a second one for hash-chain-bound jobs).
    void setup_slots(uint32_t S, bool chain) {
        const Mode md = mode();
        auto make = [](hipStream_t& x) {
            if (!x) hip_check(hipStreamCreateWithFlags(&x, hipStreamNonBlocking), "hipStreamCreate");
        };
        while (slots_.size() < S) {
            slots_.emplace_back(std::make_unique<Slot>());
            Slot& s = *slots_.back();
            hip_check(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate");
            hip_check(hipEventCreateWithFlags(&s.kdone, hipEventDisableTiming), "hipEventCreate");
            hip_check(hipEventCreateWithFlags(&s.indone, hipEventDisableTiming), "hipEventCreate");
        }
        if (!split_dirs(md)) {
            for (uint32_t i = 0; i < S; ++i) make(slots_[i]->stream);
            return;
        }
        make(up_);
        if (!zc_out(md)) make(down_);
        if (kern_streams(md)) {
            make(kern_[0]);
            if (chain) make(kern_[1]);
        }
        nkern_ = (kern_streams(md) && chain) ? 2u : 1u;
    }
    Pool& pool() {
        if (!pool_) pool_ = std::make_unique<Pool>(worker_threads());
        return *pool_;
    }
    // byte-balanced parts of the records [a, b): parts of >= min_bytes each, at most workers + 1
    template <class LenF>
    std::vector<size_t> split(size_t a, size_t b, uint64_t bytes, LenF len) {
        const uint64_t min_bytes = 256u << 10;
        const uint64_t P = std::max<uint64_t>(1, std::min<uint64_t>(worker_threads() + 1, bytes / min_bytes));
        std::vector<size_t> cut{a};
        uint64_t acc = 0, next = bytes / P;
        for (size_t i = a; i < b && cut.size() < P; ++i) {
            acc += len(i);
            if (acc >= next && i + 1 < b) {
                cut.push_back(i + 1);
                next = bytes * cut.size() / P;
            }
        }
        cut.push_back(b);
        return cut;
    }
    struct CopyTask {
        int kind;  // 0 gather records [a, b) into base + at; 1 scatter them from base + at
        Slot* s;
        size_t a, b;
        uint64_t at;
        uint8_t* base;
    };
    void stage(Slot& s, const Job& j, size_t c0, size_t c1, uint64_t in_b, uint64_t out_b, std::vector<CopyTask>& tasks);
    void fill(Slot& s, const Job& j, uint64_t in_b, uint64_t out_b, uint32_t mx);
    void run_tasks(const Job& j, std::vector<CopyTask>& tasks);
    void launch(Slot& s, const Job& j, uint64_t in_b, uint32_t mx, bool mixed);
    void retire(Slot& s, const Job& j, std::vector<CopyTask>& tasks);

    int dev_;
    Config cfg_;
    mutable std::mutex mu_;
    std::vector<std::unique_ptr<Slot>> slots_;
    hipStream_t up_ = nullptr;    // SdmaSplit*: every H2D (and SdmaSplit: every kernel)
    hipStream_t kern_[2] = {};    // SdmaSplitK: the kernels (alternating by chunk for chain-bound jobs)
    uint32_t nkern_ = 1;          // kernel streams of the current job
    hipStream_t down_ = nullptr;  // SdmaSplit*: every D2H
    std::unique_ptr<Pool> pool_;
    EngineStats st_{};
    // per job
    const uint8_t* in_dev_ = nullptr;   // device view of the caller's input arena (direct in)
    uint8_t* out_dev_ = nullptr;        // ... output arena (direct out)
    std::vector<uint64_t> lin_, lout_;  // record lengths in / out
    DevBuf table_, mid_;                // session key table + HMAC midstates on the device
    double t_wait_ = 0, t_copy_ = 0, t_fill_ = 0, t_launch_ = 0;  // ENET_HOST_TRACE
    const uint8_t* in_ptr(const Job& j, size_t i) const {
        return j.in_spans.empty() ? j.in_base + j.in_off[i] : j.in_spans[i].data();
    }
};

// Stage a chunk into slot s: layout and device buffers, and the gather tasks that copy its
// records into the pinned input arena (run by run_tasks, together with the previous chunk's scatter)
void Engine::stage(Slot& s, const Job& j, size_t c0, size_t c1, uint64_t in_b, uint64_t out_b,
                   std::vector<CopyTask>& tasks) {
    const uint32_t m = (uint32_t)(c1 - c0);
    const Mode md = mode();
    s.lay = layout(j, m);
    s.small.ensure(s.lay.total);
    if (via_copies(md)) {
        s.d_small.ensure(s.lay.total);
        s.d_in.ensure(in_b);
        if (!zc_out(md)) s.d_out.ensure(out_b);
    }
    if (in_dev_) return;  // the caller's input arena is device-accessible: used in place
    s.in.ensure(in_b);
    const auto cut = split(c0, c1, in_b, [&](size_t i) { return lin_[i]; });
    uint64_t o = 0;
    for (size_t p = 0, i = c0; p + 1 < cut.size(); ++p) {
        tasks.push_back({0, &s, cut[p], cut[p + 1], o, s.in.h});
        for (; i < cut[p + 1]; ++i) o += lin_[i];
    }
    st_.gathered_bytes += in_b;
}

// The per-record small arrays of the chunk in slot s (rebased offsets, keys, nonces, ...) and its
// output staging; after run_tasks, so the previous chunk's scatter has read the old staging
void Engine::fill(Slot& s, const Job& j, uint64_t in_b, uint64_t out_b, uint32_t mx) {
    const size_t c0 = s.c0;
    const uint32_t m = (uint32_t)(s.c1 - s.c0);
    const Layout& l = s.lay;
    if (!s.direct_out) s.out.ensure(out_b);
    uint8_t* sm = s.small.h;
    auto* io = reinterpret_cast<uint64_t*>(sm + l.in_off);
    auto* oo = reinterpret_cast<uint64_t*>(sm + l.out_off);
    io[0] = oo[0] = 0;
    for (uint32_t k = 0; k < m; ++k) {
        io[k + 1] = io[k] + lin_[c0 + k];
        oo[k + 1] = oo[k] + lout_[c0 + k];
    }
    if (!j.session) std::memcpy(sm + l.keys, j.keys + (j.key_stride ? 32ull * c0 : 0ull), l.key_bytes);
    if (j.nonces) std::memcpy(sm + l.nonces, j.nonces + 12ull * c0, 12ull * m);
    else std::memset(sm + l.nonces, 0, 12ull * m);
    if (j.counters) std::memcpy(sm + l.ctr, j.counters + c0, 4ull * m);
    if (j.tags_in) std::memcpy(sm + l.tags_in, j.tags_in + 16ull * c0, 16ull * m);
    if (j.macs_in) std::memcpy(sm + l.macs_in, j.macs_in + 32ull * c0, 32ull * m);
    if (j.ids) std::memcpy(sm + l.ids, j.ids + 32ull * c0, 32ull * m);
    if (j.session) std::memcpy(sm + l.session, j.session + c0, 4ull * m);
    // mixed lengths: longest records first, so the serial per-record chains (SHA-256 is one lane
    // per record) start at once and short records fill in behind them
    const bool mixed = in_b != (uint64_t)m * mx;
    if (mixed) {
        auto* ord = reinterpret_cast<uint32_t*>(sm + l.order);
        for (uint32_t k = 0; k < m; ++k) ord[k] = k;
        const uint64_t* len = lin_.data() + c0;
        std::stable_sort(ord, ord + m, [len](uint32_t a, uint32_t b) { return len[a] > len[b]; });
    }
}

// Gather and scatter parts of (up to) two chunks in one pool pass: independent memory streams
void Engine::run_tasks(const Job& j, std::vector<CopyTask>& tasks) {
    if (tasks.empty()) return;
    pool().parallel(tasks.size(), [&](size_t t) {
        const CopyTask& c = tasks[t];
        uint64_t o = c.at;
        // an arena's records [a, b) are one contiguous range (record i = [off[i], off[i+1])):
        // one streaming copy instead of one per record
        if (c.kind == 0) {
            if (j.in_spans.empty()) {
                copy_out(c.base + o, j.in_base + j.in_off[c.a], j.in_off[c.b] - j.in_off[c.a]);
            } else {
                for (size_t i = c.a; i < c.b; ++i) {
                    copy_out(c.base + o, in_ptr(j, i), lin_[i]);
                    o += lin_[i];
                }
            }
        } else if (j.out_vecs || !j.out_each.empty()) {
            for (size_t i = c.a; i < c.b; ++i) {
                // assign from the range: one allocation and one copy, no zero fill first
                vec_of(j, i).assign(c.base + o, c.base + o + lout_[i]);
                o += lout_[i];
            }
        } else {
            copy_out(j.out_base + j.out_off[c.a], c.base + o, j.out_off[c.b] - j.out_off[c.a]);
        }
        fence_stores();  // streamed lines are globally visible before the device / caller reads them
    });
    tasks.clear();
}

void Engine::launch(Slot& s, const Job& j, uint64_t in_b, uint32_t mx, bool mixed) {
    const Mode md = mode();
    const Layout& l = s.lay;
    const uint32_t m = (uint32_t)(s.c1 - s.c0);
    // SdmaSplit: H2D + kernel of every chunk on the up stream, D2H on the down stream;
    // SdmaSplitK: H2D on up, kernels on kern, D2H on down
    hipStream_t st = split_dirs(md) ? up_ : s.stream;
    // device addresses of this chunk's arenas and small block
    const uint8_t* din;
    uint8_t* dout;
    uint8_t* sm;
    const uint8_t* src_in = in_dev_ ? nullptr : s.in.h;
    if (via_copies(md)) {
        const uint8_t* h_in = in_dev_ ? in_ptr(j, s.c0) : src_in;
        if (in_b) hip_check(hipMemcpyAsync(s.d_in.p, h_in, in_b, hipMemcpyHostToDevice, st), "H2D arena");
        hip_check(hipMemcpyAsync(s.d_small.p, s.small.h, l.in_end, hipMemcpyHostToDevice, st), "H2D small");
        if (kern_streams(md)) {
            hip_check(hipEventRecord(s.indone, st), "hipEventRecord");
            // two kernel streams for hash-chain-bound jobs: consecutive chunks' chains overlap
            st = kern_[nkern_ > 1 ? (s.seq & 1) : 0];
            hip_check(hipStreamWaitEvent(st, s.indone, 0), "hipStreamWaitEvent");
        }
        din = s.d_in.p;
        // SdmaInZcOut: outputs straight into the caller's arena (device view) or the pinned staging
        dout = !zc_out(md) ? s.d_out.p : s.direct_out ? out_dev_ + j.out_off[s.c0] : s.out.d;
        sm = s.d_small.p;
    } else {
        din = in_dev_ ? in_dev_ + j.in_off[s.c0] : s.in.d;
        dout = s.direct_out ? out_dev_ + j.out_off[s.c0] : s.out.d;
        sm = s.small.d;
    }
    if (!din) din = sm;  // an all-empty chunk: any valid address
    if (!dout) dout = sm + l.ok;
    enet_records r{};
    r.count = m;
    r.in_offsets = reinterpret_cast<const uint64_t*>(sm + l.in_off);
    r.out_offsets = reinterpret_cast<const uint64_t*>(sm + l.out_off);
    r.in = din;
    r.out = dout;
    r.keys = j.session ? table_.p : sm + l.keys;
    r.key_stride = j.session ? 32 : j.key_stride;
    r.nonces = sm + l.nonces;
    r.order = mixed ? reinterpret_cast<const uint32_t*>(sm + l.order) : nullptr;
    r.total_bytes_hint = in_b;
    r.max_len_hint = mx;
    // the per-record outputs (tags, MACs, ok: <= 49 bytes a record) go straight from the kernel
    // into the pinned host small block over PCIe: the down stream then carries only the arena
    // copies (a small D2H behind every chunk's arena copy held the stream ~55 us per chunk,
    // profiles/r04_c2_copy_trace_summary.jsonl)
    uint8_t* smo = via_copies(md) ? s.small.d : sm;
    uint8_t* tags_out = smo + l.tags_out;
    uint8_t* macs_out = smo + l.macs_out;
    uint8_t* ok = smo + l.ok;
    const uint8_t* tags_in = j.tags_in ? sm + l.tags_in : nullptr;
    const uint8_t* macs_in = j.macs_in ? sm + l.macs_in : nullptr;
    const uint8_t* ids = j.ids ? sm + l.ids : nullptr;
    const auto* sess = reinterpret_cast<const uint32_t*>(sm + l.session);
    const auto* mid = reinterpret_cast<const uint32_t*>(mid_.p);
    switch (j.op) {
        case Op::Xor:
            enet_check(enet_chacha20_xor_batch(&r, j.counters ? reinterpret_cast<const uint32_t*>(sm + l.ctr) : nullptr, st),
                       "chacha20_xor");
            break;
        case Op::AeadSeal: enet_check(enet_aead_seal_batch(&r, nullptr, nullptr, tags_out, st), "aead_seal"); break;
        case Op::AeadOpen: enet_check(enet_aead_open_batch(&r, nullptr, nullptr, tags_in, ok, st), "aead_open"); break;
        case Op::AeadHmacSeal: enet_check(enet_aead_hmac_seal_batch(&r, tags_out, macs_out, st), "aead_hmac_seal"); break;
        case Op::AeadHmacOpen:
            enet_check(enet_aead_hmac_open_batch(&r, tags_in, macs_in, ok, st), "aead_hmac_open");
            break;
        case Op::FrameSeal: enet_check(enet_frame_seal_batch(&r, st), "frame_seal"); break;
        case Op::FrameOpen: enet_check(enet_frame_open_batch(&r, macs_out, ok, st), "frame_open"); break;
        case Op::WireSeal:
            if (j.session) enet_check(enet_wire_seal_batch_sessions(&r, sess, j.n_sessions, mid, st), "wire_seal_sessions");
            else enet_check(enet_wire_seal_batch(&r, st), "wire_seal");
            break;
        case Op::WireOpen:
            if (j.session)
                enet_check(enet_wire_open_batch_sessions(&r, sess, j.n_sessions, mid, macs_out, ok, st), "wire_open_sessions");
            else enet_check(enet_wire_open_batch(&r, macs_out, ok, st), "wire_open");
            break;
        case Op::ChunkStore: enet_check(enet_chunk_store_batch(&r, ids, macs_out, st), "chunk_store"); break;
        case Op::ChunkFetch: enet_check(enet_chunk_fetch_batch(&r, ids, macs_in, ok, st), "chunk_fetch"); break;
    }
    if (split_dirs(md) && !zc_out(md)) {
        hip_check(hipEventRecord(s.kdone, st), "hipEventRecord");
        st = down_;
        hip_check(hipStreamWaitEvent(st, s.kdone, 0), "hipStreamWaitEvent");
    }
    if (via_copies(md) && !zc_out(md)) {
        uint8_t* h_out = s.direct_out ? j.out_base + j.out_off[s.c0] : s.out.h;
        if (s.out_b) hip_check(hipMemcpyAsync(h_out, s.d_out.p, s.out_b, hipMemcpyDeviceToHost, st), "D2H arena");
    }
    hip_check(hipEventRecord(s.done, st), "hipEventRecord");
    s.busy = true;
}

// The chunk in slot s is done on the device: wait for it, copy its small outputs, and queue the
// scatter of its records (run by run_tasks)
void Engine::retire(Slot& s, const Job& j, std::vector<CopyTask>& tasks) {
    s.busy = false;
    const double t0 = now_s();
    hip_check(hipEventSynchronize(s.done), "chunk sync");
    t_wait_ += now_s() - t0;
    const size_t c0 = s.c0, c1 = s.c1;
    const uint32_t m = (uint32_t)(c1 - c0);
    const Layout& l = s.lay;
    const uint8_t* sm = s.small.h;
    if (j.tags_out && (j.op == Op::AeadSeal || j.op == Op::AeadHmacSeal))
        std::memcpy(j.tags_out + 16ull * c0, sm + l.tags_out, 16ull * m);
    if (j.macs_out && (j.op == Op::AeadHmacSeal || j.op == Op::FrameOpen || j.op == Op::WireOpen || j.op == Op::ChunkStore))
        std::memcpy(j.macs_out + 32ull * c0, sm + l.macs_out, 32ull * m);
    if (j.ok_out && is_open(j.op)) std::memcpy(j.ok_out + c0, sm + l.ok, m);
    if (s.direct_out || s.out_b == 0) {
        if (j.out_vecs || !j.out_each.empty())
            for (size_t i = c0; i < c1; ++i) vec_of(j, i).clear();
        return;
    }
    const auto cut = split(c0, c1, s.out_b, [&](size_t i) { return lout_[i]; });
    uint64_t o = 0;
    for (size_t p = 0, i = c0; p + 1 < cut.size(); ++p) {
        tasks.push_back({1, &s, cut[p], cut[p + 1], o, s.out.h});
        for (; i < cut[p + 1]; ++i) o += lout_[i];
    }
    st_.scattered_bytes += s.out_b;
}

void Engine::run(const Job& j) {
    const size_t n = j.n;
    if (n == 0) return;
    if (n > 0xFFFFFFFFull) throw std::invalid_argument("enet host batch: more than 2^32 - 1 records");
    if (!j.in_spans.empty() ? j.in_spans.size() != n : !j.in_off)
        throw std::invalid_argument("enet host batch: input records missing");
    const bool vec_out = j.out_vecs || !j.out_each.empty();
    if (!j.out_each.empty() && j.out_each.size() != n) throw std::invalid_argument("enet host batch: out_each size");
    if (!vec_out && !j.out_off) throw std::invalid_argument("enet host batch: output offsets missing");
    if (!j.keys) throw std::invalid_argument("enet host batch: keys missing");
    if (j.key_stride != 0 && j.key_stride != 32) throw std::invalid_argument("enet host batch: key_stride must be 0 or 32");
    if (!j.nonces && j.op != Op::WireOpen) throw std::invalid_argument("enet host batch: nonces missing");
    if (j.session && !j.n_sessions) throw std::invalid_argument("enet host batch: empty session table");
    std::lock_guard<std::mutex> lk(mu_);
    int prev = -1;
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev_) hip_check(hipSetDevice(dev_), "hipSetDevice");
    struct Restore {
        int prev, dev;
        ~Restore() {
            if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
        }
    } restore{prev, dev_};

    const Mode md = mode();
    static const uint32_t env_slots = [] {
        const char* e = std::getenv("ENET_HOST_SLOTS");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
    }();
    const uint32_t S = std::min<uint32_t>(cfg_.slots ? cfg_.slots : env_slots ? env_slots : 4u, 8);
    // lengths
    const int64_t delta = delta_of(j.op);
    lin_.resize(n);
    lout_.resize(n);
    uint64_t in_total = 0, out_total = 0, max_len = 0;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t a = j.in_spans.empty() ? j.in_off[i + 1] - j.in_off[i] : j.in_spans[i].size();
        if (j.in_spans.empty() && j.in_off[i + 1] < j.in_off[i])
            throw std::invalid_argument("enet host batch: input offsets must be non-decreasing");
        lin_[i] = a;
        max_len = std::max(max_len, a);
        lout_[i] = (uint64_t)std::max<int64_t>(0, (int64_t)a + delta);
        in_total += a;
        out_total += lout_[i];
        if (!vec_out && j.out_off[i + 1] - j.out_off[i] != lout_[i])
            throw std::invalid_argument("enet host batch: output offsets do not give the op's output lengths");
    }
    if (!vec_out && !j.out_base && out_total) throw std::invalid_argument("enet host batch: output arena missing");
    if (j.in_spans.empty() && !j.in_base && in_total) throw std::invalid_argument("enet host batch: input arena missing");
    if (j.out_vecs) j.out_vecs->resize(n);
    // in place where the caller's arenas are device-accessible
    in_dev_ = j.in_spans.empty() ? device_view(j.in_base + j.in_off[0], in_total) : nullptr;
    out_dev_ = vec_out ? nullptr : device_view(j.out_base + j.out_off[0], out_total);
    if (in_dev_) in_dev_ -= j.in_off[0];
    if (out_dev_) out_dev_ -= j.out_off[0];
    const bool direct_out = out_dev_ != nullptr;
    // Long records behind a hash (HMAC / SHA-256 is one serial chain per record: 1.9 ms for 64 KiB)
    // bound every chunk's kernel by that chain
    const bool hashes = j.op != Op::Xor && j.op != Op::AeadSeal && j.op != Op::AeadOpen;
    const uint64_t chain = (hashes && max_len >= (16u << 10)) ? 4 : 1;
    setup_slots(S, chain > 1);
    // sessions: key table and its HMAC midstates on the device, once per job
    if (j.session) {
        table_.ensure(32ull * j.n_sessions);
        mid_.ensure(64ull * j.n_sessions);
        hipStream_t s0 = split_dirs(md) ? up_ : slots_[0]->stream;
        hip_check(hipMemcpyAsync(table_.p, j.keys, 32ull * j.n_sessions, hipMemcpyHostToDevice, s0), "H2D sessions");
        enet_check(enet_hmac_midstates(table_.p, j.n_sessions, reinterpret_cast<uint32_t*>(mid_.p), s0), "midstates");
        hip_check(hipStreamSynchronize(s0), "session setup");
    }
    // chunk size: big enough to amortise a launch, small enough that the gather / scatter of
    // neighbouring chunks overlaps it; a job with nothing to gather or scatter takes big chunks
    // (gathered records, 16 vs 32 MiB, three interleaved pairs on one box: C2 16.2-18.0 vs
    // 13.8-17.5, C3 wire 14.9-16.4 vs 14.1-17.7 GiB/s, profiles/r04_batch_bench_gather_chunk_ab.jsonl).
    // Chain-bound jobs take 4x bigger chunks, so every chunk's kernel lasts at least its chain
    // (C5 share, 4 slots, two kernel streams: 128 / 256 MiB chunks -> 18.6 / 17.4 GiB/s,
    // profiles/r04_host_sweep_p7b.jsonl; one kernel stream peaked at 256 MiB).
    uint64_t chunk = cfg_.chunk_bytes;
    if (!chunk) chunk = (in_dev_ && direct_out) ? (md == Mode::ZeroCopy ? (256ull << 20) : (32ull << 20) * chain)
                                                : (md == Mode::ZeroCopy ? (32ull << 20) : (16ull << 20) * std::min<uint64_t>(chain, 4));
    if (!cfg_.chunk_bytes)
        if (const char* e = std::getenv("ENET_HOST_CHUNK_MIB")) chunk = std::max(1ull, std::strtoull(e, nullptr, 10)) << 20;
    st_.jobs += 1;
    st_.records += n;
    st_.in_bytes += in_total;
    st_.out_bytes += out_total;
    size_t c0 = 0, k = 0;
    std::exception_ptr err;
    t_wait_ = t_copy_ = t_fill_ = t_launch_ = 0;
    const double t_job = now_s();
    std::vector<CopyTask> tasks;
    uint64_t left = in_total;
    try {
        while (c0 < n) {
            // ramped chunk sizes: the first chunks (nothing to overlap their copy in yet) are
            // small, 1/8 .. 1/2 of the steady chunk, so the pipeline fills in a fraction of a
            // chunk's time.  Ramping down at the end as well measured ~1 % slower (every extra
            // chunk pays its small copies and event hops; C2 e2e 19.1-19.3 vs 19.46, four
            // interleaved pairs, profiles/r04_host_ramp_ab.jsonl) and costs a hash-chain-bound
            // job one more ~2 ms chain per extra chunk (C5 share 17.6-17.8 vs 18.4-18.6,
            // r04_host_ramp_c5_ab.jsonl), so it is off by default.
            // ENET_HOST_RAMP (tuning): bit 0 ramp-up, bit 1 ramp-down for unhashed jobs, bit 2
            // ramp-down for hash-chain-bound jobs.
            uint64_t target = chunk;
            static const unsigned ramp = [] {
                const char* e = std::getenv("ENET_HOST_RAMP");
                return e ? (unsigned)std::strtoul(e, nullptr, 10) & 7u : 1u;
            }();
            if (k < 3 && (ramp & 1u)) target = std::max<uint64_t>(chunk >> (3 - k), 1);
            if (left < 2 * chunk && (ramp & (chain == 1 ? 2u : 4u)))
                target = std::min<uint64_t>(target, std::max<uint64_t>(left / 2, chunk >> 3));
            size_t c1 = c0 + 1;
            uint64_t ib = lin_[c0], ob = lout_[c0];
            uint32_t mx = (uint32_t)std::min<uint64_t>(lin_[c0], 0xFFFFFFFFu);
            while (c1 < n && ib + lin_[c1] <= target && ob + lout_[c1] <= target + (target >> 2) &&
                   c1 - c0 < (1u << 22)) {
                ib += lin_[c1];
                ob += lout_[c1];
                mx = std::max<uint32_t>(mx, (uint32_t)std::min<uint64_t>(lin_[c1], 0xFFFFFFFFu));
                ++c1;
            }
            left -= ib;
            Slot& s = *slots_[k % S];
            ++k;
            if (s.busy) retire(s, j, tasks);  // its scatter runs in the same pass as this gather
            s.c0 = c0;
            s.c1 = c1;
            s.seq = k - 1;
            s.out_b = ob;
            s.direct_out = direct_out;
            const double t0 = now_s();
            stage(s, j, c0, c1, ib, ob, tasks);
            run_tasks(j, tasks);
            const double t1 = now_s();
            fill(s, j, ib, ob, mx);
            const double t2 = now_s();
            launch(s, j, ib, mx, ib != (uint64_t)(c1 - c0) * mx);
            t_copy_ += t1 - t0;
            t_fill_ += t2 - t1;
            t_launch_ += now_s() - t2;
            st_.chunks += 1;
            if (in_dev_) st_.direct_in += 1;
            if (direct_out) st_.direct_out += 1;
            c0 = c1;
        }
        for (size_t q = 0; q < S; ++q) {
            Slot& s = *slots_[(k + q) % S];
            if (s.busy) {
                retire(s, j, tasks);
                const double t0 = now_s();
                run_tasks(j, tasks);
                t_copy_ += now_s() - t0;
            }
        }
    } catch (...) {
        err = std::current_exception();
    }
    if (trace_on())
        std::fprintf(stderr,
                     "[enet host] op %d mode %d n %zu in %llu out %llu chunks %zu slots %u: total %.3f ms = "
                     "gather/scatter %.3f, small arrays %.3f, launch %.3f, wait %.3f ms (direct in %d out %d)\n",
                     (int)j.op, (int)md, n, (unsigned long long)in_total, (unsigned long long)out_total, k, S,
                     1e3 * (now_s() - t_job), 1e3 * t_copy_, 1e3 * t_fill_, 1e3 * t_launch_, 1e3 * t_wait_,
                     in_dev_ != nullptr, (int)direct_out);
    if (err) {  // drain whatever is still in flight before the caller's buffers go away
        for (auto& s : slots_) {
            if (s->stream) (void)hipStreamSynchronize(s->stream);
            s->busy = false;
        }
        for (hipStream_t x : {up_, kern_[0], kern_[1], down_})
            if (x) (void)hipStreamSynchronize(x);
        std::rethrow_exception(err);
    }
}

// ------------------------------------------------------------------------------ API
Engine& shared_engine(int dev) {
    static std::mutex mu;
    static std::map<int, Engine*>* engines = new std::map<int, Engine*>();  // never destroyed: no HIP at exit
    std::lock_guard<std::mutex> lk(mu);
    auto it = engines->find(dev);
    if (it != engines->end()) return *it->second;
    Engine* e = new Engine(dev, Config{});
    (*engines)[dev] = e;
    return *e;
}

Engine* create_engine(int dev, const Config& cfg) { return new Engine(dev, cfg); }
void destroy_engine(Engine* e) { delete e; }
void run(Engine& e, const Job& job) { e.run(job); }
EngineStats stats(const Engine& e) { return e.stats(); }

}  // namespace enet::hb
