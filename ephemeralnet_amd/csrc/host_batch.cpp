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
#include "enet_internal.hpp"
#include "host_topo.hpp"

#include <pthread.h>

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
    // workers threads bound to `cpus` (empty: unbound); spin: whether they spin briefly for the
    // next task set before sleeping (only when every thread of the process's pools has a CPU)
    Pool(unsigned workers, std::vector<int> cpus, bool spin) : cpus_(std::move(cpus)), spin_(spin) {
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
    size_t workers() const { return th_.size(); }
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
    void bind() {
        if (cpus_.empty()) return;
        const int mx = cpus_.back() + 1;
        cpu_set_t* set = CPU_ALLOC(mx);
        if (!set) return;
        const size_t sz = CPU_ALLOC_SIZE(mx);
        CPU_ZERO_S(sz, set);
        for (int c : cpus_) CPU_SET_S(c, sz, set);
        (void)pthread_setaffinity_np(pthread_self(), sz, set);
        CPU_FREE(set);
    }
    void loop() {
        bind();
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            if (spin_ && !stop_ && !(task_ && gen_ != seen)) {
                // a pipeline hands out a task set every few hundred microseconds: spin ~20 us for
                // the next one before sleeping (a futex wake-up per worker per set cost ~1.5 ms per
                // 256 MiB job) -- only when the plan gave every pool thread a CPU of its own
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
    std::vector<int> cpus_;
    bool spin_;
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
// caches the session threads use (tools build: ENET_HOST_NT=0 selects plain memcpy).  The caller issues a store
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
#ifdef ENET_TOOLS_BUILD
        const char* e = std::getenv("ENET_HOST_NT");  // tools build: 0 = plain memcpy (A/B)
        if (e && e[0] == '0') return false;
#endif
        return (bool)__builtin_cpu_supports("avx512f");
    }();
    return v;
}

void copy_out(uint8_t* d, const uint8_t* s, size_t n) {
    if (n >= 512 && use_nt()) copy_nt512(d, s, n);
    else if (n) std::memcpy(d, s, n);
}

void fence_stores() { _mm_sfence(); }

// ------------------------------------------------------------------------------ buffers
struct Pinned {  // pinned, device-mapped host memory on the engine's node, grow-only
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    size_t cap = 0;
    // node: topo::target_node of the engine's device (-1: hipHostMalloc places it); bytes: the
    // engine's running total of staging held
    void ensure(size_t n, int node, uint64_t& bytes) {
        if (n <= cap) return;
        release(bytes);
        const size_t c = std::max<size_t>(n + (n >> 3), 64u << 10);
        void* dp = nullptr;
        h = static_cast<uint8_t*>(topo::alloc_pinned(c, node, &dp));
        d = static_cast<uint8_t*>(dp);
        cap = c;
        bytes += c;
    }
    void release(uint64_t& bytes) {
        if (h) {
            topo::free_pinned(h);
            bytes -= cap;
        }
        h = d = nullptr;
        cap = 0;
    }
    ~Pinned() {
        if (h) topo::free_pinned(h);
    }
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

// Device address of [p, p + n) when the WHOLE range lies in one device-accessible allocation
// (hipHostMalloc'ed / registered host memory, device or managed memory); nullptr otherwise (the
// range is then gathered / scattered through the pinned staging).  Checking the first and last
// byte is not enough: an arena built from adjacent blocks can be pinned at both ends with a
// pageable page between, which a kernel would fault on (no XNACK).  So the allocation holding p
// is looked up (its base and size) and must cover the whole range.
uint8_t* device_view(const uint8_t* p, uint64_t n) {
    if (!p || n == 0) return nullptr;
    if (uint8_t* d = topo::known_device_view(p, n)) return d;  // our own pinned / registered blocks
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable: clear the sticky "invalid value"
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost && a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged)
        return nullptr;
    uint8_t* dp = static_cast<uint8_t*>(a.devicePointer);
    if (!dp) return nullptr;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, dp) != hipSuccess || !base) {
        (void)hipGetLastError();
        // the same facts through the pointer-attribute query
        void* start = nullptr;
        size_t len = 0;
        if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, dp) != hipSuccess ||
            hipPointerGetAttribute(&len, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, dp) != hipSuccess || !start) {
            (void)hipGetLastError();
            return nullptr;
        }
        base = start;
        size = len;
    }
    const uint8_t* b = static_cast<const uint8_t*>(base);
    if (dp < b || (uint64_t)(dp - b) > size || n > size - (uint64_t)(dp - b)) return nullptr;
    return dp;
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

std::atomic<int> g_mode{-2};  // -2: not read yet; -1: auto; else the fixed mode
std::mutex g_mode_mu;
std::atomic<int> g_engines{0};  // engines alive in the process (they share the CPU budget)

std::vector<uint8_t>& vec_of(const Job& j, size_t i) { return j.out_vecs ? (*j.out_vecs)[i] : *j.out_each[i]; }

}  // namespace

int64_t out_delta(Op op) { return delta_of(op); }

void copy_streaming(uint8_t* d, const uint8_t* s, size_t n) { copy_out(d, s, n); }

bool valid_mode(int m) { return m == (int)Mode::ZeroCopy || m == (int)Mode::SdmaSplitK || m == (int)Mode::SdmaInZcOut; }

// The auto mode's decision for jobs whose output the device writes in place (caller-pinned
// output arenas): SdmaInZcOut when it moved more than 3 % more bytes per second than SdmaSplitK,
// else SdmaSplitK; undecided (-1) until both have rates.
int mode_for(const AutoRates& r) {
    if (!(r.splitk_gibs > 0) || !(r.zcout_gibs > 0)) return -1;
    return r.zcout_gibs > 1.03 * r.splitk_gibs ? (int)Mode::SdmaInZcOut : (int)Mode::SdmaSplitK;
}

namespace {

// per device: the rates sampled so far for in-place-output jobs, and the decision
struct AutoState {
    std::mutex mu;
    AutoRates r;
    std::atomic<int> decided{-1};
};
AutoState& auto_state(int dev) {
    static std::mutex mu;
    static auto* m = new std::map<int, AutoState*>();
    std::lock_guard<std::mutex> lk(mu);
    auto& s = (*m)[dev];
    if (!s) s = new AutoState();
    return *s;
}
std::atomic<unsigned> g_auto_epoch{0};  // enet_host_set_mode(-1) forgets every device's decision

constexpr uint64_t kAutoMinBytes = 64ull << 20;  // a job shorter than this is mostly ramp-up
constexpr int kAutoSamples = 2;                  // jobs per mode before deciding (best of them)

}  // namespace

int fixed_mode() {
    int m = g_mode.load(std::memory_order_acquire);
    if (m != -2) return m;  // set (or auto) by enet_host_set_mode
    std::lock_guard<std::mutex> lk(g_mode_mu);
    m = g_mode.load(std::memory_order_relaxed);
    if (m != -2) return m;
    m = -1;
    const char* e = std::getenv("ENET_HOST_MODE");
    if (e && *e) {
        m = std::strcmp(e, "zc") == 0 || std::strcmp(e, "0") == 0         ? (int)Mode::ZeroCopy
            : std::strcmp(e, "splitk") == 0 || std::strcmp(e, "3") == 0    ? (int)Mode::SdmaSplitK
            : std::strcmp(e, "zcout") == 0 || std::strcmp(e, "4") == 0     ? (int)Mode::SdmaInZcOut
                                                                          : -1;
    }
    g_mode.store(m, std::memory_order_release);
    return m;
}

void set_default_mode(int m) {
    if (m < 0) {  // auto: decisions are learned again
        std::lock_guard<std::mutex> lk(g_mode_mu);
        g_auto_epoch.fetch_add(1, std::memory_order_acq_rel);
        g_mode.store(-1, std::memory_order_release);
        return;
    }
    g_mode.store(m, std::memory_order_release);
}

AutoRates auto_rates(int dev) {
    AutoState& a = auto_state(dev);
    std::lock_guard<std::mutex> lk(a.mu);
    AutoRates r = a.r;
    r.mode = a.decided.load();
    return r;
}

// The mode of one auto job, and whether its rate is to be recorded (sample: 0 = SdmaSplitK,
// 1 = SdmaInZcOut, -1 = not a sample)
Mode auto_mode(int dev, bool out_in_place, uint64_t bytes, bool warm, int* sample, unsigned* epoch) {
    *sample = -1;
    if (!out_in_place) return Mode::SdmaSplitK;
    AutoState& a = auto_state(dev);
    std::lock_guard<std::mutex> lk(a.mu);
    const unsigned ep = g_auto_epoch.load(std::memory_order_acquire);
    if (a.r.epoch != ep) {  // enet_host_set_mode(-1) since the last look: start over
        a.r = AutoRates{};
        a.r.epoch = ep;
        a.decided.store(-1);
    }
    const int d = a.decided.load();
    if (d >= 0) return (Mode)d;
    if (!warm || bytes < kAutoMinBytes) return Mode::SdmaSplitK;
    *sample = a.r.samples_splitk <= a.r.samples_zcout ? 0 : 1;  // alternate, SdmaSplitK first
    *epoch = ep;
    return *sample == 0 ? Mode::SdmaSplitK : Mode::SdmaInZcOut;
}

void auto_record(int dev, int sample, unsigned epoch, double gibs) {
    AutoState& a = auto_state(dev);
    std::lock_guard<std::mutex> lk(a.mu);
    if (a.r.epoch != epoch || a.decided.load() >= 0) return;
    if (sample == 0) {
        a.r.splitk_gibs = std::max(a.r.splitk_gibs, gibs);
        ++a.r.samples_splitk;
    } else {
        a.r.zcout_gibs = std::max(a.r.zcout_gibs, gibs);
        ++a.r.samples_zcout;
    }
    if (a.r.samples_splitk >= kAutoSamples && a.r.samples_zcout >= kAutoSamples) a.decided.store(mode_for(a.r));
}

// enet_host_mode_probe: the same choice made up front with a synthetic job -- 256 MiB of 4 KiB
// AEAD seals from and to caller-pinned host memory, alternating modes, best of three each; the
// result becomes the device's auto decision.
AutoRates probe_mode(int dev) {
    int prev = -1;
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (dev < 0) dev = prev;
    constexpr size_t kRec = 4096, kN = 65536, kBytes = kRec * kN;
    constexpr int kRounds = 3;
    const int node = topo::target_node(dev);
    uint8_t* in = nullptr;
    uint8_t* out = nullptr;
    Engine* eng[2] = {};
    std::exception_ptr err;
    AutoRates r;
    try {
        in = static_cast<uint8_t*>(topo::alloc_pinned(kBytes, node, nullptr));
        out = static_cast<uint8_t*>(topo::alloc_pinned(kBytes, node, nullptr));
        std::memset(in, 0x5a, kBytes);
        std::vector<uint64_t> off(kN + 1);
        for (size_t i = 0; i <= kN; ++i) off[i] = i * kRec;
        std::vector<uint8_t> keys(32 * kN, 7), nonces(12 * kN, 1), tags(16 * kN);
        Job j;
        j.op = Op::AeadSeal;
        j.n = kN;
        j.in_base = in;
        j.in_off = off.data();
        j.out_base = out;
        j.out_off = off.data();
        j.keys = keys.data();
        j.nonces = nonces.data();
        j.tags_out = tags.data();
        const Mode modes[2] = {Mode::SdmaSplitK, Mode::SdmaInZcOut};
        for (int m = 0; m < 2; ++m) {
            Config c;
            c.mode = (int)modes[m];
            eng[m] = create_engine(dev, c);
            run(*eng[m], j);  // warm: staging, streams, first launches
        }
        for (int k = 0; k < kRounds; ++k)
            for (int m = 0; m < 2; ++m) {
                const auto t0 = std::chrono::steady_clock::now();
                run(*eng[m], j);
                const double g = (double)kBytes / 1073741824.0 /
                                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (m == 0) r.splitk_gibs = std::max(r.splitk_gibs, g), ++r.samples_splitk;
                else r.zcout_gibs = std::max(r.zcout_gibs, g), ++r.samples_zcout;
            }
    } catch (...) {
        err = std::current_exception();
    }
    for (Engine* e : eng)
        if (e) destroy_engine(e);
    if (in) topo::free_pinned(in);
    if (out) topo::free_pinned(out);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (err) std::rethrow_exception(err);
    r.mode = mode_for(r);
    AutoState& a = auto_state(dev);
    std::lock_guard<std::mutex> lk(a.mu);
    const unsigned ep = g_auto_epoch.load(std::memory_order_acquire);
    a.r = r;
    a.r.epoch = ep;
    a.decided.store(r.mode);
    return r;
}

// ------------------------------------------------------------------------------ engine
bool via_copies(Mode m) { return m != Mode::ZeroCopy; }  // SDMA H2D (up), kernels, [D2H (down)]
bool zc_out(Mode m) { return m == Mode::SdmaInZcOut; }    // kernels write host memory, no D2H

// ENET_HOST_TRACE=1: one stderr line per job with where its wall time went (diagnosis)
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

#ifdef ENET_TOOLS_BUILD
// tools build only (A/B of the pipeline shape): ENET_HOST_SLOTS, ENET_HOST_CHUNK_MIB, ENET_HOST_RAMP
uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::strtoull(e, nullptr, 10) : dflt;
}
#endif

struct Slot {
    hipStream_t stream = nullptr;  // ZeroCopy: the slot's stream
    hipEvent_t done = nullptr;
    hipEvent_t kdone = nullptr;   // SdmaSplitK: the chunk's kernel has run (-> down stream)
    hipEvent_t indone = nullptr;  // SdmaSplitK / SdmaInZcOut: the chunk's H2D copies are done
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
    Engine(int dev, const Config& cfg) : dev_(dev), cfg_(cfg) {
        g_engines.fetch_add(1);
        node_ = topo::target_node(dev);
        st_.target_node = node_;
        st_.device_node = topo::device_numa_node(dev);
    }
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
        pool_.reset();
        g_engines.fetch_sub(1);
    }
    void run(const Job& j);
    EngineStats stats() const {
        std::lock_guard<std::mutex> lk(mu_);
        return st_;
    }
    void run_locked(const Job& j);  // run() with mu_ held

private:
    // Streams are created only when a job needs them: the box maps every stream of the process
    // (torch's included, when the library runs on torch's HIP runtime) onto GPU_MAX_HW_QUEUES = 4
    // hardware queues, and streams that share a queue serialise.  Eight streams put the H2D and
    // D2H streams behind each other: C2 e2e 12.4 GiB/s in bench.py (torch's runtime) against 18.5
    // with the library's own runtime, same box (profiles/r04_e2e_variants_bench_process.txt).
    // SDMA modes: up + down (+ one kernel stream, + a second one for hash-chain-bound jobs);
    // ZeroCopy: one stream per slot.
    void setup_slots(uint32_t S, bool chain) {
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
        if (!via_copies(md_)) {
            for (uint32_t i = 0; i < S; ++i) make(slots_[i]->stream);
            nkern_ = 1;
            return;
        }
        make(up_);
        if (!zc_out(md_)) make(down_);
        make(kern_[0]);
        if (chain) make(kern_[1]);
        nkern_ = chain ? 2u : 1u;
    }
    Pool& pool() {
        if (!pool_) {
            // the threads go where the staging is (the device's node unless ENET_HOST_NUMA moved it)
            const int tnode = node_ >= 0 ? node_ : st_.device_node;
            const topo::Plan p = topo::plan(topo::node_cpus(tnode), topo::allowed_cpus(),
                                            topo::cgroup_quota_cpus(), topo::env_cpus(),
                                            (uint32_t)std::max(1, g_engines.load()));
            uint32_t w = p.workers;
#ifdef ENET_TOOLS_BUILD
            if (const char* e = std::getenv("ENET_HOST_THREADS")) w = (uint32_t)std::strtoul(e, nullptr, 10);
#endif
            pool_ = std::make_unique<Pool>(w, p.cpus, p.spin);
            st_.workers = w;
            st_.cpu_budget = p.budget;
            st_.spin = p.spin ? 1 : 0;
        }
        return *pool_;
    }
    // byte-balanced parts of the records [a, b): parts of >= min_bytes each, at most workers + 1
    template <class LenF>
    std::vector<size_t> split(size_t a, size_t b, uint64_t bytes, LenF len) {
        const uint64_t min_bytes = 256u << 10;
        const uint64_t P = std::max<uint64_t>(1, std::min<uint64_t>(pool().workers() + 1, bytes / min_bytes));
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
    void ensure(Pinned& p, size_t n) {
        const bool first = p.h == nullptr && st_.staging_node < 0;
        p.ensure(n, node_, st_.pinned_bytes);
        if (first && p.h) st_.staging_node = topo::page_node(p.h);
    }
    void stage(Slot& s, const Job& j, size_t c0, size_t c1, uint64_t in_b, uint64_t out_b, std::vector<CopyTask>& tasks);
    void fill(Slot& s, const Job& j, uint64_t in_b, uint64_t out_b, uint32_t mx);
    void run_tasks(const Job& j, std::vector<CopyTask>& tasks);
    void launch(Slot& s, const Job& j, uint64_t in_b, uint32_t mx, bool mixed);
    void retire(Slot& s, const Job& j, std::vector<CopyTask>& tasks);

    int dev_;
    Config cfg_;
    int node_ = -1;  // where this engine's pinned staging goes (topo::target_node)
    mutable std::mutex mu_;
    std::vector<std::unique_ptr<Slot>> slots_;
    hipStream_t up_ = nullptr;    // SDMA modes: every H2D
    hipStream_t kern_[2] = {};    // SDMA modes: the kernels (alternating by chunk for chain-bound jobs)
    uint32_t nkern_ = 1;          // kernel streams of the current job
    hipStream_t down_ = nullptr;  // SdmaSplitK: every D2H
    std::unique_ptr<Pool> pool_;
    EngineStats st_{};
    // per job (under mu_)
    Mode md_ = Mode::SdmaSplitK;        // the job's mode, read once at its start
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
    s.lay = layout(j, m);
    ensure(s.small, s.lay.total);
    if (via_copies(md_)) {
        s.d_small.ensure(s.lay.total);
        s.d_in.ensure(in_b);
        if (!zc_out(md_)) s.d_out.ensure(out_b);
    }
    if (in_dev_) return;  // the caller's input arena is device-accessible: used in place
    ensure(s.in, in_b);
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
    if (!s.direct_out) ensure(s.out, out_b);
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
    const Mode md = md_;
    const Layout& l = s.lay;
    const uint32_t m = (uint32_t)(s.c1 - s.c0);
    // SDMA modes: H2D on up, kernels on kern, D2H on down; ZeroCopy: the slot's stream
    hipStream_t st = via_copies(md) ? up_ : s.stream;
    // device addresses of this chunk's arenas and small block
    const uint8_t* din;
    uint8_t* dout;
    uint8_t* sm;
    const uint8_t* src_in = in_dev_ ? nullptr : s.in.h;
    if (via_copies(md)) {
        const uint8_t* h_in = in_dev_ ? in_ptr(j, s.c0) : src_in;
        if (in_b) hip_check(hipMemcpyAsync(s.d_in.p, h_in, in_b, hipMemcpyHostToDevice, st), "H2D arena");
        hip_check(hipMemcpyAsync(s.d_small.p, s.small.h, l.in_end, hipMemcpyHostToDevice, st), "H2D small");
        hip_check(hipEventRecord(s.indone, st), "hipEventRecord");
        // two kernel streams for hash-chain-bound jobs: consecutive chunks' chains overlap
        st = kern_[nkern_ > 1 ? (s.seq & 1) : 0];
        hip_check(hipStreamWaitEvent(st, s.indone, 0), "hipStreamWaitEvent");
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
    if (via_copies(md) && !zc_out(md)) {
        hip_check(hipEventRecord(s.kdone, st), "hipEventRecord");
        st = down_;
        hip_check(hipStreamWaitEvent(st, s.kdone, 0), "hipStreamWaitEvent");
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
    std::lock_guard<std::mutex> lk(mu_);
    run_locked(j);
}

void Engine::run_locked(const Job& j) {
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
    int prev = -1;
    hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev_) hip_check(hipSetDevice(dev_), "hipSetDevice");
    struct Restore {
        int prev, dev;
        ~Restore() {
            if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
        }
    } restore{prev, dev_};

    uint32_t S = cfg_.slots ? cfg_.slots : 4u;
#ifdef ENET_TOOLS_BUILD
    if (!cfg_.slots) S = (uint32_t)env_u64("ENET_HOST_SLOTS", S);
#endif
    S = std::max<uint32_t>(1, std::min<uint32_t>(S, 8));
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
    // the job's mode, read ONCE: a concurrent enet_host_set_mode changes later jobs only (stage,
    // launch and the stream layout of one job must agree).  Auto (no fixed mode): SdmaSplitK, or
    // for output the device writes in place the mode the device's auto state settled on -- the
    // first such jobs of >= 64 MiB alternate the two SDMA modes and their rates decide
    const int fixed = cfg_.mode >= 0 && valid_mode(cfg_.mode) ? cfg_.mode : fixed_mode();
    int sample = -1;
    unsigned sample_epoch = 0;
    md_ = fixed >= 0 ? (Mode)fixed : auto_mode(dev_, direct_out, in_total, st_.jobs > 0, &sample, &sample_epoch);
    const Mode md = md_;
    st_.mode = (int)md;
    // Long records behind a hash (HMAC / SHA-256 is one serial chain per record: 1.9 ms for 64 KiB)
    // bound every chunk's kernel by that chain
    const bool hashes = j.op != Op::Xor && j.op != Op::AeadSeal && j.op != Op::AeadOpen;
    const uint64_t chain = (hashes && max_len >= (16u << 10)) ? 4 : 1;
    setup_slots(S, chain > 1);
    // sessions: key table and its HMAC midstates on the device, once per job
    if (j.session) {
        table_.ensure(32ull * j.n_sessions);
        mid_.ensure(64ull * j.n_sessions);
        hipStream_t s0 = via_copies(md) ? up_ : slots_[0]->stream;
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
                                                : (md == Mode::ZeroCopy ? (32ull << 20) : (16ull << 20) * chain);
#ifdef ENET_TOOLS_BUILD
    if (!cfg_.chunk_bytes) chunk = std::max<uint64_t>(1, env_u64("ENET_HOST_CHUNK_MIB", chunk >> 20)) << 20;
#endif
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
    // Ramped chunk sizes: the first chunks (nothing to overlap their copy in yet) are 1/8 .. 1/2
    // of the steady chunk, so the pipeline fills in a fraction of a chunk's time.  Ramping down at
    // the end as well measured ~1 % slower (every extra chunk pays its small copies and event
    // hops; C2 e2e 19.1-19.3 vs 19.46, profiles/r04_host_ramp_ab.jsonl) and costs a hash-chain-bound
    // job one more ~2 ms chain per extra chunk (C5 share 17.6-17.8 vs 18.4-18.6,
    // r04_host_ramp_c5_ab.jsonl).  Tools build: ENET_HOST_RAMP bit 0 ramp-up, bit 1 ramp-down for
    // unhashed jobs, bit 2 ramp-down for hash-chain-bound jobs.
    unsigned ramp = 1u;
#ifdef ENET_TOOLS_BUILD
    ramp = (unsigned)env_u64("ENET_HOST_RAMP", 1) & 7u;
#endif
    try {
        while (c0 < n) {
            uint64_t target = chunk;
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
                     "gather/scatter %.3f, small arrays %.3f, launch %.3f, wait %.3f ms (direct in %d out %d) "
                     "node dev %d staging %d workers %u budget %u\n",
                     (int)j.op, (int)md, n, (unsigned long long)in_total, (unsigned long long)out_total, k, S,
                     1e3 * (now_s() - t_job), 1e3 * t_copy_, 1e3 * t_fill_, 1e3 * t_launch_, 1e3 * t_wait_,
                     in_dev_ != nullptr, (int)direct_out, st_.device_node, st_.staging_node, st_.workers,
                     st_.cpu_budget);
    if (!err && sample >= 0 && in_total)
        auto_record(dev_, sample, sample_epoch, (double)in_total / 1073741824.0 / std::max(1e-9, now_s() - t_job));
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
namespace {

struct SharedSet {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Engine*> engines;  // never destroyed: no HIP at process exit
    std::vector<bool> busy;
};

SharedSet& shared_set(int dev) {
    static std::mutex mu;
    static auto* sets = new std::map<int, SharedSet*>();
    std::lock_guard<std::mutex> lk(mu);
    auto& s = (*sets)[dev];
    if (!s) s = new SharedSet();
    return *s;
}

}  // namespace

void run_shared(int dev, const Job& job) {
    SharedSet& set = shared_set(dev);
    size_t idx = 0;
    Engine* eng = nullptr;  // read under set.mu: another caller may grow set.engines meanwhile
    {
        std::unique_lock<std::mutex> lk(set.mu);
        for (;;) {
            size_t i = 0;
            while (i < set.engines.size() && set.busy[i]) ++i;
            if (i < set.engines.size()) {
                idx = i;
                break;
            }
            if (set.engines.size() < kSharedEngines) {
                set.engines.push_back(new Engine(dev, Config{}));
                set.busy.push_back(false);
                idx = set.engines.size() - 1;
                break;
            }
            set.cv.wait(lk);
        }
        set.busy[idx] = true;
        eng = set.engines[idx];
    }
    struct Release {
        SharedSet& set;
        size_t idx;
        ~Release() {
            {
                std::lock_guard<std::mutex> lk(set.mu);
                set.busy[idx] = false;
            }
            set.cv.notify_one();
        }
    } release{set, idx};
    eng->run(job);
}

Engine* create_engine(int dev, const Config& cfg) { return new Engine(dev, cfg); }
void destroy_engine(Engine* e) { delete e; }
void run(Engine& e, const Job& job) { e.run(job); }
EngineStats stats(const Engine& e) { return e.stats(); }

}  // namespace enet::hb
