// capi.cpp -- the extern "C" boundary (include/enet_crypto.h): argument checks, lane
// scheduling, and the kernel sequences for the composite operations (frames).
#include "enet_crypto.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "enet_internal.hpp"

// nonce(12) || BE32 length (SessionManager.cpp:85-86,376-385)
constexpr uint32_t kWireHeader = 16;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* what) {
    g_last_error = what;
    return code;
}

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) {
        g_last_error.clear();
        return ENET_OK;
    }
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return ENET_EHIP;
}

bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

// Kernel A/B knobs (ENET_NT_STORES, ENET_LOCKSTEP, ENET_STREAM, ENET_DUPLEX, ENET_COOP, ENET_LANES,
// ENET_TARGET_LANES): read from the environment by the tools build only (build.py --tools ->
// libenet_crypto_tools.so); the shipping library runs its defaults, and tests pick variants
// through the enet_set_* calls.
const char* tools_env(const char* name) {
#ifdef ENET_TOOLS_BUILD
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

int check_records(const enet_records* r, bool need_keys) {
    if (!r) return fail(ENET_EINVAL, "records descriptor is NULL");
    if (r->count == 0) return ENET_OK;
    if (!r->in_offsets || !r->out_offsets || !r->in || !r->out)
        return fail(ENET_EINVAL, "records: NULL offsets or arena");
    if (need_keys) {
        if (!r->keys || !r->nonces) return fail(ENET_EINVAL, "records: NULL keys or nonces");
        if (r->key_stride != 0 && r->key_stride != 32)
            return fail(ENET_EINVAL, "records: key_stride must be 0 or 32");
        if (!aligned4(r->keys) || !aligned4(r->nonces))
            return fail(ENET_EINVAL, "records: keys/nonces must be 4-byte aligned");
    }
    if (r->order && !aligned4(r->order)) return fail(ENET_EINVAL, "records: order misaligned");
    return ENET_OK;
}

enet::RecParams rec_params(const enet_records* r) {
    enet::RecParams p{};
    p.n = r->count;
    p.in_off = r->in_offsets;
    p.out_off = r->out_offsets;
    p.in = r->in;
    p.out = r->out;
    p.keys = r->keys;
    p.key_stride = r->key_stride;
    p.nonces = r->nonces;
    p.order = r->order;
    // hints say every record has the same length: total == n * max (record i then starts at
    // offsets[0] + i * max, since records are contiguous by construction)
    if (r->max_len_hint && r->total_bytes_hint == (uint64_t)r->count * r->max_len_hint)
        p.uniform_len = r->max_len_hint;
    p.coop = (int)enet::staging_variant();
    // variant 1 (default): line staging for unaligned one-lane records, lockstep keystream in
    // 512-thread workgroups otherwise; 4 = plain run staging (neither); 5 = lockstep run staging
    const bool dflt = p.coop == 1;
    p.coop_lines = dflt ? 1 : 0;
    static const int nt = [] {
        const char* e = tools_env("ENET_NT_STORES");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    p.nt_stores = nt;
    static const int lock = [] {
        const char* e = tools_env("ENET_LOCKSTEP");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    p.lockstep = dflt ? lock : 0;
    static const int strm = [] {
        const char* e = tools_env("ENET_STREAM");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    p.stream = dflt ? strm : 0;
#ifdef ENET_TOOLS_BUILD
    // Measurement probes of the stream kernel (skip keystream / Poly1305 / stores, clock stamps in
    // tag_out) and its memory-schedule variants.  Only the tools build of the library
    // (build.py --tools -> libenet_crypto_tools.so, loaded via ENET_LIB_PATH) reads them: a
    // probe produces wrong ciphertext and tags by design, so the shipping library cannot be
    // switched into one from the environment.
    static const int dbg = [] {
        const char* e = std::getenv("ENET_STREAM_DBG");
        return e ? (int)std::strtol(e, nullptr, 10) : 0;
    }();
    p.dbg = dbg;
    static const int var = [] {
        const char* e = std::getenv("ENET_STREAM_VAR");
        return e ? (int)std::strtol(e, nullptr, 10) : 0;
    }();
    p.var = var;
#endif

    if (p.coop == 4) p.coop = 1;
    return p;
}

// Every path with a hash beside the cipher (frames, wire frames, chunk store / fetch with given
// ids, AEAD + HMAC) runs as ONE pass through the duplex kernel (duplex.hip): any lengths, any
// alignment, any order.  ENET_DUPLEX=0 or staging variant 0 selects the two-pass path (hash kernel +
// records kernel) instead.
bool duplex_on() {
    static const bool on = [] {
        const char* e = tools_env("ENET_DUPLEX");
        return !(e && e[0] == '0');
    }();
    return on && enet::staging_variant() != 0;
}

enet::DuplexParams duplex_params(const enet_records* r) {
    enet::DuplexParams p{};
    p.n = r->count;
    p.in = r->in;
    p.in_off = r->in_offsets;
    p.out = r->out;
    p.out_off = r->out_offsets;
    p.keys = r->keys;
    p.key_stride = r->key_stride;
    p.nonces = r->nonces;
    p.order = r->order;
    p.uniform = r->max_len_hint && r->total_bytes_hint == (uint64_t)r->count * r->max_len_hint;
    p.max_len = r->max_len_hint;
    return p;
}

uint32_t lanes_for(const enet_records* r) {
    return enet::choose_lanes(r->count, r->total_bytes_hint, r->max_len_hint);
}

// ---- the sequence-parallel path (segments.hip) for long records
// -1: auto (below); otherwise every record of at least this many bytes takes the tiles, whatever
// the hints say (enet_set_seg_min: tests / tuning; INT64_MAX = never)
std::atomic<int64_t> g_seg_min{-1};
std::atomic<uint64_t> g_seg_batches{0};  // batches that took the tiles (enet_seg_batches)

// Auto: a batch whose longest record (hint) is >= kSegMin takes the tiles for its records >=
// kSegMin -- unless it is uniform and wide enough that 16 lanes per record already fill the chip
// (n * 16 >= 131 072 lanes: the record / streaming kernels run those at the C2 rate).
bool seg_wanted(const enet_records* r, uint64_t& long_min) {
    const int64_t f = g_seg_min.load(std::memory_order_relaxed);
    if (f >= 0) {
        long_min = (uint64_t)f;
        return f != INT64_MAX;
    }
    long_min = enet::kSegMin;
    if (r->max_len_hint < enet::kSegMin) return false;
    const bool uniform = r->total_bytes_hint == (uint64_t)r->count * r->max_len_hint;
    return !(uniform && (uint64_t)r->count * enet::kMaxLanesPerRecord >= 131072u);
}

// Scratch comes from a library-private, stream-ordered pool per device (hipMallocFromPoolAsync /
// hipFreeAsync on the caller's stream): no synchronisation, capturable, and concurrent calls on
// different streams get their own.  Freed memory stays in the pool.
hipMemPool_t seg_pool() {
    static std::mutex mu;
    static hipMemPool_t pools[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!pools[dev]) {
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pl = nullptr;
        if (hipMemPoolCreate(&pl, &props) != hipSuccess) return nullptr;
        uint64_t keep = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pl, hipMemPoolAttrReleaseThreshold, &keep);
        pools[dev] = pl;
    }
    return pools[dev];
}

struct SegRun {
    void* mem = nullptr;
    const uint8_t* claimed = nullptr;
};

// Per-stream state of the one-launch AEAD path (segments.hip seg_uniform_aead_kernel): arrival
// counters, zeroed when allocated and reset by each record's last arriver, so they are zero
// whenever a launch on that stream starts (launches on one stream run in order); and the tiles'
// partials.  Grown on demand, stream-ordered; otherwise reused, so a launch makes no allocation
// (a stream-ordered allocate / free pair per call cost ~4 us of gap between launches).
struct Arrivals {
    uint32_t* ptr = nullptr;
    uint32_t cap = 0;
    void* part = nullptr;
    size_t part_cap = 0;
    void* seg = nullptr;  // the plan + tiles path's scratch (seg_begin)
    size_t seg_cap = 0;
};

int arrivals_for(hipStream_t st, uint32_t n, uint32_t*& out, size_t part_bytes = 0, void** part_out = nullptr,
                 size_t seg_bytes = 0, void** seg_out = nullptr) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<int, hipStream_t>, Arrivals>> table;
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return hip_status(e, "aead tiles: hipGetDevice");
    std::lock_guard<std::mutex> lk(mu);
    Arrivals* a = nullptr;
    for (auto& kv : table)
        if (kv.first.first == dev && kv.first.second == st) a = &kv.second;
    if (!a) {
        table.push_back({{dev, st}, Arrivals{}});
        a = &table.back().second;
    }
    if (a->cap < n) {
        hipMemPool_t pool = seg_pool();
        if (!pool) return fail(ENET_EHIP, "aead tiles: no memory pool for the current device");
        const uint32_t cap = std::max<uint32_t>(n, 1024u);
        void* mem = nullptr;
        if (hipError_t e = hipMallocFromPoolAsync(&mem, 4ull * cap, pool, st)) return hip_status(e, "aead tiles: counters");
        if (hipError_t e = hipMemsetAsync(mem, 0, 4ull * cap, st)) return hip_status(e, "aead tiles: counters");
        if (a->ptr) (void)hipFreeAsync(a->ptr, st);
        a->ptr = static_cast<uint32_t*>(mem);
        a->cap = cap;
    }
    if (part_out && a->part_cap < part_bytes) {
        hipMemPool_t pool = seg_pool();
        if (!pool) return fail(ENET_EHIP, "aead tiles: no memory pool for the current device");
        const size_t cap = std::max<size_t>(part_bytes, 64u << 10);
        void* mem = nullptr;
        if (hipError_t e = hipMallocFromPoolAsync(&mem, cap, pool, st)) return hip_status(e, "aead tiles: scratch");
        if (a->part) (void)hipFreeAsync(a->part, st);
        a->part = mem;
        a->part_cap = cap;
    }
    if (part_out) *part_out = a->part;
    if (seg_out && a->seg_cap < seg_bytes) {
        hipMemPool_t pool = seg_pool();
        if (!pool) return fail(ENET_EHIP, "sequence-parallel scratch: no memory pool for the current device");
        const size_t cap = std::max<size_t>(seg_bytes, 256u << 10);
        void* mem = nullptr;
        if (hipError_t e = hipMallocFromPoolAsync(&mem, cap, pool, st)) return hip_status(e, "sequence-parallel scratch");
        if (a->seg) (void)hipFreeAsync(a->seg, st);
        a->seg = mem;
        a->seg_cap = cap;
    }
    if (seg_out) *seg_out = a->seg;
    out = a->ptr;
    return ENET_OK;
}

// RFC 8439 seal / open over a batch the hints call uniform and long: one launch
int run_uniform_aead(int mode, const enet_records* r, const enet::RecParams& p, hipStream_t st, const char* what) {
    const uint64_t L = r->max_len_hint;
    const uint64_t T = (L + enet::kSegTileBytes - 1) / enet::kSegTileBytes;
    const uint64_t tiles = (uint64_t)r->count * T;
    uint32_t* arr = nullptr;
    const uint64_t words = (uint64_t)r->count * enet::seg_uniform_arrival_words();
    if (words > UINT32_MAX) return fail(ENET_EINVAL, "aead tiles: too many records for one launch");
    void* mem = nullptr;
    if (int e = arrivals_for(st, (uint32_t)words, arr, (size_t)tiles * 32, &mem)) return e;
    enet::SegParams q{};
    q.mode = mode;
    q.n = r->count;
    q.in_off = p.in_off;
    q.out_off = p.out_off;
    q.in = p.in;
    q.out = p.out;
    q.keys = p.keys;
    q.key_stride = p.key_stride;
    q.nonces = p.nonces;
    q.aad = p.aad;
    q.aad_off = p.aad_off;
    q.tag_in = p.tag_in;
    q.tag_out = p.tag_out;
    q.ok = p.ok;
    q.partials = static_cast<uint32_t*>(mem);
    g_seg_batches.fetch_add(1, std::memory_order_relaxed);
    return hip_status(enet::launch_seg_uniform_aead(q, L, arr, st), what);
}

// Plan + tile kernels for the batch's long records; sr.claimed marks them for the record engine.
// index_n: one past the largest record index (r->count unless r->order names a subset).
int seg_begin(int mode, const enet_records* r, enet::RecParams& p, uint64_t long_min, hipStream_t st,
              SegRun& sr, uint32_t index_n) {
    const uint32_t n = r->count;
    const uint64_t total = r->total_bytes_hint ? r->total_bytes_hint
                                               : (uint64_t)std::min<uint32_t>(n, 1024u) * r->max_len_hint;
    // capacities from the hints; records past them stay with the record engine (never wrong bytes)
    const uint64_t ecap = std::min<uint64_t>(n, long_min ? total / long_min + 1 : n);
    const uint64_t tcap = std::min<uint64_t>(total / enet::kSegTileBytes + ecap + 1, 0xFFFFFFFFull);
    const size_t o_ent = 256, o_cl = o_ent + (size_t)ecap * sizeof(enet::SegEntry),
                 o_part = (o_cl + index_n + 255) & ~size_t(255), bytes = o_part + (size_t)tcap * 32;
    // per-stream scratch, reused: one seg run per call, calls on a stream run in order, and the
    // plan kernel initialises everything the tiles read (no allocate / free pair per call)
    uint32_t* unused = nullptr;
    void* mem = nullptr;
    if (int e = arrivals_for(st, 0, unused, 0, nullptr, bytes, &mem)) return e;
    uint8_t* base = static_cast<uint8_t*>(mem);
    enet::SegParams q{};
    q.mode = mode;
    q.n = n;
    q.in_off = p.in_off;
    q.out_off = p.out_off;
    q.in = p.in;
    q.out = p.out;
    q.keys = p.keys;
    q.key_stride = p.key_stride;
    q.nonces = p.nonces;
    q.counters = p.counters;
    q.counter_stride = p.counter_stride;
    q.aad = p.aad;
    q.aad_off = p.aad_off;
    q.tag_in = p.tag_in;
    q.tag_out = p.tag_out;
    q.ok = p.ok;
    q.order = p.order;
    q.hdr = reinterpret_cast<unsigned long long*>(base);
    q.entries = reinterpret_cast<enet::SegEntry*>(base + o_ent);
    q.claimed = base + o_cl;
    q.partials = reinterpret_cast<uint32_t*>(base + o_part);
    q.entry_cap = (uint32_t)ecap;
    q.tile_cap = (uint32_t)tcap;
    q.long_min = long_min;
    const uint32_t plan_blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 1024);
    const uint32_t tile_blocks = (uint32_t)std::min<uint64_t>(tcap, 4096);
    sr.claimed = q.claimed;
    g_seg_batches.fetch_add(1, std::memory_order_relaxed);
    return hip_status(enet::launch_seg(q, plan_blocks, tile_blocks, st), "sequence-parallel launch");
}

void seg_end(SegRun& sr, hipStream_t st) {
    (void)sr;
    (void)st;
}

// The record engine over the batch, with the long records on the tiles first when seg_wanted
int run_records(int mode, const enet_records* r, enet::RecParams& p, hipStream_t st, const char* what,
                uint32_t index_n = 0) {
    uint64_t long_min = 0;
    SegRun sr;
    // XOR over a batch the hints call uniform and long: one launch of tile workgroups, nothing
    // else (a record that is not as hinted is run whole by its tile-0 workgroup)
    if (mode == enet::MODE_XOR && !r->order && seg_wanted(r, long_min) && r->max_len_hint >= long_min &&
        r->total_bytes_hint == (uint64_t)r->count * r->max_len_hint) {
        enet::SegParams q{};
        q.mode = mode;
        q.n = r->count;
        q.in_off = p.in_off;
        q.out_off = p.out_off;
        q.in = p.in;
        q.out = p.out;
        q.keys = p.keys;
        q.key_stride = p.key_stride;
        q.nonces = p.nonces;
        q.counters = p.counters;
        q.counter_stride = p.counter_stride;
        g_seg_batches.fetch_add(1, std::memory_order_relaxed);
        return hip_status(enet::launch_seg_uniform_xor(q, r->max_len_hint, st), what);
    }
    // AEAD over such a batch: one launch too (the last tile of each record to arrive combines,
    // and zeroes a failed open itself)
    if ((mode == enet::MODE_SEAL || mode == enet::MODE_OPEN) && !r->order && seg_wanted(r, long_min) &&
        r->max_len_hint >= long_min && r->total_bytes_hint == (uint64_t)r->count * r->max_len_hint &&
        (uint64_t)r->count * ((r->max_len_hint + enet::kSegTileBytes - 1) / enet::kSegTileBytes) < 0x7FFFFFFFull)
        return run_uniform_aead(mode, r, p, st, what);
    if (mode <= enet::MODE_OPEN && seg_wanted(r, long_min)) {
        if (int e = seg_begin(mode, r, p, long_min, st, sr, index_n ? index_n : r->count)) {
            seg_end(sr, st);
            return e;
        }
        p.skip = sr.claimed;
        p.uniform_len = 0;  // per-lane path: the staged paths assume every record is theirs
    }
    const int rc = hip_status(enet::launch_records(mode, p, lanes_for(r), st), what);
    seg_end(sr, st);
    return rc;
}

// ---- chunk store / fetch on the device (every record on the GPU)
int chunk_store_device(const enet_records* r, const uint8_t* chunk_ids, uint8_t* chunk_hashes,
                              hipStream_t st) {
    if (chunk_ids && duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        d.chunk_ids = chunk_ids;
        d.digests = chunk_hashes;
        return hip_status(enet::launch_duplex(enet::DK_CHUNK, false, d, st), "chunk_store duplex");
    }
    // 1) chunk_hash = SHA-256(pt) (Node.cpp:1414; = derive_chunk_id, StoreProof.cpp:75-78)
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->in;
    s.off = r->in_offsets;
    s.digest = chunk_hashes;
    s.order = r->order;
    if (int e = hip_status(enet::launch_sha(s, st), "chunk_store sha")) return e;
    // 2) ChaCha20 from counter LE32(chunk_id[0..3]) (CryptoManager.cpp:8-13,38-46), the id read
    //    on the device (the fresh digests when the caller derives ids from content)
    enet::RecParams p = rec_params(r);
    p.counters = reinterpret_cast<const uint32_t*>(chunk_ids ? chunk_ids : chunk_hashes);
    p.counter_stride = 8;
    return hip_status(enet::launch_records(enet::MODE_XOR, p, lanes_for(r), st),
                      "chunk_store chacha");
}

int chunk_fetch_device(const enet_records* r, const uint8_t* chunk_ids, const uint8_t* chunk_hashes,
                              uint8_t* ok, hipStream_t st) {
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        d.chunk_ids = chunk_ids;
        d.expect = chunk_hashes;
        d.ok = ok;
        return hip_status(enet::launch_duplex(enet::DK_CHUNK, true, d, st), "chunk_fetch duplex");
    }
    // 1) decrypt_with_key (CryptoManager.cpp:49-58)
    enet::RecParams p = rec_params(r);
    p.counters = reinterpret_cast<const uint32_t*>(chunk_ids);
    p.counter_stride = 8;
    if (int e = hip_status(enet::launch_records(enet::MODE_XOR, p, lanes_for(r), st),
                           "chunk_fetch chacha"))
        return e;
    // 2) SHA-256(pt) == manifest.chunk_hash, else no plaintext (Node.cpp:1644-1655)
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->out;
    s.off = r->out_offsets;
    s.expect = chunk_hashes;
    s.ok = ok;
    s.zero_on_fail = r->out;
    s.order = r->order;
    return hip_status(enet::launch_sha(s, st), "chunk_fetch sha verify");
}


// ---- long chunks: the cipher on the device, the hash chain on host threads (chunk_hybrid.cpp)
// A record of >= kHostHashMin bytes is one serial SHA-256 chain: ~34 MB/s on a GPU lane (the 64 KiB
// duplex chain takes 1.90 ms) against ~2.1 GB/s on a SHA-NI core (490 us per MiB).
// The host route pays while the host's chains (sum over T threads) finish before the GPU's
// longest lane would: sum(long) / (T * 2.1 GB/s) < Lmax / 34 MB/s, i.e. sum(long) < ~60 T Lmax.
// Everything shorter stays on the one-pass duplex kernel.
constexpr uint64_t kHostHashMin = 256u << 10;
constexpr uint64_t kHostHashRatio = 60;
std::atomic<int64_t> g_hh_min{-1};  // enet_set_host_hash_min: -1 auto, else forced (INT64_MAX never)
std::atomic<uint64_t> g_hh_batches{0};

uint32_t host_hash_threads() {
    static const uint32_t t = [] {
        const uint32_t b = enet_host_cpu_budget();
        return b ? b : 1u;
    }();
    return t;
}

struct HostPinned {  // thread-local pinned scratch, grow-only
    void* p = nullptr;
    size_t cap = 0;
    ~HostPinned() {
        if (p) (void)hipHostFree(p);
    }
    uint8_t* get(size_t n) {
        if (n > cap) {
            if (p) (void)hipHostFree(p);
            p = nullptr;
            cap = 0;
            if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
            cap = n;
        }
        return static_cast<uint8_t*>(p);
    }
};
thread_local HostPinned t_pinned;

struct LongSplit {
    std::vector<uint64_t> in_off, out_off;
    std::vector<uint32_t> shorts, longs;
    uint64_t short_max = 0, short_sum = 0, long_max = 0, long_sum = 0;
};

// 1: the batch has long chunks for the host route (ls filled), 0: not, < 0: error
int long_split(const enet_records* r, hipStream_t st, LongSplit& ls) {
    const int64_t f = g_hh_min.load(std::memory_order_relaxed);
    if (f == INT64_MAX || r->order) return 0;  // a caller-ordered subset keeps its own schedule
    const uint64_t lmin = f >= 0 ? (uint64_t)f : kHostHashMin;
    // only when the caller's hint says a record may be that long: the route reads the offsets
    // back (a stream synchronisation), which a batch of short chunks must not pay
    if (r->max_len_hint < lmin || r->max_len_hint == 0) return 0;
    const uint32_t n = r->count;
    ls.in_off.resize(n + 1);
    ls.out_off.resize(n + 1);
    if (hipError_t e = hipMemcpyAsync(ls.in_off.data(), r->in_offsets, 8ull * (n + 1), hipMemcpyDeviceToHost, st))
        return hip_status(e, "chunk: offsets to host");
    if (hipError_t e = hipMemcpyAsync(ls.out_off.data(), r->out_offsets, 8ull * (n + 1), hipMemcpyDeviceToHost, st))
        return hip_status(e, "chunk: offsets to host");
    if (hipError_t e = hipStreamSynchronize(st)) return hip_status(e, "chunk: offsets to host");
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t a = ls.in_off[i], b = ls.in_off[i + 1];
        const uint64_t L = b >= a ? b - a : 0;
        if (b >= a && L >= lmin && ls.out_off[i + 1] >= ls.out_off[i]) {
            ls.longs.push_back(i);
            ls.long_max = std::max(ls.long_max, L);
            ls.long_sum += L;
        } else {
            ls.shorts.push_back(i);
            ls.short_max = std::max(ls.short_max, L);
            ls.short_sum += L;
        }
    }
    if (ls.longs.empty()) return 0;
    if (f < 0 && ls.long_sum > kHostHashRatio * host_hash_threads() * ls.long_max) return 0;  // GPU lanes win
    return 1;
}

// device scratch: the two index lists (and room for host results), stream-ordered from the pool
struct ChunkScratch {
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    uint32_t* d_shorts = nullptr;
    uint32_t* d_longs = nullptr;
    uint8_t* d_res = nullptr;  // [m][32] digests / [m] verdicts from the host
    uint8_t* h_res = nullptr;
};

int chunk_scratch(const LongSplit& ls, hipStream_t st, ChunkScratch& cs) {
    const size_t ns = ls.shorts.size(), m = ls.longs.size();
    const size_t o_l = (4 * ns + 255) & ~size_t(255), o_r = (o_l + 4 * m + 255) & ~size_t(255),
                 bytes = o_r + 32 * m;
    hipMemPool_t pool = seg_pool();
    if (!pool) return fail(ENET_EHIP, "chunk: no memory pool for the current device");
    void* d = nullptr;
    if (hipError_t e = hipMallocFromPoolAsync(&d, bytes, pool, st)) return hip_status(e, "chunk scratch");
    cs.dev = static_cast<uint8_t*>(d);
    cs.host = t_pinned.get(bytes);
    if (!cs.host) return fail(ENET_EHIP, "chunk: pinned host scratch");
    std::memcpy(cs.host, ls.shorts.data(), 4 * ns);
    std::memcpy(cs.host + o_l, ls.longs.data(), 4 * m);
    cs.d_shorts = reinterpret_cast<uint32_t*>(cs.dev);
    cs.d_longs = reinterpret_cast<uint32_t*>(cs.dev + o_l);
    cs.d_res = cs.dev + o_r;
    cs.h_res = cs.host + o_r;
    return hip_status(hipMemcpyAsync(cs.dev, cs.host, o_r, hipMemcpyHostToDevice, st), "chunk: index lists");
}

// the end of a host-route call: scratch back to the pool, and the stream drained (the pinned
// scratch is this thread's and is reused by its next call)
int chunk_finish(ChunkScratch& cs, hipStream_t st, int rc) {
    if (cs.dev) (void)hipFreeAsync(cs.dev, st);
    const hipError_t e = hipStreamSynchronize(st);
    return rc ? rc : hip_status(e, "chunk: drain");
}

enet_records subset(const enet_records* r, const uint32_t* order, uint32_t count, uint64_t max_len, uint64_t sum) {
    enet_records q = *r;
    q.count = count;
    q.order = order;
    q.max_len_hint = (uint32_t)std::min<uint64_t>(max_len, 0xFFFFFFFFu);
    q.total_bytes_hint = sum;
    return q;
}

int chunk_store_host_hash(const enet_records* r, const uint8_t* ids, uint8_t* hashes, hipStream_t st,
                          const LongSplit& ls) {
    ChunkScratch cs;
    int rc = chunk_scratch(ls, st, cs);
    const uint32_t m = (uint32_t)ls.longs.size();
    // the short chunks' one-pass kernel runs while the host hashes the long ones
    if (!rc && !ls.shorts.empty()) {
        enet_records q = subset(r, cs.d_shorts, (uint32_t)ls.shorts.size(), ls.short_max, ls.short_sum);
        rc = chunk_store_device(&q, ids, hashes, st);
    }
    std::string err;
    if (!rc && enet::host_hash_records(r->in, ls.in_off.data(), ls.longs.data(), m, nullptr, host_hash_threads(),
                                       cs.h_res, err))
        rc = fail(ENET_EHIP, ("chunk_store: " + err).c_str());
    if (!rc) rc = hip_status(hipMemcpyAsync(cs.d_res, cs.h_res, 32ull * m, hipMemcpyHostToDevice, st), "chunk_store: digests");
    if (!rc) rc = hip_status(enet::launch_scatter(cs.d_res, cs.d_longs, m, hashes, 32, st), "chunk_store: digests");
    if (!rc) {
        // ChaCha20 from LE32(id) -- the fresh digest when the id is derived from content
        // (CryptoManager.cpp:8-13, Node.cpp:1414-1417) -- over the long chunks, on the tiles
        enet_records q = subset(r, cs.d_longs, m, ls.long_max, ls.long_sum);
        enet::RecParams p = rec_params(&q);
        p.counters = reinterpret_cast<const uint32_t*>(ids ? ids : hashes);
        p.counter_stride = 8;
        rc = run_records(enet::MODE_XOR, &q, p, st, "chunk_store long chacha", r->count);
    }
    g_hh_batches.fetch_add(1, std::memory_order_relaxed);
    return chunk_finish(cs, st, rc);
}

int chunk_fetch_host_hash(const enet_records* r, const uint8_t* ids, const uint8_t* expect, uint8_t* ok,
                          hipStream_t st, const LongSplit& ls) {
    ChunkScratch cs;
    int rc = chunk_scratch(ls, st, cs);
    const uint32_t m = (uint32_t)ls.longs.size(), n = r->count;
    if (!rc && !ls.shorts.empty()) {
        enet_records q = subset(r, cs.d_shorts, (uint32_t)ls.shorts.size(), ls.short_max, ls.short_sum);
        rc = chunk_fetch_device(&q, ids, expect, ok, st);
    }
    if (!rc) {  // decrypt_with_key (CryptoManager.cpp:49-58) over the long chunks, on the tiles
        enet_records q = subset(r, cs.d_longs, m, ls.long_max, ls.long_sum);
        enet::RecParams p = rec_params(&q);
        p.counters = reinterpret_cast<const uint32_t*>(ids);
        p.counter_stride = 8;
        rc = run_records(enet::MODE_XOR, &q, p, st, "chunk_fetch long chacha", n);
    }
    // the expected hashes to the host, then the plaintext in pieces as the host hashes it
    std::vector<uint8_t> want(32ull * n);
    hipEvent_t ready = nullptr;
    if (!rc) rc = hip_status(hipMemcpyAsync(want.data(), expect, 32ull * n, hipMemcpyDeviceToHost, st), "chunk_fetch: hashes");
    if (!rc) rc = hip_status(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "chunk_fetch: event");
    if (!rc) rc = hip_status(hipEventRecord(ready, st), "chunk_fetch: event");
    std::string err;
    if (!rc && enet::host_hash_records(r->out, ls.out_off.data(), ls.longs.data(), m, ready, host_hash_threads(),
                                       cs.h_res, err))
        rc = fail(ENET_EHIP, ("chunk_fetch: " + err).c_str());
    if (!rc) rc = hip_status(hipEventSynchronize(ready), "chunk_fetch: hashes");
    if (ready) (void)hipEventDestroy(ready);
    if (!rc) {
        // SHA-256(pt) == manifest.chunk_hash, else no plaintext (Node.cpp:1644-1655); a chunk
        // whose output length differs from its input fails too
        std::vector<uint8_t> okl(m);
        for (uint32_t k = 0; k < m && !rc; ++k) {
            const uint32_t i = ls.longs[k];
            const bool same_len = ls.out_off[i + 1] - ls.out_off[i] == ls.in_off[i + 1] - ls.in_off[i];
            okl[k] = same_len && std::memcmp(cs.h_res + 32ull * k, want.data() + 32ull * i, 32) == 0;
            if (!okl[k])
                rc = hip_status(hipMemsetAsync(r->out + ls.out_off[i], 0, ls.out_off[i + 1] - ls.out_off[i], st),
                                "chunk_fetch: zero failed chunk");
        }
        if (!rc) {
            std::memcpy(cs.h_res, okl.data(), m);  // digests consumed: the verdicts go up from here
            rc = hip_status(hipMemcpyAsync(cs.d_res, cs.h_res, m, hipMemcpyHostToDevice, st), "chunk_fetch: verdicts");
        }
        if (!rc) rc = hip_status(enet::launch_scatter(cs.d_res, cs.d_longs, m, ok, 1, st), "chunk_fetch: verdicts");
    }
    g_hh_batches.fetch_add(1, std::memory_order_relaxed);
    return chunk_finish(cs, st, rc);
}

}  // namespace

namespace enet {

void set_last_error(const std::string& what) { g_last_error = what; }

static std::atomic<uint32_t> g_forced_lanes{0};
static std::atomic<uint32_t> g_staging{0};
static std::atomic<int> g_duplex_split{-1};

int duplex_split_mode() { return g_duplex_split.load(std::memory_order_relaxed); }

// Uniform-batch staging: 1 = register prefetch + LDS transposition (default: run staging in
// lockstep 512-thread workgroups, line staging for unaligned one-lane records), 4 = plain run
// staging, 5 = lockstep run staging; 0 = per-lane path only.  ENET_COOP / enet_set_staging
// override (tests).  (3, the LDS-DMA four-waves-per-SIMD variant, was retired in round 6.)
uint32_t staging_variant() {
    static const uint32_t env = [] {
        const char* s = tools_env("ENET_COOP");
        return s ? (uint32_t)std::strtoul(s, nullptr, 10) + 1u : 0u;
    }();
    if (uint32_t f = g_staging.load(std::memory_order_relaxed)) return f - 1u;
    if (env == 1 || env == 2 || env == 5 || env == 6) return env - 1u;
    return 1u;
}

// Give each record enough lanes that the grid holds >= ENET_TARGET_LANES lanes
// (default 2 waves per SIMD on 256 CUs = 131072), but keep >= 8 ChaCha20 blocks per lane: every
// lane pays one one-time-key block and, for P > 1, one r^e power, so thinner lanes lose more to
// that fixed cost than they gain in occupancy.  ENET_LANES / enet_set_lanes_per_record force a
// value (tuning / tests).
uint32_t choose_lanes(uint32_t n, uint64_t total_bytes, uint32_t max_len) {
    static const uint32_t forced = [] {
        const char* s = tools_env("ENET_LANES");
        return s ? (uint32_t)std::strtoul(s, nullptr, 10) : 0u;
    }();
    static const uint64_t target = [] {
        const char* s = tools_env("ENET_TARGET_LANES");
        return s ? (uint64_t)std::strtoull(s, nullptr, 10) : 131072ull;
    }();
    if (uint32_t f = g_forced_lanes.load(std::memory_order_relaxed)) return f;
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8 || forced == 16) return forced;
    if (n == 0) return 1;
    uint64_t cap = kMaxLanesPerRecord;
    const uint64_t typical = total_bytes ? total_bytes / n : max_len;
    if (typical) cap = std::max<uint64_t>(1, ((typical + 63) / 64) / 8);
    uint32_t lanes = 1;
    while (lanes < kMaxLanesPerRecord && (uint64_t)n * lanes < target && lanes * 2 <= cap)
        lanes *= 2;
    return lanes;
}

}  // namespace enet

extern "C" {

uint32_t enet_abi_version(void) { return (1u << 16) | 2u; }

const char* enet_last_error(void) { return g_last_error.c_str(); }

uint32_t enet_chunk_counter(const uint8_t chunk_id[32]) {  // CryptoManager.cpp:8-13
    return (uint32_t)chunk_id[0] | ((uint32_t)chunk_id[1] << 8) | ((uint32_t)chunk_id[2] << 16) |
           ((uint32_t)chunk_id[3] << 24);
}

uint32_t enet_lanes_per_record(uint32_t count, uint64_t total_bytes, uint32_t max_len) {
    return enet::choose_lanes(count, total_bytes, max_len);
}

int enet_set_staging(int variant) {
    if (variant != -1 && variant != 0 && variant != 1 && variant != 4 && variant != 5)
        return fail(ENET_EINVAL, "staging variant must be -1 (default), 0, 1, 4 or 5");
    enet::g_staging.store((uint32_t)(variant + 1), std::memory_order_relaxed);
    return ENET_OK;
}

int enet_set_duplex_split(int mode) {
    if (mode != -1 && mode != 0 && mode != 1) return fail(ENET_EINVAL, "duplex split mode must be -1, 0 or 1");
    enet::g_duplex_split.store(mode, std::memory_order_relaxed);
    return ENET_OK;
}

int enet_set_seg_min(int64_t bytes) {
    if (bytes < -1) return fail(ENET_EINVAL, "seg_min must be -1 (auto), 0 .. INT64_MAX");
    g_seg_min.store(bytes, std::memory_order_relaxed);
    return ENET_OK;
}

uint64_t enet_seg_batches(void) { return g_seg_batches.load(std::memory_order_relaxed); }

int enet_set_lanes_per_record(uint32_t lanes) {
    if (lanes != 0 && lanes != 1 && lanes != 2 && lanes != 4 && lanes != 8 && lanes != 16)
        return fail(ENET_EINVAL, "lanes must be 0, 1, 2, 4, 8 or 16");
    enet::g_forced_lanes.store(lanes, std::memory_order_relaxed);
    return ENET_OK;
}

int enet_chacha20_xor_batch(const enet_records* r, const uint32_t* counters, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (counters && !aligned4(counters)) return fail(ENET_EINVAL, "counters misaligned");
    enet::RecParams p = rec_params(r);
    p.counters = counters;
    return run_records(enet::MODE_XOR, r, p, (hipStream_t)stream, "chacha20_xor launch");
}

int enet_aead_seal_batch(const enet_records* r, const uint8_t* aad, const uint64_t* aad_offsets,
                         uint8_t* tags, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!tags || !aligned4(tags)) return fail(ENET_EINVAL, "tags NULL or misaligned");
    if ((aad == nullptr) != (aad_offsets == nullptr))
        return fail(ENET_EINVAL, "aad and aad_offsets must both be set or both NULL");
    enet::RecParams p = rec_params(r);
    p.aad = aad;
    p.aad_off = aad_offsets;
    p.tag_out = tags;
    return run_records(enet::MODE_SEAL, r, p, (hipStream_t)stream, "aead_seal launch");
}

int enet_aead_open_batch(const enet_records* r, const uint8_t* aad, const uint64_t* aad_offsets,
                         const uint8_t* tags, uint8_t* ok, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!tags || !aligned4(tags) || !ok) return fail(ENET_EINVAL, "tags/ok NULL or misaligned");
    if ((aad == nullptr) != (aad_offsets == nullptr))
        return fail(ENET_EINVAL, "aad and aad_offsets must both be set or both NULL");
    enet::RecParams p = rec_params(r);
    p.aad = aad;
    p.aad_off = aad_offsets;
    p.tag_in = tags;
    p.ok = ok;
    return run_records(enet::MODE_OPEN, r, p, (hipStream_t)stream, "aead_open launch");
}

int enet_sha256_batch(uint32_t n, const uint8_t* in, const uint64_t* offsets, uint8_t* digests,
                      void* stream) {
    if (n == 0) return ENET_OK;
    if (!in || !offsets || !digests) return fail(ENET_EINVAL, "sha256: NULL argument");
    enet::ShaParams p{};
    p.n = n;
    p.in = in;
    p.off = offsets;
    p.digest = digests;
    return hip_status(enet::launch_sha(p, (hipStream_t)stream), "sha256 launch");
}

static int hmac_common(uint32_t n, const uint8_t* keys, const uint64_t* key_offsets,
                       uint32_t key_stride, const uint8_t* in, const uint64_t* offsets,
                       enet::ShaParams& p) {
    if (!keys || !in || !offsets) return fail(ENET_EINVAL, "hmac: NULL argument");
    if (!key_offsets && key_stride != 0 && key_stride != 32)
        return fail(ENET_EINVAL, "hmac: key_stride must be 0 or 32");
    p.n = n;
    p.in = in;
    p.off = offsets;
    p.keys = keys;
    p.key_off = key_offsets;
    p.key_stride = key_stride;
    return ENET_OK;
}

int enet_hmac_sha256_batch(uint32_t n, const uint8_t* keys, const uint64_t* key_offsets,
                           uint32_t key_stride, const uint8_t* in, const uint64_t* offsets,
                           uint8_t* macs, void* stream) {
    if (n == 0) return ENET_OK;
    enet::ShaParams p{};
    if (int e = hmac_common(n, keys, key_offsets, key_stride, in, offsets, p)) return e;
    if (!macs) return fail(ENET_EINVAL, "hmac: NULL macs");
    p.digest = macs;
    return hip_status(enet::launch_sha(p, (hipStream_t)stream), "hmac launch");
}

int enet_hmac_sha256_verify_batch(uint32_t n, const uint8_t* keys, const uint64_t* key_offsets,
                                  uint32_t key_stride, const uint8_t* in,
                                  const uint64_t* offsets, const uint8_t* macs, uint8_t* ok,
                                  void* stream) {
    if (n == 0) return ENET_OK;
    enet::ShaParams p{};
    if (int e = hmac_common(n, keys, key_offsets, key_stride, in, offsets, p)) return e;
    if (!macs || !ok) return fail(ENET_EINVAL, "hmac verify: NULL macs/ok");
    p.expect = macs;
    p.ok = ok;
    return hip_status(enet::launch_sha(p, (hipStream_t)stream), "hmac verify launch");
}

int enet_aead_hmac_seal_batch(const enet_records* r, uint8_t* tags, uint8_t* macs,
                              void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!tags || !aligned4(tags) || !macs) return fail(ENET_EINVAL, "tags/macs NULL or misaligned");
    hipStream_t st = (hipStream_t)stream;
    if (duplex_on()) {  // one pass: Poly1305 in the cipher lanes, HMAC in the hash lanes
        enet::DuplexParams d = duplex_params(r);
        d.tags = tags;
        d.macs = macs;
        return hip_status(enet::launch_duplex(enet::DK_AEADH, false, d, st), "aead_hmac_seal duplex");
    }
    // two-pass: HMAC over the plaintext (encode_signed semantics), then the AEAD pass
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->in;
    s.off = r->in_offsets;
    s.digest = macs;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.order = r->order;
    if (int e = hip_status(enet::launch_sha(s, st), "aead_hmac_seal hmac")) return e;
    enet::RecParams p = rec_params(r);
    p.tag_out = tags;
    return hip_status(enet::launch_records(enet::MODE_SEAL, p, lanes_for(r), st),
                      "aead_hmac_seal aead");
}

int enet_aead_hmac_open_batch(const enet_records* r, const uint8_t* tags, const uint8_t* macs,
                              uint8_t* ok, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!tags || !aligned4(tags) || !macs || !ok)
        return fail(ENET_EINVAL, "tags/macs/ok NULL or misaligned");
    hipStream_t st = (hipStream_t)stream;
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        d.tags_in = tags;
        d.macs_in = macs;
        d.ok = ok;
        return hip_status(enet::launch_duplex(enet::DK_AEADH, true, d, st), "aead_hmac_open duplex");
    }
    enet::RecParams p = rec_params(r);
    p.tag_in = tags;
    p.ok = ok;
    if (int e = hip_status(enet::launch_records(enet::MODE_OPEN, p, lanes_for(r), st),
                           "aead_hmac_open aead"))
        return e;
    // HMAC verify over the decrypted plaintext, AND-ed into ok; zero the record on failure
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->out;
    s.off = r->out_offsets;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.expect = macs;
    s.ok = ok;
    s.and_ok = 1;
    s.zero_on_fail = r->out;
    s.order = r->order;
    return hip_status(enet::launch_sha(s, st), "aead_hmac_open hmac verify");
}

int enet_frame_seal_batch(const enet_records* r, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        return hip_status(enet::launch_duplex(enet::DK_FRAME, false, d, (hipStream_t)stream), "frame_seal duplex");
    }
    // 1) MAC = HMAC-SHA256(K, m) written in clear at the tail of each output record
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->in;
    s.off = r->in_offsets;
    s.digest = r->out;
    s.dest_off = r->out_offsets;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.order = r->order;
    hipStream_t st = (hipStream_t)stream;
    if (int e = hip_status(enet::launch_sha(s, st), "frame_seal hmac launch")) return e;
    // 2) body = ChaCha20(ctr 0) over m || MAC
    enet::RecParams p = rec_params(r);
    return hip_status(enet::launch_records(3, p, lanes_for(r), st), "frame_seal chacha launch");
}

int enet_frame_open_batch(const enet_records* r, uint8_t* macs, uint8_t* ok, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!macs || !ok || !aligned4(macs)) return fail(ENET_EINVAL, "frame_open: NULL/misaligned macs or NULL ok");
    hipStream_t st = (hipStream_t)stream;
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        d.macs = macs;
        d.ok = ok;
        return hip_status(enet::launch_duplex(enet::DK_FRAME, true, d, st), "frame_open duplex");
    }
    // 1) decrypt: message bytes to out, MAC bytes to macs
    enet::RecParams p = rec_params(r);
    p.tag_out = macs;
    if (int e = hip_status(enet::launch_records(4, p, lanes_for(r), st), "frame_open chacha"))
        return e;
    // 2) verify HMAC over the decrypted message; zero the message on failure
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->out;
    s.off = r->out_offsets;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.expect = macs;
    s.ok = ok;
    s.guard_off = r->in_offsets;
    s.zero_on_fail = r->out;
    s.order = r->order;
    return hip_status(enet::launch_sha(s, st), "frame_open hmac verify");
}

int enet_chunk_store_batch(const enet_records* r, const uint8_t* chunk_ids, uint8_t* chunk_hashes,
                           void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!chunk_hashes || !aligned4(chunk_hashes))
        return fail(ENET_EINVAL, "chunk_store: chunk_hashes NULL or misaligned");
    if (chunk_ids && !aligned4(chunk_ids)) return fail(ENET_EINVAL, "chunk_store: chunk_ids misaligned");
    hipStream_t st = (hipStream_t)stream;
    try {  // the host route allocates and starts threads: nothing may escape the C ABI
        LongSplit ls;
        const int route = long_split(r, st, ls);
        if (route < 0) return route;
        if (route) return chunk_store_host_hash(r, chunk_ids, chunk_hashes, st, ls);
    } catch (const std::exception& e) {
        return fail(ENET_EHIP, (std::string("chunk_store: ") + e.what()).c_str());
    }
    return chunk_store_device(r, chunk_ids, chunk_hashes, st);
}

int enet_chunk_fetch_batch(const enet_records* r, const uint8_t* chunk_ids,
                           const uint8_t* chunk_hashes, uint8_t* ok, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!chunk_ids || !aligned4(chunk_ids) || !chunk_hashes || !ok)
        return fail(ENET_EINVAL, "chunk_fetch: NULL/misaligned chunk_ids, NULL hashes or ok");
    hipStream_t st = (hipStream_t)stream;
    try {
        LongSplit ls;
        const int route = long_split(r, st, ls);
        if (route < 0) return route;
        if (route) return chunk_fetch_host_hash(r, chunk_ids, chunk_hashes, ok, st, ls);
    } catch (const std::exception& e) {
        return fail(ENET_EHIP, (std::string("chunk_fetch: ") + e.what()).c_str());
    }
    return chunk_fetch_device(r, chunk_ids, chunk_hashes, ok, st);
}

int enet_set_host_hash_min(int64_t bytes) {
    if (bytes < -1) return fail(ENET_EINVAL, "host_hash_min must be -1 (auto), 0 .. INT64_MAX");
    g_hh_min.store(bytes, std::memory_order_relaxed);
    return ENET_OK;
}

uint64_t enet_host_hash_batches(void) { return g_hh_batches.load(std::memory_order_relaxed); }

int enet_wire_seal_batch(const enet_records* r, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    hipStream_t st = (hipStream_t)stream;
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(r);
        d.hdr = kWireHeader;
        return hip_status(enet::launch_duplex(enet::DK_FRAME, false, d, st), "wire_seal duplex");
    }
    // 1) MAC = HMAC-SHA256(K, m) in clear at the tail of each frame body
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->in;
    s.off = r->in_offsets;
    s.digest = r->out + kWireHeader;
    s.dest_off = r->out_offsets;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.order = r->order;
    if (int e = hip_status(enet::launch_sha(s, st), "wire_seal hmac launch")) return e;
    // 2) header + body = ChaCha20(ctr 0) over m || MAC
    enet::RecParams p = rec_params(r);
    p.hdr = kWireHeader;
    return hip_status(enet::launch_records(3, p, lanes_for(r), st), "wire_seal chacha launch");
}

int enet_hmac_midstates(const uint8_t* keys, uint32_t n, uint32_t* mid, void* stream) {
    if (n == 0) return ENET_OK;
    if (!keys || !mid || !aligned4(keys) || !aligned4(mid)) return fail(ENET_EINVAL, "hmac_midstates: NULL/misaligned keys or mid");
    return hip_status(enet::launch_hmac_midstates(n, keys, mid, (hipStream_t)stream), "hmac_midstates");
}

// the session-keyed frame paths always run the one-pass duplex kernel
int enet_wire_seal_batch_sessions(const enet_records* r, const uint32_t* session, uint32_t sessions,
                                  const uint32_t* mid, void* stream) {
    if (int e = check_records(r, true)) return e;
    if (r->count == 0) return ENET_OK;
    if (!session || !mid || !aligned4(session) || !aligned4(mid) || sessions == 0) return fail(ENET_EINVAL, "wire_seal_sessions: NULL/misaligned session or mid, or no sessions");
    enet::DuplexParams d = duplex_params(r);
    d.hdr = kWireHeader;
    d.session = session;
    d.mid = mid;
    d.n_sessions = sessions;
    return hip_status(enet::launch_duplex(enet::DK_FRAME, false, d, (hipStream_t)stream), "wire_seal_sessions");
}

int enet_wire_open_batch_sessions(const enet_records* r, const uint32_t* session, uint32_t sessions,
                                  const uint32_t* mid, uint8_t* macs, uint8_t* ok, void* stream) {
    if (!r) return fail(ENET_EINVAL, "records descriptor is NULL");
    if (r->count == 0) return ENET_OK;
    enet_records q = *r;
    static const uint32_t kNoNonce[3] = {0, 0, 0};
    if (!q.nonces) q.nonces = reinterpret_cast<const uint8_t*>(kNoNonce);  // read from frames
    if (int e = check_records(&q, true)) return e;
    if (!macs || !ok || !aligned4(macs)) return fail(ENET_EINVAL, "wire_open_sessions: NULL/misaligned macs or NULL ok");
    if (!session || !mid || !aligned4(session) || !aligned4(mid) || sessions == 0) return fail(ENET_EINVAL, "wire_open_sessions: NULL/misaligned session or mid, or no sessions");
    enet::DuplexParams d = duplex_params(&q);
    d.hdr = kWireHeader;
    d.macs = macs;
    d.ok = ok;
    d.session = session;
    d.mid = mid;
    d.n_sessions = sessions;
    return hip_status(enet::launch_duplex(enet::DK_FRAME, true, d, (hipStream_t)stream), "wire_open_sessions");
}

int enet_wire_open_batch(const enet_records* r, uint8_t* macs, uint8_t* ok, void* stream) {
    if (!r) return fail(ENET_EINVAL, "records descriptor is NULL");
    if (r->count == 0) return ENET_OK;
    enet_records q = *r;
    static const uint32_t kNoNonce[3] = {0, 0, 0};
    if (!q.nonces) q.nonces = reinterpret_cast<const uint8_t*>(kNoNonce);  // read from frames
    if (int e = check_records(&q, true)) return e;
    if (!macs || !ok || !aligned4(macs)) return fail(ENET_EINVAL, "wire_open: NULL/misaligned macs or NULL ok");
    hipStream_t st = (hipStream_t)stream;
    if (duplex_on()) {
        enet::DuplexParams d = duplex_params(&q);
        d.hdr = kWireHeader;
        d.macs = macs;
        d.ok = ok;
        return hip_status(enet::launch_duplex(enet::DK_FRAME, true, d, st), "wire_open duplex");
    }
    enet::RecParams p = rec_params(&q);
    p.nonces = nullptr;
    p.hdr = kWireHeader;
    p.tag_out = macs;
    if (int e = hip_status(enet::launch_records(4, p, lanes_for(r), st), "wire_open chacha"))
        return e;
    enet::ShaParams s{};
    s.n = r->count;
    s.in = r->out;
    s.off = r->out_offsets;
    s.keys = r->keys;
    s.key_stride = r->key_stride;
    s.expect = macs;
    s.ok = ok;
    s.guard_off = r->in_offsets;
    s.wire_in = r->in;
    s.wire_hdr = kWireHeader;
    s.zero_on_fail = r->out;
    s.order = r->order;
    return hip_status(enet::launch_sha(s, st), "wire_open hmac verify");
}

int enet_pow_search_batch(uint32_t n, const uint8_t* prefixes, const uint64_t* prefix_offsets,
                          const uint8_t* difficulty, int schedule, uint64_t max_attempts,
                          uint64_t* nonces, uint64_t* attempts, uint8_t* found, void* stream) {
    if (n == 0) return ENET_OK;
    if (!prefixes || !prefix_offsets || !difficulty || !nonces || !found)
        return fail(ENET_EINVAL, "pow_search: NULL argument");
    if (schedule != ENET_POW_NODE && schedule != ENET_POW_STORE)
        return fail(ENET_EINVAL, "pow_search: schedule must be ENET_POW_NODE or ENET_POW_STORE");
    if (n > 0x7FFFFFFFu) return fail(ENET_EINVAL, "pow_search: too many jobs");
    // one workgroup per job: enough waves per job that the grid holds ~4 waves per SIMD
    // (1024 SIMDs), at most 16 (1024 threads), never more lanes than attempts
    uint32_t waves = 1;
    while (waves < 16 && (uint64_t)n * waves < 4096 && 64ull * waves < max_attempts) waves <<= 1;
    enet::PowParams p{};
    p.n = n;
    p.prefixes = prefixes;
    p.off = prefix_offsets;
    p.difficulty = difficulty;
    p.schedule = (uint32_t)schedule;
    p.max_attempts = max_attempts;
    if (schedule == ENET_POW_STORE) {
        uint64_t r = 1;
        while (r < 64ull * waves + 312) r <<= 1;
        p.ring = r;
    }
    p.nonces = nonces;
    p.attempts = attempts;
    p.found = found;
    return hip_status(enet::launch_pow_search(p, waves, (hipStream_t)stream), "pow_search launch");
}

int enet_pow_check_batch(uint32_t n, const uint8_t* prefixes, const uint64_t* prefix_offsets,
                         const uint64_t* nonces, const uint8_t* difficulty, uint8_t* ok,
                         void* stream) {
    if (n == 0) return ENET_OK;
    if (!prefixes || !prefix_offsets || !nonces || !difficulty || !ok)
        return fail(ENET_EINVAL, "pow_check: NULL argument");
    enet::PowParams p{};
    p.n = n;
    p.prefixes = prefixes;
    p.off = prefix_offsets;
    p.difficulty = difficulty;
    p.check_nonces = nonces;
    p.found = ok;
    return hip_status(enet::launch_pow_check(p, (hipStream_t)stream), "pow_check launch");
}

int enet_session_key_batch(uint32_t n, const uint8_t* secrets, const uint64_t* counters,
                           const int64_t* ticks, uint8_t* keys_out, void* stream) {
    if (n == 0) return ENET_OK;
    if (!secrets || !counters || !ticks || !keys_out)
        return fail(ENET_EINVAL, "session_key: NULL argument");
    return hip_status(enet::launch_session_keys(n, secrets, counters, ticks, keys_out,
                                                (hipStream_t)stream),
                      "session_key launch");
}

}  // extern "C"
