// pipeline.cpp -- host-resident record batches (include/enet_crypto.h, "host pipeline").
//
// The reference's crypto path starts and ends in host memory: socket receive buffers and relay
// payloads (SessionManager.cpp:362-387, 815-822) and chunk files (Node.cpp:1414-1417,
// 1641-1655).  This runtime takes such a batch in host memory, cuts it into chunks of about
// chunk_bytes on record boundaries, and on each of S HIP streams runs
//     H2D (arena slice + rebased offsets + keys/nonces/tags) -> kernel(s) -> D2H (arena + tags/ok)
// so the copies of one chunk overlap the kernels and copies of the others.  Per-record small
// arrays are gathered into pinned per-stream staging on the host thread (they must be rebased
// anyway); bulk arenas are copied straight from / to the caller's buffers (DMA when they are
// pinned, e.g. from enet_host_alloc).  Small outputs (tags, MACs, ok) land in pinned staging
// and are copied to the caller's arrays once every stream has drained.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "enet_crypto.h"
#include "enet_internal.hpp"

namespace {

enum class Op { Xor, Seal, Open, HmacSeal, HmacOpen };

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t staged = nullptr;   // the H2D copies out of this slot's host staging are done
    // device side
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint64_t cap_in = 0, cap_out = 0;
    uint64_t* d_in_off = nullptr;
    uint64_t* d_out_off = nullptr;
    uint8_t* d_keys = nullptr;
    uint8_t* d_nonces = nullptr;
    uint8_t* d_tags = nullptr;
    uint8_t* d_macs = nullptr;
    uint8_t* d_ok = nullptr;
    uint32_t* d_ctr = nullptr;
    uint32_t* d_order = nullptr;
    uint32_t cap_rec = 0;
    // pinned host staging of the per-record arrays
    uint64_t* h_in_off = nullptr;
    uint64_t* h_out_off = nullptr;
    uint8_t* h_keys = nullptr;
    uint8_t* h_nonces = nullptr;
    uint8_t* h_tags = nullptr;
    uint8_t* h_macs = nullptr;
    uint32_t* h_ctr = nullptr;
    uint32_t* h_order = nullptr;
};

int perr(int code, const std::string& what) {
    enet::set_last_error(what);
    return code;
}

#define PCHECK(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) return perr(ENET_EHIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

// inside the chunk loop: record the error and leave the loop (the streams are drained below)
#define LCHECK(call)                                                                   \
    {                                                                                  \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            rc = perr(ENET_EHIP, std::string(#call ": ") + hipGetErrorString(e_));     \
            break;                                                                     \
        }                                                                              \
    }

}  // namespace

struct enet_pipeline {
    int device = 0;
    uint64_t chunk_bytes = 0;
    std::vector<Slot> slots;
    // pinned staging for the small outputs of a whole call
    uint8_t* h_small = nullptr;
    uint64_t cap_small = 0;
};

namespace {

void free_slot_device(Slot& s) {
    (void)hipFree(s.d_in);
    (void)hipFree(s.d_out);
    (void)hipFree(s.d_in_off);
    (void)hipFree(s.d_out_off);
    (void)hipFree(s.d_keys);
    (void)hipFree(s.d_nonces);
    (void)hipFree(s.d_tags);
    (void)hipFree(s.d_macs);
    (void)hipFree(s.d_ok);
    (void)hipFree(s.d_ctr);
    (void)hipFree(s.d_order);
    (void)hipHostFree(s.h_in_off);
    (void)hipHostFree(s.h_out_off);
    (void)hipHostFree(s.h_keys);
    (void)hipHostFree(s.h_nonces);
    (void)hipHostFree(s.h_tags);
    (void)hipHostFree(s.h_macs);
    (void)hipHostFree(s.h_ctr);
    (void)hipHostFree(s.h_order);
    Slot keep;
    keep.stream = s.stream;
    keep.staged = s.staged;
    s = keep;
}

// Grow a slot to hold a chunk of `m` records, `in_b` input and `out_b` output bytes.  Only
// called when the slot's stream is idle (the caller synchronises it first).
int ensure(Slot& s, uint64_t in_b, uint64_t out_b, uint32_t m) {
    if (in_b > s.cap_in) {
        (void)hipFree(s.d_in);
        s.d_in = nullptr;
        s.cap_in = 0;
        PCHECK(hipMalloc(&s.d_in, std::max<uint64_t>(in_b, 16)));
        s.cap_in = in_b;
    }
    if (out_b > s.cap_out) {
        (void)hipFree(s.d_out);
        s.d_out = nullptr;
        s.cap_out = 0;
        PCHECK(hipMalloc(&s.d_out, std::max<uint64_t>(out_b, 16)));
        s.cap_out = out_b;
    }
    if (m > s.cap_rec) {
        const uint32_t c = std::max<uint32_t>(m, 1024);
        Slot fresh;
        fresh.stream = s.stream;
        fresh.staged = s.staged;
        fresh.d_in = s.d_in;
        fresh.d_out = s.d_out;
        fresh.cap_in = s.cap_in;
        fresh.cap_out = s.cap_out;
        s.d_in = s.d_out = nullptr;
        free_slot_device(s);
        s = fresh;
        PCHECK(hipMalloc(&s.d_in_off, 8ull * (c + 1)));
        PCHECK(hipMalloc(&s.d_out_off, 8ull * (c + 1)));
        PCHECK(hipMalloc(&s.d_keys, 32ull * c));
        PCHECK(hipMalloc(&s.d_nonces, 12ull * c));
        PCHECK(hipMalloc(&s.d_tags, 16ull * c));
        PCHECK(hipMalloc(&s.d_macs, 32ull * c));
        PCHECK(hipMalloc(&s.d_ok, c));
        PCHECK(hipMalloc(&s.d_ctr, 4ull * c));
        PCHECK(hipMalloc(&s.d_order, 4ull * c));
        PCHECK(hipHostMalloc(&s.h_in_off, 8ull * (c + 1), hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_out_off, 8ull * (c + 1), hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_keys, 32ull * c, hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_nonces, 12ull * c, hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_tags, 16ull * c, hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_macs, 32ull * c, hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_ctr, 4ull * c, hipHostMallocDefault));
        PCHECK(hipHostMalloc(&s.h_order, 4ull * c, hipHostMallocDefault));
        s.cap_rec = c;
    }
    return ENET_OK;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// per-record small outputs of one op, laid out [tags 16n | macs 32n | ok n] in h_small
struct SmallOut {
    uint64_t tags = 0, macs = 0, ok = 0, total = 0;
};

SmallOut small_layout(Op op, uint32_t n) {
    SmallOut l;
    uint64_t at = 0;
    if (op == Op::Seal || op == Op::HmacSeal) { l.tags = at; at += 16ull * n; }
    if (op == Op::HmacSeal) { l.macs = at; at += 32ull * n; }
    if (op == Op::Open || op == Op::HmacOpen) { l.ok = at; at += n; }
    l.total = at;
    return l;
}

int run(enet_pipeline* pp, Op op, const enet_records* r, const uint32_t* counters,
        const uint8_t* tags_in, const uint8_t* macs_in, uint8_t* tags_out, uint8_t* macs_out,
        uint8_t* ok_out) {
    if (!pp) return perr(ENET_EINVAL, "pipeline is NULL");
    if (!r) return perr(ENET_EINVAL, "records descriptor is NULL");
    const uint32_t n = r->count;
    if (n == 0) return ENET_OK;
    if (!r->in_offsets || !r->out_offsets || !r->in || !r->out || !r->keys || !r->nonces)
        return perr(ENET_EINVAL, "records: NULL offsets, arena, keys or nonces");
    if (r->key_stride != 0 && r->key_stride != 32)
        return perr(ENET_EINVAL, "records: key_stride must be 0 or 32");
    if (r->order) return perr(ENET_EINVAL, "host pipeline: order is not supported (NULL)");
    if ((op == Op::Seal || op == Op::HmacSeal) && !tags_out) return perr(ENET_EINVAL, "tags NULL");
    if (op == Op::HmacSeal && !macs_out) return perr(ENET_EINVAL, "macs NULL");
    if ((op == Op::Open || op == Op::HmacOpen) && (!tags_in || !ok_out))
        return perr(ENET_EINVAL, "tags / ok NULL");
    if (op == Op::HmacOpen && !macs_in) return perr(ENET_EINVAL, "macs NULL");
    const uint64_t* io = r->in_offsets;
    const uint64_t* oo = r->out_offsets;
    for (uint32_t i = 0; i < n; ++i)
        if (io[i + 1] < io[i] || oo[i + 1] < oo[i] || oo[i + 1] - oo[i] != io[i + 1] - io[i])
            return perr(ENET_EINVAL, "host pipeline: offsets must be non-decreasing and in/out "
                                     "records the same length");

    DeviceGuard guard(pp->device);
    const SmallOut lay = small_layout(op, n);
    if (lay.total > pp->cap_small) {
        (void)hipHostFree(pp->h_small);
        pp->h_small = nullptr;
        pp->cap_small = 0;
        PCHECK(hipHostMalloc(&pp->h_small, lay.total, hipHostMallocDefault));
        pp->cap_small = lay.total;
    }
    const uint32_t S = (uint32_t)pp->slots.size();
    int rc = ENET_OK;
    uint32_t c0 = 0, k = 0;
    while (c0 < n && rc == ENET_OK) {
        // chunk [c0, c1): at least one record, about chunk_bytes of input
        uint32_t c1 = c0 + 1;
        while (c1 < n && io[c1 + 1] - io[c0] <= pp->chunk_bytes) ++c1;
        const uint32_t m = c1 - c0;
        const uint64_t in_b = io[c1] - io[c0];
        const uint64_t out_b = oo[c1] - oo[c0];
        uint64_t mx = 0;
        for (uint32_t i = c0; i < c1; ++i) mx = std::max<uint64_t>(mx, io[i + 1] - io[i]);
        Slot& s = pp->slots[k % S];
        ++k;
        if (in_b > s.cap_in || out_b > s.cap_out || m > s.cap_rec) {
            LCHECK(hipStreamSynchronize(s.stream));
            if ((rc = ensure(s, in_b, out_b, m)) != ENET_OK) break;
        } else {
            LCHECK(hipEventSynchronize(s.staged));  // host staging free again
        }
        // gather + rebase the per-record arrays into pinned staging
        for (uint32_t i = 0; i <= m; ++i) {
            s.h_in_off[i] = io[c0 + i] - io[c0];
            s.h_out_off[i] = oo[c0 + i] - oo[c0];
        }
        const uint64_t kb = r->key_stride ? 32ull * m : 32ull;
        std::memcpy(s.h_keys, r->keys + (r->key_stride ? 32ull * c0 : 0ull), kb);
        std::memcpy(s.h_nonces, r->nonces + 12ull * c0, 12ull * m);
        if (tags_in) std::memcpy(s.h_tags, tags_in + 16ull * c0, 16ull * m);
        if (macs_in) std::memcpy(s.h_macs, macs_in + 32ull * c0, 32ull * m);
        if (counters) std::memcpy(s.h_ctr, counters + c0, 4ull * m);
        // mixed lengths: process longest records first, so the serial per-record tails
        // (SHA-256 is one lane per record) start at once and short records fill in behind them
        const bool mixed = in_b != (uint64_t)m * mx;
        if (mixed) {
            for (uint32_t i = 0; i < m; ++i) s.h_order[i] = i;
            const uint64_t* base = io + c0;
            std::stable_sort(s.h_order, s.h_order + m, [base](uint32_t a, uint32_t b) {
                return base[a + 1] - base[a] > base[b + 1] - base[b];
            });
        }
        hipStream_t st = s.stream;
        const auto h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
        LCHECK(hipMemcpyAsync(s.d_in, r->in + io[c0], in_b, h2d, st));
        LCHECK(hipMemcpyAsync(s.d_in_off, s.h_in_off, 8ull * (m + 1), h2d, st));
        LCHECK(hipMemcpyAsync(s.d_out_off, s.h_out_off, 8ull * (m + 1), h2d, st));
        LCHECK(hipMemcpyAsync(s.d_keys, s.h_keys, kb, h2d, st));
        LCHECK(hipMemcpyAsync(s.d_nonces, s.h_nonces, 12ull * m, h2d, st));
        if (tags_in) LCHECK(hipMemcpyAsync(s.d_tags, s.h_tags, 16ull * m, h2d, st));
        if (macs_in) LCHECK(hipMemcpyAsync(s.d_macs, s.h_macs, 32ull * m, h2d, st));
        if (counters) LCHECK(hipMemcpyAsync(s.d_ctr, s.h_ctr, 4ull * m, h2d, st));
        if (mixed) LCHECK(hipMemcpyAsync(s.d_order, s.h_order, 4ull * m, h2d, st));
        LCHECK(hipEventRecord(s.staged, st));
        enet_records d{};
        d.count = m;
        d.in_offsets = s.d_in_off;
        d.out_offsets = s.d_out_off;
        d.in = s.d_in;
        d.out = s.d_out;
        d.keys = s.d_keys;
        d.key_stride = r->key_stride;
        d.nonces = s.d_nonces;
        d.order = mixed ? s.d_order : nullptr;
        d.total_bytes_hint = in_b;
        d.max_len_hint = (uint32_t)std::min<uint64_t>(mx, 0xFFFFFFFFull);
        switch (op) {
            case Op::Xor: rc = enet_chacha20_xor_batch(&d, counters ? s.d_ctr : nullptr, st); break;
            case Op::Seal: rc = enet_aead_seal_batch(&d, nullptr, nullptr, s.d_tags, st); break;
            case Op::Open: rc = enet_aead_open_batch(&d, nullptr, nullptr, s.d_tags, s.d_ok, st); break;
            case Op::HmacSeal: rc = enet_aead_hmac_seal_batch(&d, s.d_tags, s.d_macs, st); break;
            case Op::HmacOpen: rc = enet_aead_hmac_open_batch(&d, s.d_tags, s.d_macs, s.d_ok, st); break;
        }
        if (rc != ENET_OK) {
            enet::set_last_error(std::string("host pipeline kernel: ") + enet_last_error());
            break;
        }
        LCHECK(hipMemcpyAsync(r->out + oo[c0], s.d_out, out_b, d2h, st));
        if (op == Op::Seal || op == Op::HmacSeal)
            LCHECK(hipMemcpyAsync(pp->h_small + lay.tags + 16ull * c0, s.d_tags, 16ull * m, d2h, st));
        if (op == Op::HmacSeal)
            LCHECK(hipMemcpyAsync(pp->h_small + lay.macs + 32ull * c0, s.d_macs, 32ull * m, d2h, st));
        if (op == Op::Open || op == Op::HmacOpen)
            LCHECK(hipMemcpyAsync(pp->h_small + lay.ok + c0, s.d_ok, m, d2h, st));
        c0 = c1;
    }
    for (Slot& s : pp->slots) {
        hipError_t e = hipStreamSynchronize(s.stream);
        if (e != hipSuccess && rc == ENET_OK)
            rc = perr(ENET_EHIP, std::string("host pipeline drain: ") + hipGetErrorString(e));
    }
    if (rc != ENET_OK) return rc;
    if (tags_out) std::memcpy(tags_out, pp->h_small + lay.tags, 16ull * n);
    if (macs_out) std::memcpy(macs_out, pp->h_small + lay.macs, 32ull * n);
    if (ok_out) std::memcpy(ok_out, pp->h_small + lay.ok, n);
    return ENET_OK;
}

}  // namespace

// Several devices of one node: one pipeline, host thread and set of streams per
// device; a batch is cut into contiguous record ranges balanced by input bytes, so a mixed
// 512 B - 64 KiB batch (C5) gives every device the same payload; no collective -- each range's
// tags / MACs / ok land at their positions in the caller's arrays.
struct enet_pipeline_group {
    std::vector<enet_pipeline*> pipes;
};

namespace {

int group_run(enet_pipeline_group* g, Op op, const enet_records* r, const uint32_t* counters,
              const uint8_t* tags_in, const uint8_t* macs_in, uint8_t* tags_out, uint8_t* macs_out,
              uint8_t* ok_out) {
    if (!g || g->pipes.empty()) return perr(ENET_EINVAL, "pipeline group is NULL or empty");
    if (!r) return perr(ENET_EINVAL, "records descriptor is NULL");
    const uint32_t n = r->count;
    if (n == 0) return ENET_OK;
    if (!r->in_offsets || !r->out_offsets) return perr(ENET_EINVAL, "records: NULL offsets");
    if (r->order) return perr(ENET_EINVAL, "pipeline group: order is not supported (NULL)");
    const uint64_t* io = r->in_offsets;
    for (uint32_t i = 0; i < n; ++i)
        if (io[i + 1] < io[i]) return perr(ENET_EINVAL, "pipeline group: offsets must be non-decreasing");
    const uint32_t D = (uint32_t)g->pipes.size();
    const uint64_t total = io[n] - io[0];
    // range d = [lo[d], lo[d + 1]): lo[d] = first record starting at or after d * total / D bytes
    std::vector<uint32_t> lo(D + 1);
    lo[0] = 0;
    lo[D] = n;
    for (uint32_t d = 1; d < D; ++d) {
        const uint64_t target = io[0] + (total * d) / D;
        lo[d] = (uint32_t)(std::lower_bound(io, io + n, target) - io);
        lo[d] = std::max(lo[d], lo[d - 1]);
    }
    std::vector<int> rc(D, ENET_OK);
    std::vector<std::string> err(D);
    std::vector<std::thread> th;
    th.reserve(D);
    for (uint32_t d = 0; d < D; ++d) {
        const uint32_t a = lo[d], b = lo[d + 1];
        if (a == b) continue;
        enet_records q = *r;
        q.count = b - a;
        q.in_offsets = r->in_offsets + a;
        q.out_offsets = r->out_offsets + a;
        if (r->keys) q.keys = r->keys + (size_t)r->key_stride * a;
        if (r->nonces) q.nonces = r->nonces + 12ull * a;
        q.total_bytes_hint = io[b] - io[a];
        th.emplace_back([=, &rc, &err] {
            rc[d] = run(g->pipes[d], op, &q, counters ? counters + a : nullptr,
                        tags_in ? tags_in + 16ull * a : nullptr, macs_in ? macs_in + 32ull * a : nullptr,
                        tags_out ? tags_out + 16ull * a : nullptr,
                        macs_out ? macs_out + 32ull * a : nullptr, ok_out ? ok_out + a : nullptr);
            if (rc[d] != ENET_OK) err[d] = enet_last_error();
        });
    }
    for (std::thread& t : th) t.join();
    for (uint32_t d = 0; d < D; ++d)
        if (rc[d] != ENET_OK) return perr(rc[d], "pipeline group, range " + std::to_string(d) + ": " + err[d]);
    return ENET_OK;
}

}  // namespace

extern "C" {

enet_pipeline_group* enet_pipeline_group_create(const int* devices, uint32_t ndev,
                                                uint64_t chunk_bytes, uint32_t streams) {
    std::vector<int> devs;
    if (devices && ndev) {
        devs.assign(devices, devices + ndev);
    } else {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
            enet::set_last_error("enet_pipeline_group_create: no devices");
            return nullptr;
        }
        for (int d = 0; d < count; ++d) devs.push_back(d);
    }
    auto* g = new enet_pipeline_group;
    for (int d : devs) {
        enet_pipeline* p = enet_pipeline_create(d, chunk_bytes, streams);
        if (!p) {
            const std::string e = enet_last_error();
            enet_pipeline_group_destroy(g);
            enet::set_last_error("enet_pipeline_group_create: device " + std::to_string(d) + ": " + e);
            return nullptr;
        }
        g->pipes.push_back(p);
    }
    return g;
}

void enet_pipeline_group_destroy(enet_pipeline_group* g) {
    if (!g) return;
    for (enet_pipeline* p : g->pipes) enet_pipeline_destroy(p);
    delete g;
}

uint32_t enet_pipeline_group_size(const enet_pipeline_group* g) {
    return g ? (uint32_t)g->pipes.size() : 0u;
}

int enet_pipeline_group_chacha20_xor(enet_pipeline_group* g, const enet_records* r,
                                     const uint32_t* counters) {
    return group_run(g, Op::Xor, r, counters, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int enet_pipeline_group_aead_seal(enet_pipeline_group* g, const enet_records* r, uint8_t* tags) {
    return group_run(g, Op::Seal, r, nullptr, nullptr, nullptr, tags, nullptr, nullptr);
}

int enet_pipeline_group_aead_open(enet_pipeline_group* g, const enet_records* r,
                                  const uint8_t* tags, uint8_t* ok) {
    return group_run(g, Op::Open, r, nullptr, tags, nullptr, nullptr, nullptr, ok);
}

int enet_pipeline_group_aead_hmac_seal(enet_pipeline_group* g, const enet_records* r,
                                       uint8_t* tags, uint8_t* macs) {
    return group_run(g, Op::HmacSeal, r, nullptr, nullptr, nullptr, tags, macs, nullptr);
}

int enet_pipeline_group_aead_hmac_open(enet_pipeline_group* g, const enet_records* r,
                                       const uint8_t* tags, const uint8_t* macs, uint8_t* ok) {
    return group_run(g, Op::HmacOpen, r, nullptr, tags, macs, nullptr, nullptr, ok);
}

enet_pipeline* enet_pipeline_create(int device, uint64_t chunk_bytes, uint32_t streams) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) {
        enet::set_last_error("enet_pipeline_create: no such device");
        return nullptr;
    }
    DeviceGuard guard(device);
    auto* p = new enet_pipeline;
    p->device = device;
    p->chunk_bytes = chunk_bytes ? chunk_bytes : (16ull << 20);
    const uint32_t S = streams ? std::min<uint32_t>(streams, 16) : 3u;
    p->slots.resize(S);
    for (Slot& s : p->slots) {
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&s.staged, hipEventDisableTiming) != hipSuccess) {
            enet::set_last_error("enet_pipeline_create: stream/event creation failed");
            enet_pipeline_destroy(p);
            return nullptr;
        }
    }
    return p;
}

void enet_pipeline_destroy(enet_pipeline* p) {
    if (!p) return;
    DeviceGuard guard(p->device);
    for (Slot& s : p->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        free_slot_device(s);
        if (s.staged) (void)hipEventDestroy(s.staged);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    (void)hipHostFree(p->h_small);
    delete p;
}

int enet_pipeline_chacha20_xor(enet_pipeline* p, const enet_records* r, const uint32_t* counters) {
    return run(p, Op::Xor, r, counters, nullptr, nullptr, nullptr, nullptr, nullptr);
}

int enet_pipeline_aead_seal(enet_pipeline* p, const enet_records* r, uint8_t* tags) {
    return run(p, Op::Seal, r, nullptr, nullptr, nullptr, tags, nullptr, nullptr);
}

int enet_pipeline_aead_open(enet_pipeline* p, const enet_records* r, const uint8_t* tags,
                            uint8_t* ok) {
    return run(p, Op::Open, r, nullptr, tags, nullptr, nullptr, nullptr, ok);
}

int enet_pipeline_aead_hmac_seal(enet_pipeline* p, const enet_records* r, uint8_t* tags,
                                 uint8_t* macs) {
    return run(p, Op::HmacSeal, r, nullptr, nullptr, nullptr, tags, macs, nullptr);
}

int enet_pipeline_aead_hmac_open(enet_pipeline* p, const enet_records* r, const uint8_t* tags,
                                 const uint8_t* macs, uint8_t* ok) {
    return run(p, Op::HmacOpen, r, nullptr, tags, macs, nullptr, nullptr, ok);
}

void* enet_host_alloc(uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void enet_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
