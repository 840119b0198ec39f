// host_path_probe.cpp -- how fast can records that start and end in HOST memory go through the
// MI355X?  Measures, on one box, in one process (JSON line per case):
//   copies   : pinned H2D, D2H, and both at once on two streams (256 MiB)
//   zc       : the AEAD seal / open kernels reading and / or writing pinned host memory directly
//              (zero-copy over PCIe: no DMA, no chunking), for several host allocation flags
//   pipe     : the library's enet_pipeline_aead_* (H2D -> kernel -> D2H per chunk, 3 streams)
//   zcout    : per-chunk H2D (SDMA) -> kernel writing the pinned host output directly
//   zcin     : kernel reading the pinned host input directly -> device out -> D2H (SDMA)
// Every case checks open(seal(x)) == x with every tag verified.
// build: hipcc --offload-arch=gfx950 -O2 -std=c++20 -Iinclude tools/host_path_probe.cpp
//        -Lephemeralnet_amd -lenet_crypto -Wl,-rpath,'$ORIGIN/../ephemeralnet_amd' -o tools/host_path_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "enet_crypto.h"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                       \
        }                                                                                       \
    } while (0)
#define EK(x)                                                                           \
    do {                                                                                \
        int r_ = (x);                                                                   \
        if (r_ != 0) {                                                                  \
            std::fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r_, enet_last_error()); \
            std::exit(3);                                                               \
        }                                                                               \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Host {
    uint8_t* h = nullptr;  // host address
    uint8_t* d = nullptr;  // device address of the same bytes
};

static Host host_alloc(size_t n, unsigned flags) {
    Host m;
    CK(hipHostMalloc((void**)&m.h, n, flags));
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, m.h, 0));
    m.d = (uint8_t*)dp;
    return m;
}

static uint8_t* dev_alloc(size_t n) {
    uint8_t* p = nullptr;
    CK(hipMalloc((void**)&p, n));
    return p;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536;
    const uint64_t L = argc > 2 ? (uint64_t)atoll(argv[2]) : 4096;
    const std::string only = argc > 3 ? argv[3] : "all";
    const uint64_t T = n * L;
    const int reps = 5;
    std::mt19937_64 rng(7);
    std::vector<uint8_t> pt(T), keys(32ull * n), nonces(12ull * n);
    for (auto* v : {&pt, &keys, &nonces})
        for (size_t i = 0; i < v->size(); i += 8) {
            uint64_t x = rng();
            std::memcpy(v->data() + i, &x, std::min<size_t>(8, v->size() - i));
        }
    std::vector<uint64_t> off(n + 1);
    for (uint32_t i = 0; i <= n; ++i) off[i] = i * L;

    // small per-record arrays on the device
    uint8_t* d_keys = dev_alloc(keys.size());
    uint8_t* d_non = dev_alloc(nonces.size());
    uint64_t* d_off = (uint64_t*)dev_alloc(8ull * (n + 1));
    uint8_t* d_tags = dev_alloc(16ull * n);
    uint8_t* d_ok = dev_alloc(n);
    CK(hipMemcpy(d_keys, keys.data(), keys.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_non, nonces.data(), nonces.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, off.data(), 8ull * (n + 1), hipMemcpyHostToDevice));
    uint8_t* d_a = dev_alloc(T);
    uint8_t* d_b = dev_alloc(T);
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto recs = [&](const uint8_t* in, uint8_t* out, uint32_t cnt, const uint64_t* offs, uint32_t first) {
        enet_records r{};
        r.count = cnt;
        r.in_offsets = offs;
        r.out_offsets = offs;
        r.in = in;
        r.out = out;
        r.keys = d_keys + 32ull * first;
        r.key_stride = 32;
        r.nonces = d_non + 12ull * first;
        r.total_bytes_hint = (uint64_t)cnt * L;
        r.max_len_hint = (uint32_t)L;
        return r;
    };
    auto gib = [&](double s) { return (double)T / s / (1ull << 30); };
    auto check = [&](const uint8_t* back_h, const char* what) {
        std::vector<uint8_t> ok(n);
        CK(hipMemcpy(ok.data(), d_ok, n, hipMemcpyDeviceToHost));
        uint64_t good = 0;
        for (uint8_t v : ok) good += v;
        const bool same = std::memcmp(back_h, pt.data(), T) == 0;
        if (good != n || !same) {
            std::fprintf(stderr, "%s: FAILED ok=%llu/%u same=%d\n", what, (unsigned long long)good, n, same);
            std::exit(4);
        }
    };

    const unsigned flag_sets[3] = {hipHostMallocDefault, hipHostMallocMapped | hipHostMallocCoherent,
                                   hipHostMallocMapped | hipHostMallocNonCoherent};
    const char* flag_names[3] = {"default", "coherent", "noncoherent"};

    // ---------------------------------------------------------------- copies
    if (only == "all" || only == "copies") {
        Host src = host_alloc(T, 0), dst = host_alloc(T, 0);
        std::memcpy(src.h, pt.data(), T);
        auto timed = [&](auto&& fn) {
            fn();
            CK(hipDeviceSynchronize());
            double t = now();
            for (int i = 0; i < reps; ++i) fn();
            CK(hipDeviceSynchronize());
            return (now() - t) / reps;
        };
        double h2d = timed([&] { CK(hipMemcpyAsync(d_a, src.h, T, hipMemcpyHostToDevice, s0)); });
        double d2h = timed([&] { CK(hipMemcpyAsync(dst.h, d_b, T, hipMemcpyDeviceToHost, s1)); });
        double both = timed([&] {
            CK(hipMemcpyAsync(d_a, src.h, T, hipMemcpyHostToDevice, s0));
            CK(hipMemcpyAsync(dst.h, d_b, T, hipMemcpyDeviceToHost, s1));
        });
        std::printf("{\"case\":\"copies\",\"bytes\":%llu,\"h2d_GBs\":%.1f,\"d2h_GBs\":%.1f,\"both_each_GBs\":%.1f}\n",
                    (unsigned long long)T, T / h2d / 1e9, T / d2h / 1e9, T / both / 1e9);
        std::fflush(stdout);
        CK(hipHostFree(src.h));
        CK(hipHostFree(dst.h));
    }

    // ---------------------------------------------------------------- zero-copy kernels
    for (int f = 0; f < 3; ++f) {
        if (only != "all" && only != "zc") break;
        Host in = host_alloc(T, flag_sets[f]), mid = host_alloc(T, flag_sets[f]), back = host_alloc(T, flag_sets[f]);
        std::memcpy(in.h, pt.data(), T);
        // (io: 3 = read host + write host, 1 = read host / write device, 2 = read device / write host)
        for (int io = 3; io >= 1; --io) {
            const uint8_t* sin = (io & 1) ? in.d : d_a;
            uint8_t* smid = (io & 2) ? mid.d : d_b;
            uint8_t* sback = (io & 2) ? back.d : d_b;  // open output (device case reuses d_b after)
            if (!(io & 1)) CK(hipMemcpy(d_a, pt.data(), T, hipMemcpyHostToDevice));
            const uint8_t* oin = (io & 1) ? (io & 2 ? mid.d : mid.d) : d_b;
            // the open reads what the seal wrote: host mid if the seal wrote host, else device d_b
            oin = (io & 2) ? mid.d : d_b;
            uint8_t* oout = (io & 2) ? back.d : d_a;
            (void)sback;
            auto seal = [&] {
                enet_records r = recs(sin, smid, n, d_off, 0);
                EK(enet_aead_seal_batch(&r, nullptr, nullptr, d_tags, s0));
            };
            auto open = [&] {
                enet_records r = recs(oin, oout, n, d_off, 0);
                EK(enet_aead_open_batch(&r, nullptr, nullptr, d_tags, d_ok, s0));
            };
            seal();
            open();
            CK(hipStreamSynchronize(s0));
            float ms_s = 0, ms_o = 0;
            for (int i = 0; i < reps; ++i) {
                float a, b;
                CK(hipEventRecord(e0, s0));
                seal();
                CK(hipEventRecord(e1, s0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&a, e0, e1));
                CK(hipEventRecord(e0, s0));
                open();
                CK(hipEventRecord(e1, s0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&b, e0, e1));
                ms_s += a;
                ms_o += b;
            }
            ms_s /= reps;
            ms_o /= reps;
            std::vector<uint8_t> backh(T);
            if (io & 2) std::memcpy(backh.data(), back.h, T);
            else CK(hipMemcpy(backh.data(), d_a, T, hipMemcpyDeviceToHost));
            check(backh.data(), "zc");
            std::printf("{\"case\":\"zc\",\"flags\":\"%s\",\"read_host\":%d,\"write_host\":%d,\"seal_ms\":%.3f,"
                        "\"open_ms\":%.3f,\"seal_open_GiBs\":%.2f}\n",
                        flag_names[f], io & 1, (io >> 1) & 1, ms_s, ms_o, gib((ms_s + ms_o) * 1e-3));
            std::fflush(stdout);
        }
        CK(hipHostFree(in.h));
        CK(hipHostFree(mid.h));
        CK(hipHostFree(back.h));
    }

    // ---------------------------------------------------------------- library pipeline (reference point)
    if (only == "all" || only == "pipe") {
        Host in = host_alloc(T, 0), mid = host_alloc(T, 0), back = host_alloc(T, 0);
        Host tags = host_alloc(16ull * n, 0), ok = host_alloc(n, 0);
        std::memcpy(in.h, pt.data(), T);
        for (int mode : {0, 1, 2})
        for (uint32_t streams : {3u, 2u, 4u}) {
            for (uint64_t chunk : {0ull, 16ull << 20, 64ull << 20}) {
                if (enet_host_set_mode(mode)) { std::fprintf(stderr, "mode %d: %s\n", mode, enet_last_error()); return 5; }
                enet_pipeline* p = enet_pipeline_create(0, chunk, streams);
                enet_records r{};
                r.count = n;
                r.in_offsets = off.data();
                r.out_offsets = off.data();
                r.keys = keys.data();
                r.key_stride = 32;
                r.nonces = nonces.data();
                r.total_bytes_hint = T;
                r.max_len_hint = (uint32_t)L;
                auto seal = [&] { r.in = in.h; r.out = mid.h; EK(enet_pipeline_aead_seal(p, &r, tags.h)); };
                auto open = [&] { r.in = mid.h; r.out = back.h; EK(enet_pipeline_aead_open(p, &r, tags.h, ok.h)); };
                seal();
                open();
                double t0 = now();
                for (int i = 0; i < reps; ++i) seal();
                double t1 = now();
                for (int i = 0; i < reps; ++i) open();
                double t2 = now();
                uint64_t good = 0;
                for (uint32_t i = 0; i < n; ++i) good += ok.h[i];
                if (good != n || std::memcmp(back.h, pt.data(), T)) { std::fprintf(stderr, "pipe FAILED\n"); return 4; }
                std::printf("{\"case\":\"pipe\",\"mode\":%d,\"streams\":%u,\"chunk_mib\":%llu,\"seal_GiBs\":%.2f,\"open_GiBs\":%.2f,"
                            "\"seal_open_GiBs\":%.2f}\n", mode, streams, (unsigned long long)(chunk >> 20),
                            gib((t1 - t0) / reps), gib((t2 - t1) / reps), gib((t2 - t0) / reps));
                std::fflush(stdout);
                enet_pipeline_destroy(p);
            }
        }
        CK(hipHostFree(in.h));
        CK(hipHostFree(mid.h));
        CK(hipHostFree(back.h));
        CK(hipHostFree(tags.h));
        CK(hipHostFree(ok.h));
    }

    // ---------------------------------------------------------------- half zero-copy pipelines
    // zcout: per chunk on stream k: H2D(chunk) -> kernel(device in -> host out)
    // zcin : per chunk on stream k: kernel(host in -> device out) -> D2H(chunk)
    for (int variant = 0; variant < 2; ++variant) {
        if (only != "all" && only != "half") break;
        Host in = host_alloc(T, 0), mid = host_alloc(T, 0), back = host_alloc(T, 0);
        std::memcpy(in.h, pt.data(), T);
        for (uint32_t S : {1u, 2u, 3u}) {
            for (uint64_t chunk : {16ull << 20, 64ull << 20}) {
                std::vector<hipStream_t> ss(S);
                for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                const uint32_t per = (uint32_t)(chunk / L);
                // per-chunk rebased offsets (uniform batches: every chunk has the same offsets)
                auto pass = [&](bool open, const uint8_t* src_h, const uint8_t* src_d, uint8_t* dst_h, uint8_t* dst_d) {
                    uint32_t k = 0;
                    for (uint32_t c0 = 0; c0 < n; c0 += per, ++k) {
                        const uint32_t m = std::min(per, n - c0);
                        hipStream_t s = ss[k % S];
                        uint8_t* dbuf_in = d_a + (uint64_t)(k % S) * chunk;   // device chunk slots
                        uint8_t* dbuf_out = d_b + (uint64_t)(k % S) * chunk;
                        enet_records r{};
                        if (variant == 0) {  // zcout
                            CK(hipMemcpyAsync(dbuf_in, src_h + c0 * L, (uint64_t)m * L, hipMemcpyHostToDevice, s));
                            r = recs(dbuf_in, dst_d + c0 * L, m, d_off, c0);
                        } else {  // zcin
                            r = recs(src_d + c0 * L, dbuf_out, m, d_off, c0);
                        }
                        if (open) EK(enet_aead_open_batch(&r, nullptr, nullptr, d_tags + 16ull * c0, d_ok + c0, s));
                        else EK(enet_aead_seal_batch(&r, nullptr, nullptr, d_tags + 16ull * c0, s));
                        if (variant == 1)
                            CK(hipMemcpyAsync(dst_h + c0 * L, dbuf_out, (uint64_t)m * L, hipMemcpyDeviceToHost, s));
                    }
                    for (auto& s : ss) CK(hipStreamSynchronize(s));
                };
                auto seal = [&] { pass(false, in.h, in.d, mid.h, mid.d); };
                auto open = [&] { pass(true, mid.h, mid.d, back.h, back.d); };
                seal();
                open();
                double t0 = now();
                for (int i = 0; i < reps; ++i) seal();
                double t1 = now();
                for (int i = 0; i < reps; ++i) open();
                double t2 = now();
                check(back.h, variant ? "zcin" : "zcout");
                std::printf("{\"case\":\"%s\",\"streams\":%u,\"chunk_mib\":%llu,\"seal_GiBs\":%.2f,\"open_GiBs\":%.2f,"
                            "\"seal_open_GiBs\":%.2f}\n", variant ? "zcin" : "zcout", S,
                            (unsigned long long)(chunk >> 20), gib((t1 - t0) / reps), gib((t2 - t1) / reps),
                            gib((t2 - t0) / reps));
                std::fflush(stdout);
                for (auto& s : ss) CK(hipStreamDestroy(s));
            }
        }
        CK(hipHostFree(in.h));
        CK(hipHostFree(mid.h));
        CK(hipHostFree(back.h));
    }
    CK(hipDeviceSynchronize());
    return 0;
}
