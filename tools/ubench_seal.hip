// ubench_seal.hip -- compute-only model of the seal stage loop (two interleaved keystream
// blocks + eight Poly1305 16-byte blocks per lane per stage, no global memory), to split the
// records kernel's time into VALU work and memory/staging overhead.  Reports G blocks/s and
// cycles per 64-lane stage at 2/3/4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "enet_device.hpp"

using namespace enet;

template <int POLY>
__global__ __launch_bounds__(256) void k_stage(uint32_t* out, int stages, uint32_t seed) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t kw[8], nw[3];
#pragma unroll
    for (int i = 0; i < 8; ++i) kw[i] = seed * (i + 3) ^ t;
#pragma unroll
    for (int i = 0; i < 3; ++i) nw[i] = seed + i * t;
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    PolyR32 PR = polyr32_make(kw[0], kw[1], kw[2], kw[3]);
    uint32_t h[5] = {0, 0, 0, 0, 0};
    uint32_t w2[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) w2[i] = t * (i + 1);
    for (int st = 0; st < stages; ++st) {
        uint32_t ka[16], kb[16];
        chacha_block2(R, 2 * st, 2 * st + 1, ka, kb);
#pragma unroll
        for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
        if (POLY) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                poly32_block(h, PR, w2[4 * u], w2[4 * u + 1], w2[4 * u + 2], w2[4 * u + 3], 1u);
        }
    }
    uint32_t acc = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= w2[i];
    out[t] = acc;
}

// The same stage body with the lockstep keystream (512-thread workgroups, both waves of a SIMD
// in one workgroup, s_barrier every 24 ChaCha instructions) -- the records kernel's default.
template <int POLY>
__global__ __launch_bounds__(512) void k_stage_l(uint32_t* out, int stages, uint32_t seed) {
    const uint32_t t = blockIdx.x * 512 + threadIdx.x;
    uint32_t kw[8], nw[3];
#pragma unroll
    for (int i = 0; i < 8; ++i) kw[i] = seed * (i + 3) ^ t;
#pragma unroll
    for (int i = 0; i < 3; ++i) nw[i] = seed + i * t;
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    PolyR32 PR = polyr32_make(kw[0], kw[1], kw[2], kw[3]);
    uint32_t h[5] = {0, 0, 0, 0, 0};
    uint32_t w2[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) w2[i] = t * (i + 1);
    for (int st = 0; st < stages; ++st) {
        uint32_t ka[16], kb[16];
        chacha_block2_lockstep(R, 2 * st, 2 * st + 1, ka, kb);
#pragma unroll
        for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
        if (POLY) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                poly32_block(h, PR, w2[4 * u], w2[4 * u + 1], w2[4 * u + 2], w2[4 * u + 3], 1u);
        }
    }
    uint32_t acc = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= w2[i];
    out[t] = acc;
}

int coop_main();
int main() {
    if (coop_main()) return 1;
    uint32_t* d;
    if (hipMalloc(&d, 64 << 20) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_stage<1>, dim3(4096), dim3(256), 0, 0, d, 200, 1u);
    hipDeviceSynchronize();
    for (int poly = 0; poly < 2; ++poly) {
        for (int occ : {1, 2, 3, 4}) {
            const int stages = 200;
            auto launch = [&](int s) {
                if (poly) hipLaunchKernelGGL(k_stage<1>, dim3(256 * occ), dim3(256), 0, 0, d, s, 1u);
                else hipLaunchKernelGGL(k_stage<0>, dim3(256 * occ), dim3(256), 0, 0, d, s, 1u);
            };
            launch(10);
            hipEventRecord(e0);
            launch(stages);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double blocks = 256.0 * occ * 256 * stages * 2;
            printf("{\"body\":\"%s\",\"waves_per_simd\":%d,\"Gblocks_per_s\":%.2f,"
                   "\"cycles_per_wave_stage_at_2.4GHz\":%.0f}\n",
                   poly ? "chacha2+poly8" : "chacha2", occ, blocks / (ms * 1e6),
                   ms * 1e-3 * 2.4e9 / (occ * (double)stages));
        }
    }
    for (int poly = 0; poly < 2; ++poly) {  // lockstep: 512-thread workgroups, 2 waves per SIMD
        const int stages = 200;
        auto launch = [&](int s) {
            if (poly) hipLaunchKernelGGL(k_stage_l<1>, dim3(256), dim3(512), 0, 0, d, s, 1u);
            else hipLaunchKernelGGL(k_stage_l<0>, dim3(256), dim3(512), 0, 0, d, s, 1u);
        };
        launch(10);
        hipEventRecord(e0);
        launch(stages);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double blocks = 256.0 * 512 * stages * 2;
        printf("{\"body\":\"%s lockstep\",\"waves_per_simd\":2,\"Gblocks_per_s\":%.2f,"
               "\"cycles_per_wave_stage_at_2.4GHz\":%.0f}\n",
               poly ? "chacha2+poly8" : "chacha2", blocks / (ms * 1e6), ms * 1e-3 * 2.4e9 / (2.0 * stages));
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------
// The COOP-1 stage loop of records_kernel (P = 2 lanes per 4096-B record, 16 stages of two
// blocks per lane) over a real 256 MiB arena, with parts switched off to price them:
//   F_LOAD  global loads of the next stage     F_STORE global stores of the outputs
//   F_LDS   the four LDS passes (off: lanes XOR their prefetch registers directly)
//   F_POLY  Poly1305 over the ciphertext
enum { F_LOAD = 1, F_STORE = 2, F_LDS = 4, F_POLY = 8 };
constexpr uint32_t kRunB = 128;

#define WAVE_LDS_SYNC()                  \
    do {                                 \
        asm volatile("" ::: "memory");   \
        __builtin_amdgcn_wave_barrier(); \
        asm volatile("" ::: "memory");   \
    } while (0)

template <int F>
__global__ __launch_bounds__(256) void k_coop(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                              uint32_t* sink, uint32_t L) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[256 * kRunB];
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    const uint32_t B = (L / 64) / 2;
    const uint32_t j = gid & 1u;
    uint32_t kw[8], nw[3];
#pragma unroll
    for (int i = 0; i < 8; ++i) kw[i] = (gid >> 1) * (i + 7) ^ 0x5a5a5a5au;
#pragma unroll
    for (int i = 0; i < 3; ++i) nw[i] = (gid >> 1) + i;
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    PolyR32 PR = polyr32_make(kw[0], kw[1], kw[2], kw[3]);
    uint32_t h[5] = {0, 0, 0, 0, 0};
    const uint32_t kk = lane & 7u;
    const uint32_t wgid0 = blockIdx.x * 256 + wbase;
    uint64_t off[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t o = 8u * i + (lane >> 3);
        const uint32_t og = (wgid0 + o) >> 1, oj = (wgid0 + o) & 1u;
        const uint32_t sw = (o >> 1) & 7u;
        off[i] = (uint64_t)og * L + 64ull * oj * B + 16u * (((F & F_LDS) ? kk ^ sw : kk));
    }
    uint8_t* wslab = slab + wbase * kRunB;
    uint8_t* myrun = slab + threadIdx.x * kRunB;
    const uint32_t msw = (lane >> 1) & 7u;
    const uint32_t Ts = B / 2;
    uint32_t pf[32];
    auto fetch = [&](uint32_t stage) {
        const uint64_t adv = (uint64_t)kRunB * stage;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (F & F_LOAD) {
                const uint4 v = *reinterpret_cast<const uint4*>(in + off[i] + adv);
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) pf[4 * i + q] = pf[4 * i + q] * 3u + stage;
            }
        }
    };
    auto land = [&]() {
        if (F & F_LDS) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                    make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
        }
    };
#pragma unroll
    for (int i = 0; i < 32; ++i) pf[i] = gid + i;
    fetch(0);
    land();
    uint32_t w2[32];
    for (uint32_t st = 0; st < Ts; ++st) {
        WAVE_LDS_SYNC();
        if (F & F_LDS) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                w2[4 * k] = v.x; w2[4 * k + 1] = v.y; w2[4 * k + 2] = v.z; w2[4 * k + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) w2[i] = pf[i];
        }
        fetch(min(st + 1, Ts - 1));
        asm volatile("" : "+v"(R.k[0]) :: "memory");
        {
            const uint32_t c0 = 1 + j * B + 2 * st;
            uint32_t ka[16], kb[16];
            chacha_block2(R, c0, c0 + 1, ka, kb);
#pragma unroll
            for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
            if (F & F_POLY) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    poly32_block(h, PR, w2[4 * u], w2[4 * u + 1], w2[4 * u + 2], w2[4 * u + 3], 1u);
            }
        }
        WAVE_LDS_SYNC();
        uint32_t o[32];
        if (F & F_LDS) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                    make_uint4(w2[4 * k], w2[4 * k + 1], w2[4 * k + 2], w2[4 * k + 3]);
            WAVE_LDS_SYNC();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                o[4 * i] = v.x; o[4 * i + 1] = v.y; o[4 * i + 2] = v.z; o[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) o[i] = w2[i];
        }
        const uint64_t adv = (uint64_t)kRunB * st;
        if (F & F_STORE) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(out + off[i] + adv) =
                    make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
        } else {
            uint32_t a = 0;
#pragma unroll
            for (int i = 0; i < 32; ++i) a ^= o[i];
            if (a == 0x12345u) sink[gid] = a;
        }
        WAVE_LDS_SYNC();
        land();
    }
    sink[gid] = h[0] ^ h[1] ^ h[2] ^ h[3] ^ h[4];
}

int coop_main() {
    const uint32_t n = 65536, L = 4096;
    uint8_t *in, *out;
    uint32_t* sink;
    if (hipMalloc(&in, (size_t)n * L) != hipSuccess || hipMalloc(&out, (size_t)n * L) != hipSuccess ||
        hipMalloc(&sink, n * 2 * 4) != hipSuccess)
        return 1;
    hipMemset(in, 7, (size_t)n * L);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int flags[] = {15, 13, 14, 11, 9, 7, 3, 12, 8, 0};
    for (int f : flags) {
        auto launch = [&]() {
            const dim3 g(n * 2 / 256), b(256);
            switch (f) {
                case 15: hipLaunchKernelGGL(k_coop<15>, g, b, 0, 0, in, out, sink, L); break;
                case 13: hipLaunchKernelGGL(k_coop<13>, g, b, 0, 0, in, out, sink, L); break;
                case 14: hipLaunchKernelGGL(k_coop<14>, g, b, 0, 0, in, out, sink, L); break;
                case 11: hipLaunchKernelGGL(k_coop<11>, g, b, 0, 0, in, out, sink, L); break;
                case 9: hipLaunchKernelGGL(k_coop<9>, g, b, 0, 0, in, out, sink, L); break;
                case 7: hipLaunchKernelGGL(k_coop<7>, g, b, 0, 0, in, out, sink, L); break;
                case 3: hipLaunchKernelGGL(k_coop<3>, g, b, 0, 0, in, out, sink, L); break;
                case 12: hipLaunchKernelGGL(k_coop<12>, g, b, 0, 0, in, out, sink, L); break;
                case 8: hipLaunchKernelGGL(k_coop<8>, g, b, 0, 0, in, out, sink, L); break;
                case 0: hipLaunchKernelGGL(k_coop<0>, g, b, 0, 0, in, out, sink, L); break;
            }
        };
        for (int w = 0; w < 20; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 50; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 50;
        printf("{\"coop_flags\":\"%s%s%s%s\",\"us\":%.1f,\"GiBs\":%.1f}\n", (f & F_LOAD) ? "load " : "",
               (f & F_STORE) ? "store " : "", (f & F_LDS) ? "lds " : "", (f & F_POLY) ? "poly" : "",
               ms * 1e3, (double)n * L / (ms * 1e-3) / (1 << 30));
    }
    return 0;
}
