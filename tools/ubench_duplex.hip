// ubench_duplex.hip -- compute-only model of duplex_kernel<FRAME, seal, 256> at C3 (1 M wire frames of
// 1 500 B): 512-thread workgroups, 4 cipher waves + 4 hash waves, lane l of cipher wave w and hash
// wave w serving the same record, one workgroup barrier per 128-byte stage, registers only (no
// global memory, no LDS slab).  Per record the real kernel runs 24 ChaCha20 blocks (12 stages of
// chacha_block2: 11 whole stages + the body tail) and 27 SHA-256 compressions (ipad, 22 in the
// stages, 2 tail blocks, opad, outer).  Also: each role alone, and SHA-256 alone at 1/2/4 waves
// per SIMD -- the issue ceiling of the hash lane's instruction mix.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I ephemeralnet_amd/csrc tools/ubench_duplex.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "enet_device.hpp"

using namespace enet;

constexpr int kStages = 11;  // whole 128-byte stages of a 1 500-byte message

// ROLE: 3 = both (the real split), 1 = cipher waves only work, 2 = hash waves only work
template <int ROLE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void k_duplex(uint32_t* out, uint32_t seed) {
    const uint32_t t = blockIdx.x * 512 + threadIdx.x;
    const bool cipher = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < 4u;
    uint32_t acc = 0;
    if (cipher) {
        uint32_t kw[8], nw[3];
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = seed * (i + 3) ^ t;
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = seed + i * t;
        ChachaRecord R;
        chacha_record_init(R, kw, nw);
        uint32_t x[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) x[i] = t * (i + 1);
#pragma unroll 1
        for (int s = 0; s <= kStages; ++s) {  // 11 stages + the tail's two blocks
            if (ROLE & 1) {
                uint32_t ka[16], kb[16];
                chacha_block2(R, 2u * s, 2u * s + 1u, ka, kb);
#pragma unroll
                for (int i = 0; i < 16; ++i) { x[i] ^= ka[i]; x[16 + i] ^= kb[i]; }
            }
            asm volatile("s_barrier" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) acc ^= x[i];
    } else {
        uint32_t st[8], w[16];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kShaIV[i] ^ t;
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = seed * (i + 1) + t;
        // 27 compressions: ipad, two per stage (12 stages: 11 whole + the tail's blocks), opad,
        // outer; the stage barrier after each stage's pair, as in the real hash lane
#pragma unroll 1
        for (int c = 0; c < 27; ++c) {
            if (ROLE & 2) {
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] ^= st[i & 7] + (uint32_t)c;
                sha256_compress(st, w);
            }
            if (c >= 2 && c <= 24 && (c & 1) == 0) asm volatile("s_barrier" ::: "memory");
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= st[i];
    }
    out[t] = acc;
}

// SHA-256 alone: 256-thread workgroups, `occ` workgroups per CU
__global__ __launch_bounds__(256) void k_sha(uint32_t* out, int blocks, uint32_t seed) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t st[8], w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = kShaIV[i] ^ t;
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = seed * (i + 1) + t;
#pragma unroll 1
    for (int b = 0; b < blocks; ++b) {
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] ^= st[i & 7] + (uint32_t)b;
        sha256_compress(st, w);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= st[i];
    out[t] = acc;
}

static float time_ms(hipEvent_t e0, hipEvent_t e1) {
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    const uint32_t n = 1u << 20;  // records (C3)
    uint32_t* d;
    if (hipMalloc(&d, (size_t)2 * n * 4 + (64u << 20)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 g(n / 256), b(512);
    const char* names[] = {"", "cipher waves only", "hash waves only", "cipher + hash (duplex model)"};
    for (int role : {3, 1, 2, 3}) {
        auto launch = [&]() {
            if (role == 3) hipLaunchKernelGGL(k_duplex<3>, g, b, 0, 0, d, 7u);
            else if (role == 1) hipLaunchKernelGGL(k_duplex<1>, g, b, 0, 0, d, 7u);
            else hipLaunchKernelGGL(k_duplex<2>, g, b, 0, 0, d, 7u);
        };
        for (int w = 0; w < 5; ++w) launch();
        hipEventRecord(e0);
        for (int r = 0; r < 20; ++r) launch();
        hipEventRecord(e1);
        const float ms = time_ms(e0, e1) / 20;
        printf("{\"body\":\"%s\",\"records\":%u,\"record_bytes\":1500,\"us_per_launch\":%.1f,"
               "\"seal_GiBs_equiv\":%.1f}\n",
               names[role], n, ms * 1e3, (double)n * 1500 / (ms * 1e-3) / (1u << 30));
    }
    for (int occ : {1, 2, 4}) {
        const int blocks = 64;
        const uint32_t wgs = 256u * occ;  // 256 CUs
        hipLaunchKernelGGL(k_sha, dim3(wgs), dim3(256), 0, 0, d, 4, 1u);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_sha, dim3(wgs), dim3(256), 0, 0, d, blocks, 1u);
        hipEventRecord(e1);
        const float ms = time_ms(e0, e1);
        // ~1 400 VALU instructions per compression (64 rounds x 14 + 48 schedule words x 10)
        const double comp = (double)wgs * 256 * blocks;
        printf("{\"body\":\"sha256_compress\",\"waves_per_simd\":%d,\"G_compressions_per_s\":%.3f,"
               "\"cycles_per_wave_compression_per_simd_at_2.4GHz\":%.0f}\n",
               occ, comp / (ms * 1e6), ms * 1e-3 * 2.4e9 / (occ * (double)blocks));
    }
    return 0;
}
