// ubench.hip -- microbenchmarks that pin the roofline of the record engine on gfx950.
//   chacha   : ChaCha20 keystream blocks in registers, no memory traffic (int32 ARX ceiling)
//   pmul     : Poly1305 26-bit-limb multiply chains (v_mad_u64_u32 ceiling)
//   copy_*   : 64-byte-per-lane block copy in the engine's access pattern (lane-per-block,
//              records of 4 KiB, P lanes per record) vs a fully coalesced dwordx4 copy
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I../ephemeralnet_amd/csrc ubench.hip -o ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "enet_device.hpp"

using namespace enet;

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ __launch_bounds__(256) void k_chacha(uint32_t* out, int iters, uint32_t seed) {
    uint32_t k[8], n[3];
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    for (int i = 0; i < 8; ++i) k[i] = seed * (i + 1) + gid;
    for (int i = 0; i < 3; ++i) n[i] = seed ^ (i * 7919u) ^ gid;
    ChachaRecord R;
    chacha_record_init(R, k, n);
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t x[16];
        chacha_block(R, (uint32_t)it, x);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= x[i];
    }
    out[gid] = acc;
}

__global__ __launch_bounds__(256) void k_pmul(uint32_t* out, int iters, uint32_t seed) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    uint32_t r[5], h[5], h2[5];
    for (int i = 0; i < 5; ++i) {
        r[i] = (seed * (i + 3) + gid) & M26;
        h[i] = (seed ^ (i * 131u) ^ gid) & M26;
        h2[i] = (seed + i + gid * 3u) & M26;
    }
    Pmul m = pmul_make(r);
    for (int it = 0; it < iters; ++it) {  // two independent chains for ILP
        pmul(h, m);
        h[0] += it;
        pmul(h2, m);
        h2[1] += it;
    }
    uint32_t a = 0;
    for (int i = 0; i < 5; ++i) a ^= h[i] ^ h2[i];
    out[gid] = a;
}

// lane-per-block pattern: record q = gid / P, lane j = gid % P; rounds over blocks j, j+P, ...
template <int P>
__global__ __launch_bounds__(256) void k_copy_blocks(const uint8_t* in, uint8_t* out, uint32_t n,
                                                     uint32_t L) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t q = gid / P, j = gid % P;
    if (q >= n) return;
    const uint32_t nb = L / 64;
    for (uint32_t c = j; c < nb; c += P) {
        const uint4* s = reinterpret_cast<const uint4*>(in + (size_t)q * L + 64ull * c);
        uint4* d = reinterpret_cast<uint4*>(out + (size_t)q * L + 64ull * c);
        uint4 a = s[0], b = s[1], cc = s[2], dd = s[3];
        d[0] = a; d[1] = b; d[2] = cc; d[3] = dd;
    }
}

// segmented: lane j of record q copies blocks [j*B, (j+1)*B) one per step
template <int P>
__global__ __launch_bounds__(256) void k_copy_seg(const uint8_t* in, uint8_t* out, uint32_t n,
                                                  uint32_t L) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t q = gid / P, j = gid % P;
    if (q >= n) return;
    const uint32_t nb = L / 64, B = nb / P;
    for (uint32_t t = 0; t < B; ++t) {
        const size_t off = (size_t)q * L + 64ull * (j * B + t);
        const uint4* s = reinterpret_cast<const uint4*>(in + off);
        uint4* d = reinterpret_cast<uint4*>(out + off);
        uint4 a = s[0], b = s[1], cc = s[2], dd = s[3];
        d[0] = a; d[1] = b; d[2] = cc; d[3] = dd;
    }
}

// segmented, but each step's 64 blocks of a wave are moved cooperatively: 4 coalesced
// dwordx4 instructions (16 blocks x 64 B each), transposed through LDS to lane-per-block.
template <int P>
__global__ __launch_bounds__(256) void k_copy_coop(const uint8_t* in, uint8_t* out, uint32_t n,
                                                   uint32_t L) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[256 * 80];
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wbase = threadIdx.x & ~63u;
    const uint32_t q = gid / P, j = gid % P;
    const uint32_t nb = L / 64, B = nb / P;
    const uint64_t mybase = (q < n) ? (uint64_t)q * L + 64ull * (j * B) : 0;
    uint64_t pbase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int srcl = 16 * i + (lane >> 2);
        pbase[i] = __shfl(mybase, srcl) + 16 * (lane & 3);
    }
    const uint32_t T = (q < n) ? B : 0;
    for (uint32_t t = 0; t < B; ++t) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const uint4*>(in + pbase[i] + 64ull * t);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            *reinterpret_cast<uint4*>(lds + (wbase + 16 * i + (lane >> 2)) * 80 + 16 * (lane & 3)) = v[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint4 w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const uint4*>(lds + threadIdx.x * 80 + 16 * i);
        // (compute would go here) -- write back own block, read transposed, store coalesced
#pragma unroll
        for (int i = 0; i < 4; ++i) { w[i].x ^= 1u; }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(lds + threadIdx.x * 80 + 16 * i) = w[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int i = 0; i < 4; ++i)
            v[i] = *reinterpret_cast<const uint4*>(lds + (wbase + 16 * i + (lane >> 2)) * 80 + 16 * (lane & 3));
        if (t < T || true) {
#pragma unroll
            for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(out + pbase[i] + 64ull * t) = v[i];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// segmented lanes (P per record, lane owns B contiguous blocks) moved in stages of S blocks:
// each global instruction covers 16/S owners x (64*S) contiguous bytes = 1 KiB (whole 128-B
// lines for S >= 2), transposed through LDS (chunk index XOR-swizzled by owner) so that each
// lane then reads / writes its own S blocks.
template <int P, int S>
__global__ __launch_bounds__(256) void k_copy_stage(const uint8_t* in, uint8_t* out, uint32_t n,
                                                    uint32_t L) {
    constexpr int RUN = 64 * S;          // bytes per owner per stage
    constexpr int CH = 4 * S;            // 16-B chunks per owner run
    constexpr int OPI = 16 / S;          // owners per instruction
    __shared__ __attribute__((aligned(16))) uint8_t lds[256 * RUN];
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wbase = threadIdx.x & ~63u;
    const uint32_t q = gid / P, j = gid % P;
    const uint32_t nb = L / 64, B = nb / P;
    const uint64_t mybase = (q < n) ? (uint64_t)q * L + 64ull * (j * B) : 0;
    uint64_t src[4 * S];
    uint32_t lofs[4 * S];
#pragma unroll
    for (int i = 0; i < 4 * S; ++i) {
        const uint32_t o = i * OPI + lane / CH;   // owner lane served by this lane in instr i
        const uint32_t k = lane % CH;              // logical chunk
        src[i] = __shfl(mybase, o) + 16 * k;
        lofs[i] = (wbase + o) * RUN + 16 * (k ^ (o % CH));
    }
    uint8_t* myrow = lds + threadIdx.x * RUN;
    const uint32_t sw = lane % CH;
    for (uint32_t t = 0; t < B; t += S) {
        uint4 v[4 * S];
#pragma unroll
        for (int i = 0; i < 4 * S; ++i) v[i] = *reinterpret_cast<const uint4*>(in + src[i] + 64ull * t);
#pragma unroll
        for (int i = 0; i < 4 * S; ++i) *reinterpret_cast<uint4*>(lds + lofs[i]) = v[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint4 w[4 * S];
#pragma unroll
        for (int k = 0; k < 4 * S; ++k) w[k] = *reinterpret_cast<const uint4*>(myrow + 16 * (k ^ sw));
#pragma unroll
        for (int k = 0; k < 4 * S; ++k) w[k].x ^= 1u;
#pragma unroll
        for (int k = 0; k < 4 * S; ++k) *reinterpret_cast<uint4*>(myrow + 16 * (k ^ sw)) = w[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int i = 0; i < 4 * S; ++i) v[i] = *reinterpret_cast<const uint4*>(lds + lofs[i]);
#pragma unroll
        for (int i = 0; i < 4 * S; ++i) *reinterpret_cast<uint4*>(out + src[i] + 64ull * t) = v[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

__global__ __launch_bounds__(256) void k_copy_coalesced(const uint4* in, uint4* out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

static float time_ms(hipEvent_t a, hipEvent_t b) {
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char** argv) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint32_t* dout;
    const int lanes = 256 * 4096;  // 1M lanes = 16 waves/CU
    CK(hipMalloc(&dout, lanes * 4));

    // chacha ARX ceiling: iters blocks per lane
    for (int occ : {1, 2, 4, 8, 16}) {
        const int blocks = 256 * occ / 4 * 4;  // occ waves per SIMD -> occ*4 waves/CU -> occ WG/CU
        const int iters = 200;
        hipLaunchKernelGGL(k_chacha, dim3(blocks), dim3(256), 0, 0, dout, 4, 1u);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_chacha, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        const double ms = time_ms(e0, e1);
        const double blk = (double)blocks * 256 * iters;
        printf("{\"bench\":\"chacha\",\"waves_per_simd\":%d,\"ms\":%.4f,\"keystream_GBs\":%.1f,"
               "\"blocks_per_s\":%.4e}\n",
               occ, ms, blk * 64 / ms / 1e6, blk / ms * 1e3);
    }
    for (int occ : {1, 2, 4, 8}) {
        const int blocks = 256 * occ;
        const int iters = 2000;
        hipLaunchKernelGGL(k_pmul, dim3(blocks), dim3(256), 0, 0, dout, 4, 1u);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_pmul, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        const double ms = time_ms(e0, e1);
        const double muls = (double)blocks * 256 * iters * 2;
        printf("{\"bench\":\"pmul\",\"waves_per_simd\":%d,\"ms\":%.4f,\"pmul_per_s\":%.4e,"
               "\"poly_GBs_equiv\":%.1f}\n",
               occ, ms, muls / ms * 1e3, muls * 16 / ms / 1e6);
    }

    // memory patterns over 256 MiB
    const uint32_t n = 65536, L = 4096;
    const size_t bytes = (size_t)n * L;
    uint8_t *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    auto run_copy = [&](auto kern, int P, const char* name) {
        const uint32_t threads = n * P;
        const uint32_t blocks = (threads + 255) / 256;
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, a, b, n, L);
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, a, b, n, L);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        const double ms = time_ms(e0, e1) / 10;
        printf("{\"bench\":\"%s\",\"P\":%d,\"ms\":%.4f,\"rw_GBs\":%.1f}\n", name, P, ms, 2.0 * bytes / ms / 1e6);
    };
    run_copy(k_copy_blocks<1>, 1, "copy_blocks");
    run_copy(k_copy_blocks<2>, 2, "copy_blocks");
    run_copy(k_copy_blocks<4>, 4, "copy_blocks");
    run_copy(k_copy_blocks<8>, 8, "copy_blocks");
    run_copy(k_copy_blocks<16>, 16, "copy_blocks");
    run_copy(k_copy_seg<1>, 1, "copy_seg");
    run_copy(k_copy_seg<2>, 2, "copy_seg");
    run_copy(k_copy_seg<4>, 4, "copy_seg");
    run_copy(k_copy_coop<1>, 1, "copy_coop");
    run_copy(k_copy_coop<2>, 2, "copy_coop");
    run_copy(k_copy_coop<4>, 4, "copy_coop");
    run_copy(k_copy_stage<2, 1>, 2, "copy_stage_S1");
    run_copy(k_copy_stage<2, 2>, 2, "copy_stage_S2");
    run_copy(k_copy_stage<2, 4>, 2, "copy_stage_S4");
    run_copy(k_copy_stage<4, 1>, 4, "copy_stage_S1");
    run_copy(k_copy_stage<4, 2>, 4, "copy_stage_S2");
    run_copy(k_copy_stage<4, 4>, 4, "copy_stage_S4");
    run_copy(k_copy_stage<1, 2>, 1, "copy_stage_S2");
    {
        const size_t n16 = bytes / 16;
        hipLaunchKernelGGL(k_copy_coalesced, dim3(4096), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16);
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r)
            hipLaunchKernelGGL(k_copy_coalesced, dim3(4096), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        const double ms = time_ms(e0, e1) / 10;
        printf("{\"bench\":\"copy_coalesced\",\"ms\":%.4f,\"rw_GBs\":%.1f}\n", ms, 2.0 * bytes / ms / 1e6);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
