// ubench_mix.hip -- which VALU instruction forms reach the 2-cycle (two waves interleaved)
// issue rate on gfx950 and which stay at 4?  Event-timed, 8 independent chains per lane,
// 1/2/4 waves per SIMD.  Prints cycles per wave64 instruction per SIMD at the measured clock
// assumption of 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int V>
__global__ __launch_bounds__(256) void k_mix(uint32_t* out, int iters, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = seed * (i + 1) + threadIdx.x * 77u + blockIdx.x;
    uint32_t b = seed ^ 0x9e3779b9u, c = seed * 3u + 1u;
    asm volatile("" : "+v"(b), "+v"(c));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                uint32_t& a = x[i];
                uint32_t& o = x[(i + 4) & 7];
                if (V == 0) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 1) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a));
                if (V == 3) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a) : "v"(b));
                if (V == 4) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a) : "v"(o));
                if (V == 5) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 6) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(a) : "v"(c));
                if (V == 7) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
                if (V == 8) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a) : "v"(b));
                if (V == 9) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
                if (V == 10) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a) : "v"(b), "v"(c));
                if (V == 11) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a));
                if (V == 12) asm volatile("v_lshlrev_b32_e32 %0, 7, %0" : "+v"(a));
                if (V == 13) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a) : "v"(o));
                if (V == 14) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 15) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a) : "v"(o));
                if (V == 16) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(a) : "v"(b) : "vcc");
                if (V == 17) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 18) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
                if (V == 19) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
                if (V == 20) asm volatile("v_lshrrev_b32_e32 %0, 7, %0" : "+v"(a));
                if (V == 21) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a) : "v"(b));
                if (V == 22) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(a) : "v"(b));
                if (V == 23) asm volatile("v_alignbit_b32 %0, %1, %0, 7" : "+v"(a) : "v"(o));
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// ChaCha quarter-round chains written as explicit asm, 8 columns (2 blocks), varied forms.
#define QRA(a, b, c, d, R16, R12, R8, R7)                                       \
    asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a) : "v"(b));                \
    asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(d) : "v"(a));                \
    R16(d);                                                                     \
    asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(c) : "v"(d));                \
    asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(b) : "v"(c));                \
    R12(b);                                                                     \
    asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a) : "v"(b));                \
    asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(d) : "v"(a));                \
    R8(d);                                                                      \
    asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(c) : "v"(d));                \
    asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(b) : "v"(c));                \
    R7(b);
#define ROT_AB(n) [&](uint32_t& v) { asm volatile("v_alignbit_b32 %0, %0, %0, " #n : "+v"(v)); }

template <int V>
__global__ __launch_bounds__(256) void k_qr(uint32_t* out, int iters, uint32_t seed) {
    uint32_t x[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = seed * (i + 1) + threadIdx.x * 77u + blockIdx.x;
    auto r16 = ROT_AB(16);
    auto r12 = ROT_AB(20);
    auto r8 = ROT_AB(24);
    auto r7 = ROT_AB(25);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (V == 0) {  // column + diagonal rounds, QR by QR (compiler may not reorder asm volatile)
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    uint32_t* y = x + 16 * blk;
                    QRA(y[0], y[4], y[8], y[12], r16, r12, r8, r7);
                    QRA(y[1], y[5], y[9], y[13], r16, r12, r8, r7);
                    QRA(y[2], y[6], y[10], y[14], r16, r12, r8, r7);
                    QRA(y[3], y[7], y[11], y[15], r16, r12, r8, r7);
                }
            } else {  // 8 QRs interleaved step by step (what the compiler emits)
#define STEP(OP) for (int q = 0; q < 8; ++q) { uint32_t* y = x + 16 * (q >> 2); const int k = q & 3; OP; }
                STEP(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(y[k]) : "v"(y[4 + k])));
                STEP(asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(y[12 + k]) : "v"(y[k])));
                STEP(r16(y[12 + k]));
                STEP(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(y[8 + k]) : "v"(y[12 + k])));
                STEP(asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(y[4 + k]) : "v"(y[8 + k])));
                STEP(r12(y[4 + k]));
                STEP(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(y[k]) : "v"(y[4 + k])));
                STEP(asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(y[12 + k]) : "v"(y[k])));
                STEP(r8(y[12 + k]));
                STEP(asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(y[8 + k]) : "v"(y[12 + k])));
                STEP(asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(y[4 + k]) : "v"(y[8 + k])));
                STEP(r7(y[4 + k]));
#undef STEP
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename F>
static double run(F launch, int occ, double instr_per_iter, int iters, hipEvent_t e0, hipEvent_t e1) {
    launch(occ, 20);
    hipEventRecord(e0);
    launch(occ, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e-3 * 2.4e9 / (occ * (double)iters * instr_per_iter);
}

#define MIX(V, NAME)                                                                            \
    for (int occ : {1, 2, 4}) {                                                                 \
        double c = run([&](int o, int it) { hipLaunchKernelGGL(k_mix<V>, dim3(256 * o), dim3(256), 0, 0, d, it, 1u); }, \
                       occ, 128.0, 2000, e0, e1);                                               \
        printf("{\"form\":\"%s\",\"waves_per_simd\":%d,\"cyc\":%.3f}\n", NAME, occ, c);       \
    }

int main() {
    uint32_t* d;
    CK(hipMalloc(&d, 64 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_mix<0>, dim3(4096), dim3(256), 0, 0, d, 20000, 1u);
    CK(hipDeviceSynchronize());
    MIX(0, "v_add_u32 a,a,b");
    MIX(1, "v_xor_b32 a,a,b");
    MIX(2, "v_alignbit a,a,a,7");
    MIX(3, "v_alignbit a,a,b,7");
    MIX(4, "v_add_u32 a,a,o(chain)");
    MIX(5, "v_add_u32_e64 a,a,b");
    MIX(6, "v_perm_b32 a,a,a,c");
    MIX(7, "v_xad_u32 a,a,b,c");
    MIX(8, "v_lshl_or_b32 a,a,7,b");
    MIX(9, "v_add3_u32 a,a,b,c");
    MIX(10, "v_bitop3 a,a,b,c");
    MIX(11, "v_alignbit a,a,a,16");
    MIX(12, "v_lshlrev_b32 a,7,a");
    MIX(13, "v_xor_b32 a,a,o(chain)");
    MIX(14, "v_pk_add_u16 a,a,b");
    MIX(15, "v_mov_b32 a,o");
    MIX(16, "v_add_co_u32 a,vcc,a,b");
    MIX(17, "v_mul_u32_u24 a,a,b");
    MIX(18, "v_mad_u32_u24 a,a,b,c");
    MIX(19, "v_and_or_b32 a,a,b,c");
    MIX(20, "v_lshrrev_b32 a,7,a");
    MIX(21, "v_cndmask_b32 a,a,b,vcc");
    MIX(22, "v_and_b32 a,a,b");
    MIX(23, "v_alignbit a,o,a,7");
    for (int v = 0; v < 2; ++v)
        for (int occ : {1, 2, 4}) {
            double c = run([&](int o, int it) {
                if (v == 0) hipLaunchKernelGGL(k_qr<0>, dim3(256 * o), dim3(256), 0, 0, d, it, 1u);
                else hipLaunchKernelGGL(k_qr<1>, dim3(256 * o), dim3(256), 0, 0, d, it, 1u);
            }, occ, 10 * 8 * 12.0, 500, e0, e1);
            printf("{\"form\":\"chacha_qr_%s\",\"waves_per_simd\":%d,\"cyc\":%.3f}\n",
                   v == 0 ? "sequential" : "interleaved8", occ, c);
        }
    return 0;
}
