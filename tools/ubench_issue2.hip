// ubench_issue2.hip -- does a second wave on the SIMD add VALU throughput for (a) a long
// unrolled body of independent adds, (b) ChaCha quarter-round chains (8 and 4 independent)?
// Reports shader cycles per wave64 VALU instruction per SIMD (kernel event time x clock).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
#define ROTL(v, n) __builtin_amdgcn_alignbit((v), (v), 32 - (n))
#define QR(a, b, c, d) \
    a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12); \
    a += b; d ^= a; d = ROTL(d, 8);  c += d; b ^= c; b = ROTL(b, 7);

template <int KIND>
__global__ __launch_bounds__(256) void k_body(uint32_t* out, int iters, uint32_t seed) {
    uint32_t x[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) x[i] = seed * (i + 1) + threadIdx.x * 77u + blockIdx.x;
    const uint32_t b = seed ^ 0x9e3779b9u;
    for (int it = 0; it < iters; ++it) {
        if (KIND == 0) {  // 2048 independent adds, 8 chains, fully unrolled (~8 KB of code)
#pragma unroll
            for (int r = 0; r < 256; ++r) {
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(b));
            }
        } else if (KIND == 1) {  // 8 ChaCha columns (two blocks) x 10 double rounds
#pragma unroll
            for (int r = 0; r < 10; ++r) {
                QR(x[0], x[4], x[8], x[12]); QR(x[16], x[20], x[24], x[28]);
                QR(x[1], x[5], x[9], x[13]); QR(x[17], x[21], x[25], x[29]);
                QR(x[2], x[6], x[10], x[14]); QR(x[18], x[22], x[26], x[30]);
                QR(x[3], x[7], x[11], x[15]); QR(x[19], x[23], x[27], x[31]);
                QR(x[0], x[5], x[10], x[15]); QR(x[16], x[21], x[26], x[31]);
                QR(x[1], x[6], x[11], x[12]); QR(x[17], x[22], x[27], x[28]);
                QR(x[2], x[7], x[8], x[13]); QR(x[18], x[23], x[24], x[29]);
                QR(x[3], x[4], x[9], x[14]); QR(x[19], x[20], x[25], x[30]);
            }
        } else {  // one block: 4 chains
#pragma unroll
            for (int r = 0; r < 10; ++r) {
                QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
                QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
                QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
                QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc ^= x[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    uint32_t* d;
    CK(hipMalloc(&d, 64 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int clk_khz = 0;
    CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
    const char* names[] = {"adds_long_body", "chacha_8chains", "chacha_4chains"};
    const double ipi[] = {2048.0, 10 * 16 * 12.0, 10 * 8 * 12.0};  // VALU instr per iteration
    // warm the clocks
    hipLaunchKernelGGL(k_body<1>, dim3(4096), dim3(256), 0, 0, d, 2000, 1u);
    CK(hipDeviceSynchronize());
    for (int kind = 0; kind < 3; ++kind) {
        for (int occ : {1, 2, 4}) {
            const int blocks = 256 * occ;
            const int iters = kind == 0 ? 400 : 600;
            auto launch = [&](int it) {
                if (kind == 0) hipLaunchKernelGGL(k_body<0>, dim3(blocks), dim3(256), 0, 0, d, it, 1u);
                if (kind == 1) hipLaunchKernelGGL(k_body<1>, dim3(blocks), dim3(256), 0, 0, d, it, 1u);
                if (kind == 2) hipLaunchKernelGGL(k_body<2>, dim3(blocks), dim3(256), 0, 0, d, it, 1u);
            };
            launch(20);
            CK(hipEventRecord(e0));
            launch(iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            // wave-instructions per SIMD = occ waves x iters x ipi; cycles at the nominal clock
            const double cyc = ms * 1e-3 * 2.4e9;
            printf("{\"body\":\"%s\",\"waves_per_simd\":%d,\"ms\":%.4f,"
                   "\"cycles_per_wave_instr_per_simd_at_2.4GHz\":%.3f}\n",
                   names[kind], occ, ms, cyc / (occ * (double)iters * ipi[kind]));
        }
    }
    printf("{\"clock_rate_khz_reported\":%d}\n", clk_khz);
    return 0;
}
