// ubench_mix3.hip -- how do full-rate (v_add/v_xor, 2 cycles with two waves) and half-rate
// (v_alignbit, 4 cycles) VALU instructions share a gfx950 SIMD?  Event-timed; 8 independent
// chains per lane; 512-thread workgroups (waves w and w+4 share a SIMD), one or more
// workgroups per CU.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

#define ADD(a) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a) : "v"(b))
#define XOR(a) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a) : "v"(b))
#define ROT(a) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a))

// P: instruction pattern per chain step.  Returns number of instructions per chain step.
//  0: A        1: R        2: A R      3: A A R     4: A X R (chacha mix, independent)
//  5: A A A R  6: specialised: waves 0-3 of the WG run A, waves 4-7 run R
//  7: specialised: waves 0-3 run A X, waves 4-7 run R R (same 2:1 totals as pattern 3 w/ A A R)
//  8: blocks of 8 A then 8 R (grouped, not interleaved)
//  9: A A R but R on the chain written two steps earlier (more slack)
template <int P>
__global__ __launch_bounds__(512) void k(uint32_t* out, int iters, uint32_t seed) {
    uint32_t x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = seed * (i + 1) + threadIdx.x * 77u + blockIdx.x;
    uint32_t b = seed ^ 0x9e3779b9u;
    asm volatile("" : "+v"(b));
    const bool upper = (threadIdx.x >> 8) & 1;  // waves 4..7
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (P == 8) {
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(x[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) ROT(x[i]);
                continue;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (P == 0) ADD(x[i]);
                if (P == 1) ROT(x[i]);
                if (P == 2) { ADD(x[i]); ROT(x[(i + 4) & 7]); }
                if (P == 3) { ADD(x[i]); ADD(x[(i + 2) & 7]); ROT(x[(i + 4) & 7]); }
                if (P == 4) { ADD(x[i]); XOR(x[(i + 2) & 7]); ROT(x[(i + 4) & 7]); }
                if (P == 5) { ADD(x[i]); ADD(x[(i + 2) & 7]); XOR(x[(i + 6) & 7]); ROT(x[(i + 4) & 7]); }
                if (P == 6) { if (!upper) ADD(x[i]); else ROT(x[i]); }
                if (P == 7) { if (!upper) { ADD(x[i]); XOR(x[(i + 4) & 7]); } else { ROT(x[i]); ROT(x[(i + 4) & 7]); } }
                if (P == 9) { ADD(x[i]); ADD(x[(i + 1) & 7]); ROT(x[(i + 6) & 7]); }
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= x[i];
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
    uint32_t* d;
    CK(hipMalloc(&d, 64 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k<0>, dim3(4096), dim3(512), 0, 0, d, 20000, 1u);
    CK(hipDeviceSynchronize());
    const char* names[] = {"A", "R", "A R", "A A R", "A X R", "A A X R", "spec A | R",
                           "spec AX | RR", "8A 8R grouped", "A A R (slack)"};
    const double ipc[] = {1, 1, 2, 3, 3, 4, 1, 2, 2, 3};
    for (int p = 0; p < 10; ++p) {
        for (int wgs : {1, 2}) {  // 512-thread WGs per CU -> 2 or 4 waves per SIMD
            auto launch = [&](int it) {
                dim3 g(256 * wgs), bl(512);
                switch (p) {
                    case 0: hipLaunchKernelGGL(k<0>, g, bl, 0, 0, d, it, 1u); break;
                    case 1: hipLaunchKernelGGL(k<1>, g, bl, 0, 0, d, it, 1u); break;
                    case 2: hipLaunchKernelGGL(k<2>, g, bl, 0, 0, d, it, 1u); break;
                    case 3: hipLaunchKernelGGL(k<3>, g, bl, 0, 0, d, it, 1u); break;
                    case 4: hipLaunchKernelGGL(k<4>, g, bl, 0, 0, d, it, 1u); break;
                    case 5: hipLaunchKernelGGL(k<5>, g, bl, 0, 0, d, it, 1u); break;
                    case 6: hipLaunchKernelGGL(k<6>, g, bl, 0, 0, d, it, 1u); break;
                    case 7: hipLaunchKernelGGL(k<7>, g, bl, 0, 0, d, it, 1u); break;
                    case 8: hipLaunchKernelGGL(k<8>, g, bl, 0, 0, d, it, 1u); break;
                    case 9: hipLaunchKernelGGL(k<9>, g, bl, 0, 0, d, it, 1u); break;
                }
            };
            const int iters = 2000;
            launch(20);
            CK(hipEventRecord(e0));
            launch(iters);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double instr_per_simd = 2.0 * wgs * iters * 8 * 8 * ipc[p];
            printf("{\"pattern\":\"%s\",\"waves_per_simd\":%d,\"cyc_per_instr\":%.3f}\n", names[p],
                   2 * wgs, ms * 1e-3 * 2.4e9 / instr_per_simd);
        }
    }
    return 0;
}
