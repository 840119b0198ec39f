// ubench_issue.hip -- VALU issue cost per instruction class on gfx950 (cycles per wave64
// instruction per SIMD), measured with s_memtime around 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int KIND>
__global__ __launch_bounds__(256) void k_issue(uint64_t* out, int iters, uint32_t seed) {
    uint32_t a[8];
    uint64_t w[8];
    for (int i = 0; i < 8; ++i) { a[i] = seed * (i + 1) + threadIdx.x; w[i] = a[i] * 7ull; }
    const uint32_t b = seed ^ 0x9e3779b9u, c = seed + 12345u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if (KIND == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]));
                if (KIND == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "v"(b) : "vcc");
                if (KIND == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(b), "v"(c));
                if (KIND == 4) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" : "+v"(a[i]), "+v"(a[(i + 4) & 7]) : "v"(b) : "vcc");
                if (KIND == 5) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[i]) : "v"(w[(i + 3) & 7]));
                if (KIND == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t acc = 0;
    for (int i = 0; i < 8; ++i) acc += a[i] + w[i];
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if (acc == 0x123456789ull) out[gridDim.x + blockIdx.x] = acc;
}

int main() {
    uint64_t* d;
    CK(hipMalloc(&d, 1 << 20));
    const char* names[] = {"v_add_u32", "v_alignbit_b32", "v_mad_u64_u32", "v_bitop3_b32",
                           "v_add_co+v_addc_co (2 instr)", "v_lshl_add_u64", "v_mul_lo_u32"};
    for (int occ : {1, 2, 4}) {
        const int blocks = 256 * occ;  // occ waves per SIMD
        for (int kind = 0; kind < 7; ++kind) {
            const int iters = 400;
            auto launch = [&](int it) {
                switch (kind) {
                    case 0: hipLaunchKernelGGL(k_issue<0>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 1: hipLaunchKernelGGL(k_issue<1>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 2: hipLaunchKernelGGL(k_issue<2>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 3: hipLaunchKernelGGL(k_issue<3>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 4: hipLaunchKernelGGL(k_issue<4>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 5: hipLaunchKernelGGL(k_issue<5>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                    case 6: hipLaunchKernelGGL(k_issue<6>, dim3(blocks), dim3(256), 0, 0, d, it, 1u); break;
                }
            };
            launch(50);
            launch(iters);
            CK(hipDeviceSynchronize());
            uint64_t h[1];
            CK(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
            const double instr = (double)iters * 16 * 8 * (kind == 4 ? 2 : 1);
            // s_memtime counts the shader clock; occ waves share one SIMD
            printf("{\"instr\":\"%s\",\"waves_per_simd\":%d,\"cycles_per_wave_instr_per_simd\":%.3f}\n",
                   names[kind], occ, (double)h[0] / (instr * occ));
        }
    }
    return 0;
}
