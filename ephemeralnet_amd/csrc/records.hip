// records.hip -- record kernels and their launch scheduling (gfx950); the body is in
// records_body.hpp.
#include "records_body.hpp"

namespace enet {


template <int LOGP, int MODE, int FRAME, int COOP>
__global__ __launch_bounds__(kWG) void records_kernel(RecParams p) {
    records_body<LOGP, MODE, FRAME, COOP>(p);
}

// 512-thread workgroups with the lockstep keystream (COOP 5, run staging)
template <int LOGP, int MODE>
__global__ __launch_bounds__(512) void records_kernel_l(RecParams p) {
    records_body<LOGP, MODE, FR_NONE, 5>(p);
}

template <int LOGP, int MODE, int FRAME>
static hipError_t launch_one(const RecParams& p, hipStream_t s) {
    const uint64_t lanes = (uint64_t)p.n << LOGP;
    const uint32_t blocks = (uint32_t)((lanes + kWG - 1) / kWG);
    if (blocks == 0) return hipSuccess;
    if (FRAME == FR_NONE && stream_eligible(p, 1u << LOGP)) {
        // the streaming kernel over whole 512-thread workgroups, the rest per lane
        const uint32_t per_wg = 512u >> LOGP;
        const uint32_t full = p.n / per_wg;
        RecParams q = p;
        q.n = full * per_wg;
        if (hipError_t e = launch_stream(MODE, q, 1u << LOGP, full, s)) return e;
        const uint32_t rest = p.n - full * per_wg;
        if (rest) {
            RecParams r = p;
            r.n = rest;
            r.rec_base = full * per_wg;
            hipLaunchKernelGGL((records_kernel<LOGP, MODE, FR_NONE, 0>),
                               dim3((uint32_t)((((uint64_t)rest << LOGP) + kWG - 1) / kWG)),
                               dim3(kWG), 0, s, r);
        }
        return hipGetLastError();
    }
    if (FRAME == FR_NONE && p.uniform_len != 0 && p.order == nullptr && p.coop >= 1) {
        // Cooperative kernels over whole workgroups of records (no dead owners, no store
        // predicates); the remaining records go through the per-lane kernel.
        // Line staging (COOP 4) for one-lane records that are not 64-byte multiples: 1 M
        // records, 1 GPU, GiB/s line vs run staging -- 1500 B 746 vs 590, 1504 B 762 vs 689,
        // 1400 B 750 vs 613; 1472 B 775 vs 789, 1536 B 835 vs 839 (tools/c3ab.sh).
        const bool lines = LOGP == 0 && p.coop == 1 && p.coop_lines && (p.uniform_len & 63u) != 0 &&
                           (p.uniform_len & 3u) == 0 && p.uniform_len < (1u << 24) &&
                           p.uniform_len * (uint64_t)p.n < 0xFFFFFF00ull;
        // Lockstep keystream in 512-thread workgroups (COOP 5) unless a plain variant is asked
        // for: C2 837 -> 864, C4 868 -> 913 GiB/s; not with line staging, where it measured
        // 765 -> 751 at C3 (the line-staging lockstep variant, retired in round 6)
        const bool lock = p.coop == 5 || (p.coop == 1 && p.lockstep && !lines);
        const uint32_t wg = lock ? 512u : (uint32_t)kWG;
        const uint32_t per_wg = wg >> LOGP;
        const uint32_t full = p.n / per_wg;
        if (full) {
            RecParams q = p;
            q.n = full * per_wg;
            if (lines)
                hipLaunchKernelGGL((records_kernel<0, MODE, FR_NONE, 4>), dim3(full), dim3(kWG), 0, s, q);
            else if (lock)
                hipLaunchKernelGGL((records_kernel_l<LOGP, MODE>), dim3(full), dim3(512), 0, s, q);
            else
                hipLaunchKernelGGL((records_kernel<LOGP, MODE, FR_NONE, 1>), dim3(full), dim3(kWG),
                                   0, s, q);
        }
        const uint32_t rest = p.n - full * per_wg;
        if (rest) {
            RecParams q = p;
            q.n = rest;
            q.rec_base = full * per_wg;
            hipLaunchKernelGGL((records_kernel<LOGP, MODE, FR_NONE, 0>),
                               dim3((uint32_t)((((uint64_t)rest << LOGP) + kWG - 1) / kWG)),
                               dim3(kWG), 0, s, q);
        }
        return hipGetLastError();
    }
    hipLaunchKernelGGL((records_kernel<LOGP, MODE, FRAME, 0>), dim3(blocks), dim3(kWG), 0, s, p);
    return hipGetLastError();
}

template <int MODE, int FRAME>
static hipError_t launch_mode(const RecParams& p, uint32_t lanes, hipStream_t s) {
    switch (lanes) {
        case 1: return launch_one<0, MODE, FRAME>(p, s);
        case 2: return launch_one<1, MODE, FRAME>(p, s);
        case 4: return launch_one<2, MODE, FRAME>(p, s);
        case 8: return launch_one<3, MODE, FRAME>(p, s);
        case 16: return launch_one<4, MODE, FRAME>(p, s);
        default: return hipErrorInvalidValue;
    }
}

// mode: MODE_XOR / MODE_SEAL / MODE_OPEN, plus frame variants encoded as 3 (seal) / 4 (open)
hipError_t launch_records(int mode, const RecParams& p, uint32_t lanes, hipStream_t s) {
    switch (mode) {
        case MODE_XOR: return launch_mode<MODE_XOR, FR_NONE>(p, lanes, s);
        case MODE_SEAL: return launch_mode<MODE_SEAL, FR_NONE>(p, lanes, s);
        case MODE_OPEN: return launch_mode<MODE_OPEN, FR_NONE>(p, lanes, s);
        case 3: return launch_mode<MODE_XOR, FR_SEAL>(p, lanes, s);
        case 4: return launch_mode<MODE_XOR, FR_OPEN>(p, lanes, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace enet
