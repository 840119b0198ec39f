// stream.hip -- the streaming ChaCha20 / ChaCha20-Poly1305 kernel for uniform batches (gfx950).
//
// Shape: every record is L bytes with L a multiple of 128*P (P = lanes per record), records
// contiguous in both arenas (C2: 65 536 x 4 KiB, C4: 64 KiB chunks).  One 512-thread workgroup
// per CU (8 waves, two per SIMD); lane j of record g owns blocks [j*B, (j+1)*B), B = L/(64 P),
// and moves them in stages of two blocks (128 bytes per lane, 8 KiB per wave).
//
// What differs from the staged paths of records_body.hpp (COOP 1/5): the memory traffic is
// spread through the keystream instead of bunched at the stage boundary.
//   * Inputs land in LDS by DMA (global_load_lds_dwordx4, whole 128-byte lines, 8 instructions
//     per stage), into a wave-private input slab; the next stage's 8 DMAs are issued one per
//     keystream half-round while the current stage computes, so the HBM reads of the whole chip
//     arrive as a steady stream rather than one burst per stage, and have most of a stage to land.
//   * Outputs go to a separate wave-private output slab; the previous stage's 8 whole-line
//     stores are likewise issued one per half-round (the lane-linear LDS read one half-round
//     ahead of its store).
//   * 2 x 64 KiB of LDS per workgroup, no prefetch registers.
//   * The keystream is the lockstep pair schedule (enet_device.hpp): both waves of a SIMD meet
//     at s_barrier every 24 ChaCha instructions, so their full-rate adds / xors pair up.
// The LDS chunk swizzle sw(o) = ((o >> 1) & 7) ^ ((o & 1) << 2) makes the own-run ds_read_b128
// (lane groups of 16: (sw, o & 1) distinct) and ds_write_b128 (8 contiguous lanes: sw distinct)
// conflict-free; the lane-linear DMA landing and store reads are contiguous.
//
// A workgroup first checks that each of its records sits at in_off[0] + g*L / out_off[0] + g*L
// (the caller's hints declared the batch uniform); if any does not, the whole workgroup runs the
// per-lane path of records_body.hpp instead (COOP 7), so a wrong hint costs speed, never bytes.
//
// Reference behaviour: ChaCha20::apply (src/crypto/ChaCha20.cpp:98-121, u32 counter wrap :110)
// for MODE_XOR; RFC 8439 AEAD (no reference implementation) for seal / open.
#include "records_body.hpp"

namespace enet {

constexpr uint32_t kStreamWG = 512;

__device__ __forceinline__ uint32_t stream_sw(uint32_t o) { return ((o >> 1) & 7u) ^ ((o & 1u) << 2); }

template <int LOGP, int MODE, int VAR = 0>
__global__ __launch_bounds__(kStreamWG) void stream_kernel(RecParams p) {
    constexpr uint32_t P = 1u << LOGP;
    constexpr bool kPoly = (MODE != MODE_XOR);
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kStreamWG * kRun];
    __shared__ __attribute__((aligned(16))) uint8_t s_out[kStreamWG * kRun];

    const uint32_t L = (uint32_t)p.uniform_len;
    const uint32_t gid = blockIdx.x * kStreamWG + threadIdx.x;
    const uint32_t rec = gid >> LOGP;  // the launch covers records [0, n), n = whole workgroups
    const uint32_t j = gid & (P - 1);
    const uint64_t i0 = p.in_off[0], o0 = p.out_off[0];
    {
        const bool mine = p.in_off[rec] == i0 + (uint64_t)rec * L &&
                          p.in_off[rec + 1] == i0 + (uint64_t)(rec + 1) * L &&
                          p.out_off[rec] == o0 + (uint64_t)rec * L &&
                          p.out_off[rec + 1] == o0 + (uint64_t)(rec + 1) * L;
        if (!__syncthreads_and(mine ? 1 : 0)) {
            records_body<LOGP, MODE, FR_NONE, 7>(p);
            return;
        }
    }

    const uint32_t lane = threadIdx.x & 63u;
    // scalar: the slot tests in the keystream stay SALU branches
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t B = L >> (6 + LOGP);  // blocks per lane (the host launches L % (128 P) == 0)
    const uint32_t S = B >> 1;           // stages
    const uint32_t kk = lane & 7u;
    const uint32_t wgid0 = blockIdx.x * kStreamWG + (wave << 6);
    // load / store roles: instruction i moves 16-byte chunk kk ^ sw(o) of owner o = 8i + lane/8
    // of the wave.  Its arena offset is off(i) = off(i & 1) + (i >> 1) * (16 / P) * L (owner o's
    // record advances by 8/P per instruction for P <= 8 and by 1 per two for P = 16, its lane
    // within the record and sw(o) ^ sw(o mod 16) only alternate).  32-bit offsets from the arena
    // bases: the host launches this kernel only for arenas < 4 GiB.
    uint32_t off01[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const uint32_t o = 8u * i + (lane >> 3);
        const uint32_t go = wgid0 + o;
        off01[i] = (go >> LOGP) * L + (((go & (P - 1)) * B) << 6) + 16u * (kk ^ stream_sw(o));
    }
    const uint32_t offD = (16u >> LOGP) * L;
    const uint32_t offA = off01[0], offAB = off01[1] - off01[0];
    auto off = [&](uint32_t i) { return offA + (i & 1u) * offAB + (i >> 1) * offD; };
    const uint8_t* ibase = p.in + i0;
    uint8_t* obase = p.out + o0;
    const bool nt = p.nt_stores && (reinterpret_cast<uintptr_t>(obase) & 127u) == 0;
    uint8_t* win = s_in + wave * (64u * kRun);
    uint8_t* wout = s_out + wave * (64u * kRun);
    uint8_t* myin = win + lane * kRun;
    uint8_t* myout = wout + lane * kRun;
    const uint32_t msw = stream_sw(lane);

    // ---- per-record ChaCha20 constants
    uint32_t kw[8], nw[3];
    {
        const uint32_t* kp = reinterpret_cast<const uint32_t*>(p.keys + (size_t)p.key_stride * rec);
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = kp[i];
        const uint32_t* np = reinterpret_cast<const uint32_t*>(p.nonces + 12ull * rec);
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = np[i];
    }
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    uint32_t ctr = 1u;  // RFC 8439 data counter
    if (MODE == MODE_XOR)  // reference ChaCha20::apply start counter (0 when not given)
        ctr = p.counters ? p.counters[(size_t)rec * (p.counter_stride ? p.counter_stride : 1u)] : 0u;
    ctr += j * B;  // this lane's first block (u32 wrap, ChaCha20.cpp:110)

    // The DMA is issued from inline asm: the compiler then sees no LDS DMA, and does not put an
    // s_waitcnt vmcnt(0) in front of every later LDS read it cannot prove disjoint from the
    // landing slab (which would wait out each DMA right after issuing it).  The landing is
    // awaited explicitly at the stage start; own-run reads are ordered after that wait by its
    // memory clobber.
    const uint32_t win_lds = (uint32_t)reinterpret_cast<uintptr_t>(win);
    auto dma = [&](uint32_t st, uint32_t i) {
        const uint32_t voff = off(i) + kRun * st;
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(win_lds + 1024u * i);
        asm volatile("s_mov_b32 m0, %1\n s_nop 0\n global_load_lds_dwordx4 %0, %2"
                     :: "v"(voff), "s"(m0), "s"(ibase) : "memory");
    };

    const int dbg = p.dbg;
    uint64_t clk0 = 0, rt0 = 0;
    if (dbg & 256) {  // clock probe: shader cycles and 100 MHz ticks around the whole body
        clk0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
    }
    const bool mem = !(dbg & 1);
    if (mem) {
#pragma unroll
        for (int i = 0; i < 8; ++i) dma(0, i);
    }

    // ---- Poly1305: one-time key from block 0 (runs while stage 0 lands); lane 0 absorbs the AAD
    uint32_t h[5] = {0, 0, 0, 0, 0};
    PolyR32 PR{};
    uint32_t pad[4] = {0, 0, 0, 0};
    uint32_t na = 0, aad_len = 0;
    if (kPoly) {
        uint32_t otk[16];
        chacha_block(R, 0u, otk);
        PR = polyr32_make(otk[0], otk[1], otk[2], otk[3]);
        pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        uint64_t aoff = 0;
        if (p.aad) {
            aoff = p.aad_off[rec];
            aad_len = (uint32_t)(p.aad_off[rec + 1] - aoff);
        }
        na = (aad_len + 15) >> 4;
        if (j == 0) {
            for (uint32_t s = 0; s < na; ++s) {
                const uint8_t* ap = p.aad + aoff + 16ull * s;
                const uint32_t cnt = min(16u, aad_len - 16u * s);
                uint32_t w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t v = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if ((uint32_t)(4 * i + b) < cnt) v |= (uint32_t)ap[4 * i + b] << (8 * b);
                    w[i] = v;
                }
                poly32_block(h, PR, w[0], w[1], w[2], w[3], 1u);
            }
        }
    }

    const uint32_t ff[16] = {kSigma0, kSigma1, kSigma2, kSigma3, R.k[0], R.k[1], R.k[2], R.k[3],
                             R.k[4], R.k[5], R.k[6], R.k[7], 0u, R.n[0], R.n[1], R.n[2]};
    for (uint32_t st = 0; st < S; ++st) {
        // Stage st has landed.  Each memory slot issues its DMA before its store, so from the
        // third stage on only the last store may still be in flight (vmcnt retires in order).
        if (mem && !(dbg & 16)) {
            if (st >= 2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        ENET_WAVE_LDS_SYNC();
        uint32_t w[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint4 v = *reinterpret_cast<const uint4*>(myin + 16u * (k ^ msw));
            w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
        }
        if (MODE == MODE_OPEN && !(dbg & 4)) {
            poly_block64(h, PR, w);
            poly_block64(h, PR, w + 16);
        }
        const bool more = mem && st + 1 < S, prev = mem && st > 0;
        uint4 pv = make_uint4(0, 0, 0, 0);
        if (prev) pv = *reinterpret_cast<const uint4*>(wout + 16u * lane);
        // Memory slot i (0..7) of this wave: DMA i of stage st+1, store i of stage st-1 and the
        // lane-linear read for store i+1.  Slot i runs in double round i+1 after lockstep step
        // `wave` (0..7), so the workgroup's waves take turns at the texture unit one step at a
        // time instead of all eight queueing at the same barrier.
        auto slot = [&](uint32_t i) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own-run reads / pv done
            if (more) dma(st + 1, i);
            if (prev) {
                store_stream(obase + (off(i) + kRun * (st - 1)), pv, nt);
                if (i < 7) pv = *reinterpret_cast<const uint4*>(wout + 1024u * (i + 1) + 16u * lane);
            }
        };
        const uint32_t c0 = ctr + 2u * st;
        uint32_t x[32];
        {
            uint32_t a0 = kSigma0, a4 = R.k[0], a8 = R.k[4], a12 = c0;
            uint32_t b0 = kSigma0, b4 = R.k[0], b8 = R.k[4], b12 = c0 + 1u;
            ENET_QR(a0, a4, a8, a12);
            ENET_QR(b0, b4, b8, b12);
            x[0] = a0; x[4] = a4; x[8] = a8; x[12] = a12;
            x[16] = b0; x[20] = b4; x[24] = b8; x[28] = b12;
#pragma unroll
            for (int c = 1; c < 4; ++c) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    x[c + 4 * r] = R.pre[4 * (c - 1) + r];
                    x[16 + c + 4 * r] = R.pre[4 * (c - 1) + r];
                }
            }
        }
        chacha_half_lockstep2<true>(x);
        // double rounds 1..9 as a loop (not unrolled: the hot loop stays a few KiB of code)
        auto dround = [&](uint32_t dr) {
            const uint32_t my_step = (dr <= 8 && (more || prev)) ? wave : 99u;
            // the slot is rare (1 step in 8): keep the common path free of taken branches -- a
            // taken branch right after the step's s_barrier stalls both waves of the SIMD for the
            // instruction refetch (~100 cycles measured; 72 per stage cost more than HBM did)
            auto at = [&](int k) {
                if (__builtin_expect((uint32_t)k == my_step, 0)) slot(dr - 1);
            };
            if constexpr (VAR & 2) {
                chacha_half_lockstep2<false>(x);
                chacha_half_lockstep2<true>(x);
            } else {
                chacha_half_lockstep2<false>(x, at, 0);
                chacha_half_lockstep2<true>(x, at, 4);
            }
        };
        if constexpr (VAR & 1) {
#pragma unroll
            for (uint32_t dr = 1; dr < 10; ++dr) dround(dr);
        } else {
#pragma unroll 1
            for (uint32_t dr = 1; dr < 10; ++dr) dround(dr);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            w[i] ^= x[i] + (i == 12 ? c0 : ff[i]);
            w[16 + i] ^= x[16 + i] + (i == 12 ? c0 + 1u : ff[i]);
        }
        if (MODE == MODE_SEAL && !(dbg & 4)) {
            poly_block64(h, PR, w);
            poly_block64(h, PR, w + 16);
        }
        // outputs into the own run of the output slab (its previous contents were read above)
#pragma unroll
        for (int k = 0; k < 8; ++k)
            *reinterpret_cast<uint4*>(myout + 16u * (k ^ msw)) =
                make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        ENET_WAVE_LDS_SYNC();
    }
    // the last stage's stores
    if (S > 0 && mem) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = *reinterpret_cast<const uint4*>(wout + 1024u * i + 16u * lane);
            store_stream(obase + (off(i) + kRun * (S - 1)), v, nt);
        }
    }

    if (dbg & 256) {  // 4 words at the workgroup's first tag slot: clk0, rt0, clk1, rt1
        const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0 && p.tag_out) {
            uint64_t* d = reinterpret_cast<uint64_t*>(p.tag_out + 16ull * rec);
            d[0] = clk0; d[1] = rt0; d[2] = clk1; d[3] = rt1;
        }
        return;
    }
    if (kPoly) {
        // length block LE64(|aad|) || LE64(|ct|), owned by the last lane of the record
        const uint32_t nct = L >> 4;
        const uint32_t N = na + nct + 1;
        uint32_t e = 0;  // contribution scale: r^(N-1-s_last)
        if (j == P - 1) poly32_block(h, PR, aad_len, 0u, L, 0u, 1u);
        else e = N - 1 - (na + 4 * (j + 1) * B - 1);
        uint32_t l[5];
        h32_to_limbs(h, l);
        if (P > 1) {
            if (e > 0) {
                uint32_t r26[5], xx[5];
                plimbs(r26, PR.r0, PR.r1, PR.r2, PR.r3);
                ppow(r26, e, xx);
                pmul(l, pmul_make(xx));
            }
#pragma unroll
            for (uint32_t o = P >> 1; o >= 1; o >>= 1) {
#pragma unroll
                for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], (int)o);
            }
        }
        uint32_t tag[4];
        pfinish(l, pad, tag);
        if (MODE == MODE_SEAL) {
            if (j == 0) {
                uint32_t* tp = reinterpret_cast<uint32_t*>(p.tag_out + 16ull * rec);
                tp[0] = tag[0]; tp[1] = tag[1]; tp[2] = tag[2]; tp[3] = tag[3];
            }
        } else {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tag_in + 16ull * rec);
            const uint32_t diff = (tag[0] ^ tp[0]) | (tag[1] ^ tp[1]) | (tag[2] ^ tp[2]) | (tag[3] ^ tp[3]);
            if (j == 0) p.ok[rec] = diff == 0 ? 1 : 0;
            if (diff != 0) {
                // authentication failed: do not release plaintext.  Other lanes of this wave
                // stored this lane's segment (owners are the wave's own lanes): let every store
                // of the wave complete before overwriting it.
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint8_t* seg = obase + (uint64_t)rec * L + ((uint64_t)j * B << 6);
                for (uint32_t c = 0; c < 4 * B; ++c)
                    *reinterpret_cast<uint4*>(seg + 16ull * c) = make_uint4(0, 0, 0, 0);
            }
        }
    }
}

template <int MODE>
static hipError_t launch_stream_mode(const RecParams& p, uint32_t lanes, uint32_t blocks, hipStream_t s) {
    switch (lanes) {
        case 1: hipLaunchKernelGGL((stream_kernel<0, MODE>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        case 2:
            // tuning variants of the C2 shape (ENET_STREAM_VAR: 1 unrolled double rounds, 2 no
            // memory slots -- timing only, 3 both)
            switch (p.var) {
                case 1: hipLaunchKernelGGL((stream_kernel<1, MODE, 1>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
                case 2: hipLaunchKernelGGL((stream_kernel<1, MODE, 2>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
                case 3: hipLaunchKernelGGL((stream_kernel<1, MODE, 3>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
                default: hipLaunchKernelGGL((stream_kernel<1, MODE>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
            }
            break;
        case 4: hipLaunchKernelGGL((stream_kernel<2, MODE>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        case 8: hipLaunchKernelGGL((stream_kernel<3, MODE>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        case 16: hipLaunchKernelGGL((stream_kernel<4, MODE>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

bool stream_eligible(const RecParams& p, uint32_t lanes) {
    const uint64_t L = p.uniform_len;
    return p.stream && L != 0 && p.order == nullptr && L % (128ull * lanes) == 0 &&
           L * (uint64_t)p.n <= 0xFFFFFFFFull && p.n >= kStreamWG / lanes;
}

hipError_t launch_stream(int mode, const RecParams& p, uint32_t lanes, uint32_t blocks, hipStream_t s) {
    switch (mode) {
        case MODE_XOR: return launch_stream_mode<MODE_XOR>(p, lanes, blocks, s);
        case MODE_SEAL: return launch_stream_mode<MODE_SEAL>(p, lanes, blocks, s);
        case MODE_OPEN: return launch_stream_mode<MODE_OPEN>(p, lanes, blocks, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace enet
