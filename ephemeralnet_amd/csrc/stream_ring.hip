// stream_ring.hip -- the streaming ChaCha20 / ChaCha20-Poly1305 kernel for uniform batches whose
// record length is NOT a multiple of 128 bytes (C3: 1 M x 1 500 B MTU frames), gfx950.
//
// The headline kernel (stream.hip) moves whole 128-byte lines because its records start on line
// boundaries.  A 1 500-byte record starts only 4-byte aligned, so its 128-byte runs straddle
// lines.  Same split of the workgroup here (8 lockstep compute waves = 512 record lanes, 4
// memory waves, one 768-thread workgroup per CU), with the two directions handled differently:
//   * loads: the memory waves' LDS DMAs fetch each owner's record-relative run directly (16-byte
//     pieces at 4-byte-aligned addresses; a load that straddles a line just touches both);
//   * stores: a partial line written now and completed a stage later is what costs (the L2 evicts
//     it half-written, and HBM3E has no byte mask), so outputs leave as whole 64-byte units of the
//     ARENA.  Each owner has a 3-unit output ring in LDS (192 B); the compute lane writes run s at
//     ring byte (d + 128 s) mod 192, d = record start mod 64, unit u in slot u mod 3.  Run s
//     completes units 2s and 2s+1 (unit 2s's first d bytes came from run s-1) and half-fills 2s+2;
//     the memory waves store units 2s, 2s+1 during stage s+1, before run s+1 overwrites their
//     slots at its end.  LDS: 64 KiB input slab + 96 KiB ring = the whole 160 KiB.
// A record's first unit holds its predecessor's last bytes and its unit 2S its own partial end,
// so neither goes through the ring: the compute lane stores record bytes [0, 64) and
// [128 S - 64, 128 S) itself (unaligned 16-byte pieces, once per record; bytes that the memory
// waves also store are written with equal values), and the ragged end (L mod 128 bytes) with
// per-lane loads and stores (16-byte windows ending at the record end).
//
// Reference behaviour: ChaCha20::apply (src/crypto/ChaCha20.cpp:98-121, u32 counter wrap :110)
// for MODE_XOR; RFC 8439 AEAD (no reference implementation) for seal / open.
#include "records_body.hpp"

namespace enet {

namespace {

constexpr uint32_t kRingLanes = 512;   // record lanes per workgroup (8 compute waves)
constexpr uint32_t kRingWG = 768;      // + 4 memory waves
constexpr uint32_t kRingBytes = 192;   // three 64-byte output units per owner
constexpr int kRingPos = 76;           // keystream barriers per stage (19 lockstep half-rounds)

typedef const __attribute__((address_space(1))) enet_u32x4 gvec4;

__device__ __forceinline__ void ring_barrier() { asm volatile("s_barrier" ::: "memory"); }

// keep bytes [0, r) of the LE byte string w[0..32)
__device__ __forceinline__ void keep_le32(uint32_t w[32], uint32_t r) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const uint32_t b = 4u * j;
        w[j] &= b + 4u <= r ? 0xffffffffu : (b >= r ? 0u : (1u << (8u * (r - b))) - 1u);
    }
}

__device__ __forceinline__ void put16(uint8_t* p, const uint32_t* w) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
        reinterpret_cast<uint4*>(p)[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

}  // namespace

// NT: non-temporal unit stores (tuning; units are line halves, which nt does not merge)
// LD: input path -- 0 dword LDS DMAs, 1 dwordx4 loads into the memory waves' VGPRs + ds_write_b128
template <int MODE, int NT, int LD = 0>
__global__ __launch_bounds__(kRingWG) void stream_ring_kernel(RecParams p) {
    constexpr bool kPoly = (MODE != MODE_XOR);
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kRingLanes * kRun];
    __shared__ __attribute__((aligned(16))) uint8_t s_ring[kRingLanes * kRingBytes];

    const uint32_t L = (uint32_t)p.uniform_len;
    const bool compute = threadIdx.x < kRingLanes;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t rec = blockIdx.x * kRingLanes + (compute ? threadIdx.x : 0u);
    const uint64_t i0 = p.in_off[0], o0 = p.out_off[0];
    const uintptr_t in0 = reinterpret_cast<uintptr_t>(p.in + i0), out0 = reinterpret_cast<uintptr_t>(p.out + o0);
    {
        // The hints declared the batch uniform: every record of the workgroup must sit at
        // in_off[0] + g L / out_off[0] + g L, and the ring needs 4-byte-aligned arenas.  Else the
        // workgroup takes the per-lane path.  (A wave ballot per wave in LDS: __syncthreads_and
        // would add a scratch word to the 160 KiB.)
        const bool mine = ((in0 | out0) & 3u) == 0 &&
                          (!compute || (p.in_off[rec] == i0 + (uint64_t)rec * L &&
                                        p.in_off[rec + 1] == i0 + (uint64_t)(rec + 1) * L &&
                                        p.out_off[rec] == o0 + (uint64_t)rec * L &&
                                        p.out_off[rec + 1] == o0 + (uint64_t)(rec + 1) * L));
        const uint64_t bal = __ballot(mine ? 1 : 0);
        volatile uint32_t* flags = reinterpret_cast<volatile uint32_t*>(s_ring);
        if (lane == 0) flags[wave] = bal == ~0ull ? 1u : 0u;
        __syncthreads();
        uint32_t all = 1;
#pragma unroll
        for (uint32_t w = 0; w < kRingWG / 64; ++w) all &= flags[w];
        __syncthreads();  // the flags are read before the ring is written
        if (!all) {
            if (compute) records_body<0, MODE, FR_NONE, 7>(p);
            return;
        }
    }
    const uint32_t S = L >> 7;       // whole 128-byte stages (host: L >= 128, L % 128 != 0)
    const uint32_t T = L & 127u;     // ragged end
    // output units: arena bytes relative to abase (= out0 rounded down to 64); record g starts at
    // unit ((d0 + g L) >> 6), byte (d0 + g L) & 63 of it
    const uintptr_t abase = out0 & ~(uintptr_t)63;
    const uint32_t d0 = (uint32_t)(out0 & 63u);

    if (!compute) {
        // ================================================================ memory waves
        // memory wave m serves compute waves 2m, 2m+1 (owners 128 m .. 128 m + 127 of the WG)
        const uint32_t m = wave - 8u;
        __builtin_amdgcn_s_setprio(3);
        // Input runs arrive by 64 dword LDS DMAs per stage (global_load_lds_dword, 256 B: two
        // owners' 128-byte runs).  A 16-byte DMA piece at a 4-byte-aligned address is split by the
        // texture path: dwordx4 DMAs of the runs took 707 us per C3 seal for the loads alone.
        // DMA i = 8a + b covers owners 2i + h (h = lane >> 5) of the wave's 128, dword w = lane & 31
        // of the run, which lands at chunk position w >> 2 of the owner's slab run and therefore
        // holds chunk (w >> 2) ^ sw(o) (the compute lanes' swizzle, sw(o) = b ^ 4h for o = 16a + 2b + h):
        // lane offset pre[b] + SGPR 16 a L.
        const uint32_t h = lane >> 5, w = lane & 31u;
        uint32_t pre[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const uint32_t g = blockIdx.x * kRingLanes + 128u * m + 2u * (uint32_t)b + h;
            pre[b] = g * L + 16u * ((w >> 2) ^ (uint32_t)b ^ (h << 2)) + 4u * (w & 3u);
        }
        // LD 1: 16 loads of 16-byte pieces per stage (slot s: owner 8 (s & 7) + lane / 8 of compute
        // wave 2m + (s >> 3), chunk (lane & 7) ^ sw(o), landing lane-linear as a DMA would)
        uint32_t doff[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const uint32_t o = 8u * (uint32_t)(s & 7) + (lane >> 3);
            const uint32_t g = blockIdx.x * kRingLanes + (2u * m + (uint32_t)(s >> 3)) * 64u + o;
            doff[s] = g * L + 16u * ((lane & 7u) ^ slab_sw(o));
        }
        uint8_t* const land = s_in + 2u * m * (64u * kRun) + 16u * lane;
        const uint32_t land_a = (uint32_t)reinterpret_cast<uintptr_t>(land);
        // store slot t (0..15): owners 8t .. 8t+7 of the wave's 128; lane -> owner 8t + ((l >> 2) & 7),
        // unit j = l >> 5 of the run's two, 16-byte piece k = l & 3 (16-lane groups of the LDS read
        // then cover four owners' same unit: 48-dword owner stride -> banks 0/48/32/16, conflict-free)
        const uint32_t op = (lane >> 2) & 7u, j = lane >> 5, k = lane & 3u;
        uint32_t soff[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint32_t g = blockIdx.x * kRingLanes + 128u * m + 8u * (uint32_t)t + op;
            soff[t] = ((d0 + g * L) & ~63u) + 64u * j + 16u * k;
        }
        auto uni = [](uintptr_t v) {
            return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
        };
        const uint8_t* ibase = reinterpret_cast<const uint8_t*>(uni(in0));
        const uint32_t in_part = (uint32_t)reinterpret_cast<uintptr_t>(s_in) + 2u * m * (64u * kRun);
        const uint8_t* rown = s_ring + kRingBytes * (128u * m + op) + 16u * k;
        auto dma = [&](const uint8_t* base, int i) {
            const uint8_t* b = base + (size_t)(16u * (uint32_t)(i >> 3)) * L;
            uint32_t keep;
            // M0 = slab part + 256 i, formed in the statement (64 precomputed M0 values would
            // spill SGPRs into VGPR lanes, i.e. VALU in the slots)
            asm volatile("s_mov_b32 %0, m0\n s_add_u32 m0, %2, %4\n s_nop 0\n global_load_lds_dword %1, %3 nt\n s_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(pre[i & 7]), "s"(in_part), "s"(b), "n"(256 * i) : "memory", "scc");
        };
        auto store = [&](uint8_t* base, int t, uint4 v) {
            enet_u32x4 d = {v.x, v.y, v.z, v.w};
            if constexpr (NT)
                asm volatile("global_store_dwordx4 %0, %1, %2 nt\n s_nop 1" :: "v"(soff[t]), "v"(d), "s"(base) : "memory");
            else
                asm volatile("global_store_dwordx4 %0, %1, %2\n s_nop 1" :: "v"(soff[t]), "v"(d), "s"(base) : "memory");
        };
        // units 2r, 2r + 1 of run r sit in slots (2r + j) mod 3; unit 0 of run 0 is not stored
        // (its head is the previous record's)
        auto unit_read = [&](const uint8_t* ru, int t) {
            return *reinterpret_cast<const uint4*>(ru + kRingBytes * 8u * (uint32_t)t);
        };
        auto run_unit_base = [&](uint32_t r) {
            uint32_t sl = (2u * r) % 3u + j;
            sl = sl >= 3u ? sl - 3u : sl;
            return rown + 64u * sl;
        };
        if constexpr (LD == 0) {
#pragma unroll
            for (int i = 0; i < 64; ++i) dma(ibase, i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2)
                *reinterpret_cast<enet_u32x4*>(land + 1024u * s2) =
                    __builtin_nontemporal_load((gvec4*)(ibase + doff[s2]));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        for (uint32_t st = 0; st < S; ++st) {
            ring_barrier();  // S0(st): run st landed; run st-1's outputs are in the ring
            const bool more = st + 1 < S && !(p.dbg & 128), prev = st > 0 && !(p.dbg & 64);
            const uint8_t* inext = ibase + (size_t)kRun * (st + 1);
            uint8_t* obase = reinterpret_cast<uint8_t*>(uni(abase + (uintptr_t)kRun * (st - 1)));
            const uint8_t* ru = prev ? run_unit_base(st - 1) : rown;
            const bool skip0 = st == 1 && j == 0;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (prev) v = unit_read(ru, 0);
            enet_u32x4 ldv[16];
            // DMAs 2 per position at 1..32 (after barrier 0: the compute waves hold their runs),
            // then the 16 unit stores at 33, 35, ..., 63: every store is younger than every DMA, so
            // the stage-end wait for the DMAs leaves the stores in flight
#pragma unroll
            for (int q = 0; q < kRingPos; ++q) {
                if (LD == 0 && q >= 1 && q <= 32) {
                    if (more) {
                        dma(inext, 2 * (q - 1));
                        dma(inext, 2 * (q - 1) + 1);
                    }
                }
                // (asm: a 64-bit address add per load would put VALU in the slots; the loaded
                // registers are only touched by the write statement, which waits for them itself)
                if (LD == 1 && q >= 1 && q <= 16) {
                    if (more)
                        asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(ldv[q - 1]) : "v"(doff[q - 1]), "s"(inext) : "memory");
                }
                if (LD == 1 && q >= 17 && q <= 32) {
                    if (more)
                        asm volatile("s_waitcnt vmcnt(%2)\n ds_write_b128 %0, %1 offset:%3"
                                     :: "v"(land_a), "v"(ldv[q - 17]), "n"(32 - q), "n"(1024 * (q - 17)) : "memory");
                }
                if (q >= 33 && (q - 33) % 2 == 0 && (q - 33) / 2 < 16) {
                    const int t = (q - 33) / 2;
                    if (prev) {
                        if (!skip0) store(obase, t, v);
                        if (t < 15) v = unit_read(ru, t + 1);
                    }
                }
                ring_barrier();
            }
            constexpr int kStoresAfter = 16;
            if (LD == 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            else if (prev) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kStoresAfter) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        ring_barrier();  // F1: the last run's outputs are in the ring
        if (!(p.dbg & 64)) {
            uint8_t* obase = reinterpret_cast<uint8_t*>(uni(abase + (uintptr_t)kRun * (S - 1)));
            const uint8_t* ru = run_unit_base(S - 1);
            const bool skip0 = S == 1 && j == 0;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const uint4 v = unit_read(ru, t);
                if (!skip0) store(obase, t, v);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store done (tamper zeroing)
        ring_barrier();  // F2
        return;
    }

    // ==================================================================== compute waves
    const uint32_t msw = slab_sw(lane);
    const uint8_t* src = p.in + i0 + (uint64_t)rec * L;
    uint8_t* dst = p.out + o0 + (uint64_t)rec * L;
    const uint32_t dlt = (d0 + rec * L) & 63u;  // record start within its first 64-byte unit
    uint8_t* const myring = s_ring + kRingBytes * threadIdx.x;

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

    // ---- Poly1305: one-time key from block 0 (runs while stage 0 lands); the AAD first
    uint32_t h[5] = {0, 0, 0, 0, 0};
    PolyR32 PR{};
    uint32_t pad[4] = {0, 0, 0, 0};
    uint32_t aad_len = 0;
    if (kPoly) {
        uint32_t otk[16];
        chacha_block(R, 0u, otk);
        PR = polyr32_make(otk[0], otk[1], otk[2], otk[3]);
        pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        if (p.aad) {
            const uint64_t aoff = p.aad_off[rec];
            aad_len = (uint32_t)(p.aad_off[rec + 1] - aoff);
            const uint32_t na = (aad_len + 15) >> 4;
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ring_barrier();  // S0(st)
        const uint8_t* myrun = s_in + threadIdx.x * kRun;
        uint32_t w[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (q ^ msw));
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
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
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slab may be refilled
        if (__builtin_expect(p.dbg & 2, 0)) {  // probe (tools build): no keystream, barriers only
#pragma unroll
            for (int q = 0; q < kRingPos; ++q) ring_barrier();
        } else {
            chacha_half_lockstep2<true>(x);
#pragma unroll
            for (int dr = 1; dr < 10; ++dr) {
                chacha_half_lockstep2<false>(x);
                chacha_half_lockstep2<true>(x);
            }
        }
        if (MODE == MODE_OPEN) {
            poly_block64(h, PR, w);
            poly_block64(h, PR, w + 16);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            w[i] ^= x[i] + (i == 12 ? c0 : ff[i]);
            w[16 + i] ^= x[16 + i] + (i == 12 ? c0 + 1u : ff[i]);
        }
        if (MODE == MODE_SEAL) {
            poly_block64(h, PR, w);
            poly_block64(h, PR, w + 16);
        }
        // the record's own first and last units (shared with the neighbours): direct stores
        if (st == 0) put16(dst, w);
        if (st == S - 1) put16(dst + (uint64_t)kRun * S - 64u, w + 16);
        // run st -> ring bytes (dlt + 128 st) mod 192 (the memory waves have read the two units
        // this overwrites by now).  Phase 0 never wraps; phases 1, 2 wrap after nw words.
        const uint32_t ph = (2u * st) % 3u;  // slot of unit 2 st
        uint32_t* ra = reinterpret_cast<uint32_t*>(myring + dlt + 64u * ph);
        if (__builtin_expect(p.dbg & 16, 0)) {  // probe: no ring writes
        } else if (ph == 0) {
#pragma unroll
            for (int i = 0; i < 32; ++i) ra[i] = w[i];
        } else {
            uint32_t* rb = ra - kRingBytes / 4u;
            const uint32_t nwr = (kRingBytes - 64u * ph - dlt) >> 2;
#pragma unroll
            for (int i = 0; i < 32; ++i) ((uint32_t)i < nwr ? ra : rb)[i] = w[i];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ring_barrier();  // F1

    // ---- ragged end: T (1..127) bytes from record byte 128 S, per lane
    if (__builtin_expect(p.dbg & 8, 0)) {  // probe: no ragged end / tag
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ring_barrier();
        return;
    }
    uint32_t t[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) t[i] = 0u;
    const uint64_t tb = (uint64_t)kRun * S;
    load_block(src + tb, min(T, 64u), t, true);
    if (T > 64u) load_block(src + tb + 64u, T - 64u, t + 16, true);
    {
        uint32_t ka[16], kb[16];
        chacha_block2(R, ctr + 2u * S, ctr + 2u * S + 1u, ka, kb);
        const uint32_t nch = (T + 15u) >> 4;
        if (MODE == MODE_OPEN) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if ((uint32_t)u < nch) poly32_block(h, PR, t[4 * u], t[4 * u + 1], t[4 * u + 2], t[4 * u + 3], 1u);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) { t[i] ^= ka[i]; t[16 + i] ^= kb[i]; }
        if (MODE == MODE_SEAL) {
            keep_le32(t, T);
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if ((uint32_t)u < nch) poly32_block(h, PR, t[4 * u], t[4 * u + 1], t[4 * u + 2], t[4 * u + 3], 1u);
        }
    }
    store_block(dst + tb, min(T, 64u), t);
    if (T > 64u) store_block(dst + tb + 64u, T - 64u, t + 16);

    uint32_t diff = 0;
    if (kPoly) {
        poly32_block(h, PR, aad_len, 0u, L, 0u, 1u);  // LE64 |aad| || LE64 |ct|
        uint32_t l[5], tag[4];
        h32_to_limbs(h, l);
        pfinish(l, pad, tag);
        if (MODE == MODE_SEAL) {
            uint32_t* tp = reinterpret_cast<uint32_t*>(p.tag_out + 16ull * rec);
            tp[0] = tag[0]; tp[1] = tag[1]; tp[2] = tag[2]; tp[3] = tag[3];
        } else {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tag_in + 16ull * rec);
            diff = (tag[0] ^ tp[0]) | (tag[1] ^ tp[1]) | (tag[2] ^ tp[2]) | (tag[3] ^ tp[3]);
            p.ok[rec] = diff == 0 ? 1 : 0;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ring_barrier();  // F2: the memory waves' stores of this workgroup are complete
    if (MODE == MODE_OPEN && diff != 0) {
        // authentication failed: do not release plaintext (16-byte pieces, the last one ending
        // at the record end)
        const uint4 z = make_uint4(0, 0, 0, 0);
        for (uint32_t c = 0; c + 16u <= L; c += 16u) *reinterpret_cast<uint4*>(dst + c) = z;
        *reinterpret_cast<uint4*>(dst + L - 16u) = z;
    }
}

bool stream_ring_eligible(const RecParams& p) {
    const uint64_t L = p.uniform_len;
    return p.stream && p.ring && L >= 128 && (L & 127u) != 0 && (L & 3u) == 0 && p.order == nullptr &&
           L * (uint64_t)p.n <= 0xFFFFFE00ull && p.n >= kRingLanes;
}

hipError_t launch_stream_ring(int mode, const RecParams& p, uint32_t blocks, hipStream_t s) {
    const int v = (p.var & 1) | ((p.var & 2) ? 2 : 0);  // tools build only: 1 nt stores, 2 VGPR loads
    const dim3 g(blocks), b(kRingWG);
#define ENET_RING_CASE(M, V) \
    case M * 4 + V: hipLaunchKernelGGL((stream_ring_kernel<M, (V & 1), (V >> 1)>), g, b, 0, s, p); break;
    switch (mode * 4 + v) {
        ENET_RING_CASE(MODE_XOR, 0) ENET_RING_CASE(MODE_XOR, 1) ENET_RING_CASE(MODE_XOR, 2) ENET_RING_CASE(MODE_XOR, 3)
        ENET_RING_CASE(MODE_SEAL, 0) ENET_RING_CASE(MODE_SEAL, 1) ENET_RING_CASE(MODE_SEAL, 2) ENET_RING_CASE(MODE_SEAL, 3)
        ENET_RING_CASE(MODE_OPEN, 0) ENET_RING_CASE(MODE_OPEN, 1) ENET_RING_CASE(MODE_OPEN, 2) ENET_RING_CASE(MODE_OPEN, 3)
        default: return hipErrorInvalidValue;
    }
#undef ENET_RING_CASE
    return hipGetLastError();
}

}  // namespace enet
