// records_body.hpp -- the ChaCha20 / ChaCha20-Poly1305 record engine body (gfx950), shared by
// records.hip (the record kernels) and stream.hip (the streaming kernel, whose workgroups fall
// back to the per-lane path here when a batch declared uniform is not).
#pragma once

// One wave = 64 lanes; each record gets P lanes (P = 1..16, a power of two chosen by the host
// scheduler from the batch shape).  Lane j of a record processes a contiguous run of ChaCha20
// blocks -- one 64-byte block per lane per step, the 4x4 state in VGPRs, the next block's
// 64 bytes prefetched into registers while the current keystream is computed.
//
// Poly1305 (seal / open) runs in the same lanes over the same bytes: Horner in the clamped r
// with radix-2^32 limbs (20 v_mad_u64_u32 per 16-byte block), then one r^e scale per lane and
// a cross-lane sum of the P partial accumulators.  No LDS: every lane MACs its own bytes.
//
// Reference behaviour (ShardianLabs/EphemeralNet):
//   ChaCha20::apply           src/crypto/ChaCha20.cpp:98-121 (u32 counter wrap :110)
//   CryptoManager chunk mode  src/crypto/CryptoManager.cpp:8-13,38-58 (start counter LE32(id))
//   session frame body        src/network/SessionManager.cpp:362-374, 815-822
// RFC 8439 AEAD (no reference implementation): keystream counter 1.., one-time
// Poly1305 key from block 0, tag over aad || pad || ct || pad || LE64 |aad| || LE64 |ct|.
#include "enet_device.hpp"
#include "enet_internal.hpp"

namespace enet {

// Frame sub-modes of MODE_XOR
enum FrameKind : int { FR_NONE = 0, FR_SEAL = 1, FR_OPEN = 2 };

__device__ __forceinline__ void mask_tail(uint32_t w[16], uint32_t n) {
    // zero bytes >= n of a 64-byte block (n < 64)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t lo = 4u * i;
        uint32_t m;
        if (n >= lo + 4) m = 0xffffffffu;
        else if (n <= lo) m = 0u;
        else m = (1u << (8 * (n - lo))) - 1u;
        w[i] &= m;
    }
}

__device__ __forceinline__ void load_full(const uint8_t* __restrict__ p, uint32_t w[16]) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = q[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
}

__device__ __forceinline__ void store_full(uint8_t* __restrict__ p, const uint32_t w[16]) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// Four Poly1305 blocks (one 64-byte ciphertext block), all full.
__device__ __forceinline__ void poly_block64(uint32_t h[5], const PolyR32& R, const uint32_t ct[16]) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
        poly32_block(h, R, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
}

// Lane layout: record = P consecutive lanes; lane j owns the contiguous ChaCha20 blocks
// [j*B, min((j+1)*B, nb)), B = ceil(nb / P), and with them the contiguous Poly1305 stream
// blocks they cover (lane 0 also the AAD prefix, the lane with the last block also the length
// block).  Each lane runs Horner in the clamped r (radix 2^32); at the end lane j scales its
// accumulator by r^(N-1-s_last_j) and the P lanes add up with cross-lane shuffles.
// COOP (uniform batches only: every record has the same length, so record g starts at
// in_off[0] + g*L): whole-block stages of kStage blocks per lane are moved wave-cooperatively.
// Load instruction i of a stage serves owners 8i..8i+7 of the wave (64 lanes x 16 B = 8 owners x
// 128 contiguous bytes = whole 128-byte lines), lands in a wave-private LDS slab
// [owner][128 B] whose 16-byte chunks are XOR-swizzled by slab_sw(owner) (conflict-free
// ds_read_b128 and ds_write_b128), and each lane then reads its own two blocks.  Outputs take the reverse trip.
// Within one wave, DS instructions execute in issue order, so handing LDS data between lanes
// of the same wave needs only a compiler barrier -- a wavefront-scope fence would also drain the
// in-flight global loads/stores (s_waitcnt vmcnt(0)) and serialise every stage.
#define ENET_WAVE_LDS_SYNC()                  \
    do {                                      \
        asm volatile("" ::: "memory");        \
        __builtin_amdgcn_wave_barrier();      \
        asm volatile("" ::: "memory");        \
    } while (0)

// Pin 16 register words: they must be computed before this point and cannot be sunk past it.
#define ENET_PIN16(a)                                                                          \
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), \
                      "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), \
                      "+v"(a[12]), "+v"(a[13]), "+v"(a[14]), "+v"(a[15])::"memory")

// 16-byte chunk c of owner o's run sits at 128 o + 16 (c ^ slab_sw(o)) in a staging slab.  The
// own-run ds_read_b128 serves lanes in groups of 16 ({0-3,12-15,20-27}, ...; bank = dword address
// mod 64) and needs (slab_sw(o), o & 1) distinct inside each group; the own-run ds_write_b128
// serves 8 contiguous lanes (bank = dword address mod 32) and needs slab_sw(o) distinct across
// them.  ((o >> 1) & 7) alone met the first only: every own-run write was a 2-way conflict
// (PMC SQ_LDS_BANK_CONFLICT 2.1 M cycles per C2 launch, profiles/pmc_r01.json); flipping bit 2
// with o & 1 meets both (0 in profiles/pmc_r02.json).
__device__ __forceinline__ uint32_t slab_sw(uint32_t o) { return ((o >> 1) & 7u) ^ ((o & 1u) << 2); }

constexpr uint32_t kStage = 2;                 // blocks per lane per cooperative stage
constexpr uint32_t kRun = 64 * kStage;         // bytes per owner per stage
constexpr uint32_t kRing = 288;                // COOP 4: two-line ring (256 B) + 32 B pad per owner

// Streaming output store: the kernel never reads its outputs back, so stores that fill whole
// 128-byte lines are non-temporal (global_store ... nt) instead of being kept dirty in the per-XCD
// L2 until the end-of-kernel write-back (C2 seal kernel 150 -> 142 us, tools/nt_ab.sh).  Stores
// covering partial lines stay cached (nt there costs up to 35 %: the halves are not merged).
typedef uint32_t enet_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_stream(uint8_t* p, uint4 v, bool nt = true) {
    if (nt) {
        enet_u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<enet_u32x4*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}

template <int LOGP, int MODE, int FRAME, int COOP>
__device__ __forceinline__ void records_body(const RecParams& p) {
    constexpr uint32_t P = 1u << LOGP;
    constexpr bool kPoly = (MODE != MODE_XOR);
    // COOP 5 = COOP 1 in 512-thread workgroups with the lockstep keystream (both waves of a SIMD
    // belong to one workgroup and meet at s_barrier every 24 ChaCha instructions)
    // (COOP 7 = the per-lane path of COOP 0 in 512-thread workgroups, the streaming kernel's
    // fallback)
    constexpr uint32_t WGS = (COOP == 5 || COOP == 7) ? 512u : (uint32_t)kWG;
    __shared__ __attribute__((aligned(16))) uint8_t
        slab[COOP == 4 ? WGS * kRing : (COOP && COOP != 7) ? WGS * kRun : 16];

    const uint32_t gid = blockIdx.x * WGS + threadIdx.x;
    const uint32_t group = gid >> LOGP;
    const uint32_t j = gid & (P - 1);
    const bool in_batch = group < p.n;
    const uint32_t rec = in_batch ? (p.order ? p.order[group] : group + p.rec_base) : 0u;
    // a record the sequence-parallel path claimed (segments.hip) is not this kernel's -- except
    // that an open whose tag failed there is zeroed here (the launch boundary orders these zero
    // stores after every tile's plaintext stores; no plaintext of a failed record is released)
    const bool claimed = COOP == 0 && in_batch && p.skip && p.skip[rec];
    if (MODE == MODE_OPEN && claimed && p.ok[rec] == 0) {
        const uint64_t a = p.out_off[rec], L = p.in_off[rec + 1] - p.in_off[rec];
        const uint32_t j0 = (blockIdx.x * WGS + threadIdx.x) & (P - 1);
        for (uint64_t b = 16ull * j0; b < L; b += 16ull * P) {
            const uint32_t nbytes = (uint32_t)min<uint64_t>(16, L - b);
            if (nbytes == 16) *reinterpret_cast<uint4*>(p.out + a + b) = make_uint4(0u, 0u, 0u, 0u);
            else for (uint32_t t = 0; t < nbytes; ++t) p.out[a + b + t] = 0;
        }
    }
    const bool live = in_batch && !claimed;

    // ---- record geometry
    uint64_t ioff = 0, ooff = 0, Lin = 0, Lout = 0;
    if (live) {
        ioff = p.in_off[rec];
        Lin = p.in_off[rec + 1] - ioff;
        ooff = p.out_off[rec];
        Lout = p.out_off[rec + 1] - ooff;
    }
    // The staged variants address record g at in_off[0] + g*Lu (uniform batch, declared by the
    // caller's hints).  Check the offsets: a workgroup holding any record that does not sit
    // there takes the per-lane path, so a wrong hint costs speed, never bytes.
    bool lay_ok = true;
    if (COOP != 0 && COOP != 7) {
        const uint64_t Lu = p.uniform_len;
        const bool mine = !live || (ioff == p.in_off[0] + (uint64_t)rec * Lu && Lin == Lu &&
                                    ooff == p.out_off[0] + (uint64_t)rec * Lu && Lout == Lu);
        lay_ok = __syncthreads_and(mine ? 1 : 0) != 0;
    }
    // wire frames: step over the nonce || BE32 length header
    uint64_t frame0 = 0;                       // frame start (seal: header goes here)
    bool hdr_ok = true;                        // open: the frame holds a whole header
    if (FRAME != FR_NONE && p.hdr) {
        if (FRAME == FR_SEAL) {
            frame0 = ooff;
            const uint64_t hb = min<uint64_t>(p.hdr, Lout);
            ooff += hb;
            Lout -= hb;
        } else {
            frame0 = ioff;
            hdr_ok = Lin >= p.hdr;
            const uint64_t hb = min<uint64_t>(p.hdr, Lin);
            ioff += hb;
            Lin -= hb;
        }
    }
    uint64_t L = Lin;                          // bytes run through the keystream
    if (FRAME == FR_SEAL) L = Lout;            // in || mac (the HMAC pass left the MAC in
                                               // clear at the tail of the out body)
    uint64_t simple = L;                       // prefix where whole blocks take the fast path
    if (FRAME == FR_SEAL) simple = Lin;
    if (FRAME == FR_OPEN) simple = Lout;
    const uint32_t nb = (uint32_t)((L + 63) >> 6);
    const uint32_t B = (nb + P - 1) >> LOGP;
    const uint32_t cbeg = min(j * B, nb);
    const uint32_t cend = min(cbeg + B, nb);
    const uint32_t cfast = max(cbeg, min(cend, (uint32_t)(simple >> 6)));
    const uint8_t* src = p.in + ioff;
    uint8_t* dst = p.out + ooff;

    // ---- per-record ChaCha20 constants
    uint32_t kw[8], nw[3];
    if (live) {
        const uint32_t* kp = reinterpret_cast<const uint32_t*>(p.keys + (size_t)p.key_stride * rec);
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = kp[i];
        if (FRAME == FR_OPEN && p.hdr) {  // nonce = first 12 bytes of the wire frame
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = hdr_ok ? ld32(p.in + frame0 + 4 * i) : 0u;
        } else {
            const uint32_t* np = reinterpret_cast<const uint32_t*>(p.nonces + 12ull * rec);
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = np[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = 0;
    }
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    uint32_t ctr0 = 1;  // RFC 8439 data counter
    if (MODE == MODE_XOR)  // reference ChaCha20::apply counter (0 when not given)
        ctr0 = (p.counters && live)
                   ? p.counters[(size_t)rec * (p.counter_stride ? p.counter_stride : 1u)]
                   : 0u;

    // ---- Poly1305: one-time key from block 0; lane 0 absorbs the AAD prefix
    uint32_t h[5] = {0, 0, 0, 0, 0};
    PolyR32 PR{};
    uint32_t pad[4] = {0, 0, 0, 0};
    uint32_t na = 0, aad_len = 0;
    const uint32_t nct = (uint32_t)((L + 15) >> 4);
    auto poly_setup = [&]() {
        if (!kPoly) return;
        uint32_t otk[16];
        chacha_block(R, 0u, otk);
        PR = polyr32_make(otk[0], otk[1], otk[2], otk[3]);
        pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        uint64_t aoff = 0;
        if (p.aad && live) {
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
    };
    if (COOP == 0 || COOP == 7) poly_setup();

    // ---- cooperative stages (uniform batches)
    uint32_t cco = cbeg;     // first block left for the per-lane fast path
    uint32_t ctail = cfast;  // first block left for the per-lane tail path
    if (COOP == 1 || COOP == 5) {
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t wbase = threadIdx.x & ~63u;
        const uint64_t Lu = p.uniform_len;
        const uint32_t nfull = (uint32_t)(Lu >> 6);
        // every lane of every record has at least fmin whole blocks (the last lane has fewest)
        const uint32_t jl = P - 1;
        const uint32_t fmin = (nfull > jl * B) ? min(B, nfull - jl * B) : 0u;
        const uint32_t Ts = lay_ok ? fmin / kStage : 0u;
        const uint32_t kk = lane & 7u;
        const uint32_t wgid0 = blockIdx.x * WGS + wbase;  // gid of lane 0 of this wave
        uint64_t off[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t o = 8u * i + (lane >> 3);
            const uint32_t og = (wgid0 + o) >> LOGP;
            const uint32_t oj = (wgid0 + o) & (P - 1);
            const uint32_t sw = slab_sw(o);
            // the host launches COOP only over whole waves of live records
            off[i] = (uint64_t)og * Lu + 64ull * oj * B + 16u * (kk ^ sw);
        }
        const uint8_t* ibase = p.in + (p.n ? p.in_off[0] : 0);
        uint8_t* obase = p.out + (p.n ? p.out_off[0] : 0);
        // every owner run covers whole aligned 64-byte halves of lines (uniform test)
        const bool lines_whole = p.nt_stores && (Lu & 63u) == 0 && ((64ull * B) & 63u) == 0 &&
                                 (reinterpret_cast<uintptr_t>(obase) & 63u) == 0;
        uint8_t* wslab = slab + wbase * kRun;
        uint8_t* myrun = slab + threadIdx.x * kRun;
        const uint32_t msw = slab_sw(lane);
        // prefetch registers as plain words (a uint4 array is copied with memcpy and stays
        // in scratch)
        uint32_t pf[32];
        auto land = [&]() {  // prefetched stage -> slab, lane-linear (whole-line layout)
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                    make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
        };
        auto fetch = [&](uint32_t stage) {
            const uint64_t adv = (uint64_t)kRun * stage;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(ibase + off[i] + adv);
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            }
        };
        if (Ts > 0) fetch(0);
        poly_setup();  // the one-time-key block runs while the first stage is in flight
        if (Ts > 0) land();
        // Loop rotated so every wait on the prefetch sits after this stage's stores in the same
        // iteration: vmcnt then waits for the (older) loads only, never for the stores.
        for (uint32_t st = 0; st < Ts; ++st) {
            ENET_WAVE_LDS_SYNC();
            // (b) each lane reads its own two blocks
            uint32_t w2[32];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                w2[4 * k] = v.x; w2[4 * k + 1] = v.y; w2[4 * k + 2] = v.z; w2[4 * k + 3] = v.w;
            }
            // (c) prefetch the next stage now, so its latency hides under this stage's ALU work
            //     (the last iteration re-reads its own stage, an L2 hit, so the prefetch
            //     registers are written unconditionally and stay in VGPRs)
            fetch(min(st + 1, Ts - 1));
            // keep the loads issued here: the keystream work below is made to depend on this
            // statement, so the scheduler cannot hoist it above the loads
            asm volatile("" : "+v"(R.k[0]) :: "memory");
            // (d) two keystream blocks (interleaved) + Poly1305
            {
                const uint32_t c0 = ctr0 + cbeg + kStage * st;
                if (MODE == MODE_OPEN) {
                    poly_block64(h, PR, w2);
                    poly_block64(h, PR, w2 + 16);
                }
                uint32_t ka[16], kb[16];
                if (COOP == 5) chacha_block2_lockstep(R, c0, c0 + 1, ka, kb);
                else chacha_block2(R, c0, c0 + 1, ka, kb);
#pragma unroll
                for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
                if (MODE == MODE_SEAL) {
                    poly_block64(h, PR, w2);
                    poly_block64(h, PR, w2 + 16);
                }
            }
            // (e) outputs back into the own run, (f) read lane-linear and store whole lines
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                    make_uint4(w2[4 * k], w2[4 * k + 1], w2[4 * k + 2], w2[4 * k + 3]);
            ENET_WAVE_LDS_SYNC();
            const uint64_t adv = (uint64_t)kRun * st;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                store_stream(obase + off[i] + adv, v, lines_whole);
            }
            ENET_WAVE_LDS_SYNC();
            // (a) land the next stage in the slab
            land();
        }
        cco = min(cfast, cbeg + kStage * Ts);
        // Ragged last stage (one lane per record): bytes [kRun*Ts, L) of every record -- the odd
        // whole block and the partial block -- through the same whole-line LDS transposition
        // instead of the per-lane paths (64 scattered records per load/store instruction).
        // rem = L - kRun*Ts is uniform; chunks [0, rem/16) move whole, and a partial chunk is
        // replaced by the 16-byte window ending at the record end (inside the record since
        // rem >= 16): loaded there and stored there, so nothing outside the record is read or
        // written (the window's overlap with the previous chunk is rewritten with equal bytes).
        const uint32_t rem = (uint32_t)(Lu - (uint64_t)kRun * Ts);
        if (P == 1 && lay_ok && Lu <= 0xFFFFFFFFull && rem >= 16u) {
            const uint32_t rem16 = rem >> 4, remb = rem & 15u;
            const uint32_t nch = rem16 + (remb ? 1u : 0u);
            const uint64_t adv = (uint64_t)kRun * Ts;
            // (a) loads: lane (owner 8i + lane/8, LDS slot kk) fetches the record chunk kk ^ sw
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t o = 8u * i + (lane >> 3);
                const uint32_t gc = kk ^ slab_sw(o);
                const uint64_t run = (uint64_t)((wgid0 + o) >> LOGP) * Lu + adv;
                if (gc < nch) {
                    const uint32_t at = gc < rem16 ? 16u * gc : rem - 16u;
                    const uint4 v = *reinterpret_cast<const uint4*>(ibase + run + at);
                    *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) = v;
                }
            }
            ENET_WAVE_LDS_SYNC();
            // (b) own run -> 32 words, zero past rem (the window slot is shifted into place)
            uint32_t x[32];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                uint32_t v4[4] = {0u, 0u, 0u, 0u};
                if ((uint32_t)k < nch) {
                    const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                    v4[0] = v.x; v4[1] = v.y; v4[2] = v.z; v4[3] = v.w;
                    if ((uint32_t)k == rem16) {  // window bytes [rem-16, rem) -> [16k, rem)
                        uint32_t sh[4];
                        extract_bytes<4, 4>(v4, 16u - remb, sh);
#pragma unroll
                        for (int t = 0; t < 4; ++t) v4[t] = sh[t];
                    }
                }
#pragma unroll
                for (int t = 0; t < 4; ++t) x[4 * k + t] = v4[t];
            }
            // (c) keystream, Poly1305 over the ciphertext chunks [0, nch)
            const uint32_t c0 = ctr0 + cbeg + kStage * Ts;
            if (MODE == MODE_OPEN) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if ((uint32_t)u < nch)
                        poly32_block(h, PR, x[4 * u], x[4 * u + 1], x[4 * u + 2], x[4 * u + 3], 1u);
            }
            {
                uint32_t ks[16];
                chacha_block(R, c0, ks);
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] ^= ks[i];
            }
            if (rem > 64u) {
                uint32_t ks[16];
                chacha_block(R, c0 + 1, ks);
#pragma unroll
                for (int i = 0; i < 16; ++i) x[16 + i] ^= ks[i];
            }
            if (MODE == MODE_SEAL) {
                // ciphertext bytes past rem are keystream: RFC 8439 pads the last block with zeros
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t lo = 16u * k;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const uint32_t b0 = lo + 4u * t;
                        const uint32_t m = rem >= b0 + 4u ? 0xffffffffu
                                         : rem <= b0      ? 0u
                                                          : (1u << (8u * (rem - b0))) - 1u;
                        if ((uint32_t)k == rem16) x[4 * k + t] &= m;
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if ((uint32_t)u < nch)
                        poly32_block(h, PR, x[4 * u], x[4 * u + 1], x[4 * u + 2], x[4 * u + 3], 1u);
            }
            // (d) outputs into the own run: whole chunks, and the window ending at rem
            uint32_t win[4] = {0u, 0u, 0u, 0u};
            if (remb) extract_bytes<32, 4>(x, rem - 16u, win);
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if ((uint32_t)k < rem16)
                    *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                        make_uint4(x[4 * k], x[4 * k + 1], x[4 * k + 2], x[4 * k + 3]);
                else if ((uint32_t)k == rem16 && remb)
                    *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                        make_uint4(win[0], win[1], win[2], win[3]);
            }
            ENET_WAVE_LDS_SYNC();
            // (e) lane-linear stores of whole chunks / the window
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t o = 8u * i + (lane >> 3);
                const uint32_t gc = kk ^ slab_sw(o);
                const uint64_t run = (uint64_t)((wgid0 + o) >> LOGP) * Lu + adv;
                if (gc < nch) {
                    const uint32_t at = gc < rem16 ? 16u * gc : rem - 16u;
                    const uint4 v = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                    *reinterpret_cast<uint4*>(obase + run + at) = v;
                }
            }
            cco = cend;
            ctail = cend;
        }
    }
    if (COOP == 4) {
        // Line-aligned staging for uniform batches whose records are not 128-byte aligned
        // (C3: 1 500-byte records), one lane per record.  Run s of a record = record bytes
        // [128s, 128s+128) straddles two arena lines (offset d = record start mod 128), so
        // staging whole runs touches twice the lines and splits 16-byte accesses.  Instead the
        // wave moves whole ALIGNED 128-byte lines: line t of owner o is arena line
        // floor(start_o / 128) + t, eight lanes per line, eight owners per instruction; each
        // owner keeps a two-line ring in LDS (slot t % 2) and reads / writes its run at ring
        // offset (d + 128s) mod 256 with dword accesses.  Line t is complete once run t is
        // written back (its first d bytes came from run t-1), and is stored whole -- except a
        // record's first and last lines, shared with the neighbouring records: only this
        // record's bytes of them are stored (dword-exact; the host launches this variant only
        // when record starts are 4-byte aligned and in / out starts agree mod 128).  Loads of
        // whole lines read at most 127 bytes outside the record, never outside its pages.
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t wbase = threadIdx.x & ~63u;
        const uint32_t Lu = (uint32_t)p.uniform_len;
        // load / store roles: instruction i serves owner 8i + rq with its 16-byte chunk rc, each
        // quad of lanes one aligned 64-byte half line (whole lines per instruction, as before).
        // The quad -> (owner, half) map below makes the ring's ds_read_b128 lane groups
        // ({0-3,12-15,20-27}, ...; bank = dword mod 64) and the ds_write_b128 8-lane groups
        // (bank = dword mod 32) conflict-free with the 72-dword ring stride (kRing = 288 B): the
        // identity map (owner = lane / 8, chunk = lane % 8) left every ds_read_b128 2- to 3-way
        // conflicted (PMC 12.3 M conflict cycles per C3 launch, profiles/pmc_c3_r02.json) and no
        // stride <= 88 dwords is conflict-free with it.  The run's own dword accesses
        // (ring_at: ds_read/write_b32, bank = dword mod 32) stay conflict-free when
        // 72 + L/4 is odd (C3: L = 1500).
        const uint32_t rk = lane >> 2;
        const uint32_t rq = 2u * ((rk >> 1) & 3u) + (rk >> 3);
        const uint32_t rc = 4u * ((rk ^ (rk >> 1) ^ (rk >> 2)) & 1u) + (lane & 3u);
        const uint32_t wgid0 = blockIdx.x * WGS + wbase;
        const uint8_t* ibase = p.in + (p.n ? p.in_off[0] : 0);
        uint8_t* obase = p.out + (p.n ? p.out_off[0] : 0);
        const uint32_t ib = (uint32_t)reinterpret_cast<uintptr_t>(ibase);
        const uint32_t ob = (uint32_t)reinterpret_cast<uintptr_t>(obase);
        const uint32_t S = (Lu + kRun - 1) / kRun;  // stages (the last one may be partial)
        // in and out must share the line phase and allow dword-exact edge stores (uniform test;
        // otherwise every record takes the per-lane paths below)
        if (lay_ok && ((ib - ob) & 127u) == 0 && (ib & 3u) == 0) {
        uint8_t* wslab = slab + (wbase >> 6) * (64u * kRing);
        uint8_t* myring = wslab + lane * kRing;
        const uint32_t dme = (ib + (wgid0 + lane) * Lu) & 127u;
        // 32-bit line offsets from the 128-byte-aligned bases (the host launches this variant only
        // for arenas < 4 GiB)
        // the line bases are workgroup-uniform: pin them in SGPRs (the compiler kept them in
        // VGPRs and re-read them with two v_readfirstlane + s_nop 4 before every line load / store)
        const uint8_t* ial =
            reinterpret_cast<const uint8_t*>(uniform_u64(reinterpret_cast<uintptr_t>(ibase - (ib & 127u))));
        uint8_t* oal = reinterpret_cast<uint8_t*>(uniform_u64(reinterpret_cast<uintptr_t>(obase - (ib & 127u))));
        uint32_t roff[8];  // line 0 of owner o
        uint32_t rgeo[8];  // d | lines << 8 | end-bytes-in-last-line << 16
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t o = 8u * i + rq;
            const uint32_t g = wgid0 + o;
            const uint32_t d = (ib + g * Lu) & 127u;
            roff[i] = g * Lu + (ib & 127u) - d;
            const uint32_t nl = (d + Lu + 127u) >> 7;
            const uint32_t e = ((d + Lu - 1u) & 127u) + 1u;
            rgeo[i] = d | (nl << 8) | (e << 16);
        }
        uint32_t pf[32];
        auto fetch = [&](uint32_t t) {  // line t of every role owner -> pf (only lines it has)
            if (t < S) {  // every record has lines 0 .. S-1 (S = ceil(L / 128) <= its line count)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ial + (roff[i] + 128u * t + 16u * rc));
                    pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
                }
                return;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (t < ((rgeo[i] >> 8) & 0xffu)) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ial + (roff[i] + 128u * t + 16u * rc));
                    pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
                }
            }
        };
        auto land = [&](uint32_t t) {  // pf -> ring slot t % 2 of every role owner
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(wslab + (8u * i + rq) * kRing + 128u * (t & 1u) + 16u * rc) =
                    make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
        };
        auto store_inner = [&](uint32_t t) {  // line t, 1 <= t <= S-2: complete in every record
#pragma unroll
            for (int i = 0; i < 8; ++i)
                store_stream(oal + (roff[i] + 128u * t + 16u * rc),
                             *reinterpret_cast<const uint4*>(wslab + (8u * i + rq) * kRing +
                                                             128u * (t & 1u) + 16u * rc));
        };
        auto store_line = [&](uint32_t t) {  // ring slot t % 2 -> line t, this record's bytes only
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t d = rgeo[i] & 0xffu, nl = (rgeo[i] >> 8) & 0xffu, e = rgeo[i] >> 16;
                if (t >= nl) continue;
                const uint32_t lo = t == 0 ? d : 0u, hi = t + 1 == nl ? e : 128u;
                const uint32_t c0 = 16u * rc;
                if (c0 + 16u <= lo || c0 >= hi) continue;
                const uint4 v = *reinterpret_cast<const uint4*>(
                    wslab + (8u * i + rq) * kRing + 128u * (t & 1u) + c0);
                uint8_t* q = oal + (roff[i] + 128u * t + c0);
                if (c0 >= lo && c0 + 16u <= hi) {
                    store_stream(q, v);
                } else {  // a record-boundary chunk: its dwords in [lo, hi) only
                    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        if (c0 + 4u * m >= lo && c0 + 4u * m < hi)
                            *reinterpret_cast<uint32_t*>(q + 4 * m) = w4[m];
                }
            }
        };
        // dword m of the run at ring offset o (wraps at 256)
        auto ring_at = [&](uint32_t o, uint32_t m) -> uint32_t* {
            return reinterpret_cast<uint32_t*>(myring + ((o + 4u * m) & 255u));
        };
        fetch(0);
        poly_setup();  // the one-time-key block runs while line 0 is in flight
        land(0);
        fetch(1);
        for (uint32_t st = 0; st < S; ++st) {
            ENET_WAVE_LDS_SYNC();
            land(st + 1);  // lines the owner does not have are never read back
            ENET_WAVE_LDS_SYNC();
            const uint32_t rl = min(kRun, Lu - kRun * st);  // uniform
            uint32_t x[32];
            uint32_t ro = dme + 128u * (st & 1u);
            // even stages: the run starts in slot 0 (ro = d < 128) and never wraps, so its dwords
            // are one base plus immediate offsets; odd stages wrap into slot 0 (ring_at's & 255,
            // two VALU per dword)
            if (rl == kRun && (st & 1u) == 0u) {
                // opaque to the compiler, which otherwise proves the two paths equal and keeps
                // only the masked one
                uint32_t eo = ro;
                asm volatile("" : "+v"(eo));
#pragma unroll
                for (int m = 0; m < 32; ++m) x[m] = *reinterpret_cast<const uint32_t*>(myring + eo + 4u * m);
            } else if (rl == kRun) {
#pragma unroll
                for (int m = 0; m < 32; ++m) x[m] = *ring_at(ro, m);
            } else {
#pragma unroll
                for (int m = 0; m < 32; ++m) x[m] = (4u * m < rl) ? *ring_at(ro, m) : 0u;
            }
            fetch(st + 2);
            asm volatile("" : "+v"(R.k[0]) :: "memory");
            const uint32_t c0 = ctr0 + kStage * st;
            const uint32_t nch = (rl + 15u) >> 4;
            if (rl == kRun) {
                if (MODE == MODE_OPEN) { poly_block64(h, PR, x); poly_block64(h, PR, x + 16); }
                uint32_t ka[16], kb[16];
                chacha_block2(R, c0, c0 + 1, ka, kb);
#pragma unroll
                for (int i = 0; i < 16; ++i) { x[i] ^= ka[i]; x[16 + i] ^= kb[i]; }
                if (MODE == MODE_SEAL) { poly_block64(h, PR, x); poly_block64(h, PR, x + 16); }
            } else {
                if (MODE == MODE_OPEN) {
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if ((uint32_t)u < nch)
                            poly32_block(h, PR, x[4 * u], x[4 * u + 1], x[4 * u + 2], x[4 * u + 3], 1u);
                }
                {
                    uint32_t ks[16];
                    chacha_block(R, c0, ks);
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] ^= ks[i];
                }
                if (rl > 64u) {
                    uint32_t ks[16];
                    chacha_block(R, c0 + 1, ks);
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[16 + i] ^= ks[i];
                }
                if (MODE == MODE_SEAL) {
#pragma unroll
                    for (int m = 0; m < 32; ++m) x[m] = (4u * m < rl) ? x[m] : 0u;  // RFC 8439 zero pad
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if ((uint32_t)u < nch)
                            poly32_block(h, PR, x[4 * u], x[4 * u + 1], x[4 * u + 2], x[4 * u + 3], 1u);
                }
            }
            // recompute the ring addresses here instead of holding 32 of them across the rounds
            asm volatile("" : "+v"(ro));
            if (rl == kRun && (st & 1u) == 0u) {
                uint32_t eo = ro;
                asm volatile("" : "+v"(eo));
#pragma unroll
                for (int m = 0; m < 32; ++m) *reinterpret_cast<uint32_t*>(myring + eo + 4u * m) = x[m];
            } else if (rl == kRun) {
#pragma unroll
                for (int m = 0; m < 32; ++m) *ring_at(ro, m) = x[m];
            } else {
#pragma unroll
                for (int m = 0; m < 32; ++m)
                    if (4u * m < rl) *ring_at(ro, m) = x[m];
            }
            ENET_WAVE_LDS_SYNC();
            if (st >= 1 && st + 2 <= S) store_inner(st);
            else store_line(st);
        }
        ENET_WAVE_LDS_SYNC();
        store_line(S);  // the last line when the record ends in line S (d + L > 128 S)
        cco = cend;
        ctail = cend;
        } else {
            // per-lane path for this workgroup: it still needs the one-time key (round 1 skipped
            // it here, so a uniform 1500-byte batch whose in / out arenas differed mod 128 got
            // all-zero tags; tests/test_gpu_parity.py::test_lying_hints_give_correct_bytes)
            poly_setup();
        }
    }
    // ---- fast path: whole blocks, next block prefetched while this one is computed
    uint32_t w[16];
    if (cco < cfast) load_full(src + 64ull * cco, w);
    for (uint32_t c = cco; c < cfast; ++c) {
        uint32_t wn[16];
        if (c + 1 < cfast) load_full(src + 64ull * (c + 1), wn);
        if (MODE == MODE_OPEN) poly_block64(h, PR, w);
        uint32_t ks[16];
        chacha_block(R, ctr0 + c, ks);  // uint32 wrap, ChaCha20.cpp:110
#pragma unroll
        for (int i = 0; i < 16; ++i) ks[i] ^= w[i];
        store_full(dst + 64ull * c, ks);
        if (MODE == MODE_SEAL) poly_block64(h, PR, ks);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = wn[i];
    }

    // ---- tail: the partial block and (frame open) the blocks that touch the MAC
    uint32_t mac[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // frame open: MAC bytes this lane decrypted
    for (uint32_t c = ctail; c < cend; ++c) {
        const uint64_t pos = 64ull * c;
        const uint32_t nbytes = (uint32_t)min<uint64_t>(64, L - pos);
        if (FRAME == FR_SEAL && pos + 64 > Lin) {
            // virtual input m[pos, Lin) || MAC, the MAC (clear, at dst + Lin) shifted in place
            const uint32_t nm = pos < Lin ? (uint32_t)(Lin - pos) : 0u;
            if (nm) {
                load_block(src + pos, nm, w, pos + nm >= 16);
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = 0u;
            }
            uint32_t m8[8];
            {
                const uint4 a = *reinterpret_cast<const uint4*>(dst + Lin);
                const uint4 b = *reinterpret_cast<const uint4*>(dst + Lin + 16);
                m8[0] = a.x; m8[1] = a.y; m8[2] = a.z; m8[3] = a.w;
                m8[4] = b.x; m8[5] = b.y; m8[6] = b.z; m8[7] = b.w;
            }
            uint32_t ins[16];
            if (pos <= Lin) {  // MAC bytes land at block offset Lin - pos
                uint32_t z[24];
#pragma unroll
                for (int i = 0; i < 16; ++i) z[i] = 0u;
#pragma unroll
                for (int i = 0; i < 8; ++i) z[16 + i] = m8[i];
                extract_bytes<24, 16>(z, 64u - (uint32_t)(Lin - pos), ins);
            } else {           // the MAC's bytes [pos - Lin, 32) open this block
                extract_bytes<8, 16>(m8, (uint32_t)(pos - Lin), ins);
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] |= ins[i];
        } else {
            load_block(src + pos, nbytes, w, pos + nbytes >= 16);
        }
        uint32_t o[16];
        chacha_block(R, ctr0 + c, o);
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] ^= w[i];
        if (FRAME == FR_OPEN) {
            // message bytes [pos, Lout) to out; MAC bytes [Lout, Lout + 32) into mac[]
            mask_tail(o, nbytes);
            if (pos < Lout) store_block(dst + pos, (uint32_t)min<uint64_t>(64, Lout - pos), o);
            if (pos + 64 > Lout && pos < Lout + 32) {
                uint32_t part[8];
                if (pos <= Lout) {
                    extract_bytes<16, 8>(o, (uint32_t)(Lout - pos), part);
                } else {  // MAC bytes [d, 32) from this block's bytes [0, 32 - d)
                    uint32_t z[16];
#pragma unroll
                    for (int i = 0; i < 8; ++i) { z[i] = 0u; z[8 + i] = o[i]; }
                    extract_bytes<16, 8>(z, 32u - (uint32_t)(pos - Lout), part);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) mac[i] |= part[i];
            }
        } else {
            store_block(dst + pos, nbytes, o);
        }
        if (kPoly) {
            uint32_t* ct = (MODE == MODE_SEAL) ? o : w;
            if (MODE == MODE_SEAL && nbytes < 64) mask_tail(ct, nbytes);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (4 * c + u < nct)
                    poly32_block(h, PR, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
        }
    }
    if (FRAME == FR_OPEN) {
        // the MAC may straddle two lanes' segments: OR over the record's lanes, lane 0 writes
#pragma unroll
        for (uint32_t off = P >> 1; off >= 1; off >>= 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) mac[i] |= __shfl_xor(mac[i], (int)off);
        }
        if (live && j == 0) {
            uint32_t* mp = reinterpret_cast<uint32_t*>(p.tag_out + 32ull * rec);
#pragma unroll
            for (int i = 0; i < 8; ++i) mp[i] = mac[i];
        }
    }

    if (FRAME == FR_SEAL && p.hdr && live && j == 0 && Lout <= 0xFFFFFFFFull) {
        // wire header: nonce(12) || BE32(|body|) (SessionManager.cpp:376-385)
        uint8_t* hp = p.out + frame0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int b = 0; b < 4; ++b) hp[4 * i + b] = (uint8_t)(nw[i] >> (8 * b));
        }
        hp[12] = (uint8_t)(Lout >> 24);
        hp[13] = (uint8_t)(Lout >> 16);
        hp[14] = (uint8_t)(Lout >> 8);
        hp[15] = (uint8_t)Lout;
    }

    if (kPoly) {
        // length block LE64(|aad|) || LE64(|ct|), owned by the lane holding the last block
        const uint32_t jlast = nb ? (nb - 1) / B : 0u;
        const uint32_t N = na + nct + 1;
        uint32_t e = 0;  // contribution scale: r^(N-1-s_last)
        if (j == jlast) {
            poly32_block(h, PR, aad_len, 0u, (uint32_t)L, (uint32_t)(L >> 32), 1u);
        } else if (cend > cbeg) {
            e = N - 1 - (na + 4 * cend - 1);
        }
        uint32_t l[5];
        h32_to_limbs(h, l);
        if (P > 1) {
            if (e > 0) {
                uint32_t r26[5], x[5];
                plimbs(r26, PR.r0, PR.r1, PR.r2, PR.r3);
                ppow(r26, e, x);
                pmul(l, pmul_make(x));
            }
#pragma unroll
            for (uint32_t off = P >> 1; off >= 1; off >>= 1) {
#pragma unroll
                for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], (int)off);
            }
        }
        uint32_t tag[4];
        pfinish(l, pad, tag);
        if (MODE == MODE_SEAL) {
            if (live && j == 0) {
                uint32_t* tp = reinterpret_cast<uint32_t*>(p.tag_out + 16ull * rec);
                tp[0] = tag[0]; tp[1] = tag[1]; tp[2] = tag[2]; tp[3] = tag[3];
            }
        } else {
            uint32_t diff = 0;
            if (live) {
                const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tag_in + 16ull * rec);
                diff = (tag[0] ^ tp[0]) | (tag[1] ^ tp[1]) | (tag[2] ^ tp[2]) | (tag[3] ^ tp[3]);
            }
            if (live && j == 0) p.ok[rec] = diff == 0 ? 1 : 0;
            if (live && diff != 0) {
                // authentication failed: do not release plaintext
                const uint32_t zero[16] = {0};
                for (uint32_t c = cbeg; c < cend; ++c) {
                    const uint64_t pos = 64ull * c;
                    store_block(dst + pos, (uint32_t)min<uint64_t>(64, L - pos), zero);
                }
            }
        }
    }
}

}  // namespace enet
