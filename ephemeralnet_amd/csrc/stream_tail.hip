// stream_tail.hip -- the streaming ChaCha20 / ChaCha20-Poly1305 kernel for uniform one-lane records
// whose length is not a multiple of 128 bytes (C3: 1 048 576 x 1 500-byte relay frames) (gfx950).
//
// Same workgroup as stream.hip: 8 compute waves (512 records, one lane each, two per SIMD in the
// lockstep keystream) and 4 memory waves that move every byte between HBM and LDS on a fixed
// schedule between the keystream barriers.  What changes is the record geometry: record g starts
// at byte g L, so its stage runs [128 st, 128 st + 128) are not 16-byte aligned.  Unaligned
// 16-byte DMAs and stores split in the texture units (a first version that used them directly
// ran at 0.6 x line staging, TA busy 61 %), so both sides move 16-BYTE-ALIGNED WINDOWS instead:
//   window t of record g = arena bytes [A_g + 128 t, A_g + 128 t + 128), A_g = (start of g) & ~15,
//   i.e. record bytes [128 t - d_g, 128 t + 128 - d_g), d_g = start mod 16 in {0, 4, 8, 12}.
//   * in: the memory waves land window st and the first chunk of window st + 1 (9 aligned chunks,
//     144 bytes) in the record's LDS slot; the compute lane reads its run at slot offset d_in with
//     dword reads (ds_read2_b32 -- a 4-byte-aligned ds_read_b128 would replay at 64 cycles).
//   * out: after the keystream the lane writes the previous run's last 3 words and its own run
//     at window offset d_out - 12 .. d_out + 127 of its output slot, so the slot's first 128
//     bytes are exactly window st: record bytes before the run from the previous stage, the rest
//     from this one.  The memory waves store that window during the next stage with aligned
//     16-byte stores.  Edges: window 0's first chunk holds the previous record's last d bytes
//     (the memory waves skip that chunk, the lane stores its 16 - d bytes itself, dword-exact);
//     the last window is stored dword-exact up to L, and bytes past it (d_out > 128 S - L) come
//     from the lane's carry.
//   * slots: lane o's record sits in slot ((o & 3) << 3 | (o >> 2) & 7 | (o & 32)) of its wave's
//     9 KiB part (144-byte slots), so a ds_read_b32 / ds_write_b32 half-wave (bank = dword mod 32)
//     sees 8 slot phases x 4 record phases: conflict-free whenever L = 4 (mod 8) (C3: 1 500).
//     The memory waves' ds_read_b128 of a store covers slots (i & 7) + 8 j with the lane -> (j,
//     chunk) map tail_store_j / tail_store_chunk, one 16-byte bank slot per lane of every 16-lane
//     group.
// The last stage is partial (rem = L - 128 (S-1) bytes): its DMA over-reads up to 128 S + 16 - L
// bytes into the NEXT record (the host keeps at least one record after the launch; each
// workgroup checks that record is long enough), its keystream is computed whole, Poly1305 takes
// only the ceil(rem / 16) remaining blocks (zero-padded, RFC 8439 2.8).
//
// Reference behaviour: ChaCha20::apply (src/crypto/ChaCha20.cpp:98-121, u32 counter wrap :110)
// for MODE_XOR; RFC 8439 AEAD (no reference implementation) for seal / open;
// relay frames of SessionManager.cpp:362-387 are the C3 shape.
#include "stream_common.hpp"

namespace enet {

constexpr uint32_t kTailSlot = 144;               // per-record LDS slot: 9 16-byte chunks
constexpr uint32_t kTailPart = 64 * kTailSlot;    // one compute wave's 64 records
constexpr int kTailDmas = 18;                     // per memory wave per stage: 2 x 64 x 9 chunks / 64

__device__ __forceinline__ uint32_t tail_slot(uint32_t o) { return ((o & 3u) << 3) | ((o >> 2) & 7u) | (o & 32u); }
__device__ __forceinline__ uint32_t tail_owner(uint32_t s) { return ((s & 7u) << 2) | ((s >> 3) & 3u) | (s & 32u); }
// store lane l reads chunk tail_store_chunk(l) of slot (i & 7) + 8 tail_store_j(l): per 16-lane group
// of ds_read_b128 ({0-3,12-15,20-27}, ...), (9 slot + chunk) mod 16 takes every value once
__device__ __forceinline__ uint32_t tail_store_chunk(uint32_t l) { return (l & 3u) | (((l >> 3) & 1u) << 2); }
__device__ __forceinline__ uint32_t tail_store_j(uint32_t l) {
    const uint32_t idx = ((l >> 4) & 1u) * 2u + (((l >> 2) ^ (l >> 3)) & 1u);
    return 4u * (l >> 5) + ((0x78u >> (2u * idx)) & 3u);
}
// lanes of a store whose chunk is 0: window 0's first chunk is not stored by the memory waves
constexpr uint64_t kTailChunk0Lanes = 0x0011001100110011ull;

// Poly1305 over the first ceil(rem / 16) 16-byte blocks of a 128-byte run, bytes >= rem zeroed
// (the last stage of a record; rem is a multiple of 4, uniform across the workgroup)
__device__ __forceinline__ void poly_run_tail(uint32_t h[5], const PolyR32& R, const uint32_t w[32], uint32_t rem) {
    const uint32_t nb16 = (rem + 15u) >> 4;
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
        if (u < nb16) {
            uint32_t m[4];
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) m[i] = (4u * (4u * u + i) < rem) ? w[4 * u + i] : 0u;
            poly32_block(h, R, m[0], m[1], m[2], m[3], 1u);
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(kStreamWG) void stream_tail_kernel(RecParams p) {
    constexpr bool kPoly = (MODE != MODE_XOR);
    constexpr int kPos = kStreamSteps;  // barrier positions per stage
    __shared__ __attribute__((aligned(16))) uint8_t s_in[kStreamLanes * kTailSlot];
    // 16 bytes of pad in front: slot 0's carry words land at offsets -12 .. -1
    __shared__ __attribute__((aligned(16))) uint8_t s_out[16 + kStreamLanes * kTailSlot];

    const uint32_t L = (uint32_t)p.uniform_len;
    const bool compute = threadIdx.x < kStreamLanes;
    const uint32_t rec = blockIdx.x * kStreamLanes + (compute ? threadIdx.x : 0u);
    const uint32_t B = (L + 63u) >> 6;       // ChaCha20 blocks per record
    const uint32_t S = (B + 1u) >> 1;        // stages (>= 2: L >= 128)
    const uint32_t rem = L - kRun * (S - 1); // bytes of the last stage
    const uint64_t i0 = p.in_off[0], o0 = p.out_off[0];
    const uint64_t ia = reinterpret_cast<uintptr_t>(p.in) + i0, oa = reinterpret_cast<uintptr_t>(p.out) + o0;
    {
        // every record at its uniform place, the next record long enough for the last stage's
        // over-read, 4-byte-aligned starts (dword-exact edge stores); else the per-lane path
        const bool mine = !compute || (p.in_off[rec] == i0 + (uint64_t)rec * L &&
                                       p.in_off[rec + 1] == i0 + (uint64_t)(rec + 1) * L &&
                                       p.out_off[rec] == o0 + (uint64_t)rec * L &&
                                       p.out_off[rec + 1] == o0 + (uint64_t)(rec + 1) * L &&
                                       p.in_off[rec + 2] >= i0 + (uint64_t)(rec + 1) * L + (kRun * S + 16u - L) &&
                                       (ia & 3u) == 0 && (oa & 3u) == 0);
        if (!__syncthreads_and(mine ? 1 : 0)) {
            if (compute) records_body<0, MODE, FR_NONE, 7>(p);
            return;
        }
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    auto din = [&](uint32_t g) { return (uint32_t)((ia + (uint64_t)g * L) & 15u); };
    auto dout = [&](uint32_t g) { return (uint32_t)((oa + (uint64_t)g * L) & 15u); };

    if (!compute) {
        // ================================================================ memory waves
        // Memory wave m serves compute waves 2m and 2m+1 (records rec0 .. rec0 + 127).  32-bit
        // offsets from SGPR bases 16 bytes before the arenas (window 0 of record 0 starts up to 12
        // bytes before them, inside their first 16-byte granule).
        const uint32_t m = wave - 8u;
        __builtin_amdgcn_s_setprio(3);
        const uint32_t rec0 = blockIdx.x * kStreamLanes + 128u * m;
        uint32_t doff[kTailDmas];
#pragma unroll
        for (int i = 0; i < kTailDmas; ++i) {
            const uint32_t q = 64u * i + lane;  // flat chunk of the two parts: slot q / 9, chunk q % 9
            const uint32_t si = q / 9u, c = q - 9u * si;
            const uint32_t g = rec0 + (si & 64u) + tail_owner(si & 63u);
            doff[i] = g * L - din(g) + 16u + 16u * c;
        }
        const uint32_t sc = tail_store_chunk(lane), sj = tail_store_j(lane);
        uint32_t soff[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t g = rec0 + 64u * (uint32_t)(i >> 3) + tail_owner((uint32_t)(i & 7) + 8u * sj);
            soff[i] = g * L - dout(g) + 16u + 16u * sc;
        }
        auto uni = [](uint64_t v) {
            return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
        };
        const uint8_t* ibase = reinterpret_cast<const uint8_t*>(uni(ia - 16u));
        uint8_t* obase = reinterpret_cast<uint8_t*>(uni(oa - 16u));
        const uint32_t in_part = (uint32_t)reinterpret_cast<uintptr_t>(s_in) + 2u * m * kTailPart;
        const uint8_t* out_lane = s_out + 16u + 2u * m * kTailPart + kTailSlot * 8u * sj + 16u * sc;
        // DMA i lands 1 KiB at in_part + 1024 i (lane-linear), i.e. slots and chunks q / 9, q % 9
        auto dma = [&](const uint8_t* base, int i) {
            const uint32_t m0 = in_part + 1024u * (uint32_t)i;
            uint32_t keep;
            // plain (not non-temporal) loads: chunk 8 of window st is chunk 0 of window st + 1
            asm volatile("s_mov_b32 %0, m0\n s_mov_b32 m0, %2\n s_nop 0\n global_load_lds_dwordx4 %1, %3\n s_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(doff[i]), "s"(m0), "s"(base) : "memory");
        };
        auto ldsread = [&](int i) {
            return *reinterpret_cast<const uint4*>(out_lane + kTailPart * (uint32_t)(i >> 3) + kTailSlot * (uint32_t)(i & 7));
        };
        // windows are 16-byte aligned but not lines: plain stores, L2 merges a line's two halves
        auto store = [&](uint8_t* base, int i, uint4 v) {
            enet_u32x4 d = {v.x, v.y, v.z, v.w};
            asm volatile("global_store_dwordx4 %0, %1, %2\n s_nop 1" :: "v"(soff[i]), "v"(d), "s"(base) : "memory");
        };
        // window 0: every lane but the chunk-0 ones (that chunk also holds the previous record's bytes)
        auto store_w0 = [&](uint8_t* base, int i, uint4 v) {
            enet_u32x4 d = {v.x, v.y, v.z, v.w};
            uint64_t save;
            asm volatile("s_mov_b64 %0, exec\n s_and_b64 exec, exec, %4\n global_store_dwordx4 %1, %2, %3\n s_mov_b64 exec, %0\n s_nop 1"
                         : "=&s"(save) : "v"(soff[i]), "v"(d), "s"(base), "s"(~kTailChunk0Lanes) : "memory");
        };
#pragma unroll
        for (int i = 0; i < kTailDmas; ++i) dma(ibase, i);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (uint32_t st = 0; st < S; ++st) {
            stream_barrier();  // S0(st): window st landed; window st-1 in the output slots
            const bool more = st + 1 < S, prev = st > 0, first = st == 1;
            const uint8_t* inext = ibase + (size_t)kRun * (st + 1);
            uint8_t* oprev = obase + (size_t)kRun * (st - 1);
            uint4 v = make_uint4(0, 0, 0, 0);
            if (__builtin_expect(prev, 1)) v = ldsread(0);
#pragma unroll
            for (int k = 0; k < kPos; ++k) {
                // DMA d at position 1 + 3 d (after keystream barrier 0: the runs are in registers)
                if (k >= 1 && (k - 1) % 3 == 0 && (k - 1) / 3 < kTailDmas) {
                    if (__builtin_expect(more, 1)) dma(inext, (k - 1) / 3);
                }
                // store s at position 2 + 3 s
                if (k >= 2 && (k - 2) % 3 == 0 && (k - 2) / 3 < 16) {
                    const int sl = (k - 2) / 3;
                    if (__builtin_expect(prev, 1)) {
                        if (__builtin_expect(first, 0)) store_w0(oprev, sl, v);
                        else store(oprev, sl, v);
                        if (sl < 15) v = ldsread(sl + 1);
                    }
                }
                stream_barrier();
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next window has landed
        }
        stream_barrier();  // F1: the last window is in the output slots
        {
            // last window: record bytes [128 (S-1) - d, ...), stored dword-exact up to L
            uint8_t* olast = obase + (size_t)kRun * (S - 1);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint4 v = ldsread(i);
                const uint32_t g = rec0 + 64u * (uint32_t)(i >> 3) + tail_owner((uint32_t)(i & 7) + 8u * sj);
                const uint32_t valid = rem + dout(g), c0 = 16u * sc;
                uint8_t* q = olast + soff[i];
                if (c0 + 16u <= valid) {
                    *reinterpret_cast<uint4*>(q) = v;
                } else if (c0 < valid) {
                    const uint32_t w4[3] = {v.x, v.y, v.z};
#pragma unroll
                    for (uint32_t j = 0; j < 3; ++j)
                        if (c0 + 4u * j < valid) reinterpret_cast<uint32_t*>(q)[j] = w4[j];
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store done (tamper zeroing)
        stream_barrier();  // F2
        return;
    }

    // ==================================================================== compute waves
    const uint32_t slot = tail_slot(lane);
    const uint32_t dq = dout(rec);
    const uint32_t* myin = reinterpret_cast<const uint32_t*>(s_in + wave * kTailPart + kTailSlot * slot + din(rec));
    uint32_t* myout = reinterpret_cast<uint32_t*>(s_out + 16u + wave * kTailPart + kTailSlot * slot + dq - 12u);
    uint8_t* rout = p.out + o0 + (uint64_t)rec * L;

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

    // ---- Poly1305: one-time key from block 0 (runs while window 0 lands), then the AAD
    uint32_t h[5] = {0, 0, 0, 0, 0};
    PolyR32 PR{};
    uint32_t pad[4] = {0, 0, 0, 0};
    uint32_t aad_len = 0;
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

    const uint32_t ff[16] = {kSigma0, kSigma1, kSigma2, kSigma3, R.k[0], R.k[1], R.k[2], R.k[3],
                             R.k[4], R.k[5], R.k[6], R.k[7], 0u, R.n[0], R.n[1], R.n[2]};
    uint32_t carry[3] = {0u, 0u, 0u};  // the previous run's last three output words
    for (uint32_t st = 0; st < S; ++st) {
        // S0(st): the memory waves saw window st land; this wave's output writes are done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stream_barrier();
        uint32_t w[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) w[k] = myin[k];
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
        // the run is in registers before keystream barrier 0: the slot may be refilled
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        chacha_half_lockstep2<true, NoStepHook, 1>(x);
#pragma unroll
        for (int dr = 1; dr < 10; ++dr) {
            chacha_half_lockstep2<false, NoStepHook, 1>(x);
            chacha_half_lockstep2<true, NoStepHook, 1>(x);
        }
        const bool part = st + 1 == S;  // the last stage holds rem record bytes (uniform)
        if (MODE == MODE_OPEN) {
            if (part) {
                poly_run_tail(h, PR, w, rem);
            } else {
                poly_block64(h, PR, w);
                poly_block64(h, PR, w + 16);
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            w[i] ^= x[i] + (i == 12 ? c0 : ff[i]);
            w[16 + i] ^= x[16 + i] + (i == 12 ? c0 + 1u : ff[i]);
        }
        if (MODE == MODE_SEAL) {
            if (part) {
                poly_run_tail(h, PR, w, rem);
            } else {
                poly_block64(h, PR, w);
                poly_block64(h, PR, w + 16);
            }
        }
        // window st = the previous run's last d words || this run's first 32 - d words
        myout[0] = carry[0]; myout[1] = carry[1]; myout[2] = carry[2];
#pragma unroll
        for (int k = 0; k < 32; ++k) myout[3 + k] = w[k];
        carry[0] = w[29]; carry[1] = w[30]; carry[2] = w[31];
        if (__builtin_expect(st == 0, 0)) {
            // window 0's first chunk also holds the previous record's bytes: its 16 - d bytes of
            // this record go out from here
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k)
                if (4u * k + dq < 16u) reinterpret_cast<uint32_t*>(rout)[k] = w[k];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stream_barrier();  // F1
    // record bytes past the last window ([128 S - d, L), from the carry)
#pragma unroll
    for (uint32_t i = 0; i < 3; ++i) {
        const uint32_t k = 29u + i;
        if (4u * k + dq >= 128u && 4u * k < rem)
            reinterpret_cast<uint32_t*>(rout + (size_t)kRun * (S - 1))[k] = carry[i];
    }
    uint32_t diff = 0;
    if (kPoly) {
        // length block LE64(|aad|) || LE64(|ct|)
        poly32_block(h, PR, aad_len, 0u, L, 0u, 1u);
        uint32_t l[5];
        h32_to_limbs(h, l);
        uint32_t tag[4];
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
    stream_barrier();  // F2: the memory waves' stores of this workgroup are complete
    if (MODE == MODE_OPEN && diff != 0) {
        // authentication failed: do not release plaintext (exactly the record's L bytes)
        for (uint32_t c = 0; c < (L >> 2); ++c) reinterpret_cast<uint32_t*>(rout)[c] = 0u;
    }
}

// One lane per record, L % 4 == 0, L >= 128 and not a multiple of 128, at least one record after
// the launched ones (n > 512: the launch covers (n - 1) / 512 whole workgroups), 32-bit offsets.
bool stream_tail_eligible(const RecParams& p, uint32_t lanes) {
    const uint64_t L = p.uniform_len;
    return (p.stream & 2) && lanes == 1 && L >= 128 && L % 128 != 0 && L % 4 == 0 && p.order == nullptr &&
           L * (uint64_t)p.n <= 0xFFFFFFFFull - 512 && p.n > kStreamLanes;
}

hipError_t launch_stream_tail(int mode, const RecParams& p, uint32_t blocks, hipStream_t s) {
    switch (mode) {
        case MODE_XOR: hipLaunchKernelGGL((stream_tail_kernel<MODE_XOR>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        case MODE_SEAL: hipLaunchKernelGGL((stream_tail_kernel<MODE_SEAL>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        case MODE_OPEN: hipLaunchKernelGGL((stream_tail_kernel<MODE_OPEN>), dim3(blocks), dim3(kStreamWG), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace enet
