// segments.hip -- the sequence-parallel axis: records too long for the record
// engine's at most 16 lanes are cut into 64 KiB TILES spread over every CU of the chip.
//
// Reference shapes this serves: a stored file is ONE chunk of up to 32 MiB
// (include/ephemeralnet/Config.hpp:62, src/main.cpp:4467, encrypted whole in
// src/core/Node.cpp:1414-1417 and decrypted whole in Node.cpp:1644-1655); session payloads go up
// to 1 MiB (src/network/SessionManager.cpp:87).  On the record engine one such record got 16
// lanes: a lone 32 MiB AEAD record was 32 768 serial ChaCha20 blocks per lane.
//
// Three steps on the caller's stream:
//   1. seg_plan_kernel: every record >= the threshold CLAIMS a contiguous range of tile indices
//      (one 64-bit CAS on a packed count|tiles word, so entries come out sorted by tile base) and
//      writes its entry -- for the AEAD also the one-time Poly1305 key and the power table
//      r^(2^k), k = 0..nbits -- and a claimed[] byte per record that the record engine skips.
//   2. seg_kernel: a grid of 256-lane workgroups walks the tiles.  Lane j of a tile owns the four
//      ChaCha20 blocks [tile*1024 + 4j, +4) of its record; a tile whose 64 KiB are all whole blocks
//      moves them through a wave-private LDS slab with whole 128-byte lines per load / store
//      instruction (the staging of records_body.hpp COOP 1), a ragged last tile goes per lane.
//      XOR mode ends there (counter = start + block index, mod 2^32 as ChaCha20.cpp:110).
//   3. AEAD: lane j's Poly1305 Horner covers its own blocks; the lane scales its accumulator by
//      r^(tile end - lane end) from the entry's power table and the workgroup sums the lanes: the
//      tile's partial, normalised at the tile's end.  The last tile of a record to finish (an
//      agent-scope arrival counter) combines the record's partials -- Horner over whole tiles in
//      r^4096, one table-power scale per lane -- adds the pad s and writes the tag (seal) or the
//      verdict (open; a failed record's plaintext is zeroed by that workgroup).
// No MFMA: nothing here is a contraction.
#include "enet_device.hpp"
#include "enet_internal.hpp"
#include "records_body.hpp"

namespace enet {

namespace {

constexpr uint32_t kSegThreads = 256;                 // lanes per tile workgroup
constexpr uint32_t kSegBPL = 4;                       // ChaCha20 blocks per lane
constexpr uint32_t kTileBlocks = kSegThreads * kSegBPL;  // 1024 blocks = 64 KiB
constexpr uint64_t kTileBytes = 64ull * kTileBlocks;
constexpr uint32_t kTilePoly = 4 * kTileBlocks;       // Poly1305 blocks per whole tile (4096)
constexpr int kTileCountBits = 40;                    // header word: count << 40 | tiles
constexpr unsigned long long kTileMask = (1ull << kTileCountBits) - 1;

}  // namespace

__device__ __forceinline__ void pcarry(uint32_t l[5]) {
    uint32_t c;
    c = l[0] >> 26; l[0] &= M26; l[1] += c;
    c = l[1] >> 26; l[1] &= M26; l[2] += c;
    c = l[2] >> 26; l[2] &= M26; l[3] += c;
    c = l[3] >> 26; l[3] &= M26; l[4] += c;
    c = l[4] >> 26; l[4] &= M26; l[0] += 5u * c;
    c = l[0] >> 26; l[0] &= M26; l[1] += c;
}

// l <- l * r^e with the table pw[k] = r^(2^k) (e < 2^nbits)
__device__ __forceinline__ void pscale(uint32_t l[5], uint32_t e, const uint32_t* pw, uint32_t nbits) {
    for (uint32_t k = 0; k < nbits; ++k) {
        if ((e >> k) & 1u) {
            uint32_t m[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) m[i] = pw[5 * k + i];
            pmul(l, pmul_make(m));
        }
    }
}

// l <- l * m (26-bit limbs)
__device__ __forceinline__ void pmul_by(uint32_t l[5], const uint32_t m[5]) { pmul(l, pmul_make(m)); }

// h <- h^2 (mod 2^130-5): 15 products instead of pmul's 25; same bounds and reduction as pmul
__device__ __forceinline__ void psquare(uint32_t h[5]) {
    const uint64_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
    const uint64_t t0 = 2 * h0, t1 = 2 * h1, f3 = 5 * h3, f4 = 5 * h4, g4 = 10 * h4;
    uint64_t d0 = h0 * h0 + h1 * g4 + h2 * (2 * f3);
    uint64_t d1 = t0 * h1 + h2 * g4 + h3 * f3;
    uint64_t d2 = t0 * h2 + h1 * h1 + h3 * g4;
    uint64_t d3 = t0 * h3 + t1 * h2 + h4 * f4;
    uint64_t d4 = t0 * h4 + t1 * h3 + h2 * h2;
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h[0] = (uint32_t)d0 & M26; d1 += c;
    c = (uint32_t)(d1 >> 26); h[1] = (uint32_t)d1 & M26; d2 += c;
    c = (uint32_t)(d2 >> 26); h[2] = (uint32_t)d2 & M26; d3 += c;
    c = (uint32_t)(d3 >> 26); h[3] = (uint32_t)d3 & M26; d4 += c;
    c = (uint32_t)(d4 >> 26); h[4] = (uint32_t)d4 & M26;
    h[0] += c * 5u;
    c = h[0] >> 26; h[0] &= M26; h[1] += c;
}

// Sum of the workgroup's 256 accumulators (limbs < 2^27) into thread 0's l (limbs < 2^27)
__device__ __forceinline__ void wg_sum(uint32_t l[5], uint32_t* red /* [4][5] shared */) {
#pragma unroll
    for (int off = 1; off <= 8; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[5 * w + i] = l[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] = red[i] + red[5 + i] + red[10 + i] + red[15 + i];
        pcarry(l);
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t seg_counter(const SegParams& p, uint32_t rec) {
    if (p.mode != MODE_XOR) return 1u;  // RFC 8439 data counter
    return p.counters ? p.counters[(size_t)rec * (p.counter_stride ? p.counter_stride : 1u)] : 0u;
}

// ---------------------------------------------------------------------------------- plan
// Thread per record (grid-stride).  A lone workgroup initialises the header itself; larger grids
// get it zeroed by the host (hipMemsetAsync) first.
__global__ __launch_bounds__(kSegThreads) void seg_plan_kernel(SegParams p) {
    if (gridDim.x == 1) {
        if (threadIdx.x == 0) __hip_atomic_store(p.hdr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
    }
    for (uint32_t pos = blockIdx.x * kSegThreads + threadIdx.x; pos < p.n; pos += gridDim.x * kSegThreads) {
        const uint32_t i = p.order ? p.order[pos] : pos;  // a subset of the batch (capi chunk paths)
        const uint64_t L = p.in_off[i + 1] - p.in_off[i];
        bool claim = L >= p.long_min && L < kSegMaxLen;
        uint32_t idx = 0, base = 0;
        const uint64_t tiles = L ? (L + kTileBytes - 1) / kTileBytes : 1;
        if (claim) {
            unsigned long long old = __hip_atomic_load(p.hdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (;;) {
                const uint64_t cnt = old >> kTileCountBits, tb = old & kTileMask;
                if (cnt >= p.entry_cap || tb + tiles > p.tile_cap) {
                    claim = false;  // over the scratch the host sized from its hints: record engine
                    break;
                }
                const unsigned long long nw = old + (1ull << kTileCountBits) + tiles;
                if (__hip_atomic_compare_exchange_strong(p.hdr, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)) {
                    idx = (uint32_t)cnt;
                    base = (uint32_t)tb;
                    break;
                }
            }
        }
        if (p.claimed) p.claimed[i] = claim ? 1 : 0;
        if (!claim) continue;
        SegEntry& e = p.entries[idx];
        e.rec = i;
        e.tile_base = base;
        e.ntiles = (uint32_t)tiles;
        e.arrived = 0;
        if (p.mode == MODE_XOR) continue;
        // AEAD: one-time key = block 0 (RFC 8439 2.6), AAD length, power table
        uint32_t kw[8], nw[3];
        const uint32_t* kp = reinterpret_cast<const uint32_t*>(p.keys + (size_t)p.key_stride * i);
#pragma unroll
        for (int t = 0; t < 8; ++t) kw[t] = kp[t];
        const uint32_t* np = reinterpret_cast<const uint32_t*>(p.nonces + 12ull * i);
#pragma unroll
        for (int t = 0; t < 3; ++t) nw[t] = np[t];
        ChachaRecord R;
        chacha_record_init(R, kw, nw);
        uint32_t otk[16];
        chacha_block(R, 0u, otk);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            e.r[t] = otk[t];
            e.s[t] = otk[4 + t];
        }
        uint32_t aad_len = 0;
        if (p.aad) aad_len = (uint32_t)(p.aad_off[i + 1] - p.aad_off[i]);
        e.aad_len = aad_len;
        const uint64_t K = (uint64_t)((aad_len + 15) >> 4) + (L + 15) / 16 + 1;  // Poly1305 blocks
        const uint32_t nbits = 64u - (uint32_t)__builtin_clzll(K);
        e.nbits = nbits;
        uint32_t x[5];
        pclamp(x, otk[0], otk[1], otk[2], otk[3]);
        for (uint32_t k = 0; k < nbits; ++k) {
#pragma unroll
            for (int t = 0; t < 5; ++t) e.pw[5 * k + t] = x[t];
            pmul(x, pmul_make(x));
        }
    }
}

// ---------------------------------------------------------------------------------- tiles
template <int MODE>
__global__ __launch_bounds__(kSegThreads) void seg_kernel(SegParams p) {
    constexpr bool kPoly = MODE != MODE_XOR;
    __shared__ __attribute__((aligned(16))) uint8_t slab[kSegThreads * kRun];
    __shared__ uint32_t red[20];
    __shared__ uint32_t last_flag;
    const unsigned long long hw = *p.hdr;
    const uint32_t count = (uint32_t)(hw >> kTileCountBits);
    const uint32_t total = (uint32_t)(hw & kTileMask);
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    const uint32_t j = threadIdx.x;

    for (uint32_t tile = blockIdx.x; tile < total; tile += gridDim.x) {
        // the entry whose tile range holds this tile (entries are sorted by tile_base)
        uint32_t lo = 0, hi = count;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (p.entries[mid].tile_base <= tile) lo = mid;
            else hi = mid;
        }
        SegEntry& E = p.entries[lo];
        const uint32_t rec = E.rec;
        const uint32_t tr = tile - E.tile_base;
        const uint64_t ioff = p.in_off[rec];
        const uint64_t L = p.in_off[rec + 1] - ioff;
        const uint64_t ooff = p.out_off[rec];
        const uint32_t nb = (uint32_t)((L + 63) >> 6);
        const uint32_t tb0 = tr * kTileBlocks;
        const uint32_t tb1 = min(tb0 + kTileBlocks, nb);
        const uint32_t c0 = min(tb0 + kSegBPL * j, tb1), c1 = min(c0 + kSegBPL, tb1);
        const uint8_t* src = p.in + ioff;
        uint8_t* dst = p.out + ooff;

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
        const uint32_t ctr0 = seg_counter(p, rec);

        // Poly1305 state: lane 0 of the record's first tile absorbs the AAD prefix
        uint32_t h[5] = {0, 0, 0, 0, 0};
        PolyR32 PR{};
        uint32_t na = 0, aad_len = 0;
        const uint32_t nct = (uint32_t)((L + 15) >> 4);
        if (kPoly) {
            PR = polyr32_make(E.r[0], E.r[1], E.r[2], E.r[3]);
            aad_len = E.aad_len;
            na = (aad_len + 15) >> 4;
            if (tr == 0 && j == 0 && na) {
                const uint8_t* ap = p.aad + p.aad_off[rec];
                for (uint32_t s = 0; s < na; ++s) {
                    const uint32_t cnt = min(16u, aad_len - 16u * s);
                    uint32_t w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        uint32_t v = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            if ((uint32_t)(4 * i + b) < cnt) v |= (uint32_t)ap[16 * s + 4 * i + b] << (8 * b);
                        w[i] = v;
                    }
                    poly32_block(h, PR, w[0], w[1], w[2], w[3], 1u);
                }
            }
        }

        const bool whole = (uint64_t)(tb0 + kTileBlocks) * 64ull <= L;  // uniform over the workgroup
        if (whole) {
            // two stages of two blocks per lane; load / store instruction i serves the owners
            // 8i .. 8i+7 of the wave, eight lanes per owner = one whole 128-byte run each
            const uint32_t kk = lane & 7u;
            const uint32_t msw = slab_sw(lane);
            uint8_t* wslab = slab + wbase * kRun;
            uint8_t* myrun = slab + threadIdx.x * kRun;
            const uint8_t* ib = src + 64ull * tb0;
            uint8_t* ob = dst + 64ull * tb0;
            const bool nt = ((reinterpret_cast<uintptr_t>(ob)) & 63u) == 0;
            uint32_t offs[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t o = 8u * i + (lane >> 3);
                offs[i] = 64u * kSegBPL * (wbase + o) + 16u * (kk ^ slab_sw(o));
            }
            uint32_t pf[32];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(ib + offs[i]);
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            }
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                ENET_WAVE_LDS_SYNC();
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                        make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
                ENET_WAVE_LDS_SYNC();
                uint32_t w2[32];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                    w2[4 * k] = v.x; w2[4 * k + 1] = v.y; w2[4 * k + 2] = v.z; w2[4 * k + 3] = v.w;
                }
                if (st == 0) {  // the second stage's lines fly under this stage's rounds
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint4 v = *reinterpret_cast<const uint4*>(ib + offs[i] + kRun);
                        pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
                    }
                    asm volatile("" : "+v"(R.k[0])::"memory");
                }
                const uint32_t cb = ctr0 + c0 + 2u * st;  // u32 wrap (ChaCha20.cpp:110)
                if (MODE == MODE_OPEN) {
                    poly_block64(h, PR, w2);
                    poly_block64(h, PR, w2 + 16);
                }
                uint32_t ka[16], kb[16];
                chacha_block2(R, cb, cb + 1u, ka, kb);
#pragma unroll
                for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
                if (MODE == MODE_SEAL) {
                    poly_block64(h, PR, w2);
                    poly_block64(h, PR, w2 + 16);
                }
                ENET_WAVE_LDS_SYNC();
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                        make_uint4(w2[4 * k], w2[4 * k + 1], w2[4 * k + 2], w2[4 * k + 3]);
                ENET_WAVE_LDS_SYNC();
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint4 v = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                    store_stream(ob + offs[i] + kRun * st, v, nt);
                }
            }
        } else {
            // the record's ragged last tile: per lane, partial block masked
            for (uint32_t c = c0; c < c1; ++c) {
                const uint64_t pos = 64ull * c;
                const uint32_t nbytes = (uint32_t)min<uint64_t>(64, L - pos);
                uint32_t w[16];
                load_block(src + pos, nbytes, w, pos + nbytes >= 16);
                uint32_t o[16];
                chacha_block(R, ctr0 + c, o);
#pragma unroll
                for (int i = 0; i < 16; ++i) o[i] ^= w[i];
                store_block(dst + pos, nbytes, o);
                if (kPoly) {
                    uint32_t* ct = (MODE == MODE_SEAL) ? o : w;
                    if (MODE == MODE_SEAL && nbytes < 64) mask_tail(ct, nbytes);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (4 * c + u < nct)
                            poly32_block(h, PR, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
                }
            }
        }

        if (kPoly) {
            // the lane holding the record's last block absorbs the length block
            const bool last_tile = tb1 == nb;
            const bool has_last = (c1 == nb && c1 > c0) || (nb == 0 && j == 0);
            if (has_last) poly32_block(h, PR, aad_len, 0u, (uint32_t)L, (uint32_t)(L >> 32), 1u);
            // positions (Poly1305 block index + 1) where this lane's and the tile's runs end
            const uint32_t lane_end = na + min(4u * c1, nct) + (has_last ? 1u : 0u);
            const uint32_t tile_end = na + min(4u * tb1, nct) + (last_tile ? 1u : 0u);
            uint32_t l[5];
            h32_to_limbs(h, l);
#ifndef ENET_SEG_PROBE_NO_SCALE  // timing probes (hand-built libraries only; wrong tags)
            if (c1 > c0 || (tr == 0 && j == 0)) pscale(l, tile_end - lane_end, E.pw, min(E.nbits, 14u));
#endif
            wg_sum(l, red);
            // Publish the tile's partial; the record's last tile to arrive finishes the record.
            // Hand-off without an L2 write-back (MI355X_MICROARCH.md, inter-workgroup visibility,
            // first row of the sc1 table): thread 0 stores the partial write-through (sc1),
            // drains it (vmcnt 0), then takes a ticket with a relaxed agent-scope add; the
            // workgroup whose add comes last reads every partial with sc1 loads after a barrier.
            // (__threadfence() here wrote back the XCD's whole L2 once per tile.)
            uint32_t* part = p.partials + 8ull * tile;
            if (threadIdx.x == 0) {
#pragma unroll
                for (int i = 0; i < 5; ++i) __hip_atomic_store(part + i, l[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t prev = __hip_atomic_fetch_add(&E.arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last_flag = prev + 1 == E.ntiles ? 1u : 0u;
            }
            __syncthreads();
#ifdef ENET_SEG_PROBE_NO_TAIL
            last_flag = 0;
#endif
            if (last_flag) {
                const uint32_t nt = E.ntiles;
                const uint32_t K = na + nct + 1;
                // whole tiles [0, nt-1) end at na + 4096 (t+1); the last one at K.  Lane j runs
                // Horner in r^4096 over its contiguous tiles, then scales by r^(K - its end).
                const uint32_t nw = nt - 1;
                const uint32_t q = (nw + kSegThreads - 1) / kSegThreads;
                const uint32_t t0 = min(j * q, nw), t1 = min(t0 + q, nw);
                uint32_t acc[5] = {0, 0, 0, 0, 0};
                auto load_part = [&](uint32_t t) {
                    const uint32_t* v = p.partials + 8ull * (E.tile_base + t);
#pragma unroll
                    for (int i = 0; i < 5; ++i) acc[i] += __hip_atomic_load(v + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    pcarry(acc);
                };
                if (t1 > t0) {
                    uint32_t m4096[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) m4096[i] = E.pw[5 * 12 + i];
                    const Pmul M = pmul_make(m4096);
                    for (uint32_t t = t0; t < t1; ++t) {
                        if (t > t0) pmul(acc, M);
                        load_part(t);
                    }
                    pscale(acc, K - (na + kTilePoly * t1), E.pw, E.nbits);
                }
                if (j == kSegThreads - 1) load_part(nt - 1);  // already normalised at K
                wg_sum(acc, red);
                if (threadIdx.x == 0) {
                    uint32_t tag[4];
                    pfinish(acc, E.s, tag);
                    if (MODE == MODE_SEAL) {
                        uint32_t* tp = reinterpret_cast<uint32_t*>(p.tag_out + 16ull * rec);
                        tp[0] = tag[0]; tp[1] = tag[1]; tp[2] = tag[2]; tp[3] = tag[3];
                    } else {
                        // a failed record's plaintext is zeroed by the record kernel launched
                        // after this one (records_body: claimed records with ok == 0): zero
                        // stores from here could be overtaken by other tiles' plaintext still
                        // dirty in their XCD's L2
                        const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tag_in + 16ull * rec);
                        const uint32_t diff = (tag[0] ^ tp[0]) | (tag[1] ^ tp[1]) | (tag[2] ^ tp[2]) | (tag[3] ^ tp[3]);
                        p.ok[rec] = diff == 0 ? 1 : 0;
                    }
                }
            }
        }
        __syncthreads();  // the slab and red[] are reused by the next tile
    }
}

// ---------------------------------------------------------------------------------- uniform XOR
// ChaCha20 (XOR mode) over a batch whose hints say every record is L >= ENET_SEG_MIN bytes: ONE
// launch, no plan and no record-engine pass.  Workgroup t serves tile t % T of record t / T
// (T = ceil(L / 64 KiB)); every workgroup checks its record against the hint, and a record whose
// real length differs is run whole by the workgroup of its tile 0, tile after tile (a wrong hint
// costs speed, never bytes).  The three-launch path (plan, tiles, record engine) cost ~4 us per
// launch whatever the launch does (profiles/r06b_long_kernel_stats.csv).

// One tile of a record in XOR mode: lane j owns blocks [tb0 + 4j, +4) clipped to the record.
__device__ __forceinline__ void xor_tile(const uint8_t* src, uint8_t* dst, uint64_t L, uint32_t tb0,
                                         uint32_t ctr0, const ChachaRecord& R, uint8_t* slab) {
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    const uint32_t j = threadIdx.x;
    const uint32_t nb = (uint32_t)((L + 63) >> 6);
    const uint32_t tb1 = min(tb0 + kTileBlocks, nb);
    const uint32_t c0 = min(tb0 + kSegBPL * j, tb1), c1 = min(c0 + kSegBPL, tb1);
    const bool whole = (uint64_t)(tb0 + kTileBlocks) * 64ull <= L;  // uniform over the workgroup
    if (whole) {
        const uint32_t kk = lane & 7u;
        const uint32_t msw = slab_sw(lane);
        uint8_t* wslab = slab + wbase * kRun;
        uint8_t* myrun = slab + threadIdx.x * kRun;
        const uint8_t* ib = src + 64ull * tb0;
        uint8_t* ob = dst + 64ull * tb0;
        const bool nt = ((reinterpret_cast<uintptr_t>(ob)) & 63u) == 0;
        uint32_t offs[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t o = 8u * i + (lane >> 3);
            offs[i] = 64u * kSegBPL * (wbase + o) + 16u * (kk ^ slab_sw(o));
        }
        uint32_t pf[32];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint4 v = *reinterpret_cast<const uint4*>(ib + offs[i]);
            pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
            const uint32_t cb = ctr0 + c0 + 2u * st;  // u32 wrap (ChaCha20.cpp:110)
            uint32_t ka[16], kb[16];
#ifndef ENET_SEG_PROBE_XOR_OLD
            chacha_block2(R, cb, cb + 1u, ka, kb);  // the keystream first, under the loads' latency
#endif
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                    make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
            ENET_WAVE_LDS_SYNC();
            uint32_t w2[32];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                w2[4 * k] = v.x; w2[4 * k + 1] = v.y; w2[4 * k + 2] = v.z; w2[4 * k + 3] = v.w;
            }
            if (st == 0) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ib + offs[i] + kRun);
                    pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
                }
            }
#ifdef ENET_SEG_PROBE_XOR_OLD
            chacha_block2(R, cb, cb + 1u, ka, kb);
#endif
#pragma unroll
            for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                    make_uint4(w2[4 * k], w2[4 * k + 1], w2[4 * k + 2], w2[4 * k + 3]);
            ENET_WAVE_LDS_SYNC();
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                store_stream(ob + offs[i] + kRun * st, v, nt);
            }
        }
    } else {
        for (uint32_t c = c0; c < c1; ++c) {
            const uint64_t pos = 64ull * c;
            const uint32_t nbytes = (uint32_t)min<uint64_t>(64, L - pos);
            uint32_t w[16];
            load_block(src + pos, nbytes, w, pos + nbytes >= 16);
            uint32_t o[16];
            chacha_block(R, ctr0 + c, o);
#pragma unroll
            for (int i = 0; i < 16; ++i) o[i] ^= w[i];
            store_block(dst + pos, nbytes, o);
        }
    }
}

__global__ __launch_bounds__(kSegThreads) void seg_uniform_xor_kernel(SegParams p, uint64_t L, uint32_t T) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[kSegThreads * kRun];
    const uint32_t rec = blockIdx.x / T, tr = blockIdx.x % T;
    const uint64_t ioff = p.in_off[rec];
    const uint64_t Lr = p.in_off[rec + 1] - ioff;
    const bool as_hinted = p.in_off[rec + 1] >= ioff && Lr == L;
    if (!as_hinted && tr != 0) return;  // the record's tile-0 workgroup runs it whole
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
    const uint32_t ctr0 = seg_counter(p, rec);
    const uint8_t* src = p.in + ioff;
    uint8_t* dst = p.out + p.out_off[rec];
    if (as_hinted) {
        xor_tile(src, dst, L, tr * kTileBlocks, ctr0, R, slab);
        return;
    }
    // the hint was wrong for this record: all of it here (empty or disordered offsets: nothing)
    if (p.in_off[rec + 1] < ioff) return;
    const uint64_t ntile = (Lr + kTileBytes - 1) / kTileBytes;
    for (uint64_t t = 0; t < ntile; ++t) {
        xor_tile(src, dst, Lr, (uint32_t)(t * kTileBlocks), ctr0, R, slab);
        __syncthreads();  // the slab is reused by the next tile
    }
}

// ---------------------------------------------------------------------------------- uniform AEAD
// RFC 8439 seal / open over a batch whose hints say every record is L >= ENET_SEG_MIN bytes: ONE
// launch (the three-launch path spent ~12 of its ~51 us per 32 MiB record in the plan and the
// record-engine pass, profiles/r06i_seg_probes.txt).  Workgroup t serves tile t % T of record
// t / T with four data waves and a fifth "power" wave:
//   * the power wave derives the record's one-time key (block 0) and r^(2^k), k <= 12, into LDS
//     (the data waves load and run their first keystream meanwhile, and wait at one barrier before
//     their first Poly1305 step); in the record's tile-0 workgroup it then goes on squaring --
//     r^(2^k) up to what the combine needs, and r^R for the last tile -- into the record's global
//     table, published before that workgroup's arrival;
//   * tiles publish their partial write-through and take an arrival ticket (as seg_kernel); the
//     last to arrive combines: Horner over q right-aligned tiles per lane in r^4096, a shuffle / LDS
//     tree whose level multipliers are table entries, then h = Q r^R + P_last;
//   * open: every tile stores its plaintext write-through (sc1) and drains it before arriving, so
//     the last arriver can zero a failed record itself (no later pass needed);
//   * the arrival counters are per-stream state, zero when the launch starts (capi.cpp) and reset
//     by each record's last arriver;
//   * a record whose real length differs from the hint is run whole by its tile-0 workgroup, tile
//     after tile, its partials combined in that workgroup (a wrong hint costs speed, never bytes).
// TPW tiles per workgroup (4 TPW data waves) + the power wave.  Past one tile per CU, two tiles
// per nine-wave workgroup (three waves of ~166 VGPRs per SIMD fit) keep a 32 MiB record's 512
// tiles resident at once; one tile per five-wave workgroup ran in two rounds there (a second such
// workgroup did not fit beside the first).  Up to one tile per CU, one tile per workgroup spreads
// the tiles over the most CUs.
#ifdef ENET_SEG_PROBE_TRACE
// timing probe: per-workgroup wall-clock stamps (100 MHz) at the phase boundaries, read back by
// tools/seg_trace.py through enet_probe_trace_read (hand-built libraries only)
__device__ uint64_t g_seg_trace[8192 * 8];
#define SEG_STAMP(k) (g_seg_trace[8ull * blockIdx.x + (k)] = wall_clock64())
#else
#define SEG_STAMP(k) ((void)0)
#endif
constexpr uint32_t kUPow = 44;                      // LDS table entries r^(2^k), k < 44
// Arrival counters per record: a top counter and kUGroups group counters, each on its own 128-byte
// line.  Tile t arrives at group t mod kUGroups; a group's last arriver arrives at the top counter.
// (One counter per record took all of a 32 MiB record's 512 arrivals at one address.)
#ifdef ENET_SEG_PROBE_GROUPS
constexpr uint32_t kUGroups = ENET_SEG_PROBE_GROUPS;  // timing probe
#else
constexpr uint32_t kUGroups = 16;
#endif
constexpr uint32_t kUArrStride = 32 * (1 + kUGroups);

typedef uint32_t enet_v4u __attribute__((ext_vector_type(4)));
// 16-byte write-through store (sc1): the line leaves this XCD's L2 for memory (MI355X_MICROARCH.md,
// inter-workgroup visibility).  asm stores are not in hipcc's vmcnt bookkeeping: the caller drains
// with s_waitcnt vmcnt(0) before publishing; s_nop 1 keeps the next instruction off the data VGPRs.
__device__ __forceinline__ void store_wt16(uint8_t* p, uint4 v) {
    enet_v4u w = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}

// Workgroup barrier for LDS hand-offs only: this wave's LDS operations retire, then s_barrier.
// __syncthreads() also drains the wave's outstanding global stores (vmcnt(0)): after a tile's
// stores that held every wave for their round trip at each barrier.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Sum of the first `nwaves` waves' accumulators into thread 0's l (the others contribute zero).
__device__ __forceinline__ void wg_sum5(uint32_t l[5], uint32_t* red /* [waves][5] shared */, uint32_t nwaves) {
#pragma unroll
    for (int off = 1; off <= 8; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0 && w < nwaves) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[5 * w + i] = l[i];
    }
    lds_barrier();
    if (threadIdx.x == 0) {
        for (uint32_t k = 1; k < nwaves; ++k) {
#pragma unroll
            for (int i = 0; i < 5; ++i) l[i] += red[5 * k + i];
            if ((k & 7u) == 7u) pcarry(l);
        }
        pcarry(l);
    }
    lds_barrier();
}

// Per-tile sums of the data waves' accumulators: the power wave's lane h gets tile h's sum (waves
// 4h..4h+3) -- the power wave stored no data, so its publishing waits for its own stores alone.
// pw (whole tiles): the r^(2^k) table; wave t of a tile is first scaled by r^(1024 (3 - t)) (lane
// j's run ends 16 (255 - j) blocks before the tile's end; the in-wave part of that scaling is the
// caller's).
template <int TPW>
__device__ __forceinline__ void wg_sum_tiles(uint32_t l[5], uint32_t* red /* [4 TPW][5] shared */, const uint32_t* pw) {
    constexpr uint32_t kUTiles = TPW, kUData = kSegThreads * TPW;
#pragma unroll
    for (int off = 1; off <= 8; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] += __shfl_xor(l[i], off);
    }
    pcarry(l);
    const uint32_t w = threadIdx.x >> 6, wt = w & 3u;
    const bool data = threadIdx.x < kUData;
    if (data && pw && wt < 3) pscale(l, (3u - wt) << 10, pw, 12u);  // wave-uniform
    if ((threadIdx.x & 63u) == 0 && data) {
#pragma unroll
        for (int i = 0; i < 5; ++i) red[5 * w + i] = l[i];
    }
    lds_barrier();
    const uint32_t h = threadIdx.x - kUData;  // the power wave's lane h < kUTiles takes tile h's sum
    if (!data && h < kUTiles) {
        const uint32_t b = 20 * h;
#pragma unroll
        for (int i = 0; i < 5; ++i) l[i] = red[b + i] + red[b + 5 + i] + red[b + 10 + i] + red[b + 15 + i];
        pcarry(l);
    }
}

template <int MODE, int TPW>
__global__ __launch_bounds__(kSegThreads * TPW + 64) void seg_uniform_aead_kernel(SegParams p, uint64_t Lh, uint32_t T,
                                                                                 uint32_t* __restrict__ arrivals) {
    constexpr uint32_t kUTiles = TPW;                    // tiles per workgroup
    constexpr uint32_t kUData = kSegThreads * kUTiles;  // data threads
    constexpr uint32_t kUThreads = kUData + 64;         // + the power wave
    __shared__ __attribute__((aligned(16))) uint8_t slab[kUData * kRun];
    __shared__ uint32_t red[(kUThreads / 64) * 5];
    __shared__ uint32_t pw_s[kUPow * 5];  // r^(2^k), 26-bit limbs
    __shared__ uint32_t t1_s[4 * 64 * 5];  // [m][i]: r^(16 i + 1024 m), a tile lane's scaling
    __shared__ uint32_t t2_s[4 * 64 * 5];  // [m][i]: r^(4096 q (i + 64 m)), the combine's lanes
    __shared__ uint32_t rr_s[5];          // r^R: the last tile's offset from tile nw-1's end
    __shared__ uint32_t ok_s[8];       // one-time key words: r (raw) then s
    __shared__ uint32_t last_flag;
    __shared__ uint32_t okr_s;  // main path: 1 once the power wave has put the one-time key in LDS
    const bool pwv = threadIdx.x >= kUData;
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    const uint32_t half = pwv ? 0u : threadIdx.x / kSegThreads;  // the workgroup's tile of this wave
    const uint32_t j = threadIdx.x & (kSegThreads - 1);         // data lane inside its tile
    const uint32_t wbase_t = wbase & (kSegThreads - 1);

    const uint32_t G = (T + kUTiles - 1) / kUTiles;  // workgroups per record
    const uint32_t rec = blockIdx.x / G, tr = blockIdx.x % G;
    if (threadIdx.x == 0) {
        last_flag = 0;  // read after the publish barrier
        okr_s = 0;
    }
    lds_barrier();  // the nine waves start together: this costs little and orders the resets
    if (threadIdx.x == 0) SEG_STAMP(0);
#ifdef ENET_SEG_PROBE_TRACE
    if (threadIdx.x == 0)  // where the workgroup runs: HW_ID (cu, sh, se) and XCC_ID
        g_seg_trace[8ull * blockIdx.x + 7] = ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) << 32) |
                                             (uint32_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
#endif
    const uint64_t ioff = p.in_off[rec], iend = p.in_off[rec + 1];
    // disordered offsets or an impossible length: handled as an empty record by the fallback
    const uint64_t L = (iend >= ioff && iend - ioff < kSegMaxLen) ? iend - ioff : 0;
    const bool as_hinted = iend >= ioff && L == Lh;
    if (!as_hinted && tr != 0) return;  // the record's tile-0 workgroup runs it whole
    const uint8_t* src = p.in + ioff;
    uint8_t* dst = p.out + p.out_off[rec];
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
    uint32_t aad_len = 0;
    uint64_t aoff = 0;
    if (p.aad) {
        aoff = p.aad_off[rec];
        aad_len = (uint32_t)(p.aad_off[rec + 1] - aoff);
    }
    const uint32_t na = (aad_len + 15) >> 4;
    const uint32_t nct = (uint32_t)((L + 15) >> 4);
    const uint32_t K = na + nct + 1;  // Poly1305 blocks
    const uint32_t nb = (uint32_t)((L + 63) >> 6);
    const uint32_t nt = as_hinted ? T : (L ? (uint32_t)((L + kTileBytes - 1) / kTileBytes) : 1u);
    // combine geometry (main path): q right-aligned tiles per lane, q a power of two
    const uint32_t nw_t = nt - 1;
    uint32_t lq = 0;
    while ((kSegThreads << lq) < nw_t) ++lq;
    const uint32_t top = max(13u, min(12 + lq + 8, kUPow));  // table entries the combine reads: k < top

    // ---- the power wave: the one-time key into LDS before barrier A; then (while the data waves
    // run the tile) the table r^(2^k), k < top, and r^R before barrier B
    if (pwv) {
        // the power wave's chain gates every tile (the key, then the table before barrier B); the
        // issue arbiter favours older waves, and this youngest wave shared its SIMD with two data
        // waves' keystream: without a raised priority each of its steps took ~1 us
        __builtin_amdgcn_s_setprio(3);
        uint32_t otk[16];
#ifdef ENET_SEG_PROBE_NO_OTK
        for (int i = 0; i < 16; ++i) otk[i] = R.k[i & 7];
#else
        chacha_block(R, 0u, otk);
#endif
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) ok_s[i] = otk[i];
        }
        __hip_atomic_store(&okr_s, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // The power wave's table, built while the data waves run their tile (main path: right after
    // the one-time key; barrier B publishes it).  Low (what a tile's own scaling reads): r^(2^k),
    // k <= 12, and in lane i r^(16 i), the product of r^(2^(4+b)) over the bits b of i.  High (read
    // only by the record's last arriver): r^(2^k), 13 <= k < top, and r^R.
    uint32_t px[5];  // the power wave's running square
    auto put = [&](uint32_t k) {
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < 5; ++i) pw_s[5 * k + i] = px[i];
        }
    };
    auto power_low = [&]() {
#ifdef ENET_SEG_PROBE_NO_TABLE
        return;
#endif
        pclamp(px, ok_s[0], ok_s[1], ok_s[2], ok_s[3]);
        // one chain at a time (few registers: this runs where the tile's key state is live).  The
        // power wave shares a SIMD with two data waves, so every step here is slow: only what a
        // tile's own scaling needs (k <= 11, and r^(16 i)) comes before barrier B
#pragma unroll 1
        for (uint32_t k = 0; k < 12; ++k) {
            put(k);
            psquare(px);
        }
        ENET_WAVE_LDS_SYNC();
        uint32_t y[5] = {1, 0, 0, 0, 0};
#pragma unroll 1
        for (uint32_t b = 0; b < 6; ++b) {
            uint32_t m[5];
            const bool on = (lane >> b) & 1u;
#pragma unroll
            for (int i = 0; i < 5; ++i) m[i] = on ? pw_s[5 * (4 + b) + i] : (i == 0 ? 1u : 0u);
            pmul_by(y, m);
        }
        // then times r^1024 per wave of the tile: entry [m][i] = r^(16 i + 1024 m)
#pragma unroll 1
        for (uint32_t m = 0; m < 4; ++m) {
#pragma unroll
            for (int i = 0; i < 5; ++i) t1_s[5 * (64 * m + lane) + i] = y[i];
            if (m < 3) pmul_by(y, pw_s + 5 * 10);
        }
    };
    auto power_high = [&]() {
#ifdef ENET_SEG_PROBE_NO_TABLE
        return;
#endif
        for (uint32_t k = 12; k < top; ++k) {
            put(k);
            psquare(px);
        }
        if (nw_t) {  // R = K - (na + 4096 nw) <= 4097
            uint32_t y[5] = {1, 0, 0, 0, 0};
            ENET_WAVE_LDS_SYNC();
            pscale(y, K - (na + kTilePoly * nw_t), pw_s, 13u);
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < 5; ++i) rr_s[i] = y[i];
            }
            // lane i: r^(4096 q i), q = 2^lq, from entries 12 + lq .. 12 + lq + 5
            uint32_t z[5] = {1, 0, 0, 0, 0};
#pragma unroll 1
            for (uint32_t b = 0; b < 6; ++b) {
                uint32_t m[5];
                const bool on = (lane >> b) & 1u;
#pragma unroll
                for (int i = 0; i < 5; ++i) m[i] = on ? pw_s[5 * (12 + lq + b) + i] : (i == 0 ? 1u : 0u);
                pmul_by(z, m);
            }
#pragma unroll 1
            for (uint32_t m = 0; m < 4; ++m) {  // times r^(4096 q 64) per wave
#pragma unroll
                for (int i = 0; i < 5; ++i) t2_s[5 * (64 * m + lane) + i] = z[i];
                if (m < 3) pmul_by(z, pw_s + 5 * (12 + lq + 6));
            }
        }
    };

    if (pwv && as_hinted) {  // while the data waves run their tiles
        power_low();
        power_high();
    }
    uint32_t hf[5] = {0, 0, 0, 0, 0};  // the record's Poly1305 sum (thread 0), normalised at K
    PolyR32 PR{};
    if (!as_hinted) {
        // fallback: the whole record here, tile after tile, per lane (lane j: blocks [tb0 + 4j, +4))
        __syncthreads();  // barrier A: r / s in LDS
        PR = polyr32_make(ok_s[0], ok_s[1], ok_s[2], ok_s[3]);
        if (pwv) {
            power_low();
            power_high();
        }
        uint32_t prev_end = 0;
        for (uint32_t v = 0; v < nt; ++v) {
            const uint32_t tb0 = v * kTileBlocks;
            const uint32_t tb1 = min(tb0 + kTileBlocks, nb);
            const uint32_t c0 = min(tb0 + kSegBPL * j, tb1), c1 = min(c0 + kSegBPL, tb1);
            uint32_t h[5] = {0, 0, 0, 0, 0};
            uint32_t l[5] = {0, 0, 0, 0, 0};
            const bool last_tile = tb1 == nb;
            const uint32_t tile_end = na + min(4u * tb1, nct) + (last_tile ? 1u : 0u);
            if (!pwv && half == 0) {
                if (v == 0 && j == 0) {
                    const uint8_t* ap = p.aad + aoff;
                    for (uint32_t s2 = 0; s2 < na; ++s2) {
                        const uint32_t cnt = min(16u, aad_len - 16u * s2);
                        uint32_t w[4];
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            uint32_t vv = 0;
#pragma unroll
                            for (int b2 = 0; b2 < 4; ++b2)
                                if ((uint32_t)(4 * i + b2) < cnt) vv |= (uint32_t)ap[16 * s2 + 4 * i + b2] << (8 * b2);
                            w[i] = vv;
                        }
                        poly32_block(h, PR, w[0], w[1], w[2], w[3], 1u);
                    }
                }
                for (uint32_t c = c0; c < c1; ++c) {
                    const uint64_t pos = 64ull * c;
                    const uint32_t nbytes = (uint32_t)min<uint64_t>(64, L - pos);
                    uint32_t w[16];
                    load_block(src + pos, nbytes, w, pos + nbytes >= 16);
                    uint32_t o[16];
                    chacha_block(R, 1u + c, o);
#pragma unroll
                    for (int i = 0; i < 16; ++i) o[i] ^= w[i];
                    store_block(dst + pos, nbytes, o);
                    uint32_t* ct = (MODE == MODE_SEAL) ? o : w;
                    if (MODE == MODE_SEAL && nbytes < 64) mask_tail(ct, nbytes);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (4 * c + u < nct)
                            poly32_block(h, PR, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
                }
                const bool has_last = (c1 == nb && c1 > c0) || (nb == 0 && j == 0);
                if (has_last) poly32_block(h, PR, aad_len, 0u, (uint32_t)L, (uint32_t)(L >> 32), 1u);
                h32_to_limbs(h, l);
            }
            if (v == 0) __syncthreads();  // barrier B: the table in LDS
            if (!pwv && half == 0) {
                const bool has_last = (c1 == nb && c1 > c0) || (nb == 0 && j == 0);
                const uint32_t lane_end = na + min(4u * c1, nct) + (has_last ? 1u : 0u);
                if (c1 > c0 || (v == 0 && j == 0)) pscale(l, tile_end - lane_end, pw_s, 13u);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wg_sum5(l, red, kSegThreads / 64);
            if (threadIdx.x == 0) {  // H = H r^(tile_end - prev_end) + P_v
                pscale(hf, tile_end - prev_end, pw_s, 13u);
#pragma unroll
                for (int i = 0; i < 5; ++i) hf[i] += l[i];
                pcarry(hf);
            }
            prev_end = tile_end;
        }
    } else {
        const uint32_t tt = kUTiles * tr + half;  // tile index inside the record (the power wave: the first)
        const bool tile_ok = tt < T;              // the record's last workgroup may hold one tile only
        const uint32_t tb0 = tt * kTileBlocks;
        const uint32_t tb1 = min(tb0 + kTileBlocks, nb);
        const uint32_t c0 = min(tb0 + kSegBPL * j, tb1), c1 = min(c0 + kSegBPL, tb1);
        // uniform over the tile's waves (an absent tile: the per-block path over no blocks)
        const bool whole = tile_ok && (uint64_t)(tb0 + kTileBlocks) * 64ull <= L;
        const bool first_iter = true;
        uint32_t h[5] = {0, 0, 0, 0, 0};
        auto barrier_a = [&]() {  // r / s in LDS: wait for the power wave's flag (no barrier)
            while (__hip_atomic_load(&okr_s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                __builtin_amdgcn_s_sleep(1);
            if (threadIdx.x == 0) SEG_STAMP(1);
            PR = polyr32_make(ok_s[0], ok_s[1], ok_s[2], ok_s[3]);
        };
        auto absorb_aad = [&]() {
            if (tt == 0 && j == 0 && !pwv) {
                const uint8_t* ap = p.aad + aoff;
                for (uint32_t s = 0; s < na; ++s) {
                    const uint32_t cnt = min(16u, aad_len - 16u * s);
                    uint32_t w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        uint32_t vv = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            if ((uint32_t)(4 * i + b) < cnt) vv |= (uint32_t)ap[16 * s + 4 * i + b] << (8 * b);
                        w[i] = vv;
                    }
                    poly32_block(h, PR, w[0], w[1], w[2], w[3], 1u);
                }
            }
        };
        if (whole) {
            const uint32_t kk = lane & 7u;
            const uint32_t msw = slab_sw(lane);
            uint8_t* wslab = slab + wbase * kRun;
            uint8_t* myrun = slab + threadIdx.x * kRun;
            const uint8_t* ib = src + 64ull * tb0;
            uint8_t* ob = dst + 64ull * tb0;
            const bool nt_ok = ((reinterpret_cast<uintptr_t>(ob)) & 63u) == 0;
            uint32_t offs[8];
            uint32_t pf[32];
            if (!pwv) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t o = 8u * i + (lane >> 3);
                    offs[i] = 64u * kSegBPL * (wbase_t + o) + 16u * (kk ^ slab_sw(o));
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint4 q = *reinterpret_cast<const uint4*>(ib + offs[i]);
                    pf[4 * i] = q.x; pf[4 * i + 1] = q.y; pf[4 * i + 2] = q.z; pf[4 * i + 3] = q.w;
                }
            }
#pragma unroll
            for (int st = 0; st < 2; ++st) {
                uint32_t w2[32], ka[16], kb[16];
                if (!pwv) {
                    // the keystream first: it needs no data, so it runs under the loads' latency
                    const uint32_t cb = 1u + c0 + 2u * st;  // RFC 8439 data counter from 1
                    chacha_block2(R, cb, cb + 1u, ka, kb);
                    ENET_WAVE_LDS_SYNC();
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                            make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
                    ENET_WAVE_LDS_SYNC();
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint4 q = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                        w2[4 * k] = q.x; w2[4 * k + 1] = q.y; w2[4 * k + 2] = q.z; w2[4 * k + 3] = q.w;
                    }
                    if (st == 0) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const uint4 q = *reinterpret_cast<const uint4*>(ib + offs[i] + kRun);
                            pf[4 * i] = q.x; pf[4 * i + 1] = q.y; pf[4 * i + 2] = q.z; pf[4 * i + 3] = q.w;
                        }
                        asm volatile("" : "+v"(R.k[0])::"memory");
                    }
                }
                if (st == 0 && first_iter) {
                    barrier_a();
                    absorb_aad();
                } else if (st == 0) {
                    PR = polyr32_make(ok_s[0], ok_s[1], ok_s[2], ok_s[3]);
                    absorb_aad();
                }
                if (!pwv) {
#ifndef ENET_SEG_PROBE_NO_POLY
                    if (MODE == MODE_OPEN) {
                        poly_block64(h, PR, w2);
                        poly_block64(h, PR, w2 + 16);
                    }
#endif
#pragma unroll
                    for (int i = 0; i < 16; ++i) { w2[i] ^= ka[i]; w2[16 + i] ^= kb[i]; }
#ifndef ENET_SEG_PROBE_NO_POLY
                    if (MODE == MODE_SEAL) {
                        poly_block64(h, PR, w2);
                        poly_block64(h, PR, w2 + 16);
                    }
#else
                    h[0] ^= w2[0];
#endif
                    ENET_WAVE_LDS_SYNC();
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        *reinterpret_cast<uint4*>(myrun + 16u * (k ^ msw)) =
                            make_uint4(w2[4 * k], w2[4 * k + 1], w2[4 * k + 2], w2[4 * k + 3]);
                    ENET_WAVE_LDS_SYNC();
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint4 q = *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
                        if (MODE == MODE_OPEN) store_wt16(ob + offs[i] + kRun * st, q);
                        else store_stream(ob + offs[i] + kRun * st, q, nt_ok);
                    }
                }
            }
        } else {
            if (first_iter) barrier_a();
            else PR = polyr32_make(ok_s[0], ok_s[1], ok_s[2], ok_s[3]);
            absorb_aad();
            if (!pwv) {
                for (uint32_t c = c0; c < c1; ++c) {
                    const uint64_t pos = 64ull * c;
                    const uint32_t nbytes = (uint32_t)min<uint64_t>(64, L - pos);
                    uint32_t w[16];
                    load_block(src + pos, nbytes, w, pos + nbytes >= 16);
                    uint32_t o[16];
                    chacha_block(R, 1u + c, o);
#pragma unroll
                    for (int i = 0; i < 16; ++i) o[i] ^= w[i];
                    if (MODE == MODE_OPEN && nbytes == 64) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            store_wt16(dst + pos + 16 * q, make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]));
                    } else if (MODE == MODE_OPEN) {
                        // the record's last partial block, write-through byte by byte (a failed
                        // record is zeroed by another workgroup, whose stores must land last)
                        for (uint32_t b = 0; b < nbytes; ++b)
                            __hip_atomic_store(dst + pos + b, (uint8_t)(o[b >> 2] >> (8 * (b & 3))), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        store_block(dst + pos, nbytes, o);
                    }
                    uint32_t* ct = (MODE == MODE_SEAL) ? o : w;
                    if (MODE == MODE_SEAL && nbytes < 64) mask_tail(ct, nbytes);
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (4 * c + u < nct)
                            poly32_block(h, PR, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
                }
            }
        }

        // this tile's partial, normalised at the tile's end
        uint32_t l[5] = {0, 0, 0, 0, 0};
        const bool last_tile = tb1 == nb;
        const uint32_t tile_end = na + min(4u * tb1, nct) + (last_tile ? 1u : 0u);
        const bool has_last = (c1 == nb && c1 > c0) || (nb == 0 && j == 0);
        if (!pwv) {
            if (has_last) poly32_block(h, PR, aad_len, 0u, (uint32_t)L, (uint32_t)(L >> 32), 1u);
            h32_to_limbs(h, l);
        }
#ifdef ENET_SEG_PROBE_NO_PUBLISH
        if (h[0] == 0x12345u) p.ok[rec] = 7;  // keep the Horner live
        return;
#endif
        // the power wave skipped the tile's body: it builds the table here, where no tile data
        // is live (inside the body its registers would count against every wave)
        if (threadIdx.x == 0) SEG_STAMP(2);
        if (threadIdx.x == kUData) SEG_STAMP(3);
#ifndef ENET_SEG_PROBE_NO_SYNC
        lds_barrier();  // barrier B: the table's low part in LDS
#endif
        if (threadIdx.x == 0) SEG_STAMP(4);

#ifndef ENET_SEG_PROBE_NO_SCALE
        if (!pwv) {
            const uint32_t lane_end = na + min(4u * c1, nct) + (has_last ? 1u : 0u);
            const uint32_t e = tile_end - lane_end;
            if (whole) {
                // e = 16 (255 - j) (+1 in the record's last tile for lanes before the length
                // block) = 16 (63 - lane) + 1024 (3 - wave of the tile): one table entry
                uint32_t m[5];
                const uint32_t wt = (threadIdx.x >> 6) & 3u;
#pragma unroll
                for (int i = 0; i < 5; ++i) m[i] = t1_s[5 * (64 * (3u - wt) + 63u - lane) + i];
                pmul_by(l, m);
                if (e != 16u * (255u - j)) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) m[i] = pw_s[i];
                    pmul_by(l, m);
                }
            } else if (c1 > c0 || (tt == 0 && j == 0)) {
                pscale(l, e, pw_s, 13u);
            }
        }
#endif
        // open: every wave drains its write-through plaintext before the arrival (the last arriver
        // may zero the record)
        if (MODE == MODE_OPEN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wg_sum_tiles<TPW>(l, red, nullptr);  // whole tiles: the wave factor is in the lane's entry
        // main path: each tile publishes (the power wave's lane h for tile h), takes a ticket; the
        // record's last tile to arrive finishes it
        uint32_t* ctr = arrivals + (size_t)kUArrStride * rec;  // [0] top, [32 (1 + g)] group g
        const uint32_t tp = kUTiles * tr + lane;  // the power wave lane's tile
        if (pwv && lane < kUTiles && tp < T) {
            uint32_t* part = p.partials + 8ull * ((size_t)rec * T + tp);
#pragma unroll
            for (int i = 0; i < 5; ++i) __hip_atomic_store(part + i, l[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef ENET_SEG_PROBE_ONECTR
            uint32_t lf = 0;
            if (lane == 0) {  // one add per workgroup at one counter per record
                const uint32_t nw = min(kUTiles, T - kUTiles * tr);
                lf = __hip_atomic_fetch_add(ctr, nw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + nw == T ? 1u : 0u;
            }
#else
            const uint32_t ng = min(T, kUGroups), g = tp % ng, members = (T - g + ng - 1) / ng;
            uint32_t* gc = ctr + 32 * (1 + g);
            const uint32_t prev = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t lf = 0;
            if (prev + 1 == members) {  // the group is complete: reset it, arrive at the top
                __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t top_prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lf = top_prev + 1 == ng ? 1u : 0u;
            }
#endif
            if (lf) last_flag = 1u;
            if (lane == 0) SEG_STAMP(5);
        }
        lds_barrier();
#ifdef ENET_SEG_PROBE_NO_TAIL
        if (threadIdx.x == 0 && last_flag) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
#endif
        if (!last_flag) return;  // uniform over the workgroup
        if (threadIdx.x >= kSegThreads) return;  // the combine runs on the first tile's four waves
        const uint32_t* parts = p.partials + 8ull * ((size_t)rec * T);
        uint32_t vl[5] = {0, 0, 0, 0, 0};  // the last tile's partial, normalised at K: loaded first
        if (threadIdx.x == 0) {
#pragma unroll
            for (int i = 0; i < 5; ++i) vl[i] = __hip_atomic_load(parts + 8ull * (T - 1) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        auto pw_at = [&](uint32_t k, uint32_t out[5]) {  // r^(2^k) from this workgroup's table
#pragma unroll
            for (int i = 0; i < 5; ++i) out[i] = pw_s[5 * k + i];
        };
        uint32_t acc[5] = {0, 0, 0, 0, 0};
        if (nw_t) {
            if (!pwv) {
                const uint32_t q = 1u << lq;
                const int64_t hi = (int64_t)nw_t - (int64_t)q * (kSegThreads - 1 - j);
                const int64_t lo = max<int64_t>(0, hi - (int64_t)q);
                uint32_t m[5];
                pw_at(12, m);
                const Pmul M4 = pmul_make(m);
                uint32_t nx[5] = {0, 0, 0, 0, 0};
                if (lo < hi) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) nx[i] = __hip_atomic_load(parts + 8 * lo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                for (int64_t t = lo; t < hi; ++t) {
                    uint32_t cur[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) cur[i] = nx[i];
                    if (t + 1 < hi) {  // the next partial's load flies under this step
#pragma unroll
                        for (int i = 0; i < 5; ++i)
                            nx[i] = __hip_atomic_load(parts + 8 * (t + 1) + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (t > lo) pmul(acc, M4);
#pragma unroll
                    for (int i = 0; i < 5; ++i) acc[i] += cur[i];
                    pcarry(acc);
                }
                // lane l of wave w: its tiles end 63 - l + 64 (3 - w) lane-runs of q tiles before
                // the last lane's: r^(4096 q (63 - l + 64 (3 - w))), one entry of the power wave's
                // table; then plain sums
                const uint32_t w = threadIdx.x >> 6;
                {
                    uint32_t mm[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) mm[i] = t2_s[5 * (64 * (3u - w) + 63u - lane) + i];
                    pmul_by(acc, mm);
                }
#pragma unroll
                for (int off = 1; off <= 8; off <<= 1) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) acc[i] += __shfl_xor(acc[i], off);
                }
                pcarry(acc);
#pragma unroll
                for (int off = 16; off <= 32; off <<= 1) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) acc[i] += __shfl_xor(acc[i], off);
                }
                pcarry(acc);
                if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) red[5 * w + i] = acc[i];
                }
            }
            lds_barrier();
            if (threadIdx.x == 0) {
                uint32_t rr[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    acc[i] = red[i] + red[5 + i] + red[10 + i] + red[15 + i];
                    rr[i] = rr_s[i];
                }
                pcarry(acc);
                pmul_by(acc, rr);
            }
        }
        if (threadIdx.x == 0) {
#pragma unroll
            for (int i = 0; i < 5; ++i) hf[i] = acc[i] + vl[i];
            pcarry(hf);
            __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
        }
    }
    // tag / verdict; a failed open's plaintext is zeroed here (every tile's stores were
    // write-through and drained before its arrival; the fallback's are this workgroup's own)
    if (threadIdx.x == 0) SEG_STAMP(6);
    if (threadIdx.x == 0) {
        uint32_t tag[4];
        pfinish(hf, ok_s + 4, tag);
        if (MODE == MODE_SEAL) {
            uint32_t* tp = reinterpret_cast<uint32_t*>(p.tag_out + 16ull * rec);
            tp[0] = tag[0]; tp[1] = tag[1]; tp[2] = tag[2]; tp[3] = tag[3];
        } else {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(p.tag_in + 16ull * rec);
            const uint32_t diff = (tag[0] ^ tp[0]) | (tag[1] ^ tp[1]) | (tag[2] ^ tp[2]) | (tag[3] ^ tp[3]);
            p.ok[rec] = diff == 0 ? 1 : 0;
            last_flag = diff == 0 ? 0u : 1u;  // reused: 1 = zero the record
        }
    }
#if defined(ENET_SEG_PROBE_NO_POLY) || defined(ENET_SEG_PROBE_NO_TABLE)
    if (MODE == MODE_OPEN) return;  // timing probes: wrong tags, nothing to zero
#endif
    if (MODE == MODE_OPEN) {
        __syncthreads();
        const uint32_t zt = as_hinted ? kSegThreads : kUThreads;  // the main path's combine: 4 waves
        if (last_flag && threadIdx.x < zt) {
            for (uint64_t b = 16ull * threadIdx.x; b < L; b += 16ull * zt) {
                const uint32_t nbytes = (uint32_t)min<uint64_t>(16, L - b);
                if (nbytes == 16 && ((reinterpret_cast<uintptr_t>(dst + b)) & 15u) == 0)
                    *reinterpret_cast<uint4*>(dst + b) = make_uint4(0u, 0u, 0u, 0u);
                else
                    for (uint32_t t = 0; t < nbytes; ++t) dst[b + t] = 0;
            }
        }
    }
}

// dst[width * list[k] ..] = src[width * k ..] for k < m (results computed on the host for a subset
// of the batch, e.g. the host-hashed digests of long chunks, capi.cpp)
__global__ void scatter_kernel(const uint8_t* __restrict__ src, const uint32_t* __restrict__ list, uint32_t m,
                               uint8_t* __restrict__ dst, uint32_t width) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)m * width) return;
    const uint32_t k = (uint32_t)(t / width), b = (uint32_t)(t % width);
    dst[(uint64_t)width * list[k] + b] = src[t];
}

hipError_t launch_scatter(const uint8_t* src, const uint32_t* list, uint32_t m, uint8_t* dst, uint32_t width,
                          hipStream_t s) {
    const uint64_t total = (uint64_t)m * width;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_kernel, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, src, list, m, dst, width);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------- host side
uint32_t seg_uniform_arrival_words() { return kUArrStride; }

#ifdef ENET_SEG_PROBE_TRACE
extern "C" __attribute__((visibility("default"))) int enet_probe_trace_read(uint64_t* out, size_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_seg_trace), 8 * std::min<size_t>(n, 8192 * 8)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_seg_uniform_aead(const SegParams& p, uint64_t L, uint32_t* arrivals, hipStream_t s) {
    const uint64_t T = (L + kTileBytes - 1) / kTileBytes;
    if ((uint64_t)p.n * T == 0) return hipSuccess;
    if (T > 0xFFFFFFFFull) return hipErrorInvalidValue;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const bool two = (uint64_t)p.n * T > (uint64_t)(cus > 0 ? cus : 256);  // tiles per workgroup
    const uint64_t blocks = (uint64_t)p.n * (two ? (T + 1) / 2 : T);
    if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    const dim3 g((uint32_t)blocks), b1(kSegThreads + 64), b2(2 * kSegThreads + 64);
    switch (p.mode) {
        case MODE_SEAL:
            if (two) hipLaunchKernelGGL((seg_uniform_aead_kernel<MODE_SEAL, 2>), g, b2, 0, s, p, L, (uint32_t)T, arrivals);
            else hipLaunchKernelGGL((seg_uniform_aead_kernel<MODE_SEAL, 1>), g, b1, 0, s, p, L, (uint32_t)T, arrivals);
            break;
        case MODE_OPEN:
            if (two) hipLaunchKernelGGL((seg_uniform_aead_kernel<MODE_OPEN, 2>), g, b2, 0, s, p, L, (uint32_t)T, arrivals);
            else hipLaunchKernelGGL((seg_uniform_aead_kernel<MODE_OPEN, 1>), g, b1, 0, s, p, L, (uint32_t)T, arrivals);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_seg_uniform_xor(const SegParams& p, uint64_t L, hipStream_t s) {
    const uint64_t T = (L + kTileBytes - 1) / kTileBytes;
    const uint64_t blocks = (uint64_t)p.n * T;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7FFFFFFFull || T > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(seg_uniform_xor_kernel, dim3((uint32_t)blocks), dim3(kSegThreads), 0, s, p, L, (uint32_t)T);
    return hipGetLastError();
}

hipError_t launch_seg(const SegParams& p, uint32_t plan_blocks, uint32_t tile_blocks, hipStream_t s) {
    if (plan_blocks > 1) {
        if (hipError_t e = hipMemsetAsync(p.hdr, 0, sizeof(unsigned long long), s)) return e;
    }
    hipLaunchKernelGGL(seg_plan_kernel, dim3(plan_blocks), dim3(kSegThreads), 0, s, p);
    switch (p.mode) {
        case MODE_XOR: hipLaunchKernelGGL(seg_kernel<MODE_XOR>, dim3(tile_blocks), dim3(kSegThreads), 0, s, p); break;
        case MODE_SEAL: hipLaunchKernelGGL(seg_kernel<MODE_SEAL>, dim3(tile_blocks), dim3(kSegThreads), 0, s, p); break;
        case MODE_OPEN: hipLaunchKernelGGL(seg_kernel<MODE_OPEN>, dim3(tile_blocks), dim3(kSegThreads), 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace enet
