// duplex_split.hip -- the duplex pass (cipher + hash, one HBM pass) for LONG records, with the
// per-record work split over four waves so that a record's serial chain is shorter (gfx950).
//
// Why: in duplex.hip a record has one cipher lane and one hash lane; SHA-256 is serial inside a
// record, so a workgroup lasts as long as its longest record's chain: per 128-byte stage one
// wave runs two SHA-256 compressions (~2 750 VALU instructions, schedule + rounds) while the other
// runs two ChaCha20 blocks + Poly1305 (~2 330), and a lone wave issues one VALU instruction per
// ~4.5 cycles.  A 64 KiB record is 512 stages: 2.63 ms measured (tools/c5_overlap_probe.py) --
// the whole time of a C5 batch (BASELINE config 5: mixed 512 B-64 KiB, VALU busy 31 %) and of a
// 64 KiB chunk store.  Here lane l of four waves serves record l of the workgroup:
//   C0, C1 (waves 0, 1)  ChaCha20, one 64-byte block of the stage each: load, keystream, store;
//               they hand the ciphertext (seal) or the plaintext (open) of each stage to S
//               through an LDS run slab;
//   S (wave 2)  the SHA-256 message schedule W[0..63] of the stage's two blocks (plaintext: seal
//               re-loads the input run, an L2 hit; open takes C's output) into an LDS W slab, and
//               Poly1305 over the ciphertext (AEAD; seal from C's slab, open re-loads the input);
//   R (wave 3)  the 64 SHA-256 rounds per block over the W slab, and the digest / HMAC finish.
// Stage u is ciphered in interval u, scheduled in u + 1 and hashed in u + 2 (one workgroup
// barrier per interval); VALU instructions per stage: C0 / C1 ~1 000 each, S ~1 350 (AEAD),
// R 1 808 (14 per round, the floor), so R is the chain: 64 KiB in 1.90 ms.  (Three waves, one C
// for both blocks at ~1 960, measured the same chain: R bound it already.  The fourth wave raised
// the throughput around it: C5 device-resident 170 -> 192 GiB/s.)
// The ragged end (< 128 bytes) follows the same three steps: C encrypts and stores the tail, S
// finishes Poly1305 (tag) and lays out the padded final SHA-256 blocks (message tail, 0x80,
// BE64 bit length: 1-3 blocks), R compresses them, finishes HMAC (opad) and writes the digest /
// MAC -- or, opening, compares tag and MAC and zeroes a failed record's plaintext.
//
// Kinds (as duplex.hip): DK_CHUNK (ChaCha20 from LE32(chunk_id) + SHA-256(m): Node::store_chunk /
// fetch_chunk, Node.cpp:1414-1417, 1644-1655, CryptoManager.cpp:8-13) and DK_AEADH (RFC 8439
// seal/open + HMAC-SHA256_K(m), HmacSha256.cpp:11-39).  Frames keep duplex.hip (their MAC sits
// inside the ciphertext).  A record whose output length differs from its input is not
// processed: output zeroed, ok = 0.
#include "enet_device.hpp"
#include "enet_internal.hpp"

namespace enet {

namespace {

constexpr uint32_t kSRun = 128;  // bytes per stage and record
constexpr uint32_t kSRec = 64;   // records per workgroup (one lane each in 4 waves)
constexpr uint32_t kSWaves = 4;  // C0, C1, S, R

#define ENET_SP_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

__device__ __forceinline__ void sp_keep_le(uint32_t* w, int n, uint32_t r) {
    for (int j = 0; j < n; ++j) {
        const uint32_t b = 4u * j;
        const uint32_t m = b + 4u <= r ? 0xffffffffu : (b >= r ? 0u : (1u << (8u * (r - b))) - 1u);
        w[j] &= m;
    }
}

__device__ __forceinline__ void sp_zero_bytes(uint8_t* p, uint64_t n) {
    const uint32_t z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint64_t o = 0; o < n; o += 64) store_block(p + o, (uint32_t)min<uint64_t>(64, n - o), z);
}

// W[16..63] from W[0..15] (Sha256.cpp:134-150)
__device__ __forceinline__ void sha256_expand(uint32_t w[64]) {
#pragma unroll
    for (int i = 16; i < 64; ++i) {
        const uint32_t s0 = xor3(rotr(w[i - 15], 7), rotr(w[i - 15], 18), w[i - 15] >> 3);
        const uint32_t s1 = xor3(rotr(w[i - 2], 17), rotr(w[i - 2], 19), w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
}

// one SHA-256 round (Sha256.cpp:152-170) with the schedule word given
__device__ __forceinline__ void sha256_round(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                             uint32_t& f, uint32_t& g, uint32_t& h, uint32_t kw) {
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
    const uint32_t t1 = h + S1 + ch + kw;
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
}

}  // namespace

template <int KIND, bool OPEN>
__global__ __launch_bounds__(kSWaves * kSRec) void duplex_split_kernel(DuplexParams p) {
    constexpr bool kAead = KIND == DK_AEADH;
    // LDS (conflict-free: chunk-major, one 16-byte chunk per record per row, so a wave's
    // ds_read/write_b128 of chunk c touches 1 KiB contiguous)
    //   run slab [2][8 chunks][64 records]      C -> S: ciphertext (AEAD seal) / plaintext (open)
    //   W slab   [2][32 chunks][64 records]     S -> R: W[0..63] of the stage's two blocks
    // 80 KiB exactly, so two workgroups share a CU (160 KiB): the longest-stage count and the
    // open verdict of Poly1305 ride in run-slab words nobody else reads at that moment
    __shared__ __attribute__((aligned(16))) uint4 runs[2][8][kSRec];
    __shared__ __attribute__((aligned(16))) uint4 wsl[2][32][kSRec];
    uint32_t& tmax_s = runs[0][0][0].x;

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t pos = blockIdx.x * kSRec + lane;
    const bool live = pos < p.n;
    const uint32_t rec = live ? (p.order ? p.order[pos] : pos) : 0u;

    // ---- geometry (every role computes it)
    uint64_t ib = 0, Li = 0, ob = 0, Lo = 0;
    bool ordered = true;
    if (live) {
        ib = p.in_off[rec];
        const uint64_t ie = p.in_off[rec + 1];
        ob = p.out_off[rec];
        const uint64_t oe = p.out_off[rec + 1];
        ordered = ie >= ib && oe >= ob;
        Li = ordered ? ie - ib : 0u;
        Lo = ordered ? oe - ob : 0u;
    }
    const bool valid = live && ordered && Lo == Li;
    const uint64_t Lm = valid ? Li : 0u;
    const uint32_t Ts = (uint32_t)(Lm / kSRun);
    const uint32_t r = (uint32_t)(Lm - (uint64_t)kSRun * Ts);
    const uint64_t tb = (uint64_t)kSRun * Ts;
    const uint8_t* src = p.in + ib;
    uint8_t* dst = p.out + ob;

    if (threadIdx.x == 0) tmax_s = 0;
    __syncthreads();
    if (wave == 0 && valid) atomicMax(&tmax_s, Ts);
    __syncthreads();
    const uint32_t Tmax = __builtin_amdgcn_readfirstlane(tmax_s);
    __syncthreads();  // every wave has read it before C reuses the slab
    const uint32_t nint = Tmax + 3;  // intervals: stage u ciphered at u, scheduled at u+1, hashed at u+2

    uint32_t kw[8];
    {
        const uint8_t* kp = p.keys + (size_t)p.key_stride * rec;
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = live ? reinterpret_cast<const uint32_t*>(kp)[i] : 0u;
    }

    if (wave < 2) {
        // ================================================================ C0 / C1: ChaCha20
        // wave hb owns block hb of every stage: bytes [128 t + 64 hb, 128 t + 64 hb + 64)
        const uint32_t hb = wave;
        uint32_t nw[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = live ? ld32(p.nonces + 12ull * rec + 4 * i) : 0u;
        ChachaRecord R;
        chacha_record_init(R, kw, nw);
        const uint32_t c0 = (KIND == DK_CHUNK ? (live ? ld32(p.chunk_ids + 32ull * rec) : 0u) : 1u) + hb;
        const uint8_t* hsrc = src + 64u * hb;
        uint8_t* hdst = dst + 64u * hb;
        uint32_t pf[16];
        auto load_blk = [&](uint32_t s) {
            const uint4* q = reinterpret_cast<const uint4*>(hsrc + (uint64_t)kSRun * s);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint4 v = q[i];
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            }
        };
        // the slab carries what S cannot re-load from the input: seal ciphertext (AEAD only:
        // Poly1305 runs over it), open plaintext (the hash input)
        constexpr bool kHand = OPEN || kAead;
        if (Ts > 0) load_blk(0);
        for (uint32_t t = 0; t < nint; ++t) {
            if (t < Ts) {
                uint32_t x[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = pf[i];
                if (t + 1 < Ts) load_blk(t + 1);
                {
                    uint32_t ka[16];
                    chacha_block(R, c0 + 2u * t, ka);
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] ^= ka[i];
                }
                uint4* o = reinterpret_cast<uint4*>(hdst + (uint64_t)kSRun * t);
#pragma unroll
                for (int i = 0; i < 4; ++i) o[i] = make_uint4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
                if (kHand) {
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        runs[t & 1u][4 * hb + c][lane] = make_uint4(x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]);
                }
            } else if (t == Ts && valid) {
                // ragged end: r < 128 bytes; this wave's part is [64 hb, min(r, 64 hb + 64)), read
                // through 16-byte windows ending at the record end
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = 0u;
                const uint32_t rh = r > 64u * hb ? min(r - 64u * hb, 64u) : 0u;
                if (rh) {
                    load_block(hsrc + tb, rh, w, tb + 64u * hb + rh >= 16u);
                    uint32_t ka[16];
                    chacha_block(R, c0 + 2u * Ts, ka);
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] ^= ka[i];
                    store_block(hdst + tb, rh, w);
                    sp_keep_le(w, 16, rh);  // RFC 8439 zero pad / clean hash input
                }
                if (kHand) {
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        runs[Ts & 1u][4 * hb + c][lane] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
                }
            }
            // a failed open is zeroed by R two intervals later: this wave's stores must be done
            // (only in intervals where one of its records ended)
            if (OPEN && __builtin_amdgcn_ballot_w64(t == Ts && valid)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ENET_SP_BARRIER();
        }
    } else if (wave == 2) {
        // ================================================================ S: schedule + Poly1305
        PolyR32 PR{};
        uint32_t h[5] = {0, 0, 0, 0, 0}, pad[4] = {0, 0, 0, 0};
        if (kAead) {
            uint32_t nw[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = live ? ld32(p.nonces + 12ull * rec + 4 * i) : 0u;
            ChachaRecord R;
            chacha_record_init(R, kw, nw);
            uint32_t otk[16];
            chacha_block(R, 0u, otk);  // one-time key = keystream block 0 (RFC 8439 2.6)
            PR = polyr32_make(otk[0], otk[1], otk[2], otk[3]);
            pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        }
        auto poly_words = [&](const uint32_t* w, uint32_t blocks) {
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q)
                if (q < blocks) poly32_block(h, PR, w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], 1u);
        };
        auto global_run = [&](uint32_t s, uint32_t* x) {
            const uint4* q = reinterpret_cast<const uint4*>(src + (uint64_t)kSRun * s);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = q[i];
                x[4 * i] = v.x; x[4 * i + 1] = v.y; x[4 * i + 2] = v.z; x[4 * i + 3] = v.w;
            }
        };
        auto slab_run = [&](uint32_t s, uint32_t* x) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint4 v = runs[s & 1u][c][lane];
                x[4 * c] = v.x; x[4 * c + 1] = v.y; x[4 * c + 2] = v.z; x[4 * c + 3] = v.w;
            }
        };
        for (uint32_t t = 0; t < nint; ++t) {
            if (t >= 1 && t <= Ts) {
                const uint32_t u = t - 1;
                uint32_t pt[32];
                if (kAead) {
                    uint32_t ct[32];
                    if (OPEN) global_run(u, ct);  // the input is the ciphertext
                    else slab_run(u, ct);         // C's output
                    poly_words(ct, 8);
                }
                if (OPEN) slab_run(u, pt);  // C's output is the plaintext
                else global_run(u, pt);     // the input is the plaintext (an L2 hit: C just read it)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    uint32_t w[64];
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = bswap32(pt[16 * b + i]);
                    sha256_expand(w);
#pragma unroll
                    for (int c = 0; c < 16; ++c)
                        wsl[u & 1u][16 * b + c][lane] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
                }
            } else if (t == Ts + 1 && valid) {
                // tail: Poly1305 finish, and the padded final SHA-256 blocks as raw W[0..15]
                uint32_t pt[32], ct[32];
                if (OPEN || kAead) slab_run(Ts, OPEN ? pt : ct);  // C parked its tail there (masked)
                if (r && !OPEN) {  // seal: plaintext tail from the input
#pragma unroll
                    for (int i = 0; i < 32; ++i) pt[i] = 0u;
                    load_block(src + tb, min(r, 64u), pt, tb + min(r, 64u) >= 16u);
                    if (r > 64u) load_block(src + tb + 64, r - 64u, pt + 16, tb + r >= 16u);
                } else if (!OPEN) {
#pragma unroll
                    for (int i = 0; i < 32; ++i) pt[i] = 0u;
                }
                if (kAead) {
                    if (OPEN) {  // ciphertext tail from the input (masked)
#pragma unroll
                        for (int i = 0; i < 32; ++i) ct[i] = 0u;
                        if (r) {
                            load_block(src + tb, min(r, 64u), ct, tb + min(r, 64u) >= 16u);
                            if (r > 64u) load_block(src + tb + 64, r - 64u, ct + 16, tb + r >= 16u);
                        }
                    }
                    poly_words(ct, (r + 15u) >> 4);
                    poly32_block(h, PR, 0u, 0u, (uint32_t)Lm, (uint32_t)(Lm >> 32), 1u);  // LE64 |aad| = 0, LE64 |ct|
                    uint32_t l[5], tag[4];
                    h32_to_limbs(h, l);
                    pfinish(l, pad, tag);
                    if (OPEN) {  // verdict for R: this record's run-slab row of the other parity is free now
                        const uint8_t* tp = p.tags_in + 16ull * rec;
                        runs[(Ts + 1u) & 1u][0][lane].x = ((tag[0] ^ ld32(tp)) | (tag[1] ^ ld32(tp + 4)) |
                                                            (tag[2] ^ ld32(tp + 8)) | (tag[3] ^ ld32(tp + 12))) == 0u;
                    } else {
                        *reinterpret_cast<uint4*>(p.tags + 16ull * rec) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
                    }
                }
                // message tail, 0x80, zeros, BE64 bit length of [ipad ||] m (Sha256.cpp:94-126)
                const uint64_t bits = ((kAead ? 64ull : 0ull) + Lm) * 8ull;
                const uint32_t nb = (r + 9u + 63u) >> 6;  // 1..3 blocks
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    uint32_t x[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t b = 64u * k + 4u * i;
                        const uint32_t v = k < 2 ? bswap32(pt[16 * k + i]) : 0u;
                        const uint32_t m = b + 4u <= r ? 0xffffffffu : (b >= r ? 0u : 0xffffffffu << (8u * (4u - (r - b))));
                        x[i] = (v & m) | ((r >> 2) == (b >> 2) ? 0x80000000u >> (8u * (r & 3u)) : 0u);
                    }
                    if ((uint32_t)k == nb - 1u) {
                        x[14] = (uint32_t)(bits >> 32);
                        x[15] = (uint32_t)bits;
                    }
                    if ((uint32_t)k < nb) {
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            wsl[Ts & 1u][4 * k + c][lane] = make_uint4(x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]);
                    }
                }
            }
            ENET_SP_BARRIER();
        }
    } else {
        // ================================================================ R: rounds + finish
        uint32_t kb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kb[i] = bswap32(kw[i]);
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
        if (kAead) {  // HMAC inner: the ipad block first (HmacSha256.cpp:24-29)
            uint32_t x[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = (i < 8 ? kb[i] : 0u) ^ 0x36363636u;
            sha256_compress(st, x);
        }
        for (uint32_t t = 0; t < nint; ++t) {
            if (t >= 2 && t <= Ts + 1) {
                const uint32_t u = t - 2;
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    uint32_t a0 = st[0], a1 = st[1], a2 = st[2], a3 = st[3], a4 = st[4], a5 = st[5],
                             a6 = st[6], a7 = st[7];
#pragma unroll
                    for (int c = 0; c < 16; ++c) {
                        const uint4 v = wsl[u & 1u][16 * b + c][lane];
                        sha256_round(a0, a1, a2, a3, a4, a5, a6, a7, kSha256K[4 * c] + v.x);
                        sha256_round(a0, a1, a2, a3, a4, a5, a6, a7, kSha256K[4 * c + 1] + v.y);
                        sha256_round(a0, a1, a2, a3, a4, a5, a6, a7, kSha256K[4 * c + 2] + v.z);
                        sha256_round(a0, a1, a2, a3, a4, a5, a6, a7, kSha256K[4 * c + 3] + v.w);
                    }
                    st[0] += a0; st[1] += a1; st[2] += a2; st[3] += a3;
                    st[4] += a4; st[5] += a5; st[6] += a6; st[7] += a7;
                }
            } else if (t == Ts + 2 && live) {
                uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // digest as LE words of its bytes
                if (valid) {
                    const uint32_t nb = (r + 9u + 63u) >> 6;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        if ((uint32_t)k < nb) {
                            uint32_t x[16];
#pragma unroll
                            for (int c = 0; c < 4; ++c) {
                                const uint4 v = wsl[Ts & 1u][4 * k + c][lane];
                                x[4 * c] = v.x; x[4 * c + 1] = v.y; x[4 * c + 2] = v.z; x[4 * c + 3] = v.w;
                            }
                            sha256_compress(st, x);
                        }
                    }
                    if (kAead) {  // HMAC outer (HmacSha256.cpp:31-38)
                        uint32_t inner[8], x[16];
#pragma unroll
                        for (int i = 0; i < 8; ++i) inner[i] = st[i];
#pragma unroll
                        for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
#pragma unroll
                        for (int i = 0; i < 16; ++i) x[i] = (i < 8 ? kb[i] : 0u) ^ 0x5c5c5c5cu;
                        sha256_compress(st, x);
#pragma unroll
                        for (int i = 0; i < 8; ++i) x[i] = inner[i];
                        x[8] = 0x80000000u;
#pragma unroll
                        for (int i = 9; i < 15; ++i) x[i] = 0u;
                        x[15] = (64 + 32) * 8;
                        sha256_compress(st, x);
                    }
#pragma unroll
                    for (int i = 0; i < 8; ++i) d[i] = bswap32(st[i]);
                }
                if (!OPEN) {
                    if (valid) {
                        uint8_t* dp = (KIND == DK_CHUNK ? p.digests : p.macs) + 32ull * rec;
                        reinterpret_cast<uint4*>(dp)[0] = make_uint4(d[0], d[1], d[2], d[3]);
                        reinterpret_cast<uint4*>(dp)[1] = make_uint4(d[4], d[5], d[6], d[7]);
                    } else {
                        sp_zero_bytes(p.out + ob, Lo);  // not processed
                    }
                } else {
                    uint32_t diff = valid ? 0u : 1u;
                    if (valid) {
                        const uint8_t* ep = (KIND == DK_CHUNK ? p.expect : p.macs_in) + 32ull * rec;
#pragma unroll
                        for (int j = 0; j < 8; ++j) diff |= ld32(ep + 4 * j) ^ d[j];
                        if (kAead && runs[(Ts + 1u) & 1u][0][lane].x == 0u) diff = 1;
                    }
                    p.ok[rec] = diff == 0u ? 1 : 0;
                    if (diff != 0u) sp_zero_bytes(p.out + ob, Lo);  // no plaintext for a failed record
                }
            }
            ENET_SP_BARRIER();
        }
    }
}

hipError_t launch_duplex_split(int kind, bool open, const DuplexParams& p, hipStream_t s) {
    const dim3 g((p.n + kSRec - 1) / kSRec), b(kSWaves * kSRec);
    switch (kind * 2 + (open ? 1 : 0)) {
        case DK_CHUNK * 2: hipLaunchKernelGGL((duplex_split_kernel<DK_CHUNK, false>), g, b, 0, s, p); break;
        case DK_CHUNK * 2 + 1: hipLaunchKernelGGL((duplex_split_kernel<DK_CHUNK, true>), g, b, 0, s, p); break;
        case DK_AEADH * 2: hipLaunchKernelGGL((duplex_split_kernel<DK_AEADH, false>), g, b, 0, s, p); break;
        case DK_AEADH * 2 + 1: hipLaunchKernelGGL((duplex_split_kernel<DK_AEADH, true>), g, b, 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace enet
