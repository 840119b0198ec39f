// duplex.hip -- one HBM pass of cipher + hash over ANY batch of records (gfx950).
//
// Three reference paths encrypt a record and hash the same bytes:
//   frames   protocol::encode_signed + SessionManager::send (Message.cpp:305-311,
//            SessionManager.cpp:362-387): body = ChaCha20_{K,N,0}(m || HMAC-SHA256_K(m)), optionally
//            behind the nonce(12) || BE32(|body|) wire header; receive reverses it
//            (SessionManager.cpp:760-822, Message.cpp:313-328);
//   chunks   Node::store_chunk / fetch_chunk (Node.cpp:1414-1417, 1644-1655): ChaCha20 from counter
//            LE32(chunk_id) (CryptoManager.cpp:8-13, 38-58) and SHA-256(m) (= derive_chunk_id);
//   AEAD+MAC RFC 8439 ChaCha20-Poly1305 with HMAC-SHA256_K(m) beside the tag (BASELINE config 5).
// SHA-256 is serial inside a record, so a record gets one lane for its hash; a 512-thread workgroup
// owns 256 records and splits into 4 "cipher" waves and 4 "hash" waves (waves w and w + 4 share a
// SIMD and a record set: lane l of both serves record 64 w + l).  The cipher lane streams its
// record in 128-byte stages (one stage prefetched in registers), runs ChaCha20 (and Poly1305 over
// the ciphertext), stores, and hands every stage's plaintext to the hash lane through a
// double-buffered LDS slab -- one workgroup barrier per stage.  The plaintext is never re-read
// from HBM.
//
// Unlike frames.hip (uniform lengths, multiple of 128 B, whole workgroups), nothing is assumed:
// every lane reads its own record's offsets, lengths may differ lane to lane (a workgroup runs
// the stages of its longest record; `order` -- e.g. length-sorted -- keeps workgroups balanced),
// record starts may have any alignment, and the ragged end of a record (< 128 bytes, plus the
// 32-byte MAC of a frame body) goes through a 160-byte LDS tail slot per record:
//   seal  T1 cipher loads the message tail and parks it in the slot (chunks / AEAD also encrypt
//            and store it); T2 hash lane hashes it (masked, SHA padding) and finishes the digest --
//            frames put the MAC bytes right behind the message tail in the slot; T3 (frames) the
//            cipher lane encrypts message tail || MAC as one run of body bytes and stores it.
//   open  T1 cipher loads the body tail, checks Poly1305 (AEAD), decrypts, stores the message
//            tail, parks it (frames: with the decrypted MAC) in the slot; T2 hash lane finishes,
//            compares, writes ok, and zeroes a failed record's output.
// A record whose output length does not match its input (frames: out = in + 32 + hdr) is not
// processed: its output range is zeroed and, when opening, ok = 0.
#include "enet_device.hpp"
#include "enet_internal.hpp"

#include <cstdlib>

namespace enet {

namespace {

constexpr uint32_t kRun = 128;  // bytes per stage and record

// one wave: its lanes' LDS writes are visible to its other lanes (DS ops of a wave execute in
// issue order; a compiler barrier and a wave barrier suffice, no vmcnt drain)
#define ENET_DX_WAVE_SYNC()               \
    do {                                  \
        asm volatile("" ::: "memory");    \
        __builtin_amdgcn_wave_barrier();  \
        asm volatile("" ::: "memory");    \
    } while (0)

// all waves: this wave's LDS traffic is done, then meet
#define ENET_DX_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// keep bytes [0, r) of the LE byte string in w[0..N)
template <int N>
__device__ __forceinline__ void keep_le(uint32_t* w, uint32_t r) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
        const uint32_t b = 4u * j;
        const uint32_t m = b + 4u <= r ? 0xffffffffu : (b >= r ? 0u : (1u << (8u * (r - b))) - 1u);
        w[j] &= m;
    }
}

__device__ __forceinline__ void zero_bytes(uint8_t* p, uint64_t n) {
    const uint32_t z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (uint64_t o = 0; o < n; o += 64) store_block(p + o, (uint32_t)min<uint64_t>(64, n - o), z);
}

__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) { return ld32(p); }

}  // namespace

// RPW records per workgroup: RPW / 64 cipher waves + RPW / 64 hash waves.
template <int KIND, bool OPEN, int RPW>
__device__ __forceinline__ void duplex_body(const DuplexParams& p) {
    constexpr uint32_t kW = RPW / 64;          // waves per role
    constexpr uint32_t kBuf = RPW * kRun;      // one stage of the workgroup (32 KB at 256 records)
    __shared__ __attribute__((aligned(16))) uint8_t ptb[2 * kBuf];  // stage slabs
    __shared__ __attribute__((aligned(16))) uint8_t text[RPW * 32];  // tail slot bytes 128..159
    __shared__ uint32_t tmax_s;
    // chunk fetch: each record's output base and whole stages, for the line-wise plaintext stores
    // (the frame and AEAD+HMAC opens keep per-lane stores: at the 128-VGPR cap the line-wise form
    // spilled there and cost C3 wire open 4 %, 1 904 -> 1 981 us, r06 prof_c3w)
    constexpr bool kLines = OPEN && KIND == DK_CHUNK;
    __shared__ uint64_t odst_s[kLines ? RPW : 1];
    __shared__ uint32_t ots_s[kLines ? RPW : 1];

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const bool cipher = wave < kW;
    const uint32_t rl = 64u * (wave % kW) + lane;
    const uint32_t pos = blockIdx.x * RPW + rl;
    const bool live = pos < p.n;
    const uint32_t rec = live ? (p.order ? p.order[pos] : pos) : 0u;
    const uint32_t H = KIND == DK_FRAME ? p.hdr : 0u;

    // ---- geometry (both lanes of a record compute it)
    uint64_t ib = 0, Li = 0, ob = 0, Lo = 0;
    bool ordered = true;  // offsets non-decreasing: a decreasing pair would wrap Li / Lo to ~2^64
    if (live) {
        ib = p.in_off[rec];
        const uint64_t ie = p.in_off[rec + 1];
        ob = p.out_off[rec];
        const uint64_t oe = p.out_off[rec + 1];
        ordered = ie >= ib && oe >= ob;
        Li = ordered ? ie - ib : 0u;
        Lo = ordered ? oe - ob : 0u;  // nothing is zeroed for a disordered record
    }
    uint64_t Lm = 0;  // message bytes
    bool valid = live && ordered;
    if (KIND == DK_FRAME && !OPEN) {
        Lm = Li;
        valid = valid && Lo == Li + 32u + H;
    } else if (KIND == DK_FRAME) {  // frames shorter than [hdr] + MAC fail (Message.cpp:315)
        valid = valid && Li >= 32ull + H;
        Lm = valid ? Li - 32u - H : 0;
        valid = valid && Lo == Lm;
    } else {
        Lm = Li;
        valid = valid && Lo == Li;
    }
    // session-keyed frames: an index outside the table fails closed -- the record is processed
    // as invalid (seal: the whole output slot zeroed, no byte encrypted under another session's
    // key; open: ok = 0, plaintext zeroed), and no key or midstate past the table is read
    const uint32_t sraw = (p.session && live) ? p.session[rec] : 0u;
    const bool sbad = p.session && sraw >= p.n_sessions;
    const uint32_t sid = sbad ? 0u : sraw;
    valid = valid && !sbad;
    if (!valid) Lm = 0;
    const uint32_t Ts = (uint32_t)(Lm / kRun);         // whole stages
    const uint32_t r = (uint32_t)(Lm - (uint64_t)kRun * Ts);  // ragged end, < 128
    const uint64_t tb = (uint64_t)kRun * Ts;            // message offset of the ragged end

    if (threadIdx.x == 0) tmax_s = 0;
    __syncthreads();
    if (cipher && Ts) atomicMax(&tmax_s, Ts);
    __syncthreads();
    const uint32_t Tmax = __builtin_amdgcn_readfirstlane(tmax_s);
    // Length-graded issue priority: a workgroup lasts as long as its longest record's serial
    // SHA-256 chain (one lane; 64 KiB = 1 027 compressions, ~2.8 ms), so with mixed lengths (C5)
    // the kernel's tail is that chain -- and when other workgroups (or, with overlapped steps, the
    // other direction's kernel) share its SIMDs, the chain only gets its share of issue slots.
    // Both waves of a long workgroup are on that chain (they meet at every stage barrier), so
    // they win arbitration over shorter workgroups'.
    if (p.prio == 0) {
        if (Tmax >= 256) __builtin_amdgcn_s_setprio(3);
        else if (Tmax >= 64) __builtin_amdgcn_s_setprio(2);
        else if (Tmax >= 16) __builtin_amdgcn_s_setprio(1);
    }

    // 16-byte chunk swizzles (row = record rl): conflict-free ds_write_b128 (8-lane groups) and
    // ds_read_b128 (16-lane groups) for the 128-byte runs and the 32-byte tail extension
    const uint32_t msw = ((lane >> 1) & 7u) ^ ((lane & 1u) << 2);
    const uint32_t xsw = ((lane >> 2) ^ (lane >> 3)) & 1u;
    uint8_t* const trow = ptb + (Tmax & 1u) * kBuf + rl * kRun;  // tail slot bytes 0..127
    uint8_t* const xrow = text + rl * 32u;                       // tail slot bytes 128..159
    auto slot_byte = [&](uint32_t i) -> uint8_t* {
        return i < kRun ? trow + 16u * ((i >> 4) ^ msw) + (i & 15u)
                        : xrow + 16u * (((i - kRun) >> 4) ^ xsw) + (i & 15u);
    };
    auto slot_put = [&](const uint32_t* w, int chunks) {  // slot words [0, 4 * chunks)
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            if (c < chunks) {
                uint8_t* d = c < 8 ? trow + 16u * (c ^ msw) : xrow + 16u * ((c - 8) ^ xsw);
                *reinterpret_cast<uint4*>(d) = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
            }
        }
    };
    auto slot_chunk = [&](int c) -> uint4 {
        const uint8_t* d = c < 8 ? trow + 16u * (c ^ msw) : xrow + 16u * ((c - 8) ^ xsw);
        return *reinterpret_cast<const uint4*>(d);
    };

    uint32_t kw[8];
    {
        const uint8_t* kp = p.session ? p.keys + 32ull * sid : p.keys + (size_t)p.key_stride * rec;
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = live ? reinterpret_cast<const uint32_t*>(kp)[i] : 0u;
    }

    if (cipher) {
        // ============================================================== cipher lane
        if (p.prio == 2) __builtin_amdgcn_s_setprio(2);
        const uint8_t* src = p.in + ib + (OPEN ? H : 0u);
        uint8_t* dst = p.out + ob + (OPEN ? 0u : H);
        const uint32_t off0 = OPEN ? H : 0u;  // offset of src inside the input record
        if (kLines) {
            odst_s[rl] = reinterpret_cast<uint64_t>(dst);  // read after the first stage barrier
            ots_s[rl] = Ts;
        }
        uint32_t nw[3];
        if (OPEN && KIND == DK_FRAME && H) {  // nonce = the frame's first 12 bytes (SessionManager.cpp:815-822)
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = valid ? ld32u(p.in + ib + 4 * i) : 0u;
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = live ? ld32u(p.nonces + 12ull * rec + 4 * i) : 0u;
        }
        ChachaRecord R;
        chacha_record_init(R, kw, nw);
        // ChaCha20::apply start counter: frames 0, chunks LE32(chunk_id) (u32 wrap), AEAD 1
        const uint32_t c0 = KIND == DK_FRAME ? 0u
                          : KIND == DK_CHUNK ? (live ? ld32u(p.chunk_ids + 32ull * rec) : 0u)
                                             : 1u;
        PolyR32 PR{};
        uint32_t h[5] = {0, 0, 0, 0, 0}, pad[4] = {0, 0, 0, 0};
        if (KIND == DK_AEADH) {  // one-time key = keystream block 0 (RFC 8439 2.6)
            uint32_t otk[16];
            chacha_block(R, 0u, otk);
            PR = polyr32_make(otk[0], otk[1], otk[2], otk[3]);
            pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        }
        auto poly_words = [&](const uint32_t* w, uint32_t blocks) {  // blocks <= 8
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q)
                if (q < blocks) poly32_block(h, PR, w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3], 1u);
        };

        uint32_t pf[32];
        auto load_run = [&](uint32_t s) {
            const uint4* q = reinterpret_cast<const uint4*>(src + (uint64_t)kRun * s);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = q[i];
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            }
        };
        auto put_run = [&](uint8_t* d, const uint32_t* v) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<uint4*>(d + 16u * (k ^ msw)) =
                    make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        };
        // Chunk fetch: every stage's plaintext is in the slab (for the hash lane); it is stored from there
        // line by line one stage later (after the barrier that hands the slab to the hash lanes,
        // which only read it; the cipher lanes rewrite it two stages on) -- instruction i serves
        // the wave's records 8i .. 8i+7, eight lanes per record, each record's whole 128-byte run
        // in one instruction.  Per-lane 16-byte stores wrote 64 records' lines in eight pieces
        // each, and the pieces the L2 wrote back separately doubled the fetch's HBM writes
        // (pmc_st_r05z.json: 2.03x the algorithmic write bytes; seal 1.42x).
        auto store_stage = [&](uint32_t t) {
            const uint32_t kk = lane & 7u;
            const uint32_t wrow = 64u * (wave % kW);
            const uint8_t* slab = ptb + (t & 1u) * kBuf;
#pragma unroll 1
            for (uint32_t i = 0; i < 8; ++i) {
                const uint32_t o = 8u * i + (lane >> 3);
                if (t < ots_s[wrow + o]) {
                    const uint32_t sw = ((o >> 1) & 7u) ^ ((o & 1u) << 2);
                    const uint4 v = *reinterpret_cast<const uint4*>(slab + (wrow + o) * kRun + 16u * kk);
                    uint8_t* d = reinterpret_cast<uint8_t*>(odst_s[wrow + o]) + (uint64_t)kRun * t + 16u * (kk ^ sw);
                    *reinterpret_cast<uint4*>(d) = v;
                }
            }
        };
        if (Ts > 0) load_run(0);
        for (uint32_t s = 0; s < Tmax; ++s) {
            if (kLines && s > 0) store_stage(s - 1);
            if (s < Ts) {
                uint32_t x[32];
#pragma unroll
                for (int i = 0; i < 32; ++i) x[i] = pf[i];
                if (s + 1 < Ts) load_run(s + 1);
                uint8_t* const pt = ptb + (s & 1u) * kBuf + rl * kRun;
                if (!OPEN) put_run(pt, x);  // plaintext for the hash lane
                if (KIND == DK_AEADH && OPEN) poly_words(x, 8);
                {
                    uint32_t ka[16], kb[16];
                    chacha_block2(R, c0 + 2u * s, c0 + 2u * s + 1u, ka, kb);
#pragma unroll
                    for (int i = 0; i < 16; ++i) { x[i] ^= ka[i]; x[16 + i] ^= kb[i]; }
                }
                if (KIND == DK_AEADH && !OPEN) poly_words(x, 8);
                if (OPEN) put_run(pt, x);
                if (!kLines) {
                    uint4* o = reinterpret_cast<uint4*>(dst + (uint64_t)kRun * s);
#pragma unroll
                    for (int i = 0; i < 8; ++i) o[i] = make_uint4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
                }
            }
            ENET_DX_BARRIER();  // stage s plaintext is in ptb[s & 1]
        }
        if (kLines && Tmax > 0) store_stage(Tmax - 1);

        // ---- ragged end
        const uint32_t tin = (OPEN && KIND == DK_FRAME) ? r + 32u : r;  // body-tail bytes read now
        uint32_t w[48];
#pragma unroll
        for (int i = 0; i < 48; ++i) w[i] = 0u;
        if (valid && tin) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if (tin > 64u * k) {
                    const uint32_t nk = min(64u, tin - 64u * k);
                    load_block(src + tb + 64u * k, nk, w + 16 * k, off0 + tb + 64u * k + nk >= 16u);
                }
            }
        }
        uint32_t ks[48];
#pragma unroll
        for (int i = 32; i < 48; ++i) ks[i] = 0u;  // the third block is only made when a body needs it
        if (valid && (tin || (!OPEN && KIND == DK_FRAME))) {
            chacha_block2(R, c0 + 2u * Ts, c0 + 2u * Ts + 1u, ks, ks + 16);
            if (KIND == DK_FRAME && r + 32u > 128u) chacha_block(R, c0 + 2u * Ts + 2u, ks + 32);
        }
        if (!OPEN) {
            if (valid) {
                // T1: the message tail to the hash lane
                slot_put(w, 8);
                if (KIND != DK_FRAME && r) {
#pragma unroll
                    for (int j = 0; j < 32; ++j) w[j] ^= ks[j];
                    store_block(dst + tb, min(r, 64u), w);
                    if (r > 64u) store_block(dst + tb + 64, r - 64u, w + 16);
                    if (KIND == DK_AEADH) {
                        keep_le<32>(w, r);
                        poly_words(w, (r + 15u) >> 4);
                    }
                }
                if (KIND == DK_AEADH) {
                    poly32_block(h, PR, 0u, 0u, (uint32_t)Lm, (uint32_t)(Lm >> 32), 1u);
                    uint32_t l[5], tag[4];
                    h32_to_limbs(h, l);
                    pfinish(l, pad, tag);
                    *reinterpret_cast<uint4*>(p.tags + 16ull * rec) = make_uint4(tag[0], tag[1], tag[2], tag[3]);
                }
            }
            ENET_DX_BARRIER();  // T1
            ENET_DX_BARRIER();  // T2: frames -- the MAC sits behind the message tail in the slot
            if (KIND == DK_FRAME && valid) {
                // T3: body tail = message tail || MAC, one run of body bytes
                const uint32_t t = r + 32u;
#pragma unroll
                for (int c = 0; c < 10; ++c) {
                    const uint4 v = slot_chunk(c);
                    w[4 * c] = v.x ^ ks[4 * c]; w[4 * c + 1] = v.y ^ ks[4 * c + 1];
                    w[4 * c + 2] = v.z ^ ks[4 * c + 2]; w[4 * c + 3] = v.w ^ ks[4 * c + 3];
                }
                store_block(dst + tb, min(t, 64u), w);
                if (t > 64u) store_block(dst + tb + 64, min(t - 64u, 64u), w + 16);
                if (t > 128u) store_block(dst + tb + 128, t - 128u, w + 32);
                if (H) {  // nonce(12) || BE32(|body|) (SessionManager.cpp:376-385)
                    *reinterpret_cast<uint4*>(p.out + ob) =
                        make_uint4(nw[0], nw[1], nw[2], bswap32((uint32_t)(Lm + 32u)));
                }
            }
        } else {
            if (valid) {
                uint32_t aok = 1;
                if (KIND == DK_AEADH) {  // Poly1305 over the ciphertext (zero beyond r), then lengths
                    poly_words(w, (r + 15u) >> 4);
                    poly32_block(h, PR, 0u, 0u, (uint32_t)Lm, (uint32_t)(Lm >> 32), 1u);
                    uint32_t l[5], tag[4];
                    h32_to_limbs(h, l);
                    pfinish(l, pad, tag);
                    const uint8_t* tp = p.tags_in + 16ull * rec;
                    aok = ((tag[0] ^ ld32u(tp)) | (tag[1] ^ ld32u(tp + 4)) | (tag[2] ^ ld32u(tp + 8)) |
                           (tag[3] ^ ld32u(tp + 12))) == 0u;
                }
                if (tin) {
#pragma unroll
                    for (int j = 0; j < 40; ++j) w[j] ^= ks[j];
                }
                if (r) {
                    store_block(dst + tb, min(r, 64u), w);
                    if (r > 64u) store_block(dst + tb + 64, r - 64u, w + 16);
                }
                slot_put(w, KIND == DK_FRAME ? 10 : 8);
                if (KIND == DK_AEADH) *slot_byte(159) = (uint8_t)aok;
            }
            // the plaintext stores are complete before a hash lane may zero them on failure
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ENET_DX_BARRIER();  // T1
        }
    } else {
        // ============================================================== hash lane
        if (p.prio == 1) __builtin_amdgcn_s_setprio(2);
        // frames / AEAD: HMAC-SHA256 (HmacSha256.cpp:11-39) with the 32-byte record key;
        // chunks: SHA-256 (Sha256::digest, Sha256.cpp:66-132)
        uint32_t kb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kb[i] = bswap32(kw[i]);
        uint32_t st[8], x[16];
        // session-keyed frames: the session's midstates replace the ipad / opad compressions
        const uint32_t* ms = (KIND == DK_FRAME && p.mid && live) ? p.mid + 16ull * sid : nullptr;
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
        if (KIND != DK_CHUNK) {
            if (ms) {
#pragma unroll
                for (int i = 0; i < 8; ++i) st[i] = ms[i];
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) x[i] = (i < 8 ? kb[i] : 0u) ^ 0x36363636u;
                sha256_compress(st, x);
            }
        }
        for (uint32_t s = 0; s < Tmax; ++s) {
            ENET_DX_BARRIER();
            if (s < Ts) {
                const uint8_t* pt = ptb + (s & 1u) * kBuf + rl * kRun;
#pragma unroll
                for (int hb = 0; hb < 2; ++hb) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint4 v = *reinterpret_cast<const uint4*>(pt + 16u * ((4 * hb + k) ^ msw));
                        x[4 * k] = bswap32(v.x); x[4 * k + 1] = bswap32(v.y);
                        x[4 * k + 2] = bswap32(v.z); x[4 * k + 3] = bswap32(v.w);
                    }
                    sha256_compress(st, x);
                }
            }
        }
        ENET_DX_BARRIER();  // T1: the ragged end is in the slot
        uint32_t d[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // digest as LE words of its bytes
        if (valid) {
            // message tail, 0x80, zeros, BE64 bit length of [ipad ||] m
            const uint64_t bits = ((KIND == DK_CHUNK ? 0ull : 64ull) + Lm) * 8ull;
            const uint32_t nb = (r + 9u + 63u) >> 6;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if ((uint32_t)k < nb) {
                    uint32_t blk[16];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const uint4 v = k < 2 ? slot_chunk(4 * k + c) : make_uint4(0u, 0u, 0u, 0u);
                        blk[4 * c] = v.x; blk[4 * c + 1] = v.y; blk[4 * c + 2] = v.z; blk[4 * c + 3] = v.w;
                    }
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t b = 64u * k + 4u * i;
                        const uint32_t v = bswap32(blk[i]);
                        const uint32_t m = b + 4u <= r ? 0xffffffffu : (b >= r ? 0u : 0xffffffffu << (8u * (4u - (r - b))));
                        x[i] = (v & m) | ((r >> 2) == (b >> 2) ? 0x80000000u >> (8u * (r & 3u)) : 0u);
                    }
                    if ((uint32_t)k == nb - 1u) {
                        x[14] = (uint32_t)(bits >> 32);
                        x[15] = (uint32_t)bits;
                    }
                    sha256_compress(st, x);
                }
            }
            if (KIND != DK_CHUNK) {
                uint32_t inner[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) inner[i] = st[i];
                if (ms) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) st[i] = ms[8 + i];
                } else {
#pragma unroll
                    for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
#pragma unroll
                    for (int i = 0; i < 16; ++i) x[i] = (i < 8 ? kb[i] : 0u) ^ 0x5c5c5c5cu;
                    sha256_compress(st, x);
                }
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
                if (KIND == DK_FRAME) {  // the MAC follows the message tail in the slot
                    for (uint32_t i = 0; i < 32u; ++i) *slot_byte(r + i) = (uint8_t)(d[i >> 2] >> (8u * (i & 3u)));
                } else {
                    uint8_t* dp = (KIND == DK_CHUNK ? p.digests : p.macs) + 32ull * rec;
                    reinterpret_cast<uint4*>(dp)[0] = make_uint4(d[0], d[1], d[2], d[3]);
                    reinterpret_cast<uint4*>(dp)[1] = make_uint4(d[4], d[5], d[6], d[7]);
                }
            } else if (live) {
                zero_bytes(p.out + ob, Lo);
            }
            ENET_DX_BARRIER();  // T2
        } else if (live) {
            uint32_t diff = valid ? 0u : 1u;
            if (valid) {
                if (KIND == DK_FRAME) {  // HmacSha256::verify (HmacSha256.cpp:41-54)
                    uint32_t e[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        uint32_t v = 0;
#pragma unroll
                        for (int b = 0; b < 4; ++b) v |= (uint32_t)*slot_byte(r + 4u * j + b) << (8 * b);
                        e[j] = v;
                        diff |= v ^ d[j];
                    }
                    uint8_t* mp = p.macs + 32ull * rec;
                    reinterpret_cast<uint4*>(mp)[0] = make_uint4(e[0], e[1], e[2], e[3]);
                    reinterpret_cast<uint4*>(mp)[1] = make_uint4(e[4], e[5], e[6], e[7]);
                    if (H) {  // the length field must give the body (SessionManager.cpp:770-796)
                        const uint32_t be = bswap32(ld32u(p.in + ib + 12));
                        if ((uint64_t)be != Li - H) diff = 1;
                    }
                } else {
                    const uint8_t* ep = (KIND == DK_CHUNK ? p.expect : p.macs_in) + 32ull * rec;
#pragma unroll
                    for (int j = 0; j < 8; ++j) diff |= ld32u(ep + 4 * j) ^ d[j];
                    if (KIND == DK_AEADH && *slot_byte(159) == 0) diff = 1;
                }
            }
            p.ok[rec] = diff == 0u ? 1 : 0;
            if (diff != 0u) zero_bytes(p.out + ob, Lo);  // no plaintext for a failed record
        }
    }
}

// Frames and chunks fit 128 VGPRs, so two workgroups share a CU (LDS 72 KB each) when the batch
// has more than 256 workgroups (C3: 1 M frames, 358 -> 388 GiB/s).  The AEAD + HMAC body would
// spill at 128, so it keeps one workgroup per CU.
template <int KIND, bool OPEN, int RPW>
__global__ __launch_bounds__(2 * RPW) __attribute__((amdgpu_waves_per_eu(4))) void duplex_kernel(DuplexParams p) {
    duplex_body<KIND, OPEN, RPW>(p);
}
template <int KIND, bool OPEN, int RPW>
__global__ __launch_bounds__(2 * RPW) void duplex_kernel_wide(DuplexParams p) {
    duplex_body<KIND, OPEN, RPW>(p);
}

template <int RPW>
hipError_t launch_duplex_rpw(int kind, bool open, const DuplexParams& p, hipStream_t s) {
    const uint32_t blocks = (p.n + RPW - 1) / RPW;
    const dim3 g(blocks), b(2 * RPW);
    switch (kind * 2 + (open ? 1 : 0)) {
        case DK_FRAME * 2: hipLaunchKernelGGL((duplex_kernel<DK_FRAME, false, RPW>), g, b, 0, s, p); break;
        case DK_FRAME * 2 + 1: hipLaunchKernelGGL((duplex_kernel<DK_FRAME, true, RPW>), g, b, 0, s, p); break;
        case DK_CHUNK * 2: hipLaunchKernelGGL((duplex_kernel<DK_CHUNK, false, RPW>), g, b, 0, s, p); break;
        case DK_CHUNK * 2 + 1: hipLaunchKernelGGL((duplex_kernel<DK_CHUNK, true, RPW>), g, b, 0, s, p); break;
        case DK_AEADH * 2: hipLaunchKernelGGL((duplex_kernel_wide<DK_AEADH, false, RPW>), g, b, 0, s, p); break;
        case DK_AEADH * 2 + 1: hipLaunchKernelGGL((duplex_kernel_wide<DK_AEADH, true, RPW>), g, b, 0, s, p); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_duplex(int kind, bool open, const DuplexParams& p, hipStream_t s) {
    if (p.n == 0) return hipSuccess;
    // long records (a 64 KiB record's serial hash chain is the whole kernel time): chunks and
    // AEAD + HMAC split each record over four waves (duplex_split.hip) -- for uniform batches
    // and batches the caller ordered (length-sorted, like C5).  The split kernel holds 2
    // workgroups per CU (80 KiB LDS) against 6 here, so an UNSORTED mixed batch, where every
    // workgroup holds some long record, runs two rounds of chains there: 45 vs 69 GiB/s at C5.
    if (kind == DK_CHUNK || kind == DK_AEADH) {
        const int m = duplex_split_mode();
        if (m == 1 || (m == -1 && p.max_len >= 16384u && (p.uniform || p.order != nullptr))) {
            DuplexParams q = p;
            return launch_duplex_split(kind, open, q, s);
        }
    }
    // A/B knobs, compiled into kernel objects built with -DENET_TOOLS_BUILD only (build.py --tools
    // --probes)
#ifdef ENET_TOOLS_BUILD
    static const int prio_env = [] {
        const char* e = std::getenv("ENET_DUPLEX_PRIO");
        return e ? (int)std::strtol(e, nullptr, 10) : 0;
    }();
    static const int rpw_env = [] {
        const char* e = std::getenv("ENET_DUPLEX_RPW");
        return e ? (int)std::strtol(e, nullptr, 10) : 0;
    }();
#else
    constexpr int prio_env = 0, rpw_env = 0;
#endif
    DuplexParams q = p;
    q.prio = prio_env;
    // Mixed lengths: 64-record workgroups, so the few long records (a workgroup lasts as long as
    // its longest record's serial hash) occupy few SIMDs and the rest of the chip keeps pulling
    // short workgroups (C5 device-resident: 88 -> 138 GiB/s).  Uniform batches: 256-record
    // workgroups once there are >= 128 of them (C4 store 64 KiB: 230 vs 217 GiB/s), else 64.
    const bool small = rpw_env ? rpw_env == 64 : (!p.uniform || p.n < 128u * 256u);
    return small ? launch_duplex_rpw<64>(kind, open, q, s) : launch_duplex_rpw<256>(kind, open, q, s);
}

}  // namespace enet
