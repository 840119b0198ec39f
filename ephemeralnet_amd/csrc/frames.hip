// frames.hip -- fused HMAC-SHA256 + ChaCha20 for uniform batches of session frames (gfx950).
//
// The reference signs then encrypts every session message (protocol::encode_signed,
// src/protocol/Message.cpp:305-311: m || HMAC-SHA256_K(m); SessionManager::send,
// src/network/SessionManager.cpp:362-387: ChaCha20 counter 0 over it behind a nonce || BE32 length
// header) and reverses it on receive (SessionManager.cpp:760-822, Message.cpp:313-328).
//
// SHA-256 is serial inside a record, so at one lane per record a batch of 65 536 frames gives one
// SHA wave per SIMD, and a single wave cannot issue faster than ~4.5 cycles per instruction on
// gfx950.  This kernel gives every SIMD a second, independent instruction stream
// instead of a second SHA wave: a 512-thread workgroup owns 256 records and splits into
//   waves 0-3  "cipher" waves -- the ChaCha20 pass with whole-line LDS staging (as records.hip
//              COOP 1: per stage each lane moves 128 bytes of its record), and
//   waves 4-7  "MAC" waves -- HMAC-SHA256 of the same 256 records, one lane per record,
// so each SIMD runs one wave of each kind (waves w and w + 4 share a SIMD).  The message bytes
// cross HBM once: the cipher lane hands every stage's plaintext (seal: what it loaded, open: what
// it decrypted) to the MAC lane of the same record through a double-buffered LDS slab, one
// workgroup barrier per stage.  After the last stage the MAC goes through LDS the other way
// (seal: MAC lane -> cipher lane, which encrypts it as the body's last 32 bytes; open: cipher lane
// decrypts it -> MAC lane, which compares).
#include "enet_device.hpp"
#include "enet_internal.hpp"

namespace enet {

namespace {

constexpr uint32_t kFWG = 512;  // threads per workgroup: 4 cipher + 4 MAC waves

// all waves of the workgroup: this wave's LDS writes are done, then meet
#define ENET_WG_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
// lanes of one wave hand LDS data to each other: DS ops of a wave execute in order
#define ENET_FR_WAVE_SYNC()                   \
    do {                                      \
        asm volatile("" ::: "memory");        \
        __builtin_amdgcn_wave_barrier();      \
        asm volatile("" ::: "memory");        \
    } while (0)

__device__ __forceinline__ void sha_iv(uint32_t st[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
}

}  // namespace

// OPEN: false = seal (in = m, out = [hdr] || body), true = open (in = [hdr] || body, out = m).
// HDR: 16 = whole wire frames (nonce || BE32 length header), 0 = frame bodies.
// CHUNK: the store / fetch pipeline instead (Node::store_chunk, src/core/Node.cpp:1414-1417;
// Node::fetch_chunk, :1644-1655): ciphertext = ChaCha20(key, nonce, LE32(chunk_id), m) with no MAC
// tail (CryptoManager.cpp:8-13,38-58), and the MAC waves compute the plain SHA-256(m) -- written
// to p.digests on store, compared with p.expect on fetch (failed chunks are zeroed).
template <bool OPEN, int HDR, bool CHUNK>
__global__ __launch_bounds__(kFWG) void frames_fused_kernel(FrameFusedParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t slab[4 * 64 * kFrameRun];           // 32 KB
    __shared__ __attribute__((aligned(16))) uint8_t ptb[2 * kFrameRecsPerWG * kFrameRun];  // 64 KB
    __shared__ __attribute__((aligned(16))) uint32_t macb[kFrameRecsPerWG * 8];          // 8 KB

    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = wave & 3u;
    const uint32_t rl = 64u * w + lane;                  // record within the workgroup
    const uint32_t rec0 = blockIdx.x * kFrameRecsPerWG;  // the host launches whole workgroups
    const uint32_t rec = rec0 + rl;
    const uint64_t Lm = p.msg_len;
    const uint32_t Ts = (uint32_t)(Lm / kFrameRun);
    const uint64_t Lb = CHUNK ? Lm : Lm + 32;  // frame body = m || MAC, chunk = m
    const uint64_t Si = OPEN ? Lb + HDR : Lm;
    const uint64_t So = OPEN ? Lm : Lb + HDR;
    const uint8_t* inb = p.in + p.in_off[0];
    uint8_t* outb = p.out + p.out_off[0];
    const uint32_t msw = (lane >> 1) & 7u;  // 16-byte chunk swizzle of a 128-byte run in LDS
    uint8_t* const myp = ptb + rl * kFrameRun;
    constexpr uint32_t kPtbBuf = kFrameRecsPerWG * kFrameRun;

    uint32_t kw[8];
    {
        const uint4* kq = reinterpret_cast<const uint4*>(p.keys + (size_t)p.key_stride * rec);
        const uint4 a = kq[0], b = kq[1];
        kw[0] = a.x; kw[1] = a.y; kw[2] = a.z; kw[3] = a.w;
        kw[4] = b.x; kw[5] = b.y; kw[6] = b.z; kw[7] = b.w;
    }

    if (wave < 4) {
        // ------------------------------------------------------------------ cipher waves
        uint32_t nw[3];
        if (OPEN && HDR) {  // nonce = the frame's first 12 bytes (SessionManager.cpp:815-822)
            const uint8_t* f = inb + Si * rec;
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = ld32(f + 4 * i);
        } else {
            const uint32_t* np = reinterpret_cast<const uint32_t*>(p.nonces + 12ull * rec);
#pragma unroll
            for (int i = 0; i < 3; ++i) nw[i] = np[i];
        }
        ChachaRecord R;
        chacha_record_init(R, kw, nw);
        // ChaCha20::apply's start counter: 0 for frames, LE32(chunk_id[0..3]) for chunks (u32 wrap)
        const uint32_t c0 = CHUNK ? ld32(p.chunk_ids + 32ull * rec) : 0u;
        // load / store instruction i serves owners 8i..8i+7 of this wave, 8 lanes x 16 B each
        const uint32_t kk = lane & 7u;
        uint64_t ioff[8], ooff[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t o = 8u * i + (lane >> 3);
            const uint32_t sw = (o >> 1) & 7u;
            const uint64_t ro = rec0 + 64u * w + o;
            ioff[i] = ro * Si + (OPEN ? HDR : 0) + 16u * (kk ^ sw);
            ooff[i] = ro * So + (OPEN ? 0 : HDR) + 16u * (kk ^ sw);
        }
        uint8_t* const wslab = slab + w * 64u * kFrameRun;
        uint8_t* const myrun = wslab + lane * kFrameRun;
        uint32_t pf[32];
        auto fetch = [&](uint32_t st) {
            const uint64_t adv = (uint64_t)kFrameRun * st;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint4 v = *reinterpret_cast<const uint4*>(inb + ioff[i] + adv);
                pf[4 * i] = v.x; pf[4 * i + 1] = v.y; pf[4 * i + 2] = v.z; pf[4 * i + 3] = v.w;
            }
        };
        auto land = [&]() {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(wslab + 1024u * i + 16u * lane) =
                    make_uint4(pf[4 * i], pf[4 * i + 1], pf[4 * i + 2], pf[4 * i + 3]);
        };
        auto put_run = [&](uint8_t* dst, const uint32_t* v) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<uint4*>(dst + 16u * (k ^ msw)) =
                    make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        };
        fetch(0);
        land();
        for (uint32_t s = 0; s < Ts; ++s) {
            ENET_FR_WAVE_SYNC();
            uint32_t x[32];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint4 v = *reinterpret_cast<const uint4*>(myrun + 16u * (k ^ msw));
                x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
            }
            fetch(min(s + 1, Ts - 1));  // the last stage re-reads its own lines (L2 hits)
            asm volatile("" : "+v"(R.k[0]) :: "memory");
            uint8_t* const pt = myp + (s & 1u) * kPtbBuf;
            if (!OPEN) put_run(pt, x);  // plaintext for the MAC lane
            {
                uint32_t ka[16], kb[16];
                chacha_block2(R, c0 + 2u * s, c0 + 2u * s + 1u, ka, kb);
#pragma unroll
                for (int i = 0; i < 16; ++i) { x[i] ^= ka[i]; x[16 + i] ^= kb[i]; }
            }
            if (OPEN) put_run(pt, x);
            ENET_FR_WAVE_SYNC();
            put_run(myrun, x);
            ENET_FR_WAVE_SYNC();
            const uint64_t adv = (uint64_t)kFrameRun * s;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<uint4*>(outb + ooff[i] + adv) =
                    *reinterpret_cast<const uint4*>(wslab + 1024u * i + 16u * lane);
            ENET_FR_WAVE_SYNC();
            land();
            ENET_WG_LDS_BARRIER();  // stage s plaintext is in ptb[s & 1]
        }
        if (CHUNK) {
            if (OPEN) {
                // the plaintext stores are complete before a MAC lane may zero them on failure
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                ENET_WG_LDS_BARRIER();
            }
            return;
        }
        uint32_t ks[16];
        chacha_block(R, (uint32_t)(Lm >> 6), ks);  // the MAC is the body's block Lm / 64
        if (!OPEN) {
            ENET_WG_LDS_BARRIER();  // MACs are in macb
            const uint4 a = *reinterpret_cast<const uint4*>(macb + 8u * rl);
            const uint4 b = *reinterpret_cast<const uint4*>(macb + 8u * rl + 4u);
            uint8_t* body = outb + So * rec + HDR;
            *reinterpret_cast<uint4*>(body + Lm) =
                make_uint4(a.x ^ ks[0], a.y ^ ks[1], a.z ^ ks[2], a.w ^ ks[3]);
            *reinterpret_cast<uint4*>(body + Lm + 16) =
                make_uint4(b.x ^ ks[4], b.y ^ ks[5], b.z ^ ks[6], b.w ^ ks[7]);
            if (HDR) {  // nonce(12) || BE32(|body|) (SessionManager.cpp:376-385)
                *reinterpret_cast<uint4*>(outb + So * rec) =
                    make_uint4(nw[0], nw[1], nw[2], bswap32((uint32_t)Lb));
            }
        } else {
            const uint8_t* body = inb + Si * rec + HDR;
            const uint4 a = *reinterpret_cast<const uint4*>(body + Lm);
            const uint4 b = *reinterpret_cast<const uint4*>(body + Lm + 16);
            const uint4 ma = make_uint4(a.x ^ ks[0], a.y ^ ks[1], a.z ^ ks[2], a.w ^ ks[3]);
            const uint4 mb = make_uint4(b.x ^ ks[4], b.y ^ ks[5], b.z ^ ks[6], b.w ^ ks[7]);
            *reinterpret_cast<uint4*>(macb + 8u * rl) = ma;
            *reinterpret_cast<uint4*>(macb + 8u * rl + 4u) = mb;
            uint4* mo = reinterpret_cast<uint4*>(p.macs + 32ull * rec);
            mo[0] = ma;
            mo[1] = mb;
            // the plaintext stores are complete before a MAC lane may zero them on failure
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ENET_WG_LDS_BARRIER();
        }
    } else {
        // ------------------------------------------------------------------ MAC waves
        // frames: HMAC-SHA256 (HmacSha256.cpp:11-39) with the 32-byte session key;
        // chunks: SHA-256 (Sha256::digest, Sha256.cpp:66-132)
        uint32_t kb[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) kb[i] = bswap32(kw[i]);
        uint32_t st[8], x[16];
        sha_iv(st);
        if (!CHUNK) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = (i < 8 ? kb[i] : 0u) ^ 0x36363636u;
            sha256_compress(st, x);
        }
        for (uint32_t s = 0; s < Ts; ++s) {
            ENET_WG_LDS_BARRIER();
            const uint8_t* pt = myp + (s & 1u) * kPtbBuf;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint4 v = *reinterpret_cast<const uint4*>(pt + 16u * ((4 * h + k) ^ msw));
                    x[4 * k] = bswap32(v.x); x[4 * k + 1] = bswap32(v.y);
                    x[4 * k + 2] = bswap32(v.z); x[4 * k + 3] = bswap32(v.w);
                }
                sha256_compress(st, x);
            }
        }
        {  // padding of [ipad ||] m: 0x80, zeros, BE64 bit length (Lm is a multiple of 64)
            const uint64_t bits = ((CHUNK ? 0ull : 64ull) + Lm) * 8ull;
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = 0u;
            x[0] = 0x80000000u;
            x[14] = (uint32_t)(bits >> 32);
            x[15] = (uint32_t)bits;
            sha256_compress(st, x);
        }
        if (CHUNK) {
            if (!OPEN) {  // chunk_hash = SHA-256(m), digest bytes big-endian
                uint4* d = reinterpret_cast<uint4*>(p.digests + 32ull * rec);
                d[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
                d[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
                return;
            }
            ENET_WG_LDS_BARRIER();  // the cipher waves' plaintext stores are complete
            // hash != manifest.chunk_hash -> no plaintext (Node.cpp:1652-1655)
            const uint8_t* e = p.expect + 32ull * rec;
            uint32_t diff = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) diff |= ld32(e + 4 * i) ^ bswap32(st[i]);
            p.ok[rec] = diff == 0 ? 1 : 0;
            if (diff != 0) {
                uint4* z = reinterpret_cast<uint4*>(outb + So * rec);
                for (uint64_t b = 0; b < Lm / 16; ++b) z[b] = make_uint4(0u, 0u, 0u, 0u);
            }
            return;
        }
        uint32_t inner[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) inner[i] = st[i];
        sha_iv(st);
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
        if (!OPEN) {
            *reinterpret_cast<uint4*>(macb + 8u * rl) =
                make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
            *reinterpret_cast<uint4*>(macb + 8u * rl + 4u) =
                make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
            ENET_WG_LDS_BARRIER();
        } else {
            ENET_WG_LDS_BARRIER();  // decrypted MACs are in macb
            // HmacSha256::verify (HmacSha256.cpp:41-54): OR-accumulated difference
            uint32_t diff = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) diff |= macb[8u * rl + i] ^ bswap32(st[i]);
            if (HDR) {  // the length field must give the body (SessionManager.cpp:770-796)
                const uint32_t be = bswap32(ld32(inb + Si * rec + 12));
                if ((uint64_t)be != Lb) diff = 1;
            }
            p.ok[rec] = diff == 0 ? 1 : 0;
            if (diff != 0) {  // no plaintext for a failed frame
                uint4* z = reinterpret_cast<uint4*>(outb + So * rec);
                for (uint64_t b = 0; b < Lm / 16; ++b) z[b] = make_uint4(0u, 0u, 0u, 0u);
            }
        }
    }
}

hipError_t launch_frames_fused(bool open, uint32_t hdr, const FrameFusedParams& p, hipStream_t s) {
    const uint32_t blocks = p.n / kFrameRecsPerWG;
    if (blocks == 0) return hipSuccess;
    if (!open && hdr)
        hipLaunchKernelGGL((frames_fused_kernel<false, 16, false>), dim3(blocks), dim3(kFWG), 0, s, p);
    else if (!open)
        hipLaunchKernelGGL((frames_fused_kernel<false, 0, false>), dim3(blocks), dim3(kFWG), 0, s, p);
    else if (hdr)
        hipLaunchKernelGGL((frames_fused_kernel<true, 16, false>), dim3(blocks), dim3(kFWG), 0, s, p);
    else
        hipLaunchKernelGGL((frames_fused_kernel<true, 0, false>), dim3(blocks), dim3(kFWG), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_chunks_fused(bool fetch, const FrameFusedParams& p, hipStream_t s) {
    const uint32_t blocks = p.n / kFrameRecsPerWG;
    if (blocks == 0) return hipSuccess;
    if (fetch)
        hipLaunchKernelGGL((frames_fused_kernel<true, 0, true>), dim3(blocks), dim3(kFWG), 0, s, p);
    else
        hipLaunchKernelGGL((frames_fused_kernel<false, 0, true>), dim3(blocks), dim3(kFWG), 0, s, p);
    return hipGetLastError();
}

}  // namespace enet
