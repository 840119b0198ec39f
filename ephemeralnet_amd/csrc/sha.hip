// sha.hip -- batched SHA-256 and HMAC-SHA256 (gfx950), one record per lane.
//
// SHA-256 is Merkle-Damgard: strictly serial inside a record, so the batch parallelises across
// records only (SURVEY.md 7 "hard parts").  Each lane streams its record in 64-byte blocks
// (four 16-byte loads, byte-swapped to big-endian words) through sha256_compress with the
// message schedule held as a rolling 16-word window in VGPRs.
//
// Reference behaviour (ShardianLabs/EphemeralNet):
//   Sha256 update/finalize/transform  src/crypto/Sha256.cpp:72-176 (BE length pad :94-126)
//   HmacSha256::compute               src/crypto/HmacSha256.cpp:11-39 (key > 64 B hashed :15-17)
//   HmacSha256::verify                src/crypto/HmacSha256.cpp:41-54 (OR-accumulated compare)
//   decode_signed short-buffer reject src/protocol/Message.cpp:315
#include "enet_device.hpp"
#include "enet_internal.hpp"

namespace enet {

// Absorb `len` message bytes at p into st (continuing a stream that already absorbed
// `prefix` bytes, a multiple of 64) and apply the final padding for prefix + len bytes.
__device__ __forceinline__ void sha_absorb_final(uint32_t st[8], const uint8_t* __restrict__ p,
                                                 uint64_t len, uint64_t prefix) {
    uint64_t done = 0;
    uint32_t w[16];
    for (; done + 64 <= len; done += 64) {
        const uint4* q = reinterpret_cast<const uint4*>(p + done);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q[i];
            w[4 * i] = bswap32(v.x); w[4 * i + 1] = bswap32(v.y);
            w[4 * i + 2] = bswap32(v.z); w[4 * i + 3] = bswap32(v.w);
        }
        sha256_compress(st, w);
    }
    // tail (0..63 bytes) + 0x80 + zeros + BE64 bit length, one or two blocks
    const uint32_t rem = (uint32_t)(len - done);
    const uint64_t bits = (prefix + len) * 8ull;
    uint32_t wl[16];
    if (rem) {
        load_block(p + done, rem, wl, done + rem >= 16);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) wl[i] = 0u;
    }
    const uint32_t mword = rem >> 2, mbit = 0x80u << (24 - 8 * (rem & 3u));
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = bswap32(wl[i]) | ((uint32_t)i == mword ? mbit : 0u);
    if (rem >= 56) {
        sha256_compress(st, w);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = 0;
    }
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    sha256_compress(st, w);
}

__device__ __forceinline__ void sha_init(uint32_t st[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = kShaIV[i];
}

__global__ __launch_bounds__(kWG) void sha_kernel(ShaParams p) {
    const uint32_t gid = blockIdx.x * kWG + threadIdx.x;
    if (gid >= p.n) return;
    const uint32_t rec = p.order ? p.order[gid] : gid;
    const uint64_t off = p.off[rec];
    const uint64_t len = p.off[rec + 1] - off;
    const uint8_t* msg = p.in + off;
    uint32_t st[8];

    if (!p.keys) {  // plain SHA-256 (Sha256::digest)
        sha_init(st);
        sha_absorb_final(st, msg, len, 0);
    } else {  // HMAC-SHA256
        const uint8_t* kp;
        uint64_t klen;
        if (p.key_off) {
            kp = p.keys + p.key_off[rec];
            klen = p.key_off[rec + 1] - p.key_off[rec];
        } else {
            kp = p.keys + (size_t)p.key_stride * rec;
            klen = 32;
        }
        uint32_t kb[16];  // key block as big-endian words
        if (klen > 64) {
            uint32_t hk[8];
            sha_init(hk);
            sha_absorb_final(hk, kp, klen, 0);
#pragma unroll
            for (int i = 0; i < 8; ++i) { kb[i] = hk[i]; kb[8 + i] = 0; }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t q = 4 * i + b;
                    if (q < klen) v |= (uint32_t)kp[q] << (24 - 8 * b);
                }
                kb[i] = v;
            }
        }
        uint32_t w[16];
        // inner = SHA(ipad || msg)
        sha_init(st);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = kb[i] ^ 0x36363636u;
        sha256_compress(st, w);
        sha_absorb_final(st, msg, len, 64);
        // outer = SHA(opad || inner)
        uint32_t inner[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) inner[i] = st[i];
        sha_init(st);
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = kb[i] ^ 0x5c5c5c5cu;
        sha256_compress(st, w);
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = inner[i];
        w[8] = 0x80000000u;
#pragma unroll
        for (int i = 9; i < 15; ++i) w[i] = 0;
        w[15] = (64 + 32) * 8;
        sha256_compress(st, w);
    }

    if (p.expect) {  // verify (HmacSha256::verify): OR-accumulate the difference
        const uint8_t* e = p.expect + 32ull * rec;
        uint32_t diff = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t ev = ((uint32_t)e[4 * i] << 24) | ((uint32_t)e[4 * i + 1] << 16) |
                                ((uint32_t)e[4 * i + 2] << 8) | (uint32_t)e[4 * i + 3];
            diff |= ev ^ st[i];
        }
        if (p.guard_off) {
            const uint64_t g0 = p.guard_off[rec], glen = p.guard_off[rec + 1] - g0;
            if (glen < 32ull + p.wire_hdr) {
                diff = 1;
            } else if (p.wire_in) {  // the receiver's length field must match the body it got
                const uint8_t* lf = p.wire_in + g0 + 12;
                const uint32_t be = ((uint32_t)lf[0] << 24) | ((uint32_t)lf[1] << 16) |
                                    ((uint32_t)lf[2] << 8) | (uint32_t)lf[3];
                if ((uint64_t)be != glen - p.wire_hdr) diff = 1;
            }
        }
        if (p.and_ok && p.ok[rec] == 0) diff |= 1;  // fused with an earlier check (AEAD tag)
        p.ok[rec] = diff == 0 ? 1 : 0;
        if (diff != 0 && p.zero_on_fail) {
            uint8_t* z = p.zero_on_fail + off;
            for (uint64_t b = 0; b < len; ++b) z[b] = 0;
        }
        return;
    }
    uint8_t* d = p.dest_off ? p.digest + p.dest_off[rec] + len : p.digest + 32ull * rec;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        d[4 * i] = (uint8_t)(st[i] >> 24);
        d[4 * i + 1] = (uint8_t)(st[i] >> 16);
        d[4 * i + 2] = (uint8_t)(st[i] >> 8);
        d[4 * i + 3] = (uint8_t)st[i];
    }
}

hipError_t launch_sha(const ShaParams& p, hipStream_t s) {
    const uint32_t blocks = (p.n + kWG - 1) / kWG;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(sha_kernel, dim3(blocks), dim3(kWG), 0, s, p);
    return hipGetLastError();
}

// KeyManager::derive_key (src/network/KeyManager.cpp:74-92): HMAC-SHA256 with the 32-byte shared
// secret over the 16-byte material BE64(counter) || BE64(ticks) -- four compressions per
// session (ipad, inner message, opad, outer), one session per lane.
__global__ __launch_bounds__(kWG) void session_key_kernel(uint32_t n, const uint8_t* __restrict__ secrets,
                                                          const uint64_t* __restrict__ counters,
                                                          const int64_t* __restrict__ ticks,
                                                          uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * kWG + threadIdx.x;
    if (i >= n) return;
    const uint4* kq = reinterpret_cast<const uint4*>(secrets + 32ull * i);
    const uint4 k0 = kq[0], k1 = kq[1];
    const uint32_t kb[8] = {bswap32(k0.x), bswap32(k0.y), bswap32(k0.z), bswap32(k0.w),
                            bswap32(k1.x), bswap32(k1.y), bswap32(k1.z), bswap32(k1.w)};
    const uint64_t c = counters[i], t = (uint64_t)ticks[i];
    uint32_t st[8], w[16];
    sha_init(st);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = (j < 8 ? kb[j] : 0u) ^ 0x36363636u;
    sha256_compress(st, w);
    w[0] = (uint32_t)(c >> 32); w[1] = (uint32_t)c; w[2] = (uint32_t)(t >> 32); w[3] = (uint32_t)t;
    w[4] = 0x80000000u;
#pragma unroll
    for (int j = 5; j < 15; ++j) w[j] = 0u;
    w[15] = (64 + 16) * 8;
    sha256_compress(st, w);
    uint32_t inner[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) inner[j] = st[j];
    sha_init(st);
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = (j < 8 ? kb[j] : 0u) ^ 0x5c5c5c5cu;
    sha256_compress(st, w);
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = inner[j];
    w[8] = 0x80000000u;
#pragma unroll
    for (int j = 9; j < 15; ++j) w[j] = 0u;
    w[15] = (64 + 32) * 8;
    sha256_compress(st, w);
    uint4* o = reinterpret_cast<uint4*>(out + 32ull * i);
    o[0] = make_uint4(bswap32(st[0]), bswap32(st[1]), bswap32(st[2]), bswap32(st[3]));
    o[1] = make_uint4(bswap32(st[4]), bswap32(st[5]), bswap32(st[6]), bswap32(st[7]));
}

// HMAC-SHA256 midstates of a session-key table (HmacSha256.cpp:11-39 with 32-byte keys: the key
// block is key || 0^32): the states after absorbing key ^ ipad and key ^ opad, one key per lane.
// Frames of one session then start their inner and outer hashes from these (duplex.hip).
__global__ __launch_bounds__(kWG) void hmac_midstate_kernel(uint32_t n, const uint8_t* __restrict__ keys,
                                                            uint32_t* __restrict__ mid) {
    const uint32_t i = blockIdx.x * kWG + threadIdx.x;
    if (i >= n) return;
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(keys + 32ull * i);
    uint32_t kb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) kb[j] = bswap32(kp[j]);
    uint32_t* o = mid + 16ull * i;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t pad = pass == 0 ? 0x36363636u : 0x5c5c5c5cu;
        uint32_t st[8], w[16];
        sha_init(st);
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = (j < 8 ? kb[j] : 0u) ^ pad;
        sha256_compress(st, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[8 * pass + j] = st[j];
    }
}

hipError_t launch_hmac_midstates(uint32_t n, const uint8_t* keys, uint32_t* mid, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(hmac_midstate_kernel, dim3((uint32_t)(((uint64_t)n + kWG - 1) / kWG)), dim3(kWG), 0, s, n, keys, mid);
    return hipGetLastError();
}

hipError_t launch_session_keys(uint32_t n, const uint8_t* secrets, const uint64_t* counters,
                               const int64_t* ticks, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(session_key_kernel, dim3((uint32_t)(((uint64_t)n + kWG - 1) / kWG)), dim3(kWG), 0, s, n, secrets,
                       counters, ticks, out);
    return hipGetLastError();
}

}  // namespace enet
