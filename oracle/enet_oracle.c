/*
 * enet_oracle.c -- CPU restatement of the EphemeralNet crypto hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see enet_oracle.h).  Deliberately scalar and
 * byte-wise, like the reference: this is also the "port" CPU baseline that
 * bench.py times next to the GPU numbers.
 *
 * Reference citations are file:line into ShardianLabs/EphemeralNet @ 2025-11-28.
 */
#include "enet_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- splitmix64 */
static uint64_t splitmix_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void orc_splitmix_bytes(uint64_t seed, uint8_t* out, size_t n) {
    size_t i = 0;
    uint64_t k = 0;
    while (i < n) {
        uint64_t v = splitmix_mix(seed + (k + 1) * 0x9E3779B97F4A7C15ull);
        for (int b = 0; b < 8 && i < n; ++b, ++i) out[i] = (uint8_t)(v >> (8 * b));
        ++k;
    }
}

/* ------------------------------------------------------------------ ChaCha20 */
/* constants "expand 32-byte k": src/crypto/ChaCha20.cpp:11-16 */
static const uint32_t kSigma[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};

static uint32_t rotl32(uint32_t v, int s) { return (v << s) | (v >> (32 - s)); } /* :20-22 */

static uint32_t load32_le(const uint8_t* p) { /* :24-29 */
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static void store32_le(uint8_t* p, uint32_t v) { /* :31-36 */
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

#define QR(a, b, c, d)                 \
    do {                               \
        a += b; d ^= a; d = rotl32(d, 16); \
        c += d; b ^= c; b = rotl32(b, 12); \
        a += b; d ^= a; d = rotl32(d, 8);  \
        c += d; b ^= c; b = rotl32(b, 7);  \
    } while (0) /* quarter_round, ChaCha20.cpp:38-54 */

void orc_chacha20_block(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                        uint8_t out[64]) { /* chacha20_block, ChaCha20.cpp:56-94 */
    uint32_t s[16], x[16];
    for (int i = 0; i < 4; ++i) s[i] = kSigma[i];
    for (int i = 0; i < 8; ++i) s[4 + i] = load32_le(key + 4 * i);
    s[12] = counter;
    s[13] = load32_le(nonce + 0);
    s[14] = load32_le(nonce + 4);
    s[15] = load32_le(nonce + 8);
    memcpy(x, s, sizeof(x));
    for (int i = 0; i < 10; ++i) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) store32_le(out + 4 * i, x[i] + s[i]);
}

void orc_chacha20_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter,
                      const uint8_t* in, uint8_t* out, size_t n) { /* ChaCha20::apply :98-121 */
    uint8_t ks[64];
    size_t done = 0;
    while (done < n) {
        orc_chacha20_block(key, nonce, counter, ks);
        ++counter; /* uint32_t: wraps mod 2^32 with the nonce unchanged (:110) */
        size_t b = n - done < 64 ? n - done : 64;
        for (size_t i = 0; i < b; ++i) out[done + i] = (uint8_t)(in[done + i] ^ ks[i]);
        done += b;
    }
    memset(ks, 0, sizeof(ks));
}

uint32_t orc_derive_counter(const uint8_t id[32]) { /* CryptoManager.cpp:8-13 */
    return (uint32_t)id[0] | ((uint32_t)id[1] << 8) | ((uint32_t)id[2] << 16) |
           ((uint32_t)id[3] << 24);
}

/* ------------------------------------------------------------------- SHA-256 */
static const uint32_t kK[64] = { /* FIPS 180-4 4.2.2; Sha256.cpp:10-20 */
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

static uint32_t rotr32(uint32_t v, int s) { return (v >> s) | (v << (32 - s)); }

typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    size_t fill;
    uint64_t bits;
} sha_ctx;

static void sha_transform(uint32_t st[8], const uint8_t blk[64]) { /* Sha256.cpp:134-176 */
    uint32_t w[64];
    for (int i = 0; i < 16; ++i)
        w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
               ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
        uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = s1 + w[i - 7] + s0 + w[i - 16];
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; ++i) {
        uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) +
                      kK[i] + w[i];
        uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

static void sha_init(sha_ctx* c) { /* Sha256.cpp:66-70 */
    static const uint32_t iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    memcpy(c->h, iv, sizeof(iv));
    c->fill = 0;
    c->bits = 0;
}

static void sha_update(sha_ctx* c, const uint8_t* p, size_t n) { /* Sha256.cpp:72-92 */
    c->bits += (uint64_t)n * 8;
    while (n) {
        size_t take = 64 - c->fill < n ? 64 - c->fill : n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += take; p += take; n -= take;
        if (c->fill == 64) { sha_transform(c->h, c->buf); c->fill = 0; }
    }
}

static void sha_final(sha_ctx* c, uint8_t out[32]) { /* Sha256.cpp:94-126 */
    c->buf[c->fill++] = 0x80;
    if (c->fill > 56) {
        memset(c->buf + c->fill, 0, 64 - c->fill);
        sha_transform(c->h, c->buf);
        c->fill = 0;
    }
    memset(c->buf + c->fill, 0, 56 - c->fill);
    for (int i = 0; i < 8; ++i) c->buf[56 + i] = (uint8_t)(c->bits >> (56 - 8 * i));
    sha_transform(c->h, c->buf);
    for (int i = 0; i < 8; ++i) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8);
        out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

void orc_sha256(const uint8_t* data, size_t n, uint8_t out[32]) { /* Sha256::digest :128-132 */
    sha_ctx c;
    sha_init(&c);
    sha_update(&c, data, n);
    sha_final(&c, out);
}

void orc_hmac_sha256(const uint8_t* key, size_t klen, const uint8_t* data, size_t n,
                     uint8_t out[32]) { /* HmacSha256::compute, HmacSha256.cpp:11-39 */
    uint8_t kb[64] = {0}, ipad[64], opad[64], inner[32];
    if (klen > 64) orc_sha256(key, klen, kb); /* keys over 64 B are hashed first (:15-17) */
    else if (klen) memcpy(kb, key, klen);
    for (int i = 0; i < 64; ++i) { ipad[i] = kb[i] ^ 0x36; opad[i] = kb[i] ^ 0x5c; }
    sha_ctx c;
    sha_init(&c); sha_update(&c, ipad, 64); sha_update(&c, data, n); sha_final(&c, inner);
    sha_init(&c); sha_update(&c, opad, 64); sha_update(&c, inner, 32); sha_final(&c, out);
}

int orc_hmac_sha256_verify(const uint8_t* key, size_t klen, const uint8_t* data, size_t n,
                           const uint8_t* mac, size_t maclen) { /* HmacSha256.cpp:41-54 */
    if (maclen != 32) return 0;
    uint8_t e[32], diff = 0;
    orc_hmac_sha256(key, klen, data, n, e);
    for (int i = 0; i < 32; ++i) diff |= (uint8_t)(e[i] ^ mac[i]);
    return diff == 0;
}

/* ------------------------------------------------------------------ Poly1305 */
/* RFC 8439 2.5, restated over three limbs of radix 2^44 / 2^44 / 2^42 held in
 * uint64_t with unsigned __int128 products (independent of the GPU kernel's
 * five 26-bit limbs, so the two formulations check each other). */
typedef unsigned __int128 u128;
#define M44 0xfffffffffffull
#define M42 0x3ffffffffffull

typedef struct {
    uint64_t r0, r1, r2, s1, s2, h0, h1, h2, pad0, pad1;
    uint8_t buf[16];
    size_t fill;
} poly_ctx;

static uint64_t le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

static void poly_init(poly_ctx* c, const uint8_t key[32]) {
    uint64_t t0 = le64(key) & 0x0ffffffc0fffffffull; /* clamp r (RFC 8439 2.5.1) */
    uint64_t t1 = le64(key + 8) & 0x0ffffffc0ffffffcull;
    c->r0 = t0 & M44;
    c->r1 = ((t0 >> 44) | (t1 << 20)) & M44;
    c->r2 = (t1 >> 24) & M42;
    c->s1 = c->r1 * 20; /* 2^132 = 4 * 2^130 == 4 * 5 (mod p) */
    c->s2 = c->r2 * 20;
    c->h0 = c->h1 = c->h2 = 0;
    c->pad0 = le64(key + 16);
    c->pad1 = le64(key + 24);
    c->fill = 0;
}

static void poly_block(poly_ctx* c, const uint8_t m[16], uint64_t hibit) {
    uint64_t t0 = le64(m), t1 = le64(m + 8);
    uint64_t h0 = c->h0 + (t0 & M44);
    uint64_t h1 = c->h1 + (((t0 >> 44) | (t1 << 20)) & M44);
    uint64_t h2 = c->h2 + (((t1 >> 24) & M42) | (hibit << 40));
    u128 d0 = (u128)h0 * c->r0 + (u128)h1 * c->s2 + (u128)h2 * c->s1;
    u128 d1 = (u128)h0 * c->r1 + (u128)h1 * c->r0 + (u128)h2 * c->s2;
    u128 d2 = (u128)h0 * c->r2 + (u128)h1 * c->r1 + (u128)h2 * c->r0;
    uint64_t k;
    k = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & M44; d1 += k;
    k = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & M44; d2 += k;
    k = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & M42;
    h0 += k * 5; k = h0 >> 44; h0 &= M44; h1 += k;
    c->h0 = h0; c->h1 = h1; c->h2 = h2;
}

static void poly_update(poly_ctx* c, const uint8_t* p, size_t n) {
    while (n) {
        size_t take = 16 - c->fill < n ? 16 - c->fill : n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += take; p += take; n -= take;
        if (c->fill == 16) { poly_block(c, c->buf, 1); c->fill = 0; }
    }
}

static void poly_final(poly_ctx* c, uint8_t tag[16]) {
    if (c->fill) { /* partial block: append 0x01, zero-fill, no 2^128 bit */
        c->buf[c->fill] = 1;
        memset(c->buf + c->fill + 1, 0, 15 - c->fill);
        poly_block(c, c->buf, 0);
    }
    uint64_t h0 = c->h0, h1 = c->h1, h2 = c->h2, k;
    for (int pass = 0; pass < 2; ++pass) { /* fully propagate carries */
        k = h1 >> 44; h1 &= M44; h2 += k;
        k = h2 >> 42; h2 &= M42; h0 += k * 5;
        k = h0 >> 44; h0 &= M44; h1 += k;
    }
    /* g = h + 5 - 2^130; keep g if it did not borrow (h >= p) */
    uint64_t g0 = h0 + 5; k = g0 >> 44; g0 &= M44;
    uint64_t g1 = h1 + k; k = g1 >> 44; g1 &= M44;
    uint64_t g2 = h2 + k - (1ull << 42);
    uint64_t keep_g = (g2 >> 63) - 1; /* all-ones when no borrow */
    h0 = (h0 & ~keep_g) | (g0 & keep_g);
    h1 = (h1 & ~keep_g) | (g1 & keep_g);
    h2 = (h2 & ~keep_g) | (g2 & keep_g & M42);
    uint64_t lo = h0 | (h1 << 44);
    uint64_t hi = (h1 >> 20) | (h2 << 24);
    u128 acc = ((u128)hi << 64 | lo) + ((u128)c->pad1 << 64 | c->pad0); /* mod 2^128 */
    for (int i = 0; i < 16; ++i) tag[i] = (uint8_t)(acc >> (8 * i));
}

void orc_poly1305(const uint8_t key[32], const uint8_t* msg, size_t n, uint8_t tag[16]) {
    poly_ctx c;
    poly_init(&c, key);
    poly_update(&c, msg, n);
    poly_final(&c, tag);
}

/* RFC 8439 2.8: otk = block(ctr 0)[0..32); ct = ChaCha20(ctr 1); mac over
 * aad || pad16 || ct || pad16 || LE64(|aad|) || LE64(|ct|). */
static void aead_tag(const uint8_t otk[32], const uint8_t* aad, size_t aad_len,
                     const uint8_t* ct, size_t n, uint8_t tag[16]) {
    static const uint8_t zeros[16] = {0};
    uint8_t lens[16];
    poly_ctx c;
    poly_init(&c, otk);
    poly_update(&c, aad, aad_len);
    if (aad_len % 16) poly_update(&c, zeros, 16 - aad_len % 16);
    poly_update(&c, ct, n);
    if (n % 16) poly_update(&c, zeros, 16 - n % 16);
    for (int i = 0; i < 8; ++i) {
        lens[i] = (uint8_t)((uint64_t)aad_len >> (8 * i));
        lens[8 + i] = (uint8_t)((uint64_t)n >> (8 * i));
    }
    poly_update(&c, lens, 16);
    poly_final(&c, tag);
}

void orc_aead_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                   size_t aad_len, const uint8_t* pt, size_t n, uint8_t* ct, uint8_t tag[16]) {
    uint8_t blk[64];
    orc_chacha20_block(key, nonce, 0, blk);
    orc_chacha20_xor(key, nonce, 1, pt, ct, n);
    aead_tag(blk, aad, aad_len, ct, n, tag);
    memset(blk, 0, sizeof(blk));
}

int orc_aead_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                  size_t aad_len, const uint8_t* ct, size_t n, const uint8_t tag[16],
                  uint8_t* pt) {
    uint8_t blk[64], t[16], diff = 0;
    orc_chacha20_block(key, nonce, 0, blk);
    aead_tag(blk, aad, aad_len, ct, n, t);
    for (int i = 0; i < 16; ++i) diff |= (uint8_t)(t[i] ^ tag[i]);
    orc_chacha20_xor(key, nonce, 1, ct, pt, n);
    memset(blk, 0, sizeof(blk));
    return diff == 0;
}

/* -------------------------------------------------------------- frame codec */
void orc_frame_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* m, size_t n,
                    uint8_t* body) {
    uint8_t* tmp = (uint8_t*)malloc(n + 32);
    if (n) memcpy(tmp, m, n);
    orc_hmac_sha256(key, 32, m, n, tmp + n);          /* encode_signed, Message.cpp:305-311 */
    orc_chacha20_xor(key, nonce, 0, tmp, body, n + 32); /* SessionManager.cpp:374 */
    free(tmp);
}

int orc_frame_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* body,
                   size_t body_len, uint8_t* m_out) {
    if (body_len < 32) return 0; /* decode_signed rejects short buffers, Message.cpp:315 */
    uint8_t* tmp = (uint8_t*)malloc(body_len);
    orc_chacha20_xor(key, nonce, 0, body, tmp, body_len); /* SessionManager.cpp:822 */
    size_t n = body_len - 32;
    int ok = orc_hmac_sha256_verify(key, 32, tmp, n, tmp + n, 32); /* Message.cpp:323 */
    if (n) memcpy(m_out, tmp, n);
    free(tmp);
    return ok;
}

/* ------------------------------------------------------------ proof of work */
void orc_mt64_seed(orc_mt64* g, uint64_t seed) { /* std::mersenne_twister_engine::seed */
    g->mt[0] = seed;
    for (int i = 1; i < 312; ++i)
        g->mt[i] = 6364136223846793005ull * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
    g->mti = 312;
}

uint64_t orc_mt64_next(orc_mt64* g) {
    if (g->mti >= 312) { /* twist, in place, index order */
        for (int i = 0; i < 312; ++i) {
            const uint64_t x = (g->mt[i] & 0xFFFFFFFF80000000ull) | (g->mt[(i + 1) % 312] & 0x7FFFFFFFull);
            g->mt[i] = g->mt[(i + 156) % 312] ^ (x >> 1) ^ ((x & 1u) ? 0xB5026F5AA96619E9ull : 0ull);
        }
        g->mti = 0;
    }
    uint64_t y = g->mt[g->mti++];
    y ^= (y >> 29) & 0x5555555555555555ull;
    y ^= (y << 17) & 0x71D67FFFEDA60000ull;
    y ^= (y << 37) & 0xFFF7EEE000000000ull;
    y ^= y >> 43;
    return y;
}

unsigned orc_leading_zero_bits(const uint8_t d[32]) { /* Node.cpp:174-190 */
    unsigned total = 0;
    for (int i = 0; i < 32; ++i) {
        if (d[i] == 0) { total += 8; continue; }
        for (int bit = 7; bit >= 0; --bit) {
            if ((d[i] >> bit) & 1u) return total;
            ++total;
        }
    }
    return total;
}

static void be64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (56 - 8 * i));
}

void orc_pow_digest(const uint8_t* prefix, size_t plen, uint64_t nonce, uint8_t out[32]) {
    sha_ctx c;
    uint8_t nb[8];
    sha_init(&c);
    sha_update(&c, prefix, plen);
    be64(nb, nonce); /* to_big_endian(nonce), StoreProof.cpp:50 / Node.cpp:168 */
    sha_update(&c, nb, 8);
    sha_final(&c, out);
}

size_t orc_store_pow_prefix(const uint8_t chunk_id[32], uint64_t payload_size, const uint8_t* hint,
                            size_t hint_len, uint8_t* out) {
    size_t o = 0;
    memcpy(out, chunk_id, 32); o += 32;          /* :41 */
    be64(out + o, payload_size); o += 8;         /* :42 */
    const uint32_t l = hint_len > 0xFFFFFFFFu ? 0xFFFFFFFFu : (uint32_t)hint_len; /* :26 */
    out[o++] = (uint8_t)(l >> 24); out[o++] = (uint8_t)(l >> 16);
    out[o++] = (uint8_t)(l >> 8); out[o++] = (uint8_t)l;
    if (hint_len) { memcpy(out + o, hint, hint_len); o += hint_len; }
    return o;
}

static size_t lp64(uint8_t* out, const uint8_t* p, size_t n) { /* Node.cpp:149-153 */
    be64(out, (uint64_t)n);
    if (n) memcpy(out + 8, p, n);
    return 8 + n;
}

size_t orc_announce_pow_prefix(const uint8_t chunk_id[32], const uint8_t peer_id[32],
                               const uint8_t* endpoint, size_t elen, const uint8_t* uri,
                               size_t ulen, const uint8_t* shards, size_t slen, int64_t ttl,
                               uint8_t* out) {
    size_t o = 0;
    o += lp64(out + o, chunk_id, 32);
    o += lp64(out + o, peer_id, 32);
    o += lp64(out + o, endpoint, elen);
    o += lp64(out + o, uri, ulen);
    o += lp64(out + o, shards, slen);
    be64(out + o, (uint64_t)ttl); o += 8; /* Node.cpp:165-166 */
    return o;
}

size_t orc_handshake_pow_prefix(const uint8_t initiator[32], const uint8_t responder[32],
                                uint32_t initiator_public, uint8_t* out) {
    size_t o = 0;
    o += lp64(out + o, initiator, 32);
    o += lp64(out + o, responder, 32);
    be64(out + o, (uint64_t)initiator_public); o += 8; /* Node.cpp:241-242 */
    return o;
}

int orc_pow_check(const uint8_t* prefix, size_t plen, uint64_t nonce, unsigned difficulty) {
    if (difficulty == 0) return 1;
    uint8_t d[32];
    orc_pow_digest(prefix, plen, nonce, d);
    return orc_leading_zero_bits(d) >= difficulty;
}

int orc_pow_search(const uint8_t* prefix, size_t plen, unsigned difficulty, int schedule,
                   uint64_t max_attempts, uint64_t* nonce, uint64_t* attempt) {
    if (difficulty == 0) { *nonce = 0; *attempt = 0; return 1; }
    uint8_t d[32];
    orc_pow_digest(prefix, plen, 0, d);
    uint64_t seed = 0;
    if (schedule == 1) { /* memcpy(&seed, digest, 8), StoreProof.cpp:136-137 */
        for (int i = 7; i >= 0; --i) seed = (seed << 8) | d[i];
    } else {             /* Node.cpp:205-207 / 261-263 */
        for (int i = 0; i < 8; ++i) seed = (seed << 8) | d[i];
    }
    orc_mt64 g;
    orc_mt64_seed(&g, seed);
    const uint64_t start = schedule == 1 ? 0 : orc_mt64_next(&g);
    for (uint64_t a = 0; a < max_attempts; ++a) {
        const uint64_t cand = schedule == 1 ? orc_mt64_next(&g) : start + a;
        if (orc_pow_check(prefix, plen, cand, difficulty)) {
            *nonce = cand;
            *attempt = a;
            return 1;
        }
    }
    return 0;
}

/* ------------------------------------------------ session key derivation */
void orc_session_key(const uint8_t secret[32], uint64_t counter, int64_t ticks, uint8_t out[32]) {
    uint8_t m[16];
    be64(m, counter);          /* KeyManager.cpp:79-81 */
    be64(m + 8, (uint64_t)ticks); /* :83-86 */
    orc_hmac_sha256(secret, 32, m, 16, out); /* :88-90 */
}

/* ----------------------------------------------------------- CPU baseline */
typedef struct {
    const uint8_t *pt, *keys, *nonces;
    uint8_t *ct, *back, *tags;
    size_t lo, hi, len;
    int phase, fails;
} bench_job;

static void* bench_worker(void* arg) {
    bench_job* j = (bench_job*)arg;
    for (size_t i = j->lo; i < j->hi; ++i) {
        const uint8_t* k = j->keys + 32 * i;
        const uint8_t* nn = j->nonces + 12 * i;
        if (j->phase == 0)
            orc_aead_seal(k, nn, NULL, 0, j->pt + i * j->len, j->len, j->ct + i * j->len,
                          j->tags + 16 * i);
        else
            j->fails += !orc_aead_open(k, nn, NULL, 0, j->ct + i * j->len, j->len,
                                       j->tags + 16 * i, j->back + i * j->len);
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int orc_bench_aead(const uint8_t* pt, uint8_t* ct, uint8_t* back, const uint8_t* keys,
                   const uint8_t* nonces, uint8_t* tags, size_t n, size_t len, int threads,
                   double out_seconds[2]) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    bench_job* jobs = (bench_job*)calloc((size_t)threads, sizeof(bench_job));
    int fails = 0;
    for (int phase = 0; phase < 2; ++phase) {
        double t0 = now_s();
        for (int t = 0; t < threads; ++t) {
            bench_job* j = &jobs[t];
            j->pt = pt; j->keys = keys; j->nonces = nonces; j->ct = ct; j->back = back;
            j->tags = tags; j->len = len; j->phase = phase; j->fails = 0;
            j->lo = n * (size_t)t / (size_t)threads;
            j->hi = n * (size_t)(t + 1) / (size_t)threads;
            pthread_create(&th[t], NULL, bench_worker, j);
        }
        for (int t = 0; t < threads; ++t) {
            pthread_join(th[t], NULL);
            fails += jobs[t].fails;
        }
        out_seconds[phase] = now_s() - t0;
    }
    free(th);
    free(jobs);
    return fails;
}

typedef struct {
    const uint8_t* prefixes;
    const uint64_t* off;
    size_t lo, hi;
    unsigned difficulty;
    uint64_t max_attempts, hashes;
} pow_job;

static void* pow_worker(void* arg) {
    pow_job* j = (pow_job*)arg;
    for (size_t i = j->lo; i < j->hi; ++i) {
        uint64_t nonce = 0, at = 0;
        const int f = orc_pow_search(j->prefixes + j->off[i], (size_t)(j->off[i + 1] - j->off[i]),
                                     j->difficulty, 0, j->max_attempts, &nonce, &at);
        j->hashes += 1 + (f ? at + 1 : j->max_attempts); /* + the seed digest */
    }
    return NULL;
}

double orc_bench_pow(const uint8_t* prefixes, const uint64_t* offsets, size_t jobs,
                     unsigned difficulty, uint64_t max_attempts, int threads, uint64_t* hashes) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    pow_job* js = (pow_job*)calloc((size_t)threads, sizeof(pow_job));
    const double t0 = now_s();
    for (int t = 0; t < threads; ++t) {
        pow_job* j = &js[t];
        j->prefixes = prefixes; j->off = offsets; j->difficulty = difficulty;
        j->max_attempts = max_attempts;
        j->lo = jobs * (size_t)t / (size_t)threads;
        j->hi = jobs * (size_t)(t + 1) / (size_t)threads;
        pthread_create(&th[t], NULL, pow_worker, j);
    }
    uint64_t h = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        h += js[t].hashes;
    }
    const double dt = now_s() - t0;
    free(th);
    free(js);
    *hashes = h;
    return dt;
}
