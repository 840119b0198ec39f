// enet_device.hpp -- CDNA4 (gfx950) device primitives for the bulk crypto engine.
//
// ChaCha20 state words live in VGPRs, one 64-byte block per lane; quarter-rounds are 32-bit
// ARX (v_add_u32 / v_xor_b32 / v_alignbit_b32).  Poly1305 uses five 26-bit limbs with 64-bit
// partial products (v_mad_u64_u32).  SHA-256 is one record per lane.  No MFMA anywhere: none of
// this is a dense contraction.
//
// Reference behaviour restated here (file:line into ShardianLabs/EphemeralNet):
//   ChaCha20 block / quarter round     src/crypto/ChaCha20.cpp:38-94
//   ChaCha20::apply u32 counter wrap   src/crypto/ChaCha20.cpp:110
//   SHA-256 compression               src/crypto/Sha256.cpp:134-176
// Poly1305 has no reference implementation; it follows RFC 8439 2.5.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chacha_lockstep_asm.hpp"

namespace enet {

// ----------------------------------------------------------------------------- ChaCha20
constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u,
                   kSigma3 = 0x6b206574u;  // "expand 32-byte k", ChaCha20.cpp:11-16

__device__ __forceinline__ uint32_t rotl(uint32_t v, int s) { return __builtin_rotateleft32(v, s); }

#define ENET_QR(a, b, c, d)                  \
    do {                                     \
        a += b; d ^= a; d = rotl(d, 16);     \
        c += d; b ^= c; b = rotl(b, 12);     \
        a += b; d ^= a; d = rotl(d, 8);      \
        c += d; b ^= c; b = rotl(b, 7);      \
    } while (0)

// Per-record ChaCha20 constants.  The first column round's quarter-rounds on columns 1..3 do
// not involve the block counter (word 12), so they are computed once per record and reused for
// every block of that record; only column 0 is recomputed per block.
struct ChachaRecord {
    uint32_t k[8];      // key words (feed-forward)
    uint32_t n[3];      // nonce words (feed-forward)
    uint32_t pre[12];   // columns 1..3 after the first column round: x1,x5,x9,x13,x2,...,x15
};

__device__ __forceinline__ void chacha_record_init(ChachaRecord& R, const uint32_t k[8],
                                                   const uint32_t n[3]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) R.k[i] = k[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) R.n[i] = n[i];
    uint32_t a1 = kSigma1, b1 = k[1], c1 = k[5], d1 = n[0];
    uint32_t a2 = kSigma2, b2 = k[2], c2 = k[6], d2 = n[1];
    uint32_t a3 = kSigma3, b3 = k[3], c3 = k[7], d3 = n[2];
    ENET_QR(a1, b1, c1, d1);
    ENET_QR(a2, b2, c2, d2);
    ENET_QR(a3, b3, c3, d3);
    R.pre[0] = a1; R.pre[1] = b1; R.pre[2] = c1; R.pre[3] = d1;
    R.pre[4] = a2; R.pre[5] = b2; R.pre[6] = c2; R.pre[7] = d2;
    R.pre[8] = a3; R.pre[9] = b3; R.pre[10] = c3; R.pre[11] = d3;
}

// Keystream block for `counter` (chacha20_block, ChaCha20.cpp:56-94), as 16 LE words.
__device__ __forceinline__ void chacha_block(const ChachaRecord& R, uint32_t counter,
                                             uint32_t x[16]) {
    uint32_t x0 = kSigma0, x4 = R.k[0], x8 = R.k[4], x12 = counter;
    ENET_QR(x0, x4, x8, x12);
    uint32_t x1 = R.pre[0], x5 = R.pre[1], x9 = R.pre[2], x13 = R.pre[3];
    uint32_t x2 = R.pre[4], x6 = R.pre[5], x10 = R.pre[6], x14 = R.pre[7];
    uint32_t x3 = R.pre[8], x7 = R.pre[9], x11 = R.pre[10], x15 = R.pre[11];
    // rest of double round 1: diagonal round
    ENET_QR(x0, x5, x10, x15);
    ENET_QR(x1, x6, x11, x12);
    ENET_QR(x2, x7, x8, x13);
    ENET_QR(x3, x4, x9, x14);
#pragma unroll
    for (int i = 1; i < 10; ++i) {
        ENET_QR(x0, x4, x8, x12);
        ENET_QR(x1, x5, x9, x13);
        ENET_QR(x2, x6, x10, x14);
        ENET_QR(x3, x7, x11, x15);
        ENET_QR(x0, x5, x10, x15);
        ENET_QR(x1, x6, x11, x12);
        ENET_QR(x2, x7, x8, x13);
        ENET_QR(x3, x4, x9, x14);
    }
    x[0] = x0 + kSigma0; x[1] = x1 + kSigma1; x[2] = x2 + kSigma2; x[3] = x3 + kSigma3;
    x[4] = x4 + R.k[0]; x[5] = x5 + R.k[1]; x[6] = x6 + R.k[2]; x[7] = x7 + R.k[3];
    x[8] = x8 + R.k[4]; x[9] = x9 + R.k[5]; x[10] = x10 + R.k[6]; x[11] = x11 + R.k[7];
    x[12] = x12 + counter; x[13] = x13 + R.n[0]; x[14] = x14 + R.n[1]; x[15] = x15 + R.n[2];
}

// Two keystream blocks of the same record, quarter-rounds interleaved (8 independent ARX
// chains instead of 4) so a wave always has independent VALU work in flight.
__device__ __forceinline__ void chacha_block2(const ChachaRecord& R, uint32_t ca, uint32_t cb,
                                              uint32_t xa[16], uint32_t xb[16]) {
    uint32_t a0 = kSigma0, a4 = R.k[0], a8 = R.k[4], a12 = ca;
    uint32_t b0 = kSigma0, b4 = R.k[0], b8 = R.k[4], b12 = cb;
    ENET_QR(a0, a4, a8, a12);
    ENET_QR(b0, b4, b8, b12);
    uint32_t a1 = R.pre[0], a5 = R.pre[1], a9 = R.pre[2], a13 = R.pre[3];
    uint32_t a2 = R.pre[4], a6 = R.pre[5], a10 = R.pre[6], a14 = R.pre[7];
    uint32_t a3 = R.pre[8], a7 = R.pre[9], a11 = R.pre[10], a15 = R.pre[11];
    uint32_t b1 = a1, b5 = a5, b9 = a9, b13 = a13;
    uint32_t b2 = a2, b6 = a6, b10 = a10, b14 = a14;
    uint32_t b3 = a3, b7 = a7, b11 = a11, b15 = a15;
    ENET_QR(a0, a5, a10, a15); ENET_QR(b0, b5, b10, b15);
    ENET_QR(a1, a6, a11, a12); ENET_QR(b1, b6, b11, b12);
    ENET_QR(a2, a7, a8, a13);  ENET_QR(b2, b7, b8, b13);
    ENET_QR(a3, a4, a9, a14);  ENET_QR(b3, b4, b9, b14);
#pragma unroll
    for (int i = 1; i < 10; ++i) {
        ENET_QR(a0, a4, a8, a12);  ENET_QR(b0, b4, b8, b12);
        ENET_QR(a1, a5, a9, a13);  ENET_QR(b1, b5, b9, b13);
        ENET_QR(a2, a6, a10, a14); ENET_QR(b2, b6, b10, b14);
        ENET_QR(a3, a7, a11, a15); ENET_QR(b3, b7, b11, b15);
        ENET_QR(a0, a5, a10, a15); ENET_QR(b0, b5, b10, b15);
        ENET_QR(a1, a6, a11, a12); ENET_QR(b1, b6, b11, b12);
        ENET_QR(a2, a7, a8, a13);  ENET_QR(b2, b7, b8, b13);
        ENET_QR(a3, a4, a9, a14);  ENET_QR(b3, b4, b9, b14);
    }
    xa[0] = a0 + kSigma0; xa[1] = a1 + kSigma1; xa[2] = a2 + kSigma2; xa[3] = a3 + kSigma3;
    xa[4] = a4 + R.k[0]; xa[5] = a5 + R.k[1]; xa[6] = a6 + R.k[2]; xa[7] = a7 + R.k[3];
    xa[8] = a8 + R.k[4]; xa[9] = a9 + R.k[5]; xa[10] = a10 + R.k[6]; xa[11] = a11 + R.k[7];
    xa[12] = a12 + ca; xa[13] = a13 + R.n[0]; xa[14] = a14 + R.n[1]; xa[15] = a15 + R.n[2];
    xb[0] = b0 + kSigma0; xb[1] = b1 + kSigma1; xb[2] = b2 + kSigma2; xb[3] = b3 + kSigma3;
    xb[4] = b4 + R.k[0]; xb[5] = b5 + R.k[1]; xb[6] = b6 + R.k[2]; xb[7] = b7 + R.k[3];
    xb[8] = b8 + R.k[4]; xb[9] = b9 + R.k[5]; xb[10] = b10 + R.k[6]; xb[11] = b11 + R.k[7];
    xb[12] = b12 + cb; xb[13] = b13 + R.n[0]; xb[14] = b14 + R.n[1]; xb[15] = b15 + R.n[2];
}

// Two keystream blocks with the quarter-round steps of all 8 chains issued in a fixed order
// (step s of every chain, then step s+1 ...) as one asm statement per instruction, and an
// s_barrier after every 24 instructions (one add / xor / rotate step of the 8 chains).  With both
// waves of a SIMD in one workgroup, the barrier keeps them in phase, so their full-rate v_add /
// v_xor runs line up and pair on gfx950's dual-rate VALU instead of colliding with the other
// wave's half-rate v_alignbit runs (tools/ubench_pair.hip: 4.29 -> 3.69 cycles per instruction).
// Every wave of the workgroup must call this the same number of times.
#define ENET_ASM_ADD(x, y) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(y))
#define ENET_ASM_XOR(x, y) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(x) : "v"(y))
#define ENET_ASM_ROT(x, r) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(x) : "I"(32 - (r)))

// one half-round (four QRs on quads Q of both blocks), steps interleaved across the 8 chains
template <bool DIAG>
__device__ __forceinline__ void chacha_half_lockstep(uint32_t x[32]) {
    constexpr int C[4][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15}};
    constexpr int D[4][4] = {{0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
    constexpr int R[4] = {16, 12, 8, 7};
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // QR line k: (a += b, d ^= a, d <<<= 16) / (c += d, b ^= c, b <<<= 12) ...
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int* q = DIAG ? D[c & 3] : C[c & 3];
            const int o = 16 * (c >> 2);
            if (k % 2 == 0) ENET_ASM_ADD(x[o + q[0]], x[o + q[1]]);
            else ENET_ASM_ADD(x[o + q[2]], x[o + q[3]]);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int* q = DIAG ? D[c & 3] : C[c & 3];
            const int o = 16 * (c >> 2);
            if (k % 2 == 0) ENET_ASM_XOR(x[o + q[3]], x[o + q[0]]);
            else ENET_ASM_XOR(x[o + q[1]], x[o + q[2]]);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int* q = DIAG ? D[c & 3] : C[c & 3];
            const int o = 16 * (c >> 2);
            if (k % 2 == 0) ENET_ASM_ROT(x[o + q[3]], R[k]);
            else ENET_ASM_ROT(x[o + q[1]], R[k]);
        }
#ifndef ENET_LOCK_EVERY
#define ENET_LOCK_EVERY 1
#endif
        if ((k + 1) % ENET_LOCK_EVERY == 0) __builtin_amdgcn_s_barrier();
    }
}

// The same half-round with each step (8 adds, 8 xors, 8 rotates, s_barrier) as ONE asm
// statement whose operands are all 32 state words (chacha_lockstep_asm.hpp, generated by
// tools/gen/gen_lockstep.py).  Single-instruction statements also get an s_nop 0 from the
// compiler's inline-asm hazard check at every add / xor / rotate group boundary, and statements
// naming only the words they touch make the register allocator shuffle words between VGPRs
// (~15 v_mov per step) once the rounds are a loop; with all 32 words tied there is neither.
// sh(base + k) runs after step k (k = 0..3), pinned there by compiler memory barriers.
struct NoStepHook {
    __device__ __forceinline__ void operator()(int) const {}
};
// BAR: s_barrier after every step (1), after steps 1 and 3 (2), after step 3 (4), never (0).
template <bool DIAG, class SH = NoStepHook, int BAR = 1>
__device__ __forceinline__ void chacha_half_lockstep2(uint32_t x[32], SH&& sh = SH{}, int base = 0) {
    auto after = [&](int k) {
        asm volatile("" ::: "memory");
        sh(base + k);
        asm volatile("" ::: "memory");
    };
    constexpr bool b0 = BAR == 1, b1 = BAR == 1 || BAR == 2, b2 = BAR == 1, b3 = BAR != 0;
#define ENET_LS_STEP(NAME, B)                               \
    do {                                                    \
        if constexpr (B) asm volatile(NAME ENET_LS_X32(x)); \
        else asm volatile(NAME##_NB ENET_LS_X32(x));        \
    } while (0)
    if constexpr (DIAG) {
        ENET_LS_STEP(ENET_LS_D0, b0);
        after(0);
        ENET_LS_STEP(ENET_LS_D1, b1);
        after(1);
        ENET_LS_STEP(ENET_LS_D2, b2);
        after(2);
        ENET_LS_STEP(ENET_LS_D3, b3);
        after(3);
    } else {
        ENET_LS_STEP(ENET_LS_C0, b0);
        after(0);
        ENET_LS_STEP(ENET_LS_C1, b1);
        after(1);
        ENET_LS_STEP(ENET_LS_C2, b2);
        after(2);
        ENET_LS_STEP(ENET_LS_C3, b3);
        after(3);
    }
#undef ENET_LS_STEP
}

__device__ __forceinline__ void chacha_block2_lockstep(const ChachaRecord& R, uint32_t ca, uint32_t cb,
                                                       uint32_t xa[16], uint32_t xb[16]) {
    uint32_t a0 = kSigma0, a4 = R.k[0], a8 = R.k[4], a12 = ca;
    uint32_t b0 = kSigma0, b4 = R.k[0], b8 = R.k[4], b12 = cb;
    ENET_QR(a0, a4, a8, a12);
    ENET_QR(b0, b4, b8, b12);
    uint32_t x[32];
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
    chacha_half_lockstep2<true>(x);
#pragma unroll
    for (int i = 1; i < 10; ++i) {
        chacha_half_lockstep2<false>(x);
        chacha_half_lockstep2<true>(x);
    }
    const uint32_t ff[16] = {kSigma0, kSigma1, kSigma2, kSigma3, R.k[0], R.k[1], R.k[2], R.k[3],
                             R.k[4], R.k[5], R.k[6], R.k[7], 0u, R.n[0], R.n[1], R.n[2]};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        xa[i] = x[i] + (i == 12 ? ca : ff[i]);
        xb[i] = x[16 + i] + (i == 12 ? cb : ff[i]);
    }
}

// ----------------------------------------------------------------------------- Poly1305
// Field elements mod 2^130-5 in five 26-bit limbs.  `Pmul` holds a multiplier and its 5x
// multiples (2^130 == 5), so h*r needs 25 v_mad_u64_u32 and a short carry chain.
constexpr uint32_t M26 = 0x3ffffffu;

struct Pmul {
    uint32_t r[5];
    uint32_t s[5];  // s[i] = 5 * r[i] (s[0] unused)
};

__device__ __forceinline__ Pmul pmul_make(const uint32_t r[5]) {
    Pmul m;
#pragma unroll
    for (int i = 0; i < 5; ++i) { m.r[i] = r[i]; m.s[i] = r[i] * 5u; }
    return m;
}

// h <- h * m (mod 2^130-5), partially reduced: limbs < 2^26 except h1 < 2^26 + 2^6.
// Inputs: limbs of h < 2^27, limbs of m.r < 2^26 (so the 64-bit sums stay < 2^58).
__device__ __forceinline__ void pmul(uint32_t h[5], const Pmul& m) {
    const uint64_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
    uint64_t d0 = h0 * m.r[0] + h1 * m.s[4] + h2 * m.s[3] + h3 * m.s[2] + h4 * m.s[1];
    uint64_t d1 = h0 * m.r[1] + h1 * m.r[0] + h2 * m.s[4] + h3 * m.s[3] + h4 * m.s[2];
    uint64_t d2 = h0 * m.r[2] + h1 * m.r[1] + h2 * m.r[0] + h3 * m.s[4] + h4 * m.s[3];
    uint64_t d3 = h0 * m.r[3] + h1 * m.r[2] + h2 * m.r[1] + h3 * m.r[0] + h4 * m.s[4];
    uint64_t d4 = h0 * m.r[4] + h1 * m.r[3] + h2 * m.r[2] + h3 * m.r[1] + h4 * m.r[0];
    uint32_t c;
    c = (uint32_t)(d0 >> 26); h[0] = (uint32_t)d0 & M26; d1 += c;
    c = (uint32_t)(d1 >> 26); h[1] = (uint32_t)d1 & M26; d2 += c;
    c = (uint32_t)(d2 >> 26); h[2] = (uint32_t)d2 & M26; d3 += c;
    c = (uint32_t)(d3 >> 26); h[3] = (uint32_t)d3 & M26; d4 += c;
    c = (uint32_t)(d4 >> 26); h[4] = (uint32_t)d4 & M26;
    h[0] += c * 5u;
    c = h[0] >> 26; h[0] &= M26; h[1] += c;
}

// h += 16-byte block (w0..w3 little-endian words) + hibit * 2^128.
__device__ __forceinline__ void padd_block(uint32_t h[5], uint32_t w0, uint32_t w1, uint32_t w2,
                                           uint32_t w3, uint32_t hibit) {
    h[0] += w0 & M26;
    h[1] += __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    h[2] += __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    h[3] += __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    h[4] += (w3 >> 8) | (hibit << 24);
}

// 128-bit value (4 LE words) into limbs, no 2^128 bit.
__device__ __forceinline__ void plimbs(uint32_t out[5], uint32_t w0, uint32_t w1, uint32_t w2,
                                       uint32_t w3) {
    out[0] = w0 & M26;
    out[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    out[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    out[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    out[4] = w3 >> 8;
}

// Fully reduce h mod 2^130-5, add the 128-bit pad s, emit the tag as 4 LE words.
__device__ __forceinline__ void pfinish(const uint32_t hin[5], const uint32_t s[4],
                                        uint32_t tag[4]) {
    uint32_t h0 = hin[0], h1 = hin[1], h2 = hin[2], h3 = hin[3], h4 = hin[4], c;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        c = h0 >> 26; h0 &= M26; h1 += c;
        c = h1 >> 26; h1 &= M26; h2 += c;
        c = h2 >> 26; h2 &= M26; h3 += c;
        c = h3 >> 26; h3 &= M26; h4 += c;
        c = h4 >> 26; h4 &= M26; h0 += c * 5u;
    }
    c = h0 >> 26; h0 &= M26; h1 += c;
    // g = h + 5 - 2^130; use g when it does not borrow (h >= p)
    uint32_t g0 = h0 + 5u; c = g0 >> 26; g0 &= M26;
    uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= M26;
    uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= M26;
    uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= M26;
    uint32_t g4 = h4 + c - (1u << 26);
    const uint32_t use_g = (g4 >> 31) - 1u;  // all ones when no borrow
    h0 = (h0 & ~use_g) | (g0 & use_g);
    h1 = (h1 & ~use_g) | (g1 & use_g);
    h2 = (h2 & ~use_g) | (g2 & use_g);
    h3 = (h3 & ~use_g) | (g3 & use_g);
    h4 = (h4 & ~use_g) | (g4 & use_g);
    // pack to 128 bits and add s mod 2^128
    uint64_t f;
    f = (uint64_t)(h0 | (h1 << 26)) + s[0]; tag[0] = (uint32_t)f;
    f = (uint64_t)((h1 >> 6) | (h2 << 20)) + s[1] + (f >> 32); tag[1] = (uint32_t)f;
    f = (uint64_t)((h2 >> 12) | (h3 << 14)) + s[2] + (f >> 32); tag[2] = (uint32_t)f;
    f = (uint64_t)((h3 >> 18) | (h4 << 8)) + s[3] + (f >> 32); tag[3] = (uint32_t)f;
}

// r clamp (RFC 8439 2.5.1) on the 4 LE words of the one-time key's first half, into limbs.
__device__ __forceinline__ void pclamp(uint32_t r[5], uint32_t w0, uint32_t w1, uint32_t w2,
                                       uint32_t w3) {
    plimbs(r, w0 & 0x0fffffffu, w1 & 0x0ffffffcu, w2 & 0x0ffffffcu, w3 & 0x0ffffffcu);
}

// Radix-2^32 Horner step with the CLAMPED r (RFC 8439 clamp clears the top 4 bits of every r
// word and the low 2 bits of r1..r3).  That makes s_j = r_j + (r_j >> 2) = 5*r_j/4 exact and
// keeps every column sum below 2^63, so h*r needs 16+4 v_mad_u64_u32 and the column carries
// ride inside the multiply-add chains (the same construction as OpenSSL's 32-bit Poly1305).
// h = (h + m + hibit*2^128) * r, partially reduced (h4 <= 4).
struct PolyR32 {
    uint32_t r0, r1, r2, r3, s1, s2, s3;
};

__device__ __forceinline__ PolyR32 polyr32_make(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    PolyR32 R;
    R.r0 = w0 & 0x0fffffffu;
    R.r1 = w1 & 0x0ffffffcu;
    R.r2 = w2 & 0x0ffffffcu;
    R.r3 = w3 & 0x0ffffffcu;
    R.s1 = R.r1 + (R.r1 >> 2);
    R.s2 = R.r2 + (R.r2 >> 2);
    R.s3 = R.r3 + (R.r3 >> 2);
    return R;
}

__device__ __forceinline__ void poly32_block(uint32_t h[5], const PolyR32& R, uint32_t m0,
                                             uint32_t m1, uint32_t m2, uint32_t m3,
                                             uint32_t hibit) {
    // carries ride on 32-bit add-with-carry (v_add_co / v_addc_co); 64-bit adds of zero-extended
    // words would cost a v_mov per operand
    unsigned cy;
    const uint32_t a0 = __builtin_addc(h[0], m0, 0u, &cy);
    const uint32_t a1 = __builtin_addc(h[1], m1, cy, &cy);
    const uint32_t a2 = __builtin_addc(h[2], m2, cy, &cy);
    const uint32_t a3 = __builtin_addc(h[3], m3, cy, &cy);
    const uint32_t a4 = h[4] + hibit + cy;
    const uint64_t d0 = (uint64_t)a0 * R.r0 + (uint64_t)a1 * R.s3 + (uint64_t)a2 * R.s2 +
                        (uint64_t)a3 * R.s1;
    const uint64_t e1 = (uint64_t)a0 * R.r1 + (uint64_t)a1 * R.r0 + (uint64_t)a2 * R.s3 +
                        (uint64_t)a3 * R.s2 + (uint64_t)a4 * R.s1;
    const uint64_t e2 = (uint64_t)a0 * R.r2 + (uint64_t)a1 * R.r1 + (uint64_t)a2 * R.r0 +
                        (uint64_t)a3 * R.s3 + (uint64_t)a4 * R.s2;
    const uint64_t e3 = (uint64_t)a0 * R.r3 + (uint64_t)a1 * R.r2 + (uint64_t)a2 * R.r1 +
                        (uint64_t)a3 * R.r0 + (uint64_t)a4 * R.s3;
    const uint32_t x0 = (uint32_t)d0;
    const uint32_t x1 = __builtin_addc((uint32_t)e1, (uint32_t)(d0 >> 32), 0u, &cy);
    const uint32_t c1 = (uint32_t)(e1 >> 32) + cy;
    const uint32_t x2 = __builtin_addc((uint32_t)e2, c1, 0u, &cy);
    const uint32_t c2 = (uint32_t)(e2 >> 32) + cy;
    const uint32_t x3 = __builtin_addc((uint32_t)e3, c2, 0u, &cy);
    const uint32_t c3 = (uint32_t)(e3 >> 32) + cy;
    const uint32_t t4 = a4 * R.r0 + c3;  // < 2^31.6
    const uint32_t f = (t4 >> 2) * 5u;   // fold 2^130 == 5; < 2^31.9
    h[0] = __builtin_addc(x0, f, 0u, &cy);
    h[1] = __builtin_addc(x1, 0u, cy, &cy);
    h[2] = __builtin_addc(x2, 0u, cy, &cy);
    h[3] = __builtin_addc(x3, 0u, cy, &cy);
    h[4] = (t4 & 3u) + cy;
}

// Radix-2^32 accumulator (h4 small) -> five 26-bit limbs (limb 4 < 2^27).
__device__ __forceinline__ void h32_to_limbs(const uint32_t h[5], uint32_t l[5]) {
    l[0] = h[0] & M26;
    l[1] = __builtin_amdgcn_alignbit(h[1], h[0], 26) & M26;
    l[2] = __builtin_amdgcn_alignbit(h[2], h[1], 20) & M26;
    l[3] = __builtin_amdgcn_alignbit(h[3], h[2], 14) & M26;
    l[4] = (h[3] >> 8) | (h[4] << 24);
}

// x = r^e (e >= 1), general radix-2^26 square-and-multiply, left to right.
__device__ __forceinline__ void ppow(const uint32_t r[5], uint32_t e, uint32_t x[5]) {
#pragma unroll
    for (int i = 0; i < 5; ++i) x[i] = r[i];
    const Pmul mr = pmul_make(r);
    const int top = 31 - __builtin_clz(e);
    for (int b = top - 1; b >= 0; --b) {
        pmul(x, pmul_make(x));
        if ((e >> b) & 1u) pmul(x, mr);
    }
}

// ----------------------------------------------------------------------------- SHA-256
__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
__device__ __forceinline__ uint32_t rotr(uint32_t v, int s) { return __builtin_rotateright32(v, s); }

__constant__ static const uint32_t kSha256K[64] = {
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

constexpr uint32_t kShaIV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the compiler emits two v_xor_b32
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One compression (Sha256::transform, Sha256.cpp:134-176) on 16 big-endian message words.
// The 64-entry schedule is kept as a rolling 16-word window in registers.
__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);  // (e & f) ^ (~e & g)
        const uint32_t t1 = h + S1 + ch + kSha256K[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        // majority in one v_bitop3 (the compiler's own form takes three VALU ops)
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ----------------------------------------------------------------------------- byte I/O
// Bytes [off, off + 4M) of the little-endian byte string in[0..4N) as M words, zero past the
// end (off <= 4N).  The per-lane word offset goes through a log2(N)-stage barrel shift over
// compile-time register indices (no dynamic VGPR indexing, no scratch), the byte offset through
// v_alignbyte.  ~(N + 1) * log2(N) v_cndmask + M v_alignbyte.
template <int N, int M>
__device__ __forceinline__ void extract_bytes(const uint32_t* in, uint32_t off, uint32_t* out) {
    constexpr int W = N + 1;
    uint32_t a[W];
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = in[i];
    a[N] = 0u;
    const uint32_t k = off >> 2;
#pragma unroll
    for (int b = 32; b >= 1; b >>= 1) {
        if (b > N) continue;
        const bool t = (k & (uint32_t)b) != 0u;
#pragma unroll
        for (int i = 0; i < W; ++i) a[i] = t ? (i + b < W ? a[i + b] : 0u) : a[i];
    }
    const uint32_t sh = off & 3u;
#pragma unroll
    for (int j = 0; j < M; ++j)
        out[j] = __builtin_amdgcn_alignbyte(j + 1 < W ? a[j + 1] : 0u, a[j], sh);
}

// Load `n` (1..64) bytes at p into 16 LE words, zero beyond n.  Full blocks: four 16-byte loads.
// A partial block whose 16 bytes before p + n lie inside the record (window_ok) takes its whole
// 16-byte chunks plus one 16-byte window ending at p + n, shifted into place in registers
// (at most 4 loads); only records shorter than 16 bytes fall back to byte loads.
__device__ __forceinline__ void load_block(const uint8_t* __restrict__ p, uint32_t n,
                                           uint32_t w[16], bool window_ok = false) {
    if (n >= 64) {
        const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q[i];
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
    } else if (window_ok) {
        const uint32_t nq = n >> 4;
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = 0u;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            if ((uint32_t)c < nq) {
                const uint4 v = reinterpret_cast<const uint4*>(p)[c];
                w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        }
        const uint4 v = *reinterpret_cast<const uint4*>(p + n - 16);
        const uint32_t win[4] = {v.x, v.y, v.z, v.w};
        uint32_t ch[4];
        extract_bytes<4, 4>(win, 16u - (n & 15u), ch);  // the n mod 16 trailing bytes
#pragma unroll
        for (int c = 0; c < 4; ++c) {
#pragma unroll
            for (int i = 0; i < 4; ++i) w[4 * c + i] = ((uint32_t)c == nq) ? ch[i] : w[4 * c + i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if ((uint32_t)(4 * i + b) < n) v |= (uint32_t)p[4 * i + b] << (8 * b);
            w[i] = v;
        }
    }
}

// Store the first `n` (0..64) bytes of 16 LE words at p.  Partial blocks of >= 16 bytes: whole
// 16-byte chunks plus one 16-byte window ending at p + n (rewriting bytes of the previous chunk
// with the same values); shorter ones: whole words, then at most 3 bytes.
__device__ __forceinline__ void store_block(uint8_t* __restrict__ p, uint32_t n,
                                            const uint32_t w[16]) {
    if (n >= 64) {
        uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            q[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
    } else if (n >= 16) {
        const uint32_t nq = n >> 4;
#pragma unroll
        for (int c = 0; c < 3; ++c)
            if ((uint32_t)c < nq)
                reinterpret_cast<uint4*>(p)[c] =
                    make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
        uint32_t win[4];
        extract_bytes<16, 4>(w, n - 16u, win);
        *reinterpret_cast<uint4*>(p + n - 16) = make_uint4(win[0], win[1], win[2], win[3]);
    } else {
        const uint32_t nw = n >> 2;
#pragma unroll
        for (int i = 0; i < 3; ++i)
            if ((uint32_t)i < nw) *reinterpret_cast<uint32_t*>(p + 4 * i) = w[i];
        const uint32_t lw = nw == 0 ? w[0] : nw == 1 ? w[1] : nw == 2 ? w[2] : w[3];
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if ((uint32_t)b < (n & 3u)) p[4 * nw + b] = (uint8_t)(lw >> (8 * b));
    }
}

// A workgroup-uniform 64-bit value (a base address) pinned in an SGPR pair.  readfirstlane is a
// 32-bit operation returning int: read both halves and zero-extend the low one (passing the
// 64-bit value to the builtin truncates it to 32 bits -- an illegal address).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

}  // namespace enet
