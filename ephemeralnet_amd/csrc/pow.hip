// pow.hip -- batched proof-of-work search and check, gfx950.
//
// Every PoW in the reference hashes  SHA-256(prefix || BE64(candidate))  and takes the FIRST
// candidate, in attempt order, whose digest has >= difficulty leading zero bits:
//   store      src/security/StoreProof.cpp:39-52 (pow_digest), :124-146 (compute_store_pow):
//              candidates = successive std::mt19937_64(LE64(digest(nonce 0)[0..8])) outputs
//   announce   src/core/Node.cpp:155-171 (digest), :200-230 (compute_announce_pow)
//   handshake  src/core/Node.cpp:233-245 (digest), :257-292 (compute_handshake_pow):
//              candidates = start + attempt, start = first std::mt19937_64(BE64(digest(0)[0..8]))
//   leading-zero count  Node.cpp:174-190 == StoreProof.cpp:61-80
//
// One workgroup per job (1..16 waves; the host picks enough waves per job that the grid holds
// ~4 waves per SIMD).  Each step tests 64*waves consecutive attempts, one per lane; a workgroup
// min-reduction over the successful attempt indices keeps the reference's first-found order
// exactly, and the job stops at the first step that finds one.  Per job, once:
//   * the prefix's whole 64-byte blocks are absorbed into a midstate;
//   * the final block(s) become a template (tail || 8 zero nonce bytes || 0x80 || BE64 length)
//     and the SHA rounds before the nonce's first word (q = tail/4 of them) are precomputed, so
//     a candidate costs 64 - q rounds (+ one more compression when the tail is > 47 bytes);
//     q is workgroup-uniform and dispatched to 16 straight-line variants;
//   * the mt19937_64 state lives in LDS; the workgroup twists it cooperatively (groups of
//     <= 156 words keep the in-place recurrence's read-old / read-new order) and tempers 312
//     candidates at a time into an LDS ring the lanes read.
// No MFMA, no atomics, no host round trips: one launch per batch.
#include "enet_device.hpp"
#include "enet_internal.hpp"

namespace enet {

constexpr uint64_t kMtUpper = 0xFFFFFFFF80000000ull, kMtLower = 0x7FFFFFFFull;
constexpr uint64_t kMtMatrix = 0xB5026F5AA96619E9ull;
constexpr int kMtN = 312, kMtM = 156;

__device__ __forceinline__ uint64_t mt_temper(uint64_t y) {
    y ^= (y >> 29) & 0x5555555555555555ull;
    y ^= (y << 17) & 0x71D67FFFEDA60000ull;
    y ^= (y << 37) & 0xFFF7EEE000000000ull;
    return y ^ (y >> 43);
}

// SHA-256 rounds [Q, 64) of one block on the rolling 16-word schedule window w, starting from
// state st (= the state after rounds [0, Q), precomputed), feed-forward ff.  Q is a template
// parameter so every variant is straight-line code (no dynamic register indexing).
template <int Q>
__device__ __forceinline__ void sha_rounds_from(uint32_t st[8], const uint32_t ff[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
#pragma unroll
    for (int i = Q; i < 64; ++i) {
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
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);   // (e & f) ^ (~e & g)
        const uint32_t t1 = h + S1 + ch + kSha256K[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);   // majority
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] = ff[0] + a; st[1] = ff[1] + b; st[2] = ff[2] + c; st[3] = ff[3] + d;
    st[4] = ff[4] + e; st[5] = ff[5] + f; st[6] = ff[6] + g; st[7] = ff[7] + h;
}

// Rounds [0, Q) only (constant words of the first final block), no feed-forward.
template <int Q>
__device__ __forceinline__ void sha_rounds_prefix(uint32_t st[8], const uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6],
             h = st[7];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
        const uint32_t t1 = h + S1 + ch + kSha256K[i] + w[i];
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
    }
    st[0] = a; st[1] = b; st[2] = c; st[3] = d; st[4] = e; st[5] = f; st[6] = g; st[7] = h;
}

// Dispatch a uniform runtime q (0..15) to the straight-line variants.
#define ENET_POW_SWITCH_Q(q, CALL)                                                              \
    switch (q) {                                                                                \
        case 0: CALL(0); break;   case 1: CALL(1); break;   case 2: CALL(2); break;             \
        case 3: CALL(3); break;   case 4: CALL(4); break;   case 5: CALL(5); break;             \
        case 6: CALL(6); break;   case 7: CALL(7); break;   case 8: CALL(8); break;             \
        case 9: CALL(9); break;   case 10: CALL(10); break; case 11: CALL(11); break;           \
        case 12: CALL(12); break; case 13: CALL(13); break; case 14: CALL(14); break;           \
        default: CALL(15); break;                                                               \
    }

// Per-job hashing template for SHA-256(prefix || BE64(x)).
struct PowTemplate {
    uint32_t mid[8];  // state after the prefix's whole 64-byte blocks
    uint32_t stq[8];  // mid after rounds [0, q) of the first final block
    uint32_t w[32];   // final block(s), nonce bytes zero, padding and bit length in place
    uint32_t q, s;    // the nonce starts at byte 4q + s of the final block(s)
    uint32_t two;     // two final blocks (tail > 47 bytes)
};

__device__ __forceinline__ void pow_prepare(const uint8_t* __restrict__ p, uint64_t plen,
                                            PowTemplate& T) {
#pragma unroll
    for (int i = 0; i < 8; ++i) T.mid[i] = kShaIV[i];
    const uint64_t full = plen >> 6;
    uint32_t w[16];
    for (uint64_t b = 0; b < full; ++b) {
        const uint4* q4 = reinterpret_cast<const uint4*>(p + 64 * b);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = q4[i];
            w[4 * i] = bswap32(v.x); w[4 * i + 1] = bswap32(v.y);
            w[4 * i + 2] = bswap32(v.z); w[4 * i + 3] = bswap32(v.w);
        }
        sha256_compress(T.mid, w);
    }
    const uint32_t t = (uint32_t)(plen & 63u);
    uint32_t wl[16];
    if (t) {
        load_block(p + 64 * full, t, wl, plen >= 16);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) wl[i] = 0u;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) { T.w[i] = bswap32(wl[i]); T.w[16 + i] = 0u; }
    T.q = t >> 2;
    T.s = t & 3u;
    T.two = (t + 17u > 64u) ? 1u : 0u;
    const uint32_t pad_word = (t + 8u) >> 2, pad_bits = 0x80u << (24u - 8u * T.s);
    const uint64_t bits = (plen + 8ull) * 8ull;
    const uint32_t len_word = T.two ? 30u : 14u;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        T.w[i] |= ((uint32_t)i == pad_word) ? pad_bits : 0u;
        T.w[i] |= ((uint32_t)i == len_word) ? (uint32_t)(bits >> 32) : 0u;
        T.w[i] |= ((uint32_t)i == len_word + 1u) ? (uint32_t)bits : 0u;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) T.stq[i] = T.mid[i];
#define ENET_POW_PREFIX(Q) sha_rounds_prefix<Q>(T.stq, T.w)
    ENET_POW_SWITCH_Q(T.q, ENET_POW_PREFIX)
#undef ENET_POW_PREFIX
}

// Make every template field wave-uniform (SGPRs): all lanes of a workgroup prepare the same job.
__device__ __forceinline__ void pow_uniform(PowTemplate& T) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        T.mid[i] = __builtin_amdgcn_readfirstlane(T.mid[i]);
        T.stq[i] = __builtin_amdgcn_readfirstlane(T.stq[i]);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) T.w[i] = __builtin_amdgcn_readfirstlane(T.w[i]);
    T.q = __builtin_amdgcn_readfirstlane(T.q);
    T.s = __builtin_amdgcn_readfirstlane(T.s);
    T.two = __builtin_amdgcn_readfirstlane(T.two);
}

// Leading zero bits of SHA-256(prefix || BE64(x)) (digest words in st on return).  SKIP: start
// the first final block at round q from the precomputed state (the hot path, 16 straight-line
// variants); otherwise run it whole from the midstate (seed digest, checks).
template <bool SKIP>
__device__ __forceinline__ uint32_t pow_hash(const PowTemplate& T, uint64_t x, uint32_t st[8]) {
    uint32_t w[16];
    const uint32_t s8 = 8u * T.s;
    const uint32_t na = (uint32_t)(x >> (32u + s8));
    const uint32_t nb = (uint32_t)(x >> s8);
    const uint32_t nc = T.s ? (uint32_t)(x << (32u - s8)) : 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint32_t v = T.w[i];
        v |= ((uint32_t)i == T.q) ? na : 0u;
        v |= ((uint32_t)i == T.q + 1u) ? nb : 0u;
        v |= ((uint32_t)i == T.q + 2u) ? nc : 0u;
        w[i] = v;
    }
    if (SKIP) {
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = T.stq[i];
#define ENET_POW_FROM(Q) sha_rounds_from<Q>(st, T.mid, w)
        ENET_POW_SWITCH_Q(T.q, ENET_POW_FROM)
#undef ENET_POW_FROM
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) st[i] = T.mid[i];
        sha_rounds_from<0>(st, T.mid, w);
    }
    if (T.two) {
        // the nonce spills into the second block only when it starts at byte >= 57 (q >= 14)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t v = T.w[16 + i];
            v |= ((uint32_t)(16 + i) == T.q + 1u) ? nb : 0u;
            v |= ((uint32_t)(16 + i) == T.q + 2u) ? nc : 0u;
            w[i] = v;
        }
        uint32_t ff[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) ff[i] = st[i];
        sha_rounds_from<0>(st, ff, w);
    }
    uint32_t lz = 0, done = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        lz += done ? 0u : (st[i] ? (uint32_t)__builtin_clz(st[i]) : 32u);
        done |= st[i];
    }
    return lz;
}

// Workgroup twist of the mt19937_64 state in LDS: words in index order, groups of <= 156, so
// word i >= 156 reads the NEW word i-156 and word i < 156 reads the OLD word i+156, exactly as
// the sequential in-place recurrence does (std::mersenne_twister_engine::_M_gen_rand).
__device__ __forceinline__ void mt_twist(uint64_t* mt, uint32_t tid, uint32_t nthreads) {
    const uint32_t G = nthreads < (uint32_t)kMtM ? nthreads : (uint32_t)kMtM;
    for (uint32_t g = 0; g < (uint32_t)kMtN; g += G) {
        const uint32_t i = g + tid;
        uint64_t v = 0;
        const bool mine = tid < G && i < (uint32_t)kMtN;
        if (mine) {
            const uint64_t x = (mt[i] & kMtUpper) | (mt[i + 1 == (uint32_t)kMtN ? 0 : i + 1] & kMtLower);
            const uint32_t j = i < (uint32_t)kMtM ? i + kMtM : i - kMtM;
            v = mt[j] ^ (x >> 1) ^ ((x & 1u) ? kMtMatrix : 0ull);
        }
        __syncthreads();
        if (mine) mt[i] = v;
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void pow_search_kernel(PowParams P) {
    extern __shared__ uint64_t smem[];
    uint64_t* mt = smem;                       // [312]
    uint64_t* ring = smem + kMtN;              // [ring]
    uint64_t* wres = ring + P.ring;            // [waves]
    const uint32_t job = blockIdx.x;
    const uint32_t tid = threadIdx.x, nthreads = blockDim.x, waves = nthreads >> 6;
    const uint32_t diff = P.difficulty[job];
    if (diff == 0u) {  // compute_store_pow / compute_*_pow: difficulty 0 -> nonce 0
        if (tid == 0) {
            P.nonces[job] = 0;
            if (P.attempts) P.attempts[job] = 0;
            P.found[job] = 1;
        }
        return;
    }
    const uint64_t off = P.off[job];
    PowTemplate T;
    // The prefix address is workgroup-uniform, so the compiler would fetch it with scalar
    // (SMEM) loads -- which ignore the low two address bits.  Prefixes start at arbitrary byte
    // offsets: keep the pointer in VGPRs so the loads are vector loads (unaligned-safe).
    const uint8_t* pre = P.prefixes + off;
    asm volatile("" : "+v"(pre));
    pow_prepare(pre, P.off[job + 1] - off, T);
    pow_uniform(T);
    uint32_t st[8];
    (void)pow_hash<false>(T, 0ull, st);  // seed digest: the same prefix with nonce 0
    const uint64_t seed = P.schedule == 1
        ? ((uint64_t)bswap32(st[1]) << 32) | bswap32(st[0])   // memcpy LE, StoreProof.cpp:137
        : ((uint64_t)st[0] << 32) | st[1];                     // BE, Node.cpp:205-207
    if (tid == 0) {  // std::mt19937_64(seed): sequential 311-step recurrence
        uint64_t v = seed;
        mt[0] = v;
        for (int i = 1; i < kMtN; ++i) {
            v = 6364136223846793005ull * (v ^ (v >> 62)) + (uint64_t)i;
            mt[i] = v;
        }
    }
    __syncthreads();
    const uint64_t R = P.ring, rmask = R - 1;
    const uint64_t step = nthreads;
    uint64_t gen = 0;  // stream positions generated into the ring
    uint64_t start = 0;
    if (P.schedule == 0) {  // first draw of the distribution = first engine output
        mt_twist(mt, tid, nthreads);
        start = mt_temper(mt[0]);
    }
    const uint64_t max_att = P.max_attempts;
    uint64_t best = ~0ull;
    for (uint64_t base = 0; base < max_att; base += step) {
        if (P.schedule == 1) {
            while (gen < base + step) {
                mt_twist(mt, tid, nthreads);
                for (uint32_t k = tid; k < (uint32_t)kMtN; k += nthreads)
                    ring[(gen + k) & rmask] = mt_temper(mt[k]);
                gen += kMtN;
                __syncthreads();
            }
        }
        const uint64_t a = base + tid;
        bool hit = false;
        if (a < max_att) {
            const uint64_t cand = P.schedule == 1 ? ring[a & rmask] : start + a;
            hit = pow_hash<true>(T, cand, st) >= diff;
        }
        const uint64_t mask = __ballot(hit);
        if ((tid & 63u) == 0)
            wres[tid >> 6] = mask ? base + (tid & ~63u) + (uint64_t)__builtin_ctzll(mask) : ~0ull;
        __syncthreads();
        for (uint32_t w = 0; w < waves; ++w) best = wres[w] < best ? wres[w] : best;
        if (best != ~0ull) break;
        __syncthreads();  // wres is rewritten next step
    }
    if (tid == 0) {
        const bool ok = best != ~0ull;
        P.found[job] = ok ? 1 : 0;
        P.nonces[job] = ok ? (P.schedule == 1 ? ring[best & rmask] : start + best) : 0ull;
        if (P.attempts) P.attempts[job] = ok ? best : max_att;
    }
}

// store_pow_valid / announce_pow_valid: one lane per job (difficulty 0 -> valid).
__global__ __launch_bounds__(kWG) void pow_check_kernel(PowParams P) {
    const uint32_t job = blockIdx.x * kWG + threadIdx.x;
    if (job >= P.n) return;
    const uint32_t diff = P.difficulty[job];
    uint8_t ok = 1;
    if (diff != 0u) {
        const uint64_t off = P.off[job];
        PowTemplate T;
        pow_prepare(P.prefixes + off, P.off[job + 1] - off, T);
        uint32_t st[8];
        ok = pow_hash<false>(T, P.check_nonces[job], st) >= diff ? 1 : 0;
    }
    P.found[job] = ok;
}

hipError_t launch_pow_search(const PowParams& p, uint32_t waves, hipStream_t s) {
    if (p.n == 0) return hipSuccess;
    const size_t lds = (size_t)(kMtN + p.ring + waves) * sizeof(uint64_t);
    hipLaunchKernelGGL(pow_search_kernel, dim3(p.n), dim3(64 * waves), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_pow_check(const PowParams& p, hipStream_t s) {
    if (p.n == 0) return hipSuccess;
    hipLaunchKernelGGL(pow_check_kernel, dim3((p.n + kWG - 1) / kWG), dim3(kWG), 0, s, p);
    return hipGetLastError();
}

}  // namespace enet
