// records.hip -- the ChaCha20 / ChaCha20-Poly1305 record engine (gfx950).
//
// One wave = 64 lanes; each record gets P lanes (P = 1..16, a power of two chosen by the host
// scheduler so the chip holds >= 2 waves per SIMD).  Lane j of a record processes ChaCha20
// blocks j, j+P, j+2P, ... -- one 64-byte block per lane per round, the 4x4 state in VGPRs.
//
// Poly1305 (seal / open) runs in the same lanes, interleaved by 16-byte block: lane j owns the
// Poly1305 stream blocks s == j (mod P) and keeps a Horner accumulator in the multiplier r^P;
// at the end each lane multiplies by r^(e_j) (e_j in [1, P]) and the P lanes add up their
// contributions with cross-lane shuffles.  For P > 1 each round's ciphertext is exchanged
// through a wave-private LDS slab (80-byte lane slots: conflict-free b128 writes and reads).
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

constexpr int kSlot = 80;  // LDS bytes per lane (64 data + 16 pad)

// Frame sub-modes of MODE_XOR
enum FrameKind : int { FR_NONE = 0, FR_SEAL = 1, FR_OPEN = 2 };

// r^(2^b) table and the small power r^e, e in [1, 2^LOGP]
template <int LOGP>
__device__ __forceinline__ void poly_powers(const uint32_t r[5], Pmul& RP, Pmul& E, uint32_t e) {
    uint32_t pw[LOGP + 1][5];
#pragma unroll
    for (int i = 0; i < 5; ++i) pw[0][i] = r[i];
#pragma unroll
    for (int b = 1; b <= LOGP; ++b) {
#pragma unroll
        for (int i = 0; i < 5; ++i) pw[b][i] = pw[b - 1][i];
        pmul(pw[b], pmul_make(pw[b - 1]));
    }
    RP = pmul_make(pw[LOGP]);
    if (LOGP == 0) {
        E = RP;
        return;
    }
    // x = r^e by binary powering over the table (e == 2^LOGP handled by the top bit)
    uint32_t x[5] = {1, 0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b <= LOGP; ++b) {
        if ((e >> b) & 1u) {
            uint32_t y[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) y[i] = x[i];
            pmul(y, pmul_make(pw[b]));
#pragma unroll
            for (int i = 0; i < 5; ++i) x[i] = y[i];
        }
    }
    E = pmul_make(x);
}

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

template <int LOGP, int MODE, int FRAME>
__global__ __launch_bounds__(kWG) void records_kernel(RecParams p) {
    constexpr uint32_t P = 1u << LOGP;
    constexpr bool kPoly = (MODE != MODE_XOR);
    constexpr bool kLds = kPoly && (P > 1);
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds ? kWG * kSlot : 16];

    const uint32_t gid = blockIdx.x * kWG + threadIdx.x;
    const uint32_t group = gid >> LOGP;
    const uint32_t j = gid & (P - 1);
    const bool live = group < p.n;
    const uint32_t rec = live ? (p.order ? p.order[group] : group) : 0u;

    // ---- record geometry
    uint64_t ioff = 0, ooff = 0, Lin = 0, Lout = 0;
    if (live) {
        ioff = p.in_off[rec];
        Lin = p.in_off[rec + 1] - ioff;
        ooff = p.out_off[rec];
        Lout = p.out_off[rec + 1] - ooff;
    }
    // bytes run through the keystream
    uint64_t L = Lin;
    if (FRAME == FR_SEAL) L = Lout;  // in || mac(out tail)
    const uint32_t nb = (uint32_t)((L + 63) >> 6);
    const uint8_t* __restrict__ src = p.in + ioff;
    uint8_t* __restrict__ dst = p.out + ooff;

    // ---- per-record ChaCha20 constants
    uint32_t kw[8], nw[3];
    if (live) {
        const uint32_t* kp = reinterpret_cast<const uint32_t*>(p.keys + (size_t)p.key_stride * rec);
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = kp[i];
        const uint32_t* np = reinterpret_cast<const uint32_t*>(p.nonces + 12ull * rec);
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = np[i];
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) kw[i] = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) nw[i] = 0;
    }
    ChachaRecord R;
    chacha_record_init(R, kw, nw);
    uint32_t ctr0 = 1;  // RFC 8439 data counter
    if (MODE == MODE_XOR) ctr0 = (p.counters && live) ? p.counters[rec] : 0u;

    // ---- Poly1305 setup: one-time key from block 0, stream geometry
    uint32_t g[5] = {0, 0, 0, 0, 0};
    uint32_t rl[5], pad[4];
    Pmul RP, E;
    uint32_t na = 0, nct = 0, aad_len = 0, oj = 0;
    uint64_t aoff = 0;
    if (kPoly) {
        uint32_t otk[16];
        chacha_block(R, 0u, otk);
        pclamp(rl, otk[0], otk[1], otk[2], otk[3]);
        pad[0] = otk[4]; pad[1] = otk[5]; pad[2] = otk[6]; pad[3] = otk[7];
        if (p.aad && live) {
            aoff = p.aad_off[rec];
            aad_len = (uint32_t)(p.aad_off[rec + 1] - aoff);
        }
        na = (aad_len + 15) >> 4;
        nct = (uint32_t)((L + 15) >> 4);
        const uint32_t N = na + nct + 1;
        const uint32_t e = 1u + ((N - 1u - j) & (P - 1u));
        poly_powers<LOGP>(rl, RP, E, e);
        oj = (j - na) & (P - 1u);
        // AAD prefix: stream blocks s < na with s == j (mod P)
        for (uint32_t s = j; s < na; s += P) {
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
            pmul(g, RP);
            padd_block(g, w[0], w[1], w[2], w[3], 1u);
        }
    }

    // ---- main loop: one ChaCha20 block per lane per round
    const uint32_t T = (nb + P - 1) >> LOGP;
    for (uint32_t t = 0; t < T; ++t) {
        const uint32_t c = (t << LOGP) + j;
        const bool act = c < nb;
        uint32_t ks[16];
        chacha_block(R, ctr0 + c, ks);  // uint32 wrap, ChaCha20.cpp:110
        uint32_t w[16];
        uint32_t nbytes = 0;
        if (act) {
            const uint64_t pos = 64ull * c;
            nbytes = (uint32_t)min<uint64_t>(64, L - pos);
            if (FRAME == FR_SEAL && pos + 64 > Lin) {
                // virtual input in[0, Lin) || out[Lin, Lout): the plaintext MAC written by the
                // HMAC pass sits in the output record's tail
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    uint32_t v = 0;
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint64_t q = pos + 4 * i + b;
                        uint32_t byte = 0;
                        if (q < Lin) byte = src[q];
                        else if (q < L) byte = dst[q];
                        v |= byte << (8 * b);
                    }
                    w[i] = v;
                }
            } else {
                load_block(src + pos, nbytes, w);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = 0;
        }
        uint32_t o[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] = w[i] ^ ks[i];
        if (act) {
            const uint64_t pos = 64ull * c;
            if (FRAME == FR_OPEN && pos + 64 > Lout) {
                // decrypted MAC (bytes >= Lout) goes to the tag buffer
#pragma unroll
                for (int i = 0; i < 16; ++i) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint64_t q = pos + 4 * i + b;
                        const uint8_t byte = (uint8_t)(o[i] >> (8 * b));
                        if (q < Lout) dst[q] = byte;
                        else if (q < L) p.tag_out[32ull * rec + (q - Lout)] = byte;
                    }
                }
            } else {
                store_block(dst + pos, nbytes, o);
            }
        }
        if (kPoly) {
            // ciphertext of this block, zero beyond the record (Poly1305 pads with zeros)
            uint32_t ct[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) ct[i] = (MODE == MODE_SEAL) ? o[i] : w[i];
            if (MODE == MODE_SEAL && nbytes < 64) mask_tail(ct, nbytes);
            const uint32_t qbase = t << (LOGP + 2);  // first ct stream block of this round
            if (P == 1) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (qbase + u < nct) {
                        pmul(g, RP);
                        padd_block(g, ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3], 1u);
                    }
                }
            } else {
                uint4* mine = reinterpret_cast<uint4*>(lds + threadIdx.x * kSlot);
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    mine[u] = make_uint4(ct[4 * u], ct[4 * u + 1], ct[4 * u + 2], ct[4 * u + 3]);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t lane0 = threadIdx.x - j;  // first lane of this record's group
                uint4 blk[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t q = oj + P * u;  // stream block within the round
                    blk[u] = *reinterpret_cast<const uint4*>(lds + (lane0 + (q >> 2)) * kSlot +
                                                             (q & 3) * 16);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (qbase + oj + P * u < nct) {
                        pmul(g, RP);
                        padd_block(g, blk[u].x, blk[u].y, blk[u].z, blk[u].w, 1u);
                    }
                }
            }
        }
    }

    if (kPoly) {
        // length block: stream index na + nct, owned by lane (na + nct) mod P
        if (((na + nct) & (P - 1u)) == j) {
            pmul(g, RP);
            padd_block(g, aad_len, 0u, (uint32_t)L, (uint32_t)(L >> 32), 1u);
        }
        pmul(g, E);
#pragma unroll
        for (uint32_t off = P >> 1; off >= 1; off >>= 1) {
#pragma unroll
            for (int i = 0; i < 5; ++i) g[i] += __shfl_xor(g[i], (int)off);
        }
        uint32_t tag[4];
        pfinish(g, pad, tag);
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
                for (uint32_t c = j; c < nb; c += P) {
                    const uint64_t pos = 64ull * c;
                    store_block(dst + pos, (uint32_t)min<uint64_t>(64, L - pos), zero);
                }
            }
        }
    }
}

template <int LOGP, int MODE, int FRAME>
static hipError_t launch_one(const RecParams& p, hipStream_t s) {
    const uint64_t lanes = (uint64_t)p.n << LOGP;
    const uint32_t blocks = (uint32_t)((lanes + kWG - 1) / kWG);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((records_kernel<LOGP, MODE, FRAME>), dim3(blocks), dim3(kWG), 0, s, p);
    return hipGetLastError();
}

template <int MODE, int FRAME>
static hipError_t launch_mode(const RecParams& p, uint32_t lanes, hipStream_t s) {
    switch (lanes) {
        case 1: return launch_one<0, MODE, FRAME>(p, s);
        case 2: return launch_one<1, MODE, FRAME>(p, s);
        case 4: return launch_one<2, MODE, FRAME>(p, s);
        case 8: return launch_one<3, MODE, FRAME>(p, s);
        case 16: return launch_one<4, MODE, FRAME>(p, s);
        default: return hipErrorInvalidValue;
    }
}

// mode: MODE_XOR / MODE_SEAL / MODE_OPEN, plus frame variants encoded as 3 (seal) / 4 (open)
hipError_t launch_records(int mode, const RecParams& p, uint32_t lanes, hipStream_t s) {
    switch (mode) {
        case MODE_XOR: return launch_mode<MODE_XOR, FR_NONE>(p, lanes, s);
        case MODE_SEAL: return launch_mode<MODE_SEAL, FR_NONE>(p, lanes, s);
        case MODE_OPEN: return launch_mode<MODE_OPEN, FR_NONE>(p, lanes, s);
        case 3: return launch_mode<MODE_XOR, FR_SEAL>(p, lanes, s);
        case 4: return launch_mode<MODE_XOR, FR_OPEN>(p, lanes, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace enet
