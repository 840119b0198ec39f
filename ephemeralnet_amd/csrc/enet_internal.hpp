// enet_internal.hpp -- launch-side declarations shared by the kernel TUs and the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace enet {

constexpr int kWG = 256;           // threads per workgroup (4 waves of 64)
constexpr int kMaxLanesPerRecord = 16;

enum RecMode : int { MODE_XOR = 0, MODE_SEAL = 1, MODE_OPEN = 2 };

// Kernel parameters for the ChaCha20 / AEAD record engine (passed by value).
struct RecParams {
    uint32_t n;
    const uint64_t* in_off;
    const uint64_t* out_off;
    const uint8_t* in;
    uint8_t* out;
    const uint8_t* keys;
    uint32_t key_stride;
    const uint8_t* nonces;
    const uint32_t* counters;  // MODE_XOR start counters (nullable -> 0)
    uint32_t counter_stride;   // words between records' counters (0 -> 1; 8 = LE32 of 32-B ids)
    const uint8_t* aad;        // nullable
    const uint64_t* aad_off;   // nullable
    const uint8_t* tag_in;     // open: expected tags
    uint8_t* tag_out;          // seal: produced tags
    uint8_t* ok;               // open: verdicts
    const uint32_t* order;     // nullable
    // frame mode (MODE_XOR over in || mac): when non-null, bytes [len_in, len_in+32) of the
    // virtual input come from append[32*rec]
    const uint8_t* append;
    // uniform batch: every record is exactly uniform_len bytes in and out (0 = not uniform)
    uint64_t uniform_len;
    int coop;  // uniform-batch staging variant: 0 none, 1 register prefetch (default), 5 lockstep
    // COOP 1 with one lane per record and L % 128 != 0: stage whole aligned 128-byte lines
    // (COOP 4; needs 4-byte-aligned record starts and in / out starts equal mod 128)
    int coop_lines;
    int nt_stores;  // non-temporal whole-line output stores (ENET_NT_STORES=0 disables)
    int lockstep;   // staging 1: lockstep keystream in 512-thread workgroups (ENET_LOCKSTEP=0 disables)
    int stream;     // uniform batches with L % (128 P) == 0: the streaming kernel (stream.hip;
                    // ENET_STREAM=0 disables)
    int dbg;        // streaming kernel timing probes (ENET_STREAM_DBG bitmask, tools only; wrong
                    // output): 1 no HBM traffic, 2 no keystream, 4 no Poly1305, 64 no stores,
                    // 128 no DMA, 256 clock stamps
    int var;        // streaming kernel code variant (ENET_STREAM_VAR, tuning)
    uint32_t rec_base;  // first record index of this launch (record = group + rec_base)
    // wire frames (frame modes only): every frame starts with a hdr-byte header
    // nonce(12) || BE32(|body|) (SessionManager.cpp:376-387).  Seal writes it in front of the
    // body; open reads the nonce from it.
    uint32_t hdr;
    // records the sequence-parallel path (segments.hip) claimed: skip[rec] != 0 -> not this
    // kernel's record (nullable; per-lane path only)
    const uint8_t* skip;
};

// lanes: 1, 2, 4, 8 or 16 lanes per record.
hipError_t launch_records(int mode, const RecParams& p, uint32_t lanes, hipStream_t s);
// The streaming kernel (stream.hip): whole 512-thread workgroups of a uniform batch.
bool stream_eligible(const RecParams& p, uint32_t lanes);
hipError_t launch_stream(int mode, const RecParams& p, uint32_t lanes, uint32_t blocks, hipStream_t s);

struct ShaParams {
    uint32_t n;
    const uint8_t* in;
    const uint64_t* off;
    uint8_t* digest;           // [n][32], or an arena when dest_off != null
    const uint64_t* dest_off;  // nullable: digest i goes to digest + dest_off[i] + len_i
    // HMAC: when keys != null the lane computes HMAC(key_i, msg_i) (HmacSha256.cpp:11-39)
    const uint8_t* keys;
    const uint64_t* key_off;   // nullable: fixed 32-byte keys
    uint32_t key_stride;       // 32 or 0 (shared key) when key_off == null
    const uint8_t* expect;     // verify: expected MACs [n][32] (nullable -> compute only)
    uint8_t* ok;               // verify verdicts
    const uint64_t* guard_off; // verify: records whose guard length is < 32 fail (Message.cpp:315)
    uint8_t* zero_on_fail;     // verify: arena (indexed like `in`) to zero for failed records
    int and_ok;                // verify: ok[i] &= (mac matches) instead of ok[i] = ...
    // verify on wire frames: guard_off indexes the frames in wire_in; a frame shorter than
    // wire_hdr + 32 or whose BE32 length field differs from its body length fails
    const uint8_t* wire_in;
    uint32_t wire_hdr;
    const uint32_t* order;     // nullable
};
hipError_t launch_sha(const ShaParams& p, hipStream_t s);

// One-pass cipher + hash over ANY batch (duplex.hip): every record length, every alignment, any
// order.  A cipher lane and a hash lane per record; the message crosses HBM once.
enum DuplexKind : int {
    DK_FRAME = 0,  // frames: body = ChaCha20_{K,N,0}(m || HMAC_K(m)), [hdr] in front
    DK_CHUNK = 1,  // chunk store / fetch: ChaCha20 from LE32(chunk_id) + SHA-256(m)
    DK_AEADH = 2,  // RFC 8439 AEAD (counter 1, Poly1305 over the ciphertext) + HMAC_K(m)
};
constexpr uint32_t kDuplexRecsPerWG = 256;
struct DuplexParams {
    uint32_t n;
    const uint8_t* in;
    const uint64_t* in_off;
    uint8_t* out;
    const uint64_t* out_off;
    const uint8_t* keys;
    uint32_t key_stride;
    const uint8_t* nonces;     // [rec][12]; wire open (hdr 16) reads the frame header instead
    const uint32_t* order;     // nullable: position -> record (e.g. length-sorted)
    uint32_t hdr;              // frames: 0 or 16 (nonce || BE32 body length)
    const uint8_t* chunk_ids;  // chunks: start counter LE32(id[0..3])
    uint8_t* digests;          // chunk store: SHA-256(m)
    const uint8_t* expect;     // chunk fetch: expected SHA-256(m)
    uint8_t* macs;             // frame open: decrypted MACs; AEADH seal: HMAC_K(m)
    const uint8_t* macs_in;    // AEADH open: expected HMAC_K(m)
    uint8_t* tags;             // AEADH seal: Poly1305 tags
    const uint8_t* tags_in;    // AEADH open: expected tags
    uint8_t* ok;               // open / fetch verdicts
    int uniform;               // host hint: every record the same length (scheduling only)
    uint32_t max_len;          // host hint: longest record (scheduling only; 0 = unknown)
    int prio;                  // issue priority: 0 = length-graded (default), -1 = none,
                               // 1 = hash waves first, 2 = cipher waves first
    // session-keyed frames (nullable): record i uses key keys[32 * session[i]] and the session's
    // HMAC midstates mid[16 * session[i]] (inner state, outer state) instead of absorbing
    // key ^ ipad / key ^ opad itself
    const uint32_t* session;
    const uint32_t* mid;
    uint32_t n_sessions;  // session[i] >= n_sessions: the frame never authenticates
};
hipError_t launch_duplex(int kind, bool open, const DuplexParams& p, hipStream_t s);
// chunk / AEAD+HMAC kinds with each record's work split over cipher, schedule and rounds waves
// (duplex_split.hip): a shorter serial chain for long records
hipError_t launch_duplex_split(int kind, bool open, const DuplexParams& p, hipStream_t s);
// -1 auto (split when the longest record is >= 16 KiB), 0 never, 1 always (chunk / AEADH kinds)
int duplex_split_mode();

// Proof-of-work search / check (pow.hip): SHA-256(prefix_i || BE64(candidate)).
struct PowParams {
    uint32_t n;
    const uint8_t* prefixes;
    const uint64_t* off;
    const uint8_t* difficulty;     // per job, 0 -> nonce 0 / valid
    uint32_t schedule;             // 0 = start + attempt (Node.cpp), 1 = mt19937_64 stream (StoreProof.cpp)
    uint64_t max_attempts;
    uint64_t ring;                 // LDS candidate ring (power of two >= 64*waves + 312; 0 for schedule 0)
    uint64_t* nonces;              // search: found nonce
    uint64_t* attempts;            // search: attempt index of the nonce (nullable)
    uint8_t* found;                // search: found flag; check: valid flag
    const uint64_t* check_nonces;  // check: nonce per job
};
hipError_t launch_pow_search(const PowParams& p, uint32_t waves, hipStream_t s);
hipError_t launch_pow_check(const PowParams& p, hipStream_t s);

// HMAC-SHA256 midstates of n 32-byte keys: mid[16 i .. 16 i + 8) = state after (key ^ ipad),
// mid[16 i + 8 .. 16 i + 16) = state after (key ^ opad) (sha.hip)
hipError_t launch_hmac_midstates(uint32_t n, const uint8_t* keys, uint32_t* mid, hipStream_t s);

// KeyManager::derive_key for many sessions (sha.hip)
hipError_t launch_session_keys(uint32_t n, const uint8_t* secrets, const uint64_t* counters,
                               const int64_t* ticks, uint8_t* out, hipStream_t s);


// ---- sequence-parallel path for long records (segments.hip)
// A claimed record's entry; entries are sorted by tile_base (claimed by CAS on one packed word).
struct SegEntry {
    uint32_t rec, tile_base, ntiles, arrived;
    uint32_t aad_len, nbits, pad0, pad1;
    uint32_t r[4], s[4];     // AEAD: one-time key halves (r unclamped words; s the pad)
    uint32_t pw[5 * 40];     // AEAD: r^(2^k) in 26-bit limbs, k < nbits
};
constexpr uint64_t kSegMin = 256u << 10;   // records this long take the tiles (seg_wanted)
constexpr uint64_t kSegTileBytes = 64u << 10;
constexpr uint64_t kSegMaxLen = 1ull << 35;  // 32-bit Poly1305 block positions inside a record
struct SegParams {
    int mode;                  // MODE_XOR / MODE_SEAL / MODE_OPEN
    uint32_t n;
    const uint64_t* in_off;
    const uint64_t* out_off;
    const uint8_t* in;
    uint8_t* out;
    const uint8_t* keys;
    uint32_t key_stride;
    const uint8_t* nonces;
    const uint32_t* counters;  // MODE_XOR start counters (nullable -> 0)
    uint32_t counter_stride;
    const uint8_t* aad;
    const uint64_t* aad_off;
    const uint8_t* tag_in;
    uint8_t* tag_out;
    uint8_t* ok;
    const uint32_t* order;     // nullable: the records to plan are order[0 .. n) (a subset)
    // scratch (stream-ordered, capi.cpp seg_begin)
    unsigned long long* hdr;   // count << 40 | tiles claimed
    SegEntry* entries;         // [entry_cap]
    uint8_t* claimed;          // [index bound]: indexed by record
    uint32_t* partials;        // [tile_cap][8]
    uint32_t entry_cap, tile_cap;
    uint64_t long_min;
};
hipError_t launch_seg(const SegParams& p, uint32_t plan_blocks, uint32_t tile_blocks, hipStream_t s);
// ChaCha20 over a batch whose hints say every record is L >= kSegMin bytes: one launch of n *
// ceil(L / 64 KiB) tile workgroups; records whose real length differs are run whole by their
// tile-0 workgroup (p.n, offsets, arenas, keys, nonces, counters used; no scratch)
hipError_t launch_seg_uniform_xor(const SegParams& p, uint64_t L, hipStream_t s);
// RFC 8439 seal / open over such a batch, one launch (segments.hip seg_uniform_aead_kernel):
// p.partials [n * T][8] scratch; arrivals [n][seg_uniform_arrival_words()] zero at launch (reset
// by the kernel)
hipError_t launch_seg_uniform_aead(const SegParams& p, uint64_t L, uint32_t* arrivals, hipStream_t s);
uint32_t seg_uniform_arrival_words();
// dst[width * list[k] + b] = src[width * k + b], k < m, b < width
hipError_t launch_scatter(const uint8_t* src, const uint32_t* list, uint32_t m, uint8_t* dst, uint32_t width,
                          hipStream_t s);

// ---- long chunks: SHA-256 on host threads (chunk_hybrid.cpp)
// digests[32 k] = SHA-256 of record list[k] of the batch at `base` (device memory, or host memory
// the device maps), off = a HOST copy of its offsets; `ready` (nullable): an event the copies wait
// for.  0 or -1 (err set).
int host_hash_records(const uint8_t* base, const uint64_t* off, const uint32_t* list, uint32_t m,
                      hipEvent_t ready, uint32_t threads, uint8_t* digests, std::string& err);

uint32_t choose_lanes(uint32_t n, uint64_t total_bytes, uint32_t max_len);
uint32_t staging_variant();
// the text enet_last_error() returns on this host thread
void set_last_error(const std::string& what);

}  // namespace enet
