// Batch.hpp -- crypto::batch: the many-records-per-call form of the reference API, for callers
// that collect work across sessions / chunks (batched session-frame codec, store
// pipeline).  Host memory in, host memory out (see below).  Device-resident callers use the C ABI
// (enet_crypto.h) directly.
#pragma once

#include <array>
#include <chrono>
#include <cstdint>
#include <future>
#include <optional>
#include <span>
#include <string_view>
#include <vector>

#include "ephemeralnet/crypto/CryptoTypes.hpp"
#include "ephemeralnet/crypto/ChaCha20.hpp"

namespace ephemeralnet::crypto::batch {

struct Sealed {
    std::vector<std::uint8_t> data;
    std::array<std::uint8_t, 16> tag{};
};

// Every call below takes host memory and runs on the MI355X of the calling thread's device
// through the host-memory batch runtime: the records are gathered by host worker threads into
// pinned, device-mapped staging, chunk by chunk, while earlier chunks run on the device and
// later results are scattered back -- never a pageable hipMemcpy.  Outputs come either as one
// vector per record (the reference's own shape) or, for throughput, written into ONE
// caller-provided contiguous span: record i at packed_offsets(inputs, delta)[i], where delta is
// the op's length change (0 cipher / AEAD, +48 wire seal, -48 wire open, clamped at 0).
ENET_CXX_API std::vector<std::uint64_t> packed_offsets(std::span<const std::span<const std::uint8_t>> records,
                                                       std::int64_t delta);

// ChaCha20::apply for many records (counters[i] = start counter; empty span = all 0).
ENET_CXX_API std::vector<std::vector<std::uint8_t>> chacha20_apply(
    std::span<const Key> keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> inputs, std::span<const std::uint32_t> counters);
ENET_CXX_API void chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                                 std::span<const std::span<const std::uint8_t>> inputs,
                                 std::span<const std::uint32_t> counters, std::span<std::uint8_t> out);

// RFC 8439 ChaCha20-Poly1305 (no AAD) for many records.
ENET_CXX_API std::vector<Sealed> aead_seal(std::span<const Key> keys,
                                           std::span<const Nonce> nonces,
                                           std::span<const std::span<const std::uint8_t>> plaintexts);
// Returns one entry per record; an empty optional-like flag vector `ok` says which verified.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> aead_open(
    std::span<const Key> keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> ciphertexts,
    std::span<const std::array<std::uint8_t, 16>> tags, std::vector<std::uint8_t>& ok);
// contiguous forms: ciphertexts / plaintexts packed into `out` (packed_offsets(.., 0)), tags[i],
// ok[i] (a failed record's plaintext is zeroed)
ENET_CXX_API void aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
                            std::span<const std::span<const std::uint8_t>> plaintexts, std::span<std::uint8_t> out,
                            std::span<std::array<std::uint8_t, 16>> tags);
ENET_CXX_API void aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
                            std::span<const std::span<const std::uint8_t>> ciphertexts,
                            std::span<const std::array<std::uint8_t, 16>> tags, std::span<std::uint8_t> out,
                            std::span<std::uint8_t> ok);

// Vector-per-record outputs into caller-owned vectors that may be reused from call to call: `out`
// is resized to one entry per record and every entry is assigned its result, keeping its
// capacity -- a caller that keeps its result vectors (a relay's per-session buffers) pays no
// allocation per record.  The forms above that return fresh vectors allocate every record; with
// the system allocator that costs more than the crypto (host runtime).
ENET_CXX_API void chacha20_apply(std::span<const Key> keys, std::span<const Nonce> nonces,
                                 std::span<const std::span<const std::uint8_t>> inputs,
                                 std::span<const std::uint32_t> counters, std::vector<std::vector<std::uint8_t>>& out);
ENET_CXX_API void aead_seal(std::span<const Key> keys, std::span<const Nonce> nonces,
                            std::span<const std::span<const std::uint8_t>> plaintexts, std::vector<Sealed>& out);
ENET_CXX_API void aead_open(std::span<const Key> keys, std::span<const Nonce> nonces,
                            std::span<const std::span<const std::uint8_t>> ciphertexts,
                            std::span<const std::array<std::uint8_t, 16>> tags,
                            std::vector<std::vector<std::uint8_t>>& out, std::vector<std::uint8_t>& ok);

// SHA-256 digests of many messages (Sha256::digest).
ENET_CXX_API std::vector<std::array<std::uint8_t, 32>> sha256(
    std::span<const std::span<const std::uint8_t>> messages);

// Session frame bodies: ChaCha20_{K,N,0}(m || HMAC_K(m)) (Message.cpp:305-311 +
// SessionManager.cpp:362-374) and the inverse with MAC verification.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> frame_seal(
    std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> messages);
ENET_CXX_API std::vector<std::vector<std::uint8_t>> frame_open(
    std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> bodies, std::vector<std::uint8_t>& ok);

// Chunk store pipeline (Node.cpp:1414-1417): chunk_hash = SHA-256(chunk) and the chunk sealed by
// CryptoManager::encrypt_with_key(key, chunk_id, chunk); chunk_ids empty = derive each id from
// content (security::derive_chunk_id, as the daemon does, ControlServer.cpp:1101).
struct StoredChunk {
    std::vector<std::uint8_t> data;
    std::array<std::uint8_t, 32> chunk_hash{};
};
ENET_CXX_API std::vector<StoredChunk> chunk_store(std::span<const Key> keys,
                                                  std::span<const Nonce> nonces,
                                                  std::span<const std::span<const std::uint8_t>> chunks,
                                                  std::span<const ChunkId> chunk_ids);
// Fetch side (Node.cpp:1641-1655): decrypt_with_key, then keep the plaintext only when its
// SHA-256 equals the manifest's chunk_hash (ok[i] = 1); failed entries come back zeroed.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> chunk_fetch(
    std::span<const Key> keys, std::span<const Nonce> nonces, std::span<const ChunkId> chunk_ids,
    std::span<const std::span<const std::uint8_t>> ciphertexts,
    std::span<const std::array<std::uint8_t, 32>> chunk_hashes, std::vector<std::uint8_t>& ok);

// Whole wire frames nonce(12) || BE32(|body|) || ChaCha20_{K,N,0}(m || HMAC_K(m)) -- what
// SessionManager::send writes (SessionManager.cpp:362-387) -- and their inverse, which takes the
// nonce from the frame and rejects frames whose length field disagrees with the body.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> wire_seal(
    std::span<const std::array<std::uint8_t, 32>> session_keys, std::span<const Nonce> nonces,
    std::span<const std::span<const std::uint8_t>> messages);
ENET_CXX_API std::vector<std::vector<std::uint8_t>> wire_open(
    std::span<const std::array<std::uint8_t, 32>> session_keys,
    std::span<const std::span<const std::uint8_t>> frames, std::vector<std::uint8_t>& ok);
// contiguous forms: frames packed into `frames` (packed_offsets(messages, 48)); messages packed
// into `messages` (packed_offsets(frames, -48)), ok[i] (a failed message is zeroed)
ENET_CXX_API void wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys,
                            std::span<const Nonce> nonces, std::span<const std::span<const std::uint8_t>> messages,
                            std::span<std::uint8_t> frames);
ENET_CXX_API void wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                            std::span<const std::span<const std::uint8_t>> frames, std::span<std::uint8_t> messages,
                            std::span<std::uint8_t> ok);
// ... into reusable caller-owned vectors (see chacha20_apply above)
ENET_CXX_API void wire_seal(std::span<const std::array<std::uint8_t, 32>> session_keys,
                            std::span<const Nonce> nonces, std::span<const std::span<const std::uint8_t>> messages,
                            std::vector<std::vector<std::uint8_t>>& frames);
ENET_CXX_API void wire_open(std::span<const std::array<std::uint8_t, 32>> session_keys,
                            std::span<const std::span<const std::uint8_t>> frames,
                            std::vector<std::vector<std::uint8_t>>& messages, std::vector<std::uint8_t>& ok);
// The same frames from a table of session keys: frame i belongs to session_table[session[i]]
// (bytes identical to wire_seal / wire_open with session_keys[i] = session_table[session[i]]).
// The HMAC key-block midstates are computed once per table entry on the device
// (enet_hmac_midstates, enet_wire_*_batch_sessions).  Throws std::invalid_argument for a size
// mismatch or a session index outside the table.
ENET_CXX_API std::vector<std::vector<std::uint8_t>> wire_seal_sessions(
    std::span<const std::array<std::uint8_t, 32>> session_table, std::span<const std::uint32_t> session,
    std::span<const Nonce> nonces, std::span<const std::span<const std::uint8_t>> messages);
ENET_CXX_API std::vector<std::vector<std::uint8_t>> wire_open_sessions(
    std::span<const std::array<std::uint8_t, 32>> session_table, std::span<const std::uint32_t> session,
    std::span<const std::span<const std::uint8_t>> frames, std::vector<std::uint8_t>& ok);

// Cross-session frame queues.  SessionManager runs one detached reader
// thread per session (SessionManager.cpp:332-333, receive_loop :703-854) and sends from whatever
// thread calls Node::send_secure (:337-388), one ChaCha20 + HMAC per frame on that thread.  Here
// every thread hands its frame to a shared queue instead: the submitting thread reserves a slot in
// the queue's current PASS -- pinned, device-mapped staging -- and copies its frame, key and nonce
// straight into it (no lock on that path); a worker thread closes the pass once it is large enough,
// when frames stop arriving (30 us gap) or 250 us after its first frame, runs ONE wire-frame
// kernel over it on the MI355X
// (the kernel writes the pinned pass and reads it, or for a large pass -- 640+ frames sealing,
// 512+ opening -- a device copy of its input side), and every submitter copies its own result out
// of the pass (FrameTicket::get) or reads it in place (FrameTicket::view).  Passes grow with the offered load; several are in
// flight at once (max_inflight workers).  Results are matched by slot, so sessions never see each
// other's frames; bytes are identical to the per-frame reference path.
// Routing (enet_scalar_set_policy): blocking seal() / open() run on the calling thread's host
// engine under ENET_SCALAR_AUTO (default) and ENET_SCALAR_HOST -- one blocked caller per frame
// never builds a batch at which the device pays -- and through the queue under ENET_SCALAR_DEVICE.
// Non-blocking submit() / seal_async() / open_async() (a relay draining a socket buffer keeps
// many frames in flight) go through the queue under DEVICE, and under AUTO when the device is
// present and the submitting thread holds >= 320 submitted, uncollected frames (the measured
// crossover where the device queue overtakes the host engine in frames/s); on the
// host engine otherwise and under HOST.  A pass the device cannot run
// is finished on the host engine (never an exception into a session thread).
struct FrameQueueOptions {
    std::size_t max_frames = 4096;                     // at most this many frames per pass
    std::size_t max_bytes = 8u << 20;                  // ... and this many input bytes (a frame of
                                                       // the maximum payload always fits)
    std::chrono::microseconds max_delay{0};            // 0: a pass closes at max_frames / 4 or
                                                       // max_bytes / 4, after a 30 us arrival gap,
                                                       // or 250 us after its first frame; > 0: at
                                                       // the size limits or this long after its
                                                       // first frame
    std::size_t max_inflight = 8;                      // device passes in flight at once (one
                                                       // worker thread + HIP stream each; 1-16)
    int device = 0;                                    // HIP device of the device passes
};
struct FrameQueueStats {
    std::uint64_t frames = 0;   // frames served
    std::uint64_t flushes = 0;  // batched passes (frames / flushes = mean batch)
    std::uint64_t host_flushes = 0;  // passes served by the host engine (policy, no device, failure)
    std::uint64_t evicted = 0;  // results copied out of a pass to free it for new frames
    double pass_us = 0;         // mean wall time of a device pass (close -> results ready)
    double kernel_us = 0;       // ... of which the kernel (launch to completion)
    double worker_cpu_s = 0;    // CPU time of the queue's worker threads
    std::uint64_t cas_retries = 0;  // reservations that found their pass full and moved on
};

// One submitted frame's result.  Move-only; get() blocks until the pass carrying the frame has
// run and returns the sealed frame / opened message (nullopt as seal() / open()); the ticket is
// empty afterwards.  A ticket may outlive its queue.
class ENET_CXX_API FrameTicket {
public:
    struct State;
    FrameTicket() noexcept = default;
    explicit FrameTicket(State* s) noexcept : s_(s) {}
    FrameTicket(FrameTicket&& o) noexcept : s_(o.s_) { o.s_ = nullptr; }
    FrameTicket& operator=(FrameTicket&& o) noexcept;
    FrameTicket(const FrameTicket&) = delete;
    FrameTicket& operator=(const FrameTicket&) = delete;
    ~FrameTicket();
    bool valid() const noexcept { return s_ != nullptr; }
    bool ready() const noexcept;  // get() would not block
    std::optional<std::vector<std::uint8_t>> get();
    // The same into a caller-owned vector, keeping its capacity (a session's send / receive
    // buffer: no allocation per frame): true and `out` = the result, or false (nullopt above;
    // `out` cleared)
    bool get(std::vector<std::uint8_t>& out);
    // Zero-copy: blocks like get(); on success `out` views the result where it lies (the queue's
    // pinned pass, or the ticket's own buffer) and stays valid until release(), get() or the
    // ticket's destruction.  Hold a view briefly (a relay's socket write): its pass cannot be
    // reused meanwhile.  false where get() returns nullopt.  Release every view before the
    // queue is destroyed.
    bool view(std::span<const std::uint8_t>& out);
    void release() noexcept;  // ends the ticket and its view; the ticket is empty afterwards

private:
    State* s_ = nullptr;
};

// Send side: nonce(12) || BE32(|body|) || ChaCha20_{K,nonce,0}(m || HMAC_K(m)), the frame
// SessionManager::send writes (SessionManager.cpp:362-387).  Nonces: 12 random bytes per frame
// (the reference draws them from std::random_device, SessionManager.cpp:365-371; here from a
// per-thread ChaCha20 keystream keyed from std::random_device, re-keyed every 2^20 nonces).
class ENET_CXX_API FrameQueue {
public:
    static constexpr std::size_t kMaxPayloadSize = 1024 * 1024;  // SessionManager.cpp:87
    FrameQueue();
    explicit FrameQueue(FrameQueueOptions options);
    ~FrameQueue();
    FrameQueue(const FrameQueue&) = delete;
    FrameQueue& operator=(const FrameQueue&) = delete;

    // Seal one message for one session; blocks until done.  nullopt when the signed payload
    // (message + 32-byte MAC) exceeds kMaxPayloadSize, as SessionManager::send returns false
    // (:358-360).
    std::optional<std::vector<std::uint8_t>> seal(const std::array<std::uint8_t, 32>& session_key,
                                                  std::span<const std::uint8_t> message);
    // Non-blocking seal: the message is copied into the queue before this returns.
    FrameTicket submit(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> message);
    // DEPRECATED (ABI 1.2): the same as a std::future with std::launch::deferred -- get() / wait()
    // collect the result on the calling thread, but wait_for / wait_until return
    // std::future_status::deferred and never report readiness.  Before ABI 1.2 the future became
    // ready when its pass had run; a caller that polls futures must move to submit() and
    // FrameTicket::ready() / view() (a promise per frame cost ~0.45 us of CPU per frame, DESIGN.md
    // section 6).  Kept for source compatibility of get()-style callers.
    [[deprecated("poll with submit() + FrameTicket::ready(); the returned future is deferred")]]
    std::future<std::optional<std::vector<std::uint8_t>>> seal_async(const std::array<std::uint8_t, 32>& session_key,
                                                                      std::vector<std::uint8_t> message);
    // Explicit batching (a sender that collects frames itself): push queues a message (false =
    // too large, nothing queued), flush() seals every pushed message in one pass and returns the
    // wire frames in push order.  Thread-safe; independent of the queue above.
    bool push(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> message);
    std::size_t size() const;
    std::vector<std::vector<std::uint8_t>> flush();
    FrameQueueStats stats() const;

private:
    struct Impl;
    Impl* impl_;
};

// Receive side: the inverse for frames read off any session's socket (receive_loop :744-822 +
// decode_signed, Message.cpp:313-328): nullopt when the frame is shorter than its header, its
// BE32 length disagrees with the body or exceeds kMaxPayloadSize, the body is shorter than the
// MAC, or the HMAC does not verify; otherwise the message (the body minus its 32-byte MAC).
class ENET_CXX_API FrameReceiveQueue {
public:
    FrameReceiveQueue();
    explicit FrameReceiveQueue(FrameQueueOptions options);
    ~FrameReceiveQueue();
    FrameReceiveQueue(const FrameReceiveQueue&) = delete;
    FrameReceiveQueue& operator=(const FrameReceiveQueue&) = delete;

    std::optional<std::vector<std::uint8_t>> open(const std::array<std::uint8_t, 32>& session_key,
                                                  std::span<const std::uint8_t> frame);
    // Non-blocking open (see FrameQueue::submit / seal_async).
    FrameTicket submit(const std::array<std::uint8_t, 32>& session_key, std::span<const std::uint8_t> frame);
    // DEPRECATED (ABI 1.2): a deferred future, as FrameQueue::seal_async.
    [[deprecated("poll with submit() + FrameTicket::ready(); the returned future is deferred")]]
    std::future<std::optional<std::vector<std::uint8_t>>> open_async(const std::array<std::uint8_t, 32>& session_key,
                                                                     std::vector<std::uint8_t> frame);
    FrameQueueStats stats() const;

private:
    struct Impl;
    Impl* impl_;
};

// Proof of work.  Every PoW in the reference hashes
// SHA-256(prefix || BE64(nonce)) and takes the first nonce, in attempt order, with >= difficulty
// leading zero bits.  Node: compute_announce_pow / compute_handshake_pow (Node.cpp:212-230,
// 269-292; candidates start + attempt).  Store: security::compute_store_pow (StoreProof.cpp;
// successive mt19937_64 outputs) -- see also ephemeralnet/security/StoreProof.hpp.
enum class PowSchedule : int { Node = 0, Store = 1 };
struct PowResult {
    bool found{false};
    std::uint64_t nonce{0};
    std::uint64_t attempts{0};  // index of the nonce in attempt order (max_attempts if not found)
};
// difficulty[i] as given (no clamp; 0 -> nonce 0); one device pass for the whole batch
ENET_CXX_API std::vector<PowResult> pow_search(std::span<const std::span<const std::uint8_t>> prefixes,
                                               std::span<const std::uint8_t> difficulty,
                                               PowSchedule schedule, std::uint64_t max_attempts);
// announce_pow_valid / handshake_pow_valid / store_pow_valid without the clamp; 1 = valid
ENET_CXX_API std::vector<std::uint8_t> pow_check(std::span<const std::span<const std::uint8_t>> prefixes,
                                                 std::span<const std::uint64_t> nonces,
                                                 std::span<const std::uint8_t> difficulty);
// Node.cpp:155-171 (announce_pow_digest without the nonce): BE64-length-prefixed chunk_id,
// peer_id, endpoint, manifest_uri, assigned_shards, then BE64(ttl seconds)
ENET_CXX_API std::vector<std::uint8_t> announce_pow_prefix(const ChunkId& chunk_id, const PeerId& peer_id,
                                                           std::string_view endpoint,
                                                           std::string_view manifest_uri,
                                                           std::span<const std::uint8_t> assigned_shards,
                                                           std::int64_t ttl_seconds);
// Node.cpp:233-245 (handshake_pow_digest without the nonce)
ENET_CXX_API std::vector<std::uint8_t> handshake_pow_prefix(const PeerId& initiator, const PeerId& responder,
                                                            std::uint32_t initiator_public);

// Drop-ins for Node.cpp's file-local searches compute_announce_pow (Node.cpp:212-230) and
// compute_handshake_pow (:269-292): same start (mt19937_64 seeded by the nonce-0 digest), same
// attempt order and 500'000-attempt cap (Node.cpp:40,43), same nonce.  difficulty 0 -> nonce 0,
// true.  Not found -> false and nonce_out untouched.  One device search replaces up to 500'000
// host Sha256 constructions; a maintainer makes the Node.cpp helpers forward here.
inline constexpr std::uint64_t kNodePowAttempts = 500'000;
ENET_CXX_API bool compute_announce_pow(const ChunkId& chunk_id, const PeerId& peer_id, std::string_view endpoint,
                                       std::string_view manifest_uri,
                                       std::span<const std::uint8_t> assigned_shards, std::int64_t ttl_seconds,
                                       std::uint8_t difficulty, std::uint64_t& nonce_out);
ENET_CXX_API bool compute_handshake_pow(const PeerId& initiator, const PeerId& responder,
                                        std::uint32_t initiator_public, std::uint8_t difficulty,
                                        std::uint64_t& nonce_out);

// KeyManager::derive_key (KeyManager.cpp:74-92) for many sessions:
// HMAC-SHA256(secret_i, BE64(counter_i) || BE64(ticks_i)), ticks in ns since the steady_clock epoch
ENET_CXX_API std::vector<std::array<std::uint8_t, 32>> session_keys(std::span<const Key> secrets,
                                                                    std::span<const std::uint64_t> counters,
                                                                    std::span<const std::int64_t> ticks);

}  // namespace ephemeralnet::crypto::batch
