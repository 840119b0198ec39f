// scalar.hpp -- routing state of the scalar C++ drop-in (enet_crypto.h "scalar"), shared by the
// translation units that serve reference signatures (crypto_api.cpp, frame_queue.cpp).
#pragma once

#include <atomic>
#include <cstdint>
#include <exception>
#include <new>

namespace enet::scalar {

extern std::atomic<int> g_policy;          // ENET_SCALAR_AUTO / DEVICE / HOST
extern std::atomic<uint64_t> g_crossover;  // ChaCha20 bytes from which AUTO uses the device
extern std::atomic<uint64_t> g_launches, g_records;

// does a call with a device kernel and `bytes` of payload go to the MI355X?
bool device_for(uint64_t bytes, bool has_crossover);
void host_call();
void device_call();
// throws like a failed HIP call when a test injected failures
void maybe_inject();
// a device call of the scalar API failed: count it, say so once on stderr (or abort)
void device_failed(const char* what, const char* why) noexcept;

// Run `dev` (a device path); on any failure except bad_alloc, report it and return false so the
// caller finishes on the host engine.
template <class F>
bool try_device(const char* what, F&& dev) {
    try {
        maybe_inject();
        dev();
        device_call();
        return true;
    } catch (const std::bad_alloc&) {
        throw;
    } catch (const std::exception& e) {
        device_failed(what, e.what());
    } catch (...) {
        device_failed(what, "unknown error");
    }
    return false;
}

}  // namespace enet::scalar
