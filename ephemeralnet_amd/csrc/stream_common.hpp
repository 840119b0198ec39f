// stream_common.hpp -- shape constants of the streaming kernel (stream.hip).
#pragma once
#include "records_body.hpp"

namespace enet {

constexpr uint32_t kStreamLanes = 512;    // record lanes per workgroup (8 compute waves)
constexpr uint32_t kStreamWG = 768;       // + 4 memory waves
constexpr int kStreamSteps = 76;          // keystream barriers per stage (19 lockstep half-rounds)

__device__ __forceinline__ void stream_barrier() { asm volatile("s_barrier" ::: "memory"); }

}  // namespace enet
