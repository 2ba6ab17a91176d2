// Completion flag of the synchronous drop-in calls (runtime.cpp wait_stream):
// one lane stores the call's sequence number into a coherent, device-mapped host word once every
// earlier command of the stream has finished, and the host spins on that word.  On the box a
// flag written by a kernel is seen 6.3-6.7 us after the launch, against 10.4 us for a
// hipStreamSynchronize of an empty kernel and 7.8-8.8 us for hipStreamWriteValue32
// (tools/latency/launch_floor.hip, profiles/r04/probes/launch_floor_*.json).
#include "common.hpp"
#include "kernels.hpp"

namespace mi355x {

__global__ void done_flag_kernel(uint32_t* flag, uint32_t v) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t done_flag_launch(uint32_t* dflag, uint32_t v, hipStream_t st) {
  hipLaunchKernelGGL(done_flag_kernel, dim3(1), dim3(64), 0, st, dflag, v);
  return hipGetLastError();
}

}  // namespace mi355x
