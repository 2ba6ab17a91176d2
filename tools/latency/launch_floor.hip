// Launch + completion floor of one small GPU call on this box: what the
// drop-in API (one transform / block per call, host buffers) cannot go below.
//   empty+sync        : empty kernel, hipStreamSynchronize (the drop-in's current completion)
//   empty+event       : empty kernel, hipEventRecord + hipEventSynchronize
//   flag+spin         : kernel stores a flag into coherent pinned host memory, host spins on it
//   graph+sync/spin   : the same kernels launched as a captured one-node hipGraph
//   copy8k+spin       : kernel reads 8 KiB from coherent pinned memory and writes 8 KiB back
//                       (the cfft N=1024 drop-in's data movement), host spins on a flag
//   writevalue+spin   : kernel, then hipStreamWriteValue32 of a sequence number into the mapped
//                       host flag (no change to the kernel), host spins on it
// Each under hipDeviceScheduleAuto (default) and hipDeviceScheduleSpin.  Prints one JSON line.
// Usage: launch_floor [calls] [spin]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void empty_kernel() {}

__global__ void flag_kernel(volatile unsigned* flag, unsigned v) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    *flag = v;
  }
}

__global__ void copy_flag_kernel(const float4* __restrict__ in, float4* __restrict__ out, volatile unsigned* flag,
                                 unsigned v) {
  const int t = threadIdx.x;                 // 512 threads x 16 B = 8 KiB
  float4 a = in[t];
  a.x = -a.x;
  out[t] = a;
  __syncthreads();
  if (t == 0) {
    __threadfence_system();
    *flag = v;
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename F>
static double per_call_us(F&& f, int calls) {
  for (int i = 0; i < 200; ++i) f(i);
  std::vector<double> t;
  for (int r = 0; r < 5; ++r) {
    const double t0 = now_us();
    for (int i = 0; i < calls; ++i) f(i);
    t.push_back((now_us() - t0) / calls);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

#define CK(x) do { if ((x) != hipSuccess) { std::fprintf(stderr, "%s failed\n", #x); std::exit(1); } } while (0)

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  const bool spin = argc > 2 && std::atoi(argv[2]) != 0;
  if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned* flag = nullptr;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  float4 *zin = nullptr, *zout = nullptr;
  CK(hipHostMalloc((void**)&zin, 8192, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&zout, 8192, hipHostMallocCoherent | hipHostMallocMapped));
  *flag = 0;
  unsigned seq = 0;
  auto wait_flag = [&](unsigned v) {
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
    }
  };

  const double empty_sync = per_call_us([&](int) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
    (void)hipStreamSynchronize(st);
  }, calls);
  const double empty_event = per_call_us([&](int) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
    (void)hipEventRecord(ev, st);
    (void)hipEventSynchronize(ev);
  }, calls);
  const double flag_spin = per_call_us([&](int) {
    ++seq;
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, seq);
    wait_flag(seq);
  }, calls);
  const double copy_spin = per_call_us([&](int) {
    ++seq;
    hipLaunchKernelGGL(copy_flag_kernel, dim3(1), dim3(512), 0, st, zin, zout, flag, seq);
    wait_flag(seq);
  }, calls);
  const double copy_sync = per_call_us([&](int) {
    ++seq;
    hipLaunchKernelGGL(copy_flag_kernel, dim3(1), dim3(512), 0, st, zin, zout, flag, seq);
    (void)hipStreamSynchronize(st);
  }, calls);
  // empty kernel, then a stream write of the sequence number into the mapped host flag
  unsigned* dflag = nullptr;
  CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
  const double wv_spin = per_call_us([&](int) {
    ++seq;
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
    (void)hipStreamWriteValue32(st, dflag, seq, 0);
    wait_flag(seq);
  }, calls);
  const double copy_wv_spin = per_call_us([&](int) {
    ++seq;
    hipLaunchKernelGGL(copy_flag_kernel, dim3(1), dim3(512), 0, st, zin, zout, flag, seq + 1000000000u);
    (void)hipStreamWriteValue32(st, dflag, seq, 0);
    wait_flag(seq);
  }, calls);
  // one-node graph of the empty kernel
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  const double graph_sync = per_call_us([&](int) {
    (void)hipGraphLaunch(ge, st);
    (void)hipStreamSynchronize(st);
  }, calls);
  (void)hipStreamSynchronize(st);
  std::printf("{\"spin_schedule\": %s, \"calls\": %d, \"empty_sync_us\": %.2f, \"empty_event_us\": %.2f, "
              "\"flag_spin_us\": %.2f, \"copy8k_spin_us\": %.2f, \"copy8k_sync_us\": %.2f, \"graph_sync_us\": %.2f, "
              "\"writevalue_spin_us\": %.2f, \"copy8k_writevalue_spin_us\": %.2f}\n",
              spin ? "true" : "false", calls, empty_sync, empty_event, flag_spin, copy_spin, copy_sync, graph_sync, wv_spin,
              copy_wv_spin);
  return 0;
}
