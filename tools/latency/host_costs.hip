// Host-side pieces of one synchronous drop-in call, timed one by one (what
// separates arm_cfft_f32's 12.5-13.5 us from the 8.2 us copy8k+spin floor on the box).
//   attr       : hipPointerGetAttributes on a malloc'ed host pointer (the is_device_ptr test)
//   cpy_in_coh : memcpy 8 KiB host -> coherent pinned (hipHostMallocCoherent | Mapped)
//   cpy_out_coh: memcpy 8 KiB coherent pinned -> host, after a kernel wrote it
//   cpy_*_def  : the same with default (non-coherent) pinned memory
//   enqueue    : hipLaunchKernelGGL of an empty kernel, host time only (2000 in a row, then sync)
// Usage: host_costs [calls]   -> one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void empty_kernel() {}
__global__ void touch_kernel(float4* p) { p[threadIdx.x].x += 1.0f; }

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x) do { if ((x) != hipSuccess) { std::fprintf(stderr, "%s failed\n", #x); std::exit(1); } } while (0)

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<char> host(8192, 1);
  void *coh = nullptr, *def = nullptr;
  CK(hipHostMalloc(&coh, 8192, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(&def, 8192, hipHostMallocDefault));
  auto med = [&](auto&& f) {
    std::vector<double> t;
    for (int r = 0; r < 5; ++r) {
      const double t0 = now_us();
      for (int i = 0; i < calls; ++i) f();
      t.push_back((now_us() - t0) / calls);
    }
    std::sort(t.begin(), t.end());
    return t[2];
  };
  hipPointerAttribute_t a;
  const double attr = med([&] { (void)hipPointerGetAttributes(&a, host.data()); (void)hipGetLastError(); });
  const double in_coh = med([&] { std::memcpy(coh, host.data(), 8192); });
  const double in_def = med([&] { std::memcpy(def, host.data(), 8192); });
  // out: the GPU wrote the buffer first (so no host cache holds it), then one copy out
  auto out_after_gpu = [&](void* p) {
    std::vector<double> t;
    for (int i = 0; i < 200; ++i) {
      hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(512), 0, st, (float4*)p);
      CK(hipStreamSynchronize(st));
      const double t0 = now_us();
      std::memcpy(host.data(), p, 8192);
      t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const double out_coh = out_after_gpu(coh), out_def = out_after_gpu(def);
  CK(hipStreamSynchronize(st));
  std::vector<double> t;
  for (int r = 0; r < 5; ++r) {
    const double t0 = now_us();
    for (int i = 0; i < calls; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
    t.push_back((now_us() - t0) / calls);
    CK(hipStreamSynchronize(st));
  }
  std::sort(t.begin(), t.end());
  std::printf("{\"calls\": %d, \"attr_us\": %.3f, \"cpy_in_coh_us\": %.3f, \"cpy_in_def_us\": %.3f, \"cpy_out_coh_us\": %.3f, "
              "\"cpy_out_def_us\": %.3f, \"enqueue_us\": %.3f}\n",
              calls, attr, in_coh, in_def, out_coh, out_def, t[2]);
  return 0;
}
