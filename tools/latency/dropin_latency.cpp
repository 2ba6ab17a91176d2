// Per-call latency of the host-pointer drop-in API against the reference's scalar C, on the
// call shapes of the reference's own examples:
//   arm_cfft_f32 N=1024 in place, bitReverseFlag=1 (Examples/ARM/arm_fft_bin_example/
//     arm_fft_bin_example_f32.c:111-143: one transform per call on a host buffer);
//   arm_fir_f32 29 taps x 32-sample blocks (Examples/ARM/arm_fir_example/arm_fir_example_f32.c:
//     141-239: a streaming FIR called once per block).
// Both libraries export the same symbols, so each is dlopen'ed RTLD_LOCAL and bound by dlsym.
// Usage: dropin_latency <product.so> <reference.so> [calls]   -> one JSON line on stdout.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/arm_math.h"

struct Lib {
  void* h = nullptr;
  void (*cfft)(const arm_cfft_instance_f32*, float*, uint8_t, uint8_t) = nullptr;
  const arm_cfft_instance_f32* sR1024 = nullptr;
  void (*fir_init)(arm_fir_instance_f32*, uint16_t, const float*, float*, uint32_t) = nullptr;
  void (*fir)(const arm_fir_instance_f32*, const float*, float*, uint32_t) = nullptr;
  bool open(const char* path) {
    h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) { std::fprintf(stderr, "dlopen %s: %s\n", path, dlerror()); return false; }
    cfft = (decltype(cfft))dlsym(h, "arm_cfft_f32");
    sR1024 = (const arm_cfft_instance_f32*)dlsym(h, "arm_cfft_sR_f32_len1024");
    fir_init = (decltype(fir_init))dlsym(h, "arm_fir_init_f32");
    fir = (decltype(fir))dlsym(h, "arm_fir_f32");
    return cfft && sR1024 && fir_init && fir;
  }
};

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// median of per-call times over `reps` timed batches of `calls` calls
template <typename F>
static double per_call_us(F&& f, int calls) {
  for (int i = 0; i < 50; ++i) f(i);                          // warm: uploads, caches, clocks
  std::vector<double> t;
  for (int r = 0; r < 5; ++r) {
    const double t0 = now_us();
    for (int i = 0; i < calls; ++i) f(i);
    t.push_back((now_us() - t0) / calls);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: %s product.so reference.so [calls]\n", argv[0]); return 2; }
  const int calls = argc > 3 ? std::atoi(argv[3]) : 2000;
  Lib gpu, ref;
  if (!gpu.open(argv[1]) || !ref.open(argv[2])) return 1;
  std::vector<float> x(2048), xr(2048);
  for (int i = 0; i < 2048; ++i) x[i] = xr[i] = std::sin(0.01f * i);
  // in place, alternating forward / inverse keeps the data bounded
  const double g_cfft = per_call_us([&](int i) { gpu.cfft(gpu.sR1024, x.data(), (uint8_t)(i & 1), 1); }, calls);
  const double r_cfft = per_call_us([&](int i) { ref.cfft(ref.sR1024, xr.data(), (uint8_t)(i & 1), 1); }, calls);
  bool same = true;
  for (int i = 0; i < 2048; ++i) same &= x[i] == xr[i];       // identical call sequences
  const int taps = 29, block = 32;
  std::vector<float> c(taps), sg(taps + block - 1), sr(taps + block - 1), in(block), og(block), orr(block);
  for (int k = 0; k < taps; ++k) c[k] = 0.03f * (float)(k % 7) - 0.05f;
  arm_fir_instance_f32 Sg, Sr;
  gpu.fir_init(&Sg, taps, c.data(), sg.data(), block);
  ref.fir_init(&Sr, taps, c.data(), sr.data(), block);
  auto src = [&](int i) { for (int k = 0; k < block; ++k) in[k] = std::sin(0.05f * (i * block + k)); };
  const double g_fir = per_call_us([&](int i) { src(i); gpu.fir(&Sg, in.data(), og.data(), block); }, calls);
  const double r_fir = per_call_us([&](int i) { src(i); ref.fir(&Sr, in.data(), orr.data(), block); }, calls);
  bool fsame = true;
  for (int k = 0; k < block; ++k) fsame &= og[k] == orr[k];
  std::printf("{\"calls\": %d, \"cfft_f32_1024\": {\"product_us\": %.2f, \"reference_us\": %.2f, \"bit_exact\": %s}, "
              "\"fir_f32_29x32\": {\"product_us\": %.2f, \"reference_us\": %.2f, \"bit_exact\": %s}}\n",
              calls, g_cfft, r_cfft, same ? "true" : "false", g_fir, r_fir, fsame ? "true" : "false");
  return 0;
}
