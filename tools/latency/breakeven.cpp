// Break-even batch size of the MI355X backend against the reference's scalar C on one host core
// (VERDICT r3 item 8), for the two example shapes of the drop-in API:
//   arm_cfft_f32 N=1024 (Examples/ARM/arm_fft_bin_example), arm_fir_f32 29 taps x 32-sample blocks
//   (Examples/ARM/arm_fir_example).
// For b = 1, 2, 4, ... items per call, times (median of 5 runs of `reps` calls):
//   gpu_host  : host buffers -> hipMemcpyAsync H2D -> arm_cfft_f32_batch / arm_fir_f32_batch ->
//               hipMemcpyAsync D2H -> stream sync  (what a host application pays end to end);
//   gpu_dev   : the batched call alone on device-resident buffers + stream sync;
//   ref       : b calls of the reference on one core.
// The product library is linked (its batched API needs device pointers); the reference is
// dlopen'ed RTLD_LOCAL (same symbol names).  Prints one JSON line.
// Build: hipcc -O2 -std=c++17 tools/latency/breakeven.cpp -Iinclude -Lcmsis-dsp_amd/lib -lcmsisdsp_mi355x -ldl
//        -Wl,-rpath,$PWD/cmsis-dsp_amd/lib -o tools/latency/breakeven
// Usage: breakeven <reference.so> [reps]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "arm_const_structs.h"
#include "arm_math_mi355x.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
template <typename F>
static double per_call_us(F&& f, int reps) {
  for (int i = 0; i < 20; ++i) f();
  std::vector<double> t;
  for (int r = 0; r < 5; ++r) {
    const double t0 = now_us();
    for (int i = 0; i < reps; ++i) f();
    t.push_back((now_us() - t0) / reps);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: %s reference.so [reps]\n", argv[0]); return 2; }
  const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) { std::fprintf(stderr, "dlopen: %s\n", dlerror()); return 1; }
  auto rcfft = (void (*)(const arm_cfft_instance_f32*, float*, uint8_t, uint8_t))dlsym(h, "arm_cfft_f32");
  auto rS = (const arm_cfft_instance_f32*)dlsym(h, "arm_cfft_sR_f32_len1024");
  auto rfir_init = (void (*)(arm_fir_instance_f32*, uint16_t, const float*, float*, uint32_t))dlsym(h, "arm_fir_init_f32");
  auto rfir = (void (*)(const arm_fir_instance_f32*, const float*, float*, uint32_t))dlsym(h, "arm_fir_f32");
  if (!rcfft || !rS || !rfir_init || !rfir) return 1;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  const int maxb = 4096, n = 1024, taps = 29, blk = 32;
  float *hbuf, *dbuf, *dout, *dhist, *dcoef;
  if (hipHostMalloc((void**)&hbuf, sizeof(float) * 2 * n * maxb, hipHostMallocDefault) != hipSuccess) return 1;
  if (hipMalloc((void**)&dbuf, sizeof(float) * 2 * n * maxb) != hipSuccess) return 1;
  if (hipMalloc((void**)&dout, sizeof(float) * blk * maxb) != hipSuccess) return 1;
  if (hipMalloc((void**)&dhist, sizeof(float) * (taps - 1) * maxb) != hipSuccess) return 1;
  if (hipMalloc((void**)&dcoef, sizeof(float) * taps) != hipSuccess) return 1;
  std::vector<float> coef(taps);
  for (int k = 0; k < taps; ++k) coef[k] = 0.03f * (float)(k % 7) - 0.05f;
  (void)hipMemcpy(dcoef, coef.data(), sizeof(float) * taps, hipMemcpyHostToDevice);
  (void)hipMemset(dhist, 0, sizeof(float) * (taps - 1) * maxb);
  for (int i = 0; i < 2 * n * maxb; ++i) hbuf[i] = std::sin(0.001f * (float)(i % 9973));
  (void)hipMemcpy(dbuf, hbuf, sizeof(float) * 2 * n * maxb, hipMemcpyHostToDevice);
  std::vector<float> rbuf(2 * n), rstate(taps + blk - 1), rin(blk), rout(blk);
  for (int i = 0; i < 2 * n; ++i) rbuf[i] = hbuf[i];
  arm_fir_instance_f32 Sg, Sr;
  Sg.numTaps = taps;
  Sg.pCoeffs = dcoef;
  Sg.pState = nullptr;
  rfir_init(&Sr, taps, coef.data(), rstate.data(), blk);
  for (int k = 0; k < blk; ++k) rin[k] = std::sin(0.05f * k);
  const double ref_cfft = per_call_us([&] { rcfft(rS, rbuf.data(), 0, 1); }, reps * 10);
  const double ref_fir = per_call_us([&] { rfir(&Sr, rin.data(), rout.data(), blk); }, reps * 10);
  std::printf("{\"reference_one_core_us\": {\"cfft_f32_1024\": %.3f, \"fir_f32_29x32\": %.3f}, \"batches\": [", ref_cfft,
              ref_fir);
  bool first = true;
  for (int b = 1; b <= maxb; b *= 4) {
    const size_t cb = sizeof(float) * 2 * n * b, fb = sizeof(float) * blk * b;
    const double c_host = per_call_us([&] {
      (void)hipMemcpyAsync(dbuf, hbuf, cb, hipMemcpyHostToDevice, st);
      (void)arm_cfft_f32_batch(&arm_cfft_sR_f32_len1024, dbuf, b, 0, 1, st);
      (void)hipMemcpyAsync(hbuf, dbuf, cb, hipMemcpyDeviceToHost, st);
      (void)hipStreamSynchronize(st);
    }, reps);
    const double c_dev = per_call_us([&] {
      (void)arm_cfft_f32_batch(&arm_cfft_sR_f32_len1024, dbuf, b, 0, 1, st);
      (void)hipStreamSynchronize(st);
    }, reps);
    const double f_host = per_call_us([&] {
      (void)hipMemcpyAsync(dbuf, hbuf, fb, hipMemcpyHostToDevice, st);
      (void)arm_fir_f32_batch(&Sg, dbuf, dout, blk, b, dhist, st);
      (void)hipMemcpyAsync(hbuf, dout, fb, hipMemcpyDeviceToHost, st);
      (void)hipStreamSynchronize(st);
    }, reps);
    const double f_dev = per_call_us([&] {
      (void)arm_fir_f32_batch(&Sg, dbuf, dout, blk, b, dhist, st);
      (void)hipStreamSynchronize(st);
    }, reps);
    std::printf("%s{\"b\": %d, \"cfft_gpu_host_us\": %.2f, \"cfft_gpu_dev_us\": %.2f, \"cfft_ref_us\": %.2f, "
                "\"fir_gpu_host_us\": %.2f, \"fir_gpu_dev_us\": %.2f, \"fir_ref_us\": %.2f}",
                first ? "" : ", ", b, c_host, c_dev, ref_cfft * b, f_host, f_dev, ref_fir * b);
    first = false;
    // keep the in-place data bounded: restore the input
    (void)hipMemcpy(dbuf, hbuf, sizeof(float) * 2 * n * maxb, hipMemcpyHostToDevice);
  }
  std::printf("]}\n");
  return 0;
}
