// Issue rate of v_mfma_i32_32x32x32_i8 / v_mfma_i32_16x16x64_i8 on one MI355X: each wave runs
// ITER x A independent accumulator chains (no memory traffic in the loop); waves per SIMD
// set by the grid.  Prints i8 TOPS and cycles per MFMA per SIMD at the measured clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

template <int A>
__global__ __launch_bounds__(256) void k32(int* out, int iters, int seed) {
  i32x16 acc[A];
  for (int a = 0; a < A; ++a) acc[a] = i32x16{};
  i32x4 x = {seed + (int)threadIdx.x, seed * 3, seed ^ 5, 7}, y = {seed, 11, (int)threadIdx.x, 13};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int a = 0; a < A; ++a) acc[a] = __builtin_amdgcn_mfma_i32_32x32x32_i8(x, y, acc[a], 0, 0, 0);
  }
  int s = 0;
  for (int a = 0; a < A; ++a) for (int r = 0; r < 16; ++r) s += acc[a][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int A>
__global__ __launch_bounds__(256) void k16(int* out, int iters, int seed) {
  i32x4 acc[A];
  for (int a = 0; a < A; ++a) acc[a] = i32x4{};
  i32x4 x = {seed + (int)threadIdx.x, seed * 3, seed ^ 5, 7}, y = {seed, 11, (int)threadIdx.x, 13};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int a = 0; a < A; ++a) acc[a] = __builtin_amdgcn_mfma_i32_16x16x64_i8(x, y, acc[a], 0, 0, 0);
  }
  int s = 0;
  for (int a = 0; a < A; ++a) for (int r = 0; r < 4; ++r) s += acc[a][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int* out;
  hipMalloc(&out, 256 * 4096 * sizeof(int));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 4000;
  for (int wps : {1, 2, 4}) {
    const int blocks = 256 * wps;            // 4 waves per block = 1 per SIMD
    for (int kind = 0; kind < 4; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        if (kind == 0) k32<4><<<blocks, 256>>>(out, iters, rep);
        if (kind == 1) k32<1><<<blocks, 256>>>(out, iters * 4, rep);
        if (kind == 2) k16<4><<<blocks, 256>>>(out, iters * 2, rep);
        if (kind == 3) k16<1><<<blocks, 256>>>(out, iters * 8, rep);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double mfmas = (double)blocks * 4 * iters * 4 * (kind >= 2 ? 2 : 1);   // per wave: iters*4 (32x32) or iters*8 (16x16)
      const double ops = mfmas * (kind >= 2 ? 16.0 * 16 * 64 * 2 : 32.0 * 32 * 32 * 2);
      const char* nm[4] = {"32x32x32 4 chains", "32x32x32 1 chain ", "16x16x64 4 chains", "16x16x64 1 chain "};
      printf("%s waves/SIMD=%d  %.3f ms  %.0f TOPS  %.1f ns per MFMA per SIMD\n", nm[kind], wps, best,
             ops / (best * 1e-3) * 1e-12, best * 1e6 / (mfmas / 1024.0));
    }
  }
  return 0;
}
