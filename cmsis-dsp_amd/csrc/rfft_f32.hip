// Real FFT (fast) f32 split / merge passes — MI355X kernels, bit-exact.
//
// arm_rfft_fast_f32 (Source/TransformFunctions/arm_rfft_fast_f32.c:675-699) is
//   forward: arm_cfft_f32(Sint, p, 0, 1) then stage_rfft_f32 (:316-402)
//   inverse: merge_rfft_f32 (:405-462) then arm_cfft_f32(Sint, pOut, 1, 1).
// The CFFT runs through cfft_f32_launch; these kernels are the O(N) passes, one thread
// per output complex bin, with the reference's expression trees kept verbatim.
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace mi355x {

// forward split: X = CFFT(p) of length H = N/2 (interleaved), output N floats
__global__ __launch_bounds__(kBlock) void rfft_stage_kernel(const float2* __restrict__ X, float2* __restrict__ out,
                                                            uint64_t total, int H, const float2* __restrict__ tw) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= total) return;
  const uint64_t t = g / H;
  const int i = (int)(g % H);
  const float2* x = X + t * H;
  if (i == 0) {
    // arm_rfft_fast_f32.c:335-353: first and last bins packed into out[0], out[1]
    const float2 a = x[0];
    const float t1a = a.x + a.x, t1b = a.y + a.y;
    out[t * H] = make_float2(0.5f * (t1a + t1b), 0.5f * (t1a - t1b));
    return;
  }
  const float2 A = x[i], B = x[H - i], w = tw[i];
  const float t1a = B.x - A.x, t1b = B.y + A.y;
  const float p0 = w.x * t1a, p1 = w.y * t1a, p2 = w.x * t1b, p3 = w.y * t1b;
  out[t * H + i] = make_float2(0.5f * (A.x + B.x + p0 + p3), 0.5f * (A.y - B.y + p1 - p2));
}

// inverse merge: p holds the packed half spectrum (N floats), output feeds the inverse CFFT
__global__ __launch_bounds__(kBlock) void rfft_merge_kernel(const float2* __restrict__ X, float2* __restrict__ out,
                                                            uint64_t total, int H, const float2* __restrict__ tw) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= total) return;
  const uint64_t t = g / H;
  const int i = (int)(g % H);
  const float2* x = X + t * H;
  if (i == 0) {
    const float2 a = x[0];   // arm_rfft_fast_f32.c:420-429
    out[t * H] = make_float2(0.5f * (a.x + a.y), 0.5f * (a.x - a.y));
    return;
  }
  const float2 A = x[i], B = x[H - i], w = tw[i];
  const float t1a = A.x - B.x, t1b = A.y + B.y;
  const float r = w.x * t1a, s = w.y * t1b, tt = w.y * t1a, u = w.x * t1b;
  out[t * H + i] = make_float2(0.5f * (A.x + B.x - r - s), 0.5f * (A.y - B.y + tt - u));
}

static hipError_t launch_pass(bool merge, int n_real, const float* p, float* out, uint32_t batch,
                              const float* tw, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const int H = n_real / 2;
  const uint64_t total = (uint64_t)batch * H;
  const uint32_t grid = (uint32_t)((total + kBlock - 1) / kBlock);
  auto k = merge ? rfft_merge_kernel : rfft_stage_kernel;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, st, (const float2*)p, (float2*)out, total, H,
                     (const float2*)tw);
  return hipGetLastError();
}

hipError_t rfft_f32_stage_launch(int n_real, const float* p, float* out, uint32_t batch, const float* tw,
                                 hipStream_t st) {
  return launch_pass(false, n_real, p, out, batch, tw, st);
}
hipError_t rfft_f32_merge_launch(int n_real, const float* p, float* out, uint32_t batch, const float* tw,
                                 hipStream_t st) {
  return launch_pass(true, n_real, p, out, batch, tw, st);
}

}  // namespace mi355x
