// Batched FIR filters f32 / q15 — MI355X kernels, bit-exact.
//
// Replaces Source/FilteringFunctions/arm_fir_f32.c:911-1280 and arm_fir_q15.c:458-726
// (host scalar path, ARM_MATH_LOOPUNROLL on).  Per output n of a block, with the state
// s = [history (numTaps-1) ; block input]:
//   f32:  acc = 0.0f; for k in 0..T-1: acc = acc + s[n+k]*c[k]      (mul, then add; no FMA)
//   q15:  unrolled outputs (n < B - B%4): acc = sum over tap PAIRS of int32-wrapped
//         (s[n+2m]*c[2m] + s[n+2m+1]*c[2m+1])  -- the __SMLALD emulation, none.h:497-506;
//         tail outputs (n >= B - B%4): acc = sum of int64 products, taps in pairs (:649-681);
//         y = __SSAT(acc >> 15, 16).
//
// Geometry: one workgroup = one filter x a chunk of CHUNK outputs.  The chunk's input
// window (CHUNK + T - 1 samples) is staged into LDS with coalesced loads (history from
// the per-filter state, block samples from the input); each lane then produces R
// consecutive outputs with a register-rotated window, coefficients wave-uniform.
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace mi355x {

constexpr int kFirR = 8;                       // outputs per lane
constexpr int kFirChunk = kBlock * kFirR;      // outputs per workgroup (2048)
constexpr int kFirMaxTaps = 1024;              // LDS budget: (2048 + 1023) * 4 B

// LDS index with one pad word every 32 (lanes read at a stride of R words)
__device__ __forceinline__ int padx(int i) { return i + (i >> 5); }

template <typename T>
__device__ __forceinline__ void stage_window(T* win, const T* __restrict__ hist, const T* __restrict__ src,
                                             int T1, int n0, int count) {
  // window[j] = s[n0 + j], j < count + T1, where s = [hist(T1) ; src]
  const int total = count + T1;
  for (int j = threadIdx.x; j < total; j += kBlock) {
    const int sidx = n0 + j;
    win[padx(j)] = sidx < T1 ? hist[sidx] : src[sidx - T1];
  }
}

__global__ __launch_bounds__(kBlock) void fir_f32_kernel(const float* __restrict__ coeffs, int T,
                                                         const float* __restrict__ src, float* __restrict__ dst,
                                                         uint32_t B, const float* __restrict__ hist_in) {
  __shared__ float win[(kFirChunk + kFirMaxTaps) * 33 / 32 + 32];
  const uint32_t f = blockIdx.y;
  const int n0 = blockIdx.x * kFirChunk;
  const int count = min((int)B - n0, kFirChunk);
  const int T1 = T - 1;
  const float* s_src = src + (uint64_t)f * B;
  const float* s_hist = hist_in + (uint64_t)f * T1;
  stage_window(win, s_hist, s_src, T1, n0, count);
  __syncthreads();

  const int base = threadIdx.x * kFirR;           // local output index of this lane
  if (base < count) {
    // w is a ring over s[base + k .. base + k + R-1]; k advances R taps per unrolled round,
    // so every ring index is a compile-time constant (no register shuffling).
    float acc[kFirR], w[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) { acc[r] = 0.0f; w[r] = win[padx(base + r)]; }
    int k = 0;
    for (; k + kFirR <= T; k += kFirR) {
#pragma unroll
      for (int u = 0; u < kFirR; ++u) {
        const float c = coeffs[k + u];
#pragma unroll
        for (int r = 0; r < kFirR; ++r) acc[r] = acc[r] + w[(r + u) % kFirR] * c;
        w[u] = win[padx(base + k + u + kFirR)];
      }
    }
    for (; k < T; ++k) {
      const float c = coeffs[k];
#pragma unroll
      for (int r = 0; r < kFirR; ++r) acc[r] = acc[r] + w[r] * c;
#pragma unroll
      for (int r = 0; r < kFirR - 1; ++r) w[r] = w[r + 1];
      w[kFirR - 1] = win[padx(base + kFirR + k)];
    }
    float* o = dst + (uint64_t)f * B + n0 + base;
#pragma unroll
    for (int r = 0; r < kFirR; ++r)
      if (base + r < count) o[r] = acc[r];
  }
}

__global__ __launch_bounds__(kBlock) void fir_q15_kernel(const int16_t* __restrict__ coeffs, int T,
                                                         const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                         uint32_t B, const int16_t* __restrict__ hist_in) {
  __shared__ int16_t win[(kFirChunk + kFirMaxTaps) * 33 / 32 + 32];
  const uint32_t f = blockIdx.y;
  const int n0 = blockIdx.x * kFirChunk;
  const int count = min((int)B - n0, kFirChunk);
  const int T1 = T - 1;
  stage_window(win, hist_in + (uint64_t)f * T1, src + (uint64_t)f * B, T1, n0, count);
  __syncthreads();
  const int unrolled_end = (int)(B - (B & 3u));   // outputs before this use the pair-wrap path
  const int pairs = T >> 1;
  const int base = threadIdx.x * kFirR;
  for (int r = 0; r < kFirR; ++r) {
    const int ln = base + r;
    if (ln >= count) break;
    const bool pairwrap = (n0 + ln) < unrolled_end;
    int64_t acc = 0;
    for (int m = 0; m < pairs; ++m) {
      const int32_t x0 = win[padx(ln + 2 * m)], x1 = win[padx(ln + 2 * m + 1)];
      const int32_t c0 = coeffs[2 * m], c1 = coeffs[2 * m + 1];
      if (pairwrap) acc += (int32_t)((uint32_t)(x0 * c0) + (uint32_t)(x1 * c1));
      else          acc += (int64_t)(x0 * c0) + (int64_t)(x1 * c1);
    }
    // __SSAT takes an int32_t: (acc >> 15) is narrowed first (arm_fir_q15.c:674)
    dst[(uint64_t)f * B + n0 + ln] = (int16_t)ssat16((int32_t)(acc >> 15));
  }
}

// new history = last T-1 samples of [hist ; src]  (arm_fir_f32.c:1242-1278)
template <typename T>
__global__ void fir_hist_kernel(const T* __restrict__ src, T* __restrict__ hist, const T* __restrict__ hist_in,
                                uint32_t B, int T1, uint32_t batch) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= (uint64_t)batch * T1) return;
  const uint64_t f = g / T1;
  const int j = (int)(g % T1);
  const int64_t sidx = (int64_t)B + j;              // index into s of the new history word j
  hist[g] = sidx < T1 ? hist_in[f * T1 + sidx] : src[f * B + (sidx - T1)];
}

template <typename T>
static hipError_t fir_launch(const T* coeffs, int T_, const T* src, T* dst, uint32_t B, uint32_t batch,
                             T* hist, hipStream_t st) {
  if (batch == 0 || B == 0) return hipSuccess;
  if (T_ < 1 || T_ > kFirMaxTaps) return hipErrorInvalidValue;
  const int T1 = T_ - 1;
  // The history is read by the filter pass and rewritten afterwards; if the new tail
  // depends on old history (B < T1) keep a copy of the old one.
  const T* hist_in = hist;
  T* tmp = nullptr;
  if (T1 > 0 && (int64_t)B < T1) {
    hipError_t e = hipMallocAsync((void**)&tmp, sizeof(T) * (size_t)batch * T1, st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(tmp, hist, sizeof(T) * (size_t)batch * T1, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
    hist_in = tmp;
  }
  dim3 grid((B + kFirChunk - 1) / kFirChunk, batch);
  if constexpr (sizeof(T) == 4)
    hipLaunchKernelGGL(fir_f32_kernel, grid, dim3(kBlock), 0, st, (const float*)coeffs, T_, (const float*)src,
                       (float*)dst, B, (const float*)hist_in);
  else
    hipLaunchKernelGGL(fir_q15_kernel, grid, dim3(kBlock), 0, st, (const int16_t*)coeffs, T_,
                       (const int16_t*)src, (int16_t*)dst, B, (const int16_t*)hist_in);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (T1 > 0) {
    const uint64_t n = (uint64_t)batch * T1;
    // stream order: the filter pass has read hist_in before it is overwritten here
    hipLaunchKernelGGL(fir_hist_kernel<T>, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       src, hist, hist_in, B, T1, batch);
    e = hipGetLastError();
  }
  if (tmp) (void)hipFreeAsync(tmp, st);
  return e;
}

hipError_t fir_f32_launch(const float* coeffs, int num_taps, const float* src, float* dst, uint32_t block_size,
                          uint32_t batch, float* hist, hipStream_t st) {
  return fir_launch<float>(coeffs, num_taps, src, dst, block_size, batch, hist, st);
}
hipError_t fir_q15_launch(const int16_t* coeffs, int num_taps, const int16_t* src, int16_t* dst,
                          uint32_t block_size, uint32_t batch, int16_t* hist, hipStream_t st) {
  return fir_launch<int16_t>(coeffs, num_taps, src, dst, block_size, batch, hist, st);
}

}  // namespace mi355x
