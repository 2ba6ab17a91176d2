// Batched linear convolution / correlation family — MI355X kernels, bit-exact.
//
// Replaces the host scalar paths of Source/FilteringFunctions:
//   arm_conv_f32.c, arm_conv_q15.c (!ARM_MATH_DSP), arm_conv_q31.c       (full convolution)
//   arm_conv_partial_f32.c / _q15.c / _q31.c (!ARM_MATH_DSP branch, :635-679 / :715-759)
//   arm_correlate_f32.c / _q15.c / _q31.c   (!ARM_MATH_DSP branch, :1013-1096 / :814-895)
//   arm_conv_fast_q15.c, arm_conv_fast_q31.c, arm_correlate_fast_q15.c, _fast_q31.c
//   arm_conv_q7.c, arm_conv_partial_q7.c (!ARM_MATH_DSP, :688-735), arm_correlate_q7.c:
//     q31_t sum of q7 x q7 products (int32 adds / __SMLAD pairs, both wrap: a modular sum,
//     any order), output __SSAT(sum >> 7, 8)
// Every exact variant sums each output over the overlap in ASCENDING index of the summed
// input x (conv: pSrcA, whichever is longer; correlate: the longer input), f32 mul then add
// from 0.0f, q15/q31 an exact q63 sum.  Correlation is the convolution of x with the time-
// reversed shorter input, written forward at (srcALen - srcBLen) or, when srcALen <
// srcBLen, backward from srcALen + srcBLen - 2 (the reference's `inv` / `inc = -1`).
// The fast variants are modular sums (any order gives the reference's bits):
//   fast q31: acc += (x*y) >> 32 mod 2^32 (((q63)acc << 32 + x*y) >> 32), output acc << 1;
//   fast q15: acc += x*y mod 2^32 through __SMLAD, output (q15)(acc >> 15).  A single-sample
//   __SMLAD(*px, *py, acc) (none.h:455-463) also multiplies the HIGH halfwords of the two
//   sign-extended samples, (-1)*(-1) = +1 when both are negative; the reference does that
//   for the last count % 4 MACs of its stage-1 / stage-3 outputs (and, in arm_conv_fast_q15,
//   for every MAC of the stage-3 outputs after the first (srcBLen-1)/4), never in stage 2.
//   The stage-2 outputs take the windowed kernel; the edge outputs take the direct kernel,
//   which adds that +1 term (probe: tools/probes/conv_family_model.py, 0 mismatches).
//
// Windowed kernel: as a FIR over a zero-padded window, with c[t] = h[B-1-t] (conv) or h[t]
// (correlate), v[n] = sum_t w[n+t]*c[t], w[j] = x[j-(B-1)] (0 outside x), t ascending = k
// ascending.  The padded terms add +-0 to an accumulator that can never be -0.0 (it starts
// at +0.0 and an exact cancellation rounds to +0.0), so they change nothing -- for finite h
// (an infinite or NaN h would turn a padded 0*h into NaN where the reference skips the
// term).  Integer sums are exact.  One workgroup = one item x 2048 outputs, window staged in
// LDS, 8 outputs per lane from a register ring; c read wave-uniformly.  srcBLen >
// kConvMaxB: one thread per output, sum over the exact overlap.
#include "common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace mi355x {

constexpr int kConvR = 8, kConvChunk = kBlock * kConvR, kConvMaxB = 1024;
constexpr int kConvPre = (kConvChunk + kConvMaxB - 1 + kBlock - 1) / kBlock;

__device__ __forceinline__ int cpad(int i) { return i + (i >> 3); }   // as the f32 FIR window

// Accumulator semantics per op (ConvOp in kernels.hpp).
template <int OP> struct ConvT;
template <> struct ConvT<kConvF32> {
  using T = float; using Acc = float;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { const float p = w * c; return a + p; }
  static __device__ __forceinline__ T out(Acc a) { return a; }
};
template <> struct ConvT<kConvQ15> {
  using T = int16_t; using Acc = int64_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (int64_t)((int32_t)w * (int32_t)c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat16((int32_t)(a >> 15)); }
};
template <> struct ConvT<kConvQ31> {
  using T = int32_t; using Acc = uint64_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint64_t)((int64_t)w * c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)(int32_t)((int64_t)a >> 31); }
};
template <> struct ConvT<kConvFastQ15> {
  using T = int16_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)((int32_t)w * (int32_t)c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)((int32_t)a >> 15); }
};
// arm_conv_fast_opt_q15.c / arm_correlate_fast_opt_q15.c / arm_conv_partial_fast_opt_q15.c:
// __SMLAD over zero-padded scratch copies (no single-sample high-halfword term), a modular q31
// sum, output __SSAT(acc >> 15, 16) -- saturating, unlike arm_conv_fast_q15's (q15) cast.
template <> struct ConvT<kConvFastOptQ15> {
  using T = int16_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)((int32_t)w * (int32_t)c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat16((int32_t)a >> 15); }
};
template <> struct ConvT<kConvQ7> {
  using T = int8_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)((int32_t)w * (int32_t)c); }
  static __device__ __forceinline__ T out(Acc a) {
    const int32_t v = (int32_t)a >> 7;
    return (T)(v > 127 ? 127 : v < -128 ? -128 : v);
  }
};
template <> struct ConvT<kConvFastQ31> {
  using T = int32_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)__mulhi(w, c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)(a << 1); }
};

template <int OP, bool CORR>
__global__ __launch_bounds__(kBlock) void conv_kernel(const typename ConvT<OP>::T* __restrict__ X, uint32_t A,
                                                      uint64_t sx, const typename ConvT<OP>::T* __restrict__ Hh,
                                                      uint32_t B, uint64_t sh, typename ConvT<OP>::T* __restrict__ Y,
                                                      uint64_t sy, int64_t yoff, int ydir, uint32_t first,
                                                      uint32_t num, uint32_t nchunks) {
  using Op = ConvT<OP>;
  using T = typename Op::T;
  using Acc = typename Op::Acc;
  __shared__ T win[(kConvChunk + kConvMaxB) * 9 / 8 + 32];
  const uint32_t item = blockIdx.x / nchunks;
  const uint32_t cofs = (blockIdx.x - item * nchunks) * kConvChunk;
  const int n0 = (int)(first + cofs);
  const int count = min((int)(num - cofs), kConvChunk);
  const int total = count + (int)B - 1;
  const T* x = X + item * sx;
  const T* h = Hh + item * sh;
  T pre[kConvPre];
#pragma unroll
  for (int k = 0; k < kConvPre; ++k) {
    const int j = threadIdx.x + k * kBlock;
    const int xi = n0 + j - ((int)B - 1);                     // window word j = x[xi]
    const bool in = j < total && xi >= 0 && xi < (int)A;
    const T v = x[in ? xi : 0];
    pre[k] = in ? v : (T)0;
  }
#pragma unroll
  for (int k = 0; k < kConvPre; ++k) {
    const int j = threadIdx.x + k * kBlock;
    if (j < total) win[cpad(j)] = pre[k];
  }
  __syncthreads();
  const int base = threadIdx.x * kConvR;
  if (base >= count) return;
  Acc acc[kConvR];
  T w[kConvR];
#pragma unroll
  for (int r = 0; r < kConvR; ++r) { acc[r] = (Acc)0; w[r] = win[cpad(base + r)]; }
  const int Bi = (int)B;
  auto tap = [&](int t) { return CORR ? h[t] : h[Bi - 1 - t]; };
  int t = 0;
  for (; t + kConvR <= Bi; t += kConvR) {
#pragma unroll
    for (int u = 0; u < kConvR; ++u) {
      const T c = tap(t + u);
#pragma unroll
      for (int r = 0; r < kConvR; ++r) acc[r] = Op::mac(acc[r], w[(r + u) % kConvR], c);
      w[u] = win[cpad(base + t + u + kConvR)];
    }
  }
  for (; t < Bi; ++t) {
    const T c = tap(t);
#pragma unroll
    for (int r = 0; r < kConvR; ++r) acc[r] = Op::mac(acc[r], w[r], c);
#pragma unroll
    for (int r = 0; r < kConvR - 1; ++r) w[r] = w[r + 1];
    w[kConvR - 1] = win[cpad(base + kConvR + t)];
  }
  T* y = Y + (uint64_t)item * sy;
#pragma unroll
  for (int r = 0; r < kConvR; ++r)
    if (base + r < count) y[yoff + (int64_t)ydir * (n0 + base + r)] = Op::out(acc[r]);
}

// One thread per output over the exact overlap, k (index of x) ascending: long h, and the
// fast-q15 edge outputs (stage 1 / stage 3 of the reference), which add the single-sample
// __SMLAD high-halfword term over the k range the reference runs one sample at a time.
template <int OP, bool CORR>
__global__ __launch_bounds__(kBlock) void conv_direct_kernel(const typename ConvT<OP>::T* __restrict__ X, uint32_t A,
                                                             uint64_t sx, const typename ConvT<OP>::T* __restrict__ Hh,
                                                             uint32_t B, uint64_t sh,
                                                             typename ConvT<OP>::T* __restrict__ Y, uint64_t sy,
                                                             int64_t yoff, int ydir, uint32_t first, uint32_t num,
                                                             uint32_t batch) {
  using Op = ConvT<OP>;
  using T = typename Op::T;
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= (uint64_t)num * batch) return;
  const uint64_t item = g / num;
  const int64_t n = (int64_t)first + (int64_t)(g - item * num);
  const T* x = X + item * sx;
  const T* h = Hh + item * sh;
  const int64_t Ai = A, Bi = B;
  const int64_t k0 = n - Bi + 1 > 0 ? n - Bi + 1 : 0;
  const int64_t k1 = n < Ai - 1 ? n : Ai - 1;
  auto g_at = [&](int64_t m) { return CORR ? h[Bi - 1 - m] : h[m]; };   // g[m], m = n - k
  typename Op::Acc acc = 0;
  for (int64_t k = k0; k <= k1; ++k) acc = Op::mac(acc, x[k], g_at(n - k));
  if constexpr (OP == kConvFastQ15) {
    int64_t s0 = 1, s1 = 0;                                  // single-sample MAC range of k
    if (n <= Bi - 2) {                                       // stage 1: count = n + 1 MACs
      s0 = n + 1 - (n + 1) % 4; s1 = n;
    } else if (n >= Ai) {                                    // stage 3
      const int64_t cnt = Ai + Bi - 1 - n;
      s1 = Ai - 1;
      s0 = (!CORR && n - Ai >= (Bi - 1) / 4) ? n - Bi + 1 : Ai - cnt % 4;
    }
    for (int64_t k = s0; k <= s1; ++k) acc += (x[k] < 0 && g_at(n - k) < 0) ? 1u : 0u;
  }
  Y[item * sy + yoff + ydir * n] = Op::out(acc);
}

template <int OP, bool CORR>
static hipError_t launch_direct(const ConvJob& j, uint32_t first, uint32_t num, hipStream_t st) {
  using T = typename ConvT<OP>::T;
  if (num == 0) return hipSuccess;
  const uint64_t blocks = ((uint64_t)num * j.batch + kBlock - 1) / kBlock;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_direct_kernel<OP, CORR>), dim3((uint32_t)blocks), dim3(kBlock), 0, st, (const T*)j.x, j.A,
                     j.sx, (const T*)j.h, j.B, j.sh, (T*)j.y, j.sy, j.yoff, j.ydir, first, num, j.batch);
  return hipGetLastError();
}

// c[t] = h[B-1-t] per item row (the convolution's taps in the FIR's order)
__global__ void reverse_rows_kernel(const float* __restrict__ h, uint64_t sh, float* __restrict__ c, uint32_t B,
                                    uint32_t rows) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= (uint64_t)rows * B) return;
  const uint64_t r = g / B, t = g - r * B;
  c[g] = h[r * sh + (B - 1 - t)];
}

template <int OP, bool CORR>
static hipError_t launch_window(const ConvJob& j, uint32_t first, uint32_t num, hipStream_t st) {
  using T = typename ConvT<OP>::T;
  if (num == 0) return hipSuccess;
  if constexpr (OP == kConvF32) {
    // f32: the FIR kernel's register-window pass (fir.hip), taps in ascending index of x
    const float* c = (const float*)j.h;
    uint64_t cs = j.sh;
    float* rev = nullptr;
    if (!CORR) {
      const uint32_t rows = j.sh ? j.batch : 1u;
      hipError_t e = hipMallocAsync((void**)&rev, sizeof(float) * (size_t)rows * j.B, st);
      if (e != hipSuccess) return e;
      const uint64_t n = (uint64_t)rows * j.B;
      hipLaunchKernelGGL(reverse_rows_kernel, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                         (const float*)j.h, j.sh, rev, j.B, rows);
      c = rev;
      cs = j.sh ? j.B : 0;
    }
    hipError_t e = fir_f32_conv_pass(c, cs, (int)j.B, (const float*)j.x, j.sx, j.A, first, (float*)j.y, j.sy,
                                     j.yoff + (int64_t)j.ydir * first, j.ydir, num, j.batch, st);
    if (rev) (void)hipFreeAsync(rev, st);
    return e;
  }
  const uint64_t nchunks = ((uint64_t)num + kConvChunk - 1) / kConvChunk;
  if (nchunks * j.batch > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_kernel<OP, CORR>), dim3((uint32_t)(nchunks * j.batch)), dim3(kBlock), 0, st,
                     (const T*)j.x, j.A, j.sx, (const T*)j.h, j.B, j.sh, (T*)j.y, j.sy, j.yoff, j.ydir, first, num,
                     (uint32_t)nchunks);
  return hipGetLastError();
}

template <int OP, bool CORR>
static hipError_t conv_family_launch(const ConvJob& j, hipStream_t st) {
  const uint64_t L = (uint64_t)j.A + j.B - 1;
  if ((uint64_t)j.first + j.num > L || L > 0x7FFFFFFFull) return hipErrorInvalidValue;
  if (j.B > (uint32_t)kConvMaxB) return launch_direct<OP, CORR>(j, j.first, j.num, st);
  if constexpr (OP == kConvFastQ15) {
    // stage-1 outputs [0, B-1) and stage-3 outputs [A, L) carry the single-sample term
    const uint32_t end = j.first + j.num;
    const uint32_t s2b = j.B - 1, s2e = j.A;                  // stage 2: [B-1, A)
    const uint32_t m0 = j.first > s2b ? j.first : s2b, m1 = end < s2e ? end : s2e;
    hipError_t e = hipSuccess;
    if (j.first < s2b) e = launch_direct<OP, CORR>(j, j.first, (end < s2b ? end : s2b) - j.first, st);
    if (e == hipSuccess && m0 < m1) e = launch_window<OP, CORR>(j, m0, m1 - m0, st);
    if (e == hipSuccess && end > s2e) {
      const uint32_t a = j.first > s2e ? j.first : s2e;
      e = launch_direct<OP, CORR>(j, a, end - a, st);
    }
    return e;
  }
  return launch_window<OP, CORR>(j, j.first, j.num, st);
}

hipError_t conv_family_run(const ConvJob& j, hipStream_t st) {
  if (j.batch == 0 || j.A == 0 || j.B == 0 || j.num == 0) return hipSuccess;
  if (j.op == kConvFastQ15 && j.A < j.B) return hipErrorInvalidValue;  // host passes x = the longer input
#define MI355X_CONV_CASE(OP)                                                           \
  case OP: return j.corr ? conv_family_launch<OP, true>(j, st) : conv_family_launch<OP, false>(j, st);
  switch (j.op) {
    MI355X_CONV_CASE(kConvF32)
    MI355X_CONV_CASE(kConvQ15)
    MI355X_CONV_CASE(kConvQ31)
    MI355X_CONV_CASE(kConvFastQ15)
    MI355X_CONV_CASE(kConvFastQ31)
    MI355X_CONV_CASE(kConvQ7)
    MI355X_CONV_CASE(kConvFastOptQ15)
    default: return hipErrorInvalidValue;
  }
#undef MI355X_CONV_CASE
}

}  // namespace mi355x
