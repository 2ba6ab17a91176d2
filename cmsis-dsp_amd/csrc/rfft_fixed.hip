// Real FFT, q31 and q15 — the split / merge passes around the batched fixed-point CFFT
// (MI355X, gfx950), bit-exact.
//
// Replaces the host scalar path of
//   q31: Source/TransformFunctions/arm_rfft_q31.c:148-183 (dispatch),
//        arm_split_rfft_q31 :256-341, arm_split_rifft_q31 :397-476 (scalar branches);
//   q15: arm_rfft_q15.c dispatch, arm_split_rfft_q15 / arm_split_rifft_q15
//        (!ARM_MATH_DSP branches);
//   the inverse's arm_shift_q31 / arm_shift_q15 by +1 is folded into the inverse CFFT's
//   store (kSatShl1, cfft_fixed.hip).
// L = N/2 complex bins of the inner CFFT.  One thread per k for 8 signals, k in [0, L):
//   forward: reads bins k and L-k of the CFFT output, writes spectrum bin k and, for
//            k >= 1, its mirror N-k (thread k = 0 writes bins 0 and L) -> 2N words out;
//   inverse: reads bins k and L-k of the 2N-word spectrum row, writes bin k of the N-word
//            CFFT input.
// Twiddle c = 2*modifier*k into realCoef{A,B} (shared 8192-entry tables, L2-resident).
#include "common.hpp"
#include "kernels.hpp"
#include "rfft_fixed_split.hpp"

namespace mi355x {

namespace {

// Work mapping: a workgroup takes kper = min(L, 256) consecutive k for R signals at a time
// (256 / kper signals side by side); each thread loads its k's twiddles once — a strided
// gather, realCoef index 2*mod*k — and reuses them for its R signals (the gather per element
// bound the pass: 1.39 ms for 2^18 x 1024-point q31 splits at one signal per thread).
constexpr int kRfftRows = 8;
struct RfftMap {
  uint64_t row0;    // first signal of this thread
  uint32_t rstep;   // signals between this thread's consecutive rows
  int k;
};
__device__ __forceinline__ RfftMap rfft_map(int L) {
  const int kper = L < 256 ? L : 256;
  const uint32_t nk = (uint32_t)(L / kper), side = 256u / (uint32_t)kper;
  const uint32_t kc = blockIdx.x % nk, rg = blockIdx.x / nk;
  RfftMap m;
  m.k = (int)(kc * kper + threadIdx.x % kper);
  m.rstep = side;
  m.row0 = (uint64_t)rg * side * kRfftRows + threadIdx.x / kper;
  return m;
}

template <typename T>
__global__ __launch_bounds__(256) void rfft_fx_split_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                            uint64_t rows, int n, const T* __restrict__ ta,
                                                            const T* __restrict__ tb, uint32_t mod) {
  const int L = n >> 1;
  const RfftMap mp = rfft_map(L);
  const int k = mp.k;
  const uint32_t c = 2u * mod * (uint32_t)k;
  const int32_t a1 = ta[c], a2 = ta[c + 1], b1 = tb[c], b2 = tb[c + 1];
  // all rows' loads first (rows past the batch re-read the last row and store nothing), so
  // each thread has 16 loads in flight instead of one row's latency at a time
  int2 av[kRfftRows], bv[kRfftRows];
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = min(mp.row0 + (uint64_t)r * mp.rstep, rows - 1);
    const T* x = src + row * (uint64_t)n;
    av[r] = Cx<T>::ld(x + 2 * k);
    bv[r] = Cx<T>::ld(x + (k == 0 ? 0 : 2 * (L - k)));   // bin L would lie past the row (k = 0 uses a only)
  }
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = mp.row0 + (uint64_t)r * mp.rstep;
    if (row >= rows) break;
    T* y = dst + row * (uint64_t)(2 * n);
    const int2 a = av[r], b = bv[r];
    if (k == 0) {
      const int2 v = a;     // bin 0: x[0], x[1]
      if constexpr (sizeof(T) == 4) {
        Cx<T>::st(y + n, wsub(v.x, v.y) >> 1, 0);
        Cx<T>::st(y, wadd(v.x, v.y) >> 1, 0);
      } else {
        Cx<T>::st(y + n, (v.x - v.y) >> 1, 0);
        Cx<T>::st(y, (v.x + v.y) >> 1, 0);
      }
      continue;
    }
    if constexpr (sizeof(T) == 4) {
      // arm_rfft_q31.c:293-326
      int32_t re = mult_R(a.x, a1), im = mult_R(a.x, a2);
      re = multSub_R(re, a.y, a2); im = multAcc_R(im, a.y, a1);
      re = multSub_R(re, b.y, a2); im = multSub_R(im, b.y, b1);
      re = multAcc_R(re, b.x, b1); im = multSub_R(im, b.x, a2);
      Cx<T>::st(y + 2 * k, re, im);
      Cx<T>::st(y + 2 * n - 2 * k, re, wneg(im));
    } else {
      // arm_rfft_q15.c scalar branch: wrapping int sums, >> 16, stores truncate to q15_t
      const int32_t re = (int32_t)(p16(a.x, a1) - p16(a.y, a2) + p16(b.x, b1) + p16(b.y, b2)) >> 16;
      const int32_t im = (int32_t)(p16(b.x, b2) - p16(b.y, b1) + p16(a.y, a1) + p16(a.x, a2)) >> 16;
      Cx<T>::st(y + 2 * k, re, im);
      Cx<T>::st(y + 2 * n - 2 * k, re, -im);
    }
  }
}

// Paired forward split (rfft_fixed_split.hpp): bins k and L - k read the same two CFFT bins
// (x[k], x[L-k]), so one thread forms both (j in [1, L/2): bins j and L - j; j = 0: bins 0, L and
// L/2) and every CFFT word is read once instead of twice.
template <typename T>
__global__ __launch_bounds__(256) void rfft_fx_split2_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                             uint64_t rows, int n, const T* __restrict__ ta,
                                                             const T* __restrict__ tb, uint32_t mod) {
  const int L = n >> 1, H = L >> 1;
  const RfftMap mp = rfft_map(H);
  const int j = mp.k;
  const int k2 = j == 0 ? H : L - j;                   // the partner bin
  const uint32_t c1 = 2u * mod * (uint32_t)j, c2 = 2u * mod * (uint32_t)k2;
  const int32_t a1 = ta[c1], a2 = ta[c1 + 1], b1 = tb[c1], b2 = tb[c1 + 1];
  const int32_t e1 = ta[c2], e2 = ta[c2 + 1], f1 = tb[c2], f2 = tb[c2 + 1];
  int2 av[kRfftRows], bv[kRfftRows];
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = min(mp.row0 + (uint64_t)r * mp.rstep, rows - 1);
    const T* x = src + row * (uint64_t)n;
    av[r] = Cx<T>::ld(x + 2 * j);
    bv[r] = Cx<T>::ld(x + 2 * k2);
  }
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = mp.row0 + (uint64_t)r * mp.rstep;
    if (row >= rows) break;
    T* y = dst + row * (uint64_t)(2 * n);
    const int2 a = av[r], b = bv[r];
    if (j == 0) {
      if constexpr (sizeof(T) == 4) {
        Cx<T>::st(y + n, wsub(a.x, a.y) >> 1, 0);
        Cx<T>::st(y, wadd(a.x, a.y) >> 1, 0);
      } else {
        Cx<T>::st(y + n, (a.x - a.y) >> 1, 0);
        Cx<T>::st(y, (a.x + a.y) >> 1, 0);
      }
      rfft_st_pair<T>(y, H, n, rfft_split_bin<T>(b, b, e1, e2, f1, f2));   // bin L/2: x[L/2] both ways
      continue;
    }
    rfft_st_pair<T>(y, j, n, rfft_split_bin<T>(a, b, a1, a2, b1, b2));
    rfft_st_pair<T>(y, k2, n, rfft_split_bin<T>(b, a, e1, e2, f1, f2));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void rfft_fx_merge_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                            uint64_t rows, int n, const T* __restrict__ ta,
                                                            const T* __restrict__ tb, uint32_t mod) {
  const int L = n >> 1;
  const RfftMap mp = rfft_map(L);
  const int k = mp.k;
  const uint32_t c = 2u * mod * (uint32_t)k;
  const int32_t a1 = ta[c], a2 = ta[c + 1], b1 = tb[c], b2 = tb[c + 1];
  int2 av[kRfftRows], bv[kRfftRows];
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = min(mp.row0 + (uint64_t)r * mp.rstep, rows - 1);
    const T* x = src + row * (uint64_t)(2 * n);
    av[r] = Cx<T>::ld(x + 2 * k);
    bv[r] = Cx<T>::ld(x + 2 * (L - k));
  }
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = mp.row0 + (uint64_t)r * mp.rstep;
    if (row >= rows) break;
    T* y = dst + row * (uint64_t)n;
    const int2 a = av[r], b = bv[r];
    if constexpr (sizeof(T) == 4) {
      // arm_rfft_q31.c:430-466
      int32_t re = mult_R(a.x, a1), im = mult_R(a.x, wneg(a2));
      re = multAcc_R(re, a.y, a2); im = multAcc_R(im, a.y, a1);
      re = multAcc_R(re, b.y, a2); im = multSub_R(im, b.y, b1);
      re = multAcc_R(re, b.x, b1); im = multAcc_R(im, b.x, a2);
      Cx<T>::st(y + 2 * k, re, im);
    } else {
      const int32_t re = (int32_t)(p16(b.x, b1) - p16(b.y, b2) + p16(a.x, a1) + p16(a.y, a2)) >> 16;
      const int32_t im = (int32_t)(p16(a.y, a1) - p16(a.x, a2) - p16(b.x, b2) - p16(b.y, b1)) >> 16;
      Cx<T>::st(y + 2 * k, re, im);
    }
  }
}

// Paired inverse merge: bins k and L - k of the N-word CFFT input read the same two spectrum
// bins (X[k], X[L-k]); j in [1, L/2) forms both, j = 0 forms bin 0 (X[0], X[L]) and bin L/2.
template <typename T>
__global__ __launch_bounds__(256) void rfft_fx_merge2_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                             uint64_t rows, int n, const T* __restrict__ ta,
                                                             const T* __restrict__ tb, uint32_t mod) {
  const int L = n >> 1, H = L >> 1;
  const RfftMap mp = rfft_map(H);
  const int j = mp.k;
  const int k2 = j == 0 ? H : L - j;
  const uint32_t c1 = 2u * mod * (uint32_t)j, c2 = 2u * mod * (uint32_t)k2;
  const int32_t a1 = ta[c1], a2 = ta[c1 + 1], b1 = tb[c1], b2 = tb[c1 + 1];
  const int32_t e1 = ta[c2], e2 = ta[c2 + 1], f1 = tb[c2], f2 = tb[c2 + 1];
  int2 av[kRfftRows], bv[kRfftRows], hv[kRfftRows];
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = min(mp.row0 + (uint64_t)r * mp.rstep, rows - 1);
    const T* x = src + row * (uint64_t)(2 * n);
    av[r] = Cx<T>::ld(x + 2 * j);
    bv[r] = Cx<T>::ld(x + 2 * (L - j));                // j = 0: X[L], bin 0's partner
    hv[r] = j == 0 ? Cx<T>::ld(x + 2 * H) : make_int2(0, 0);
  }
#pragma unroll
  for (int r = 0; r < kRfftRows; ++r) {
    const uint64_t row = mp.row0 + (uint64_t)r * mp.rstep;
    if (row >= rows) break;
    T* y = dst + row * (uint64_t)n;
    const int2 a = av[r], b = bv[r];
    const int2 v1 = rfft_merge_bin<T>(a, b, a1, a2, b1, b2);
    Cx<T>::st(y + 2 * j, v1.x, v1.y);
    const int2 v2 = j == 0 ? rfft_merge_bin<T>(hv[r], hv[r], e1, e2, f1, f2) : rfft_merge_bin<T>(b, a, e1, e2, f1, f2);
    Cx<T>::st(y + 2 * k2, v2.x, v2.y);
  }
}

}  // namespace

template <typename T>
static hipError_t rfft_fx_pass(bool inverse, int n, const T* src, T* dst, uint32_t batch, const T* ta, const T* tb,
                               uint32_t mod, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const int L = n / 2, kper = L < 256 ? L : 256;
  const uint64_t side = 256 / kper, groups = (batch + side * kRfftRows - 1) / (side * kRfftRows);
  const uint64_t blocks = groups * (uint64_t)(L / kper);
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  if (L >= 4) {   // paired kernels (every length the reference's init accepts)
    const int H = L / 2, hper = H < 256 ? H : 256;
    const uint64_t hside = 256 / hper, hgroups = (batch + hside * kRfftRows - 1) / (hside * kRfftRows);
    const dim3 g2((uint32_t)(hgroups * (uint64_t)(H / hper)));
    if (inverse)
      hipLaunchKernelGGL((rfft_fx_merge2_kernel<T>), g2, dim3(256), 0, st, src, dst, (uint64_t)batch, n, ta, tb, mod);
    else
      hipLaunchKernelGGL((rfft_fx_split2_kernel<T>), g2, dim3(256), 0, st, src, dst, (uint64_t)batch, n, ta, tb, mod);
  } else if (inverse)
    hipLaunchKernelGGL((rfft_fx_merge_kernel<T>), dim3((uint32_t)blocks), dim3(256), 0, st, src, dst, (uint64_t)batch,
                       n, ta, tb, mod);
  else
    hipLaunchKernelGGL((rfft_fx_split_kernel<T>), dim3((uint32_t)blocks), dim3(256), 0, st, src, dst, (uint64_t)batch,
                       n, ta, tb, mod);
  return hipGetLastError();
}

hipError_t rfft_q31_pass_launch(bool inverse, int n, const int32_t* src, int32_t* dst, uint32_t batch,
                                const int32_t* ta, const int32_t* tb, uint32_t mod, hipStream_t st) {
  return rfft_fx_pass<int32_t>(inverse, n, src, dst, batch, ta, tb, mod, st);
}
hipError_t rfft_q15_pass_launch(bool inverse, int n, const int16_t* src, int16_t* dst, uint32_t batch,
                                const int16_t* ta, const int16_t* tb, uint32_t mod, hipStream_t st) {
  return rfft_fx_pass<int16_t>(inverse, n, src, dst, batch, ta, tb, mod, st);
}

}  // namespace mi355x
