// The fixed-point RFFT's forward split per bin (arm_split_rfft_q31, arm_rfft_q31.c:256-341;
// arm_split_rfft_q15, the scalar branch of arm_rfft_q15.c), shared by the split pass
// (rfft_fixed.hip) and the fused forward RFFTs (cfft_fixed.hip N = 8192, cfft_fixed_r16.hip
// N = 512 .. 4096); the inverse's merge per bin (arm_split_rifft_q31, arm_rfft_q31.c:397-476; the
// q15 scalar branch), shared by the merge pass and the fused inverse (cfft_fixed_r16.hip).
#pragma once
#include "common.hpp"

namespace mi355x {

// ((q63)x*y + 2^31) >> 32 forms of none.h:184-194 (SMMULR / SMMLAR / SMMLSR) -> common.hpp
__device__ __forceinline__ int32_t wneg(int32_t a) { return (int32_t)(0u - (uint32_t)a); }
// q15 x q15 product as a wrapping int32 term
__device__ __forceinline__ uint32_t p16(int32_t a, int32_t b) { return (uint32_t)(a * b); }

template <typename T> struct Cx;
template <> struct Cx<int32_t> {
  using C = int2;
  __device__ static int2 ld(const int32_t* p) { return *reinterpret_cast<const int2*>(p); }
  __device__ static void st(int32_t* p, int32_t re, int32_t im) { *reinterpret_cast<int2*>(p) = make_int2(re, im); }
};
template <> struct Cx<int16_t> {
  __device__ static int2 ld(const int16_t* p) {
    const short2 s = *reinterpret_cast<const short2*>(p);
    return make_int2(s.x, s.y);
  }
  __device__ static void st(int16_t* p, int32_t re, int32_t im) {
    *reinterpret_cast<short2*>(p) = make_short2((short)re, (short)im);
  }
};


// spectrum bin k from CFFT bins a = x[k], b = x[L - k] and the k-th twiddle record (a1, a2, b1, b2) =
// (A[2 mod k], A[2 mod k + 1], B[2 mod k], B[2 mod k + 1])
template <typename T>
__device__ __forceinline__ int2 rfft_split_bin(int2 a, int2 b, int32_t a1, int32_t a2, int32_t b1, int32_t b2) {
  if constexpr (sizeof(T) == 4) {
    int32_t re = mult_R(a.x, a1), im = mult_R(a.x, a2);
    re = multSub_R(re, a.y, a2); im = multAcc_R(im, a.y, a1);
    re = multSub_R(re, b.y, a2); im = multSub_R(im, b.y, b1);
    re = multAcc_R(re, b.x, b1); im = multSub_R(im, b.x, a2);
    return make_int2(re, im);
  } else {
    const int32_t re = (int32_t)(p16(a.x, a1) - p16(a.y, a2) + p16(b.x, b1) + p16(b.y, b2)) >> 16;
    const int32_t im = (int32_t)(p16(b.x, b2) - p16(b.y, b1) + p16(a.y, a1) + p16(a.x, a2)) >> 16;
    return make_int2(re, im);
  }
}
// CFFT input element k of the inverse from spectrum bins a = X[k], b = X[L - k] and the k-th record
template <typename T>
__device__ __forceinline__ int2 rfft_merge_bin(int2 a, int2 b, int32_t a1, int32_t a2, int32_t b1, int32_t b2) {
  if constexpr (sizeof(T) == 4) {
    // arm_rfft_q31.c:430-466
    int32_t re = mult_R(a.x, a1), im = mult_R(a.x, wneg(a2));
    re = multAcc_R(re, a.y, a2); im = multAcc_R(im, a.y, a1);
    re = multAcc_R(re, b.y, a2); im = multSub_R(im, b.y, b1);
    re = multAcc_R(re, b.x, b1); im = multAcc_R(im, b.x, a2);
    return make_int2(re, im);
  } else {
    const int32_t re = (int32_t)(p16(b.x, b1) - p16(b.y, b2) + p16(a.x, a1) + p16(a.y, a2)) >> 16;
    const int32_t im = (int32_t)(p16(a.y, a1) - p16(a.x, a2) - p16(b.x, b2) - p16(b.y, b1)) >> 16;
    return make_int2(re, im);
  }
}
template <typename T>
__device__ __forceinline__ void rfft_st_pair(T* y, int k, int n, int2 v) {   // bin k and its mirror 2n - 2k
  Cx<T>::st(y + 2 * k, v.x, v.y);
  if constexpr (sizeof(T) == 4) Cx<T>::st(y + 2 * n - 2 * k, v.x, wneg(v.y));
  else Cx<T>::st(y + 2 * n - 2 * k, v.x, -v.y);
}
// The split's twiddle record of bin k, (A0, A1, B0, B1) = (A[2 mod k], A[2 mod k + 1], B[2 mod k],
// B[2 mod k + 1]) (arm_rfft_q31.c:293-326 index), from one of two sources:
//  * SplitRecTab: packed per-bin records (device_split_records, runtime.hpp; int4 for q31, 8-B
//    short4 for q15), one load per bin -- the radix-16 fused RFFTs, whose mod = 8192 / N >= 2
//    would otherwise read four words at a stride of 2 mod;
//  * SplitStridedTab: the instance's tables as they are -- the N = 8192 fused RFFTs (mod = 1, the
//    words of a bin are adjacent): measured faster there than the records (q15 610 vs 564-567
//    Gsamples/s on one box, profiles/r05/ab_o2; q31 equal).
template <typename T> struct SplitRec;
template <> struct SplitRec<int32_t> { using R = int4; };
template <> struct SplitRec<int16_t> { using R = short4; };
template <typename T> struct SplitRecTab {
  const typename SplitRec<T>::R* rec;
  __device__ int4 operator()(int k) const {
    const auto r = rec[k];
    return make_int4(r.x, r.y, r.z, r.w);
  }
};
template <typename T> struct SplitStridedTab {
  const T* ta;
  const T* tb;
  uint32_t mod;
  __device__ int4 operator()(int k) const {
    const uint32_t c = 2u * mod * (uint32_t)k;
    return make_int4(ta[c], ta[c + 1], tb[c], tb[c + 1]);
  }
};

// Arguments of a CFFT kernel that runs the split on its own output (the fused forward RFFT)
template <typename T> struct RfSplitArgs {
  T* dst = nullptr;                                  // [batch][2 * fftLenReal] spectrum rows
  const typename SplitRec<T>::R* rec = nullptr;      // SplitRecTab (split and merge)
  const T* spec = nullptr;                           // the fused inverse's input spectrum rows
  const T* ta = nullptr;                             // SplitStridedTab
  const T* tb = nullptr;
  uint32_t mod = 0;
};

// Paired split unit j of one row (j in [0, L/2)): bins j and L - j with their mirrors (j = 0: bins
// 0, L and L/2), from get(i) = CFFT bin i of the row and tab(k) = the record of bin k; y = the
// row's 2N-word spectrum.
template <typename T, typename Get, typename Tab>
__device__ __forceinline__ void rfft_split_pair(Get get, T* __restrict__ y, int j, int n, const Tab& tab) {
  const int L = n >> 1, H = L >> 1;
  const int k2 = j == 0 ? H : L - j;
  const int2 a = get(j), b = get(k2);
  const int4 r2 = tab(k2);
  const int2 v2 = rfft_split_bin<T>(b, j == 0 ? b : a, r2.x, r2.y, r2.z, r2.w);
  if (j == 0) {
    if constexpr (sizeof(T) == 4) {
      Cx<T>::st(y + n, wsub(a.x, a.y) >> 1, 0);
      Cx<T>::st(y, wadd(a.x, a.y) >> 1, 0);
    } else {
      Cx<T>::st(y + n, (a.x - a.y) >> 1, 0);
      Cx<T>::st(y, (a.x + a.y) >> 1, 0);
    }
  } else {
    const int4 r1 = tab(j);
    rfft_st_pair<T>(y, j, n, rfft_split_bin<T>(a, b, r1.x, r1.y, r1.z, r1.w));
  }
  rfft_st_pair<T>(y, k2, n, v2);
}

}  // namespace mi355x
