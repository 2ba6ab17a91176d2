// Element arithmetic of the MFCC q31 / q15 front end (arm_mfcc_q31.c:119-138, arm_mfcc_q15.c:
// 128-146 and the functions they call: arm_absmax, arm_divide, arm_scale, arm_mult), shared by
// the MFCC kernels (mfcc_fixed.hip) and the radix-16 CFFT's MFCC prologue (cfft_fixed_r16.hip).
#pragma once
#include "common.hpp"

namespace mi355x {

__device__ __forceinline__ int32_t mq_sat_abs(int32_t x) { return x > 0 ? x : (x == INT32_MIN ? INT32_MAX : -x); }
__device__ __forceinline__ uint32_t mq_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }
__device__ __forceinline__ int32_t mq_shl(int32_t x, int k) { return (int32_t)((uint32_t)x << (k & 31)); }
__device__ __forceinline__ int32_t mq_ssat31(int32_t v) {
  return v > 0x3FFFFFFF ? 0x3FFFFFFF : (v < -0x40000000 ? -0x40000000 : v);
}
__device__ __forceinline__ int32_t mq_hi(int32_t a, int32_t b) { return (int32_t)(((int64_t)a * b) >> 32); }

// arm_scale_q31.c, one element: in = (x * frac) >> 32, then << kShift with saturation, or
// >> -kShift (kShift = shift + 1 as int8_t)
__device__ __forceinline__ int32_t mq_scale(int32_t x, int32_t frac, int k) {
  const int32_t in = mq_hi(x, frac);
  if (k >= 0) {
    const int32_t out = mq_shl(in, k);
    return in != (out >> (k & 31)) ? (0x7FFFFFFF ^ (in >> 31)) : out;
  }
  return in >> ((-k) & 31);
}

__device__ __forceinline__ int32_t mq_sat_abs15(int32_t x) { return x > 0 ? x : (x == -32768 ? 32767 : -x); }
__device__ __forceinline__ int32_t mq_ssat16(int32_t v) { return v > 32767 ? 32767 : (v < -32768 ? -32768 : v); }

// The per-frame pre pass: m = max sat|x|; if m is neither 0 nor full scale, x = arm_scale(x,
// arm_divide(full, m)); then x = arm_mult(x, window).
template <typename T> struct MqPre;
template <> struct MqPre<int32_t> {
  static constexpr int32_t kFull = 0x7FFFFFFF;
  __device__ static int32_t sat_abs(int32_t x) { return mq_sat_abs(x); }
  // arm_divide_q31(0x7FFFFFFF, m): both positive, temp = (num << 31) / den, normalised to 32 bits;
  // k = (int8_t)(shift + 1), the arm_scale_q31 exponent
  __device__ static void divide(int32_t m, int32_t& quot, int& k) {
    int64_t t = (int64_t)(((uint64_t)0x7FFFFFFF << 31) / (uint64_t)m);
    const int sn = 32 - (int)mq_clz((uint32_t)(t >> 31));
    int sh = 0;
    if (sn > 0) {
      sh = sn;
      t >>= sn;
    }
    quot = (int32_t)t;
    k = (int)(int8_t)(sh + 1);
  }
  __device__ static int32_t pre(int32_t x, int32_t w, bool scale, int32_t quot, int k) {
    if (scale) x = mq_scale(x, quot, k);
    return mq_shl(mq_ssat31(mq_hi(x, w)), 1);          // arm_mult_q31: __SSAT((a*b) >> 32, 31) << 1
  }
};
template <> struct MqPre<int16_t> {
  static constexpr int32_t kFull = 0x7FFF;
  __device__ static int32_t sat_abs(int32_t x) { return mq_sat_abs15(x); }
  // arm_divide_q15(0x7FFF, m): temp = (0x7FFF << 15) / m, normalised by 17 - clz(temp); k = 15 - shift
  __device__ static void divide(int32_t m, int32_t& quot, int& k) {
    int32_t t = (int32_t)((0x7FFFu << 15) / (uint32_t)m);
    const int sn = 17 - (int)mq_clz((uint32_t)t);
    int sh = 0;
    if (sn > 0) {
      sh = sn;
      t >>= sn;
    }
    quot = (int32_t)(int16_t)t;
    k = (int)(int8_t)(15 - sh);
  }
  __device__ static int32_t pre(int32_t x, int32_t w, bool scale, int32_t quot, int k) {
    if (scale) x = mq_ssat16((x * quot) >> k);       // arm_scale_q15
    return mq_ssat16((x * w) >> 15);                  // arm_mult_q15
  }
};

}  // namespace mi355x
