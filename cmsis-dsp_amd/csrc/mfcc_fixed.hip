// Batched MFCC q31 / q15 — MI355X kernels around the batched fixed-point real FFT, bit-exact.
//
// Replaces Source/TransformFunctions/arm_mfcc_q31.c:88-225 (RFFT-based default build, host
// scalar path: ARM_MATH_LOOPUNROLL, no ARM_MATH_DSP) for `batch` frames, in three
// stream-ordered launches:
//   mfcc_q31_pre   m = max sat|x| (arm_absmax_q31), (quot, sh) = arm_divide_q31(0x7FFFFFFF, m),
//                  x = arm_scale_q31(x, quot, sh) if m != 0, 0x7FFFFFFF, x = arm_mult_q31(x, w)
//                  -> X (in place), m -> dst[frame][0]               [one wave per frame]
//   rfft           arm_rfft_q31 forward on X -> Y                     [the bit-exact batched RFFT]
//   mfcc_q31_post  |Y_k|, k <= fftLen/2 (arm_cmplx_mag_q31 + arm_sqrt_q31), Mel dot products
//                  (arm_dot_prod_q31: Σ (a·b) >> 14, + MICRO_Q31, >> 28, __SSAT(int32, 31)),
//                  arm_scale_q31(., m, 0), arm_vlog_q31, arm_offset_q31, arm_shift_q31(-3),
//                  DCT rows (arm_mat_vec_mult_q31: (q31)(Σ a·b >> 31)) [one wave per frame, LDS]
// Every stage is integer arithmetic; the sums are exact int64 (order-free), so each lane may
// own whole Mel filters / DCT rows.  Shift counts are taken mod 32 as on the reference's host
// (only m = 1 reaches a count of 32).
#include "common.hpp"
#include "kernels.hpp"
#include "cfft_fixed_core.hpp"
#include "mfcc_fixed_ops.hpp"
#include "mfcc_fixed_post.hpp"

namespace mi355x {

constexpr int kMqWaves = 4;   // frames (waves) per 256-thread workgroup

__device__ __forceinline__ int32_t wave_max_i(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// src and x may alias (in place): each lane rewrites only the words it read
__global__ __launch_bounds__(256) void mfcc_q31_pre_kernel(const int32_t* src, const int32_t* __restrict__ win,
                                                           int32_t* x, int32_t* maxv, int maxv_stride, int n,
                                                           uint32_t batch) {
  const int lane = threadIdx.x & 63;
  const uint32_t frame = blockIdx.x * kMqWaves + (threadIdx.x >> 6);
  if (frame >= batch) return;
  const int4* s = reinterpret_cast<const int4*>(src + (size_t)frame * n);
  const int4* w = reinterpret_cast<const int4*>(win);
  int4* o = reinterpret_cast<int4*>(x + (size_t)frame * n);
  const int n4 = n >> 2;
  // max of the saturated magnitudes (the reference's index is not used by the MFCC)
  int32_t m = 0;
  for (int i = lane; i < n4; i += 64) {
    const int4 v = s[i];
    m = max(m, max(max(mq_sat_abs(v.x), mq_sat_abs(v.y)), max(mq_sat_abs(v.z), mq_sat_abs(v.w))));
  }
  m = wave_max_i(m);
  // arm_divide_q31(0x7FFFFFFF, m): both positive, temp = (num << 31) / den, normalised to 32 bits
  const bool scale = m != 0 && m != 0x7FFFFFFF;
  int32_t quot = 0;
  int k = 1;
  if (scale) {
    int64_t t = (int64_t)(((uint64_t)0x7FFFFFFF << 31) / (uint64_t)m);
    const int sn = 32 - (int)mq_clz((uint32_t)(t >> 31));
    int sh = 0;
    if (sn > 0) {
      sh = sn;
      t >>= sn;
    }
    quot = (int32_t)t;
    k = (int)(int8_t)(sh + 1);     // kShift = (int8_t)(shift + 1)
  }
  for (int i = lane; i < n4; i += 64) {
    int4 v = s[i];
    if (scale) {
      v.x = mq_scale(v.x, quot, k); v.y = mq_scale(v.y, quot, k);
      v.z = mq_scale(v.z, quot, k); v.w = mq_scale(v.w, quot, k);
    }
    const int4 c = w[i];   // arm_mult_q31: __SSAT((a*b) >> 32, 31) << 1
    o[i] = make_int4(mq_shl(mq_ssat31(mq_hi(v.x, c.x)), 1), mq_shl(mq_ssat31(mq_hi(v.y, c.y)), 1),
                     mq_shl(mq_ssat31(mq_hi(v.z, c.z)), 1), mq_shl(mq_ssat31(mq_hi(v.w, c.w)), 1));
  }
  if (lane == 0) maxv[(size_t)frame * maxv_stride] = m;
}

constexpr int kMqFpw = 6;   // frames per wave (two groups of 3 with the suite's 20 Mel filters)

// The post kernel: frames' CFFT outputs in global memory (y), maxima in maxv.  A wave runs
// kMqFpw frames in groups of G = mq_group(nb_mel): the Mel sums of every frame of a group, then
// the group's finishes (one lane per (frame, filter)) and DCT rows (one lane per (frame, row)).
template <typename T, typename Ops>
__device__ __forceinline__ void mq_post_body(const Ops& op, const T* __restrict__ y, const int4* __restrict__ tw,
                                             const T* maxv, int maxv_stride, int n, int kmin, int kcnt, int nb_mel,
                                             const T* __restrict__ coefs, const uint32_t* __restrict__ bf, int total,
                                             int nb_dct, const T* __restrict__ dct, const int32_t* __restrict__ lut,
                                             T* dst, uint32_t batch, int stage) {
  extern __shared__ int32_t shq[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const MqTabs tb = mq_stage_tables<T>(shq, coefs, bf, total, nb_mel, nb_dct, dct, stage);
  int32_t* mag = shq + (stage ? mq_tab_words(total, nb_mel, nb_dct) : 0) + wave * mq_wave_words(n, nb_mel);
  int32_t* mel = mag + mq_mel_off(n, nb_mel);
  int32_t* mv = mag + mq_m_off(n, nb_mel);
  int64_t* acc = reinterpret_cast<int64_t*>(mag + mq_acc_off(n, nb_mel));
  auto dctw = [&](int i) { return tb.stage ? tb.dc[i] : (int32_t)dct[i]; };
  const int32_t lutv = lut[lane & 31];
  const int G = mq_group(nb_mel);
  const uint32_t first = (blockIdx.x * kMqWaves + wave) * kMqFpw;   // this wave's kMqFpw consecutive frames
  for (int it = 0; it < kMqFpw; it += G) {
    const uint32_t f0 = first + it;
    if (f0 >= batch) break;                            // wave-uniform: no workgroup barrier below
    const int g = (int)min((uint32_t)min(G, kMqFpw - it), batch - f0);
    for (int j = 0; j < g; ++j) {
      const uint32_t frame = f0 + j;
      if (lane == 0) mv[j] = (int32_t)maxv[(size_t)frame * maxv_stride];   // read before dst is written
      const T* X = y + (size_t)frame * n;              // CFFT output, L complex
      auto get = [X](int i) {
        if constexpr (sizeof(T) == 4) return reinterpret_cast<const int2*>(X)[i];
        else { const short2 v = reinterpret_cast<const short2*>(X)[i]; return make_int2(v.x, v.y); }
      };
      mq_mel_frame<T>(op, get, tw, n, kmin, kcnt, nb_mel, total, tb, coefs, lutv, mag, acc + j * nb_mel);
    }
    mq_finish_group(op, g, nb_mel, nb_dct, acc, mv, mel, dctw,
                    [&](int j, int r, int32_t v) { dst[(size_t)(f0 + j) * nb_dct + r] = (T)v; });
  }
}

__global__ __launch_bounds__(256) void mfcc_q31_post_kernel(const int32_t* __restrict__ y, const int4* __restrict__ tw,
                                                            const int32_t* maxv, int maxv_stride, int n, int kmin, int kcnt,
                                                            int nb_mel, const int32_t* __restrict__ coefs,
                                                            const uint32_t* __restrict__ bf, int total, int nb_dct,
                                                            const int32_t* __restrict__ dct,
                                                            const int32_t* __restrict__ lut, int32_t* dst,
                                                            uint32_t batch, int stage) {
  mq_post_body<int32_t>(MqOpsQ31(n, nb_mel, nb_dct), y, tw, maxv, maxv_stride, n, kmin, kcnt, nb_mel, coefs, bf, total, nb_dct, dct,
                        lut, dst, batch, stage);
}

// ---------------------------------------------------------------- q15
// arm_mfcc_q15.c:96-228: the same three launches on q15 frames.  pre: m = max sat|x| (q15),
// arm_divide_q15(0x7FFF, m) -> x = __SSAT((x * quot) >> (15 - shift), 16) (arm_scale_q15),
// x = __SSAT((x * w) >> 15, 16) (arm_mult_q15).  post: |Y_k| = sqrt_q31(((u32)re² + (u32)im²)
// >> 1) >> 16 (arm_cmplx_mag_q15), Mel = __SSAT((Σ mag·c + MICRO_Q15) >> 10, 31), scale_q31 by
// m << 16, log_q31, offset, >> 19, truncated to q15; DCT rows as arm_mat_vec_mult_q15 with
// its __SMLALD column pairs (int32-wrapped pair sums, none.h:497-506).

__global__ __launch_bounds__(256) void mfcc_q15_pre_kernel(const int16_t* src, const int16_t* __restrict__ win,
                                                           int16_t* x, int16_t* maxv, int maxv_stride, int n,
                                                           uint32_t batch) {
  const int lane = threadIdx.x & 63;
  const uint32_t frame = blockIdx.x * kMqWaves + (threadIdx.x >> 6);
  if (frame >= batch) return;
  const short4* s = reinterpret_cast<const short4*>(src + (size_t)frame * n);
  const short4* w = reinterpret_cast<const short4*>(win);
  short4* o = reinterpret_cast<short4*>(x + (size_t)frame * n);
  const int n4 = n >> 2;
  int32_t m = 0;
  for (int i = lane; i < n4; i += 64) {
    const short4 v = s[i];
    m = max(m, max(max(mq_sat_abs15(v.x), mq_sat_abs15(v.y)), max(mq_sat_abs15(v.z), mq_sat_abs15(v.w))));
  }
  m = wave_max_i(m);
  const bool scale = m != 0 && m != 0x7FFF;
  int32_t quot = 0, k = 15;
  if (scale) {   // arm_divide_q15(0x7FFF, m): temp = (0x7FFF << 15) / m, normalised by 17 - clz(temp)
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
  for (int i = lane; i < n4; i += 64) {
    short4 v = s[i];
    int32_t a[4] = {v.x, v.y, v.z, v.w};
    const short4 c = w[i];
    const int32_t cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (scale) a[j] = mq_ssat16((a[j] * quot) >> k);
      a[j] = mq_ssat16((a[j] * cw[j]) >> 15);
    }
    o[i] = make_short4((short)a[0], (short)a[1], (short)a[2], (short)a[3]);
  }
  if (lane == 0) maxv[(size_t)frame * maxv_stride] = (int16_t)m;
}

__global__ __launch_bounds__(256) void mfcc_q15_post_kernel(const int16_t* __restrict__ y, const int4* __restrict__ tw,
                                                            const int16_t* maxv, int maxv_stride, int n, int kmin, int kcnt,
                                                            int nb_mel, const int16_t* __restrict__ coefs,
                                                            const uint32_t* __restrict__ bf, int total, int nb_dct,
                                                            const int16_t* __restrict__ dct,
                                                            const int32_t* __restrict__ lut, int16_t* dst,
                                                            uint32_t batch, int stage) {
  mq_post_body<int16_t>(MqOpsQ15(n, nb_mel, nb_dct), y, tw, maxv, maxv_stride, n, kmin, kcnt, nb_mel, coefs, bf, total,
                        nb_dct, dct, lut, dst, batch, stage);
}

hipError_t mfcc_q15_pre_launch(int n, const int16_t* src, const int16_t* win, int16_t* x, int16_t* maxv,
                               uint32_t batch, int maxv_stride, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  if (n < 32 || (n & 3)) return hipErrorInvalidValue;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  hipLaunchKernelGGL(mfcc_q15_pre_kernel, dim3(grid), dim3(64 * kMqWaves), 0, st, src, win, x, maxv, maxv_stride, n,
                     batch);
  return hipGetLastError();
}

hipError_t mfcc_q15_post_launch(int n, const int16_t* y, const int4* tw, const int16_t* maxv, int maxv_stride, int nb_mel,
                                int kmin, int kcnt, const int16_t* coefs, const uint32_t* bf, int total, int nb_dct, const int16_t* dct, const int32_t* lut, int16_t* dst, uint32_t batch,
                                hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  const uint32_t grid2 = (batch + kMqFpw * kMqWaves - 1) / (kMqFpw * kMqWaves);
  const size_t tab = sizeof(int32_t) * (size_t)mq_tab_words(total, nb_mel, nb_dct);
  const int stage = mfcc_q31_post_lds(n, nb_mel) + tab <= 65536 ? 1 : 0;
  (void)grid;
  hipLaunchKernelGGL(mfcc_q15_post_kernel, dim3(grid2), dim3(64 * kMqWaves),
                     mfcc_q31_post_lds(n, nb_mel) + (stage ? tab : 0), st, y, tw, maxv, maxv_stride, n, kmin, kcnt, nb_mel,
                     coefs, bf, total, nb_dct, dct, lut, dst, batch, stage);
  return hipGetLastError();
}

hipError_t mfcc_q31_pre_launch(int n, const int32_t* src, const int32_t* win, int32_t* x, int32_t* maxv,
                               uint32_t batch, int maxv_stride, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  if (n < 32 || (n & 3)) return hipErrorInvalidValue;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  hipLaunchKernelGGL(mfcc_q31_pre_kernel, dim3(grid), dim3(64 * kMqWaves), 0, st, src, win, x, maxv, maxv_stride, n,
                     batch);
  return hipGetLastError();
}

size_t mfcc_q31_post_lds(int n, int nb_mel) { return sizeof(int32_t) * kMqWaves * (size_t)mq_wave_words(n, nb_mel); }

hipError_t mfcc_q31_post_launch(int n, const int32_t* y, const int4* tw, const int32_t* maxv, int maxv_stride, int nb_mel,
                                int kmin, int kcnt, const int32_t* coefs, const uint32_t* bf, int total, int nb_dct, const int32_t* dct, const int32_t* lut, int32_t* dst, uint32_t batch,
                                hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  const uint32_t grid2 = (batch + kMqFpw * kMqWaves - 1) / (kMqFpw * kMqWaves);
  const size_t tab = sizeof(int32_t) * (size_t)mq_tab_words(total, nb_mel, nb_dct);
  const int stage = mfcc_q31_post_lds(n, nb_mel) + tab <= 65536 ? 1 : 0;
  (void)grid;
  hipLaunchKernelGGL(mfcc_q31_post_kernel, dim3(grid2), dim3(64 * kMqWaves),
                     mfcc_q31_post_lds(n, nb_mel) + (stage ? tab : 0), st, y, tw, maxv, maxv_stride, n, kmin, kcnt, nb_mel,
                     coefs, bf, total, nb_dct, dct, lut, dst, batch, stage);
  return hipGetLastError();
}

}  // namespace mi355x
