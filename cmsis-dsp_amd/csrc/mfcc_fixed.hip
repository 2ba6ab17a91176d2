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

// arm_sqrt_q31.c:55-125 (Newton on 1/sqrt from sqrt_initial_lut_q31, 3 iterations)
// lutv: lane l holds sqrt_initial_lut_q31[l & 31]; the entry is fetched with a lane shuffle
// (every lane of the wave must be active: callers run uniform loops)
__device__ __forceinline__ int32_t mq_sqrt(int32_t in, int32_t lutv) {
  const int sb = (int)mq_clz((uint32_t)in) - 1;
  const int e = sb & ~1;                             // signBits1 rounded down to even
  const int32_t number = in << e;
  int32_t v = __shfl(lutv, ((number >> 26) - (0x20000000 >> 26)) & 31, 64);
  if (in <= 0) return 0;
#pragma unroll
  for (int it = 0; it < 3; ++it) {
    int32_t t = (int32_t)(((int64_t)v * v) >> 28);
    t = (int32_t)(((int64_t)number * t) >> 31);
    t = 0x30000000 - t;
    v = (int32_t)(((int64_t)v * t) >> 29);
  }
  v = (int32_t)(((int64_t)number * v) >> 28);
  return v >> (e >> 1);
}

// arm_vlog_q31.c:55-121 (arm_scalar_log_q31): q5.26 natural log of a q31 value
__device__ __forceinline__ int32_t mq_log(uint32_t src) {
  const int c = (int)mq_clz(src);
  uint32_t x = c == 0 ? src >> 1 : src << (c - 1), y = 0, inc = (1u << 31) >> 6;
#pragma unroll
  for (int i = 0; i < 31; ++i) {
    x = (uint32_t)(((uint64_t)x * x) >> 30);         // x < 2^31: the product fits 62 bits
    if (x >= (1u << 31)) {
      y += inc;
      x >>= 1;
    }
    inc >>= 1;
  }
  const int32_t tmp = (int32_t)(y - ((uint32_t)c << 26));
  return (int32_t)(((int64_t)tmp * (int64_t)0x58b90bfb) >> 31);
}


// LDS per wave (int32 words): |X_k| (fftLen/2 + 1, at mq_mpad(k)), Mel values (nb_mel), then
// int64 Mel sums.  mq_mpad(k) = k + k / 16: the Mel sums read the magnitudes at lane strides of
// a slice length (often a multiple of 16 words), which the pad spreads over distinct banks.
__host__ __device__ inline int mq_mpad(int k) { return k + (k >> 4); }
__host__ __device__ inline int mq_mag_words(int n) { return mq_mpad(n / 2) + 1; }
__host__ __device__ inline int mq_wave_words(int n, int nb_mel) { return ((mq_mag_words(n) + nb_mel + 1) & ~1) + 2 * nb_mel; }

// The Mel sums spread over the wave: the filters' coefficients as one flat list (bf[g] =
// bin << 16 | filter), lane t summing the contiguous slice t of it and adding each filter's
// partial sum to its int64 LDS total (ds_add_u64).  The sums are exact int64 of exact (or
// per-term floor-shifted) products, so any order gives the reference's value (mq_post_body).


// Spectrum bin k (0 <= k <= L = fftLen/2) of the real FFT, formed from the inner CFFT output
// x (L complex) as arm_split_rfft_q31 / _q15 do (arm_rfft_q31.c:256-341, arm_rfft_q15.c scalar
// branch), with the k-th twiddle record tw[k] = {A[2mk], A[2mk+1], B[2mk], B[2mk+1]} (m = the
// instance's twidCoefRModifier; built contiguous on the host, so the loads coalesce): the
// post kernels take the magnitudes straight from the CFFT output, with no 2N-word spectrum.
// get(i) returns CFFT bin i of the frame (the CFFT output in global memory).
template <typename Get>
__device__ __forceinline__ int2 mq_split_q31(Get get, int k, int L, int4 t) {
  if (k == 0 || k == L) {
    const int2 v = get(0);
    return make_int2((k == 0 ? wadd(v.x, v.y) : wsub(v.x, v.y)) >> 1, 0);
  }
  const int2 a = get(k), b = get(L - k);
  int32_t re = mult_R(a.x, t.x), im = mult_R(a.x, t.y);
  re = multSub_R(re, a.y, t.y); im = multAcc_R(im, a.y, t.x);
  re = multSub_R(re, b.y, t.y); im = multSub_R(im, b.y, t.z);
  re = multAcc_R(re, b.x, t.z); im = multSub_R(im, b.x, t.y);
  return make_int2(re, im);
}
template <typename Get>   // get(i): bin i as int2 of sign-extended q15 words
__device__ __forceinline__ int2 mq_split_q15(Get get, int k, int L, int4 t) {
  if (k == 0 || k == L) {
    const int2 v = get(0);
    return make_int2((k == 0 ? v.x + v.y : v.x - v.y) >> 1, 0);
  }
  const int2 a = get(k), b = get(L - k);
  auto p = [](int32_t u, int32_t v) { return (uint32_t)(u * v); };
  const int32_t re = (int32_t)(p(a.x, t.x) - p(a.y, t.y) + p(b.x, t.z) + p(b.y, t.w)) >> 16;
  const int32_t im = (int32_t)(p(b.x, t.w) - p(b.y, t.z) + p(a.y, t.x) + p(a.x, t.y)) >> 16;
  return make_int2((int16_t)re, (int16_t)im);     // the split stores q15_t
}

// maxv may alias dst (frame maxima carried in dst[frame][0]): read before any output store.
// A workgroup stages the frame-invariant tables (flat Mel list, coefficients, DCT rows) in LDS
// once when they fit, then each wave runs kMqFpw frames; a wave's LDS region is its own, so the
// stages are ordered by wave barriers only (waves run independently; PMC of the one-frame,
// global-table version: 71 % of wave time waiting, VALU issue at 34 %).
constexpr int kMqFpw = 4;   // frames per wave
__device__ __forceinline__ void mq_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__host__ __device__ inline int mq_tab_words(int total, int nb_mel, int nb_dct) {
  return (2 * total + nb_mel * nb_dct + 3) & ~3;
}

// The frame-invariant tables a workgroup reads: staged in LDS (shq) when `stage`, else global.
struct MqTabs {
  const uint32_t* bf;       // flat Mel list: bin << 16 | filter
  const int32_t* cf;        // staged coefficients (stage) ...
  const int32_t* dc;        // ... and DCT rows
  bool stage;
};
template <typename T>
__device__ __forceinline__ MqTabs mq_stage_tables(int32_t* tab, const T* __restrict__ coefs, const uint32_t* __restrict__ bf,
                                                  int total, int nb_mel, int nb_dct, const T* __restrict__ dct, int stage) {
  if (stage) {
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      tab[i] = (int32_t)bf[i];
      tab[total + i] = (int32_t)coefs[i];
    }
    for (int i = threadIdx.x; i < nb_mel * nb_dct; i += blockDim.x) tab[2 * total + i] = (int32_t)dct[i];
  }
  __syncthreads();
  return MqTabs{stage ? reinterpret_cast<const uint32_t*>(tab) : bf, tab + total, tab + 2 * total, stage != 0};
}

// One frame on one wave, from the CFFT output get(i) (i < L = n/2) and the frame maximum m:
// |X_k| for k <= L (split + magnitude) into mag, the Mel sums (int64 LDS totals, acc), the
// per-filter finish (fin) into mel, the DCT rows into o.  mag / mel / acc are the wave's own.
// Bins 0 .. L - 1 take one lane each per step; bin L (from get(0) only) comes last.
template <typename T, typename Ops, typename Get>
__device__ __forceinline__ void mq_post_frame(const Ops& op, Get get, const int4* __restrict__ tw, int n,
                                              int32_t m, T* o,
                                              int nb_mel, int nb_dct, int total, const MqTabs& tb,
                                              const T* __restrict__ coefs, const T* __restrict__ dct, int32_t lutv,
                                              int32_t* mag, int32_t* mel, int64_t* acc) {
  const int lane = threadIdx.x & 63;
  const int lim = (n >> 1) + 1;
  auto coef = [&](int g) { return tb.stage ? tb.cf[g] : (int32_t)coefs[g]; };
  auto dctw = [&](int i) { return tb.stage ? tb.dc[i] : (int32_t)dct[i]; };
  for (int i = lane; i < nb_mel; i += 64) acc[i] = 0;
  const int L = lim - 1;
#pragma unroll 4
  for (int p0 = 0; p0 < L; p0 += 64) {                 // uniform: the shuffle needs all lanes
    const int p = p0 + lane, k = min(p, L - 1);
    const int32_t v = op.mag(op.split(get, k, L, tw[k]), lutv);
    if (p < L) mag[mq_mpad(k)] = v;
  }
  {
    const int32_t v = op.mag(op.split(get, L, L, tw[L]), lutv);   // bin L (every lane: the shuffle)
    if (lane == 0) mag[mq_mpad(L)] = v;
  }
  mq_wave_sync();
  {   // the Mel sums over the flat list (see mq_mel_sums)
    const int per = (total + 63) >> 6;
    const int g0 = lane * per, g1 = min(total, g0 + per);
    int cur = -1;
    int64_t r = 0;
    for (int g = g0; g < g1; ++g) {
      const uint32_t e = tb.bf[g];
      const int f = (int)(e & 0xFFFFu);
      if (f != cur) {
        if (cur >= 0) atomicAdd(reinterpret_cast<unsigned long long*>(acc + cur), (unsigned long long)r);
        cur = f;
        r = 0;
      }
      r += op.term(mag[mq_mpad((int)(e >> 16))], coef(g));
    }
    if (cur >= 0) atomicAdd(reinterpret_cast<unsigned long long*>(acc + cur), (unsigned long long)r);
  }
  mq_wave_sync();
  for (int i = lane; i < nb_mel; i += 64) mel[i] = op.fin(acc[i], m);
  mq_wave_sync();
  for (int r = lane; r < nb_dct; r += 64) o[r] = op.dct(r, mel, dctw);
  mq_wave_sync();                                      // mel / acc reused by the next frame
}

// The three-launch path's post kernel: frames' CFFT outputs in global memory (y), maxima in maxv.
template <typename T, typename Ops>
__device__ __forceinline__ void mq_post_body(const Ops& op, const T* __restrict__ y, const int4* __restrict__ tw,
                                             const T* maxv, int maxv_stride, int n, int nb_mel,
                                             const T* __restrict__ coefs, const uint32_t* __restrict__ bf, int total,
                                             int nb_dct, const T* __restrict__ dct, const int32_t* __restrict__ lut,
                                             T* dst, uint32_t batch, int stage) {
  extern __shared__ int32_t shq[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lim = (n >> 1) + 1;
  const MqTabs tb = mq_stage_tables<T>(shq, coefs, bf, total, nb_mel, nb_dct, dct, stage);
  int32_t* mag = shq + (stage ? mq_tab_words(total, nb_mel, nb_dct) : 0) + wave * mq_wave_words(n, nb_mel);
  int32_t* mel = mag + mq_mag_words(n);
  int64_t* acc = reinterpret_cast<int64_t*>(mag + ((mq_mag_words(n) + nb_mel + 1) & ~1));
  const int32_t lutv = lut[lane & 31];
  (void)lim;
  for (int it = 0; it < kMqFpw; ++it) {
    const uint32_t frame = (blockIdx.x * kMqFpw + it) * kMqWaves + wave;
    if (frame >= batch) break;                         // wave-uniform: no workgroup barrier below
    const int32_t m = (int32_t)maxv[(size_t)frame * maxv_stride];
    const T* X = y + (size_t)frame * n;                // CFFT output, L complex
    auto get = [X](int i) {
      if constexpr (sizeof(T) == 4) return reinterpret_cast<const int2*>(X)[i];
      else { const short2 v = reinterpret_cast<const short2*>(X)[i]; return make_int2(v.x, v.y); }
    };
    mq_post_frame<T>(op, get, tw, n, m, dst + (size_t)frame * nb_dct, nb_mel, nb_dct, total,
                     tb, coefs, dct, lutv, mag, mel, acc);
  }
}

// The q31 chain of arm_mfcc_q31.c:119-223 as per-element operations: pre (MqPre, shared with the
// radix-16 CFFT's MFCC prologue) = arm_absmax_q31 / arm_divide_q31 / arm_scale_q31 /
// arm_mult_q31; post = arm_split_rfft_q31 + arm_cmplx_mag_q31, arm_dot_prod_q31, the Mel
// finish, the DCT rows.
struct MqOpsQ31 : MqPre<int32_t> {
  int32_t le;      // log exponent (fftShift + 2 + SHIFT_MELFILTER_SATURATION_Q31) * LOG2TOLOG_Q31
  int nb_mel;
  __device__ MqOpsQ31(int n, int nm, int /*nd*/)
      : le((int32_t)((uint32_t)(31 - (int)mq_clz((uint32_t)n) + 12) * 0x02C5C860u)), nb_mel(nm) {}
  template <typename Get> __device__ int2 split(Get get, int k, int L, int4 t) const { return mq_split_q31(get, k, L, t); }
  __device__ int32_t mag(int2 c, int32_t lutv) const {   // arm_cmplx_mag_q31
    const int32_t a0 = (int32_t)(((int64_t)c.x * c.x) >> 33), a1 = (int32_t)(((int64_t)c.y * c.y) >> 33);
    return mq_sqrt(a0 + a1, lutv);
  }
  __device__ int64_t term(int32_t a, int32_t c) const { return ((int64_t)a * c) >> 14; }   // arm_dot_prod_q31
  __device__ int32_t fin(int64_t r, int32_t m) const {
    r += 0x08637BD0;                                 // MICRO_Q31
    r >>= 28;                                        // SHIFT_MELFILTER_SATURATION_Q31 + 18
    int32_t v = mq_ssat31((int32_t)r);               // __SSAT takes the low 32 bits
    if (m != 0 && m != 0x7FFFFFFF) v = mq_scale(v, m, 1);   // arm_scale_q31(., m, 0)
    v = mq_log((uint32_t)v);
    const int64_t s = (int64_t)v + le;               // arm_offset_q31 (saturating)
    v = s > INT32_MAX ? INT32_MAX : (s < INT32_MIN ? INT32_MIN : (int32_t)s);
    return v >> 3;                                   // arm_shift_q31(., -3)
  }
  template <typename W> __device__ int32_t dct(int r, const int32_t* mel, W dctw) const {   // arm_mat_vec_mult_q31
    int64_t sum = 0;
    for (int i = 0; i < nb_mel; ++i) sum += (int64_t)dctw(r * nb_mel + i) * mel[i];
    return (int32_t)(sum >> 31);
  }
};

__global__ __launch_bounds__(256) void mfcc_q31_post_kernel(const int32_t* __restrict__ y, const int4* __restrict__ tw,
                                                            const int32_t* maxv, int maxv_stride, int n, int nb_mel,
                                                            const int32_t* __restrict__ coefs,
                                                            const uint32_t* __restrict__ bf, int total, int nb_dct,
                                                            const int32_t* __restrict__ dct,
                                                            const int32_t* __restrict__ lut, int32_t* dst,
                                                            uint32_t batch, int stage) {
  mq_post_body<int32_t>(MqOpsQ31(n, nb_mel, nb_dct), y, tw, maxv, maxv_stride, n, nb_mel, coefs, bf, total, nb_dct, dct, lut,
                        dst, batch, stage);
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

struct MqOpsQ15 : MqPre<int16_t> {
  int32_t le;
  int nb_mel, nb_dct;
  __device__ MqOpsQ15(int n, int nm, int nd)
      : le((int32_t)((uint32_t)(31 - (int)mq_clz((uint32_t)n) + 12) * 0x02C5C860u)), nb_mel(nm), nb_dct(nd) {}
  template <typename Get> __device__ int2 split(Get get, int k, int L, int4 t) const { return mq_split_q15(get, k, L, t); }
  __device__ int32_t mag(int2 c, int32_t lutv) const {   // arm_cmplx_mag_q15
    const uint32_t s2 = ((uint32_t)(c.x * c.x) + (uint32_t)(c.y * c.y)) >> 1;
    return mq_sqrt((int32_t)s2, lutv) >> 16;
  }
  __device__ int64_t term(int32_t a, int32_t c) const { return (int64_t)(a * c); }   // arm_dot_prod_q15
  __device__ int32_t fin(int64_t r, int32_t m) const {
    r += 0x219;                                      // MICRO_Q15
    r >>= 10;                                        // SHIFT_MELFILTER_SATURATION_Q15
    int32_t v = mq_ssat31((int32_t)r);
    if (m != 0 && m != 0x7FFF) v = mq_scale(v, (int32_t)((uint32_t)m << 16), 1);
    const int64_t s = (int64_t)mq_log((uint32_t)v) + le;
    v = s > INT32_MAX ? INT32_MAX : (s < INT32_MIN ? INT32_MIN : (int32_t)s);
    return (int32_t)(int16_t)(v >> 19);              // (q15_t) truncation
  }
  template <typename W> __device__ int16_t dct(int r, const int32_t* mel, W dctw) const {   // arm_mat_vec_mult_q15
    const int paired = r < (nb_dct & ~3) ? (nb_mel & ~1) : (nb_mel & ~3);
    int64_t sum = 0;
    for (int i = 0; i < paired; i += 2)
      sum += (int32_t)((uint32_t)(dctw(r * nb_mel + i) * mel[i]) + (uint32_t)(dctw(r * nb_mel + i + 1) * mel[i + 1]));
    for (int i = paired; i < nb_mel; ++i) sum += (int64_t)(dctw(r * nb_mel + i) * mel[i]);
    return (int16_t)mq_ssat16((int32_t)(sum >> 15));
  }
};

__global__ __launch_bounds__(256) void mfcc_q15_post_kernel(const int16_t* __restrict__ y, const int4* __restrict__ tw,
                                                            const int16_t* maxv, int maxv_stride, int n, int nb_mel,
                                                            const int16_t* __restrict__ coefs,
                                                            const uint32_t* __restrict__ bf, int total, int nb_dct,
                                                            const int16_t* __restrict__ dct,
                                                            const int32_t* __restrict__ lut, int16_t* dst,
                                                            uint32_t batch, int stage) {
  mq_post_body<int16_t>(MqOpsQ15(n, nb_mel, nb_dct), y, tw, maxv, maxv_stride, n, nb_mel, coefs, bf, total, nb_dct,
                        dct, lut, dst, batch, stage);
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
                                const uint32_t* pos, const uint32_t* len, const uint32_t* off, const int16_t* coefs,
                                const uint32_t* bf, int total, int nb_dct, const int16_t* dct, const int32_t* lut, int16_t* dst, uint32_t batch,
                                hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  (void)pos; (void)len; (void)off;
  const uint32_t grid2 = (batch + kMqFpw * kMqWaves - 1) / (kMqFpw * kMqWaves);
  const size_t tab = sizeof(int32_t) * (size_t)mq_tab_words(total, nb_mel, nb_dct);
  const int stage = mfcc_q31_post_lds(n, nb_mel) + tab <= 65536 ? 1 : 0;
  (void)grid;
  hipLaunchKernelGGL(mfcc_q15_post_kernel, dim3(grid2), dim3(64 * kMqWaves),
                     mfcc_q31_post_lds(n, nb_mel) + (stage ? tab : 0), st, y, tw, maxv, maxv_stride, n, nb_mel, coefs,
                     bf, total, nb_dct, dct, lut, dst, batch, stage);
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
                                const uint32_t* pos, const uint32_t* len, const uint32_t* off, const int32_t* coefs,
                                const uint32_t* bf, int total, int nb_dct, const int32_t* dct, const int32_t* lut, int32_t* dst, uint32_t batch,
                                hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMqWaves - 1) / kMqWaves;
  (void)pos; (void)len; (void)off;
  const uint32_t grid2 = (batch + kMqFpw * kMqWaves - 1) / (kMqFpw * kMqWaves);
  const size_t tab = sizeof(int32_t) * (size_t)mq_tab_words(total, nb_mel, nb_dct);
  const int stage = mfcc_q31_post_lds(n, nb_mel) + tab <= 65536 ? 1 : 0;
  (void)grid;
  hipLaunchKernelGGL(mfcc_q31_post_kernel, dim3(grid2), dim3(64 * kMqWaves),
                     mfcc_q31_post_lds(n, nb_mel) + (stage ? tab : 0), st, y, tw, maxv, maxv_stride, n, nb_mel, coefs,
                     bf, total, nb_dct, dct, lut, dst, batch, stage);
  return hipGetLastError();
}

}  // namespace mi355x
