// Device arithmetic of the MFCC q31 / q15 back end (arm_mfcc_q31.c:139-223, arm_mfcc_q15.c:
// 147-226 and the functions they call: arm_split_rfft, arm_cmplx_mag + arm_sqrt_q31,
// arm_dot_prod, arm_scale, arm_vlog_q31, arm_offset, arm_shift, arm_mat_vec_mult), shared by the
// post kernel (mfcc_fixed.hip) and the fused front-CFFT-back kernel (cfft_fixed_r16.hip).
#pragma once
#include "common.hpp"
#include "cfft_fixed_core.hpp"
#include "mfcc_fixed_ops.hpp"

namespace mi355x {

typedef short s2x __attribute__((ext_vector_type(2)));

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


// Frames per group: the per-filter finish (31-step log per Mel value) and the DCT rows run
// one lane per (frame, filter) / (frame, row), so a group of G frames fills G * nb_mel lanes
// instead of nb_mel (20 of 64 with the suite's tables: the log ran on a third of the wave).
__host__ __device__ inline int mq_group(int nb_mel) { return nb_mel >= 32 ? 1 : (64 / nb_mel > 4 ? 4 : 64 / nb_mel); }
// LDS per wave (int32 words): |X_k| (fftLen/2 + 1, at mq_mpad(k)), the group's Mel values
// (G nb_mel), frame maxima (G), then the group's int64 Mel sums (G nb_mel).  mq_mpad(k) = k + k /
// 16: the Mel sums read the magnitudes at lane strides of a slice length (often a multiple of 16
// words), which the pad spreads over distinct banks.
constexpr int kMqBinU = MI355X_MQ_BIN_U;   // magnitude steps in flight per wave (tuning.hpp)
__host__ __device__ inline int mq_mpad(int k) { return k + (k >> 4); }
__host__ __device__ inline int mq_mag_words(int n) { return mq_mpad(n / 2) + 1; }
__host__ __device__ inline int mq_mel_off(int n, int nb_mel) { return mq_mag_words(n); }
__host__ __device__ inline int mq_m_off(int n, int nb_mel) { return mq_mag_words(n) + mq_group(nb_mel) * nb_mel; }
__host__ __device__ inline int mq_acc_off(int n, int nb_mel) { return (mq_m_off(n, nb_mel) + mq_group(nb_mel) + 1) & ~1; }
__host__ __device__ inline int mq_wave_words(int n, int nb_mel) { return mq_acc_off(n, nb_mel) + 2 * mq_group(nb_mel) * nb_mel; }

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
  // branch-free (the magnitude loop is unrolled over independent bins): bins 0 and L take get(0)
  // through the masked indices and select their own form at the end
  const int2 a = get(k & (L - 1)), b = get((L - k) & (L - 1));
  int32_t re = mult_R(a.x, t.x), im = mult_R(a.x, t.y);
  re = multSub_R(re, a.y, t.y); im = multAcc_R(im, a.y, t.x);
  re = multSub_R(re, b.y, t.y); im = multSub_R(im, b.y, t.z);
  re = multAcc_R(re, b.x, t.z); im = multSub_R(im, b.x, t.y);
  const bool edge = k == 0 || k == L;
  const int32_t ev = (k == 0 ? wadd(a.x, a.y) : wsub(a.x, a.y)) >> 1;
  return make_int2(edge ? ev : re, edge ? 0 : im);
}
template <typename Get>   // get(i): bin i as int2 of sign-extended q15 words
__device__ __forceinline__ int2 mq_split_q15(Get get, int k, int L, int4 t) {
  // t: the packed record of bin k (mfcc_fx_prepare): {(A0, ~A1), (B0, B1), (B1, ~B0), (A1, A0)} as
  // q15 pairs, A0 = A[2mk] ... B1 = B[2mk + 1].  A difference x*w is x*~w + x (~w = -w - 1 fits a
  // q15 word for every w), so each output is two v_dot2_i32_i16 (int32 wrap, as the reference's
  // uint32 sums) with the missing term as the accumulator:
  //   re = a.x A0 - a.y A1 + b.x B0 + b.y B1,   im = b.x B1 - b.y B0 + a.y A0 + a.x A1
  const int2 a = get(k & (L - 1)), b = get((L - k) & (L - 1));
  auto pk = [](int2 v) { return __builtin_bit_cast(s2x, __builtin_amdgcn_perm((uint32_t)v.y, (uint32_t)v.x, 0x05040100u)); };
  const s2x A = pk(a), B = pk(b);
  const int32_t re = __builtin_amdgcn_sdot2(B, __builtin_bit_cast(s2x, t.y),
                                            __builtin_amdgcn_sdot2(A, __builtin_bit_cast(s2x, t.x), a.y, false), false) >> 16;
  const int32_t im = __builtin_amdgcn_sdot2(A, __builtin_bit_cast(s2x, t.w),
                                            __builtin_amdgcn_sdot2(B, __builtin_bit_cast(s2x, t.z), b.y, false), false) >> 16;
  const bool edge = k == 0 || k == L;
  const int32_t ev = (k == 0 ? a.x + a.y : a.x - a.y) >> 1;
  return make_int2(edge ? ev : (int16_t)re, edge ? 0 : (int16_t)im);     // the split stores q15_t
}

// maxv may alias dst (frame maxima carried in dst[frame][0]): read before any output store.
// A workgroup stages the frame-invariant tables (flat Mel list, coefficients, DCT rows) in LDS
// once when they fit, then each wave runs kMqFpw frames; a wave's LDS region is its own, so the
// stages are ordered by wave barriers only (waves run independently; PMC of the one-frame,
// global-table version: 71 % of wave time waiting, VALU issue at 34 %).
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

// One frame on one wave, from the CFFT output get(i) (i < L = n/2): |X_k| (split + magnitude)
// into mag for the bins kmin .. kmin + kcnt - 1 that some Mel filter reads (the host's range of
// the filter positions: the reference computes all L + 1 magnitudes, but only these reach its
// output), then the Mel sums into the int64 LDS totals acc[0 .. nb_mel).  mag / acc are the
// wave's own.  The bins take one lane each, kMqBinU steps unrolled: the steps' loads and splits
// are independent, so their latencies overlap.
template <typename T, typename Ops, typename Get>
__device__ __forceinline__ void mq_mel_frame(const Ops& op, Get get, const int4* __restrict__ tw, int n, int kmin,
                                             int kcnt, int nb_mel, int total, const MqTabs& tb,
                                             const T* __restrict__ coefs, int32_t lutv, int32_t* mag, int64_t* acc) {
  const int lane = threadIdx.x & 63;
  auto coef = [&](int g) { return tb.stage ? tb.cf[g] : (int32_t)coefs[g]; };
  for (int i = lane; i < nb_mel; i += 64) acc[i] = 0;
  const int L = n >> 1;
  for (int p0 = 0; p0 < kcnt; p0 += 64 * kMqBinU) {    // uniform: the shuffle needs all lanes
    int2 sp[kMqBinU];
#pragma unroll
    for (int u = 0; u < kMqBinU; ++u) {                 // past the range: a repeat of the last bin
      const int k = kmin + min(p0 + 64 * u + lane, kcnt - 1);
      sp[u] = op.split(get, k, L, tw[k]);
    }
#pragma unroll
    for (int u = 0; u < kMqBinU; ++u) {
      if (p0 + 64 * u < kcnt) {                         // uniform
        const int p = p0 + 64 * u + lane;
        const int32_t v = op.mag(sp[u], lutv);
        if (p < kcnt) mag[mq_mpad(kmin + p)] = v;
      }
    }
  }
  mq_wave_sync();
  {   // the Mel sums over the flat list (lane t sums slice t, adds each filter's part to its total)
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
  mq_wave_sync();                                      // mag is rewritten by the next frame
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

struct MqOpsQ15 : MqPre<int16_t> {
  int32_t le;
  int nb_mel, nb_dct;
  __device__ MqOpsQ15(int n, int nm, int nd)
      : le((int32_t)((uint32_t)(31 - (int)mq_clz((uint32_t)n) + 12) * 0x02C5C860u)), nb_mel(nm), nb_dct(nd) {}
  template <typename Get> __device__ int2 split(Get get, int k, int L, int4 t) const { return mq_split_q15(get, k, L, t); }
  __device__ int32_t mag(int2 c, int32_t lutv) const {   // arm_cmplx_mag_q15
    // (uint32)(x^2 + y^2) >> 1 as one v_dot2 (the same sum mod 2^32; x, y are q15 values)
    const s2x p = __builtin_bit_cast(s2x, __builtin_amdgcn_perm((uint32_t)c.y, (uint32_t)c.x, 0x05040100u));
    const uint32_t s2 = (uint32_t)__builtin_amdgcn_sdot2(p, p, 0, false) >> 1;
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


// The per-filter finish and the DCT rows of a group of g frames whose Mel sums are in acc
// (g nb_mel int64, frame-major) and maxima in mv: one lane per (frame, filter), then one lane per
// (frame, row); row r of frame j is stored by out(j, r, value).
template <typename Ops, typename W, typename Out>
__device__ __forceinline__ void mq_finish_group(const Ops& op, int g, int nb_mel, int nb_dct, const int64_t* acc,
                                                const int32_t* mv, int32_t* mel, W dctw, Out out) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < g * nb_mel; i += 64) mel[i] = op.fin(acc[i], mv[i / nb_mel]);
  mq_wave_sync();
  for (int i = lane; i < g * nb_dct; i += 64) {
    const int j = i / nb_dct, r = i - j * nb_dct;
    out(j, r, op.dct(r, mel + j * nb_mel, dctw));
  }
  mq_wave_sync();                                    // mel / acc / mv reused by the next group
}

}  // namespace mi355x
