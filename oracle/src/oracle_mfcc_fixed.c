/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * CPU restatement of the reference's host scalar MFCC q31 (RFFT-based default build,
 * ARM_MATH_LOOPUNROLL, no ARM_MATH_DSP):
 *   arm_mfcc_init_q31  Source/TransformFunctions/arm_mfcc_init_q31.c (fields + rfft init 0,1)
 *   arm_mfcc_q31       Source/TransformFunctions/arm_mfcc_q31.c:88-225, stage by stage:
 *     m      = max sat|x|                              arm_absmax_q31.c (value only)
 *     if m != 0 and m != 0x7FFFFFFF:
 *       (quot, sh) = divide(0x7FFFFFFF, m)             arm_divide_q31.c:55-101
 *       x = scale(x, quot, sh)                         arm_scale_q31.c (kShift = sh + 1)
 *     x      = ssat31((x*w) >> 32) << 1                arm_mult_q31.c
 *     tmp    = rfft_q31(x)                             arm_rfft_q31.c (x is overwritten)
 *     mag_k  = sqrt_q31((re² >> 33) + (im² >> 33))    arm_cmplx_mag_q31.c, arm_sqrt_q31.c,
 *              k = 0 .. fftLen/2                       (Newton with sqrt_initial_lut_q31)
 *     mel_i  = ssat31((int32)((Σ (mag·c) >> 14) + MICRO_Q31) >> 28))   arm_dot_prod_q31.c
 *     mel    = scale(mel, m, 0)  if m != 0, 0x7FFFFFFF arm_scale_q31.c
 *     mel    = log_q31(mel)                            arm_vlog_q31.c (Clay Turner, 31 steps)
 *     mel    = qadd(mel, (fftShift + 12)·LOG2TOLOG_Q31) >> 3   arm_offset_q31.c, arm_shift_q31.c
 *     out_r  = (int32)((Σ dct[r][i]·mel_i) >> 31)      arm_mat_vec_mult_q31.c
 * All sums are exact int64 (order-free).  Shift counts of 32 (x86 and the GPU both use the
 * low five bits of a 32-bit shift count) only arise for m = 1 in the divide/scale pair.
 * Pinned by tests/test_mfcc_q31.py against oracle/_ref and the reference's MFCC Q31 patterns.
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

extern const int32_t sqrt_initial_lut_q31[32];

#define O_LOG2TOLOG_Q31 0x02C5C860
#define O_MICRO_Q31 0x08637BD0
#define O_SHIFT_MELFILTER_SATURATION_Q31 10

static uint32_t o_clz(uint32_t x) { return x ? (uint32_t)__builtin_clz(x) : 32u; }
static int32_t o_sat_abs(int32_t x) { return x > 0 ? x : (x == INT32_MIN ? INT32_MAX : -x); }
static int32_t o_ssat(int32_t v, int bits) {
  const int32_t mx = (int32_t)((1u << (bits - 1)) - 1u), mn = -1 - mx;
  return v > mx ? mx : (v < mn ? mn : v);
}
static int32_t o_shl(int32_t x, int k) { return (int32_t)((uint32_t)x << (k & 31)); }

/* arm_divide_q31.c:55-101 (denominator != 0) */
static void o_divide(int32_t num, int32_t den, int32_t *quot, int16_t *shift) {
  const int sign = (num < 0) ^ (den < 0);
  *shift = 0;
  num = o_sat_abs(num);
  den = o_sat_abs(den);
  int64_t t = ((int64_t)num << 31) / (int64_t)den;
  const int16_t sn = (int16_t)(32 - o_clz((uint32_t)(t >> 31)));
  if (sn > 0) {
    *shift = sn;
    t >>= sn;
  }
  if (sign) t = -t;
  *quot = (int32_t)t;
}

/* arm_scale_q31.c (generic): kShift = shift + 1 as int8_t */
static void o_scale(int32_t *p, uint32_t n, int32_t frac, int8_t shift) {
  const int8_t k = (int8_t)(shift + 1);
  for (uint32_t i = 0; i < n; ++i) {
    const int32_t in = (int32_t)(((int64_t)p[i] * frac) >> 32);
    if (!(k & 0x80)) {
      int32_t out = o_shl(in, k);
      if (in != (out >> (k & 31))) out = 0x7FFFFFFF ^ (in >> 31);
      p[i] = out;
    } else {
      p[i] = in >> ((-k) & 31);
    }
  }
}

/* arm_sqrt_q31.c:55-125 */
static int32_t o_sqrt(int32_t in) {
  if (in <= 0) return 0;
  const int32_t sb = (int32_t)o_clz((uint32_t)in) - 1;
  const int32_t number = in << ((sb % 2) == 0 ? sb : sb - 1);
  int32_t v = sqrt_initial_lut_q31[(number >> 26) - (0x20000000 >> 26)];
  for (int it = 0; it < 3; ++it) {
    int32_t t = (int32_t)(((int64_t)v * v) >> 28);
    t = (int32_t)(((int64_t)number * t) >> 31);
    t = 0x30000000 - t;
    v = (int32_t)(((int64_t)v * t) >> 29);
  }
  v = (int32_t)(((int64_t)number * v) >> 28);
  return (sb % 2) == 0 ? v >> (sb / 2) : v >> ((sb - 1) / 2);
}

/* arm_vlog_q31.c:55-121 (arm_scalar_log_q31) */
static int32_t o_log(uint32_t src) {
  const int32_t c = (int32_t)o_clz(src);
  uint32_t inc = (1u << 31) >> 6, x = c - 1 < 0 ? src >> (1 - c) : src << (c - 1), y = 0;
  for (int i = 0; i < 31; ++i) {
    x = (uint32_t)(((int64_t)x * x) >> 30);
    if (x >= (1u << 31)) {
      y += inc;
      x >>= 1;
    }
    inc >>= 1;
  }
  const int32_t tmp = (int32_t)(y - ((uint32_t)c << 26));   /* int32 wrap, as the reference's */
  return (int32_t)(((int64_t)tmp * (int64_t)0x58b90bfb) >> 31);
}

arm_status oracle_arm_mfcc_init_q31(arm_mfcc_instance_q31 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const int32_t *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const int32_t *filterCoefs,
                                    const int32_t *windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
  return oracle_arm_rfft_init_q31(&S->rfft, fftLen, 0, 1);
}

arm_status oracle_arm_mfcc_q31(const arm_mfcc_instance_q31 *S, int32_t *pSrc, int32_t *pDst, int32_t *pTmp) {
  const uint32_t n = S->fftLen;
  int32_t m = o_sat_abs(pSrc[0]);
  for (uint32_t i = 1; i < n; ++i) {
    const int32_t a = o_sat_abs(pSrc[i]);
    if (a > m) m = a;
  }
  if (m != 0 && m != 0x7FFFFFFF) {
    int32_t q;
    int16_t sh;
    o_divide(0x7FFFFFFF, m, &q, &sh);
    o_scale(pSrc, n, q, (int8_t)sh);
  }
  for (uint32_t i = 0; i < n; ++i) {
    const int32_t o = o_ssat((int32_t)(((int64_t)pSrc[i] * S->windowCoefs[i]) >> 32), 31);
    pSrc[i] = o_shl(o, 1);
  }
  const uint32_t fftShift = 31 - o_clz(n);
  oracle_arm_rfft_q31(&S->rfft, pSrc, pTmp);
  const uint32_t lim = 1 + (n >> 1);
  for (uint32_t k = 0; k < lim; ++k) {
    const int32_t re = pTmp[2 * k], im = pTmp[2 * k + 1];
    const int32_t a0 = (int32_t)(((int64_t)re * re) >> 33), a1 = (int32_t)(((int64_t)im * im) >> 33);
    pSrc[k] = o_sqrt(a0 + a1);
  }
  uint32_t cp = 0;
  for (uint32_t i = 0; i < S->nbMelFilters; ++i) {
    int64_t r = 0;
    for (uint32_t j = 0; j < S->filterLengths[i]; ++j)
      r += ((int64_t)pSrc[S->filterPos[i] + j] * S->filterCoefs[cp + j]) >> 14;
    cp += S->filterLengths[i];
    r += O_MICRO_Q31;
    r >>= (O_SHIFT_MELFILTER_SATURATION_Q31 + 18);
    pTmp[i] = o_ssat((int32_t)r, 31);
  }
  if (m != 0 && m != 0x7FFFFFFF) o_scale(pTmp, S->nbMelFilters, m, 0);
  for (uint32_t i = 0; i < S->nbMelFilters; ++i) pTmp[i] = o_log((uint32_t)pTmp[i]);
  const int32_t le = (int32_t)((fftShift + 2 + O_SHIFT_MELFILTER_SATURATION_Q31) * O_LOG2TOLOG_Q31);
  for (uint32_t i = 0; i < S->nbMelFilters; ++i) {
    const int64_t s = (int64_t)pTmp[i] + le;
    const int32_t v = s > INT32_MAX ? INT32_MAX : (s < INT32_MIN ? INT32_MIN : (int32_t)s);
    pTmp[i] = v >> 3;
  }
  for (uint32_t r = 0; r < S->nbDctOutputs; ++r) {
    int64_t s = 0;
    for (uint32_t i = 0; i < S->nbMelFilters; ++i) s += (int64_t)S->dctCoefs[r * S->nbMelFilters + i] * pTmp[i];
    pDst[r] = (int32_t)(s >> 31);
  }
  return ARM_MATH_SUCCESS;
}

/*
 * arm_mfcc_q15 (Source/TransformFunctions/arm_mfcc_q15.c:96-228), q15 frames, q31 work:
 *   m      = max sat|x| (q15)                           arm_absmax_q15.c
 *   if m != 0 and m != 0x7FFF:
 *     (quot, sh) = divide_q15(0x7FFF, m)               arm_divide_q15.c (temp = (n << 15) / d,
 *                                                       normalised by 17 - clz(temp))
 *     x = ssat16((x·quot) >> (15 - sh))                arm_scale_q15.c
 *   x      = ssat16((x·w) >> 15)                        arm_mult_q15.c
 *   tmp    = rfft_q15(x)
 *   mag_k  = sqrt_q31(((u32)re² + (u32)im²) >> 1) >> 16, k = 0 .. fftLen/2   arm_cmplx_mag_q15.c
 *   mel_i  = ssat31((int32)((Σ mag·c + MICRO_Q15) >> 10))                    arm_dot_prod_q15.c
 *   mel    = scale_q31(mel, m << 16, 0) if m != 0, 0x7FFF
 *   mel    = (q15)(qadd(log_q31(mel), (fftShift + 12)·LOG2TOLOG) >> 19)     (a truncation)
 *   out_r  = ssat16((int32)(Σ dct[r][i]·mel_i >> 15))   arm_mat_vec_mult_q15.c, whose __SMLALD
 *            column pairs wrap in int32 (none.h:497-506): rows in groups of four pair columns
 *            (0,1),(2,3).. up to numCols & ~1; the other rows pair within whole column quads;
 *            the remaining columns add exactly.
 */
#define O_MICRO_Q15 0x00000219

static int16_t o_sat_abs15(int16_t x) { return x > 0 ? x : (x == INT16_MIN ? INT16_MAX : (int16_t)-x); }
static int16_t o_ssat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }

arm_status oracle_arm_mfcc_init_q15(arm_mfcc_instance_q15 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const int16_t *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const int16_t *filterCoefs,
                                    const int16_t *windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
  return oracle_arm_rfft_init_q15(&S->rfft, fftLen, 0, 1);
}

arm_status oracle_arm_mfcc_q15(const arm_mfcc_instance_q15 *S, int16_t *pSrc, int16_t *pDst, int32_t *pTmp) {
  const uint32_t n = S->fftLen, nm = S->nbMelFilters;
  int16_t *pTmp2 = (int16_t *)pTmp;
  int16_t m = o_sat_abs15(pSrc[0]);
  for (uint32_t i = 1; i < n; ++i) {
    const int16_t a = o_sat_abs15(pSrc[i]);
    if (a > m) m = a;
  }
  const int scale = m != 0 && m != 0x7FFF;
  if (scale) {
    int32_t t = ((int32_t)0x7FFF << 15) / (int32_t)m;
    int sh = 0;
    const int sn = 17 - (int)o_clz((uint32_t)t);
    if (sn > 0) {
      sh = sn;
      t >>= sn;
    }
    const int16_t quot = (int16_t)t;
    const int k = (int)(int8_t)(15 - sh);
    for (uint32_t i = 0; i < n; ++i) pSrc[i] = o_ssat16(((int32_t)pSrc[i] * quot) >> k);
  }
  for (uint32_t i = 0; i < n; ++i) pSrc[i] = o_ssat16(((int32_t)pSrc[i] * S->windowCoefs[i]) >> 15);
  const uint32_t fftShift = 31 - o_clz(n);
  oracle_arm_rfft_q15(&S->rfft, pSrc, pTmp2);
  for (uint32_t k = 0; k < 1 + (n >> 1); ++k) {
    const int32_t re = pTmp2[2 * k], im = pTmp2[2 * k + 1];
    const uint32_t s2 = ((uint32_t)(re * re) + (uint32_t)(im * im)) >> 1;
    pSrc[k] = (int16_t)(o_sqrt((int32_t)s2) >> 16);
  }
  uint32_t cp = 0;
  for (uint32_t i = 0; i < nm; ++i) {
    int64_t r = 0;
    for (uint32_t j = 0; j < S->filterLengths[i]; ++j)
      r += (int64_t)((int32_t)pSrc[S->filterPos[i] + j] * S->filterCoefs[cp + j]);
    cp += S->filterLengths[i];
    r += O_MICRO_Q15;
    r >>= O_SHIFT_MELFILTER_SATURATION_Q31;
    pTmp[i] = o_ssat((int32_t)r, 31);
  }
  if (scale) o_scale(pTmp, nm, (int32_t)((uint32_t)(int32_t)m << 16), 0);
  const int32_t le = (int32_t)((fftShift + 2 + O_SHIFT_MELFILTER_SATURATION_Q31) * O_LOG2TOLOG_Q31);
  for (uint32_t i = 0; i < nm; ++i) {
    const int64_t s = (int64_t)o_log((uint32_t)pTmp[i]) + le;
    const int32_t v = s > INT32_MAX ? INT32_MAX : (s < INT32_MIN ? INT32_MIN : (int32_t)s);
    pSrc[i] = (int16_t)(v >> 19);
  }
  const uint32_t nd = S->nbDctOutputs, grouped = nd & ~3u;
  for (uint32_t r = 0; r < nd; ++r) {
    const int16_t *a = S->dctCoefs + (size_t)r * nm;
    const uint32_t paired = r < grouped ? (nm & ~1u) : (nm & ~3u);
    int64_t s = 0;
    for (uint32_t i = 0; i < paired; i += 2)
      s += (int32_t)((uint32_t)((int32_t)a[i] * pSrc[i]) + (uint32_t)((int32_t)a[i + 1] * pSrc[i + 1]));
    for (uint32_t i = paired; i < nm; ++i) s += (int64_t)a[i] * pSrc[i];
    pDst[r] = o_ssat16((int32_t)(s >> 15));
  }
  return ARM_MATH_SUCCESS;
}
