/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * CPU restatement of the reference's host scalar MFCC (RFFT-based default build):
 *   arm_mfcc_init_f32   Source/TransformFunctions/arm_mfcc_init_f32.c (fields + rfft init)
 *   arm_mfcc_f32        Source/TransformFunctions/arm_mfcc_f32.c:83-160, stage by stage:
 *     max   = max |x|                     arm_absmax_f32.c (LOOPUNROLL: strict '>' scan)
 *     x    *= (1.0f / max)  if max != 0   arm_scale_f32.c (one rounded product per sample)
 *     x    *= window                      arm_mult_f32.c
 *     tmp   = rfft_fast(x), tmp[1] = 0    arm_rfft_fast_f32.c:675-699, arm_mfcc_f32.c:124-125
 *     mag_k = sqrtf(re*re + im*im)        arm_cmplx_mag_f32.c (LOOPUNROLL tail form),
 *                                         arm_sqrt_f32 (fast_math_functions.h: sqrtf for in >= 0)
 *     mag  *= max           if max != 0   arm_scale_f32.c
 *     mel_i = sum_j mag[pos_i + j]*c_ij   arm_dot_prod_f32.c (sequential from 0.0f)
 *     mel   = logf(mel + 1.0e-6f)         arm_offset_f32.c, arm_vlog_f32.c (scalar logf)
 *     out_r = sum_i dct[r][i]*mel_i       arm_mat_vec_mult_f32.c (sequential per row)
 * Every sum is k-ordered mul-then-add (no FMA; built with -ffp-contract=off).  The
 * reference computes magnitudes for all fftLen bins from a 2*fftLen tmp buffer whose upper
 * half is never written; Mel filters stay below fftLen/2, so only those bins are formed
 * here (bins >= fftLen/2 read as 0).
 * Pinned by tests/test_oracle.py against oracle/_ref and the reference's MFCC F32 patterns.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

arm_status oracle_arm_rfft_fast_init_f32(arm_rfft_fast_instance_f32 *S, uint16_t n);

arm_status oracle_arm_mfcc_init_f32(arm_mfcc_instance_f32 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const float *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const float *filterCoefs,
                                    const float *windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
  return oracle_arm_rfft_fast_init_f32(&S->rfft, (uint16_t)fftLen);
}

void oracle_arm_mfcc_f32(const arm_mfcc_instance_f32 *S, float *pSrc, float *pDst, float *pTmp) {
  const uint32_t n = S->fftLen;
  float mx = pSrc[0] > 0.0f ? pSrc[0] : -pSrc[0];
  for (uint32_t i = 1; i < n; ++i) {
    const float a = pSrc[i] > 0.0f ? pSrc[i] : -pSrc[i];
    if (a > mx) mx = a;
  }
  if (mx != 0.0f) {
    const float inv = 1.0f / mx;
    for (uint32_t i = 0; i < n; ++i) pSrc[i] = pSrc[i] * inv;
  }
  for (uint32_t i = 0; i < n; ++i) pSrc[i] = pSrc[i] * S->windowCoefs[i];
  oracle_arm_rfft_fast_f32(&S->rfft, pSrc, pTmp, 0);
  pTmp[1] = 0.0f;
  for (uint32_t k = 0; k < n; ++k) {
    float m = 0.0f;
    if (k < n / 2) {
      const float re = pTmp[2 * k], im = pTmp[2 * k + 1];
      const float rr = re * re, ii = im * im;
      const float s = rr + ii;
      m = s >= 0.0f ? sqrtf(s) : 0.0f;
    }
    pSrc[k] = m;
  }
  if (mx != 0.0f)
    for (uint32_t k = 0; k < n; ++k) pSrc[k] = pSrc[k] * mx;
  const float *c = S->filterCoefs;
  for (uint32_t i = 0; i < S->nbMelFilters; ++i) {
    float sum = 0.0f;
    for (uint32_t j = 0; j < S->filterLengths[i]; ++j) {
      const float prod = pSrc[S->filterPos[i] + j] * c[j];
      sum = sum + prod;
    }
    c += S->filterLengths[i];
    pTmp[i] = sum;
  }
  for (uint32_t i = 0; i < S->nbMelFilters; ++i) pTmp[i] = logf(pTmp[i] + 1.0e-6f);
  for (uint32_t r = 0; r < S->nbDctOutputs; ++r) {
    float sum = 0.0f;
    for (uint32_t i = 0; i < S->nbMelFilters; ++i) {
      const float prod = S->dctCoefs[r * S->nbMelFilters + i] * pTmp[i];
      sum = sum + prod;
    }
    pDst[r] = sum;
  }
}
