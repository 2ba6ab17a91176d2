/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 *
 * CPU restatement of the reference's host scalar FIR and matrix multiply:
 *   arm_fir_f32  Source/FilteringFunctions/arm_fir_f32.c:911-1280: y[n] = sum_k s[n+k]*c[k],
 *                the accumulator starts at +0.0f, mul then add (no FMA), k ascending; the
 *                8-way unrolled and the tail loops give the same order.
 *   arm_fir_q15  arm_fir_q15.c:458-726 with ARM_MATH_LOOPUNROLL: outputs in groups of four
 *                accumulate tap PAIRS as an int32-wrapped sum (__SMLALD, none.h:497-506),
 *                the blockSize%4 tail accumulates every product in int64 (:649-681);
 *                y = __SSAT((int32)(acc >> 15), 16).
 *   state        s = [history (numTaps-1) ; block]; afterwards the state holds
 *                [last numTaps-1 samples of s ; block] (:1242-1278).
 *   arm_mat_mult_f32  arm_mat_mult_f32.c:600-730: per element, k-ordered mul-then-add.
 *   oracle_mat_mult_f32_fmaf: NOT a reference function -- the MI355X product's own stated
 *                semantics for arm_mat_mult_f32 (v_mfma_f32_32x32x2_f32 accumulates as a
 *                k-ordered fmaf chain from +0.0f, one rounding per term), used to pin the GPU
 *                kernel bit for bit (tests/test_gpu_rfft_fir_mat.py); same k order as the
 *                reference, one rounding fewer per term.
 * Pinned by tests/test_oracle.py against oracle/_ref bit for bit.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

void oracle_arm_fir_f32(const arm_fir_instance_f32 *S, const float *pSrc, float *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps;
  float *s = S->pState;
  memcpy(s + taps - 1, pSrc, sizeof(float) * blockSize);      /* append the block */
  for (uint32_t n = 0; n < blockSize; ++n) {
    float acc = 0.0f;
    for (uint32_t k = 0; k < taps; ++k) {
      const float prod = s[n + k] * S->pCoeffs[k];
      acc = acc + prod;
    }
    pDst[n] = acc;
  }
  memmove(s, s + blockSize, sizeof(float) * (taps - 1));     /* carry the history */
}

static int16_t oracle_sat_q15(int32_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

void oracle_arm_fir_q15(const arm_fir_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps, pairs = taps >> 1;
  int16_t *s = S->pState;
  const int16_t *c = S->pCoeffs;
  memcpy(s + taps - 1, pSrc, sizeof(int16_t) * blockSize);
  const uint32_t grouped = blockSize & ~3u;
  for (uint32_t n = 0; n < blockSize; ++n) {
    int64_t acc = 0;
    for (uint32_t m = 0; m < pairs; ++m) {
      const int32_t p0 = (int32_t)s[n + 2 * m] * c[2 * m];
      const int32_t p1 = (int32_t)s[n + 2 * m + 1] * c[2 * m + 1];
      if (n < grouped) acc += (int32_t)((uint32_t)p0 + (uint32_t)p1);   /* int32 pair sum */
      else             acc += (int64_t)p0 + (int64_t)p1;
    }
    pDst[n] = oracle_sat_q15((int32_t)(acc >> 15));
  }
  memmove(s, s + blockSize, sizeof(int16_t) * (taps - 1));
}

/* arm_fir_fast_q15.c: q31_t accumulator fed by __SMLAD/__SMLADX and int32 adds (none.h) —
 * every partial sum wraps mod 2^32, pairs or not; y = __SSAT(acc >> 15, 16). */
void oracle_arm_fir_fast_q15(const arm_fir_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps, used = taps & ~1u;
  int16_t *s = S->pState;
  const int16_t *c = S->pCoeffs;
  memcpy(s + taps - 1, pSrc, sizeof(int16_t) * blockSize);
  for (uint32_t n = 0; n < blockSize; ++n) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < used; ++k) acc += (uint32_t)((int32_t)s[n + k] * c[k]);
    pDst[n] = oracle_sat_q15((int32_t)acc >> 15);
  }
  memmove(s, s + blockSize, sizeof(int16_t) * (taps - 1));
}

/* arm_fir_q7.c:446-560 (LOOPUNROLL and tail alike): q31_t accumulator of q7 x q7 products,
 * plain int32 adds (wrapping), y = __SSAT(acc >> 7, 8). */
void oracle_arm_fir_q7(const arm_fir_instance_q7 *S, const int8_t *pSrc, int8_t *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps;
  int8_t *s = S->pState;
  const int8_t *c = S->pCoeffs;
  memcpy(s + taps - 1, pSrc, blockSize);
  for (uint32_t n = 0; n < blockSize; ++n) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < taps; ++k) acc += (uint32_t)((int32_t)s[n + k] * c[k]);
    const int32_t v = (int32_t)acc >> 7;
    pDst[n] = (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v);
  }
  memmove(s, s + blockSize, taps - 1);
}

/* arm_fir_q31.c: q63 accumulator of exact products (wrapping, as gcc x86-64 adds do),
 * y = (q31)(acc >> 31). */
void oracle_arm_fir_q31(const arm_fir_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps;
  int32_t *s = S->pState;
  const int32_t *c = S->pCoeffs;
  memcpy(s + taps - 1, pSrc, sizeof(int32_t) * blockSize);
  for (uint32_t n = 0; n < blockSize; ++n) {
    uint64_t acc = 0;
    for (uint32_t k = 0; k < taps; ++k) acc += (uint64_t)((int64_t)s[n + k] * c[k]);
    pDst[n] = (int32_t)((int64_t)acc >> 31);
  }
  memmove(s, s + blockSize, sizeof(int32_t) * (taps - 1));
}

/* arm_fir_fast_q31.c: multAcc_32x32_keep32_R (none.h:185-186) per tap, taps in order:
 * acc = (q31)((((q63)acc << 32) + x*c + 0x80000000) >> 32); y = (q31)(acc << 1). */
void oracle_arm_fir_fast_q31(const arm_fir_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, uint32_t blockSize) {
  const uint32_t taps = S->numTaps;
  int32_t *s = S->pState;
  const int32_t *c = S->pCoeffs;
  memcpy(s + taps - 1, pSrc, sizeof(int32_t) * blockSize);
  for (uint32_t n = 0; n < blockSize; ++n) {
    int32_t acc = 0;
    for (uint32_t k = 0; k < taps; ++k) {
      const uint64_t wide = ((uint64_t)(int64_t)acc << 32) + (uint64_t)((int64_t)s[n + k] * c[k]) + 0x80000000ull;
      acc = (int32_t)(uint32_t)((int64_t)wide >> 32);
    }
    pDst[n] = (int32_t)((uint32_t)acc << 1);
  }
  memmove(s, s + blockSize, sizeof(int32_t) * (taps - 1));
}

arm_status oracle_arm_mat_mult_f32(const arm_matrix_instance_f32 *A, const arm_matrix_instance_f32 *B,
                                   arm_matrix_instance_f32 *Cm) {
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      float acc = 0.0f;
      for (uint32_t k = 0; k < K; ++k) {
        const float prod = A->pData[i * K + k] * B->pData[k * N + j];
        acc = acc + prod;
      }
      Cm->pData[i * N + j] = acc;
    }
  return ARM_MATH_SUCCESS;
}

/* C[i][j] = fmaf(A[i][K-1], B[K-1][j], ... fmaf(A[i][0], B[0][j], +0.0f)): k ascending, exact
 * products, one rounding per term (libm fmaf is correctly rounded; no contraction elsewhere). */
arm_status oracle_mat_mult_f32_fmaf(const arm_matrix_instance_f32 *A, const arm_matrix_instance_f32 *B,
                                    arm_matrix_instance_f32 *Cm) {
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  if (K != B->numRows || M != Cm->numRows || N != Cm->numCols) return ARM_MATH_SIZE_MISMATCH;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      float acc = 0.0f;
      for (uint32_t k = 0; k < K; ++k) acc = fmaf(A->pData[i * K + k], B->pData[k * N + j], acc);
      Cm->pData[i * N + j] = acc;
    }
  return ARM_MATH_SUCCESS;
}

/* arm_mat_mult_q15.c:741-912 (!ARM_MATH_DSP): q63 sum of exact q15 products in k order,
 * __SSAT((sum >> 15), 16) with the shifted sum narrowed to int32 first. */
arm_status oracle_arm_mat_mult_q15(const arm_matrix_instance_q15 *A, const arm_matrix_instance_q15 *B,
                                   arm_matrix_instance_q15 *Cm, int16_t *pState) {
  (void)pState;
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      int64_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) sum += (int32_t)A->pData[i * K + k] * B->pData[k * N + j];
      Cm->pData[i * N + j] = oracle_sat_q15((int32_t)(sum >> 15));
    }
  return ARM_MATH_SUCCESS;
}

/* arm_mat_mult_q7.c:689-790 (scalar branch): q31_t sum of exact q7 products -- it cannot wrap,
 * |sum| <= 65535 * 2^14 < 2^31 -- then (q7)__SSAT(sum >> 7, 8).  pState unused.  The reference
 * keeps the output row offset in a uint16_t (`i`, :704, :782), so for numRows * numColsB > 65536
 * it writes later rows over earlier ones; this restatement (and the product) writes every element
 * at its row-major place: equal to the reference wherever the reference's offset does not wrap. */
arm_status oracle_arm_mat_mult_q7(const arm_matrix_instance_q7 *A, const arm_matrix_instance_q7 *B,
                                  arm_matrix_instance_q7 *Cm, int8_t *pState) {
  (void)pState;
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      int32_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) sum += (int32_t)A->pData[i * K + k] * B->pData[k * N + j];
      const int32_t v = sum >> 7;
      Cm->pData[i * N + j] = (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v);
    }
  return ARM_MATH_SUCCESS;
}

/* arm_mat_mult_q31.c:53-163: q63 sum of exact q31 products (wrapping), (q31)(sum >> 31). */
arm_status oracle_arm_mat_mult_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                   arm_matrix_instance_q31 *Cm) {
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      uint64_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) sum += (uint64_t)((int64_t)A->pData[i * K + k] * B->pData[k * N + j]);
      Cm->pData[i * N + j] = (int32_t)((int64_t)sum >> 31);
    }
  return ARM_MATH_SUCCESS;
}

/* arm_mat_mult_opt_q31.c:648-780 (the scalar branch): the q31 product above, pState unused. */
arm_status oracle_arm_mat_mult_opt_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                       arm_matrix_instance_q31 *Cm, int32_t *pState) {
  (void)pState;
  return oracle_arm_mat_mult_q31(A, B, Cm);
}

/* arm_mat_mult_fast_q15.c:351-401 (!ARM_MATH_DSP): q31_t sum += a*b (wrapping), output
 * (q15)(sum >> 15) -- truncation, no saturation.  arm_mat_mult_fast_q31.c:152-166, :215-266:
 * sum = (q31)(((q63)sum << 32 + (q63)a*b) >> 32) per product (= sum + ((a*b) >> 32) mod 2^32),
 * output sum << 1. */
arm_status oracle_arm_mat_mult_fast_q15(const arm_matrix_instance_q15 *A, const arm_matrix_instance_q15 *B,
                                        arm_matrix_instance_q15 *Cm, int16_t *pState) {
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      uint32_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) sum += (uint32_t)((int32_t)A->pData[i * K + k] * B->pData[k * N + j]);
      Cm->pData[i * N + j] = (int16_t)((int32_t)sum >> 15);
    }
  return ARM_MATH_SUCCESS;
}
arm_status oracle_arm_mat_mult_fast_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                        arm_matrix_instance_q31 *Cm) {
  const uint32_t M = A->numRows, K = A->numCols, N = B->numCols;
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t j = 0; j < N; ++j) {
      uint32_t sum = 0;
      for (uint32_t k = 0; k < K; ++k) sum += (uint32_t)(int32_t)(((int64_t)A->pData[i * K + k] * B->pData[k * N + j]) >> 32);
      Cm->pData[i * N + j] = (int32_t)(sum << 1);
    }
  return ARM_MATH_SUCCESS;
}

/* arm_conv_f32.c / arm_conv_q15.c (!ARM_MATH_DSP) / arm_conv_q31.c: y[n] = sum over the
 * overlap of a[k]*b[n-k] with k (index of pSrcA) ASCENDING whichever input is longer
 * (the reference's internal swap of the two inputs does not change that order; checked
 * against oracle/_ref for both orders of the lengths), from 0.0f (f32: mul then add) or an
 * exact q63 sum (q15: __SSAT((q31)(sum >> 15), 16); q31: (q31)(sum >> 31), wrapping). */
#define ORACLE_CONV_SETUP(T)                                                    \
  const T *x = pSrcA, *h = pSrcB;                                              \
  const uint32_t A = srcALen, B = srcBLen, L = A + B - 1;
void oracle_arm_conv_f32(const float *pSrcA, uint32_t srcALen, const float *pSrcB, uint32_t srcBLen, float *pDst) {
  ORACLE_CONV_SETUP(float)
  for (uint32_t n = 0; n < L; ++n) {
    const uint32_t k0 = n + 1 > B ? n + 1 - B : 0, k1 = n < A - 1 ? n : A - 1;
    float sum = 0.0f;
    for (uint32_t k = k0; k <= k1; ++k) { const float p = x[k] * h[n - k]; sum = sum + p; }
    pDst[n] = sum;
  }
}
void oracle_arm_conv_q15(const int16_t *pSrcA, uint32_t srcALen, const int16_t *pSrcB, uint32_t srcBLen, int16_t *pDst) {
  ORACLE_CONV_SETUP(int16_t)
  for (uint32_t n = 0; n < L; ++n) {
    const uint32_t k0 = n + 1 > B ? n + 1 - B : 0, k1 = n < A - 1 ? n : A - 1;
    int64_t sum = 0;
    for (uint32_t k = k0; k <= k1; ++k) sum += (int32_t)x[k] * h[n - k];
    pDst[n] = oracle_sat_q15((int32_t)(sum >> 15));
  }
}
void oracle_arm_conv_q31(const int32_t *pSrcA, uint32_t srcALen, const int32_t *pSrcB, uint32_t srcBLen, int32_t *pDst) {
  ORACLE_CONV_SETUP(int32_t)
  for (uint32_t n = 0; n < L; ++n) {
    const uint32_t k0 = n + 1 > B ? n + 1 - B : 0, k1 = n < A - 1 ? n : A - 1;
    uint64_t sum = 0;
    for (uint32_t k = k0; k <= k1; ++k) sum += (uint64_t)((int64_t)x[k] * h[n - k]);
    pDst[n] = (int32_t)((int64_t)sum >> 31);
  }
}
