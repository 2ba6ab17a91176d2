/* ORACLE — test infrastructure only (never linked into the product).
 *
 * Plain-C restatement of the reference's correlation / partial-convolution / fast
 * fixed-point convolution paths (Source/FilteringFunctions), as the host build runs them:
 *   arm_correlate_f32.c:1013-1096, arm_correlate_q15.c:814-895, arm_correlate_q31.c:789-871
 *     (!ARM_MATH_DSP branches): the longer input x slides over the shorter y; output i sums
 *     x[j] * y[yLen-1 + j - i] over j ascending; written forward from pDst + (A - B), or,
 *     when srcALen < srcBLen (inputs swapped, `inv`), backward from pDst + A + B - 2.
 *   arm_conv_partial_{f32,q15,q31}.c (!ARM_MATH_DSP, :635-679 / :715-759 / :579-628):
 *     outputs firstIndex .. firstIndex + numPoints - 1 of the full convolution at pDst[i].
 *   arm_conv_fast_q15.c / arm_correlate_fast_q15.c: q31_t accumulators fed by __SMLAD /
 *     __SMLADX (none.h:455-480), modular; single-sample __SMLAD(*px, *py, sum) also adds
 *     (x >> 16) * (y >> 16) of the sign-extended samples = 1 when both are negative.  Which
 *     MACs run one sample at a time is the reference's loop structure:
 *       stage 1 (count = 1 .. B-1 MACs): the last count % 4 (conv :150-239, corr :179-228);
 *       stage 2: none (pairs, or plain q31 sums in the remainder loops);
 *       stage 3: corr: the last count % 4 (:558-607); conv: the last count % 4 for the
 *       first (B-1)/4 outputs (:569-622), then every MAC (:629-656).
 *   arm_conv_q7.c, arm_conv_partial_q7.c (!ARM_MATH_DSP :688-735), arm_correlate_q7.c: q31_t
 *     sum of q7 x q7 products (int32 adds / __SMLAD pairs, wrapping), __SSAT(sum >> 7, 8).
 *   arm_conv_fast_q31.c / arm_correlate_fast_q31.c: sum = (q31)(((q63)sum << 32 + x*y) >> 32)
 *     per MAC (= sum + ((x*y) >> 32) mod 2^32), output sum << 1.
 *   the scratch-buffer forms (arm_conv_opt_q15.c, arm_conv_opt_q7.c, arm_correlate_opt_q15.c,
 *   arm_correlate_opt_q7.c, arm_conv_partial_opt_q15.c / _q7.c): the exact sums above;
 *   arm_conv_fast_opt_q15.c, arm_correlate_fast_opt_q15.c, arm_conv_partial_fast_opt_q15.c:
 *   __SMLAD pairs over zero-padded scratch copies -- a modular q31 sum with no single-sample
 *   term -- and __SSAT(sum >> 15, 16).
 * Pinned against oracle/_ref by tests/test_oracle.py::test_conv_family_oracle_equals_reference
 * and tests/test_conv_opt.py. */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

enum { OP_F32, OP_Q15, OP_Q31, OP_FQ15, OP_FQ31, OP_Q7, OP_FOQ15 };

static int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

/* v[n] = sum_{k asc} x[k] * g(n - k), g(m) = corr ? y[B-1-m] : y[m]; stores word n at out[n]. */
static void engine(int op, int corr, const void *xv, uint32_t A, const void *yv, uint32_t B, uint32_t n0, uint32_t n1,
                   void *out, int64_t yoff, int ydir) {
  for (uint32_t n = n0; n < n1; ++n) {
    const uint32_t k0 = n + 1 > B ? n + 1 - B : 0, k1 = n < A - 1 ? n : A - 1;
    const int64_t pos = yoff + (int64_t)ydir * n;
#define G(T) (corr ? ((const T *)yv)[B - 1 - (n - k)] : ((const T *)yv)[n - k])
    if (op == OP_F32) {
      const float *x = xv;
      float s = 0.0f;
      for (uint32_t k = k0; k <= k1; ++k) { const float p = x[k] * G(float); s = s + p; }
      ((float *)out)[pos] = s;
    } else if (op == OP_Q15) {
      const int16_t *x = xv;
      int64_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (int32_t)x[k] * G(int16_t);
      ((int16_t *)out)[pos] = sat16((int32_t)(s >> 15));
    } else if (op == OP_Q31) {
      const int32_t *x = xv;
      uint64_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (uint64_t)((int64_t)x[k] * G(int32_t));
      ((int32_t *)out)[pos] = (int32_t)((int64_t)s >> 31);
    } else if (op == OP_Q7) {
      const int8_t *x = xv;
      uint32_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (uint32_t)((int32_t)x[k] * G(int8_t));
      const int32_t v = (int32_t)s >> 7;
      ((int8_t *)out)[pos] = (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v);
    } else if (op == OP_FOQ15) {
      const int16_t *x = xv;
      uint32_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (uint32_t)((int32_t)x[k] * G(int16_t));
      ((int16_t *)out)[pos] = sat16((int32_t)s >> 15);
    } else if (op == OP_FQ31) {
      const int32_t *x = xv;
      uint32_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (uint32_t)(int32_t)(((int64_t)x[k] * G(int32_t)) >> 32);
      ((int32_t *)out)[pos] = (int32_t)(s << 1);
    } else {
      const int16_t *x = xv;
      uint32_t s = 0;
      for (uint32_t k = k0; k <= k1; ++k) s += (uint32_t)((int32_t)x[k] * G(int16_t));
      int64_t s0 = 1, s1 = 0;                         /* single-sample __SMLAD range of k */
      if ((int64_t)n <= (int64_t)B - 2) {
        s0 = (int64_t)n + 1 - ((int64_t)n + 1) % 4; s1 = n;
      } else if (n >= A) {
        const int64_t cnt = (int64_t)A + B - 1 - n;
        s1 = A - 1;
        s0 = (!corr && (int64_t)(n - A) >= ((int64_t)B - 1) / 4) ? (int64_t)n - B + 1 : (int64_t)A - cnt % 4;
      }
      for (int64_t k = s0; k <= s1; ++k) s += (x[k] < 0 && G(int16_t) < 0) ? 1u : 0u;
      ((int16_t *)out)[pos] = (int16_t)((int32_t)s >> 15);
    }
#undef G
  }
}

static void correlate(int op, const void *a, uint32_t A, const void *b, uint32_t B, void *dst) {
  if (A == 0 || B == 0) return;
  const uint32_t L = A + B - 1;
  if (A >= B) engine(op, 1, a, A, b, B, 0, L, dst, A - B, 1);
  else engine(op, 1, b, B, a, A, 0, L, dst, L - 1, -1);
}

static void conv_fast(int op, const void *a, uint32_t A, const void *b, uint32_t B, void *dst) {
  if (A == 0 || B == 0) return;
  if (A >= B) engine(op, 0, a, A, b, B, 0, A + B - 1, dst, 0, 1);
  else engine(op, 0, b, B, a, A, 0, A + B - 1, dst, 0, 1);
}

static arm_status partial(int op, const void *a, uint32_t A, const void *b, uint32_t B, void *dst, uint32_t first,
                          uint32_t num) {
  if ((uint64_t)first + num > (uint64_t)A + B - 1) return ARM_MATH_ARGUMENT_ERROR;
  engine(op, 0, a, A, b, B, first, first + num, dst, 0, 1);
  return ARM_MATH_SUCCESS;
}

void oracle_arm_correlate_f32(const float *a, uint32_t A, const float *b, uint32_t B, float *d) { correlate(OP_F32, a, A, b, B, d); }
void oracle_arm_correlate_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d) { correlate(OP_Q15, a, A, b, B, d); }
void oracle_arm_correlate_q31(const int32_t *a, uint32_t A, const int32_t *b, uint32_t B, int32_t *d) { correlate(OP_Q31, a, A, b, B, d); }
void oracle_arm_correlate_fast_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d) { correlate(OP_FQ15, a, A, b, B, d); }
void oracle_arm_correlate_fast_q31(const int32_t *a, uint32_t A, const int32_t *b, uint32_t B, int32_t *d) { correlate(OP_FQ31, a, A, b, B, d); }
void oracle_arm_conv_fast_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d) { conv_fast(OP_FQ15, a, A, b, B, d); }
void oracle_arm_conv_fast_q31(const int32_t *a, uint32_t A, const int32_t *b, uint32_t B, int32_t *d) { conv_fast(OP_FQ31, a, A, b, B, d); }
arm_status oracle_arm_conv_partial_f32(const float *a, uint32_t A, const float *b, uint32_t B, float *d, uint32_t f,
                                       uint32_t n) { return partial(OP_F32, a, A, b, B, d, f, n); }
arm_status oracle_arm_conv_partial_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                       uint32_t f, uint32_t n) { return partial(OP_Q15, a, A, b, B, d, f, n); }
arm_status oracle_arm_conv_partial_q31(const int32_t *a, uint32_t A, const int32_t *b, uint32_t B, int32_t *d,
                                       uint32_t f, uint32_t n) { return partial(OP_Q31, a, A, b, B, d, f, n); }
void oracle_arm_conv_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d) { conv_fast(OP_Q7, a, A, b, B, d); }
void oracle_arm_correlate_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d) { correlate(OP_Q7, a, A, b, B, d); }
arm_status oracle_arm_conv_partial_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d,
                                      uint32_t f, uint32_t n) { return partial(OP_Q7, a, A, b, B, d, f, n); }

/* scratch-buffer forms (the reference's signatures; the scratch buffers are not needed) */
void oracle_arm_conv_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d, int16_t *s1,
                             int16_t *s2) { conv_fast(OP_Q15, a, A, b, B, d); }
void oracle_arm_conv_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d, int16_t *s1,
                                  int16_t *s2) { conv_fast(OP_FOQ15, a, A, b, B, d); }
void oracle_arm_conv_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d, int16_t *s1,
                            int16_t *s2) { conv_fast(OP_Q7, a, A, b, B, d); }
void oracle_arm_correlate_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                  int16_t *s) { correlate(OP_Q15, a, A, b, B, d); }
void oracle_arm_correlate_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                       int16_t *s) { correlate(OP_FOQ15, a, A, b, B, d); }
void oracle_arm_correlate_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d, int16_t *s1,
                                 int16_t *s2) { correlate(OP_Q7, a, A, b, B, d); }
arm_status oracle_arm_conv_partial_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                           uint32_t f, uint32_t n, int16_t *s1, int16_t *s2) {
  return partial(OP_Q15, a, A, b, B, d, f, n);
}
arm_status oracle_arm_conv_partial_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B,
                                                int16_t *d, uint32_t f, uint32_t n, int16_t *s1, int16_t *s2) {
  return partial(OP_FOQ15, a, A, b, B, d, f, n);
}
arm_status oracle_arm_conv_partial_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d,
                                          uint32_t f, uint32_t n, int16_t *s1, int16_t *s2) {
  return partial(OP_Q7, a, A, b, B, d, f, n);
}
