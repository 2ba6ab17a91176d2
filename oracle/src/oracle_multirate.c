/* ORACLE — test infrastructure only (never linked into the product).
 *
 * Plain-C restatement of the reference's multirate FIR paths (Source/FilteringFunctions,
 * generic C branches, as the host build runs them):
 *   arm_fir_decimate_{f32,q15,fast_q15,q31,fast_q31}.c: the block is appended to the state
 *     s = [history (numTaps-1) ; block]; output j (j < blockSize / M) = sum over t ascending
 *     of s[M j + t] * h[t] from a zero accumulator; then the numTaps - 1 words from
 *     s[(blockSize / M) M] are moved to the front.  Accumulators: f32 mul then add; q15 q63
 *     (__SSAT(acc >> 15, 16)); fast q15 q31_t with wrapping adds (__SSAT(acc >> 15, 16)); q31
 *     q63 ((q31)(acc >> 31)); fast q31 acc = (q31)((((q63)acc << 32) + x*h) >> 32) with no
 *     rounding term, output (q31)(acc << 1).
 *   arm_fir_interpolate_{f32,q15,q31}.c: s = [history (phaseLength-1) ; block]; output
 *     n L + q = sum over i ascending of s[n + i] * h[(L-1-q) + i L]; f32 mul then add, q15 q63
 *     (__SSAT(acc >> 15, 16)), q31 q63 ((q31)(acc >> 31)); the last phaseLength - 1 words move
 *     to the front.
 *   arm_fir_decimate_init_*.c / arm_fir_interpolate_init_*.c: ARM_MATH_LENGTH_ERROR unless
 *     blockSize % M == 0 / numTaps % L == 0; the state is zeroed.
 *   arm_fir_sparse_{f32,q31,q15,q7}.c: the block is written into the circular state (L =
 *     maxDelay + blockSize words) at stateIndex, which advances by blockSize mod L
 *     (arm_circularWrite_f32); tap k reads blockSize words from (stateIndex - blockSize -
 *     D_k) (+ L if negative), wrapping at L (arm_circularRead_f32).  The first tap stores x c,
 *     later taps add: f32 mul then add; q31 (q31)((q63 x c) >> 32) with wrap, output << 1; q15 /
 *     q7 q31 products with wrap, __SSAT(>> 15, 16) / __SSAT(>> 7, 8).  arm_fir_sparse_init_*.c
 *     zeroes maxDelay + blockSize words and stateIndex.
 *   arm_fir_lattice_{f32,q31,q15}.c: per sample f = g = x(n); stage m: f' = g_{m-1}(n-1) k + f,
 *     g' = f k + g_{m-1}(n-1) (f32 mul then add; q31 ((q31)((q63 a k) >> 32) << 1) + b with
 *     wrap; q15 __SSAT(((a k) >> 15) + b, 16)), state[m-1] <- g_{m-1}(n); y = f_M.
 * Pinned against oracle/_ref by tests/test_multirate.py, tests/test_sparse.py and
 * tests/test_lattice.py. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum { MR_F32, MR_Q15, MR_FQ15, MR_Q31, MR_FQ31 };

static int16_t sat16(int64_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

/* one output: sum_{i < n} x[i * xs] * h[i * hs], ascending */
static void mr_dot(int op, const void *x, int xs, const void *h, int hs, int n, void *out) {
  if (op == MR_F32) {
    const float *a = x, *b = h;
    float s = 0.0f;
    for (int i = 0; i < n; ++i) { const float p = a[i * xs] * b[i * hs]; s = s + p; }
    *(float *)out = s;
  } else if (op == MR_Q15 || op == MR_FQ15) {
    const int16_t *a = x, *b = h;
    if (op == MR_Q15) {
      int64_t s = 0;
      for (int i = 0; i < n; ++i) s += (int32_t)a[i * xs] * b[i * hs];
      *(int16_t *)out = sat16(s >> 15);
    } else {
      uint32_t s = 0;
      for (int i = 0; i < n; ++i) s += (uint32_t)((int32_t)a[i * xs] * b[i * hs]);
      *(int16_t *)out = sat16((int32_t)s >> 15);
    }
  } else {
    const int32_t *a = x, *b = h;
    if (op == MR_Q31) {
      uint64_t s = 0;
      for (int i = 0; i < n; ++i) s += (uint64_t)((int64_t)a[i * xs] * b[i * hs]);
      *(int32_t *)out = (int32_t)((int64_t)s >> 31);
    } else {
      int32_t s = 0;
      for (int i = 0; i < n; ++i) {
        const uint64_t wide = ((uint64_t)(int64_t)s << 32) + (uint64_t)((int64_t)a[i * xs] * b[i * hs]);
        s = (int32_t)(uint32_t)((int64_t)wide >> 32);
      }
      *(int32_t *)out = (int32_t)((uint32_t)s << 1);
    }
  }
}

static void decimate(int op, size_t es, uint8_t M, uint16_t taps, const void *h, void *state, const void *src,
                     void *dst, uint32_t B) {
  char *s = state;
  memcpy(s + es * (taps - 1), src, es * B);
  const uint32_t outs = B / M;
  for (uint32_t j = 0; j < outs; ++j) mr_dot(op, s + es * ((size_t)M * j), 1, h, 1, taps, (char *)dst + es * j);
  memmove(s, s + es * ((size_t)outs * M), es * (taps - 1));
}

static void interpolate(int op, size_t es, uint8_t L, uint16_t P, const void *h, void *state, const void *src,
                        void *dst, uint32_t B) {
  char *s = state;
  memcpy(s + es * (P - 1), src, es * B);
  for (uint32_t n = 0; n < B; ++n)
    for (uint32_t q = 0; q < L; ++q)
      mr_dot(op, s + es * n, 1, (const char *)h + es * (L - 1 - q), L, P, (char *)dst + es * ((size_t)n * L + q));
  memmove(s, s + es * B, es * (P - 1));
}

#define DECIM(NAME, INST, T, OP)                                                              \
  void oracle_##NAME(const INST *S, const T *pSrc, T *pDst, uint32_t blockSize) {             \
    decimate(OP, sizeof(T), S->M, S->numTaps, S->pCoeffs, S->pState, pSrc, pDst, blockSize); \
  }
DECIM(arm_fir_decimate_f32, arm_fir_decimate_instance_f32, float, MR_F32)
DECIM(arm_fir_decimate_q15, arm_fir_decimate_instance_q15, int16_t, MR_Q15)
DECIM(arm_fir_decimate_fast_q15, arm_fir_decimate_instance_q15, int16_t, MR_FQ15)
DECIM(arm_fir_decimate_q31, arm_fir_decimate_instance_q31, int32_t, MR_Q31)
DECIM(arm_fir_decimate_fast_q31, arm_fir_decimate_instance_q31, int32_t, MR_FQ31)

#define INTERP(NAME, INST, T, OP)                                                                  \
  void oracle_##NAME(const INST *S, const T *pSrc, T *pDst, uint32_t blockSize) {                  \
    interpolate(OP, sizeof(T), S->L, S->phaseLength, S->pCoeffs, S->pState, pSrc, pDst, blockSize); \
  }
INTERP(arm_fir_interpolate_f32, arm_fir_interpolate_instance_f32, float, MR_F32)
INTERP(arm_fir_interpolate_q15, arm_fir_interpolate_instance_q15, int16_t, MR_Q15)
INTERP(arm_fir_interpolate_q31, arm_fir_interpolate_instance_q31, int32_t, MR_Q31)

#define DINIT(T, ET)                                                                                          \
  arm_status oracle_arm_fir_decimate_init_##T(arm_fir_decimate_instance_##T *S, uint16_t numTaps, uint8_t M,   \
                                              const ET *pCoeffs, ET *pState, uint32_t blockSize) {             \
    if (M == 0 || blockSize % M) return ARM_MATH_LENGTH_ERROR;                                                \
    S->numTaps = numTaps; S->pCoeffs = pCoeffs; S->pState = pState; S->M = M;                                \
    memset(pState, 0, sizeof(ET) * ((size_t)numTaps + blockSize - 1));                                        \
    return ARM_MATH_SUCCESS;                                                                                  \
  }                                                                                                           \
  arm_status oracle_arm_fir_interpolate_init_##T(arm_fir_interpolate_instance_##T *S, uint8_t L, uint16_t numTaps, \
                                                 const ET *pCoeffs, ET *pState, uint32_t blockSize) {         \
    if (L == 0 || numTaps % L) return ARM_MATH_LENGTH_ERROR;                                                  \
    S->pCoeffs = pCoeffs; S->L = L; S->phaseLength = numTaps / L; S->pState = pState;                         \
    memset(pState, 0, sizeof(ET) * ((size_t)blockSize + S->phaseLength - 1));                                 \
    return ARM_MATH_SUCCESS;                                                                                  \
  }
DINIT(f32, float)
DINIT(q15, int16_t)
DINIT(q31, int32_t)

/* ---- sparse FIR ---- */
enum { SP_F32, SP_Q31, SP_Q15, SP_Q7 };

static int32_t sp_word(int op, const void *s, int32_t i) {
  switch (op) {
    case SP_Q31: return ((const int32_t *)s)[i];
    case SP_Q15: return ((const int16_t *)s)[i];
    default: return ((const int8_t *)s)[i];
  }
}

static void sparse(int op, size_t es, uint16_t taps, uint16_t *stateIndex, uint16_t maxDelay, const void *h,
                   const int32_t *delays, void *state, const void *src, void *dst, uint32_t B) {
  const int32_t L = (int32_t)maxDelay + (int32_t)B;
  int32_t w = *stateIndex;
  for (uint32_t n = 0; n < B; ++n) {           /* circular write */
    memcpy((char *)state + es * w, (const char *)src + es * n, es);
    if (++w >= L) w -= L;
  }
  *stateIndex = (uint16_t)w;
  float *yf = dst;
  uint32_t *acc = NULL;
  if (op != SP_F32) acc = calloc(B, sizeof(uint32_t));
  for (uint16_t k = 0; k < taps; ++k) {
    int32_t r = (int32_t)(*stateIndex - B) - delays[k];
    if (r < 0) r += L;
    for (uint32_t n = 0; n < B; ++n) {
      if (op == SP_F32) {
        const float p = ((const float *)state)[r] * ((const float *)h)[k];
        yf[n] = k == 0 ? p : yf[n] + p;
      } else {
        const int32_t x = sp_word(op, state, r), c = sp_word(op, h, k);
        const uint32_t t = op == SP_Q31 ? (uint32_t)(int32_t)(((int64_t)x * c) >> 32) : (uint32_t)(x * c);
        acc[n] = k == 0 ? t : acc[n] + t;
      }
      if (++r >= L) r -= L;
    }
  }
  for (uint32_t n = 0; op != SP_F32 && n < B; ++n) {
    const int32_t a = (int32_t)acc[n];
    if (op == SP_Q31) ((int32_t *)dst)[n] = (int32_t)((uint32_t)a << 1);
    else if (op == SP_Q15) ((int16_t *)dst)[n] = sat16(a >> 15);
    else ((int8_t *)dst)[n] = (int8_t)((a >> 7) > 127 ? 127 : (a >> 7) < -128 ? -128 : (a >> 7));
  }
  free(acc);
}

#define SPARSE_INIT(T, ET)                                                                                       \
  void oracle_arm_fir_sparse_init_##T(arm_fir_sparse_instance_##T *S, uint16_t numTaps, const ET *pCoeffs,       \
                                      ET *pState, int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize) {   \
    S->numTaps = numTaps; S->pCoeffs = pCoeffs; S->pTapDelay = pTapDelay; S->maxDelay = maxDelay;                \
    S->stateIndex = 0;                                                                                           \
    memset(pState, 0, sizeof(ET) * ((size_t)maxDelay + blockSize));                                              \
    S->pState = pState;                                                                                          \
  }
SPARSE_INIT(f32, float)
SPARSE_INIT(q31, int32_t)
SPARSE_INIT(q15, int16_t)
SPARSE_INIT(q7, int8_t)
#define SPARSE_RUN(T, OP) \
  sparse(OP, sizeof(*pSrc), S->numTaps, &S->stateIndex, S->maxDelay, S->pCoeffs, S->pTapDelay, S->pState, pSrc, pDst, blockSize)
/* the reference's signatures; the scratch buffers are not needed */
void oracle_arm_fir_sparse_f32(arm_fir_sparse_instance_f32 *S, const float *pSrc, float *pDst, float *pScratchIn,
                               uint32_t blockSize) { SPARSE_RUN(f32, SP_F32); }
void oracle_arm_fir_sparse_q31(arm_fir_sparse_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, int32_t *pScratchIn,
                               uint32_t blockSize) { SPARSE_RUN(q31, SP_Q31); }
void oracle_arm_fir_sparse_q15(arm_fir_sparse_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, int16_t *pScratchIn,
                               int32_t *pScratchOut, uint32_t blockSize) { SPARSE_RUN(q15, SP_Q15); }
void oracle_arm_fir_sparse_q7(arm_fir_sparse_instance_q7 *S, const int8_t *pSrc, int8_t *pDst, int8_t *pScratchIn,
                              int32_t *pScratchOut, uint32_t blockSize) { SPARSE_RUN(q7, SP_Q7); }

/* ---- FIR lattice ---- */
static float lat_f32(float a, float k, float b) { const float p = a * k; return p + b; }
static int32_t lat_q31(int32_t a, int32_t k, int32_t b) {
  return (int32_t)(((uint32_t)(int32_t)(((int64_t)a * k) >> 32) << 1) + (uint32_t)b);
}
static int32_t lat_q15(int32_t a, int32_t k, int32_t b) { return sat16(((a * k) >> 15) + (int64_t)b); }

#define LATTICE(T, ET, VT, STEP)                                                                                \
  void oracle_arm_fir_lattice_init_##T(arm_fir_lattice_instance_##T *S, uint16_t numStages, const ET *pCoeffs,  \
                                       ET *pState) {                                                            \
    S->numStages = numStages; S->pCoeffs = pCoeffs; S->pState = pState;                                         \
    memset(pState, 0, sizeof(ET) * numStages);                                                                  \
  }                                                                                                             \
  void oracle_arm_fir_lattice_##T(const arm_fir_lattice_instance_##T *S, const ET *pSrc, ET *pDst,              \
                                  uint32_t blockSize) {                                                         \
    ET *g = S->pState;                                                                                          \
    for (uint32_t n = 0; n < blockSize; ++n) {                                                                  \
      VT f = pSrc[n], gc = f;                                                                                   \
      for (uint16_t m = 0; m < S->numStages; ++m) {                                                             \
        const VT k = S->pCoeffs[m], gp = g[m], fo = f;                                                          \
        g[m] = (ET)gc;                                                                                          \
        f = STEP(gp, k, fo);                                                                                    \
        gc = STEP(fo, k, gp);                                                                                   \
      }                                                                                                         \
      pDst[n] = (ET)f;                                                                                          \
    }                                                                                                           \
  }
LATTICE(f32, float, float, lat_f32)
LATTICE(q31, int32_t, int32_t, lat_q31)
LATTICE(q15, int16_t, int32_t, lat_q15)
