// Host-side instance initialisation and the pre-initialised const instances.
//
// Mirrors Source/TransformFunctions/arm_cfft_init_{f32,q31,q15}.c (per-size CFFTINIT
// macros + the fftLen switch), arm_rfft_fast_init_f32.c, arm_rfft_init_{q31,q15}.c,
// Source/FilteringFunctions/
// arm_fir_init_{f32,q15}.c, Source/MatrixFunctions/arm_mat_init_f32.c and the const
// structs of Source/CommonTables/arm_const_structs.c.  Pure host code: filling a struct
// involves no device work (tables are uploaded lazily by the processing functions).
#include <string.h>

#include "../../include/arm_const_structs.h"
#include "../../include/arm_math.h"

extern "C" {

// ---- pre-initialised CFFT / RFFT instances (arm_const_structs.c:79-300)
#define MI_CFFT_CONSTS(N)                                                                              \
  const arm_cfft_instance_f32 arm_cfft_sR_f32_len##N = {N, twiddleCoef_##N, armBitRevIndexTable##N,     \
                                                        ARMBITREVINDEXTABLE_##N##_TABLE_LENGTH};        \
  const arm_cfft_instance_q31 arm_cfft_sR_q31_len##N = {N, twiddleCoef_##N##_q31,                       \
                                                        armBitRevIndexTable_fixed_##N,                  \
                                                        ARMBITREVINDEXTABLE_FIXED_##N##_TABLE_LENGTH};  \
  const arm_cfft_instance_q15 arm_cfft_sR_q15_len##N = {N, twiddleCoef_##N##_q15,                       \
                                                        armBitRevIndexTable_fixed_##N,                  \
                                                        ARMBITREVINDEXTABLE_FIXED_##N##_TABLE_LENGTH};
MI_CFFT_CONSTS(16)
MI_CFFT_CONSTS(32)
MI_CFFT_CONSTS(64)
MI_CFFT_CONSTS(128)
MI_CFFT_CONSTS(256)
MI_CFFT_CONSTS(512)
MI_CFFT_CONSTS(1024)
MI_CFFT_CONSTS(2048)
MI_CFFT_CONSTS(4096)
#undef MI_CFFT_CONSTS

#define MI_RFFT_CONST(N, H)                                                                         \
  const arm_rfft_fast_instance_f32 arm_rfft_fast_sR_f32_len##N = {                                 \
      {H, twiddleCoef_##H, armBitRevIndexTable##H, ARMBITREVINDEXTABLE_##H##_TABLE_LENGTH}, N,      \
      twiddleCoef_rfft_##N};
MI_RFFT_CONST(32, 16)
MI_RFFT_CONST(64, 32)
MI_RFFT_CONST(128, 64)
MI_RFFT_CONST(256, 128)
MI_RFFT_CONST(512, 256)
MI_RFFT_CONST(1024, 512)
MI_RFFT_CONST(2048, 1024)
MI_RFFT_CONST(4096, 2048)
#undef MI_RFFT_CONST

// ---- per-size CFFT init: copy the const instance (arm_cfft_init_f32.c:121-136)
#define MI_CFFT_INIT(N, T)                                                     \
  arm_status arm_cfft_init_##N##_##T(arm_cfft_instance_##T* S) {               \
    if (!S) return ARM_MATH_ARGUMENT_ERROR;                                    \
    *S = arm_cfft_sR_##T##_len##N;                                             \
    return ARM_MATH_SUCCESS;                                                   \
  }
#define MI_CFFT_INIT_ALL(T)                                                    \
  MI_CFFT_INIT(16, T) MI_CFFT_INIT(32, T) MI_CFFT_INIT(64, T)                  \
  MI_CFFT_INIT(128, T) MI_CFFT_INIT(256, T) MI_CFFT_INIT(512, T)               \
  MI_CFFT_INIT(1024, T) MI_CFFT_INIT(2048, T) MI_CFFT_INIT(4096, T)            \
  arm_status arm_cfft_init_##T(arm_cfft_instance_##T* S, uint16_t fftLen) {    \
    switch (fftLen) {                                                          \
      case 16: return arm_cfft_init_16_##T(S);                                 \
      case 32: return arm_cfft_init_32_##T(S);                                 \
      case 64: return arm_cfft_init_64_##T(S);                                 \
      case 128: return arm_cfft_init_128_##T(S);                               \
      case 256: return arm_cfft_init_256_##T(S);                               \
      case 512: return arm_cfft_init_512_##T(S);                               \
      case 1024: return arm_cfft_init_1024_##T(S);                             \
      case 2048: return arm_cfft_init_2048_##T(S);                             \
      case 4096: return arm_cfft_init_4096_##T(S);                             \
      default: return ARM_MATH_ARGUMENT_ERROR;                                 \
    }                                                                          \
  }
MI_CFFT_INIT_ALL(f32)
MI_CFFT_INIT_ALL(q31)
MI_CFFT_INIT_ALL(q15)
#undef MI_CFFT_INIT_ALL
#undef MI_CFFT_INIT

// ---- RFFT fast init (arm_rfft_fast_init_f32.c): inner CFFT of N/2 + RFFT twiddles
#define MI_RFFT_INIT(N)                                                        \
  arm_status arm_rfft_fast_init_##N##_f32(arm_rfft_fast_instance_f32* S) {     \
    if (!S) return ARM_MATH_ARGUMENT_ERROR;                                    \
    *S = arm_rfft_fast_sR_f32_len##N;                                          \
    return ARM_MATH_SUCCESS;                                                   \
  }
MI_RFFT_INIT(32)
MI_RFFT_INIT(64)
MI_RFFT_INIT(128)
MI_RFFT_INIT(256)
MI_RFFT_INIT(512)
MI_RFFT_INIT(1024)
MI_RFFT_INIT(2048)
MI_RFFT_INIT(4096)
#undef MI_RFFT_INIT

arm_status arm_rfft_fast_init_f32(arm_rfft_fast_instance_f32* S, uint16_t fftLen) {
  switch (fftLen) {
    case 32: return arm_rfft_fast_init_32_f32(S);
    case 64: return arm_rfft_fast_init_64_f32(S);
    case 128: return arm_rfft_fast_init_128_f32(S);
    case 256: return arm_rfft_fast_init_256_f32(S);
    case 512: return arm_rfft_fast_init_512_f32(S);
    case 1024: return arm_rfft_fast_init_1024_f32(S);
    case 2048: return arm_rfft_fast_init_2048_f32(S);
    case 4096: return arm_rfft_fast_init_4096_f32(S);
    default: return ARM_MATH_ARGUMENT_ERROR;
  }
}

// ---- RFFT q31 / q15 init (arm_rfft_init_q31.c:99-124 RFFTINIT_Q31 + the switch at
// :429-478; arm_rfft_init_q15.c likewise): split tables realCoef{A,B}Q31 / Q15 shared by
// every length with modifier 8192 / N, the inner CFFT of N/2 from the const instances.
#define MI_RFFTQ_INIT(N, H, MOD, T, TAB)                                                           \
  arm_status arm_rfft_init_##N##_##T(arm_rfft_instance_##T* S, uint32_t ifftFlagR, uint32_t bitReverseFlag) { \
    if (!S) return ARM_MATH_ARGUMENT_ERROR;                                                         \
    S->fftLenReal = N;                                                                              \
    S->pTwiddleAReal = realCoefA##TAB;                                                              \
    S->pTwiddleBReal = realCoefB##TAB;                                                              \
    S->ifftFlagR = (uint8_t)ifftFlagR;                                                              \
    S->bitReverseFlagR = (uint8_t)bitReverseFlag;                                                   \
    S->twidCoefRModifier = MOD;                                                                     \
    S->pCfft = &arm_cfft_sR_##T##_len##H;                                                           \
    return ARM_MATH_SUCCESS;                                                                        \
  }
#define MI_RFFTQ_ALL(T, TAB)                                                                       \
  MI_RFFTQ_INIT(8192, 4096, 1, T, TAB) MI_RFFTQ_INIT(4096, 2048, 2, T, TAB)                        \
  MI_RFFTQ_INIT(2048, 1024, 4, T, TAB) MI_RFFTQ_INIT(1024, 512, 8, T, TAB)                         \
  MI_RFFTQ_INIT(512, 256, 16, T, TAB) MI_RFFTQ_INIT(256, 128, 32, T, TAB)                          \
  MI_RFFTQ_INIT(128, 64, 64, T, TAB) MI_RFFTQ_INIT(64, 32, 128, T, TAB)                            \
  MI_RFFTQ_INIT(32, 16, 256, T, TAB)                                                               \
  arm_status arm_rfft_init_##T(arm_rfft_instance_##T* S, uint32_t fftLenReal, uint32_t ifftFlagR,  \
                               uint32_t bitReverseFlag) {                                          \
    switch (fftLenReal) {                                                                          \
      case 8192: return arm_rfft_init_8192_##T(S, ifftFlagR, bitReverseFlag);                      \
      case 4096: return arm_rfft_init_4096_##T(S, ifftFlagR, bitReverseFlag);                      \
      case 2048: return arm_rfft_init_2048_##T(S, ifftFlagR, bitReverseFlag);                      \
      case 1024: return arm_rfft_init_1024_##T(S, ifftFlagR, bitReverseFlag);                      \
      case 512: return arm_rfft_init_512_##T(S, ifftFlagR, bitReverseFlag);                        \
      case 256: return arm_rfft_init_256_##T(S, ifftFlagR, bitReverseFlag);                        \
      case 128: return arm_rfft_init_128_##T(S, ifftFlagR, bitReverseFlag);                        \
      case 64: return arm_rfft_init_64_##T(S, ifftFlagR, bitReverseFlag);                          \
      case 32: return arm_rfft_init_32_##T(S, ifftFlagR, bitReverseFlag);                          \
      default: return ARM_MATH_ARGUMENT_ERROR;                                                     \
    }                                                                                              \
  }
MI_RFFTQ_ALL(q31, Q31)
MI_RFFTQ_ALL(q15, Q15)
#undef MI_RFFTQ_ALL
#undef MI_RFFTQ_INIT

// ---- MFCC init (arm_mfcc_init_f32.c): record the tables, initialise the inner RFFT
static void mfcc_fields(arm_mfcc_instance_f32* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                        const float32_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                        const float32_t* filterCoefs, const float32_t* windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
}

arm_status arm_mfcc_init_f32(arm_mfcc_instance_f32* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                             const float32_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                             const float32_t* filterCoefs, const float32_t* windowCoefs) {
  mfcc_fields(S, fftLen, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs, windowCoefs);
  return fftLen > 0xFFFFu ? ARM_MATH_ARGUMENT_ERROR : arm_rfft_fast_init_f32(&S->rfft, (uint16_t)fftLen);
}

#define MI_MFCC_INIT(N)                                                                                        \
  arm_status arm_mfcc_init_##N##_f32(arm_mfcc_instance_f32* S, uint32_t nbMelFilters, uint32_t nbDctOutputs,   \
                                     const float32_t* dctCoefs, const uint32_t* filterPos,                     \
                                     const uint32_t* filterLengths, const float32_t* filterCoefs,              \
                                     const float32_t* windowCoefs) {                                           \
    mfcc_fields(S, N, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs, windowCoefs); \
    return arm_rfft_fast_init_##N##_f32(&S->rfft);                                                             \
  }
MI_MFCC_INIT(32)
MI_MFCC_INIT(64)
MI_MFCC_INIT(128)
MI_MFCC_INIT(256)
MI_MFCC_INIT(512)
MI_MFCC_INIT(1024)
MI_MFCC_INIT(2048)
MI_MFCC_INIT(4096)
#undef MI_MFCC_INIT

// ---- MFCC q31 init (arm_mfcc_init_q31.c): the fields, then the inner RFFT forward with
// bit reversal (RFFT_INIT(L) = arm_rfft_init_q31(&S->rfft, L, 0, 1))
static void mfcc_q31_fields(arm_mfcc_instance_q31* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                            const q31_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                            const q31_t* filterCoefs, const q31_t* windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
}

arm_status arm_mfcc_init_q31(arm_mfcc_instance_q31* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                             const q31_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                             const q31_t* filterCoefs, const q31_t* windowCoefs) {
  mfcc_q31_fields(S, fftLen, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs,
                  windowCoefs);
  return arm_rfft_init_q31(&S->rfft, fftLen, 0, 1);
}

#define MI_MFCC_Q31_INIT(N)                                                                                    \
  arm_status arm_mfcc_init_##N##_q31(arm_mfcc_instance_q31* S, uint32_t nbMelFilters, uint32_t nbDctOutputs,   \
                                     const q31_t* dctCoefs, const uint32_t* filterPos,                         \
                                     const uint32_t* filterLengths, const q31_t* filterCoefs,                  \
                                     const q31_t* windowCoefs) {                                               \
    mfcc_q31_fields(S, N, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs,         \
                    windowCoefs);                                                                              \
    return arm_rfft_init_##N##_q31(&S->rfft, 0, 1);                                                            \
  }
MI_MFCC_Q31_INIT(32)
MI_MFCC_Q31_INIT(64)
MI_MFCC_Q31_INIT(128)
MI_MFCC_Q31_INIT(256)
MI_MFCC_Q31_INIT(512)
MI_MFCC_Q31_INIT(1024)
MI_MFCC_Q31_INIT(2048)
MI_MFCC_Q31_INIT(4096)
#undef MI_MFCC_Q31_INIT

// ---- MFCC q15 init (arm_mfcc_init_q15.c): fields + arm_rfft_init_q15(&S->rfft, L, 0, 1)
static void mfcc_q15_fields(arm_mfcc_instance_q15* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                            const q15_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                            const q15_t* filterCoefs, const q15_t* windowCoefs) {
  S->fftLen = fftLen;
  S->nbMelFilters = nbMelFilters;
  S->nbDctOutputs = nbDctOutputs;
  S->dctCoefs = dctCoefs;
  S->filterPos = filterPos;
  S->filterLengths = filterLengths;
  S->filterCoefs = filterCoefs;
  S->windowCoefs = windowCoefs;
}

arm_status arm_mfcc_init_q15(arm_mfcc_instance_q15* S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                             const q15_t* dctCoefs, const uint32_t* filterPos, const uint32_t* filterLengths,
                             const q15_t* filterCoefs, const q15_t* windowCoefs) {
  mfcc_q15_fields(S, fftLen, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs,
                  windowCoefs);
  return arm_rfft_init_q15(&S->rfft, fftLen, 0, 1);
}

#define MI_MFCC_Q15_INIT(N)                                                                                    \
  arm_status arm_mfcc_init_##N##_q15(arm_mfcc_instance_q15* S, uint32_t nbMelFilters, uint32_t nbDctOutputs,   \
                                     const q15_t* dctCoefs, const uint32_t* filterPos,                         \
                                     const uint32_t* filterLengths, const q15_t* filterCoefs,                  \
                                     const q15_t* windowCoefs) {                                               \
    mfcc_q15_fields(S, N, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs,         \
                    windowCoefs);                                                                              \
    return arm_rfft_init_##N##_q15(&S->rfft, 0, 1);                                                            \
  }
MI_MFCC_Q15_INIT(32)
MI_MFCC_Q15_INIT(64)
MI_MFCC_Q15_INIT(128)
MI_MFCC_Q15_INIT(256)
MI_MFCC_Q15_INIT(512)
MI_MFCC_Q15_INIT(1024)
MI_MFCC_Q15_INIT(2048)
MI_MFCC_Q15_INIT(4096)
#undef MI_MFCC_Q15_INIT

// (FIR init zeroes a state buffer that may be device memory: it lives in api.cpp.)

// ---- matrix init (arm_mat_init_f32.c, arm_mat_init_q7.c, arm_mat_init_q15.c, arm_mat_init_q31.c)
void arm_mat_init_q7(arm_matrix_instance_q7* S, uint16_t nRows, uint16_t nColumns, q7_t* pData) {
  S->numRows = nRows;
  S->numCols = nColumns;
  S->pData = pData;
}
void arm_mat_init_q15(arm_matrix_instance_q15* S, uint16_t nRows, uint16_t nColumns, q15_t* pData) {
  S->numRows = nRows;
  S->numCols = nColumns;
  S->pData = pData;
}
void arm_mat_init_q31(arm_matrix_instance_q31* S, uint16_t nRows, uint16_t nColumns, q31_t* pData) {
  S->numRows = nRows;
  S->numCols = nColumns;
  S->pData = pData;
}
void arm_mat_init_f32(arm_matrix_instance_f32* S, uint16_t nRows, uint16_t nColumns, float32_t* pData) {
  S->numRows = nRows;
  S->numCols = nColumns;
  S->pData = pData;
}

}  // extern "C"
