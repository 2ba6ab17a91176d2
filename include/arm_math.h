/*
 * arm_math.h — drop-in subset of the CMSIS-DSP public API, served by the MI355X backend
 * (libcmsisdsp_mi355x.so).  Only the hot path named in BASELINE.json `north_star` lives
 * here: complex FFT f32/q31/q15, real FFT (fast) f32, FIR f32/q15, matrix multiply f32.
 *
 * Every type and prototype keeps the reference's layout and signature so that existing
 * C callers recompile unchanged.  Each declaration cites the reference interface it
 * replaces (paths relative to the reference tree, xavierbrgt/CMSIS-DSP).
 *
 * Semantics contract:
 *   - processing functions are synchronous: when they return, the result is in p1/pDst;
 *   - buffers may be host memory (staged through pinned memory) or device memory
 *     (hipMalloc'd; used in place, no copies);
 *   - an unsupported fftLen is a silent no-op, exactly like the reference switch;
 *   - no processing function aborts or throws: a device failure is reported through
 *     arm_mi355x_last_error() (arm_math_mi355x.h).
 * The batched, stream-ordered, device-pointer API lives in arm_math_mi355x.h.
 */
#ifndef ARM_MATH_MI355X_DROPIN_H
#define ARM_MATH_MI355X_DROPIN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar types: Include/arm_math_types.h:324-351 ---------------------------- */
typedef int8_t   q7_t;
typedef int16_t  q15_t;
typedef int32_t  q31_t;
typedef int64_t  q63_t;
typedef float    float32_t;
typedef double   float64_t;

/* ---- status codes: Include/arm_math_types.h:603-613 ---------------------------- */
typedef enum {
  ARM_MATH_SUCCESS               =  0,
  ARM_MATH_ARGUMENT_ERROR        = -1,
  ARM_MATH_LENGTH_ERROR          = -2,
  ARM_MATH_SIZE_MISMATCH         = -3,
  ARM_MATH_NANINF                = -4,
  ARM_MATH_SINGULAR              = -5,
  ARM_MATH_TEST_FAILURE          = -6,
  ARM_MATH_DECOMPOSITION_FAILURE = -7
} arm_status;

/* ---- transform buffer-size helpers: Include/arm_math_types.h:667-700 (enums, default target)
 * and Include/dsp/transform_functions.h:1307-1398 (functions; bodies in
 * Source/TransformFunctions/arm_transform_buffer_sizes.c:47-330).  Lengths in real elements;
 * 0 = buffer not needed, -1 = configuration not supported.  This library is a scalar-API build:
 * ARM_MATH_DEFAULT_TARGET_ARCH is ARM_MATH_SCALAR_ARCH, and the MFCC is RFFT-based
 * (ARM_MFCC_USE_CFFT undefined, as in the reference's default build). ---------------------- */
typedef enum {
  ARM_MATH_F16 = 16,
  ARM_MATH_F32 = 32,
  ARM_MATH_F64 = 64,
  ARM_MATH_Q7  = 7,
  ARM_MATH_Q15 = 15,
  ARM_MATH_Q31 = 31
} arm_math_datatype;

typedef enum {
  ARM_MATH_SCALAR_ARCH         = 1,
  ARM_MATH_DSP_EXTENSIONS_ARCH = 2,
  ARM_MATH_HELIUM_ARCH         = 3,
  ARM_MATH_NEON_ARCH           = 4
} arm_math_target_arch;

#define ARM_MATH_DEFAULT_TARGET_ARCH ARM_MATH_SCALAR_ARCH

int32_t arm_cfft_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id);
int32_t arm_cfft_output_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples);
int32_t arm_cifft_output_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples);
int32_t arm_rfft_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id);
int32_t arm_rfft_output_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples);
int32_t arm_rifft_input_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples);
int32_t arm_mfcc_tmp_buffer_size(arm_math_target_arch arch, arm_math_datatype dt, uint32_t nb_samples,
                                 uint32_t buf_id, uint32_t use_cfft);

/* ---- complex FFT instances: Include/dsp/transform_functions.h:282-296,347-361,410-424
 * (scalar/non-Helium layout: {fftLen, pTwiddle, pBitRevTable, bitRevLength}) -------- */
typedef struct {
        uint16_t   fftLen;
  const float32_t *pTwiddle;
  const uint16_t  *pBitRevTable;
        uint16_t   bitRevLength;
} arm_cfft_instance_f32;

typedef struct {
        uint16_t   fftLen;
  const q31_t     *pTwiddle;
  const uint16_t  *pBitRevTable;
        uint16_t   bitRevLength;
} arm_cfft_instance_q31;

typedef struct {
        uint16_t   fftLen;
  const q15_t     *pTwiddle;
  const uint16_t  *pBitRevTable;
        uint16_t   bitRevLength;
} arm_cfft_instance_q15;

/* ---- real FFT (fast) instance: Include/dsp/transform_functions.h:813-818 ---------- */
typedef struct {
        arm_cfft_instance_f32 Sint;
        uint16_t              fftLenRFFT;
  const float32_t            *pTwiddleRFFT;
} arm_rfft_fast_instance_f32;

/* ---- real FFT instances, q31 / q15 (non-Neon, non-MVE build):
 * Include/dsp/transform_functions.h:636-649 (q31), :508-521 (q15) */
typedef struct {
        uint32_t   fftLenReal;            /* real length N (32 ... 8192) */
        uint8_t    ifftFlagR;             /* 0 forward, 1 inverse */
        uint8_t    bitReverseFlagR;       /* passed to the inner CFFT */
        uint32_t   twidCoefRModifier;     /* 8192 / N: stride into realCoefA/BQ31 */
  const q31_t     *pTwiddleAReal;
  const q31_t     *pTwiddleBReal;
  const arm_cfft_instance_q31 *pCfft;     /* inner CFFT of N/2 */
} arm_rfft_instance_q31;

typedef struct {
        uint32_t   fftLenReal;
        uint8_t    ifftFlagR;
        uint8_t    bitReverseFlagR;
        uint32_t   twidCoefRModifier;
  const q15_t     *pTwiddleAReal;
  const q15_t     *pTwiddleBReal;
  const arm_cfft_instance_q15 *pCfft;
} arm_rfft_instance_q15;

/* ---- MFCC instance (RFFT-based default build): Include/dsp/transform_functions.h:856-873 */
typedef struct {
  const float32_t *dctCoefs;        /* nbDctOutputs x nbMelFilters, row-major */
  const float32_t *filterCoefs;     /* concatenated Mel filters (sum of filterLengths) */
  const float32_t *windowCoefs;     /* fftLen */
  const uint32_t  *filterPos;       /* first FFT bin of each Mel filter */
  const uint32_t  *filterLengths;   /* bins per Mel filter */
        uint32_t   fftLen;
        uint32_t   nbMelFilters;
        uint32_t   nbDctOutputs;
  arm_rfft_fast_instance_f32 rfft;
} arm_mfcc_instance_f32;

/* Include/dsp/transform_functions.h:1000-1020 (RFFT-based default build) */
typedef struct {
  const q31_t    *dctCoefs;
  const q31_t    *filterCoefs;
  const q31_t    *windowCoefs;
  const uint32_t *filterPos;
  const uint32_t *filterLengths;
        uint32_t   fftLen;
        uint32_t   nbMelFilters;
        uint32_t   nbDctOutputs;
  arm_rfft_instance_q31 rfft;
} arm_mfcc_instance_q31;

/* Include/dsp/transform_functions.h:1150-1168 (RFFT-based default build) */
typedef struct {
  const q15_t    *dctCoefs;
  const q15_t    *filterCoefs;
  const q15_t    *windowCoefs;
  const uint32_t *filterPos;
  const uint32_t *filterLengths;
        uint32_t   fftLen;
        uint32_t   nbMelFilters;
        uint32_t   nbDctOutputs;
  arm_rfft_instance_q15 rfft;
} arm_mfcc_instance_q15;

/* ---- FIR instances: Include/dsp/filtering_functions.h:56-61 (q7), 66-71, 76-81, 86-91 */
typedef struct {
        uint16_t   numTaps;
        q7_t      *pState;
  const q7_t      *pCoeffs;
} arm_fir_instance_q7;

typedef struct {
        uint16_t   numTaps;
        q15_t     *pState;
  const q15_t     *pCoeffs;
} arm_fir_instance_q15;

typedef struct {
        uint16_t   numTaps;
        q31_t     *pState;
  const q31_t     *pCoeffs;
} arm_fir_instance_q31;

typedef struct {
        uint16_t   numTaps;
        float32_t *pState;
  const float32_t *pCoeffs;
} arm_fir_instance_f32;

/* ---- multirate FIR instances: Include/dsp/filtering_functions.h:803-831 (decimators),
 * :1012-1040 (interpolators) */
typedef struct {
        uint8_t    M;
        uint16_t   numTaps;
  const q15_t     *pCoeffs;
        q15_t     *pState;
} arm_fir_decimate_instance_q15;

typedef struct {
        uint8_t    M;
        uint16_t   numTaps;
  const q31_t     *pCoeffs;
        q31_t     *pState;
} arm_fir_decimate_instance_q31;

typedef struct {
        uint8_t    M;
        uint16_t   numTaps;
  const float32_t *pCoeffs;
        float32_t *pState;
} arm_fir_decimate_instance_f32;

typedef struct {
        uint8_t    L;
        uint16_t   phaseLength;
  const q15_t     *pCoeffs;
        q15_t     *pState;
} arm_fir_interpolate_instance_q15;

typedef struct {
        uint8_t    L;
        uint16_t   phaseLength;
  const q31_t     *pCoeffs;
        q31_t     *pState;
} arm_fir_interpolate_instance_q31;

typedef struct {
        uint8_t    L;
        uint16_t   phaseLength;
  const float32_t *pCoeffs;
        float32_t *pState;
} arm_fir_interpolate_instance_f32;

/* Sparse FIR instances (Include/dsp/filtering_functions.h:2033-2091), same layout for each type. */
#define MI355X_SPARSE_INST(T, ET)                                                               \
  typedef struct {                                                                              \
          uint16_t numTaps;    /* nonzero taps */                                               \
          uint16_t stateIndex; /* circular write position in pState */                          \
          ET      *pState;     /* maxDelay + blockSize words (circular) */                      \
    const ET      *pCoeffs;    /* numTaps */                                                    \
          uint16_t maxDelay;                                                                    \
          int32_t *pTapDelay;  /* numTaps delays, each in [0, maxDelay] */                      \
  } arm_fir_sparse_instance_##T;
MI355X_SPARSE_INST(f32, float32_t)
MI355X_SPARSE_INST(q31, q31_t)
MI355X_SPARSE_INST(q15, q15_t)
MI355X_SPARSE_INST(q7, q7_t)
#undef MI355X_SPARSE_INST

/* FIR lattice instances (Include/dsp/filtering_functions.h:1312-1340), same layout per type. */
#define MI355X_LATTICE_INST(T, ET)                                                              \
  typedef struct {                                                                              \
          uint16_t numStages;                                                                   \
          ET      *pState;     /* numStages words: g_m at the previous sample */                \
    const ET      *pCoeffs;    /* numStages reflection coefficients */                          \
  } arm_fir_lattice_instance_##T;
MI355X_LATTICE_INST(q15, q15_t)
MI355X_LATTICE_INST(q31, q31_t)
MI355X_LATTICE_INST(f32, float32_t)
#undef MI355X_LATTICE_INST

/* ---- matrix instances: Include/dsp/matrix_functions.h:118-123 (f32), :139-143 (q7),
 * :139-144 (q15), :149-154 (q31) */
typedef struct {
  uint16_t   numRows;
  uint16_t   numCols;
  q7_t      *pData;
} arm_matrix_instance_q7;

typedef struct {
  uint16_t   numRows;
  uint16_t   numCols;
  float32_t *pData;
} arm_matrix_instance_f32;

typedef struct {
  uint16_t   numRows;
  uint16_t   numCols;
  q15_t     *pData;
} arm_matrix_instance_q15;

typedef struct {
  uint16_t   numRows;
  uint16_t   numCols;
  q31_t     *pData;
} arm_matrix_instance_q31;

/* ===================================================================================
 * Complex FFT, f32.  Prototypes: Include/dsp/transform_functions.h:428-460
 * Reference bodies: Source/TransformFunctions/arm_cfft_init_f32.c:121-136,291-354,
 *                   Source/TransformFunctions/arm_cfft_f32.c:1243-1298
 * =================================================================================== */
arm_status arm_cfft_init_4096_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_2048_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_1024_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_512_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_256_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_128_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_64_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_32_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_16_f32(arm_cfft_instance_f32 *S);
arm_status arm_cfft_init_f32(arm_cfft_instance_f32 *S, uint16_t fftLen);
void arm_cfft_f32(const arm_cfft_instance_f32 *S, float32_t *p1,
                  uint8_t ifftFlag, uint8_t bitReverseFlag);

/* ===================================================================================
 * Complex FFT, q31.  Prototypes: Include/dsp/transform_functions.h:364-394
 * Reference bodies: Source/TransformFunctions/arm_cfft_init_q31.c,
 *                   Source/TransformFunctions/arm_cfft_q31.c:704-755
 * =================================================================================== */
arm_status arm_cfft_init_4096_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_2048_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_1024_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_512_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_256_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_128_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_64_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_32_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_16_q31(arm_cfft_instance_q31 *S);
arm_status arm_cfft_init_q31(arm_cfft_instance_q31 *S, uint16_t fftLen);
void arm_cfft_q31(const arm_cfft_instance_q31 *S, q31_t *p1,
                  uint8_t ifftFlag, uint8_t bitReverseFlag);

/* ===================================================================================
 * Complex FFT, q15.  Prototypes: Include/dsp/transform_functions.h:299-331
 * Reference bodies: Source/TransformFunctions/arm_cfft_init_q15.c,
 *                   Source/TransformFunctions/arm_cfft_q15.c:671-722
 * =================================================================================== */
arm_status arm_cfft_init_4096_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_2048_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_1024_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_512_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_256_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_128_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_64_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_32_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_16_q15(arm_cfft_instance_q15 *S);
arm_status arm_cfft_init_q15(arm_cfft_instance_q15 *S, uint16_t fftLen);
void arm_cfft_q15(const arm_cfft_instance_q15 *S, q15_t *p1,
                  uint8_t ifftFlag, uint8_t bitReverseFlag);

/* ===================================================================================
 * Real FFT (fast), f32.  Prototypes: Include/dsp/transform_functions.h:820-849
 * Reference bodies: Source/TransformFunctions/arm_rfft_fast_init_f32.c:228-244,
 *                   Source/TransformFunctions/arm_rfft_fast_f32.c:675-699
 * Note (reference behaviour kept): the forward transform overwrites p.
 * =================================================================================== */
arm_status arm_rfft_fast_init_32_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_64_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_128_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_256_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_512_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_1024_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_2048_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_4096_f32(arm_rfft_fast_instance_f32 *S);
arm_status arm_rfft_fast_init_f32(arm_rfft_fast_instance_f32 *S, uint16_t fftLen);
void arm_rfft_fast_f32(const arm_rfft_fast_instance_f32 *S, float32_t *p,
                       float32_t *pOut, uint8_t ifftFlag);

/* ===================================================================================
 * Real FFT, q31 / q15.  Prototypes: Include/dsp/transform_functions.h:695-749 (q31),
 * :566-620 (q15).  Reference bodies: Source/TransformFunctions/arm_rfft_init_q31.c:99-124,
 * :429-478, arm_rfft_q31.c:148-183 (+ arm_split_rfft_q31 / arm_split_rifft_q31, scalar
 * branches), arm_rfft_init_q15.c, arm_rfft_q15.c (scalar, !ARM_MATH_DSP branches).
 * Lengths 32 ... 8192.  Forward: pSrc (N words) is overwritten by the inner CFFT, pDst
 * receives 2N words (the full conjugate-symmetric spectrum).  Inverse: pSrc holds the
 * spectrum (words 0 .. N+1 are read), pDst receives N words (<< 1, saturated).
 * =================================================================================== */
#define ARM_MI355X_DECL_RFFT_INIT(N)                                                        \
  arm_status arm_rfft_init_##N##_q31(arm_rfft_instance_q31 *S, uint32_t ifftFlagR,          \
                                     uint32_t bitReverseFlag);                              \
  arm_status arm_rfft_init_##N##_q15(arm_rfft_instance_q15 *S, uint32_t ifftFlagR,          \
                                     uint32_t bitReverseFlag);
ARM_MI355X_DECL_RFFT_INIT(32)
ARM_MI355X_DECL_RFFT_INIT(64)
ARM_MI355X_DECL_RFFT_INIT(128)
ARM_MI355X_DECL_RFFT_INIT(256)
ARM_MI355X_DECL_RFFT_INIT(512)
ARM_MI355X_DECL_RFFT_INIT(1024)
ARM_MI355X_DECL_RFFT_INIT(2048)
ARM_MI355X_DECL_RFFT_INIT(4096)
ARM_MI355X_DECL_RFFT_INIT(8192)
#undef ARM_MI355X_DECL_RFFT_INIT
arm_status arm_rfft_init_q31(arm_rfft_instance_q31 *S, uint32_t fftLenReal, uint32_t ifftFlagR,
                             uint32_t bitReverseFlag);
arm_status arm_rfft_init_q15(arm_rfft_instance_q15 *S, uint32_t fftLenReal, uint32_t ifftFlagR,
                             uint32_t bitReverseFlag);
void arm_rfft_q31(const arm_rfft_instance_q31 *S, q31_t *pSrc, q31_t *pDst);
void arm_rfft_q15(const arm_rfft_instance_q15 *S, q15_t *pSrc, q15_t *pDst);

/* ===================================================================================
 * MFCC, f32.  Prototypes: Include/dsp/transform_functions.h:875-990
 * Reference bodies: Source/TransformFunctions/arm_mfcc_init_f32.c (init by length and
 * generic), Source/TransformFunctions/arm_mfcc_f32.c:83-160 (RFFT-based path).
 * pTmp: 2*fftLen floats as in the reference.  After the call the contents of pSrc and
 * pTmp are unspecified (the reference documents pSrc as modified); Mel filters must lie
 * within bins [0, fftLen/2) -- the reference reads uninitialised pTmp words beyond them.
 * =================================================================================== */
arm_status arm_mfcc_init_32_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                const float32_t *dctCoefs, const uint32_t *filterPos,
                                const uint32_t *filterLengths, const float32_t *filterCoefs,
                                const float32_t *windowCoefs);
arm_status arm_mfcc_init_64_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                const float32_t *dctCoefs, const uint32_t *filterPos,
                                const uint32_t *filterLengths, const float32_t *filterCoefs,
                                const float32_t *windowCoefs);
arm_status arm_mfcc_init_128_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                 const float32_t *dctCoefs, const uint32_t *filterPos,
                                 const uint32_t *filterLengths, const float32_t *filterCoefs,
                                 const float32_t *windowCoefs);
arm_status arm_mfcc_init_256_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                 const float32_t *dctCoefs, const uint32_t *filterPos,
                                 const uint32_t *filterLengths, const float32_t *filterCoefs,
                                 const float32_t *windowCoefs);
arm_status arm_mfcc_init_512_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                 const float32_t *dctCoefs, const uint32_t *filterPos,
                                 const uint32_t *filterLengths, const float32_t *filterCoefs,
                                 const float32_t *windowCoefs);
arm_status arm_mfcc_init_1024_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                  const float32_t *dctCoefs, const uint32_t *filterPos,
                                  const uint32_t *filterLengths, const float32_t *filterCoefs,
                                  const float32_t *windowCoefs);
arm_status arm_mfcc_init_2048_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                  const float32_t *dctCoefs, const uint32_t *filterPos,
                                  const uint32_t *filterLengths, const float32_t *filterCoefs,
                                  const float32_t *windowCoefs);
arm_status arm_mfcc_init_4096_f32(arm_mfcc_instance_f32 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                                  const float32_t *dctCoefs, const uint32_t *filterPos,
                                  const uint32_t *filterLengths, const float32_t *filterCoefs,
                                  const float32_t *windowCoefs);
arm_status arm_mfcc_init_f32(arm_mfcc_instance_f32 *S, uint32_t fftLen, uint32_t nbMelFilters,
                             uint32_t nbDctOutputs, const float32_t *dctCoefs, const uint32_t *filterPos,
                             const uint32_t *filterLengths, const float32_t *filterCoefs,
                             const float32_t *windowCoefs);
void arm_mfcc_f32(const arm_mfcc_instance_f32 *S, float32_t *pSrc, float32_t *pDst, float32_t *pTmp);

/* MFCC q31.  Reference bodies: Source/TransformFunctions/arm_mfcc_init_q31.c (generic and
 * per-length init: RFFT q31 forward with bit reversal), arm_mfcc_q31.c:88-225 (RFFT-based
 * default path; output q8.23).  pSrc and pTmp are work buffers of the reference; the GPU
 * path uses device scratch and leaves them as they were.  Mel filters must lie within the
 * fftLen/2 + 1 spectrum magnitudes (ARM_MATH_ARGUMENT_ERROR otherwise). */
arm_status arm_mfcc_init_q31(arm_mfcc_instance_q31 *S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                             const q31_t *dctCoefs, const uint32_t *filterPos, const uint32_t *filterLengths,
                             const q31_t *filterCoefs, const q31_t *windowCoefs);
#define ARM_MI355X_DECL_MFCC_Q31_INIT(N)                                                                    \
  arm_status arm_mfcc_init_##N##_q31(arm_mfcc_instance_q31 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs, \
                                     const q31_t *dctCoefs, const uint32_t *filterPos,                       \
                                     const uint32_t *filterLengths, const q31_t *filterCoefs,                \
                                     const q31_t *windowCoefs);
ARM_MI355X_DECL_MFCC_Q31_INIT(32)
ARM_MI355X_DECL_MFCC_Q31_INIT(64)
ARM_MI355X_DECL_MFCC_Q31_INIT(128)
ARM_MI355X_DECL_MFCC_Q31_INIT(256)
ARM_MI355X_DECL_MFCC_Q31_INIT(512)
ARM_MI355X_DECL_MFCC_Q31_INIT(1024)
ARM_MI355X_DECL_MFCC_Q31_INIT(2048)
ARM_MI355X_DECL_MFCC_Q31_INIT(4096)
#undef ARM_MI355X_DECL_MFCC_Q31_INIT
arm_status arm_mfcc_q31(const arm_mfcc_instance_q31 *S, q31_t *pSrc, q31_t *pDst, q31_t *pTmp);

/* MFCC q15.  Reference bodies: Source/TransformFunctions/arm_mfcc_init_q15.c, arm_mfcc_q15.c:96-228
 * (RFFT-based default path; q15 input, q8.7 output, q31 work buffer).  Same buffer contract as
 * arm_mfcc_q31. */
arm_status arm_mfcc_init_q15(arm_mfcc_instance_q15 *S, uint32_t fftLen, uint32_t nbMelFilters, uint32_t nbDctOutputs,
                             const q15_t *dctCoefs, const uint32_t *filterPos, const uint32_t *filterLengths,
                             const q15_t *filterCoefs, const q15_t *windowCoefs);
#define ARM_MI355X_DECL_MFCC_Q15_INIT(N)                                                                    \
  arm_status arm_mfcc_init_##N##_q15(arm_mfcc_instance_q15 *S, uint32_t nbMelFilters, uint32_t nbDctOutputs, \
                                     const q15_t *dctCoefs, const uint32_t *filterPos,                       \
                                     const uint32_t *filterLengths, const q15_t *filterCoefs,                \
                                     const q15_t *windowCoefs);
ARM_MI355X_DECL_MFCC_Q15_INIT(32)
ARM_MI355X_DECL_MFCC_Q15_INIT(64)
ARM_MI355X_DECL_MFCC_Q15_INIT(128)
ARM_MI355X_DECL_MFCC_Q15_INIT(256)
ARM_MI355X_DECL_MFCC_Q15_INIT(512)
ARM_MI355X_DECL_MFCC_Q15_INIT(1024)
ARM_MI355X_DECL_MFCC_Q15_INIT(2048)
ARM_MI355X_DECL_MFCC_Q15_INIT(4096)
#undef ARM_MI355X_DECL_MFCC_Q15_INIT
arm_status arm_mfcc_q15(const arm_mfcc_instance_q15 *S, q15_t *pSrc, q15_t *pDst, q31_t *pTmp);

/* ===================================================================================
 * FIR.  Prototypes: Include/dsp/filtering_functions.h:141-145,175-180,233-237,260-265
 * Reference bodies: Source/FilteringFunctions/arm_fir_f32.c:911-1280,
 *                   arm_fir_init_f32.c:74-95, arm_fir_q15.c:458-726, arm_fir_init_q15.c:86-139
 * pState holds numTaps+blockSize-1 samples; the last numTaps-1 are carried to the
 * next call (streaming state), as in the reference.
 * =================================================================================== */
void arm_fir_init_f32(arm_fir_instance_f32 *S, uint16_t numTaps,
                      const float32_t *pCoeffs, float32_t *pState, uint32_t blockSize);
void arm_fir_f32(const arm_fir_instance_f32 *S, const float32_t *pSrc,
                 float32_t *pDst, uint32_t blockSize);
arm_status arm_fir_init_q15(arm_fir_instance_q15 *S, uint16_t numTaps,
                            const q15_t *pCoeffs, q15_t *pState, uint32_t blockSize);
void arm_fir_q15(const arm_fir_instance_q15 *S, const q15_t *pSrc,
                 q15_t *pDst, uint32_t blockSize);

/* Further FIR variants.  Prototypes: Include/dsp/filtering_functions.h
 * :154-158 (fast q15), :189-193 (q31), :202-206 (fast q31), :219-224 (init q31).
 * Reference bodies: Source/FilteringFunctions/arm_fir_fast_q15.c (q31_t accumulator, __SMLAD:
 * mod-2^32 sum, __SSAT(acc >> 15, 16)), arm_fir_q31.c (q63 sum of exact products,
 * (q31)(acc >> 31)), arm_fir_fast_q31.c (multAcc_32x32_keep32_R per tap, (q31)(acc << 1)),
 * arm_fir_init_q31.c.  numTaps must be even for the q15 variants, as in the reference. */
void arm_fir_init_q31(arm_fir_instance_q31 *S, uint16_t numTaps,
                      const q31_t *pCoeffs, q31_t *pState, uint32_t blockSize);
void arm_fir_q31(const arm_fir_instance_q31 *S, const q31_t *pSrc,
                 q31_t *pDst, uint32_t blockSize);
void arm_fir_fast_q31(const arm_fir_instance_q31 *S, const q31_t *pSrc,
                      q31_t *pDst, uint32_t blockSize);
void arm_fir_fast_q15(const arm_fir_instance_q15 *S, const q15_t *pSrc,
                      q15_t *pDst, uint32_t blockSize);
/* q7 FIR.  Prototypes: Include/dsp/filtering_functions.h:110-114 (arm_fir_q7), :127-132
 * (arm_fir_init_q7).  Reference bodies: Source/FilteringFunctions/arm_fir_q7.c:446-560 (q31_t
 * accumulator of q7 x q7 products, wrapping int32 adds, __SSAT(acc >> 7, 8)),
 * arm_fir_init_q7.c:67-85 (state numTaps + blockSize - 1 words, zeroed). */
void arm_fir_init_q7(arm_fir_instance_q7 *S, uint16_t numTaps, const q7_t *pCoeffs, q7_t *pState,
                     uint32_t blockSize);
void arm_fir_q7(const arm_fir_instance_q7 *S, const q7_t *pSrc, q7_t *pDst, uint32_t blockSize);

/* ===================================================================================
 * Multirate FIR.  Prototypes: Include/dsp/filtering_functions.h:886-1007 (decimators),
 * :1050-1150 (interpolators).  Reference bodies: Source/FilteringFunctions/
 * arm_fir_decimate_{f32,q15,fast_q15,q31,fast_q31}.c and arm_fir_interpolate_{f32,q15,q31}.c
 * (generic C paths), arm_fir_decimate_init_*.c (ARM_MATH_LENGTH_ERROR unless blockSize % M
 * == 0; state numTaps + blockSize - 1 words), arm_fir_interpolate_init_*.c
 * (ARM_MATH_LENGTH_ERROR unless numTaps % L == 0; phaseLength = numTaps / L; state
 * blockSize + phaseLength - 1 words).  Decimator output j = sum_t s[M j + t] h[t] (blockSize / M
 * outputs); interpolator output n L + q = sum_i s[n + i] h[(L-1-q) + i L] (blockSize L outputs);
 * s = [history ; block].  Accumulators: f32 mul then add, q15 / q31 q63 sums (__SSAT(>> 15) /
 * >> 31), fast q15 a wrapping q31 sum with __SSAT(>> 15), fast q31 acc + floor(x h / 2^32)
 * (no rounding term), output << 1.  M == 0 / L == 0 return ARM_MATH_LENGTH_ERROR (the
 * reference divides by zero).
 * =================================================================================== */
arm_status arm_fir_decimate_init_f32(arm_fir_decimate_instance_f32 *S, uint16_t numTaps, uint8_t M,
                                     const float32_t *pCoeffs, float32_t *pState, uint32_t blockSize);
arm_status arm_fir_decimate_init_q15(arm_fir_decimate_instance_q15 *S, uint16_t numTaps, uint8_t M,
                                     const q15_t *pCoeffs, q15_t *pState, uint32_t blockSize);
arm_status arm_fir_decimate_init_q31(arm_fir_decimate_instance_q31 *S, uint16_t numTaps, uint8_t M,
                                     const q31_t *pCoeffs, q31_t *pState, uint32_t blockSize);
void arm_fir_decimate_f32(const arm_fir_decimate_instance_f32 *S, const float32_t *pSrc, float32_t *pDst,
                          uint32_t blockSize);
void arm_fir_decimate_q15(const arm_fir_decimate_instance_q15 *S, const q15_t *pSrc, q15_t *pDst,
                          uint32_t blockSize);
void arm_fir_decimate_fast_q15(const arm_fir_decimate_instance_q15 *S, const q15_t *pSrc, q15_t *pDst,
                               uint32_t blockSize);
void arm_fir_decimate_q31(const arm_fir_decimate_instance_q31 *S, const q31_t *pSrc, q31_t *pDst,
                          uint32_t blockSize);
void arm_fir_decimate_fast_q31(const arm_fir_decimate_instance_q31 *S, const q31_t *pSrc, q31_t *pDst,
                               uint32_t blockSize);
arm_status arm_fir_interpolate_init_f32(arm_fir_interpolate_instance_f32 *S, uint8_t L, uint16_t numTaps,
                                        const float32_t *pCoeffs, float32_t *pState, uint32_t blockSize);
arm_status arm_fir_interpolate_init_q15(arm_fir_interpolate_instance_q15 *S, uint8_t L, uint16_t numTaps,
                                        const q15_t *pCoeffs, q15_t *pState, uint32_t blockSize);
arm_status arm_fir_interpolate_init_q31(arm_fir_interpolate_instance_q31 *S, uint8_t L, uint16_t numTaps,
                                        const q31_t *pCoeffs, q31_t *pState, uint32_t blockSize);
void arm_fir_interpolate_f32(const arm_fir_interpolate_instance_f32 *S, const float32_t *pSrc, float32_t *pDst,
                             uint32_t blockSize);
void arm_fir_interpolate_q15(const arm_fir_interpolate_instance_q15 *S, const q15_t *pSrc, q15_t *pDst,
                             uint32_t blockSize);
void arm_fir_interpolate_q31(const arm_fir_interpolate_instance_q31 *S, const q31_t *pSrc, q31_t *pDst,
                             uint32_t blockSize);

/* ===================================================================================
 * Sparse FIR (widening).  Prototypes: Include/dsp/filtering_functions.h:2094-2231.  Reference
 * bodies: Source/FilteringFunctions/arm_fir_sparse_{f32,q31,q15,q7}.c, inits
 * arm_fir_sparse_init_*.c.  y[n] = sum over k ascending of x[n - pTapDelay[k]] pCoeffs[k]:
 * f32 first tap x c, then mul-then-add; q31 (q31)((q63 x c) >> 32) terms summed with wrap,
 * output << 1; q15 / q7 q31 product sums (wrap) then __SSAT(>> 15, 16) / __SSAT(>> 7, 8).
 * The block is written into the circular pState at stateIndex and every tap read back from it
 * at the reference's indices, so the state and stateIndex evolve exactly as the reference's.
 * pScratchIn / pScratchOut are accepted and not used.  numTaps == 1 is one product per output
 * (the reference's numTaps - 2 tap loop counter underflows there).
 * =================================================================================== */
void arm_fir_sparse_init_f32(arm_fir_sparse_instance_f32 *S, uint16_t numTaps, const float32_t *pCoeffs,
                             float32_t *pState, int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize);
void arm_fir_sparse_init_q31(arm_fir_sparse_instance_q31 *S, uint16_t numTaps, const q31_t *pCoeffs, q31_t *pState,
                             int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize);
void arm_fir_sparse_init_q15(arm_fir_sparse_instance_q15 *S, uint16_t numTaps, const q15_t *pCoeffs, q15_t *pState,
                             int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize);
void arm_fir_sparse_init_q7(arm_fir_sparse_instance_q7 *S, uint16_t numTaps, const q7_t *pCoeffs, q7_t *pState,
                            int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize);
void arm_fir_sparse_f32(arm_fir_sparse_instance_f32 *S, const float32_t *pSrc, float32_t *pDst,
                        float32_t *pScratchIn, uint32_t blockSize);
void arm_fir_sparse_q31(arm_fir_sparse_instance_q31 *S, const q31_t *pSrc, q31_t *pDst, q31_t *pScratchIn,
                        uint32_t blockSize);
void arm_fir_sparse_q15(arm_fir_sparse_instance_q15 *S, const q15_t *pSrc, q15_t *pDst, q15_t *pScratchIn,
                        q31_t *pScratchOut, uint32_t blockSize);
void arm_fir_sparse_q7(arm_fir_sparse_instance_q7 *S, const q7_t *pSrc, q7_t *pDst, q7_t *pScratchIn,
                       q31_t *pScratchOut, uint32_t blockSize);

/* ===================================================================================
 * FIR lattice (widening).  Prototypes: Include/dsp/filtering_functions.h:1350-1410.
 * Reference bodies: Source/FilteringFunctions/arm_fir_lattice_{f32,q31,q15}.c, inits
 * arm_fir_lattice_init_*.c (zero numStages state words).  f_m(n) = g_{m-1}(n-1) k_m +
 * f_{m-1}(n), g_m(n) = f_{m-1}(n) k_m + g_{m-1}(n-1), y = f_M: f32 mul then add; q31
 * ((q31)((q63 a k) >> 32) << 1) + b with wrap; q15 __SSAT(((a k) >> 15) + b, 16).
 * =================================================================================== */
void arm_fir_lattice_init_f32(arm_fir_lattice_instance_f32 *S, uint16_t numStages, const float32_t *pCoeffs,
                              float32_t *pState);
void arm_fir_lattice_init_q31(arm_fir_lattice_instance_q31 *S, uint16_t numStages, const q31_t *pCoeffs,
                              q31_t *pState);
void arm_fir_lattice_init_q15(arm_fir_lattice_instance_q15 *S, uint16_t numStages, const q15_t *pCoeffs,
                              q15_t *pState);
void arm_fir_lattice_f32(const arm_fir_lattice_instance_f32 *S, const float32_t *pSrc, float32_t *pDst,
                         uint32_t blockSize);
void arm_fir_lattice_q31(const arm_fir_lattice_instance_q31 *S, const q31_t *pSrc, q31_t *pDst, uint32_t blockSize);
void arm_fir_lattice_q15(const arm_fir_lattice_instance_q15 *S, const q15_t *pSrc, q15_t *pDst, uint32_t blockSize);

/* ===================================================================================
 * Convolution.  Prototypes: Include/dsp/filtering_functions.h
 * (arm_conv_f32 / _q15 / _q31).  Reference bodies: Source/FilteringFunctions/arm_conv_f32.c
 * (per output a sum over the overlap from 0.0f in ascending index of pSrcA, mul then add), arm_conv_q15.c (!ARM_MATH_DSP: q63 sum,
 * __SSAT(sum >> 15, 16)), arm_conv_q31.c (q63 sum, (q31)(sum >> 31)).  pDst holds
 * srcALen + srcBLen - 1 samples.
 * =================================================================================== */
void arm_conv_f32(const float32_t *pSrcA, uint32_t srcALen, const float32_t *pSrcB, uint32_t srcBLen,
                  float32_t *pDst);
void arm_conv_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst);
void arm_conv_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen, q31_t *pDst);

/* Fast fixed-point convolution (filtering_functions.h:503,555; arm_conv_fast_q15.c,
 * arm_conv_fast_q31.c): modular q31_t accumulators.  q15: __SMLAD sums, (q15)(sum >> 15),
 * including the reference's single-sample __SMLAD high-halfword term (+1 per MAC with both
 * samples negative in its stage-1/stage-3 remainder loops); q31: sum of (x*y) >> 32, output
 * sum << 1. */
void arm_conv_fast_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst);
void arm_conv_fast_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen, q31_t *pDst);

/* Partial convolution (filtering_functions.h:610,656,723; arm_conv_partial_{f32,q15,q31}.c
 * !ARM_MATH_DSP branch): outputs firstIndex .. firstIndex + numPoints - 1 of arm_conv_*,
 * written at pDst[firstIndex ...]; ARM_MATH_ARGUMENT_ERROR when firstIndex + numPoints >
 * srcALen + srcBLen - 1. */
arm_status arm_conv_partial_f32(const float32_t *pSrcA, uint32_t srcALen, const float32_t *pSrcB, uint32_t srcBLen,
                                float32_t *pDst, uint32_t firstIndex, uint32_t numPoints);
arm_status arm_conv_partial_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen,
                                q15_t *pDst, uint32_t firstIndex, uint32_t numPoints);
arm_status arm_conv_partial_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen,
                                q31_t *pDst, uint32_t firstIndex, uint32_t numPoints);
/* filtering_functions.h:677,744 (arm_conv_partial_fast_q15.c / _q31.c): words firstIndex ..
 * firstIndex + numPoints - 1 of arm_conv_fast_q15 / _q31.  The reference's bodies read
 * outside the inputs for most ranges on the host build (segfault), so parity is pinned to
 * arm_conv_fast_* over the range. */
arm_status arm_conv_partial_fast_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen,
                                     q15_t *pDst, uint32_t firstIndex, uint32_t numPoints);
arm_status arm_conv_partial_fast_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen,
                                     q31_t *pDst, uint32_t firstIndex, uint32_t numPoints);

/* Correlation (filtering_functions.h:1873,1923,1939,1973,1989; arm_correlate_f32.c:1013-1096,
 * arm_correlate_q15.c:814-895, arm_correlate_q31.c, arm_correlate_fast_q15.c,
 * arm_correlate_fast_q31.c).  pDst has 2 * max(srcALen, srcBLen) - 1 words; the
 * srcALen + srcBLen - 1 computed ones are written from pDst[srcALen - srcBLen] forward, or,
 * when srcALen < srcBLen, from pDst[srcALen + srcBLen - 2] backward; the others are left
 * untouched (the reference asks the caller to zero pDst). */
void arm_correlate_f32(const float32_t *pSrcA, uint32_t srcALen, const float32_t *pSrcB, uint32_t srcBLen,
                       float32_t *pDst);
void arm_correlate_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst);
void arm_correlate_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen, q31_t *pDst);
void arm_correlate_fast_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst);
void arm_correlate_fast_q31(const q31_t *pSrcA, uint32_t srcALen, const q31_t *pSrcB, uint32_t srcBLen, q31_t *pDst);

/* q7 convolution family.  Prototypes: Include/dsp/filtering_functions.h:591-596
 * (arm_conv_q7), :790-797 (arm_conv_partial_q7), :2025-2030 (arm_correlate_q7).  Reference
 * bodies: Source/FilteringFunctions/arm_conv_q7.c, arm_conv_partial_q7.c (!ARM_MATH_DSP,
 * :688-735), arm_correlate_q7.c: q31_t sum of q7 x q7 products (int32 adds and __SMLAD pairs,
 * both wrapping: a modular sum), __SSAT(sum >> 7, 8).  Output placement as the q15 forms. */
void arm_conv_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen, q7_t *pDst);
arm_status arm_conv_partial_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen,
                               q7_t *pDst, uint32_t firstIndex, uint32_t numPoints);
void arm_correlate_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen, q7_t *pDst);

/* Scratch-buffer ("_opt") forms.  Prototypes: Include/dsp/filtering_functions.h:469-476,
 * :521-528, :573-580, :633-642, :700-709, :767-776, :1906-1912, :1956-1962, :2007-2014.
 * Reference bodies: Source/FilteringFunctions/arm_conv_opt_q15.c, arm_conv_opt_q7.c,
 * arm_conv_fast_opt_q15.c, arm_conv_partial_opt_q15.c, arm_conv_partial_opt_q7.c,
 * arm_conv_partial_fast_opt_q15.c, arm_correlate_opt_q15.c, arm_correlate_opt_q7.c,
 * arm_correlate_fast_opt_q15.c.  The exact forms return the plain functions' words; the fast
 * q15 forms are a modular q31 sum with __SSAT(acc >> 15, 16) (arm_conv_fast_q15 casts
 * instead).  The scratch buffers may be NULL: the GPU path does not use them.  (The exact q15
 * forms accumulate exactly, as the Arm SMLALD instruction does; the reference's host C
 * emulation of __SMLALD, Include/dsp/none.h:503-505, wraps a pair of two (-32768)^2 products
 * in int32.) */
void arm_conv_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst,
                      q15_t *pScratch1, q15_t *pScratch2);
void arm_conv_fast_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst,
                           q15_t *pScratch1, q15_t *pScratch2);
void arm_conv_opt_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen, q7_t *pDst,
                     q15_t *pScratch1, q15_t *pScratch2);
arm_status arm_conv_partial_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen,
                                    q15_t *pDst, uint32_t firstIndex, uint32_t numPoints, q15_t *pScratch1,
                                    q15_t *pScratch2);
arm_status arm_conv_partial_fast_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen,
                                         q15_t *pDst, uint32_t firstIndex, uint32_t numPoints, q15_t *pScratch1,
                                         q15_t *pScratch2);
arm_status arm_conv_partial_opt_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen,
                                   q7_t *pDst, uint32_t firstIndex, uint32_t numPoints, q15_t *pScratch1,
                                   q15_t *pScratch2);
void arm_correlate_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen, q15_t *pDst,
                           q15_t *pScratch);
void arm_correlate_fast_opt_q15(const q15_t *pSrcA, uint32_t srcALen, const q15_t *pSrcB, uint32_t srcBLen,
                                q15_t *pDst, q15_t *pScratch);
void arm_correlate_opt_q7(const q7_t *pSrcA, uint32_t srcALen, const q7_t *pSrcB, uint32_t srcBLen, q7_t *pDst,
                          q15_t *pScratch1, q15_t *pScratch2);

/* ===================================================================================
 * Matrix multiply, f32.  Prototypes: Include/dsp/matrix_functions.h:341-344,630-634
 * Reference bodies: Source/MatrixFunctions/arm_mat_mult_f32.c:600-730,
 *                   Source/MatrixFunctions/arm_mat_init_f32.c
 * Size check: always performed (the reference checks only under ARM_MATH_MATRIX_CHECK,
 * arm_mat_mult_f32.c:618-630; a mismatched call is undefined there).
 * =================================================================================== */
void arm_mat_init_f32(arm_matrix_instance_f32 *S, uint16_t nRows, uint16_t nColumns,
                      float32_t *pData);
arm_status arm_mat_mult_f32(const arm_matrix_instance_f32 *pSrcA,
                            const arm_matrix_instance_f32 *pSrcB,
                            arm_matrix_instance_f32 *pDst);

/* Matrix multiply q15 / q31.  Prototypes: Include/dsp/matrix_functions.h
 * (arm_mat_mult_q15 with its pState transpose buffer, arm_mat_mult_q31, arm_mat_init_q15/_q31).
 * Reference bodies: Source/MatrixFunctions/arm_mat_mult_q15.c:741-912 (!ARM_MATH_DSP: q63
 * sum of exact products, __SSAT(sum >> 15, 16)), arm_mat_mult_q31.c:53-163 (q63 sum,
 * (q31)(sum >> 31)).  Bit-exact; pState is accepted and unused.  Size check always on. */
void arm_mat_init_q15(arm_matrix_instance_q15 *S, uint16_t nRows, uint16_t nColumns, q15_t *pData);
/* q7: matrix_functions.h:379-383 (arm_mat_mult_q7), :617-621 (arm_mat_init_q7); body
 * Source/MatrixFunctions/arm_mat_mult_q7.c:689-790 (scalar branch: q31_t sum of exact products,
 * (q7)__SSAT(sum >> 7, 8)), Source/MatrixFunctions/arm_mat_init_q7.c.  Bit-exact on one i8 MFMA
 * plane; pState is accepted and unused. */
void arm_mat_init_q7(arm_matrix_instance_q7 *S, uint16_t nRows, uint16_t nColumns, q7_t *pData);
arm_status arm_mat_mult_q7(const arm_matrix_instance_q7 *pSrcA, const arm_matrix_instance_q7 *pSrcB,
                           arm_matrix_instance_q7 *pDst, q7_t *pState);
void arm_mat_init_q31(arm_matrix_instance_q31 *S, uint16_t nRows, uint16_t nColumns, q31_t *pData);
arm_status arm_mat_mult_q15(const arm_matrix_instance_q15 *pSrcA, const arm_matrix_instance_q15 *pSrcB,
                            arm_matrix_instance_q15 *pDst, q15_t *pState);
arm_status arm_mat_mult_q31(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                            arm_matrix_instance_q31 *pDst);
/* matrix_functions.h:459-463.  The scalar branch of Source/MatrixFunctions/arm_mat_mult_opt_q31.c:
 * 648-780 is arm_mat_mult_q31's (q63 sum of exact products, (q31)(sum >> 31)) with an unused
 * pState, so this runs the same bit-exact i8-plane GEMM. */
arm_status arm_mat_mult_opt_q31(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                                arm_matrix_instance_q31 *pDst, q31_t *pState);
/* Fast fixed-point matrix multiply (matrix_functions.h:431-435,484-487):
 * arm_mat_mult_fast_q15.c (!ARM_MATH_DSP): q31_t modular sum of q15 products, (q15)(sum >> 15);
 * arm_mat_mult_fast_q31.c: sum = (q31)(((q63)sum << 32 + a*b) >> 32) per product, output
 * sum << 1.  pState (the reference's transpose buffer) is not used. */
arm_status arm_mat_mult_fast_q15(const arm_matrix_instance_q15 *pSrcA, const arm_matrix_instance_q15 *pSrcB,
                                 arm_matrix_instance_q15 *pDst, q15_t *pState);
arm_status arm_mat_mult_fast_q31(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                                 arm_matrix_instance_q31 *pDst);

#ifdef __cplusplus
}
#endif

#include "arm_const_structs.h"

#endif /* ARM_MATH_MI355X_DROPIN_H */
