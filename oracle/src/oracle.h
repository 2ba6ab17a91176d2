/* ORACLE — test infrastructure only.  Prototypes of the CPU restatement; the instance
 * types are the reference layouts (include/arm_math.h). */
#ifndef ORACLE_H
#define ORACLE_H
#include "../../include/arm_math.h"
#include "../../include/arm_const_structs.h"

void oracle_arm_cfft_f32(const arm_cfft_instance_f32 *S, float *p1, uint8_t ifftFlag, uint8_t bitReverseFlag);
void oracle_arm_cfft_q31(const arm_cfft_instance_q31 *S, int32_t *p1, uint8_t ifftFlag, uint8_t bitReverseFlag);
void oracle_arm_cfft_q15(const arm_cfft_instance_q15 *S, int16_t *p1, uint8_t ifftFlag, uint8_t bitReverseFlag);
void oracle_arm_rfft_fast_f32(const arm_rfft_fast_instance_f32 *S, float *p, float *pOut, uint8_t ifftFlag);
void oracle_arm_rfft_q31(const arm_rfft_instance_q31 *S, int32_t *pSrc, int32_t *pDst);
void oracle_arm_rfft_q15(const arm_rfft_instance_q15 *S, int16_t *pSrc, int16_t *pDst);
arm_status oracle_arm_rfft_init_q31(arm_rfft_instance_q31 *S, uint32_t n, uint32_t ifftFlagR, uint32_t bitReverseFlag);
arm_status oracle_arm_rfft_init_q15(arm_rfft_instance_q15 *S, uint32_t n, uint32_t ifftFlagR, uint32_t bitReverseFlag);
void oracle_arm_fir_f32(const arm_fir_instance_f32 *S, const float *pSrc, float *pDst, uint32_t blockSize);
void oracle_arm_fir_q15(const arm_fir_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, uint32_t blockSize);
void oracle_arm_fir_fast_q15(const arm_fir_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, uint32_t blockSize);
void oracle_arm_fir_q7(const arm_fir_instance_q7 *S, const int8_t *pSrc, int8_t *pDst, uint32_t blockSize);
void oracle_arm_fir_init_q7(arm_fir_instance_q7 *S, uint16_t numTaps, const int8_t *pCoeffs, int8_t *pState,
                            uint32_t blockSize);
void oracle_arm_fir_q31(const arm_fir_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, uint32_t blockSize);
void oracle_arm_fir_fast_q31(const arm_fir_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, uint32_t blockSize);
arm_status oracle_arm_mat_mult_f32(const arm_matrix_instance_f32 *A, const arm_matrix_instance_f32 *B,
                                   arm_matrix_instance_f32 *C);
arm_status oracle_mat_mult_f32_fmaf(const arm_matrix_instance_f32 *A, const arm_matrix_instance_f32 *B,
                                    arm_matrix_instance_f32 *Cm);
arm_status oracle_arm_mat_mult_q7(const arm_matrix_instance_q7 *A, const arm_matrix_instance_q7 *B,
                                  arm_matrix_instance_q7 *C, int8_t *pState);
arm_status oracle_arm_mat_mult_q15(const arm_matrix_instance_q15 *A, const arm_matrix_instance_q15 *B,
                                   arm_matrix_instance_q15 *C, int16_t *pState);
arm_status oracle_arm_mat_mult_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                   arm_matrix_instance_q31 *C);
arm_status oracle_arm_mat_mult_opt_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                       arm_matrix_instance_q31 *C, int32_t *pState);
arm_status oracle_arm_mat_mult_fast_q15(const arm_matrix_instance_q15 *A, const arm_matrix_instance_q15 *B,
                                        arm_matrix_instance_q15 *C, int16_t *pState);
arm_status oracle_arm_mat_mult_fast_q31(const arm_matrix_instance_q31 *A, const arm_matrix_instance_q31 *B,
                                        arm_matrix_instance_q31 *C);
void oracle_arm_conv_f32(const float *pSrcA, uint32_t srcALen, const float *pSrcB, uint32_t srcBLen, float *pDst);
void oracle_arm_conv_q15(const int16_t *pSrcA, uint32_t srcALen, const int16_t *pSrcB, uint32_t srcBLen, int16_t *pDst);
void oracle_arm_conv_q31(const int32_t *pSrcA, uint32_t srcALen, const int32_t *pSrcB, uint32_t srcBLen, int32_t *pDst);
arm_status oracle_arm_mfcc_init_f32(arm_mfcc_instance_f32 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const float *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const float *filterCoefs,
                                    const float *windowCoefs);
void oracle_arm_mfcc_f32(const arm_mfcc_instance_f32 *S, float *pSrc, float *pDst, float *pTmp);
arm_status oracle_arm_mfcc_init_q31(arm_mfcc_instance_q31 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const int32_t *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const int32_t *filterCoefs,
                                    const int32_t *windowCoefs);
arm_status oracle_arm_mfcc_q31(const arm_mfcc_instance_q31 *S, int32_t *pSrc, int32_t *pDst, int32_t *pTmp);
arm_status oracle_arm_mfcc_init_q15(arm_mfcc_instance_q15 *S, uint32_t fftLen, uint32_t nbMelFilters,
                                    uint32_t nbDctOutputs, const int16_t *dctCoefs, const uint32_t *filterPos,
                                    const uint32_t *filterLengths, const int16_t *filterCoefs,
                                    const int16_t *windowCoefs);
arm_status oracle_arm_mfcc_q15(const arm_mfcc_instance_q15 *S, int16_t *pSrc, int16_t *pDst, int32_t *pTmp);
/* sparse FIR (oracle_multirate.c), the reference's signatures */
#define ORACLE_SPARSE_PROTO(T, ET)                                                                          \
  void oracle_arm_fir_sparse_init_##T(arm_fir_sparse_instance_##T *S, uint16_t numTaps, const ET *pCoeffs, \
                                      ET *pState, int32_t *pTapDelay, uint16_t maxDelay, uint32_t blockSize);
ORACLE_SPARSE_PROTO(f32, float)
ORACLE_SPARSE_PROTO(q31, int32_t)
ORACLE_SPARSE_PROTO(q15, int16_t)
ORACLE_SPARSE_PROTO(q7, int8_t)
void oracle_arm_fir_sparse_f32(arm_fir_sparse_instance_f32 *S, const float *pSrc, float *pDst, float *pScratchIn,
                               uint32_t blockSize);
void oracle_arm_fir_sparse_q31(arm_fir_sparse_instance_q31 *S, const int32_t *pSrc, int32_t *pDst, int32_t *pScratchIn,
                               uint32_t blockSize);
void oracle_arm_fir_sparse_q15(arm_fir_sparse_instance_q15 *S, const int16_t *pSrc, int16_t *pDst, int16_t *pScratchIn,
                               int32_t *pScratchOut, uint32_t blockSize);
void oracle_arm_fir_sparse_q7(arm_fir_sparse_instance_q7 *S, const int8_t *pSrc, int8_t *pDst, int8_t *pScratchIn,
                              int32_t *pScratchOut, uint32_t blockSize);
#undef ORACLE_SPARSE_PROTO

/* FIR lattice (oracle_multirate.c) */
void oracle_arm_fir_lattice_init_f32(arm_fir_lattice_instance_f32 *S, uint16_t numStages, const float *pCoeffs,
                                     float *pState);
void oracle_arm_fir_lattice_init_q31(arm_fir_lattice_instance_q31 *S, uint16_t numStages, const int32_t *pCoeffs,
                                     int32_t *pState);
void oracle_arm_fir_lattice_init_q15(arm_fir_lattice_instance_q15 *S, uint16_t numStages, const int16_t *pCoeffs,
                                     int16_t *pState);
void oracle_arm_fir_lattice_f32(const arm_fir_lattice_instance_f32 *S, const float *pSrc, float *pDst,
                                uint32_t blockSize);
void oracle_arm_fir_lattice_q31(const arm_fir_lattice_instance_q31 *S, const int32_t *pSrc, int32_t *pDst,
                                uint32_t blockSize);
void oracle_arm_fir_lattice_q15(const arm_fir_lattice_instance_q15 *S, const int16_t *pSrc, int16_t *pDst,
                                uint32_t blockSize);

/* scratch-buffer convolution forms (oracle_conv.c) */
void oracle_arm_conv_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d, int16_t *s1,
                             int16_t *s2);
void oracle_arm_conv_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d, int16_t *s1,
                                  int16_t *s2);
void oracle_arm_conv_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d, int16_t *s1,
                            int16_t *s2);
void oracle_arm_correlate_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d, int16_t *s);
void oracle_arm_correlate_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                       int16_t *s);
void oracle_arm_correlate_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d, int16_t *s1,
                                 int16_t *s2);
arm_status oracle_arm_conv_partial_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B, int16_t *d,
                                           uint32_t f, uint32_t n, int16_t *s1, int16_t *s2);
arm_status oracle_arm_conv_partial_fast_opt_q15(const int16_t *a, uint32_t A, const int16_t *b, uint32_t B,
                                                int16_t *d, uint32_t f, uint32_t n, int16_t *s1, int16_t *s2);
arm_status oracle_arm_conv_partial_opt_q7(const int8_t *a, uint32_t A, const int8_t *b, uint32_t B, int8_t *d,
                                          uint32_t f, uint32_t n, int16_t *s1, int16_t *s2);

#endif
