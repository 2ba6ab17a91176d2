/* Prints the byte layout of the hot-path instance structs.  Compiled against the
 * reference headers (tools/make_golden.py -> tests/golden/abi_layout.json) and against
 * include/ (tests/test_abi.py); the two must agree for the drop-in promise. */
#include <stddef.h>
#include <stdio.h>
#include "arm_math.h"

#define S(T) printf("  \"" #T "\": {\"size\": %zu", sizeof(T));
#define F(T, f) printf(", \"" #f "\": %zu", offsetof(T, f));
#define E() printf("},\n");

int main(void) {
  printf("{\n");
  S(arm_cfft_instance_f32) F(arm_cfft_instance_f32, fftLen) F(arm_cfft_instance_f32, pTwiddle)
    F(arm_cfft_instance_f32, pBitRevTable) F(arm_cfft_instance_f32, bitRevLength) E()
  S(arm_cfft_instance_q31) F(arm_cfft_instance_q31, fftLen) F(arm_cfft_instance_q31, pTwiddle)
    F(arm_cfft_instance_q31, pBitRevTable) F(arm_cfft_instance_q31, bitRevLength) E()
  S(arm_cfft_instance_q15) F(arm_cfft_instance_q15, fftLen) F(arm_cfft_instance_q15, pTwiddle)
    F(arm_cfft_instance_q15, pBitRevTable) F(arm_cfft_instance_q15, bitRevLength) E()
  S(arm_rfft_fast_instance_f32) F(arm_rfft_fast_instance_f32, Sint) F(arm_rfft_fast_instance_f32, fftLenRFFT)
    F(arm_rfft_fast_instance_f32, pTwiddleRFFT) E()
  S(arm_fir_instance_f32) F(arm_fir_instance_f32, numTaps) F(arm_fir_instance_f32, pState)
    F(arm_fir_instance_f32, pCoeffs) E()
  S(arm_fir_instance_q15) F(arm_fir_instance_q15, numTaps) F(arm_fir_instance_q15, pState)
    F(arm_fir_instance_q15, pCoeffs) E()
  S(arm_matrix_instance_f32) F(arm_matrix_instance_f32, numRows) F(arm_matrix_instance_f32, numCols)
    F(arm_matrix_instance_f32, pData) E()
  S(arm_matrix_instance_q15) F(arm_matrix_instance_q15, numRows) F(arm_matrix_instance_q15, numCols)
    F(arm_matrix_instance_q15, pData) E()
  S(arm_matrix_instance_q31) F(arm_matrix_instance_q31, numRows) F(arm_matrix_instance_q31, numCols)
    F(arm_matrix_instance_q31, pData) E()
  S(arm_fir_instance_q31) F(arm_fir_instance_q31, numTaps) F(arm_fir_instance_q31, pState)
    F(arm_fir_instance_q31, pCoeffs) E()
  S(arm_mfcc_instance_f32) F(arm_mfcc_instance_f32, dctCoefs) F(arm_mfcc_instance_f32, filterCoefs)
    F(arm_mfcc_instance_f32, windowCoefs) F(arm_mfcc_instance_f32, filterPos) F(arm_mfcc_instance_f32, filterLengths)
    F(arm_mfcc_instance_f32, fftLen) F(arm_mfcc_instance_f32, nbMelFilters) F(arm_mfcc_instance_f32, nbDctOutputs)
    F(arm_mfcc_instance_f32, rfft) E()
  S(arm_fir_sparse_instance_f32) F(arm_fir_sparse_instance_f32, numTaps) F(arm_fir_sparse_instance_f32, stateIndex)
    F(arm_fir_sparse_instance_f32, pState) F(arm_fir_sparse_instance_f32, pCoeffs)
    F(arm_fir_sparse_instance_f32, maxDelay) F(arm_fir_sparse_instance_f32, pTapDelay) E()
  S(arm_fir_sparse_instance_q7) F(arm_fir_sparse_instance_q7, numTaps) F(arm_fir_sparse_instance_q7, stateIndex)
    F(arm_fir_sparse_instance_q7, pState) F(arm_fir_sparse_instance_q7, pCoeffs)
    F(arm_fir_sparse_instance_q7, maxDelay) F(arm_fir_sparse_instance_q7, pTapDelay) E()
  S(arm_fir_decimate_instance_q15) F(arm_fir_decimate_instance_q15, M) F(arm_fir_decimate_instance_q15, numTaps)
    F(arm_fir_decimate_instance_q15, pCoeffs) F(arm_fir_decimate_instance_q15, pState) E()
  S(arm_fir_interpolate_instance_f32) F(arm_fir_interpolate_instance_f32, L)
    F(arm_fir_interpolate_instance_f32, phaseLength) F(arm_fir_interpolate_instance_f32, pCoeffs)
    F(arm_fir_interpolate_instance_f32, pState) E()
  S(arm_fir_instance_q7) F(arm_fir_instance_q7, numTaps) F(arm_fir_instance_q7, pState) F(arm_fir_instance_q7, pCoeffs) E()
  S(arm_fir_lattice_instance_q15) F(arm_fir_lattice_instance_q15, numStages) F(arm_fir_lattice_instance_q15, pState)
    F(arm_fir_lattice_instance_q15, pCoeffs) E()
  S(arm_fir_lattice_instance_f32) F(arm_fir_lattice_instance_f32, numStages) F(arm_fir_lattice_instance_f32, pState)
    F(arm_fir_lattice_instance_f32, pCoeffs) E()
  S(arm_rfft_instance_q31) F(arm_rfft_instance_q31, fftLenReal) F(arm_rfft_instance_q31, ifftFlagR)
    F(arm_rfft_instance_q31, bitReverseFlagR) F(arm_rfft_instance_q31, twidCoefRModifier)
    F(arm_rfft_instance_q31, pTwiddleAReal) F(arm_rfft_instance_q31, pTwiddleBReal) F(arm_rfft_instance_q31, pCfft) E()
  S(arm_rfft_instance_q15) F(arm_rfft_instance_q15, fftLenReal) F(arm_rfft_instance_q15, ifftFlagR)
    F(arm_rfft_instance_q15, bitReverseFlagR) F(arm_rfft_instance_q15, twidCoefRModifier)
    F(arm_rfft_instance_q15, pTwiddleAReal) F(arm_rfft_instance_q15, pTwiddleBReal) F(arm_rfft_instance_q15, pCfft) E()
  printf("  \"arm_status\": {\"size\": %zu, \"ARM_MATH_SIZE_MISMATCH\": %d}\n}\n", sizeof(arm_status),
         (int)ARM_MATH_SIZE_MISMATCH);
  return 0;
}
