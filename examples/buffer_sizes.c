/* A reference-style application that sizes its transform buffers with the CMSIS-DSP buffer-size
 * helpers (Include/dsp/transform_functions.h:1307-1398) and links against the MI355X drop-in
 * library unchanged.  Prints "name=value" per buffer; tests/test_abi.py checks the numbers. */
#include <stdio.h>
#include <stdlib.h>

#include "arm_math.h"

int main(void) {
  const arm_math_target_arch arch = ARM_MATH_DEFAULT_TARGET_ARCH;
  const uint32_t n = 1024;
  const int32_t cfft_out = arm_cfft_output_buffer_size(arch, ARM_MATH_F32, n);
  const int32_t cfft_tmp = arm_cfft_tmp_buffer_size(arch, ARM_MATH_F32, n, 1);
  const int32_t rfft_out = arm_rfft_output_buffer_size(arch, ARM_MATH_F32, n);
  const int32_t rfft_q31_out = arm_rfft_output_buffer_size(arch, ARM_MATH_Q31, n);
  const int32_t rifft_q15_in = arm_rifft_input_buffer_size(arch, ARM_MATH_Q15, n);
  const int32_t mfcc_tmp = arm_mfcc_tmp_buffer_size(arch, ARM_MATH_F32, n, 1, 0);
  const int32_t mfcc_neon = arm_mfcc_tmp_buffer_size(ARM_MATH_NEON_ARCH, ARM_MATH_F32, n, 1, 1);
  /* the buffers an FFT application would allocate from them */
  float32_t *spectrum = (float32_t *)malloc(sizeof(float32_t) * (size_t)rfft_out);
  q31_t *spectrum_q31 = (q31_t *)malloc(sizeof(q31_t) * (size_t)rfft_q31_out);
  if (!spectrum || !spectrum_q31) return 1;
  printf("cfft_out=%d cfft_tmp=%d rfft_out=%d rfft_q31_out=%d rifft_q15_in=%d mfcc_tmp=%d mfcc_tmp_neon_cfft=%d\n",
         (int)cfft_out, (int)cfft_tmp, (int)rfft_out, (int)rfft_q31_out, (int)rifft_q15_in, (int)mfcc_tmp,
         (int)mfcc_neon);
  free(spectrum);
  free(spectrum_q31);
  return 0;
}
