/*
 * Drop-in check: the reference's arm_fft_bin_example (Examples/ARM/arm_fft_bin_example/
 * arm_fft_bin_example_f32.c:111-143) restated against libcmsisdsp_mi355x.so.  Unchanged
 * call sequence: arm_cfft_f32(&arm_cfft_sR_f32_len1024, buf, 0, 1), then the magnitude
 * and the peak search on the host.  Input: the example's 10 kHz test signal, read from a
 * raw float32 file (tests/golden fixture) because the C initialiser is the reference's.
 * Build:  gcc -Iinclude examples/fft_bin_dropin.c -Lcmsis-dsp_amd/lib -lcmsisdsp_mi355x -lm
 * Run:    LD_LIBRARY_PATH=cmsis-dsp_amd/lib ./a.out input.f32    -> prints "SUCCESS 213"
 */
#include <math.h>
#include <stdio.h>

#include "arm_math.h"
#include "arm_const_structs.h"

#define TEST_LENGTH_SAMPLES 2048

int main(int argc, char **argv) {
  static float32_t buf[TEST_LENGTH_SAMPLES];
  FILE *f = fopen(argc > 1 ? argv[1] : "input.f32", "rb");
  if (!f || fread(buf, sizeof(float32_t), TEST_LENGTH_SAMPLES, f) != TEST_LENGTH_SAMPLES) {
    fprintf(stderr, "cannot read input\n");
    return 2;
  }
  fclose(f);
  arm_cfft_f32(&arm_cfft_sR_f32_len1024, buf, 0, 1);          /* same call as the example */
  uint32_t best = 0;
  float32_t best_mag = -1.0f;
  for (uint32_t k = 0; k < TEST_LENGTH_SAMPLES / 2; ++k) {
    const float32_t m = sqrtf(buf[2 * k] * buf[2 * k] + buf[2 * k + 1] * buf[2 * k + 1]);
    if (m > best_mag) { best_mag = m; best = k; }
  }
  printf("%s %u\n", best == 213 ? "SUCCESS" : "FAILURE", best);   /* refIndex = 213 */
  return best == 213 ? 0 : 1;
}
