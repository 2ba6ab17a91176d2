/*
 * The batched device API from plain C + HIP runtime: 4096 transforms of 1024 points,
 * forward then inverse on one stream, bit-identical to 4096 arm_cfft_f32 calls.
 * Build: gcc -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude examples/batched_cfft.c \
 *          -Lcmsis-dsp_amd/lib -lcmsisdsp_mi355x -L/opt/rocm/lib -lamdhip64 -lm
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "arm_const_structs.h"
#include "arm_math_mi355x.h"

int main(void) {
  const uint32_t n = 1024, batch = 4096;
  const size_t bytes = sizeof(float) * 2 * n * batch;
  float *h = (float *)malloc(bytes), *d = NULL;
  for (size_t i = 0; i < 2 * (size_t)n * batch; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.0f - 0.5f;
  hipStream_t s;
  if (hipMalloc((void **)&d, bytes) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 2;
  hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
  arm_status st = arm_cfft_f32_batch(&arm_cfft_sR_f32_len1024, d, batch, 0, 1, s);   /* forward */
  if (st == ARM_MATH_SUCCESS) st = arm_cfft_f32_batch(&arm_cfft_sR_f32_len1024, d, batch, 1, 1, s);  /* inverse */
  hipStreamSynchronize(s);
  float *r = (float *)malloc(bytes);
  hipMemcpy(r, d, bytes, hipMemcpyDeviceToHost);
  double err = 0;
  for (size_t i = 0; i < 2 * (size_t)n * batch; ++i) { double e = r[i] - h[i]; err = e * e > err ? e * e : err; }
  printf("status %d, round-trip max |err| %.3g -> %s\n", (int)st, err > 0 ? __builtin_sqrt(err) : 0.0,
         st == ARM_MATH_SUCCESS && err < 1e-10 ? "OK" : "FAIL");
  return st == ARM_MATH_SUCCESS ? 0 : 1;
}
