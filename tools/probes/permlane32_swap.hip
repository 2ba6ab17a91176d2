// Semantics of __builtin_amdgcn_permlane32_swap on gfx950: prints, for a few lanes, what the two
// returned values hold when vdst_old = 1000 + lane and src_old = 2000 + lane.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(1000u + l, 2000u + l, false, false);
  out[2 * l] = r[0];
  out[2 * l + 1] = r[1];
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 128 * 4);
  k<<<1, 64>>>(d);
  unsigned h[128];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: r0 = %u  r1 = %u\n", l, h[2 * l], h[2 * l + 1]);
  return 0;
}
