// In-kernel timestamps of the persistent ping-pong q7 GEMM (mat_mult_q7.hip, MI355X_Q7_STAMP):
// s_memtime at every barrier of waves 0 (group 0) and 4 (group 1) of workgroups 0-63, for the
// bench shape 1024^3 x 64.  Prints one JSON object: {"stamps": [[wg][group][k] ...]} (shader
// clock ticks), analysed by tools/probes/q7_stamps.py.  With -DMI355X_Q7_STAMP=2 (the 128-deep
// kernel) the same buffer holds per-segment tick sums instead (q7_stamps.py --phases).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMI355X_Q7_STAMP=1 \
//          tools/probes/q7_stamps.hip -o tools/probes/q7_stamps
#include "../../cmsis-dsp_amd/csrc/mat_mult_q7.hip"
#include <stdio.h>
#include <stdlib.h>
#include <vector>

int main(int argc, char** argv) {
  const int n = 1024, batch = argc > 1 ? atoi(argv[1]) : 64;
  const size_t mat = (size_t)n * n;
  std::vector<int8_t> h(mat * batch);
  unsigned s = 12345u;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (int8_t)(s >> 24); }
  int8_t *a, *b, *c;
  if (hipMalloc(&a, mat * batch) || hipMalloc(&b, mat * batch) || hipMalloc(&c, mat * batch)) return 1;
  (void)hipMemcpy(a, h.data(), mat * batch, hipMemcpyHostToDevice);
  (void)hipMemcpy(b, h.data(), mat * batch, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0, 0);
    if (mi355x::mat_mult_q7_launch(n, n, n, a, b, c, batch, 0) != hipSuccess) return 2;
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  static unsigned long long st[64][2][160];
  if (hipMemcpyFromSymbol(st, HIP_SYMBOL(mi355x::q7_stamp_buf), sizeof(st)) != hipSuccess) return 3;
  static unsigned long long rt[64][2][2];
  if (hipMemcpyFromSymbol(rt, HIP_SYMBOL(mi355x::q7_stamp_real), sizeof(rt)) != hipSuccess) return 4;
  // "real": s_memrealtime (100 MHz) at the first / last stamp of group 0, to calibrate the s_memtime ticks
  printf("{\"ms\": %.5f, \"batch\": %d, \"real\": [", ms, batch);
  for (int w = 0; w < 64; ++w) printf("%s[%llu,%llu]", w ? "," : "", rt[w][0][0], rt[w][0][1]);
  printf("], \"stamps\": [");
  for (int w = 0; w < 64; ++w) {
    printf("%s[", w ? "," : "");
    for (int g = 0; g < 2; ++g) {
      printf("%s[", g ? "," : "");
      for (int k = 0; k < 160; ++k) printf("%s%llu", k ? "," : "", st[w][g][k]);
      printf("]");
    }
    printf("]");
  }
  printf("]}\n");
  return 0;
}
