// In-kernel phase timestamps of the arm_fir_q15 i8-MFMA kernel (fir_mfma.hip, MI355X_FIR_STAMP):
// s_memtime at the loop top (0), after the first barrier (1), after staging (2), after the second
// barrier (3), after issuing the next window's loads (4), after the MFMAs + output arithmetic (5)
// and after the stores (6), for the first 64 items of workgroups 0-63 (wave 0), on the bench shape
// (128 taps x 4096 x 2^16).  Prints {"ms": ..., "stamps": [wg][item][event]}; tools/probes/fir_stamps.py.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMI355X_FIR_STAMP=1 \
//          tools/probes/fir_stamps.hip -o tools/probes/fir_stamps
#include "../../cmsis-dsp_amd/csrc/fir_mfma.hip"
#include <stdio.h>
#include <vector>

int main() {
  const int T = 128;
  const uint32_t B = 4096, batch = 1u << 16;
  std::vector<int16_t> h((size_t)B * batch), c(T), hi((size_t)(T - 1) * batch, 0);
  unsigned s = 12345u;
  for (auto& v : h) { s = s * 1664525u + 1013904223u; v = (int16_t)(s >> 16); }
  for (auto& v : c) { s = s * 1664525u + 1013904223u; v = (int16_t)(s >> 16); }
  int16_t *src, *dst, *coef, *hist;
  if (hipMalloc(&src, h.size() * 2) || hipMalloc(&dst, h.size() * 2) || hipMalloc(&coef, T * 2) ||
      hipMalloc(&hist, hi.size() * 2))
    return 1;
  (void)hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(coef, c.data(), T * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(hist, hi.data(), hi.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0, 0);
    if (!mi355x::fir_q15_mfma_launch(coef, T, src, dst, B, batch, hist, 0)) return 2;
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  static unsigned long long st[64][64][8];
  if (hipMemcpyFromSymbol(st, HIP_SYMBOL(mi355x::fir_stamp_buf), sizeof(st)) != hipSuccess) return 3;
  printf("{\"ms\": %.5f, \"stamps\": [", ms);
  for (int w = 0; w < 64; ++w) {
    printf("%s[", w ? "," : "");
    for (int k = 0; k < 64; ++k) {
      printf("%s[", k ? "," : "");
      for (int e = 0; e < 8; ++e) printf("%s%llu", e ? "," : "", st[w][k][e]);
      printf("]");
    }
    printf("]");
  }
  printf("]}\n");
  return 0;
}
