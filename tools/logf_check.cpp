// Exhaustive check: mi355x::host_logf (cmsis-dsp_amd/csrc/host_logf.hpp, the device logf of
// the MFCC f32 kernels, compiled here on the host from the same source) equals the host libm
// logf on all 2^32 float inputs (NaN results compared as NaN).  ~2 minutes on one core.
//   g++ -O2 -std=c++17 -ffp-contract=off tools/logf_check.cpp -o /tmp/logf_check && /tmp/logf_check
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../cmsis-dsp_amd/csrc/host_logf.hpp"

int main() {
  uint64_t bad = 0;
  for (uint64_t u = 0; u < (1ull << 32); ++u) {
    float x, a, b;
    const uint32_t w = (uint32_t)u;
    std::memcpy(&x, &w, 4);
    a = logf(x);
    b = mi355x::host_logf(x);
    uint32_t ua, ub;
    std::memcpy(&ua, &a, 4);
    std::memcpy(&ub, &b, 4);
    if (ua != ub && !(std::isnan(a) && std::isnan(b)) && bad++ < 8) std::printf("x=%a libm=%a mine=%a\n", x, a, b);
  }
  std::printf("host_logf vs libm logf: %llu mismatches over 2^32 inputs\n", (unsigned long long)bad);
  return bad != 0;
}
