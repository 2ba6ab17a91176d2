// ORACLE — test infrastructure only.  Compares the host libm logf with the product's device
// restatement of glibc 2.35's __logf_fma (cmsis-dsp_amd/csrc/host_logf.hpp, compiled here from
// the same source) on a strided sample of all 2^32 float inputs.  MFCC f32 is bit-exact against
// the reference build only when they agree (the reference calls the host logf,
// Source/FastMathFunctions/arm_vlog_f32.c:110); tests/mfcc_cfg.py::host_libm_status() uses this
// to tell "libm differs" from a parity failure.  tools/logf_check.cpp is the exhaustive form.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../cmsis-dsp_amd/csrc/host_logf.hpp"

extern "C" uint64_t logf_probe_mismatches(uint32_t stride, uint32_t offset) {
  uint64_t bad = 0;
  for (uint64_t u = offset; u < (1ull << 32); u += stride) {
    const uint32_t w = (uint32_t)u;
    float x, a, b;
    std::memcpy(&x, &w, 4);
    a = logf(x);
    b = mi355x::host_logf(x);
    uint32_t ua, ub;
    std::memcpy(&ua, &a, 4);
    std::memcpy(&ub, &b, 4);
    if (ua != ub && !(std::isnan(a) && std::isnan(b))) ++bad;
  }
  return bad;
}
