// logf as the reference's host build computes it: glibc 2.35's logf (the table-driven
// algorithm of sysdeps/ieee754/flt-32/e_logf.c, Arm optimized-routines; x86-64 selects the
// FMA-compiled instance __logf_fma on CPUs with FMA/AVX2, which this restates operation for
// operation).  The reference's only libm call on the MFCC path is this logf
// (Source/FastMathFunctions/arm_vlog_f32.c:110, from arm_mfcc_f32.c:163), so with it the
// device MFCC f32 is bit-identical to the host build.
//
// Algorithm: x = 2^k z with z in [0x3f330000, 2 * 0x3f330000) exact; the 16 subintervals of
// that range have centres c_i with tabulated (1/c_i, log c_i) in double;
//   r = z / c_i - 1 (one fma), log x = log1p(r) + log c_i + k ln2, log1p by a cubic in r.
// Constants: the pinned glibc's __logf_data (16 x {invc, logc}, ln2, poly[3]), read from the
// installed libm by tools/logf_table.py; tools/logf_check.cpp proves this restatement equal to the host
// logf on all 2^32 inputs (NaN payloads aside).
#pragma once
#include <stdint.h>

// Also compiled on the host by tools/logf_check.cpp (g++), which checks this exact source.
#ifdef __HIPCC__
#define MI355X_LOGF_FN __device__ __forceinline__
#define MI355X_LOGF_TAB static __constant__ const
#else
#define MI355X_LOGF_FN static inline
#define MI355X_LOGF_TAB static const
#endif

namespace mi355x {

struct HostLogfTab { double invc, logc; };

MI355X_LOGF_TAB HostLogfTab kHostLogfTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};

MI355X_LOGF_FN float host_logf(float x) {
  constexpr double kLn2 = 0x1.62e42fefa39efp-1;
  constexpr double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
  uint32_t ix = __builtin_bit_cast(uint32_t, x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {       // x < 0x1p-126, inf or nan
    if (ix * 2 == 0) return -__builtin_inff();
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
    ix = __builtin_bit_cast(uint32_t, x * 0x1p23f);          // subnormal: normalise
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) & 15u);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const HostLogfTab t = kHostLogfTab[i];
  const double z = (double)__builtin_bit_cast(float, iz);
  const double r = __builtin_fma(z, t.invc, -1.0);
  const double y0 = __builtin_fma((double)k, kLn2, t.logc);
  const double r2 = r * r;
  double y = __builtin_fma(A1, r, A2);
  y = __builtin_fma(A0, r2, y);
  y = __builtin_fma(y, r2, y0 + r);
  return (float)y;
}

}  // namespace mi355x
