// Shared f32 CFFT building blocks (device code): the reference's radix-8 butterfly, the
// radix8by2 / radix8by4 first passes and the radix-8 stage loop on transforms held in LDS.
// Used by the batched CFFT (cfft_f32.hip) and by the fused MFCC kernel (mfcc_f32.hip), so
// both run the identical, bit-exact arithmetic.  Include after common.hpp with
// `#pragma clang fp contract(off)` in effect.
#pragma once
#include "common.hpp"

#pragma clang fp contract(off)

namespace mi355x {

constexpr float kC81 = 0.70710678118f;  // arm_cfft_radix8_f32.c:68

// --- radix-8 DIF butterfly, arm_cfft_radix8_f32.c:188-281 (twiddled) and :87-138 (j==0).
// v[m] = x[i1 + m*n2].  The j==0 group stores exactly the values the twiddled groups feed
// to their twiddle multiply, so the butterfly is: untwiddled core, then (optionally) the
// reference's complex multiply (co*r + si*s, co*s - si*r) on outputs 1..7.
__device__ __forceinline__ void r8_core(float2 (&v)[8]) {
  float r1, r2, r3, r4, r5, r6, r7, r8v, t1, t2;
  float s1, s2, s3, s4, s5, s6, s7, s8;
  r1 = v[0].x + v[4].x;  r5 = v[0].x - v[4].x;
  r2 = v[1].x + v[5].x;  r6 = v[1].x - v[5].x;
  r3 = v[2].x + v[6].x;  r7 = v[2].x - v[6].x;
  r4 = v[3].x + v[7].x;  r8v = v[3].x - v[7].x;
  t1 = r1 - r3;  r1 = r1 + r3;
  r3 = r2 - r4;  r2 = r2 + r4;
  const float o0x = r1 + r2;
  r2 = r1 - r2;
  s1 = v[0].y + v[4].y;  s5 = v[0].y - v[4].y;
  s2 = v[1].y + v[5].y;  s6 = v[1].y - v[5].y;
  s3 = v[2].y + v[6].y;  s7 = v[2].y - v[6].y;
  s4 = v[3].y + v[7].y;  s8 = v[3].y - v[7].y;
  t2 = s1 - s3;  s1 = s1 + s3;
  s3 = s2 - s4;  s2 = s2 + s4;
  r1 = t1 + s3;  t1 = t1 - s3;
  const float o0y = s1 + s2;
  s2 = s1 - s2;
  s1 = t2 - r3;  t2 = t2 + r3;
  const float2 o4 = make_float2(r2, s2), o2 = make_float2(r1, s1), o6 = make_float2(t1, t2);
  r1 = (r6 - r8v) * kC81;  r6 = (r6 + r8v) * kC81;
  s1 = (s6 - s8) * kC81;   s6 = (s6 + s8) * kC81;
  t1 = r5 - r1;  r5 = r5 + r1;
  r8v = r7 - r6; r7 = r7 + r6;
  t2 = s5 - s1;  s5 = s5 + s1;
  s8 = s7 - s6;  s7 = s7 + s6;
  r1 = r5 + s7;  r5 = r5 - s7;
  r6 = t1 + s8;  t1 = t1 - s8;
  s1 = s5 - r7;  s5 = s5 + r7;
  s6 = t2 - r8v; t2 = t2 + r8v;
  v[0] = make_float2(o0x, o0y);
  v[1] = make_float2(r1, s1); v[2] = o2; v[3] = make_float2(t1, t2); v[4] = o4;
  v[5] = make_float2(r6, s6); v[6] = o6; v[7] = make_float2(r5, s5);
}

// reference twiddle multiply: p1 = co*r, p2 = si*s, p3 = co*s, p4 = si*r -> (p1+p2, p3-p4)
__device__ __forceinline__ float2 twmul(float2 o, float2 c) {
  return make_float2(c.x * o.x + c.y * o.y, c.x * o.y - c.y * o.x);
}

template <bool TW>
__device__ __forceinline__ void r8(float2 (&v)[8], const float2* __restrict__ w) {
  r8_core(v);
  if (TW) {
#pragma unroll
    for (int m = 1; m < 8; ++m) v[m] = twmul(v[m], w[m - 1]);
  }
}

// lane-dependent j==0 without divergence: twiddle, then select (v_cndmask)
__device__ __forceinline__ void r8_sel(float2 (&v)[8], const float2 (&w)[7], bool tw) {
  r8_core(v);
#pragma unroll
  for (int m = 1; m < 8; ++m) {
    const float2 t = twmul(v[m], w[m - 1]);
    v[m] = make_float2(tw ? t.x : v[m].x, tw ? t.y : v[m].y);
  }
}

template <int N> struct PlanF32 {
  static constexpr int FIRST = (N == 16 || N == 128 || N == 1024) ? 2
                             : (N == 32 || N == 256 || N == 2048) ? 4 : 1;
  static constexpr int L = N / FIRST;              // length handed to the radix-8 core
  static constexpr int STAGES = Log2<L>::v / 3;    // radix-8 stages
  static constexpr int LPT = N / 16;               // lanes per transform
  static constexpr int TPB = kBlock / LPT;         // transforms per workgroup
};

// position (before bit reversal) that holds frequency k: inverse of the mixed-radix digit
// reversal [FIRST, 8, 8, ...] the reference tables encode (checked on the host).
template <int N> __device__ __forceinline__ int f32_src(int k) {
  constexpr int FIRST = PlanF32<N>::FIRST;
  int p = 0, rem = N;
  if (FIRST > 1) { rem /= FIRST; p += (k % FIRST) * rem; k /= FIRST; }
#pragma unroll
  for (int s = 0; s < PlanF32<N>::STAGES; ++s) { rem >>= 3; p += (k & 7) * rem; k >>= 3; }
  return p;
}

// Forward CFFT core of one length-N transform held in LDS (`x`, natural order in,
// digit-reversed order out: frequency k sits at x[f32_src<N>(k)]), computed by the LPT =
// N/16 lanes `lane` = 0..LPT-1 of its group.  Every thread of the workgroup must call it
// (it contains __syncthreads); the first pass and stages follow arm_cfft_f32.c:1263-1280.
// LDS image index of element i of a length-N transform: for N >= 512 (whole waves inside
// one transform) bits 1-4 are XORed with bits 4-7, which takes the radix-8 stages' strided
// patterns from 4-8-way bank conflicts down to 1-2 (bijective on every aligned 256-block;
// modelled over all stage access patterns).  Every LDS access to a
// transform image -- here and in the kernels that load / store it -- goes through swz<N>.
template <int N>
__device__ __forceinline__ int swz(int i) {
  if constexpr (N >= 512) return i ^ (((i >> 4) & 15) << 1);
  else return i;
}

template <int N>
__device__ __forceinline__ void cfft_f32_lds_fwd(float2* __restrict__ x, int lane, const float2* __restrict__ tw) {
  using P = PlanF32<N>;
#define XS(i) x[swz<N>(i)]
  // ---- first pass
  if constexpr (P::FIRST == 2) {
    // arm_cfft_radix8by2_f32, arm_cfft_f32.c:867-951
    constexpr int Q = N / 4, H = N / 2;
#pragma unroll
    for (int it = 0; it < Q / P::LPT; ++it) {
      const int k = lane + it * P::LPT;
      const float2 w = tw[k];
      float2 a = XS(k), b = XS(k + H), c = XS(k + Q), d = XS(k + H + Q);
      XS(k) = make_float2(a.x + b.x, a.y + b.y);
      float2 t2 = make_float2(a.x - b.x, a.y - b.y);
      XS(k + Q) = make_float2(c.x + d.x, c.y + d.y);
      float2 t4 = make_float2(d.x - c.x, d.y - c.y);
      XS(k + H) = make_float2(t2.x * w.x + t2.y * w.y, t2.y * w.x - t2.x * w.y);
      XS(k + H + Q) = make_float2(t4.x * w.y - t4.y * w.x, t4.y * w.y + t4.x * w.x);
    }
    __syncthreads();
  } else if constexpr (P::FIRST == 4) {
    // arm_cfft_radix8by4_f32, arm_cfft_f32.c:992-1188.  Work item w <= N/8: "top" row k=w
    // (k=0 untwiddled, k=N/8 the "middle" row); w > N/8: "bottom" row kb = Q - i.
    constexpr int Q = N / 4, E = N / 8;
#pragma unroll
    for (int it = 0; it < Q / P::LPT; ++it) {
      const int w = lane + it * P::LPT;
      if (w <= E) {
        const int k = w;
        float2 A = XS(k), B = XS(k + Q), C = XS(k + 2 * Q), D = XS(k + 3 * Q);
        float ap0 = A.x + C.x, as0 = A.x - C.x, ap1 = A.y + C.y, as1 = A.y - C.y;
        float2 t2 = make_float2(as0 + B.y - D.y, as1 - B.x + D.x);
        float2 t3 = make_float2(ap0 - B.x - D.x, ap1 - B.y - D.y);
        float2 t4 = make_float2(as0 - B.y + D.y, as1 + B.x - D.x);
        XS(k) = make_float2(ap0 + B.x + D.x, ap1 + B.y + D.y);
        if (k == 0) {
          XS(k + Q) = t2; XS(k + 2 * Q) = t3; XS(k + 3 * Q) = t4;
        } else {
          const float2 w2 = tw[k], w3 = tw[2 * k], w4 = tw[3 * k];
          XS(k + Q)     = make_float2(t2.x * w2.x + t2.y * w2.y, t2.y * w2.x - t2.x * w2.y);
          XS(k + 2 * Q) = make_float2(t3.x * w3.x + t3.y * w3.y, t3.y * w3.x - t3.x * w3.y);
          XS(k + 3 * Q) = make_float2(t4.x * w4.x + t4.y * w4.y, t4.y * w4.x - t4.x * w4.y);
        }
      } else {
        const int i = w - E, kb = Q - i;
        float2 A = XS(kb), B = XS(kb + Q), C = XS(kb + 2 * Q), D = XS(kb + 3 * Q);
        float ap1 = A.x + C.x, as1 = A.x - C.x, ap0 = A.y + C.y, as0 = A.y - C.y;
        float t22 = B.y - D.y + as1;
        float t23 = A.y - C.y - B.x + D.x;
        float t32 = ap1 - B.x - D.x;
        float t33 = ap0 - B.y - D.y;
        float t42 = B.y - D.y - as1;
        float t43 = D.x - B.x - as0;
        XS(kb) = make_float2(ap1 + B.x + D.x, ap0 + B.y + D.y);
        const float2 w2 = tw[i], w3 = tw[2 * i], w4 = tw[3 * i];
        XS(kb + Q)     = make_float2(t22 * w2.y + t23 * w2.x, t23 * w2.y - t22 * w2.x);
        XS(kb + 2 * Q) = make_float2(t33 * w3.y - t32 * w3.x, -t33 * w3.x - t32 * w3.y);
        XS(kb + 3 * Q) = make_float2(t42 * w4.y + t43 * w4.x, t43 * w4.y - t42 * w4.x);
      }
    }
    __syncthreads();
  }

  // ---- radix-8 stages (arm_cfft_radix8_f32.c:72-290), on FIRST sub-transforms of length L
  constexpr int L = P::L;
#pragma unroll
  for (int s = 0; s < P::STAGES; ++s) {
    const int n1 = L >> (3 * s), n2 = n1 >> 3;
    const int mod = P::FIRST << (3 * s);
#pragma unroll
    for (int r = 0; r < (N / 8) / P::LPT; ++r) {
      const int b = lane + r * P::LPT;
      const int c = b / (L / 8), rr = b % (L / 8);
      const int j = rr % n2, q = rr / n2;
      const int bi = c * L + q * n1 + j;
      float2 v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = XS(bi + m * n2);
      if (n2 == 1) {                    // last stage: every group is the j == 0 group
        r8<false>(v, nullptr);
      } else {
        // j == 0 lanes sit in every wave of the middle stages: twiddle everywhere and
        // select (tw[0] is a valid load) instead of running both branch bodies
        float2 w[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) w[m] = tw[(m + 1) * j * mod];
        r8_sel(v, w, j != 0);
      }
#pragma unroll
      for (int m = 0; m < 8; ++m) XS(bi + m * n2) = v[m];
    }
    __syncthreads();
  }

#undef XS
}

}  // namespace mi355x
