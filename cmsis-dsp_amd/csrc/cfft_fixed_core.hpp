// Fixed-point CFFT building blocks shared by the q31 / q15 kernels (cfft_fixed.hip,
// cfft_fixed_r16.hip): the reference's radix-4 butterflies with its exact integer semantics
// (q31: arm_cfft_radix4_q31.c; q15: arm_cfft_radix4_q15.c scalar branches), the packed
// 16-bit q15 restatement, element access and buffer-resource I/O.
#pragma once
#include "common.hpp"

namespace mi355x {

// ------------------------------------------------------------------ q31 butterflies
// stage kinds: 0 = first (>>4 in, <<1 out), 1 = middle (>>2 / >>1), 2 = last (no twiddle)
template <bool INV, int KIND>
__device__ __forceinline__ void bfly_q31(int2& a, int2& b, int2& c, int2& d,
                                         int2 w1, int2 w2, int2 w3) {
  if constexpr (KIND == 2) {
    // arm_cfft_radix4_q31.c:411-464 (fwd) / :774-826 (inv)
    const int32_t xa = a.x, ya = a.y, xb = b.x, yb = b.y, xc = c.x, yc = c.y, xd = d.x, yd = d.y;
    a = make_int2(wadd(wadd(xa, xb), wadd(xc, xd)), wadd(wadd(ya, yb), wadd(yc, yd)));
    b = make_int2(wsub(wadd(wsub(xa, xb), xc), xd), wsub(wadd(wsub(ya, yb), yc), yd));
    if (!INV) {
      c = make_int2(wsub(wsub(wadd(xa, yb), xc), yd), wadd(wsub(wsub(ya, xb), yc), xd));
      d = make_int2(wadd(wsub(wsub(xa, yb), xc), yd), wsub(wsub(wadd(ya, xb), yc), xd));
    } else {
      c = make_int2(wadd(wsub(wsub(xa, yb), xc), yd), wsub(wsub(wadd(ya, xb), yc), xd));
      d = make_int2(wsub(wsub(wadd(xa, yb), xc), yd), wadd(wsub(wsub(ya, xb), yc), xd));
    }
    return;
  } else {
    // first stage: arm_cfft_radix4_q31.c:187-282; middle: :297-395 (inverse :555-756)
    constexpr int SH_IN = KIND == 0 ? 4 : 0;
    const int32_t xa = a.x >> SH_IN, ya = a.y >> SH_IN, xb = b.x >> SH_IN, yb = b.y >> SH_IN;
    const int32_t xc = c.x >> SH_IN, yc = c.y >> SH_IN, xd = d.x >> SH_IN, yd = d.y >> SH_IN;
    int32_t r1 = wadd(xa, xc), r2 = wsub(xa, xc);
    int32_t t1 = wadd(xb, xd);
    int32_t s1 = wadd(ya, yc), s2 = wsub(ya, yc);
    int32_t oax = wadd(r1, t1);
    r1 = wsub(r1, t1);
    int32_t t2 = wadd(yb, yd);
    int32_t oay = wadd(s1, t2);
    s1 = wsub(s1, t2);
    t1 = wsub(yb, yd);
    t2 = wsub(xb, xd);
    int32_t obx, oby, ocx, ocy, odx, ody;
    auto fin = [](int32_t v) { return KIND == 0 ? wshl(v, 1) : (v >> 1); };
    if (!INV) {
      obx = fin(wadd(mulhi(r1, w2.x), mulhi(s1, w2.y)));
      oby = fin(wsub(mulhi(s1, w2.x), mulhi(r1, w2.y)));
      r1 = wadd(r2, t1); r2 = wsub(r2, t1);
      s1 = wsub(s2, t2); s2 = wadd(s2, t2);
      ocx = fin(wadd(mulhi(r1, w1.x), mulhi(s1, w1.y)));
      ocy = fin(wsub(mulhi(s1, w1.x), mulhi(r1, w1.y)));
      odx = fin(wadd(mulhi(r2, w3.x), mulhi(s2, w3.y)));
      ody = fin(wsub(mulhi(s2, w3.x), mulhi(r2, w3.y)));
    } else {
      obx = fin(wsub(mulhi(r1, w2.x), mulhi(s1, w2.y)));
      oby = fin(wadd(mulhi(s1, w2.x), mulhi(r1, w2.y)));
      r1 = wsub(r2, t1); r2 = wadd(r2, t1);
      s1 = wadd(s2, t2); s2 = wsub(s2, t2);
      ocx = fin(wsub(mulhi(r1, w1.x), mulhi(s1, w1.y)));
      ocy = fin(wadd(mulhi(s1, w1.x), mulhi(r1, w1.y)));
      odx = fin(wsub(mulhi(r2, w3.x), mulhi(s2, w3.y)));
      ody = fin(wadd(mulhi(s2, w3.x), mulhi(r2, w3.y)));
    }
    if (KIND == 1) { oax >>= 2; oay >>= 2; }
    // xc' goes to i1 and xb' to i2 (the reference's output swap -> bit-reversed order)
    a = make_int2(oax, oay); b = make_int2(obx, oby); c = make_int2(ocx, ocy); d = make_int2(odx, ody);
  }
}

// ------------------------------------------------------------------ q15 butterflies
// Values live in int32 registers but carry the reference's q15_t storage semantics.
__device__ __forceinline__ int32_t t16(int32_t v) { return (int32_t)(int16_t)v; }          // store to q15_t
__device__ __forceinline__ int32_t q15mul(int32_t p, int32_t q, int32_t r, int32_t s, bool plus) {
  // (q15_t)((p*q +/- r*s) >> 16) with int32 wrap of the sum
  uint32_t u = (uint32_t)(p * q);
  uint32_t v = (uint32_t)(r * s);
  return t16((int32_t)(plus ? u + v : u - v) >> 16);
}

template <bool INV, int KIND>
__device__ __forceinline__ void bfly_q15(int2& a, int2& b, int2& c, int2& d,
                                         int2 w1, int2 w2, int2 w3) {
  constexpr int SH = KIND == 0 ? 2 : 0;
  int32_t T0 = a.x >> SH, T1 = a.y >> SH;
  int32_t S0 = c.x >> SH, S1 = c.y >> SH;
  int32_t R0 = ssat16(T0 + S0), R1 = ssat16(T1 + S1);
  S0 = ssat16(T0 - S0); S1 = ssat16(T1 - S1);
  T0 = b.x >> SH; T1 = b.y >> SH;
  int32_t U0 = d.x >> SH, U1 = d.y >> SH;
  T0 = ssat16(T0 + U0); T1 = ssat16(T1 + U1);
  int2 oa, ob, oc, od;
  if (KIND == 1) oa = make_int2(t16(((R0 >> 1) + (T0 >> 1)) >> 1), t16(((R1 >> 1) + (T1 >> 1)) >> 1));
  else           oa = make_int2(t16((R0 >> 1) + (T0 >> 1)), t16((R1 >> 1) + (T1 >> 1)));
  if (KIND == 0) { R0 = ssat16(R0 - T0); R1 = ssat16(R1 - T1); }
  else           { R0 = t16((R0 >> 1) - (T0 >> 1)); R1 = t16((R1 >> 1) - (T1 >> 1)); }
  if (KIND == 2) {
    ob = make_int2(R0, R1);
  } else if (!INV) {
    ob = make_int2(q15mul(w2.x, R0, w2.y, R1, true), q15mul(-w2.y, R0, w2.x, R1, true));
  } else {
    ob = make_int2(q15mul(w2.x, R0, w2.y, R1, false), q15mul(w2.y, R0, w2.x, R1, true));
  }
  T0 = b.x >> SH; T1 = b.y >> SH;
  U0 = d.x >> SH; U1 = d.y >> SH;
  T0 = ssat16(T0 - U0); T1 = ssat16(T1 - U1);
  if (KIND == 2) {
    if (!INV) {
      oc = make_int2(t16((S0 >> 1) + (T1 >> 1)), t16((S1 >> 1) - (T0 >> 1)));
      od = make_int2(t16((S0 >> 1) - (T1 >> 1)), t16((S1 >> 1) + (T0 >> 1)));
    } else {
      oc = make_int2(t16((S0 >> 1) - (T1 >> 1)), t16((S1 >> 1) + (T0 >> 1)));
      od = make_int2(t16((S0 >> 1) + (T1 >> 1)), t16((S1 >> 1) - (T0 >> 1)));
    }
  } else {
    int32_t nR0, nR1, nS0, nS1;
    if (KIND == 0) {
      if (!INV) { nR0 = ssat16(S0 - T1); nR1 = ssat16(S1 + T0); nS0 = ssat16(S0 + T1); nS1 = ssat16(S1 - T0); }
      else      { nR0 = ssat16(S0 + T1); nR1 = ssat16(S1 - T0); nS0 = ssat16(S0 - T1); nS1 = ssat16(S1 + T0); }
    } else {
      if (!INV) { nR0 = t16((S0 >> 1) - (T1 >> 1)); nR1 = t16((S1 >> 1) + (T0 >> 1));
                  nS0 = t16((S0 >> 1) + (T1 >> 1)); nS1 = t16((S1 >> 1) - (T0 >> 1)); }
      else      { nR0 = t16((S0 >> 1) + (T1 >> 1)); nR1 = t16((S1 >> 1) - (T0 >> 1));
                  nS0 = t16((S0 >> 1) - (T1 >> 1)); nS1 = t16((S1 >> 1) + (T0 >> 1)); }
    }
    if (!INV) {
      oc = make_int2(q15mul(w1.y, nS1, w1.x, nS0, true), q15mul(-w1.y, nS0, w1.x, nS1, true));
      od = make_int2(q15mul(w3.y, nR1, w3.x, nR0, true), q15mul(-w3.y, nR0, w3.x, nR1, true));
    } else {
      oc = make_int2(q15mul(w1.x, nS0, w1.y, nS1, false), q15mul(w1.y, nS0, w1.x, nS1, true));
      od = make_int2(q15mul(w3.x, nR0, w3.y, nR1, false), q15mul(w3.y, nR0, w3.x, nR1, true));
    }
  }
  a = oa; b = ob; c = oc; d = od;
}

// ------------------------------------------------------------------ q15 butterflies, packed
// (restated from bfly_q15, see cfft_q15_4096_pk_kernel for the mapping)
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 pk(uint32_t u) { return __builtin_bit_cast(s16x2, u); }
__device__ __forceinline__ uint32_t upk(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ s16x2 pk_sat_add(s16x2 a, s16x2 b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ s16x2 pk_sat_sub(s16x2 a, s16x2 b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ s16x2 pk_swap(s16x2 v) { return __builtin_shufflevector(v, v, 1, 0); }

struct TwP { s16x2 p, q; };      // the two packed twiddle words of one complex product
template <bool INV> __device__ __forceinline__ TwP twp(short2 w) {
  const short nx = (short)~w.y;   // ~w.y: forward imaginary / inverse real difference term
  if (!INV) return TwP{s16x2{w.x, w.y}, s16x2{nx, w.x}};
  return TwP{s16x2{w.x, nx}, s16x2{w.y, w.x}};
}
// forward: {hi(w.x R0 + w.y R1), hi(w.x R1 - w.y R0)}; inverse: {hi(w.x R0 - w.y R1),
// hi(w.y R0 + w.x R1)} -- bfly_q15's q15mul pairs.
template <bool INV> __device__ __forceinline__ s16x2 cmul_pk(TwP w, s16x2 R) {
  const uint32_t u = upk(R);
  int32_t x, y;
  if (!INV) {
    x = __builtin_amdgcn_sdot2(w.p, R, 0, false);
    y = __builtin_amdgcn_sdot2(w.q, R, (int32_t)(int16_t)u, false);
  } else {
    x = __builtin_amdgcn_sdot2(w.p, R, (int32_t)u >> 16, false);
    y = __builtin_amdgcn_sdot2(w.q, R, 0, false);
  }
  return pk(__builtin_amdgcn_perm((uint32_t)y, (uint32_t)x, 0x07060302u));
}

template <bool INV, int KIND>
__device__ __forceinline__ void bfly_pk(s16x2& a, s16x2& b, s16x2& c, s16x2& d, TwP w1, TwP w2, TwP w3) {
  constexpr short SH = KIND == 0 ? 2 : 0;
  const s16x2 A = a >> SH, B = b >> SH, Cc = c >> SH, D = d >> SH;
  s16x2 R = pk_sat_add(A, Cc), S = pk_sat_sub(A, Cc), T = pk_sat_add(B, D);
  const s16x2 Rh = R >> (short)1, Th = T >> (short)1;
  const s16x2 oa = KIND == 1 ? (s16x2)((Rh + Th) >> (short)1) : (s16x2)(Rh + Th);
  R = KIND == 0 ? pk_sat_sub(R, T) : (s16x2)(Rh - Th);
  const s16x2 ob = KIND == 2 ? R : cmul_pk<INV>(w2, R);
  T = pk_sat_sub(B, D);
  s16x2 nR, nS;                          // forward nR = {S0 - T1, S1 + T0}, nS = {S0 + T1, S1 - T0}
  if constexpr (KIND == 0) {
    const s16x2 Ts = pk_swap(T);
    const s16x2 add = pk_sat_add(S, Ts), sub = pk_sat_sub(S, Ts);   // {S0+T1, S1+T0}, {S0-T1, S1-T0}
    const s16x2 r = __builtin_shufflevector(sub, add, 0, 3), s = __builtin_shufflevector(add, sub, 0, 3);
    nR = INV ? s : r; nS = INV ? r : s;
  } else {
    const s16x2 Sh = S >> (short)1;
    const s16x2 Tn = pk_swap(T >> (short)1) * s16x2{1, -1};          // {T1', -T0'} (|T'| < 2^14)
    const s16x2 r = Sh - Tn, s = Sh + Tn;
    nR = INV ? s : r; nS = INV ? r : s;
  }
  if constexpr (KIND == 2) { c = nS; d = nR; }
  else { c = cmul_pk<INV>(w1, nS); d = cmul_pk<INV>(w3, nR); }
  a = oa; b = ob;
}


// ------------------------------------------------------------------ element access
template <typename T> struct Fx;
template <> struct Fx<int32_t> {   // q31: complex = int2 in LDS and HBM
  using C = int2;
  using S = int;
  __device__ static int2 ld(const C* p) { return *p; }
  __device__ static void st(C* p, int2 v) { *p = v; }
};
template <> struct Fx<int16_t> {   // q15: complex = short2
  using C = short2;
  using S = short;
  __device__ static int2 ld(const C* p) { short2 s = *p; return make_int2(s.x, s.y); }
  __device__ static void st(C* p, int2 v) { *p = make_short2((short)v.x, (short)v.y); }
};

// the RFFT inverse's arm_shift_<q31|q15>(pDst, 1, ...) on a complex word pair
template <typename T> __device__ __forceinline__ int2 sat_shl1(int2 v) {
  if constexpr (sizeof(T) == 4) return make_int2(sat_shl1_q31(v.x), sat_shl1_q31(v.y));
  else return make_int2(sat_shl1_q15(v.x), sat_shl1_q15(v.y));
}

template <typename T, bool INV, int KIND>
__device__ __forceinline__ void bfly(int2& a, int2& b, int2& c, int2& d, int2 w1, int2 w2, int2 w3) {
  if constexpr (sizeof(T) == 4) bfly_q31<INV, KIND>(a, b, c, d, w1, w2, w3);
  else bfly_q15<INV, KIND>(a, b, c, d, w1, w2, w3);
}

// Global I/O through a buffer resource per transform (gfx9 raw buffer, dword 3 = 0x00020000):
// one VGPR byte offset per lane, the (a, b) element offsets as SGPR soffsets, so no 64-bit
// address arithmetic per access.  MI355X_FX_NT = 2 marks the streamed words nontemporal.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fx_rsrc(const void* p, uint32_t bytes) { return buf_rsrc(p, bytes); }
template <typename C> struct FxIO;
template <> struct FxIO<int2> {
  __device__ static int2 ld(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    const v2i v = __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, MI355X_FX_NT);
    return make_int2(v.x, v.y);
  }
  __device__ static void st(__amdgpu_buffer_rsrc_t r, int vo, int so, int2 x) {
    __builtin_amdgcn_raw_buffer_store_b64(v2i{x.x, x.y}, r, vo, so, MI355X_FX_NT);
  }
};
template <> struct FxIO<short2> {
  __device__ static short2 ld(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(short2, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, MI355X_FX_NT));
  }
  __device__ static void st(__amdgpu_buffer_rsrc_t r, int vo, int so, short2 x) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, x), r, vo, so, MI355X_FX_NT);
  }
};

// Work mapping of the N = 4096 kernels (q31: MI355X_FX_T, q15: MI355X_FXQ15_T).  T = 0:
// persistent grid walking the batch with stride = grid; T > 0: workgroup b takes the T
// consecutive transforms bT .. bT+T-1 (grid = batch / T; the prefetch runs inside the run).
// Measured at 2^20 transforms (profiles/r02/variants_fx4096/): T = 8 ran at the ceiling of
// the kernels' own access pattern (a probe build with the butterflies removed) on
// every box, while the persistent walk ranged 316-354 Gsamples/s (q31) from box to box.
struct FxWalk { uint32_t begin, end, step; };
template <uint32_t kT> __device__ __forceinline__ FxWalk fx_walk(uint32_t batch) {
  if constexpr (kT == 0) return FxWalk{blockIdx.x, batch, gridDim.x};
  const uint32_t b = blockIdx.x * kT;
  return FxWalk{b, min(batch, b + kT), 1u};
}
template <uint32_t kT> __host__ __forceinline__ int fx_grid(const void* k, uint32_t batch) {
  return kT ? (int)((batch + kT - 1) / kT) : persistent_grid(k, 256, 0, batch);
}


// ------------------------------------------------------------------ LDS-resident transform
// One transform of N complex at x in LDS, N/16 lanes (`lane`) per transform, every radix-4
// stage an LDS -> VGPR -> LDS pass with 4 butterflies per lane; the whole workgroup calls it
// together (stages are separated by __syncthreads).  Output in x in bit-reversed order; for
// the radix4by2 sizes the reference's final "<<1" post-pass is left to the caller (fx_by2_out).
// Used by the generic batched kernel (cfft_fixed.hip) and the fused MFCC kernels.
template <int N> struct PlanFx {
  static constexpr bool BY2 = (Log2<N>::v & 1) != 0;       // 32,128,512,2048
  static constexpr int M = BY2 ? N / 2 : N;                 // radix-4 length
  static constexpr int STAGES = Log2<M>::v / 2;
  static constexpr int LPT = N / 16;
  static constexpr int TPB = kBlock / LPT;
};


template <typename T, int N, bool INV>
__device__ __forceinline__ void radix4_stages(typename Fx<T>::C* x, const typename Fx<T>::C* __restrict__ tw,
                                              int lane) {
  using P = PlanFx<N>;
  using F = Fx<T>;
  constexpr int M = P::M;
  constexpr int mod0 = P::BY2 ? 2 : 1;
#pragma unroll
  for (int s = 0; s < P::STAGES; ++s) {
    const int n1 = M >> (2 * s), n2 = n1 >> 2;
    const int mod = mod0 << (2 * s);
#pragma unroll
    for (int r = 0; r < (N / 4) / P::LPT; ++r) {
      const int bi = lane + r * P::LPT;
      const int c = bi / (M / 4), rr = bi % (M / 4);
      const int j = rr % n2, q = rr / n2;
      typename F::C* p = x + c * M + q * n1 + j;
      if constexpr (sizeof(T) == 2 && MI355X_FX_Q15_PACKED) {
        uint32_t* pu = reinterpret_cast<uint32_t*>(p);
        s16x2 A = pk(pu[0]), B = pk(pu[n2]), C = pk(pu[2 * n2]), D = pk(pu[3 * n2]);
        if (s == P::STAGES - 1) {
          const TwP z{};
          bfly_pk<INV, 2>(A, B, C, D, z, z, z);
        } else {
          const int ia = j * mod;
          const TwP w1 = twp<INV>(tw[ia]), w2 = twp<INV>(tw[2 * ia]), w3 = twp<INV>(tw[3 * ia]);
          if (s == 0) bfly_pk<INV, 0>(A, B, C, D, w1, w2, w3);
          else        bfly_pk<INV, 1>(A, B, C, D, w1, w2, w3);
        }
        pu[0] = upk(A); pu[n2] = upk(B); pu[2 * n2] = upk(C); pu[3 * n2] = upk(D);
        continue;
      }
      int2 A = F::ld(p), B = F::ld(p + n2), C = F::ld(p + 2 * n2), D = F::ld(p + 3 * n2);
      if (s == P::STAGES - 1) {
        bfly<T, INV, 2>(A, B, C, D, int2{}, int2{}, int2{});
      } else {
        const int ia = j * mod;
        const int2 w1 = F::ld(tw + ia), w2 = F::ld(tw + 2 * ia), w3 = F::ld(tw + 3 * ia);
        if (s == 0) bfly<T, INV, 0>(A, B, C, D, w1, w2, w3);
        else        bfly<T, INV, 1>(A, B, C, D, w1, w2, w3);
      }
      F::st(p, A); F::st(p + n2, B); F::st(p + 2 * n2, C); F::st(p + 3 * n2, D);
    }
    __syncthreads();
  }
}

template <typename T, int N, bool INV>
__device__ __forceinline__ void cfft_fx_lds_body(typename Fx<T>::C* x, const typename Fx<T>::C* __restrict__ tw,
                                                 int lane) {
  using P = PlanFx<N>;
  using F = Fx<T>;
  if constexpr (P::BY2) {
    // radix-2 pre-pass: arm_cfft_q31.c:774-794 / :835-855, arm_cfft_q15.c:782-800 / :881-899
    constexpr int H = N / 2;
#pragma unroll
    for (int it = 0; it < H / P::LPT; ++it) {
      const int i = lane + it * P::LPT;
      const int2 w = F::ld(tw + i);
      int2 a = F::ld(x + i), b = F::ld(x + i + H);
      if constexpr (sizeof(T) == 4) {
        const int32_t xt = wsub(a.x >> 2, b.x >> 2);
        const int32_t yt = wsub(a.y >> 2, b.y >> 2);
        F::st(x + i, make_int2(wadd(a.x >> 2, b.x >> 2), wadd(b.y >> 2, a.y >> 2)));
        int32_t p0 = mult_R(xt, w.x), p1 = mult_R(yt, w.x);
        if (!INV) { p0 = multAcc_R(p0, yt, w.y); p1 = multSub_R(p1, xt, w.y); }
        else      { p0 = multSub_R(p0, yt, w.y); p1 = multAcc_R(p1, xt, w.y); }
        F::st(x + i + H, make_int2(wshl(p0, 1), wshl(p1, 1)));
      } else {
        const int32_t xt = t16((a.x >> 1) - (b.x >> 1));
        const int32_t yt = t16((a.y >> 1) - (b.y >> 1));
        F::st(x + i, make_int2(((a.x >> 1) + (b.x >> 1)) >> 1, ((b.y >> 1) + (a.y >> 1)) >> 1));
        const int32_t xc = t16((xt * w.x) >> 16), ys = t16((yt * w.y) >> 16);
        const int32_t yc = t16((yt * w.x) >> 16), xs = t16((xt * w.y) >> 16);
        if (!INV) F::st(x + i + H, make_int2(t16(xc + ys), t16(yc - xs)));
        else      F::st(x + i + H, make_int2(t16(xc - ys), t16(yc + xs)));
      }
    }
    __syncthreads();
  }

  radix4_stages<T, N, INV>(x, tw, lane);
}
// the radix4by2 post-pass (arm_cfft_q31.c:796-812 "<< 1", arm_cfft_q15.c:810-827) of one word
template <typename T, int N>
__device__ __forceinline__ int2 fx_by2_out(int2 v) {
  if constexpr (PlanFx<N>::BY2) {
    if constexpr (sizeof(T) == 4) return make_int2(wshl(v.x, 1), wshl(v.y, 1));
    else return make_int2(t16(v.x << 1), t16(v.y << 1));
  }
  return v;
}

}  // namespace mi355x
