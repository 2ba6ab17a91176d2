// Batched complex FFT, q31 and q15, N = 256 / 512 / 1024 / 2048 — radix-16 register passes.
//
// Replaces the host scalar path of arm_cfft_q31 / arm_cfft_q15 (arm_cfft_q31.c:704-755,
// radix4by2 :763-881; arm_cfft_q15.c:671-722, radix4by2 scalar :782-827 / :881-926;
// arm_cfft_radix4_q31.c:153-473 / :524-834; arm_cfft_radix4_q15.c:572-970 / :1434-1813) and
// arm_bitreversal_32 / _16 with armBitRevIndexTable_fixed_N, for the reference's own tables.
// Same arithmetic as cfft_fx4096_kernel (cfft_fixed_core.hpp), generalised:
//   * P = N/16 threads per transform, 16 complex per thread, 256 / P transforms per workgroup;
//   * radix-4 stages fused in pairs (radix-16 register passes) with one LDS exchange between
//     passes; N = 2M with M = 4^K odd powers of two (512, 2048) run the radix4by2 pre-pass and
//     the first radix-4 stage of both halves in registers;
//   * thread t' of a transform holds, per pass (stages s, s+1 of the radix-4 length M, group
//     span L = M / 4^(s-1), strides d1 = L/4, d2 = L/16; j = t' mod d2, g = t' / d2):
//       e(a, b) = h M + g L + j + d2 a + d1 b            (stage s over b, stage s+1 over a)
//     with the first pass e = t' + P a + 4P b (coalesced loads) and the last pass on groups
//     g = rev(t') -- 16-element groups for two stages, or four 4-element groups for one --
//     so that the binary bit reversal of the output is free: every store instruction writes
//     consecutive bins across the threads (by2 halves interleave: h = t' & 1);
//   * LDS paddings s(e) = e + c1 (e >> k1) + c2 (e >> k2) and the per-transform stride found
//     by tools/fx_r16_plan.py: conflict free under the ds_read2_b64 / ds_write_b64 (q31) and
//     ds_read2_b32 / ds_write_b32 (q15) banking (N = 512: 1 extra cycle per 4 accesses);
//   * buffer-resource I/O per group of transforms (out-of-range loads return 0 and stores are
//     dropped, so a partial last group needs no bounds code), nontemporal; workgroup b takes
//     the MI355X_FXR_T consecutive groups, the next group's words prefetched into registers
//     under passes 2+, the loop entered after the first pass (see cfft_fx4096_kernel).
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"
#include "cfft_fixed_core.hpp"
#include "mfcc_fixed_ops.hpp"
#include "mfcc_fixed_post.hpp"
#include "rfft_fixed_split.hpp"

namespace mi355x {

// N = 32 / 64 / 128 stay on the generic kernel: with 2-8 threads per transform each load
// instruction would scatter over 32-8 transforms (measured on this kernel, bit-exact: q31
// 42 / 201 / 254 Gsamples/s against 342 / 334 / 324 for the generic kernel).

template <int N> struct R16 {
  static constexpr int LOG = Log2<N>::v;
  static constexpr bool BY2 = (LOG & 1) != 0;
  static constexpr int M = BY2 ? N / 2 : N;      // radix-4 length
  static constexpr int K = Log2<M>::v / 2;       // radix-4 stages
  static constexpr int P = N / 16;               // threads per transform
  static constexpr int PH = BY2 ? P / 2 : P;     // threads per radix-4 transform
  static constexpr int TPW = kBlock / P;         // transforms per workgroup
  static constexpr int MOD0 = BY2 ? 2 : 1;       // twiddle modifier of radix-4 stage 1
  // stages handled by the first pass, then at most one middle pass, then the last pass
  static constexpr int S_MID = BY2 ? 2 : 3;      // first stage of the middle pass
  static constexpr bool HAS_MID = S_MID + 1 < K; // a two-stage middle pass before the last
  static constexpr int S_LAST = HAS_MID ? S_MID + 2 : S_MID;
  static constexpr bool LAST2 = S_LAST + 1 == K; // last pass holds two stages
  static_assert(S_LAST == K || LAST2, "plan");
};
__device__ __forceinline__ constexpr int pow4(int s) { return 1 << (2 * s); }

template <int N, bool Q31> struct R16Pad;   // tools/fx_r16_plan.py
template <> struct R16Pad<32, true>    { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 34; };
template <> struct R16Pad<32, false>   { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 34; };
template <> struct R16Pad<64, true>    { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 68; };
template <> struct R16Pad<64, false>   { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 68; };
template <> struct R16Pad<128, true>   { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 136; };
template <> struct R16Pad<128, false>  { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 136; };
template <> struct R16Pad<256, true>   { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 271; };
template <> struct R16Pad<256, false>  { static constexpr int k1 = 3, c1 = 0, k2 = 4, c2 = 1, stride = 272; };
template <> struct R16Pad<512, true>   { static constexpr int k1 = 3, c1 = 0, k2 = 5, c2 = 1, stride = 527; };
template <> struct R16Pad<512, false>  { static constexpr int k1 = 3, c1 = 0, k2 = 5, c2 = 1, stride = 527; };
template <> struct R16Pad<1024, true>  { static constexpr int k1 = 6, c1 = 4, k2 = 8, c2 = 1, stride = 1087; };
template <> struct R16Pad<1024, false> { static constexpr int k1 = 5, c1 = 2, k2 = 9, c2 = 1, stride = 1087; };
template <> struct R16Pad<2048, true>  { static constexpr int k1 = 3, c1 = 0, k2 = 7, c2 = 1, stride = 2063; };
template <> struct R16Pad<2048, false> { static constexpr int k1 = 3, c1 = 0, k2 = 6, c2 = 1, stride = 2079; };

// Per-type register / LDS / global representations and the reference's butterflies.
template <typename T, bool INV> struct R16Ops;
template <bool INV> struct R16Ops<int32_t, INV> {
  using V = int2;     // value in registers
  using Tw = int2;    // twiddle operand
  using W = int2;     // LDS word
  using C = int2;     // global complex
  static __device__ __forceinline__ V from_w(W w) { return w; }
  static __device__ __forceinline__ W to_w(V v) { return v; }
  static __device__ __forceinline__ Tw tw(const C* t, int i) { return t[i]; }
  template <int KIND> static __device__ __forceinline__ void bf(V& a, V& b, V& c, V& d, Tw w1, Tw w2, Tw w3) {
    bfly<int32_t, INV, KIND>(a, b, c, d, w1, w2, w3);
  }
  static __device__ __forceinline__ V ld(__amdgpu_buffer_rsrc_t r, int vo, int so) { return FxIO<int2>::ld(r, vo, so); }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int vo, int so, V v) { FxIO<int2>::st(r, vo, so, v); }
  static __device__ __forceinline__ V by2_post(V v) { return make_int2(wshl(v.x, 1), wshl(v.y, 1)); }
  static __device__ __forceinline__ int2 unpack(V v) { return v; }
  static __device__ __forceinline__ V pack(int32_t x, int32_t y) { return make_int2(x, y); }
  static __device__ __forceinline__ V sat(V v) { return sat_shl1<int32_t>(v); }
  // radix4by2 pre-pass pair (arm_cfft_q31.c:774-794 forward, :835-855 inverse)
  static __device__ __forceinline__ void by2_pre(V& a, V& b, C w) {
    const int32_t xt = wsub(a.x >> 2, b.x >> 2), yt = wsub(a.y >> 2, b.y >> 2);
    a = make_int2(wadd(a.x >> 2, b.x >> 2), wadd(b.y >> 2, a.y >> 2));
    int32_t p0 = mult_R(xt, w.x), p1 = mult_R(yt, w.x);
    if (!INV) { p0 = multAcc_R(p0, yt, w.y); p1 = multSub_R(p1, xt, w.y); }
    else      { p0 = multSub_R(p0, yt, w.y); p1 = multAcc_R(p1, xt, w.y); }
    b = make_int2(wshl(p0, 1), wshl(p1, 1));
  }
};
template <bool INV> struct R16Ops<int16_t, INV> {
  using V = s16x2;    // one VGPR per complex (packed butterflies, cfft_fixed_core.hpp)
  using Tw = TwP;
  using W = uint32_t;
  using C = short2;
  static __device__ __forceinline__ V from_w(W w) { return pk(w); }
  static __device__ __forceinline__ W to_w(V v) { return upk(v); }
  static __device__ __forceinline__ Tw tw(const C* t, int i) { return twp<INV>(t[i]); }
  template <int KIND> static __device__ __forceinline__ void bf(V& a, V& b, V& c, V& d, Tw w1, Tw w2, Tw w3) {
    bfly_pk<INV, KIND>(a, b, c, d, w1, w2, w3);
  }
  static __device__ __forceinline__ V ld(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return pk((uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, vo, so, MI355X_FX_NT));
  }
  static __device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int vo, int so, V v) {
    __builtin_amdgcn_raw_buffer_store_b32((int)upk(v), r, vo, so, MI355X_FX_NT);
  }
  static __device__ __forceinline__ V by2_post(V v) { return v << (short)1; }        // t16(x << 1)
  static __device__ __forceinline__ int2 unpack(V v) { return make_int2(v.x, v.y); }
  static __device__ __forceinline__ V pack(int32_t x, int32_t y) { return s16x2{(short)x, (short)y}; }
  static __device__ __forceinline__ V sat(V v) { return pk_sat_add(v, v); }          // __SSAT(x << 1, 16)
  // radix4by2 pre-pass pair, scalar branch (arm_cfft_q15.c:782-800 forward, :881-899 inverse)
  static __device__ __forceinline__ void by2_pre(V& A, V& B, C w) {
    const int32_t ax = A.x, ay = A.y, bx = B.x, by = B.y;
    const int32_t xt = t16((ax >> 1) - (bx >> 1)), yt = t16((ay >> 1) - (by >> 1));
    A = s16x2{(short)(((ax >> 1) + (bx >> 1)) >> 1), (short)(((by >> 1) + (ay >> 1)) >> 1)};
    const int32_t xc = t16((xt * w.x) >> 16), ys = t16((yt * w.y) >> 16);
    const int32_t yc = t16((yt * w.x) >> 16), xs = t16((xt * w.y) >> 16);
    if (!INV) B = s16x2{(short)(xc + ys), (short)(yc - xs)};
    else      B = s16x2{(short)(xc - ys), (short)(yc + xs)};
  }
};

// PRE: the MFCC q31 / q15 front end on the RFFT's inner CFFT (arm_mfcc_q31.c:119-138, the N
// complex words of a transform being the frame's 2N real samples): the transform's P threads find
// max sat|x| (lane shuffles; an LDS pair for P = 128), scale and window their 32 words in
// registers (MqPre) before the first pass, and lane 0 leaves m in maxv[frame * mstride] for the
// post kernel -- the separate pre pass (one read and one write of every frame) disappears.
// POST (round 4): the whole MFCC in this kernel.  The last pass leaves the
// group's spectra in the LDS image (the CFFT's storage order, unpadded) instead of HBM, and the
// four waves then run the MFCC back end on them (mfcc_fixed_post.hpp: split + magnitudes, Mel
// sums, the grouped finish and DCT rows) while the next group's frames are already in flight;
// only the DCT outputs are written.  Traffic per frame: the frame once + nbDct words.
template <typename T> struct MqPostArgs {
  const int4* tw = nullptr;        // split twiddle records per bin (MfccFxDev::tw)
  const T* coefs = nullptr;
  const uint32_t* bf = nullptr;    // flat Mel list
  const T* dct = nullptr;
  const int32_t* lut = nullptr;    // sqrt_initial_lut_q31
  T* dst = nullptr;                // [batch][nb_dct]
  int nb_mel = 0, total = 0, nb_dct = 0, stage = 0;
  int kmin = 0, kcnt = 0;          // the bins the Mel filters read
};
// RSPLIT (round 5): the forward arm_rfft_q31 / _q15 of fftLenReal = 2N in one launch, as
// cfft_fx4096_kernel's RSPLIT: after the bit-reversed CFFT store (pSrc keeps the CFFT output, as
// the reference leaves it) the bins go to the LDS image in natural order and the transform's P
// threads run the split on them (8 bin pairs each) straight into its 4N-word spectrum row.
// RMERGE (round 5): the inverse arm_rfft_q31 / _q15 of fftLenReal = 2N in one launch.  The first
// pass's loads read spectrum bins X[e] and X[N - e] of the input row (rs.spec, 4N words per row)
// instead of the CFFT input, and the merge (rfft_merge_bin, arm_rfft_q31.c:397-476) forms element
// e in registers from them and the bin's record (staged once per workgroup in LDS) before the
// butterflies; the CFFT (inverse, the final arm_shift(+1) folded into the store) then writes the
// output rows in place of `data`.  The merge pass's write and the CFFT's re-read disappear.
template <typename T, int N, bool INV, bool BREV, bool SAT, bool PRE = false, bool POST = false, bool RSPLIT = false,
          bool RMERGE = false>
// (RMERGE: registers capped at two waves per SIMD, MI355X_RFFT_MERGE_WAVES.  With the lane exchange
// (MI355X_RFFT_MERGE_XCH) q31 N = 1024 then spills 21 VGPRs and still runs 464-476 against 414-416
// at one wave (ab_w1); without it the cap had spilled 60 there and lost, 294 against 388 (ab_u1).
// RSPLIT at N = 1024 capped at three waves spills 4 and loses, 307 against 320: ab_v1)
__global__ __launch_bounds__(kBlock, POST ? MI355X_MQF_WG : RMERGE ? MI355X_RFFT_MERGE_WAVES : 1) void cfft_fx_r16_kernel(typename R16Ops<T, INV>::C* __restrict__ data,
                                                             uint32_t batch,
                                                             const typename R16Ops<T, INV>::C* __restrict__ tw,
                                                             const typename R16Ops<T, INV>::C* __restrict__ win = nullptr,
                                                             T* __restrict__ maxv = nullptr, int mstride = 0,
                                                             MqPostArgs<T> pa = {}, RfSplitArgs<T> rs = {}) {
  static_assert(!POST || (PRE && !INV && !SAT), "the fused MFCC runs the forward front end");
  static_assert(!RSPLIT || (!PRE && !POST && !INV && BREV && !SAT), "the fused split follows the forward, bit-reversed CFFT");
  static_assert(!RMERGE || (!PRE && !POST && !RSPLIT && INV && SAT), "the fused merge precedes the inverse CFFT");
  using R = R16<N>;
  using O = R16Ops<T, INV>;
  using V = typename O::V;
  using Tw = typename O::Tw;
  using W = typename O::W;
  using C = typename O::C;
  using PD = R16Pad<N, sizeof(T) == 4>;
  constexpr int kC = (int)sizeof(C);
  constexpr int P = R::P, M = R::M, K = R::K;
  auto sfx = [](int e) { return e + PD::c1 * (e >> PD::k1) + PD::c2 * (e >> PD::k2); };

  __shared__ __attribute__((aligned(16))) W lds_all[R::TPW * PD::stride];
  const int t = threadIdx.x;
  const int w = t / P, tp = t % P;                    // transform in the group, thread in it
  W* lds = lds_all + w * PD::stride;
  const int h = R::BY2 ? (tp & 1) : 0;                // by2 half of the later passes
  const int tq = R::BY2 ? (tp >> 1) : tp;             // thread within that radix-4 transform

  // ---- twiddles, lane-constant for the kernel's life
  // first pass: non-by2 stage 1 (j = tp + P a) and stage 2 (j = tp); by2 pre-pass (i = tp + P u)
  // and stage 1 of the halves (j = tp + P c, c < 2)
  constexpr int NA0 = R::BY2 ? 2 : 4;
  Tw tw0a[NA0][3], tw0b[3];
  C twpre[R::BY2 ? 8 : 1];
#pragma unroll
  for (int a = 0; a < NA0; ++a)
#pragma unroll
    for (int k = 0; k < 3; ++k) tw0a[a][k] = O::tw(tw, (k + 1) * (tp + P * a) * R::MOD0);
#pragma unroll
  for (int k = 0; k < 3; ++k) tw0b[k] = O::tw(tw, (k + 1) * tp * 4 * R::MOD0);
  if constexpr (R::BY2) {
#pragma unroll
    for (int u = 0; u < 8; ++u) twpre[u] = tw[tp + P * u];
  }
  // middle pass (stages S_MID, S_MID + 1): j = tq mod d2
  constexpr int LM = M / pow4(R::S_MID - 1), D1M = LM / 4, D2M = LM / 16;
  constexpr int MODM = R::MOD0 * pow4(R::S_MID - 1);
  Tw twma[4][3], twmb[3];
  if constexpr (R::HAS_MID) {
    const int j = tq % D2M;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int k = 0; k < 3; ++k) twma[a][k] = O::tw(tw, (k + 1) * (j + D2M * a) * MODM);
#pragma unroll
    for (int k = 0; k < 3; ++k) twmb[k] = O::tw(tw, (k + 1) * j * 4 * MODM);
  }
  // two-stage last pass: stage K-1 twiddles depend on a only
  constexpr int MODL = R::MOD0 * pow4(K - 2);
  Tw twl[4][3];
  if constexpr (R::LAST2) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int k = 0; k < 3; ++k) twl[a][k] = O::tw(tw, (k + 1) * a * MODL);
  }

  // ---- work: groups of TPW transforms; workgroup b takes MI355X_FXR_T consecutive groups
  const uint32_t ngroups = (batch + R::TPW - 1) / R::TPW;
  const uint32_t g0 = blockIdx.x * MI355X_FXR_T;
  const uint32_t gend = min(ngroups, g0 + MI355X_FXR_T);
  if (g0 >= gend) return;
  // POST: the back end's tables (LDS when they fit) and each wave's work area
  using PostOps = typename std::conditional<sizeof(T) == 4, MqOpsQ31, MqOpsQ15>::type;
  constexpr int kFrameLen = 2 * N;                    // the MFCC frame: fftLen real samples
  extern __shared__ int32_t shq[];
  MqTabs tb{};
  int32_t *mag = nullptr, *mel = nullptr, *mv = nullptr;
  int64_t* acc = nullptr;
  if constexpr (POST) {
    tb = mq_stage_tables<T>(shq, pa.coefs, pa.bf, pa.total, pa.nb_mel, pa.nb_dct, pa.dct, pa.stage);
    mag = shq + (pa.stage ? mq_tab_words(pa.total, pa.nb_mel, pa.nb_dct) : 0) + (t >> 6) * mq_wave_words(kFrameLen, pa.nb_mel);
    mel = mag + mq_mel_off(kFrameLen, pa.nb_mel);
    mv = mag + mq_m_off(kFrameLen, pa.nb_mel);
    acc = reinterpret_cast<int64_t*>(mag + mq_acc_off(kFrameLen, pa.nb_mel));
  }
  auto group_rsrc = [&](uint32_t g) {
    const uint32_t first = g * R::TPW;
    const uint32_t valid = min((uint32_t)R::TPW, batch - first);
    return fx_rsrc(data + (size_t)first * N, valid * N * kC);
  };
  const int vin = (w * N + tp) * kC;                  // byte offset of the thread's first word
  V nq[16];
  // RMERGE, P > 64: bins X[N - e] prefetched too.  P <= 64 (MI355X_RFFT_MERGE_XCH): a transform's
  // lanes sit in one wave and X[N - e] = X[(P - tp) + P (15 - u)] is lane P - tp's own word u' =
  // 15 - u (lane tp = 0: its own word 16 - u, and X[N], loaded once) -- a ds_bpermute instead of a
  // second set of loads and 16-32 prefetch VGPRs.
  constexpr bool kXch = RMERGE && MI355X_RFFT_MERGE_XCH && P <= 64;
  // P = 128 (MI355X_RFFT_MERGE_LDSX): the transform spans two waves, so the raw words go through the
  // transform's LDS image instead (two extra barriers per group)
  constexpr bool kLdsX = RMERGE && MI355X_RFFT_MERGE_LDSX && P > 64;
  V nq2[RMERGE && !kXch && !kLdsX ? 16 : 1];
  V nqN{};                                            // kXch / kLdsX: X[N] of the lane's transform
  using Rec = typename SplitRec<T>::R;
  __shared__ Rec recl[RMERGE ? N : 1];                // RMERGE: the merge records of bins 0 .. N-1
  if constexpr (RMERGE) {
    for (int i = t; i < N; i += kBlock) recl[i] = rs.rec[i];
    __syncthreads();
  }
  // RMERGE: spectrum row f at rs.spec + f * 4N words (2N complex); X[e] at complex e, X[N - e]
  // at complex N - tp - P u = (P - tp) + P (15 - u), a non-negative immediate per u
  const int vsa = (w * 2 * N + tp) * kC, vsb = (w * 2 * N + P - tp) * kC;
  auto fetch = [&](uint32_t g) {
    if constexpr (RMERGE) {
      const uint32_t first = g * R::TPW;
      const uint32_t valid = min((uint32_t)R::TPW, batch - first);
      const __amdgpu_buffer_rsrc_t r = fx_rsrc((const C*)(rs.spec + (size_t)first * 4 * N), valid * 2 * N * kC);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        nq[u] = O::ld(r, vsa, P * u * kC);
        if constexpr (!kXch && !kLdsX) nq2[u] = O::ld(r, vsb, P * (15 - u) * kC);
      }
      if constexpr (kXch || kLdsX) nqN = O::ld(r, (w * 2 * N + N) * kC, 0);
    } else {
      const __amdgpu_buffer_rsrc_t r = group_rsrc(g);
#pragma unroll
      for (int u = 0; u < 16; ++u) nq[u] = O::ld(r, vin, P * u * kC);   // e = tp + P u
    }
  };
  V v[16];
  __shared__ int32_t red[PRE && P > 64 ? 2 * R::TPW : 1];
  __shared__ int32_t mvals[POST ? R::TPW : 1];        // POST: the group's frame maxima
  // first pass from nq, then the next group's loads (they fly under the later passes)
  auto pass0 = [&](uint32_t g) {
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = nq[u];
    if constexpr (RMERGE) {
      // The records are the same for every group: an opaque index keeps their LDS reads here
      // (hoisted out of the group loop they held 64 VGPRs for the kernel's life), in blocks of
      // MI355X_RFFT_MERGE_BLK elements read and merged before the next block's.
      if constexpr (kLdsX) {
        __syncthreads();                              // the previous group's last-pass reads are done
#pragma unroll
        for (int u = 0; u < 16; ++u) lds[tp + P * u] = O::to_w(nq[u]);   // natural order, unpadded
        __syncthreads();
      }
      int ri = tp;
      asm volatile("" : "+v"(ri));
      const int xsrc = ((t & 63) + P - 2 * tp) * 4;  // kXch: byte index of lane P - tp of this transform
      auto xch = [&](V x) -> V {
        if constexpr (sizeof(T) == 4)
          return make_int2(__builtin_amdgcn_ds_bpermute(xsrc, x.x), __builtin_amdgcn_ds_bpermute(xsrc, x.y));
        else
          return __builtin_bit_cast(V, __builtin_amdgcn_ds_bpermute(xsrc, __builtin_bit_cast(int, x)));
      };
#pragma unroll
      for (int u0 = 0; u0 < 16; u0 += MI355X_RFFT_MERGE_BLK) {
        Rec rc[MI355X_RFFT_MERGE_BLK];
#pragma unroll
        for (int u = 0; u < MI355X_RFFT_MERGE_BLK; ++u) rc[u] = recl[ri + P * (u0 + u)];
#pragma unroll
        for (int u = 0; u < MI355X_RFFT_MERGE_BLK; ++u) {
          const int uu = u0 + u;
          V bm;
          if constexpr (kXch) {
            bm = xch(nq[15 - uu]);
            if (tp == 0) bm = uu == 0 ? nqN : nq[(16 - uu) & 15];
          } else if constexpr (kLdsX) {
            bm = O::from_w(lds[(N - tp - P * uu) & (N - 1)]);
            if (uu == 0 && tp == 0) bm = nqN;
          } else {
            bm = nq2[uu];
          }
          const int2 m = rfft_merge_bin<T>(O::unpack(v[uu]), O::unpack(bm), rc[u].x, rc[u].y, rc[u].z, rc[u].w);
          v[u0 + u] = O::pack(m.x, m.y);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    int32_t mframe = 0;                               // POST: this transform's frame maximum
    if constexpr (PRE) {
      using Pre = MqPre<T>;
      int32_t m = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int2 z = O::unpack(v[u]);
        m = max(m, max(Pre::sat_abs(z.x), Pre::sat_abs(z.y)));
      }
#pragma unroll
      for (int o = (P < 64 ? P : 64) >> 1; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
      if constexpr (P > 64) {                         // the transform spans two waves
        if ((tp & 63) == 0) red[2 * w + (tp >> 6)] = m;
        __syncthreads();
        m = max(red[2 * w], red[2 * w + 1]);
      }
      const bool scale = m != 0 && m != Pre::kFull;
      int32_t quot = 0;
      int k = 0;
      if (scale) Pre::divide(m, quot, k);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const C wv = win[tp + P * u];                 // window words 2e, 2e + 1 of element e
        const int2 z = O::unpack(v[u]);
        v[u] = O::pack(Pre::pre(z.x, (int32_t)wv.x, scale, quot, k), Pre::pre(z.y, (int32_t)wv.y, scale, quot, k));
      }
      const uint32_t f = g * R::TPW + (uint32_t)w;
      if constexpr (POST) {
        mframe = m;                                   // published after the barrier below
      } else {
        if (tp == 0 && f < batch) maxv[(size_t)f * mstride] = (T)m;
      }
    }
    if constexpr (R::BY2) {
#pragma unroll
      for (int u = 0; u < 8; ++u) O::by2_pre(v[u], v[u + 8], twpre[u]);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          O::template bf<0>(v[8 * hh + c], v[8 * hh + c + 2], v[8 * hh + c + 4], v[8 * hh + c + 6],
                            tw0a[c][0], tw0a[c][1], tw0a[c][2]);
    } else {
      // v[4a + b] holds e = tp + P a + 4P b: stage 1 over b, stage 2 over a
      V x[16];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) x[4 * a + b] = v[a + 4 * b];
#pragma unroll
      for (int a = 0; a < 4; ++a)
        O::template bf<0>(x[4 * a], x[4 * a + 1], x[4 * a + 2], x[4 * a + 3], tw0a[a][0], tw0a[a][1], tw0a[a][2]);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        O::template bf<K == 2 ? 2 : 1>(x[b], x[4 + b], x[8 + b], x[12 + b], tw0b[0], tw0b[1], tw0b[2]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) v[a + 4 * b] = x[4 * a + b];
    }
    __syncthreads();                                  // the previous group's last reads are done
    // POST: mvals is read by every wave's back end of the previous group; a wave that finished
    // its share early must not overwrite it before the slowest one is done
    if constexpr (POST)
      if (tp == 0) mvals[w] = mframe;
#pragma unroll
    for (int u = 0; u < 16; ++u) lds[sfx(tp + P * u)] = O::to_w(v[u]);
    if (g + 1 < gend) fetch(g + 1);
    __syncthreads();
  };

  fetch(g0);
  pass0(g0);
  for (uint32_t g = g0;;) {
    // ---------------- middle pass: stages S_MID, S_MID + 1
    if constexpr (R::HAS_MID) {
      const int j = tq % D2M, gg = tq / D2M;
      const int base = h * M + gg * LM + j;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) v[4 * a + b] = O::from_w(lds[sfx(base + D2M * a + D1M * b)]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        O::template bf<1>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], twma[a][0], twma[a][1], twma[a][2]);
#pragma unroll
      for (int b = 0; b < 4; ++b)
        O::template bf<1>(v[b], v[4 + b], v[8 + b], v[12 + b], twmb[0], twmb[1], twmb[2]);
      __syncthreads();
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) lds[sfx(base + D2M * a + D1M * b)] = O::to_w(v[4 * a + b]);
      __syncthreads();
    }
    // ---------------- last pass, output with the bit reversal folded into the store
    const __amdgpu_buffer_rsrc_t rx = group_rsrc(g);
    int epos[16];                                     // element position of v[u] (bitReverseFlag 0)
    int bin[16];                                      // output bin of v[u] minus tp (bitReverseFlag 1)
    if constexpr (R::LAST2) {
      const int gg = (int)(__brev((uint32_t)tq) >> (32 - Log2<M / 16>::v));
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          epos[4 * a + b] = h * M + 16 * gg + a + 4 * b;
          v[4 * a + b] = O::from_w(lds[sfx(epos[4 * a + b])]);
          bin[4 * a + b] = (int)(__brev((uint32_t)a) >> 30) * (N / 4) + (int)(__brev((uint32_t)b) >> 30) * (N / 16);
        }
#pragma unroll
      for (int a = 0; a < 4; ++a)
        O::template bf<1>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], twl[a][0], twl[a][1], twl[a][2]);
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const Tw z{};
        O::template bf<2>(v[b], v[4 + b], v[8 + b], v[12 + b], z, z, z);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int gc = (int)(__brev((uint32_t)(tq + R::PH * c)) >> (32 - Log2<M / 4>::v));
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          epos[4 * c + b] = h * M + 4 * gc + b;
          v[4 * c + b] = O::from_w(lds[sfx(epos[4 * c + b])]);
          bin[4 * c + b] = (int)(__brev((uint32_t)b) >> 30) * (N / 4) + P * c;
        }
        const Tw z{};
        O::template bf<2>(v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3], z, z, z);
      }
    }
    if constexpr (POST) {
      __syncthreads();                                // every thread is done reading the image
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if constexpr (R::BY2) v[u] = O::by2_post(v[u]);
        lds[BREV ? tp + bin[u] : epos[u]] = O::to_w(v[u]);   // storage order, unpadded
      }
      __syncthreads();
      // the back end: wave wv takes the group's transforms wv, wv + 4, ... in chunks of G
      const PostOps op(kFrameLen, pa.nb_mel, pa.nb_dct);
      const int wv = t >> 6, lane = t & 63;
      const int32_t lutv = pa.lut[lane & 31];
      const int G = mq_group(pa.nb_mel);
      auto dctw = [&](int i) { return tb.stage ? tb.dc[i] : (int32_t)pa.dct[i]; };
      const uint32_t fbase = g * R::TPW;
      for (int s0 = wv; s0 < R::TPW; s0 += 4 * G) {
        int gn = 0;
        for (int s = s0; s < R::TPW && s < s0 + 4 * G && fbase + s < batch; s += 4, ++gn) {
          const W* img = lds_all + s * PD::stride;
          auto get = [img](int i) { return O::unpack(O::from_w(img[i])); };
          if (lane == 0) mv[gn] = mvals[s];
          mq_mel_frame<T>(op, get, pa.tw, kFrameLen, pa.kmin, pa.kcnt, pa.nb_mel, pa.total, tb, pa.coefs, lutv,
                          mag, acc + gn * pa.nb_mel);
        }
        if (gn == 0) break;
        mq_finish_group(op, gn, pa.nb_mel, pa.nb_dct, acc, mv, mel, dctw, [&](int j, int r, int32_t val) {
          pa.dst[(size_t)(fbase + s0 + 4 * j) * pa.nb_dct + r] = (T)val;
        });
      }
    } else {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (R::BY2) v[u] = O::by2_post(v[u]);   // radix4by2 post-pass <<1
      if constexpr (SAT) v[u] = O::sat(v[u]);
      if constexpr (BREV) O::st(rx, vin, bin[u] * kC, v[u]);
      else O::st(rx, (w * N + epos[u]) * kC, 0, v[u]);
    }
    if constexpr (RSPLIT) {
      __syncthreads();                                // every thread is done reading the image
#pragma unroll
      for (int u = 0; u < 16; ++u) lds[tp + bin[u]] = O::to_w(v[u]);   // natural bin order, unpadded
      __syncthreads();
      const uint32_t f = g * R::TPW + (uint32_t)w;
      if (f < batch) {
        T* y = rs.dst + (size_t)f * (4 * N);
        auto get = [&](int i) { return O::unpack(O::from_w(lds[i])); };
        const SplitRecTab<T> tab{rs.rec};
#pragma unroll MI355X_RFFT_SPLIT_UNROLL
        for (int i = 0; i < 8; ++i) rfft_split_pair<T>(get, y, tp + P * i, 2 * N, tab);
      }
    }                                                 // (the next pass 0 starts with a barrier)
    }
    if (++g >= gend) return;
    pass0(g);
  }
}

template <typename T, int N, bool INV, bool BREV, bool SAT>
static void launch_r16_t(void* data, uint32_t batch, const void* tw, hipStream_t st) {
  using C = typename R16Ops<T, INV>::C;
  const uint32_t ngroups = (batch + R16<N>::TPW - 1) / R16<N>::TPW;
  const uint32_t grid = (ngroups + MI355X_FXR_T - 1) / MI355X_FXR_T;
  hipLaunchKernelGGL((cfft_fx_r16_kernel<T, N, INV, BREV, SAT>), dim3(grid), dim3(kBlock), 0, st, (C*)data, batch,
                     (const C*)tw, (const C*)nullptr, (T*)nullptr, 0, MqPostArgs<T>{}, RfSplitArgs<T>{});
}

template <typename T, int N>
static void launch_r16(void* data, uint32_t batch, const void* tw, uint32_t flags, hipStream_t st) {
  const bool inv = flags & kIfft, brev = flags & kBitrev, sat = flags & kSatShl1;
  if (inv) {
    if (brev) sat ? launch_r16_t<T, N, true, true, true>(data, batch, tw, st) : launch_r16_t<T, N, true, true, false>(data, batch, tw, st);
    else      sat ? launch_r16_t<T, N, true, false, true>(data, batch, tw, st) : launch_r16_t<T, N, true, false, false>(data, batch, tw, st);
  } else {
    if (brev) sat ? launch_r16_t<T, N, false, true, true>(data, batch, tw, st) : launch_r16_t<T, N, false, true, false>(data, batch, tw, st);
    else      sat ? launch_r16_t<T, N, false, false, true>(data, batch, tw, st) : launch_r16_t<T, N, false, false, false>(data, batch, tw, st);
  }
}

template <typename T, int N>
static void launch_r16_mfcc(void* data, uint32_t batch, const void* tw, const void* win, T* maxv, int mstride,
                            bool brev, hipStream_t st) {
  using C = typename R16Ops<T, false>::C;
  const uint32_t ngroups = (batch + R16<N>::TPW - 1) / R16<N>::TPW;
  const uint32_t grid = (ngroups + MI355X_FXR_T - 1) / MI355X_FXR_T;
  auto k = brev ? cfft_fx_r16_kernel<T, N, false, true, false, true> : cfft_fx_r16_kernel<T, N, false, false, false, true>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, st, (C*)data, batch, (const C*)tw, (const C*)win, maxv, mstride,
                     MqPostArgs<T>{}, RfSplitArgs<T>{});
}

template <typename T, int N>
static hipError_t launch_r16_mfcc_fused(const void* data, uint32_t batch, const void* tw, const void* win, bool brev,
                                        const MqPostArgs<T>& pa0, hipStream_t st) {
  using C = typename R16Ops<T, false>::C;
  MqPostArgs<T> pa = pa0;
  const size_t tab = sizeof(int32_t) * (size_t)mq_tab_words(pa.total, pa.nb_mel, pa.nb_dct);
  const size_t waves = sizeof(int32_t) * 4 * (size_t)mq_wave_words(2 * N, pa.nb_mel);
  pa.stage = MI355X_MQF_STAGE && waves + tab <= 32768 ? 1 : 0;
  const size_t lds = waves + (pa.stage ? tab : 0);
  auto k = brev ? cfft_fx_r16_kernel<T, N, false, true, false, true, true>
                : cfft_fx_r16_kernel<T, N, false, false, false, true, true>;
  if (lds > 65536) {
    if (lds > 100 * 1024) return hipErrorInvalidValue;
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const uint32_t ngroups = (batch + R16<N>::TPW - 1) / R16<N>::TPW;
  const uint32_t grid = (ngroups + MI355X_FXR_T - 1) / MI355X_FXR_T;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), lds, st, (C*)data, batch, (const C*)tw, (const C*)win, (T*)nullptr,
                     0, pa, RfSplitArgs<T>{});
  return hipGetLastError();
}

// The whole MFCC q31 / q15 of fftLen 2n frames in one launch (n = 256..2048, the reference's own
// bit-reversal table); hipErrorNotSupported: not handled here (the caller takes the two-launch
// schedule).
template <typename T>
static hipError_t dispatch_r16_mfcc_fused(int n, const T* frames, uint32_t batch, const T* tw, const T* win, bool brev,
                                          const MqPostArgs<T>& pa, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  switch (n) {
    case 256:  return launch_r16_mfcc_fused<T, 256>(frames, batch, tw, win, brev, pa, st);
    case 512:  return launch_r16_mfcc_fused<T, 512>(frames, batch, tw, win, brev, pa, st);
    case 1024: return launch_r16_mfcc_fused<T, 1024>(frames, batch, tw, win, brev, pa, st);
    case 2048: return launch_r16_mfcc_fused<T, 2048>(frames, batch, tw, win, brev, pa, st);
    default:   return hipErrorNotSupported;
  }
}
hipError_t mfcc_q31_fused_launch(int n, const int32_t* frames, uint32_t batch, const int32_t* tw, const int32_t* win,
                                 bool brev, const int4* stw, int nb_mel, const int32_t* coefs, const uint32_t* bf,
                                 int total, int kmin, int kcnt, int nb_dct, const int32_t* dct, const int32_t* lut,
                                 int32_t* dst, hipStream_t st) {
  MqPostArgs<int32_t> pa;
  pa.tw = stw; pa.coefs = coefs; pa.bf = bf; pa.dct = dct; pa.lut = lut; pa.dst = dst;
  pa.nb_mel = nb_mel; pa.total = total; pa.nb_dct = nb_dct; pa.kmin = kmin; pa.kcnt = kcnt;
  return dispatch_r16_mfcc_fused<int32_t>(n, frames, batch, tw, win, brev, pa, st);
}
hipError_t mfcc_q15_fused_launch(int n, const int16_t* frames, uint32_t batch, const int16_t* tw, const int16_t* win,
                                 bool brev, const int4* stw, int nb_mel, const int16_t* coefs, const uint32_t* bf,
                                 int total, int kmin, int kcnt, int nb_dct, const int16_t* dct, const int32_t* lut,
                                 int16_t* dst, hipStream_t st) {
  MqPostArgs<int16_t> pa;
  pa.tw = stw; pa.coefs = coefs; pa.bf = bf; pa.dct = dct; pa.lut = lut; pa.dst = dst;
  pa.nb_mel = nb_mel; pa.total = total; pa.nb_dct = nb_dct; pa.kmin = kmin; pa.kcnt = kcnt;
  return dispatch_r16_mfcc_fused<int16_t>(n, frames, batch, tw, win, brev, pa, st);
}

// MFCC front end + the RFFT's inner forward CFFT of length n in place (n = fftLen / 2 in
// 256..2048, the reference's own bit-reversal table); false: not handled here.
template <typename T>
static bool dispatch_r16_mfcc(int n, T* data, uint32_t batch, const T* tw, const T* win, T* maxv, int mstride,
                              bool brev, hipStream_t st) {
  switch (n) {
    case 256:  launch_r16_mfcc<T, 256>(data, batch, tw, win, maxv, mstride, brev, st); return true;
    case 512:  launch_r16_mfcc<T, 512>(data, batch, tw, win, maxv, mstride, brev, st); return true;
    case 1024: launch_r16_mfcc<T, 1024>(data, batch, tw, win, maxv, mstride, brev, st); return true;
    case 2048: launch_r16_mfcc<T, 2048>(data, batch, tw, win, maxv, mstride, brev, st); return true;
    default:   return false;
  }
}
bool cfft_q31_r16_mfcc_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, const int32_t* win,
                              int32_t* maxv, int mstride, bool brev, hipStream_t st) {
  return dispatch_r16_mfcc<int32_t>(n, data, batch, tw, win, maxv, mstride, brev, st);
}
bool cfft_q15_r16_mfcc_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, const int16_t* win,
                              int16_t* maxv, int mstride, bool brev, hipStream_t st) {
  return dispatch_r16_mfcc<int16_t>(n, data, batch, tw, win, maxv, mstride, brev, st);
}

// The forward arm_rfft_q31 / _q15 of fftLenReal = 2n in one launch (n = 256 .. 2048, the
// reference's own bit-reversal table, bitReverseFlag 1); false: not handled here.
template <typename T, int N>
static void launch_r16_rfft(T* src, T* dst, uint32_t batch, const T* tw, const void* rec, hipStream_t st) {
  using C = typename R16Ops<T, false>::C;
  const uint32_t ngroups = (batch + R16<N>::TPW - 1) / R16<N>::TPW;
  const uint32_t grid = (ngroups + MI355X_FXR_T - 1) / MI355X_FXR_T;
  RfSplitArgs<T> rs;
  rs.dst = dst;
  rs.rec = (const typename SplitRec<T>::R*)rec;
  hipLaunchKernelGGL((cfft_fx_r16_kernel<T, N, false, true, false, false, false, true>), dim3(grid), dim3(kBlock), 0, st,
                     (C*)src, batch, (const C*)tw, (const C*)nullptr, (T*)nullptr, 0, MqPostArgs<T>{}, rs);
}
template <typename T>
static bool dispatch_r16_rfft(int n, T* src, T* dst, uint32_t batch, const T* tw, const void* rec, hipStream_t st) {
  if (batch == 0 && n >= 256 && n <= 2048) return true;
  switch (n) {
    case 256:  launch_r16_rfft<T, 256>(src, dst, batch, tw, rec, st); return true;
    case 512:  launch_r16_rfft<T, 512>(src, dst, batch, tw, rec, st); return true;
    case 1024: launch_r16_rfft<T, 1024>(src, dst, batch, tw, rec, st); return true;
    case 2048: launch_r16_rfft<T, 2048>(src, dst, batch, tw, rec, st); return true;
    default:   return false;
  }
}
// The inverse arm_rfft_q31 / _q15 of fftLenReal = 2n in one launch (n = 256 .. 2048, the
// reference's own bit-reversal table, bitReverseFlag 1): spec [batch][4n] spectrum rows (bins 0..n
// read), dst [batch][2n]; false: not handled here.
template <typename T, int N>
static void launch_r16_irfft(const T* spec, T* dst, uint32_t batch, const T* tw, const void* rec, hipStream_t st) {
  using C = typename R16Ops<T, true>::C;
  const uint32_t ngroups = (batch + R16<N>::TPW - 1) / R16<N>::TPW;
  const uint32_t grid = (ngroups + MI355X_FXR_T - 1) / MI355X_FXR_T;
  RfSplitArgs<T> rs;
  rs.spec = spec;
  rs.rec = (const typename SplitRec<T>::R*)rec;
  hipLaunchKernelGGL((cfft_fx_r16_kernel<T, N, true, true, true, false, false, false, true>), dim3(grid), dim3(kBlock), 0,
                     st, (C*)dst, batch, (const C*)tw, (const C*)nullptr, (T*)nullptr, 0, MqPostArgs<T>{}, rs);
}
template <typename T>
static bool dispatch_r16_irfft(int n, const T* spec, T* dst, uint32_t batch, const T* tw, const void* rec, hipStream_t st) {
  if (batch == 0 && n >= 256 && n <= 2048) return true;
  switch (n) {
    case 256:  launch_r16_irfft<T, 256>(spec, dst, batch, tw, rec, st); return true;
    case 512:  launch_r16_irfft<T, 512>(spec, dst, batch, tw, rec, st); return true;
    case 1024: launch_r16_irfft<T, 1024>(spec, dst, batch, tw, rec, st); return true;
    case 2048: launch_r16_irfft<T, 2048>(spec, dst, batch, tw, rec, st); return true;
    default:   return false;
  }
}
bool rfft_q31_r16_inv_fused_launch(int n, const int32_t* spec, int32_t* dst, uint32_t batch, const int32_t* tw,
                                   const void* rec, hipStream_t st) {
  return dispatch_r16_irfft<int32_t>(n, spec, dst, batch, tw, rec, st);
}
bool rfft_q15_r16_inv_fused_launch(int n, const int16_t* spec, int16_t* dst, uint32_t batch, const int16_t* tw,
                                   const void* rec, hipStream_t st) {
  return dispatch_r16_irfft<int16_t>(n, spec, dst, batch, tw, rec, st);
}

bool rfft_q31_r16_fused_launch(int n, int32_t* src, int32_t* dst, uint32_t batch, const int32_t* tw, const void* rec,
                               hipStream_t st) {
  return dispatch_r16_rfft<int32_t>(n, src, dst, batch, tw, rec, st);
}
bool rfft_q15_r16_fused_launch(int n, int16_t* src, int16_t* dst, uint32_t batch, const int16_t* tw, const void* rec,
                               hipStream_t st) {
  return dispatch_r16_rfft<int16_t>(n, src, dst, batch, tw, rec, st);
}

// Returns true if N is handled here (the reference's own bit-reversal table only).
template <typename T>
static bool dispatch_r16(int n, void* data, uint32_t batch, const void* tw, uint32_t flags, hipStream_t st) {
  switch (n) {
    case 256:  launch_r16<T, 256>(data, batch, tw, flags, st); return true;
    case 512:  launch_r16<T, 512>(data, batch, tw, flags, st); return true;
    case 1024: launch_r16<T, 1024>(data, batch, tw, flags, st); return true;
    case 2048: launch_r16<T, 2048>(data, batch, tw, flags, st); return true;
    default:   return false;
  }
}

bool cfft_q31_r16_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, uint32_t flags, hipStream_t st) {
  return dispatch_r16<int32_t>(n, data, batch, tw, flags, st);
}
bool cfft_q15_r16_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, uint32_t flags, hipStream_t st) {
  return dispatch_r16<int16_t>(n, data, batch, tw, flags, st);
}

}  // namespace mi355x
