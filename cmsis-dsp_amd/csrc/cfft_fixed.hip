// Batched complex FFT, q31 and q15 — MI355X (gfx950) kernels, bit-exact.
//
// Replaces the host scalar path (ARM_MATH_DSP undefined) of
//   q31: Source/TransformFunctions/arm_cfft_q31.c:704-755 (dispatch), :763-881 (radix4by2),
//        arm_cfft_radix4_q31.c:153-473 (forward), :524-834 (inverse);
//   q15: Source/TransformFunctions/arm_cfft_q15.c:671-722, :782-827 / :881-926 (radix4by2
//        scalar branch), arm_cfft_radix4_q15.c:572-970 (forward, scalar branch),
//        :1434-1813 (inverse, scalar branch);
//   arm_bitreversal_32 / _16 (arm_bitreversal2.c:84-148) with armBitRevIndexTable_fixed_N.
//
// Geometry as the f32 kernel: 256-thread workgroups, N/16 lanes per transform, every
// radix-4 stage is an LDS -> VGPR -> LDS pass with 4 butterflies per lane.  Integer
// semantics are the reference's on gcc/x86-64: int32 wrap, arithmetic right shifts,
// v_mul_hi_i32 for ((q63)a*b)>>32, int16 truncation on q15 stores, __SSAT(.,16).
#include "common.hpp"
#include "kernels.hpp"
#include "cfft_fixed_core.hpp"
#include "rfft_fixed_split.hpp"

namespace mi355x {

template <typename T, int N, bool INV>
__global__ __launch_bounds__(kBlock) void cfft_fx_kernel(typename Fx<T>::C* __restrict__ data, uint32_t batch,
                                                         const typename Fx<T>::C* __restrict__ tw,
                                                         const uint16_t* __restrict__ perm, uint32_t flags) {
  using P = PlanFx<N>;
  using F = Fx<T>;
  using C = typename F::C;
  // transforms sit SP complex apart in LDS: for N <= 64 (LPT <= 4: many transforms per
  // 32-lane group, all at the same offset) one pad element keeps their lanes on distinct
  // banks; larger N pay more in occupancy than they would gain (measured)
  constexpr int SP = N + (P::LPT <= 4 ? 1 : 0);
  __shared__ __attribute__((aligned(16))) C lds[P::TPB * SP];
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * P::TPB;
  const int valid = (int)min<uint64_t>((uint64_t)P::TPB, batch - t0);

  {  // coalesced 16-B load, scattered to the padded LDS image
    constexpr int PER16 = 16 / (int)sizeof(C);
    const int4* src = reinterpret_cast<const int4*>(data + t0 * N);
    const int n16 = valid * N / PER16;
#pragma unroll 4
    for (int i = tid; i < n16; i += kBlock) {
      const int4 v = src[i];
      const int e = i * PER16, t = e / N, k = e % N;
      const C* c = reinterpret_cast<const C*>(&v);
#pragma unroll
      for (int u = 0; u < PER16; ++u) lds[t * SP + k + u] = c[u];
    }
  }
  __syncthreads();

  const int tr = tid / P::LPT, lane = tid % P::LPT;
  C* x = lds + tr * SP;

  cfft_fx_lds_body<T, N, INV>(x, tw, lane);

  {  // store: binary bit reversal as an LDS gather; radix4by2 post-pass "<<1" folded here
    constexpr int LOG = Log2<N>::v;
    constexpr int PER16 = 16 / (int)sizeof(C);     // complex per 16-B store
    const bool brev = flags & kBitrev;
    int4* dst = reinterpret_cast<int4*>(data + t0 * N);
    const int n16 = valid * N / PER16;
#pragma unroll 2
    for (int i = tid; i < n16; i += kBlock) {
      const int e = i * PER16, t = e / N, k0 = e % N;
      int2 v[PER16];
#pragma unroll
      for (int u = 0; u < PER16; ++u) {
        const int k = k0 + u;
        const int src = brev ? (perm ? (int)perm[k] : bitrev<LOG>(k)) : k;
        v[u] = F::ld(lds + t * SP + src);
        if constexpr (P::BY2) {
          if constexpr (sizeof(T) == 4) v[u] = make_int2(wshl(v[u].x, 1), wshl(v[u].y, 1));
          else v[u] = make_int2(t16(v[u].x << 1), t16(v[u].y << 1));
        }
        if (flags & kSatShl1) v[u] = sat_shl1<T>(v[u]);
      }
      if constexpr (sizeof(T) == 4) {
        dst[i] = make_int4(v[0].x, v[0].y, v[1].x, v[1].y);
      } else {
        int4 o;
        o.x = (v[0].x & 0xFFFF) | (v[0].y << 16);
        o.y = (v[1].x & 0xFFFF) | (v[1].y << 16);
        o.z = (v[2].x & 0xFFFF) | (v[2].y << 16);
        o.w = (v[3].x & 0xFFFF) | (v[3].y << 16);
        dst[i] = o;
      }
    }
  }
}

// ============================================================================================
// N = 4096 specialist (BASELINE configs[3]).  4096 = 4^6: six radix-4 stages fused in
// pairs (radix-16 register passes), one 256-thread workgroup per transform, persistent.
//   pass 1: thread c holds e = c + 256a + 1024b   -> stage 1 (over b), stage 2 (over a)
//   pass 2: thread (q, j) = (t/16, t%16) holds e = 256q + j + 64a + 16b
//                                                   -> stage 3 (over a), stage 4 (over b)
//   pass 3: thread t holds e = 16*rev8(t) + 4a + b  -> stage 5 (over a), stage 6 (over b)
// Output position e = 16*rev8(t) + u goes to bin rev12(e) = rev4(u)*256 + t: for every u
// the 256 threads store 256 consecutive bins, so the bit reversal is free.
// LDS paddings are additive (every access is lane base + immediate) and bank-conflict free
// under the banking of the instructions the compiler emits (MI355X_MICROARCH.md §LDS):
//  * 8-B complex (q31): reads pair into ds_read2_b64, writes are ds_write(2)_b64, all
//    serviced in 16-lane groups on (dword mod 32) banks.  Passes 1-2 touch 16 consecutive e
//    per group; pass 3's group reads e = 256*rev4(i) + K (i < 16), which s(e) = e + (e >> 8)
//    puts on 16 distinct bank pairs.  The round-1 padding s4096 was chosen for ds_read_b64's
//    32-lane / mod-64 banking and left pass 3 two-way conflicted under ds_read2_b64: 64
//    extra LDS cycles per wave per transform (profiles/r02/cfft_q31_4096_strong1M/pmc.json).
//  * 4-B complex (q15): ds_write_b32 / ds_read2_b32 in 32-lane groups on mod-32 banks; pass
//    3's group reads e = 256*rev4(i) + 128g + K, which s4096 keeps conflict free (PMC: 0).
__device__ __forceinline__ int s4096(int e) { return e + 8 * (e >> 7) + (e >> 9); }
template <typename C> __device__ __forceinline__ int sfx(int e) {
  if constexpr (sizeof(C) == 8) return e + (e >> 8);
  else return s4096(e);
}
// LDS complex slots of the q31 N = 4096 kernel: 4112 are used; the image is sized to 6912 (54 KiB)
// so that two workgroups share a CU (three fit by registers): configs[3] q31 344-348 -> 350-352
// Gsamples/s, bit-exact (profiles/r03/experiments/fx4096_residency.json; one workgroup per CU
// 274, and the q15 kernel is fastest at its register-bound three).  The in-place streaming probe
// of this access pattern ranks the same way (profiles/r03/probe_hbm_wgtile.txt, lds = 55296).
template <typename C> constexpr int kFxSlots = sizeof(C) == 8 ? MI355X_FX_Q31_SLOTS : 4351;

// Twiddle placement.  Lane-distinct twiddles (stage 1: 12 words per lane, stage 2: 3) stay in
// VGPRs for the kernel's life; stage 3 depends only on (t % 16, a) and stage 4 on t % 16, so
// MI355X_FX_TW3_LDS / MI355X_FX_TW4_LDS keep them in small LDS tables (1.5 KiB / 384 B, read
// as conflict-free broadcasts) instead of 24 / 6 VGPRs.  Stage 5 is lane-uniform (SGPRs).
// MI355X_FX_PF = d >= 1: the next d transforms' 16 loads are held in registers (the first under
// passes 2-3 of the current one), 32 VGPRs per transform for q31.
// BREV / SAT are the bitReverseFlag and the RFFT inverse's saturating <<1 (kSatShl1) as
// template parameters: as run-time flags the compiler if-converted them into selects on
// every output word and address.
// RSPLIT (the forward arm_rfft_q31 of N = 8192, whose inner CFFT this is): after pass 3 the
// transform's bins also go to LDS in natural order, and the workgroup runs the RFFT's split on
// them (rfft_fixed_split.hpp, arm_rfft_q31.c:256-341) straight into the 2N-word spectrum row --
// the CFFT output is still stored to `data`, as the reference leaves pSrc, but never read back.
// RMERGE (q31): the inverse arm_rfft_q31 of N = 8192 in one launch, as cfft_q15_4096_pk_kernel's
// RMERGE, from half the records (the tables' symmetry) and the minimal image: two workgroups per CU.
template <typename T, bool INV, bool BREV, bool SAT, bool RSPLIT = false, bool RMERGE = false>
__global__ __launch_bounds__(256, RMERGE ? 2 : MI355X_FX_WAVES) void cfft_fx4096_kernel(typename Fx<T>::C* __restrict__ data, uint32_t batch,
                                                          const typename Fx<T>::C* __restrict__ tw,
                                                          RfSplitArgs<T> rs = {}) {
  static_assert(!RSPLIT || (!INV && BREV && !SAT), "the fused split follows the forward, bit-reversed CFFT");
  static_assert(!RMERGE || (sizeof(T) == 4 && !RSPLIT && INV && BREV && SAT), "the fused merge precedes the inverse CFFT");
  using F = Fx<T>;
  using C = typename F::C;
  using IO = FxIO<C>;
  constexpr int kC = (int)sizeof(C);
  // RMERGE: the minimal image (4112 slots) beside 32 KiB of records, so two workgroups share a CU
  __shared__ __attribute__((aligned(16))) C lds[RMERGE ? 4112 : kFxSlots<C>];
  const int t = threadIdx.x;
  const int q2 = t >> 4, j2 = t & 15;
  const int q3 = (int)(__brev((uint32_t)t) >> 24);        // rev8(t)
  const FxWalk wk = fx_walk<MI355X_FX_T>(batch);
  const uint32_t tr0 = wk.begin, tend = wk.end, step = wk.step;

  // Lane-constant twiddles (stored in the table's word type).  (w1, w2, w3) = table[ia],
  // table[2ia], table[3ia] of the butterfly's index ia.
  C tw1[4][3], tw2[3], tw5[4][3];
  // RMERGE keeps the stage-3/4 twiddles in LDS tables (30 VGPRs) to stay at two waves per SIMD
  constexpr bool kTw3L = MI355X_FX_TW3_LDS || RMERGE, kTw4L = MI355X_FX_TW4_LDS || RMERGE;
  __shared__ __attribute__((aligned(16))) C tw3l[kTw3L ? 64 * 3 : 1];
  __shared__ __attribute__((aligned(16))) C tw4l[kTw4L ? 16 * 3 : 1];
  C tw3[4][3], tw4[3];
  if constexpr (kTw3L)
    if (t < 192) tw3l[t] = tw[(t % 3 + 1) * (t / 3) * 16];        // visible after the loop's barriers
  if constexpr (kTw4L)
    if (t < 48) tw4l[t] = tw[(t % 3 + 1) * 64 * (t / 3)];
  auto TW3 = [&](int a, int k) -> C {
    if constexpr (kTw3L) return tw3l[(j2 + 16 * a) * 3 + k];
    else return tw3[a][k];
  };
  auto TW4 = [&](int k) -> C {
    if constexpr (kTw4L) return tw4l[j2 * 3 + k];
    else return tw4[k];
  };
#pragma unroll
  for (int a = 0; a < 4; ++a) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      tw1[a][k] = tw[(k + 1) * (t + 256 * a)];
      if constexpr (!kTw3L) tw3[a][k] = tw[(k + 1) * (j2 + 16 * a) * 16];
      tw5[a][k] = tw[(k + 1) * a * 256];
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    tw2[k] = tw[(k + 1) * 4 * t];
    if constexpr (!kTw4L) tw4[k] = tw[(k + 1) * 64 * j2];
  }
  auto W = [](C c) { return make_int2(c.x, c.y); };
  // RMERGE: the records of bins 0 .. 2048 only -- the caller checked that its tables are symmetric
  // (record 4096 - e = record e with A1, B1 negated, true of the reference's realCoefAQ31 / BQ31)
  __shared__ int4 recl[RMERGE ? 2049 : 1];
  if constexpr (RMERGE) {
    for (int i = t; i <= 2048; i += 256) recl[i] = reinterpret_cast<const int4*>(rs.rec)[i];
    __syncthreads();
  }

  // walk: nq[d] holds transform tr + (d + 1) * step (FxWalk)
  constexpr int PFD = MI355X_FX_PF > 0 ? MI355X_FX_PF : 1;
  const int vin = t * kC;                                    // byte offset of element t
  auto fetch = [&](C (&dst)[16], C (&dst2)[16], uint32_t tr) {
    if constexpr (RMERGE) {
      // spectrum row tr: 8192 complex words; X[e] at e = t + 256 a + 1024 b, X[4096 - e] at
      // (256 - t) + 256 (3 - a) + 1024 (3 - b)
      const __amdgpu_buffer_rsrc_t r = fx_rsrc(rs.spec + (size_t)tr * 16384, 8192 * kC);
      const int vneg = (256 - t) * kC;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          dst[4 * a + b] = IO::ld(r, vin, (256 * a + 1024 * b) * kC);
          dst2[4 * a + b] = IO::ld(r, vneg, (256 * (3 - a) + 1024 * (3 - b)) * kC);
        }
    } else {
      const __amdgpu_buffer_rsrc_t r = fx_rsrc(data + (size_t)tr * 4096, 4096 * kC);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) dst[4 * a + b] = IO::ld(r, vin, (256 * a + 1024 * b) * kC);
    }
  };
  int2 v[16];
  C nq[PFD][16], nq2[PFD][16];                              // nq2: RMERGE's X[4096 - e] words
  // Pass 1 of transform tr from nq[0]; then the prefetch of transform tr + PFD * step.
  auto pass1 = [&](C (&buf)[16], C (&buf2)[16], uint32_t tr) {
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = W(buf[u]);
    if constexpr (RMERGE) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int u = 4 * a + b;
          int4 rc;
          if (b < 2) {
            rc = recl[t + 256 * a + 1024 * b];
          } else {                                           // e >= 2048: mirrored record
            const int4 r = recl[4096 - (t + 256 * a + 1024 * b)];
            rc = make_int4(r.x, wneg(r.y), r.z, wneg(r.w));
          }
          v[u] = rfft_merge_bin<T>(v[u], W(buf2[u]), rc.x, rc.y, rc.z, rc.w);
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
      bfly<T, INV, 0>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], W(tw1[a][0]), W(tw1[a][1]), W(tw1[a][2]));
#pragma unroll
    for (int b = 0; b < 4; ++b) bfly<T, INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], W(tw2[0]), W(tw2[1]), W(tw2[2]));
    __syncthreads();                    // the previous transform's pass-3 reads are done
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) F::st(lds + sfx<C>(t + 256 * a + 1024 * b), v[4 * a + b]);
    if (tr + PFD * step < tend) fetch(buf, buf2, tr + PFD * step);   // flies under passes 2-3
    __syncthreads();
  };
  // The loop is entered after pass 1, so that at the point where pass 1 of the next
  // transform waits for its prefetched words, the only younger vector-memory operations are
  // the current transform's 16 stores and the deeper prefetches, on every path: the compiler
  // then waits with vmcnt(16 * PFD) instead of draining the stores.  (With pass 1 at the
  // loop head, the merge of the entry path -- prefetch loads youngest -- with the back edge
  // made it wait for vmcnt(0), i.e. for the previous transform's stores to complete.)  The
  // loop is unrolled PFD times so the prefetch buffers rotate by name: copying a buffer
  // whose loads are in flight would wait for them.
  if (tr0 >= tend) return;
#pragma unroll
  for (int d = 0; d < PFD; ++d)
    if (tr0 + d * step < tend) fetch(nq[d], nq2[d], tr0 + d * step);
  pass1(nq[0], nq2[0], tr0);
  uint32_t tr = tr0;
  auto pass23 = [&]() {
    const __amdgpu_buffer_rsrc_t rx = fx_rsrc(data + (size_t)tr * 4096, 4096 * kC);
    // ---------------- pass 2: stages 3 and 4
    {
      const int base = 256 * q2 + j2;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) v[4 * a + b] = F::ld(lds + sfx<C>(base + 64 * a + 16 * b));
#pragma unroll
      for (int b = 0; b < 4; ++b)
        bfly<T, INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], W(TW3(b, 0)), W(TW3(b, 1)), W(TW3(b, 2)));
#pragma unroll
      for (int a = 0; a < 4; ++a)
        bfly<T, INV, 1>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], W(TW4(0)), W(TW4(1)), W(TW4(2)));
      __syncthreads();
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) F::st(lds + sfx<C>(base + 64 * a + 16 * b), v[4 * a + b]);
    }
    __syncthreads();
    // ---------------- pass 3: stages 5 and 6 (last)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) v[4 * a + b] = F::ld(lds + sfx<C>(16 * q3 + 4 * a + b));
#pragma unroll
    for (int b = 0; b < 4; ++b)
      bfly<T, INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], W(tw5[b][0]), W(tw5[b][1]), W(tw5[b][2]));
#pragma unroll
    for (int a = 0; a < 4; ++a)
      bfly<T, INV, 2>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], int2{}, int2{}, int2{});
    if constexpr (SAT) {
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = sat_shl1<T>(v[u]);
    }
    C o[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) o[u] = C{(typename F::S)v[u].x, (typename F::S)v[u].y};
    if constexpr (BREV) {
#pragma unroll
      for (int u = 0; u < 16; ++u) IO::st(rx, vin, (int)(__brev((uint32_t)u) >> 28) * 256 * kC, o[u]);
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) IO::st(rx, 16 * q3 * kC, u * kC, o[u]);
    }
    if constexpr (RSPLIT) {
      __syncthreads();                  // every thread's pass-3 LDS reads are done
#pragma unroll
      for (int u = 0; u < 16; ++u) F::st(lds + sfx<C>((int)(__brev((uint32_t)u) >> 28) * 256 + t), v[u]);
      __syncthreads();
      T* y = rs.dst + (size_t)tr * (2 * 8192);
      auto get = [&](int i) { return F::ld(lds + sfx<C>(i)); };
      const SplitStridedTab<T> tab{rs.ta, rs.tb, rs.mod};
#pragma unroll 2
      for (int i = 0; i < 8; ++i) rfft_split_pair<T>(get, y, t + 256 * i, 8192, tab);
    }                                   // (the next pass 1 starts with a barrier before its LDS writes)
  };
  for (;;) {
#pragma unroll
    for (int d = 0; d < PFD; ++d) {
      pass23();
      tr += step;
      if (tr >= tend) return;
      pass1(nq[(d + 1) % PFD], nq2[(d + 1) % PFD], tr);
    }
  }
}


// ============================================================================================
// q15 N = 4096 on packed 16-bit math: one VGPR holds a complex sample {re, im} and every
// radix-4 butterfly of bfly_q15 is restated on v_pk_* / v_dot2 with identical bits:
//   __SSAT(x + y, 16), __SSAT(x - y, 16)  -> v_pk_add_i16 / v_pk_sub_i16 with clamp
//   t16((x >> 1) +- (y >> 1)) (never wraps) -> v_pk_ashrrev_i16 + v_pk_add/sub_u16
//   (q15)((p*q +- r*s) >> 16) (int32 wrap)  -> v_dot2_i32_i16 (modular) and the high half;
//     a difference uses the twiddle word ~w (= -w - 1) and adds the missing +R back through
//     the dot's accumulator: w.x*R1 - w.y*R0 = dot2({~w.y, w.x}, R) + R0 (mod 2^32).
// Each twiddle is held as the two packed words its products need (forward {w.x, w.y} and
// {~w.y, w.x}; inverse {w.x, ~w.y} and {w.y, w.x}).  Same work mapping as
// cfft_fx4096_kernel (three radix-16 register passes, s4096 LDS padding, free bit reversal).
// MI355X_FXQ15_TW34_LDS = 1: the stage-3/4 twiddle pairs (functions of t % 16 only) live in
// LDS tables (1.5 KiB + 384 B) instead of 30 VGPRs; MI355X_FXQ15_WAVES = the minimum waves per
// SIMD the register allocation must allow.
// RSPLIT: the forward arm_rfft_q15 of N = 8192 fused as in cfft_fx4096_kernel.
// RMERGE: the inverse arm_rfft_q15 of N = 8192 in one launch (as cfft_fx_r16_kernel's RMERGE): the
// prefetch reads spectrum bins X[e] and X[4096 - e] of the input row (rs.spec), pass 1 forms the
// merge from them and the bin's record (32 KiB of short4 records in LDS, staged once), and the
// inverse CFFT's saturating <<1 store writes the output row to `data`.
template <bool INV, bool BREV, bool SAT, bool RSPLIT = false, bool RMERGE = false>
__global__ __launch_bounds__(256, RMERGE ? 3 : MI355X_FXQ15_WAVES) void cfft_q15_4096_pk_kernel(short2* __restrict__ data, uint32_t batch,
                                                                    const short2* __restrict__ tw,
                                                                    RfSplitArgs<int16_t> rs) {
  static_assert(!RSPLIT || (!INV && BREV && !SAT), "the fused split follows the forward, bit-reversed CFFT");
  static_assert(!RMERGE || (!RSPLIT && INV && BREV && SAT), "the fused merge precedes the inverse CFFT");
  __shared__ __attribute__((aligned(16))) uint32_t lds[MI355X_FXQ15_SLOTS];
  const int t = threadIdx.x;
  const int q2 = t >> 4, j2 = t & 15;
  const int q3 = (int)(__brev((uint32_t)t) >> 24);        // rev8(t)
  const FxWalk wk = fx_walk<MI355X_FXQ15_T>(batch);
  const uint32_t tr0 = wk.begin, tend = wk.end, step = wk.step;
  TwP tw1[4][3], tw2[3], tw5[4][3];
  // RMERGE keeps the stage-3/4 twiddles in LDS too: its X[4096 - e] prefetch words need the 30
  // VGPRs to stay at three waves per SIMD (172 -> 142)
  constexpr bool kTwL = MI355X_FXQ15_TW34_LDS || RMERGE;
  __shared__ TwP tw3l[kTwL ? 64 * 3 : 1], tw4l[kTwL ? 16 * 3 : 1];
  TwP tw3[4][3], tw4[3];
  if constexpr (kTwL) {
    if (t < 192) tw3l[t] = twp<INV>(tw[(t % 3 + 1) * (t / 3) * 16]);    // visible after the loop's barriers
    else if (t < 240) tw4l[t - 192] = twp<INV>(tw[((t - 192) % 3 + 1) * 64 * ((t - 192) / 3)]);
  }
  auto TW3Q = [&](int a, int k) -> TwP {
    if constexpr (kTwL) return tw3l[(j2 + 16 * a) * 3 + k];
    else return tw3[a][k];
  };
  auto TW4Q = [&](int k) -> TwP {
    if constexpr (kTwL) return tw4l[j2 * 3 + k];
    else return tw4[k];
  };
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      tw1[a][k] = twp<INV>(tw[(k + 1) * (t + 256 * a)]);
      if constexpr (!kTwL) tw3[a][k] = twp<INV>(tw[(k + 1) * (j2 + 16 * a) * 16]);
      tw5[a][k] = twp<INV>(tw[(k + 1) * a * 256]);
    }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    tw2[k] = twp<INV>(tw[(k + 1) * 4 * t]);
    if constexpr (!kTwL) tw4[k] = twp<INV>(tw[(k + 1) * 64 * j2]);
  }
  const TwP z{};
  __shared__ short4 recl[RMERGE ? 4096 : 1];               // RMERGE: the merge records of bins 0 .. 4095
  if constexpr (RMERGE) {
    for (int i = t; i < 4096; i += 256) recl[i] = rs.rec[i];
    __syncthreads();
  }

  s16x2 v[16];
  const int vin = t * 4;                                   // byte offset of element t
  auto fetch = [&](uint32_t (&dst)[16], uint32_t (&dst2)[16], uint32_t tr) {
    if constexpr (RMERGE) {
      // spectrum row tr: 8192 complex words; X[e] at e = t + 256 a + 1024 b, X[4096 - e] at
      // (256 - t) + 256 (3 - a) + 1024 (3 - b): non-negative immediates
      const __amdgpu_buffer_rsrc_t r = fx_rsrc(rs.spec + (size_t)tr * 16384, 8192 * 4);
      const int vneg = (256 - t) * 4;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          dst[4 * a + b] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, vin, (256 * a + 1024 * b) * 4, MI355X_FX_NT);
          dst2[4 * a + b] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, vneg, (256 * (3 - a) + 1024 * (3 - b)) * 4,
                                                                           MI355X_FX_NT);
        }
    } else {
      const __amdgpu_buffer_rsrc_t r = fx_rsrc(data + (size_t)tr * 4096, 4096 * 4);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          dst[4 * a + b] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, vin, (256 * a + 1024 * b) * 4, MI355X_FX_NT);
    }
  };
  // Register prefetch MI355X_FX_Q15_PFD transforms deep: nq[d] holds transform tr + (d+1)*step.
  // q15 moves 4 B per load, so at the workgroups a CU holds one transform of look-ahead
  // (16 KiB per workgroup) does not cover the HBM latency; two measured +8.5 %.
  constexpr int PFD = MI355X_FX_Q15_PFD;
  uint32_t nq[PFD][16], nq2[PFD][16];                     // nq2: RMERGE's X[4096 - e] words
#pragma unroll
  for (int d = 0; d < PFD; ++d)
    if (tr0 + d * step < tend) fetch(nq[d], nq2[d], tr0 + d * step);
  // Loop entered after pass 1, as in cfft_fx4096_kernel: the wait for the prefetched words
  // then covers only the older loads (vmcnt = the younger stores + deeper prefetches).
  auto pass1 = [&](uint32_t (&buf)[16], uint32_t (&buf2)[16], uint32_t tr) {
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = pk(buf[u]);
    if constexpr (RMERGE) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int u = 4 * a + b;
          const short4 rc = recl[t + 256 * a + 1024 * b];
          const s16x2 y = pk(buf2[u]);
          const int2 m = rfft_merge_bin<int16_t>(make_int2(v[u].x, v[u].y), make_int2(y.x, y.y), rc.x, rc.y, rc.z, rc.w);
          v[u] = s16x2{(short)m.x, (short)m.y};
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
      bfly_pk<INV, 0>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], tw1[a][0], tw1[a][1], tw1[a][2]);
#pragma unroll
    for (int b = 0; b < 4; ++b) bfly_pk<INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], tw2[0], tw2[1], tw2[2]);
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) lds[s4096(t + 256 * a + 1024 * b)] = upk(v[4 * a + b]);
    if (tr + PFD * step < tend) fetch(buf, buf2, tr + PFD * step);
    __syncthreads();
  };
  if (tr0 >= tend) return;
  pass1(nq[0], nq2[0], tr0);
  uint32_t tr = tr0;
  auto pass23 = [&]() {
    const __amdgpu_buffer_rsrc_t rx = fx_rsrc(data + (size_t)tr * 4096, 4096 * 4);
    {
      const int base = 256 * q2 + j2;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) v[4 * a + b] = pk(lds[s4096(base + 64 * a + 16 * b)]);
#pragma unroll
      for (int b = 0; b < 4; ++b) bfly_pk<INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], TW3Q(b, 0), TW3Q(b, 1), TW3Q(b, 2));
#pragma unroll
      for (int a = 0; a < 4; ++a)
        bfly_pk<INV, 1>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], TW4Q(0), TW4Q(1), TW4Q(2));
      __syncthreads();
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) lds[s4096(base + 64 * a + 16 * b)] = upk(v[4 * a + b]);
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) v[4 * a + b] = pk(lds[s4096(16 * q3 + 4 * a + b)]);
#pragma unroll
    for (int b = 0; b < 4; ++b) bfly_pk<INV, 1>(v[b], v[4 + b], v[8 + b], v[12 + b], tw5[b][0], tw5[b][1], tw5[b][2]);
#pragma unroll
    for (int a = 0; a < 4; ++a) bfly_pk<INV, 2>(v[4 * a], v[4 * a + 1], v[4 * a + 2], v[4 * a + 3], z, z, z);
    if constexpr (SAT) {
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = pk_sat_add(v[u], v[u]);    // arm_shift_q15(+1): __SSAT(x << 1, 16)
    }
    if constexpr (BREV) {
#pragma unroll
      for (int u = 0; u < 16; ++u)
        __builtin_amdgcn_raw_buffer_store_b32((int)upk(v[u]), rx, vin, (int)(__brev((uint32_t)u) >> 28) * 1024, MI355X_FX_NT);
    } else {
#pragma unroll
      for (int u = 0; u < 16; ++u) __builtin_amdgcn_raw_buffer_store_b32((int)upk(v[u]), rx, 64 * q3, 4 * u, MI355X_FX_NT);
    }
    if constexpr (RSPLIT) {
      __syncthreads();                  // every thread's pass-3 LDS reads are done
#pragma unroll
      for (int u = 0; u < 16; ++u) lds[s4096((int)(__brev((uint32_t)u) >> 28) * 256 + t)] = upk(v[u]);
      __syncthreads();
      int16_t* y = rs.dst + (size_t)tr * (2 * 8192);
      auto get = [&](int i) {
        const uint32_t w = lds[s4096(i)];
        return make_int2((int)(int16_t)(w & 0xffffu), (int)(int16_t)(w >> 16));
      };
      const SplitStridedTab<int16_t> tab{rs.ta, rs.tb, rs.mod};
#pragma unroll 2
      for (int i = 0; i < 8; ++i) rfft_split_pair<int16_t>(get, y, t + 256 * i, 8192, tab);
    }                                   // (the next pass 1 starts with a barrier before its LDS writes)
  };
  for (;;) {
#pragma unroll
    for (int d = 0; d < PFD; ++d) {
      pass23();
      tr += step;
      if (tr >= tend) return;
      pass1(nq[(d + 1) % PFD], nq2[(d + 1) % PFD], tr);
    }
  }
}


// ============================================================================================
// A one-wave-per-transform q31 N = 4096 kernel (the one-wave f32 pattern; lane l holds x[l + 64m],
// one LDS transpose) was bit-exact but ran 273 vs 345 Gsamples/s: a 32 KiB transform needs 33 KiB
// of LDS per wave and 128 data VGPRs, leaving no room for the next transform's loads
// (profiles/r02/variants_fx4096w/).  Removed in round 3.

// The forward arm_rfft_q31 of N = 8192 in one launch: the inner CFFT-4096 (bit-reversed, pSrc
// overwritten as the reference leaves it) with the split fused into its last pass.
hipError_t rfft_q31_8192_fused_launch(int32_t* src, int32_t* dst, uint32_t batch, const int32_t* tw, const int32_t* ta,
                                      const int32_t* tb, uint32_t mod, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  auto k = cfft_fx4096_kernel<int32_t, false, true, false, true>;
  const int grid = fx_grid<MI355X_FX_T>((const void*)k, batch);
  RfSplitArgs<int32_t> rs;
  rs.dst = dst; rs.ta = ta; rs.tb = tb; rs.mod = mod;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (int2*)src, batch, (const int2*)tw, rs);
  return hipGetLastError();
}

hipError_t rfft_q15_8192_fused_launch(int16_t* src, int16_t* dst, uint32_t batch, const int16_t* tw, const int16_t* ta,
                                      const int16_t* tb, uint32_t mod, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  auto k = cfft_q15_4096_pk_kernel<false, true, false, true>;
  const int grid = fx_grid<MI355X_FXQ15_T>((const void*)k, batch);
  RfSplitArgs<int16_t> rs;
  rs.dst = dst; rs.ta = ta; rs.tb = tb; rs.mod = mod;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (short2*)src, batch, (const short2*)tw, rs);
  return hipGetLastError();
}

// The inverse arm_rfft_q31 of N = 8192 in one launch: spec [batch][16384] spectrum rows (bins
// 0..4096 read), dst [batch][8192]; rec = device_split_records(A, B, mod, 4096, 4).
hipError_t rfft_q31_8192_inv_fused_launch(const int32_t* spec, int32_t* dst, uint32_t batch, const int32_t* tw,
                                          const void* rec, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  auto k = cfft_fx4096_kernel<int32_t, true, true, true, false, true>;
  const int grid = fx_grid<MI355X_FX_T>((const void*)k, batch);
  RfSplitArgs<int32_t> rs;
  rs.spec = spec;
  rs.rec = (const int4*)rec;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (int2*)dst, batch, (const int2*)tw, rs);
  return hipGetLastError();
}

// The inverse arm_rfft_q15 of N = 8192 in one launch: spec [batch][16384] spectrum rows (bins
// 0..4096 read), dst [batch][8192]; rec = device_split_records(A, B, mod, 4096, 2).
hipError_t rfft_q15_8192_inv_fused_launch(const int16_t* spec, int16_t* dst, uint32_t batch, const int16_t* tw,
                                          const void* rec, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  auto k = cfft_q15_4096_pk_kernel<true, true, true, false, true>;
  const int grid = fx_grid<MI355X_FXQ15_T>((const void*)k, batch);
  RfSplitArgs<int16_t> rs;
  rs.spec = spec;
  rs.rec = (const short4*)rec;
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (short2*)dst, batch, (const short2*)tw, rs);
  return hipGetLastError();
}

template <typename T, bool INV, bool BREV, bool SAT>
static void launch_fx4096_t(void* data, uint32_t batch, const void* tw, hipStream_t st) {
  using C = typename Fx<T>::C;
  if constexpr (sizeof(T) == 2 && MI355X_FX_Q15_PACKED) {
    auto k = cfft_q15_4096_pk_kernel<INV, BREV, SAT>;
    const int grid = fx_grid<MI355X_FXQ15_T>((const void*)k, batch);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (short2*)data, batch, (const short2*)tw, RfSplitArgs<int16_t>{});
  } else {
    auto k = cfft_fx4096_kernel<T, INV, BREV, SAT>;
    const int grid = fx_grid<MI355X_FX_T>((const void*)k, batch);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, (C*)data, batch, (const C*)tw, RfSplitArgs<T>{});
  }
}

template <typename T, bool INV>
static void launch_fx4096_i(void* data, uint32_t batch, const void* tw, uint32_t flags, hipStream_t st) {
  const bool brev = flags & kBitrev, sat = flags & kSatShl1;
  if (brev && !sat) launch_fx4096_t<T, INV, true, false>(data, batch, tw, st);
  else if (brev) launch_fx4096_t<T, INV, true, true>(data, batch, tw, st);
  else if (!sat) launch_fx4096_t<T, INV, false, false>(data, batch, tw, st);
  else launch_fx4096_t<T, INV, false, true>(data, batch, tw, st);
}

template <typename T>
static hipError_t launch_fx4096(void* data, uint32_t batch, const void* tw, uint32_t flags, hipStream_t st) {
  if (flags & kIfft) launch_fx4096_i<T, true>(data, batch, tw, flags, st);
  else launch_fx4096_i<T, false>(data, batch, tw, flags, st);
  return hipGetLastError();
}

template <typename T, int N>
static hipError_t launch_fx(void* data, uint32_t batch, const void* tw, const uint16_t* perm,
                            uint32_t flags, hipStream_t st) {
  using P = PlanFx<N>;
  using C = typename Fx<T>::C;
  const uint32_t grid = (uint32_t)((batch + P::TPB - 1) / P::TPB);
  if (flags & kIfft)
    hipLaunchKernelGGL((cfft_fx_kernel<T, N, true>), dim3(grid), dim3(kBlock), 0, st,
                       (C*)data, batch, (const C*)tw, perm, flags);
  else
    hipLaunchKernelGGL((cfft_fx_kernel<T, N, false>), dim3(grid), dim3(kBlock), 0, st,
                       (C*)data, batch, (const C*)tw, perm, flags);
  return hipGetLastError();
}

template <typename T>
static hipError_t dispatch_fx(int n, void* data, uint32_t batch, const void* tw, const uint16_t* perm,
                              uint32_t flags, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  if (!perm) {   // the reference's own table: radix-16-pass kernels (the MFCC front end uses them too)
    const bool done = sizeof(T) == 4
        ? cfft_q31_r16_launch(n, (int32_t*)data, batch, (const int32_t*)tw, flags, st)
        : cfft_q15_r16_launch(n, (int16_t*)data, batch, (const int16_t*)tw, flags, st);
    if (done) return hipGetLastError();
  }
  switch (n) {
    case 16:   return launch_fx<T, 16>(data, batch, tw, perm, flags, st);
    case 32:   return launch_fx<T, 32>(data, batch, tw, perm, flags, st);
    case 64:   return launch_fx<T, 64>(data, batch, tw, perm, flags, st);
    case 128:  return launch_fx<T, 128>(data, batch, tw, perm, flags, st);
    case 256:  return launch_fx<T, 256>(data, batch, tw, perm, flags, st);
    case 512:  return launch_fx<T, 512>(data, batch, tw, perm, flags, st);
    case 1024: return launch_fx<T, 1024>(data, batch, tw, perm, flags, st);
    case 2048: return launch_fx<T, 2048>(data, batch, tw, perm, flags, st);
    case 4096:
      if (!perm) return launch_fx4096<T>(data, batch, tw, flags, st);   // reference table: specialist
      return launch_fx<T, 4096>(data, batch, tw, perm, flags, st);
    default:   return hipSuccess;   // reference: unsupported length is a silent no-op
  }
}

hipError_t cfft_q31_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st) {
  return dispatch_fx<int32_t>(n, data, batch, tw, perm, flags, st);
}
hipError_t cfft_q15_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st) {
  return dispatch_fx<int16_t>(n, data, batch, tw, perm, flags, st);
}

}  // namespace mi355x
