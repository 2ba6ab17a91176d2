// Batched FIR filters f32 / q15 — MI355X kernels, bit-exact.
//
// Replaces Source/FilteringFunctions/arm_fir_f32.c:911-1280 and arm_fir_q15.c:458-726
// (host scalar path, ARM_MATH_LOOPUNROLL on).  Per output n of a block, with the state
// s = [history (numTaps-1) ; block input]:
//   f32:  acc = 0.0f; for k in 0..T-1: acc = acc + s[n+k]*c[k]      (mul, then add; no FMA)
//   q15:  unrolled outputs (n < B - B%4): acc = sum over tap PAIRS of int32-wrapped
//         (s[n+2m]*c[2m] + s[n+2m+1]*c[2m+1])  -- the __SMLALD emulation, none.h:497-506;
//         tail outputs (n >= B - B%4): acc = sum of int64 products, taps in pairs (:649-681);
//         y = __SSAT(acc >> 15, 16).
//
// Geometry: one workgroup = one filter x a chunk of CHUNK outputs.  The chunk's input
// window (CHUNK + T - 1 samples) is staged into LDS with coalesced loads (history from
// the per-filter state, block samples from the input); each lane then produces R
// consecutive outputs with a register-rotated window, coefficients wave-uniform.
#include "common.hpp"
#include "kernels.hpp"

#include <type_traits>

#pragma clang fp contract(off)

namespace mi355x {

constexpr int kFirR = 8;                       // outputs per lane (fixed-point kernels)
constexpr int kFirChunk = kBlock * kFirR;      // outputs per workgroup (2048)
constexpr int kFirMaxTaps = 1024;              // LDS budget: (2048 + 1023) * 4 B

// Work items are (filter, chunk) pairs, item = f * nchunks + chunk.  The kernels are
// persistent (grid = what the CUs hold): while a workgroup filters item i from LDS, the
// window of item i + gridDim.x is already in flight into registers, so the HBM latency of
// the staging overlaps the MACs instead of stalling every co-resident workgroup at once.
struct FirItem {
  uint32_t f;
  int n0, count, total;   // first output, outputs in the chunk, window samples (count + T - 1)
  int a = 0;              // tap offset of the window (long filters run in tap segments)
};
__device__ __forceinline__ FirItem fir_item(uint32_t item, uint32_t nchunks, uint32_t B, int T1,
                                            int chunk = kFirChunk) {
  FirItem it;
  it.f = item / nchunks;
  it.n0 = (int)(item - it.f * nchunks) * chunk;
  it.count = min((int)B - it.n0, chunk);
  it.total = it.count + T1;
  return it;
}
// window sample j of an item: s[n0 + j] with s = [history (T-1) ; block input], 0 past the
// window.  Branch-free (pointer select, index clamped in bounds) so that a thread's loads
// all issue back to back instead of each waiting at a divergent join.
template <typename T>
__device__ __forceinline__ T fir_sample(const T* __restrict__ hist, const T* __restrict__ src, const FirItem& it,
                                        uint32_t B, int T1, int j) {
  const int sidx = it.n0 + it.a + min(j, it.total - 1);
  const T* p = sidx < T1 ? hist + ((uint64_t)it.f * T1 + sidx) : src + ((uint64_t)it.f * B + (sidx - T1));
  const T v = *p;
  return j < it.total ? v : (T)0;
}

// ---------------------------------------------------------------- f32
// fir_f32_kernel runs R = 16 outputs per lane (4096-output items) or R = 8 (2048): fir_f32_pass
// takes 8 when the 4096-output items would pad the outputs per filter by > 12 % more (e.g. the
// 4096 + 128 - 1 outputs of a convolution: 8192 against 6144 output slots).
template <int R> constexpr int kF32Chunk = kBlock * R;     // outputs per workgroup item
constexpr int kF32ChunkMin = kF32Chunk<8>;
constexpr int kFirPre = (kFirChunk + kFirMaxTaps - 1 + kBlock - 1) / kBlock;   // q31 window samples per thread

// LDS index with one pad word every 8: lanes read at a stride of R = 8 words from any
// offset, and i + i/8 keeps every ds_read_b32 32-lane group on 32 distinct banks (one
// pad per 32 words is conflict-free only at offsets that are multiples of 32).
__device__ __forceinline__ int padx(int i) { return i + (i >> 3); }

// ---- fir_f32_kernel: a register-window formulation with no ring rotation.
// A round is 8 consecutive taps k..k+7; output r of a lane (base = R * lane) needs window
// samples base + r + k .. base + r + k + 7, i.e. the R/8 + 1 8-sample groups from base + k.
// Four 8-register group buffers rotate by name over an unrolled block of four rounds: round q
// computes from buffers q .. q + R/8 while group q + R/8 + 1 is read from LDS, one round
// (8R VALU) ahead of its use, so every operand index is a compile-time constant and no register
// moves.  Coefficients are wave-uniform scalar loads into SGPRs (the v_mul operand: no VGPRs,
// no LDS reads); the loop is 2 VALU per tap and output (1 with FMA) plus a few per round.
// R = 16 (round 3) halves the LDS reads and the per-item overhead (barriers, staging) per MAC
// against R = 8 (PMC at R = 8: SQ_INSTS_VALU = 1.019 x the MAC minimum but VALU busy 82 %).
//
// LDS window layout: 8-sample group g at word gword(g) = 10 g (+ 2 when bit 4 of g is set, R =
// 16), so each 16-lane access of a group's ds_read2_b64 (lanes R/8 groups apart) lands on 32
// distinct banks; staging writes go through fir_stage_lane, a thread -> sample permutation under
// which every 32-lane ds_write_b32 group covers 32 distinct banks (round 2's identity mapping
// was two-way conflicted: 9.4 M conflict cycles per launch, profiles/r02/fir_f32/pmc.json).
// Both checked by tools/fir_lds_model.py.
template <int R> __host__ __device__ constexpr int gword(int g) { return 10 * g + (R == 16 ? 2 * ((g >> 4) & 1) : 0); }
template <int R> __host__ __device__ constexpr int wpos(int j) { return gword<R>(j >> 3) + (j & 7); }
__device__ __forceinline__ int fir_stage_lane(int tid) {
  const int h = tid >> 5, q = tid & 31, a = q >> 3, e = q & 7;
  return 8 * (16 * (h >> 2) + 4 * a + (h & 3)) + e;     // groups c, c+4, c+8, c+12 per half-wave
}

struct F32Grp { float v[8]; };
// group g of the window: two ds_read2_b64
template <int R>
__device__ __forceinline__ void ld_grp(F32Grp& g, const float* win, int grp) {
  const float2* q = reinterpret_cast<const float2*>(win + gword<R>(grp));
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const float2 x = q[h];
    g.v[2 * h] = x.x;
    g.v[2 * h + 1] = x.y;
  }
}
__device__ __forceinline__ void ld_coef(float (&c)[8], const float* cl, int k) {
  const float4 a = *reinterpret_cast<const float4*>(cl + k), b = *reinterpret_cast<const float4*>(cl + k + 4);
  c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w; c[4] = b.x; c[5] = b.y; c[6] = b.z; c[7] = b.w;
}
// one round: acc[r] += s[base + r + k + u] * c[k + u], u ascending (the reference's order);
// FMA: the opt-in tolerance path (arm_fir_f32_batch_fma), one v_fma_f32 per MAC in the same order
template <bool FMA>
__device__ __forceinline__ float f32_mac(float acc, float x, float c) {
  if constexpr (FMA) return __builtin_fmaf(x, c, acc);
  else return acc + x * c;
}
// groups A, B (, C for R = 16) hold window samples base + k + [0, 8), [8, 16), [16, 24)
template <int R, bool FMA>
__device__ __forceinline__ void f32_round(float (&acc)[R], const F32Grp& A, const F32Grp& B, const F32Grp& C,
                                          const float (&c)[8]) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float cu = c[u];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = r + u;
      acc[r] = f32_mac<FMA>(acc[r], j < 8 ? A.v[j] : j < 16 ? B.v[j - 8] : C.v[j - 16], cu);
    }
  }
#if MI355X_FIR_SCHED_BARRIER
  __builtin_amdgcn_sched_barrier(0);   // keep each round's products next to their adds
#endif
}

// R = 16 rounds with coefficients read from LDS one round ahead (the FMA path: v_fmac_f32
// takes its coefficient from a VGPR at full rate).  win: the window image, g: the lane's first
// group, cp: the unit's taps in LDS (read-ahead of up to 40 words past the last round).
template <bool FMA>
__device__ __forceinline__ void f32_rounds_ldsc(float (&acc)[16], const float* win, int g, const float* cp,
                                                int rounds) {
  constexpr int R = 16;
  F32Grp X0, X1, X2, X3;
  float c0[8], c1[8];
  ld_grp<R>(X0, win, g);
  ld_grp<R>(X1, win, g + 1);
  ld_grp<R>(X2, win, g + 2);
  ld_coef(c0, cp, 0);
  int nb = rounds >> 2;
  if (nb > 0) {
    do {
      ld_coef(c1, cp, 8);  ld_grp<R>(X3, win, g + 3); f32_round<R, FMA>(acc, X0, X1, X2, c0);
      ld_coef(c0, cp, 16); ld_grp<R>(X0, win, g + 4); f32_round<R, FMA>(acc, X1, X2, X3, c1);
      ld_coef(c1, cp, 24); ld_grp<R>(X1, win, g + 5); f32_round<R, FMA>(acc, X2, X3, X0, c0);
      ld_coef(c0, cp, 32); ld_grp<R>(X2, win, g + 6); f32_round<R, FMA>(acc, X3, X0, X1, c1);
      g += 4;
      cp += 32;
    } while (--nb);
  }
  const int rem = rounds & 3;
  if (rem > 0) {
    ld_coef(c1, cp, 8);
    ld_grp<R>(X3, win, g + 3);
    f32_round<R, FMA>(acc, X0, X1, X2, c0);
    if (rem > 1) {
      ld_coef(c0, cp, 16);
      ld_grp<R>(X0, win, g + 4);
      f32_round<R, FMA>(acc, X1, X2, X3, c1);
      if (rem > 2) f32_round<R, FMA>(acc, X2, X3, X0, c0);
    }
  }
}

// Window rows staged per thread: KPRE * 256 >= chunk + T + 8 (the last block reads one group
// past its taps), so the LDS image, the staging loads and the zero tail scale with numTaps.
template <int R> __host__ __device__ constexpr int fir_f32_kpre(int T) { return (kF32Chunk<R> + T + 8 + kBlock - 1) / kBlock; }

// Window staging of one item into registers, through buffer resources: window sample j is
// block sample s = n0 - T1 + j, read from [0, n0 + count) of the filter's block (a negative
// offset or one past the window is out of range and returns 0), OR-ed with history word
// n0 + j, read from [0, T1) of the filter's history (only the first chunk, n0 < T1, reaches
// it).  The per-row offsets pass through an empty asm so that the compiler cannot split a
// constant part into the instruction's immediate: the range check takes the VGPR offset
// alone, and a negative one would not be wrapped back into range by a positive immediate.
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
// Rows k >= KPRE - R never reach the history (T1 < 256 (KPRE - R)); the history words are
// kept apart and OR-ed in when the window is written to LDS, so no wait is placed before the
// MACs that the fetch is meant to overlap.  A tap segment of a long filter (LONG, numTaps >
// kFirSeg) starts a tap offset a into s, so any row can reach the history: all rows get one.
template <int R, int KPRE, bool LONG>
struct F32Win {
  static constexpr int kH = LONG ? KPRE : KPRE - R;
  int x[KPRE];
  int h[kH];
};
// Input addressing of fir_f32_kernel: filter f reads block samples from src + f * stride, of
// which the first len are valid (beyond, and before 0, reads return 0), shifted by so (window
// sample j of the chunk at n0 is block sample n0 - T1 + j + so), with the history (T1 words at
// hist_in + f * T1) in front when hist != 0; coefficients at coeffs + f * cstride.
//   FIR / multirate: {B, B, 0, 1, 0};  convolution family: x rows, so = first output, no history.
struct FirIn {
  uint64_t stride;
  uint32_t len;
  int so;
  uint32_t hist;
  uint64_t cstride;
};
// window of the tap segment starting at tap a: sample j = s[n0 + a + j]
template <int R, int KPRE, bool LONG>
__device__ __forceinline__ void fir_f32_fetch(F32Win<R, KPRE, LONG>& w, const FirItem& it, const float* __restrict__ src,
                                              const float* __restrict__ hist_in, const FirIn& in, int T1, int jl) {
  // jl = fir_stage_lane(thread): the row sample this thread stages
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(src + it.f * in.stride, in.len * 4u);
  const __amdgpu_buffer_rsrc_t rh = in.hist ? buf_rsrc(hist_in + (uint64_t)it.f * T1, (uint32_t)T1 * 4u)
                                            : buf_rsrc(src, 0u);
  const int v0 = (jl + it.n0 + it.a - T1 + in.so) * 4, h0 = (jl + it.n0 + it.a) * 4;
#pragma unroll
  for (int k = 0; k < KPRE; ++k) w.x[k] = __builtin_amdgcn_raw_buffer_load_b32(r, opaque(v0 + 1024 * k), 0, 0);
#pragma unroll
  for (int k = 0; k < w.kH; ++k)
    w.h[k] = __builtin_amdgcn_raw_buffer_load_b32(rh, opaque(h0 + 1024 * k), 0, 0);   // past the history: 0
}
// Rows are 320 words apart (a multiple of 64), so the compiler would pair them into
// ds_write2st64_b32, which is banked like ds_write_b64 (16-lane groups, both dwords of a lane
// on one bank: 2-way conflicted).  Volatile stores stay single ds_write_b32 (32-lane groups,
// conflict free under fir_stage_lane).
template <int R, int KPRE, bool LONG>
__device__ __forceinline__ void fir_f32_put(float* wl, const F32Win<R, KPRE, LONG>& w) {
  auto* v = (__attribute__((address_space(3))) volatile float*)wl;
#pragma unroll
  for (int k = 0; k < KPRE; ++k)
    v[wpos<R>(k * kBlock)] = __builtin_bit_cast(float, k < w.kH ? (w.x[k] | w.h[k < w.kH ? k : 0]) : w.x[k]);
}

// FMA path: the unit's taps are staged to LDS with its window and read as broadcast VGPRs,
// because v_fmac_f32 with an SGPR operand issues at half rate on gfx950 (a VGPR coefficient:
// full rate; tools/probes/fmac_bank.hip, profiles/r03/probe_fmac_bank.txt), while the
// bit-exact path's v_mul_f32 takes its SGPR coefficient at full rate.  Thread t holds taps
// t + 256 q of the next unit (zero past Ts: range-checked loads).
constexpr int kFirSeg = kFirMaxTaps;
struct F32Coef {
  int c[kFirSeg / kBlock];
};
__device__ __forceinline__ void fir_f32_cfetch(F32Coef& w, const float* __restrict__ coeffs, const FirItem& it,
                                               const FirIn& in, int Ts, int tid) {
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(coeffs + it.f * in.cstride + it.a, (uint32_t)Ts * 4u);
#pragma unroll
  for (int q = 0; q < kFirSeg / kBlock; ++q) w.c[q] = __builtin_amdgcn_raw_buffer_load_b32(r, opaque((tid + kBlock * q) * 4), 0, 0);
}
__device__ __forceinline__ void fir_f32_cput(float* cl, const F32Coef& w, int tid) {
#pragma unroll
  for (int q = 0; q < kFirSeg / kBlock; ++q) cl[tid + kBlock * q] = __builtin_bit_cast(float, w.c[q]);
}

// Items per workgroup.  Workgroups of identical work started together finish together, so with
// one item each every generation of co-resident workgroups stages its window at the same time
// and the SIMDs idle for the load latency (≈10 % of the launch, PMC: 89.5 % VALU busy).  A
// workgroup instead walks ipw consecutive items with the next item's window in registers
// while it filters the current one.  MI355X_FIR_IPW > 0: fixed ipw (default 16); 0: ipw =
// items / (resident workgroups x CUs), one generation of persistent workgroups.  Measured at
// 2^17 items (Gsamples/s): ipw 1 209, 2 214, 4 216, 8 219, 16 217-222, 32 210-215,
// persistent (64) 206-208.

// Output lattice of fir_f32_kernel: output n of filter f (n % M == 0 only) is stored at
// y[f per_filter + off + dir ((n / M) L + q)]: the FIR {1, 1, 0, 1, 0, B}; the decimator
// {M, 1, 0, 1, 0, B / M}; the convolution family {1, 1, 0, ydir, yoff + ydir first, sy}.
// M = L = dir = 1 is a contiguous run (16-B stores when aligned).
struct FirOut {
  uint32_t M, L, q;
  int dir;
  int64_t off;
  uint64_t per_filter;
};

// Long filters (numTaps > kFirSeg) run in tap segments of kFirSeg: a work unit is (item,
// segment), the accumulators stay in registers from a unit with segment 0 to the one with the
// last segment, so every output still sums its products k = 0, 1, .., numTaps - 1 in order.
struct FirUnit {
  FirItem it;
  int Ts;              // taps in this segment
  bool first, last;    // first / last segment of the item
};
template <int R, bool LONG>
__device__ __forceinline__ FirUnit fir_unit(uint32_t u, uint32_t nseg, uint32_t nchunks, uint32_t B, int T) {
  FirUnit x;
  const uint32_t item = LONG ? u / nseg : u;
  const int seg = LONG ? (int)(u - item * nseg) : 0;
  x.it = fir_item(item, nchunks, B, T - 1, kF32Chunk<R>);
  x.it.a = seg * kFirSeg;
  x.Ts = LONG ? min(T - x.it.a, kFirSeg) : T;
  x.first = seg == 0;
  x.last = !LONG || seg == (int)nseg - 1;
  return x;
}
// (Round 4 measured a double-buffered-window variant -- two LDS images, one barrier per item,
// VERDICT r3 item 7 -- at 212.7 vs 215-216 Gsamples/s for this kernel on the same box, bit-exact:
// at three workgroups per CU instead of five the staging it overlaps is worth less than the
// occupancy it costs; not kept.  profiles/r04/README.md.)
template <int R, int KPRE, bool LONG, bool FMA>
__global__ __launch_bounds__(kBlock, LONG ? (FMA ? 3 : 4) : FMA ? MI355X_FIR_F32_FMA_WAVES : MI355X_FIR_F32_WAVES(R)) void fir_f32_kernel(
    const float* __restrict__ coeffs, int T, const float* __restrict__ src, float* __restrict__ dst, uint32_t B,
    const float* __restrict__ hist_in, uint32_t nchunks, uint32_t items, uint32_t ipw, FirIn in, FirOut fo) {
  static_assert(R == 16 || (R == 8 && !FMA), "R = 16, or R = 8 for the bit-exact path");
  constexpr int kWin = KPRE * kBlock;
  __shared__ __attribute__((aligned(16))) float win[wpos<R>(kWin) + 32];
  __shared__ __attribute__((aligned(16))) float cl[FMA ? kFirSeg + 64 : 4];   // FMA: the unit's taps (+ read-ahead)
  const int T1 = T - 1;
  const uint32_t i0 = blockIdx.x * ipw;
  if (i0 >= items) return;
  const uint32_t nseg = LONG ? (uint32_t)((T + kFirSeg - 1) / kFirSeg) : 1u;
  const uint32_t u0 = i0 * nseg, u1 = min(items, i0 + ipw) * nseg;
  const int tid = threadIdx.x;
  const int base = tid * R;                         // local output index of this lane
  const int jl = fir_stage_lane(tid);               // the row sample this thread stages
  float* wl = win + wpos<R>(jl);                       // wpos(jl + 256 k) = wpos(jl) + 320 k
  F32Win<R, KPRE, LONG> pre;
  F32Coef pc;
  FirUnit cur = fir_unit<R, LONG>(u0, nseg, nchunks, B, T);
  fir_f32_fetch<R, KPRE, LONG>(pre, cur.it, src, hist_in, in, T1, jl);
  fir_f32_put<R, KPRE, LONG>(wl, pre);
  if constexpr (FMA) {
    fir_f32_cfetch(pc, coeffs, cur.it, in, cur.Ts, tid);
    fir_f32_cput(cl, pc, tid);
  }
  float acc[R];
  // Per unit: barrier (window ready) -> next window's loads -> MACs -> barrier (window free)
  // -> next window to LDS -> output stores.  The window write waits only for loads that had a
  // whole unit of MACs to land; the stores are issued after it, so no wait ever covers them.
  for (uint32_t u = u0;;) {
    __syncthreads();
    const bool more = u + 1 < u1;
    const FirUnit nxt = more ? fir_unit<R, LONG>(u + 1, nseg, nchunks, B, T) : cur;
    if (more) fir_f32_fetch<R, KPRE, LONG>(pre, nxt.it, src, hist_in, in, T1, jl);
    if (FMA && more) fir_f32_cfetch(pc, coeffs, nxt.it, in, nxt.Ts, tid);
    if (base < cur.it.count) {
      if (cur.first) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0f;
      }
      const int Ts = cur.Ts, rounds = Ts >> 3;
      F32Grp X0, X1, X2, X3;
      float c0[8], c1[8];
      // Four group buffers rotate by name over a block of four rounds; round q uses buffers
      // q .. q + R/8 and reads group q + R/8 + 1.  Coefficients are wave-uniform: scalar loads
      // (s_load_dwordx8 per round) into SGPRs, the v_mul operand (no VGPRs, no LDS reads).
      int g = base >> 3;                            // the lane's first group
      const float* const ci = coeffs + cur.it.f * in.cstride + cur.it.a;
      const float* cp = FMA ? cl : ci;
      ld_grp<R>(X0, win, g);
      ld_grp<R>(X1, win, g + 1);
      if constexpr (R == 16) ld_grp<R>(X2, win, g + 2);
      int nb = rounds >> 2;
      if constexpr (FMA && R == 16) {
        f32_rounds_ldsc<FMA>(acc, win, g, cp, rounds);
      } else {
      if (nb > 0) {
        do {
          if constexpr (R == 8) {
            ld_coef(c0, cp, 0);  ld_grp<R>(X2, win, g + 2); f32_round<R, FMA>(acc, X0, X1, X1, c0);
            ld_coef(c1, cp, 8);  ld_grp<R>(X3, win, g + 3); f32_round<R, FMA>(acc, X1, X2, X2, c1);
            ld_coef(c0, cp, 16); ld_grp<R>(X0, win, g + 4); f32_round<R, FMA>(acc, X2, X3, X3, c0);
            ld_coef(c1, cp, 24); ld_grp<R>(X1, win, g + 5); f32_round<R, FMA>(acc, X3, X0, X0, c1);
          } else {
            ld_coef(c0, cp, 0);  ld_grp<R>(X3, win, g + 3); f32_round<R, FMA>(acc, X0, X1, X2, c0);
            ld_coef(c1, cp, 8);  ld_grp<R>(X0, win, g + 4); f32_round<R, FMA>(acc, X1, X2, X3, c1);
            ld_coef(c0, cp, 16); ld_grp<R>(X1, win, g + 5); f32_round<R, FMA>(acc, X2, X3, X0, c0);
            ld_coef(c1, cp, 24); ld_grp<R>(X2, win, g + 6); f32_round<R, FMA>(acc, X3, X0, X1, c1);
          }
          g += 4;
          cp += 32;
        } while (--nb);
      }
      // 0..3 remaining whole rounds, same buffer order
      const int rem = rounds & 3;
      if (rem > 0) {
        if constexpr (R == 8) {
          ld_coef(c0, cp, 0);
          ld_grp<R>(X2, win, g + 2);
          f32_round<R, FMA>(acc, X0, X1, X1, c0);
          if (rem > 1) {
            ld_coef(c1, cp, 8);
            ld_grp<R>(X3, win, g + 3);
            f32_round<R, FMA>(acc, X1, X2, X2, c1);
            if (rem > 2) {
              ld_coef(c0, cp, 16);
              f32_round<R, FMA>(acc, X2, X3, X3, c0);
            }
          }
        } else {
          ld_coef(c0, cp, 0);
          ld_grp<R>(X3, win, g + 3);
          f32_round<R, FMA>(acc, X0, X1, X2, c0);
          if (rem > 1) {
            ld_coef(c1, cp, 8);
            ld_grp<R>(X0, win, g + 4);
            f32_round<R, FMA>(acc, X1, X2, X3, c1);
            if (rem > 2) {
              ld_coef(c0, cp, 16);
              f32_round<R, FMA>(acc, X2, X3, X0, c0);
            }
          }
        }
      }
      }
      // numTaps % 8 tail taps, straight from LDS
      for (int k = 8 * rounds; k < Ts; ++k) {
        const float c = ci[k];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = f32_mac<FMA>(acc[r], win[wpos<R>(base + k + r)], c);
      }
    }
    if (more) {
      __syncthreads();                              // every wave is done reading this window
      fir_f32_put<R, KPRE, LONG>(wl, pre);
      if constexpr (FMA) fir_f32_cput(cl, pc, tid);
    }
    if (cur.last && base < cur.it.count) {
      const FirItem& it = cur.it;
      const bool run = fo.M == 1 && fo.L == 1 && fo.dir == 1;
      if (run) {                                    // contiguous outputs
        float* o = dst + it.f * fo.per_filter + fo.off + it.n0 + base;
        if (((fo.per_filter | (uint64_t)fo.off) & 3u) == 0 && ((uintptr_t)dst & 15u) == 0 && base + R <= it.count) {
#pragma unroll
          for (int q = 0; q < R / 4; ++q)
            reinterpret_cast<float4*>(o)[q] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (base + r < it.count) o[r] = acc[r];
        }
      } else {                                      // decimator / reversed runs
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t n = (uint32_t)(it.n0 + base + r);
          if (base + r < it.count && n % fo.M == 0)
            dst[(int64_t)(it.f * fo.per_filter) + fo.off + (int64_t)fo.dir * ((int64_t)(n / fo.M) * fo.L + fo.q)] =
                acc[r];
        }
      }
    }
    if (!more) break;
    cur = nxt;
    ++u;
  }
}

// ---------------------------------------------------------------- q15
// A tap pair (c[2m], c[2m+1]) times a sample pair is one v_dot2_i32_i16 whose int32 result
// wraps exactly like __SMLALD's pair sum (none.h:497-506).  The window is staged as words of
// two samples, in four LDS planes: even pairs E[i] = (x[2i], x[2i+1]) and odd pairs
// O[i] = (x[2i+1], x[2i+2]), each split into x>>8 ("h") and x&255 ("l") halves.  A lane's
// R = 8 outputs need words wb+m .. wb+m+3 of every plane at tap pair m: one ds_read_b128 per
// plane per 4 pairs (lane stride 16 B: conflict-free) feeds 64 v_dot2.
typedef short s16x2 __attribute__((ext_vector_type(2)));
constexpr int kQ15W = (kFirChunk + kFirMaxTaps) / 2 + 16;   // words per plane (+ look-ahead)
constexpr int kQ15Chunk = 120;                               // tap pairs per int32 flush

__device__ __forceinline__ int32_t dot2(uint32_t x, uint32_t c, int32_t acc) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, x), __builtin_bit_cast(s16x2, c), acc, false);
}
__device__ __forceinline__ uint32_t hi8(uint32_t w) { return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, w) >> (short)8); }
__device__ __forceinline__ uint32_t lo8(uint32_t w) { return w & 0x00FF00FFu; }
__device__ __forceinline__ uint32_t join8(uint32_t h, uint32_t l) { return ((h << 8) & 0xFF00FF00u) | l; }
__device__ __forceinline__ uint32_t lane_word(const uint4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

// Split accumulation, valid when no coefficient pair is (-32768, -32768) -- only then can an
// int32 pair sum wrap, and without wraps the unrolled and tail outputs (arm_fir_q15.c:482-640
// vs :649-681) both equal the exact sum:  sum = 256*H + L  with  H = sum(h*c), L = sum(l*c),
// int32-exact over kQ15Chunk pairs (|H| <= 2^30, 0 <= L < 255*2^15*240 < 2^31), flushed to
// int64 after each chunk.
struct Q15Ring { uint4 eh[3], el[3], oh[3], ol[3]; };   // three 4-word quads per plane

template <int S>
__device__ __forceinline__ void q15_fetch(Q15Ring& r, const uint32_t* lds, int w) {
  r.eh[S] = *reinterpret_cast<const uint4*>(lds + 0 * kQ15W + w);
  r.el[S] = *reinterpret_cast<const uint4*>(lds + 1 * kQ15W + w);
  r.oh[S] = *reinterpret_cast<const uint4*>(lds + 2 * kQ15W + w);
  r.ol[S] = *reinterpret_cast<const uint4*>(lds + 3 * kQ15W + w);
}

// 4 tap pairs starting at a multiple of 4 held in slot P (the next quad in slot P+1); the
// quad after that is fetched into the free slot first, one block ahead of its use.
template <int P>
__device__ __forceinline__ void q15_block(Q15Ring& r, const uint32_t* lds, int w_ahead, const uint4 c4,
                                          int32_t (&H)[kFirR], int32_t (&L)[kFirR]) {
  q15_fetch<(P + 2) % 3>(r, lds, w_ahead);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t c = lane_word(c4, u);
#pragma unroll
    for (int j = 0; j < kFirR / 2; ++j) {
      const int i = u + j, s = i < 4 ? P : (P + 1) % 3, e = i & 3;
      H[2 * j] = dot2(lane_word(r.eh[s], e), c, H[2 * j]);
      L[2 * j] = dot2(lane_word(r.el[s], e), c, L[2 * j]);
      H[2 * j + 1] = dot2(lane_word(r.oh[s], e), c, H[2 * j + 1]);
      L[2 * j + 1] = dot2(lane_word(r.ol[s], e), c, L[2 * j + 1]);
    }
  }
}

template <bool kFlush>   // pairs > kQ15Chunk: fold H, L into int64 every kQ15Chunk pairs
__device__ __forceinline__ void fir_q15_split(const uint32_t* lds, const uint32_t* cw, int pairs, int wb,
                                              int64_t (&acc)[kFirR]) {
  int32_t H[kFirR], L[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) { H[r] = 0; L[r] = 0; acc[r] = 0; }
  const uint4* c4 = reinterpret_cast<const uint4*>(cw);
  Q15Ring r;
  q15_fetch<0>(r, lds, wb);
  q15_fetch<1>(r, lds, wb + 4);
  int m = 0, blocks = 0;
  for (; m + 12 <= pairs; m += 12) {
    q15_block<0>(r, lds, wb + m + 8, c4[m / 4], H, L);
    q15_block<1>(r, lds, wb + m + 12, c4[m / 4 + 1], H, L);
    q15_block<2>(r, lds, wb + m + 16, c4[m / 4 + 2], H, L);
    if (kFlush && ++blocks == kQ15Chunk / 12) {
      blocks = 0;
#pragma unroll
      for (int k = 0; k < kFirR; ++k) { acc[k] += (int64_t)H[k] * 256 + L[k]; H[k] = 0; L[k] = 0; }
    }
  }
  if (m + 4 <= pairs) {
    q15_block<0>(r, lds, wb + m + 8, c4[m / 4], H, L);
    m += 4;
    if (m + 4 <= pairs) {
      q15_block<1>(r, lds, wb + m + 8, c4[m / 4], H, L);
      m += 4;
    }
  }
  for (; m < pairs; ++m) {                         // pairs % 4 leftovers, straight from LDS
    const uint32_t c = cw[m];
#pragma unroll
    for (int j = 0; j < kFirR / 2; ++j) {
      const int w = wb + m + j;
      H[2 * j] = dot2(lds[w], c, H[2 * j]);
      L[2 * j] = dot2(lds[kQ15W + w], c, L[2 * j]);
      H[2 * j + 1] = dot2(lds[2 * kQ15W + w], c, H[2 * j + 1]);
      L[2 * j + 1] = dot2(lds[3 * kQ15W + w], c, L[2 * j + 1]);
    }
  }
#pragma unroll
  for (int k = 0; k < kFirR; ++k) acc[k] += (int64_t)H[k] * 256 + L[k];
}

// General accumulation: int64 sum of int32 pair sums; outputs at or past `tail_from` (the
// blockSize%4 tail, arm_fir_q15.c:649-681) add the unwrapped pair sum instead.  A pair sum
// is INT32_MIN only when it wrapped from +2^31 (the most negative true pair sum is
// -2147418112), so the tail correction is exact.
__device__ __forceinline__ void fir_q15_wide(const uint32_t* lds, const uint32_t* cw, int pairs, int wb,
                                             int tail_from, int64_t (&acc)[kFirR]) {
#pragma unroll
  for (int r = 0; r < kFirR; ++r) acc[r] = 0;
  for (int m = 0; m < pairs; ++m) {
    const uint32_t c = cw[m];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) {
      const int w = wb + m + r / 2, plane = (r & 1) ? 2 : 0;
      const int32_t p = dot2(join8(lds[plane * kQ15W + w], lds[(plane + 1) * kQ15W + w]), c, 0);
      acc[r] += (r >= tail_from && p == INT32_MIN) ? (int64_t)2147483648LL : (int64_t)p;
    }
  }
}

// arm_fir_fast_q15: mod-2^32 sum over all tap pairs with one accumulating v_dot2 each,
// planes 0/1 hold the raw even / odd sample-pair words; 4-word quads read one block ahead.
struct Q15FastRing { uint4 e[3], o[3]; };
template <int S>
__device__ __forceinline__ void q15f_fetch(Q15FastRing& r, const uint32_t* lds, int w) {
  r.e[S] = *reinterpret_cast<const uint4*>(lds + w);
  r.o[S] = *reinterpret_cast<const uint4*>(lds + kQ15W + w);
}
template <int P>
__device__ __forceinline__ void q15f_block(Q15FastRing& r, const uint32_t* lds, int w_ahead, const uint4 c4,
                                           int32_t (&A)[kFirR]) {
  q15f_fetch<(P + 2) % 3>(r, lds, w_ahead);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t c = lane_word(c4, u);
#pragma unroll
    for (int j = 0; j < kFirR / 2; ++j) {
      const int i = u + j, s = i < 4 ? P : (P + 1) % 3, e = i & 3;
      A[2 * j] = dot2(lane_word(r.e[s], e), c, A[2 * j]);
      A[2 * j + 1] = dot2(lane_word(r.o[s], e), c, A[2 * j + 1]);
    }
  }
}
__device__ __forceinline__ void fir_q15_fast(const uint32_t* lds, const uint32_t* cw, int pairs, int wb,
                                             int32_t (&A)[kFirR]) {
#pragma unroll
  for (int k = 0; k < kFirR; ++k) A[k] = 0;
  const uint4* c4 = reinterpret_cast<const uint4*>(cw);
  Q15FastRing r;
  q15f_fetch<0>(r, lds, wb);
  q15f_fetch<1>(r, lds, wb + 4);
  int m = 0;
  for (; m + 12 <= pairs; m += 12) {
    q15f_block<0>(r, lds, wb + m + 8, c4[m / 4], A);
    q15f_block<1>(r, lds, wb + m + 12, c4[m / 4 + 1], A);
    q15f_block<2>(r, lds, wb + m + 16, c4[m / 4 + 2], A);
  }
  if (m + 4 <= pairs) {
    q15f_block<0>(r, lds, wb + m + 8, c4[m / 4], A);
    m += 4;
    if (m + 4 <= pairs) {
      q15f_block<1>(r, lds, wb + m + 8, c4[m / 4], A);
      m += 4;
    }
  }
  for (; m < pairs; ++m) {
    const uint32_t c = cw[m];
#pragma unroll
    for (int j = 0; j < kFirR / 2; ++j) {
      A[2 * j] = dot2(lds[wb + m + j], c, A[2 * j]);
      A[2 * j + 1] = dot2(lds[kQ15W + wb + m + j], c, A[2 * j + 1]);
    }
  }
}

// FAST = arm_fir_fast_q15 (arm_fir_fast_q15.c): the accumulator is a q31_t fed by __SMLAD /
// __SMLADX and plain int32 adds (none.h) -- every partial sum wraps mod 2^32, so the result
// is the mod-2^32 sum of the products in ANY order: one accumulating v_dot2 per tap pair on
// the raw sample-pair words (planes 0/1 = even/odd pairs), y = __SSAT(acc >> 15, 16).
// numTaps > kFirMaxTaps: the window and the tap pairs are staged per segment of kFirMaxTaps
// taps (an even count, so pairs never straddle segments) and the segment sums are added in
// int64 (the reference's accumulator is one q63 sum of the pair sums: order-free).
template <bool FAST, bool LONG>
__global__ __launch_bounds__(kBlock, MI355X_FIR_Q15_WAVES) void fir_q15_kernel(const int16_t* __restrict__ coeffs, int T,
                                                         const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                         uint32_t B, const int16_t* __restrict__ hist_in,
                                                         uint32_t nchunks) {
  __shared__ uint4 lds4[kQ15W];                    // 4 planes x kQ15W words
  __shared__ uint4 cw4[kFirMaxTaps / 8];           // tap pairs as words
  uint32_t* lds = reinterpret_cast<uint32_t*>(lds4);
  uint32_t* cw = reinterpret_cast<uint32_t*>(cw4);
  const int T1 = T - 1;
  const FirItem it0 = fir_item(blockIdx.x, nchunks, B, T1);
  const int base = threadIdx.x * kFirR;
  const bool active = base < it0.count;
  int64_t tot[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) tot[r] = 0;
  for (int a = 0; a < (LONG ? T : 1); a += kFirMaxTaps) {   // !LONG: one pass, T <= kFirMaxTaps
    const int Ts = LONG ? min(T - a, kFirMaxTaps) : T;
    FirItem it = it0;
    it.a = a;
    it.total = it.count + Ts - 1;
    if (LONG && a) __syncthreads();                          // the previous segment is done with LDS
    // staging: every load of this thread is issued before the first LDS write
    const int words = min((it.total + 1) / 2 + 12, kQ15W);
    constexpr int kPer = (kQ15W + kBlock - 1) / kBlock;
    uint32_t x[kPer][3];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = threadIdx.x + k * kBlock;
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        const int i = 2 * j + h;
        x[k][h] = (uint16_t)fir_sample(hist_in, src, it, B, T1, i);
      }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = threadIdx.x + k * kBlock;
      if (j < words) {
        const uint32_t e = x[k][0] | (x[k][1] << 16), o = x[k][1] | (x[k][2] << 16);
        if constexpr (FAST) {
          lds[j] = e;
          lds[kQ15W + j] = o;
        } else {
          lds[j] = hi8(e);
          lds[kQ15W + j] = lo8(e);
          lds[2 * kQ15W + j] = hi8(o);
          lds[3 * kQ15W + j] = lo8(o);
        }
      }
    }
    const int pairs = Ts >> 1;
    const int16_t* cs = coeffs + a;
    int wrap = 0;
    for (int m = threadIdx.x; m < pairs; m += kBlock) {
      const uint32_t c = (uint32_t)(uint16_t)cs[2 * m] | ((uint32_t)(uint16_t)cs[2 * m + 1] << 16);
      cw[m] = c;
      wrap |= c == 0x80008000u;
    }
    const bool split = !__syncthreads_or(wrap);
    if (active) {
      int64_t acc[kFirR];
      if constexpr (FAST) {
        int32_t a32[kFirR];
        fir_q15_fast(lds, cw, pairs, base >> 1, a32);
#pragma unroll
        for (int r = 0; r < kFirR; ++r) acc[r] = a32[r];
      } else if (split && pairs <= kQ15Chunk) {
        fir_q15_split<false>(lds, cw, pairs, base >> 1, acc);
      } else if (split) {
        fir_q15_split<true>(lds, cw, pairs, base >> 1, acc);
      } else {
        const int unrolled_end = (int)(B - (B & 3u));  // outputs before this use the pair-wrap path
        fir_q15_wide(lds, cw, pairs, base >> 1, unrolled_end - (it.n0 + base), acc);
      }
#pragma unroll
      for (int r = 0; r < kFirR; ++r) tot[r] += acc[r];
    }
  }
  if (!active) return;
  int16_t y[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) {
    // FAST: the q31_t accumulator wraps mod 2^32 (acc >> 15 of the int32 sum)
    const int64_t acc = FAST ? (int64_t)(int32_t)(uint32_t)(uint64_t)tot[r] : tot[r];
    y[r] = (int16_t)ssat16((int32_t)(acc >> 15));   // arm_fir_q15.c:674
  }
  int16_t* o = dst + (uint64_t)it0.f * B + it0.n0 + base;
  if ((B & 7u) == 0 && ((uintptr_t)dst & 15u) == 0 && base + kFirR <= it0.count) {
    *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(y);
  } else {
#pragma unroll
    for (int r = 0; r < kFirR; ++r)
      if (base + r < it0.count) o[r] = y[r];
  }
}

// ---------------------------------------------------------------- q31 (exact and fast)
// arm_fir_q31 (arm_fir_q31.c, LOOPUNROLL by 3 and tail alike): q63 accumulator of exact
// q31 x q31 products, y = (q31)(acc >> 31).  arm_fir_fast_q31 (arm_fir_fast_q31.c):
// multAcc_32x32_keep32_R(acc, x, c) = (q31)(((q63)acc << 32) + x*c + 2^31) >> 32)
// = acc + ((x*c + 2^31) >> 32) mod 2^32 (acc << 32 has a zero low word), y = (q31)(acc << 1).
// Both accumulators only ever wrap (gcc x86-64 semantics of the reference build): the
// results are mod-2^64 / mod-2^32 sums, the same in any order.  Structure as fir_f32.
template <bool FAST, bool LONG>
__global__ __launch_bounds__(kBlock) void fir_q31_kernel(const int32_t* __restrict__ coeffs, int T,
                                                         const int32_t* __restrict__ src, int32_t* __restrict__ dst,
                                                         uint32_t B, const int32_t* __restrict__ hist_in,
                                                         uint32_t nchunks) {
  __shared__ int32_t win[(kFirChunk + kFirMaxTaps) * 9 / 8 + 32];
  const int T1 = T - 1;
  const FirItem it0 = fir_item(blockIdx.x, nchunks, B, T1);
  const int base = threadIdx.x * kFirR;
  const bool active = base < it0.count;
  using Acc = typename std::conditional<FAST, uint32_t, uint64_t>::type;
  Acc acc[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) acc[r] = 0;
  auto mac = [](Acc a, int32_t x, int32_t c) -> Acc {
    const int64_t p = (int64_t)x * c;
    if constexpr (FAST) return a + (uint32_t)((p + 0x80000000LL) >> 32);
    else return a + (uint64_t)p;
  };
  // numTaps > kFirMaxTaps: one window per tap segment, the modular sums carried in registers
  for (int a = 0; a < (LONG ? T : 1); a += kFirMaxTaps) {   // !LONG: one pass, T <= kFirMaxTaps
    const int Ts = LONG ? min(T - a, kFirMaxTaps) : T;
    FirItem it = it0;
    it.a = a;
    it.total = it.count + Ts - 1;
    if (LONG && a) __syncthreads();
    int32_t pre[kFirPre];
#pragma unroll
    for (int k = 0; k < kFirPre; ++k) pre[k] = fir_sample(hist_in, src, it, B, T1, (int)threadIdx.x + k * kBlock);
#pragma unroll
    for (int k = 0; k < kFirPre; ++k) {
      const int j = threadIdx.x + k * kBlock;
      if (j < it.total) win[padx(j)] = pre[k];
    }
    __syncthreads();
    if (!active) continue;
    const int32_t* cs = coeffs + a;
    int32_t w[kFirR];
#pragma unroll
    for (int r = 0; r < kFirR; ++r) w[r] = win[padx(base + r)];
    int k = 0;
    for (; k + kFirR <= Ts; k += kFirR) {
#pragma unroll
      for (int u = 0; u < kFirR; ++u) {
        const int32_t c = cs[k + u];
#pragma unroll
        for (int r = 0; r < kFirR; ++r) acc[r] = mac(acc[r], w[(r + u) % kFirR], c);
        w[u] = win[padx(base + k + u + kFirR)];
      }
    }
    for (; k < Ts; ++k) {
      const int32_t c = cs[k];
#pragma unroll
      for (int r = 0; r < kFirR; ++r) acc[r] = mac(acc[r], w[r], c);
#pragma unroll
      for (int r = 0; r < kFirR - 1; ++r) w[r] = w[r + 1];
      w[kFirR - 1] = win[padx(base + kFirR + k)];
    }
  }
  if (!active) return;
  int32_t y[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) {
    if constexpr (FAST) y[r] = (int32_t)(acc[r] << 1);
    else y[r] = (int32_t)((int64_t)acc[r] >> 31);
  }
  int32_t* o = dst + (uint64_t)it0.f * B + it0.n0 + base;
  if ((B & 3u) == 0 && ((uintptr_t)dst & 15u) == 0 && base + kFirR <= it0.count) {
    reinterpret_cast<int4*>(o)[0] = make_int4(y[0], y[1], y[2], y[3]);
    reinterpret_cast<int4*>(o)[1] = make_int4(y[4], y[5], y[6], y[7]);
  } else {
#pragma unroll
    for (int r = 0; r < kFirR; ++r)
      if (base + r < it0.count) o[r] = y[r];
  }
}

// ---------------------------------------------------------------- q7
// arm_fir_q7 (arm_fir_q7.c:446-560, LOOPUNROLL and tail alike): q31_t accumulator of q7 x q7
// products with plain int32 adds (wrapping on the gcc x86-64 build: a modular sum, the same
// in any order), y = __SSAT(acc >> 7, 8).  A tap quad c[4m..4m+3] times a sample quad is one
// v_dot4_i32_i8 (no clamp: modular).  The window is staged as aligned byte-quad words W, then
// as four LDS planes, plane p word i = (x[4i+p], .., x[4i+p+3]) = alignbyte(W[i+1], W[i], p);
// output base + r at tap quad m reads plane r & 3, word base/4 + (r >> 2) + m.  Two quads per
// block: each plane is read as an aligned 2-word pair one block ahead (3-slot ring).
constexpr int kQ7W = (kFirChunk + kFirMaxTaps) / 4 + 16;   // words per plane (+ look-ahead)
__device__ __forceinline__ int32_t dot4(uint32_t x, uint32_t c, int32_t acc) {
  return __builtin_amdgcn_sdot4((int)x, (int)c, acc, false);
}
struct Q7Ring { uint2 p[4][3]; };
template <int S>
__device__ __forceinline__ void q7_fetch(Q7Ring& r, const uint32_t* lds, int w) {
#pragma unroll
  for (int q = 0; q < 4; ++q) r.p[q][S] = *reinterpret_cast<const uint2*>(lds + q * kQ7W + w);
}
template <int P>
__device__ __forceinline__ void q7_block(Q7Ring& r, const uint32_t* lds, int w_ahead, const uint2 c2,
                                         int32_t (&A)[kFirR]) {
  q7_fetch<(P + 2) % 3>(r, lds, w_ahead);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t c = u ? c2.y : c2.x;
#pragma unroll
    for (int rr = 0; rr < kFirR; ++rr) {
      const int q = rr & 3, i = u + (rr >> 2), s = i < 2 ? P : (P + 1) % 3;
      A[rr] = dot4((i & 1) ? r.p[q][s].y : r.p[q][s].x, c, A[rr]);
    }
  }
}

template <bool LONG>
__global__ __launch_bounds__(kBlock) void fir_q7_kernel(const int8_t* __restrict__ coeffs, int T,
                                                        const int8_t* __restrict__ src, int8_t* __restrict__ dst,
                                                        uint32_t B, const int8_t* __restrict__ hist_in,
                                                        uint32_t nchunks) {
  __shared__ uint32_t wq[kQ7W + 4];                 // aligned window words
  __shared__ uint2 planes2[2 * kQ7W];              // 4 planes x kQ7W words
  __shared__ uint2 cq2[kFirMaxTaps / 8 + 2];       // tap quads as words, zero past numTaps
  uint32_t* lds = reinterpret_cast<uint32_t*>(planes2);
  uint32_t* cq = reinterpret_cast<uint32_t*>(cq2);
  const int T1 = T - 1;
  const FirItem it0 = fir_item(blockIdx.x, nchunks, B, T1);
  const int base = threadIdx.x * kFirR;
  const bool active = base < it0.count;
  const int wb = base >> 2;
  int32_t A[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) A[r] = 0;
  // numTaps > kFirMaxTaps: one window per tap segment, the modular int32 sums carried on
  for (int a = 0; a < (LONG ? T : 1); a += kFirMaxTaps) {   // !LONG: one pass, T <= kFirMaxTaps
    const int Ts = LONG ? min(T - a, kFirMaxTaps) : T;
    FirItem it = it0;
    it.a = a;
    it.total = it.count + Ts - 1;
    const int quads = (Ts + 3) >> 2;
    const int nw = kFirChunk / 4 + quads + 1;      // plane words any lane reads (<= kQ7W)
    if (LONG && a) __syncthreads();
    for (int i = threadIdx.x; i <= nw; i += kBlock) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) w |= (uint32_t)(uint8_t)fir_sample(hist_in, src, it, B, T1, 4 * i + b) << (8 * b);
      wq[i] = w;
    }
    const int8_t* cs = coeffs + a;
    for (int m = threadIdx.x; m < 2 * ((quads + 1) >> 1); m += kBlock) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int k = 4 * m + b;
        w |= k < Ts ? (uint32_t)(uint8_t)cs[k] << (8 * b) : 0u;
      }
      cq[m] = w;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nw; i += kBlock) {
      const uint32_t a0 = wq[i], b0 = wq[i + 1];
      lds[i] = a0;
      lds[kQ7W + i] = __builtin_amdgcn_alignbyte(b0, a0, 1);
      lds[2 * kQ7W + i] = __builtin_amdgcn_alignbyte(b0, a0, 2);
      lds[3 * kQ7W + i] = __builtin_amdgcn_alignbyte(b0, a0, 3);
    }
    __syncthreads();
    if (!active) continue;
    Q7Ring ring;
    q7_fetch<0>(ring, lds, wb);
    q7_fetch<1>(ring, lds, wb + 2);
    int m = 0;
    for (; m + 6 <= quads; m += 6) {
      q7_block<0>(ring, lds, wb + m + 4, cq2[m / 2], A);
      q7_block<1>(ring, lds, wb + m + 6, cq2[m / 2 + 1], A);
      q7_block<2>(ring, lds, wb + m + 8, cq2[m / 2 + 2], A);
    }
    if (m + 2 <= quads) {
      q7_block<0>(ring, lds, wb + m + 4, cq2[m / 2], A);
      m += 2;
      if (m + 2 <= quads) {
        q7_block<1>(ring, lds, wb + m + 4, cq2[m / 2], A);
        m += 2;
      }
    }
    if (m < quads) {                                  // odd quad count: the last one from LDS
      const uint32_t c = cq[m];
#pragma unroll
      for (int r = 0; r < kFirR; ++r) A[r] = dot4(lds[(r & 3) * kQ7W + wb + (r >> 2) + m], c, A[r]);
    }
  }
  if (!active) return;
  int8_t y[kFirR];
#pragma unroll
  for (int r = 0; r < kFirR; ++r) {
    const int32_t v = A[r] >> 7;
    y[r] = (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v);                   // arm_fir_q7.c:530
  }
  int8_t* o = dst + (uint64_t)it0.f * B + it0.n0 + base;
  if ((B & 7u) == 0 && ((uintptr_t)dst & 7u) == 0 && base + kFirR <= it0.count) {
    *reinterpret_cast<uint2*>(o) = *reinterpret_cast<const uint2*>(y);
  } else {
#pragma unroll
    for (int r = 0; r < kFirR; ++r)
      if (base + r < it0.count) o[r] = y[r];
  }
}

// new history = samples start .. start + T1 - 1 of s = [hist ; src]: the last T-1 for the FIR
// (start = B, arm_fir_f32.c:1242-1278), from outBlockSize * M for the decimator
// (arm_fir_decimate_f32.c), the last phaseLength - 1 for the interpolator (start = B)
template <typename T>
__global__ void fir_hist_kernel(const T* __restrict__ src, T* __restrict__ hist, const T* __restrict__ hist_in,
                                uint32_t B, int T1, uint32_t batch, uint32_t start) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= (uint64_t)batch * T1) return;
  uint64_t f;
  int j;
  if ((uint64_t)batch * T1 <= 0xffffffffull) {      // 32-bit division (the 64-bit one was most of the kernel)
    const uint32_t g32 = (uint32_t)g;
    f = g32 / (uint32_t)T1;
    j = (int)(g32 - (uint32_t)f * (uint32_t)T1);
  } else {
    f = g / T1;
    j = (int)(g % T1);
  }
  const int64_t sidx = (int64_t)start + j;          // index into s of the new history word j
  hist[g] = sidx < T1 ? hist_in[f * T1 + sidx] : src[f * B + (sidx - T1)];
}

// Latency path for the drop-in arm_fir_f32 (one short block per call, e.g. the 29-tap x
// 32-sample arm_fir_example_f32.c:141-239): one workgroup per filter stages s = [history ;
// block] in LDS, every output sums its taps k = 0 .. T-1 in order (mul then add, the
// reference's rounding), and the new history s[B .. B+T-1) is written from the LDS image -- one
// launch instead of filter pass + history kernel, and in place / B < T-1 need no copies (every
// read of src and hist_in precedes the barrier, every write follows it).
constexpr int kFirSmallMax = 8192;           // T - 1 + B words of LDS
__global__ __launch_bounds__(kBlock) void fir_f32_small_kernel(const float* __restrict__ coeffs, int T,
                                                               const float* src, float* dst, uint32_t B,
                                                               float* hist, const float* hist_in, uint32_t* done,
                                                               uint32_t seq) {
  __shared__ float s[kFirSmallMax];
  const int T1 = T - 1, tid = threadIdx.x;
  const uint64_t f = blockIdx.x;
  for (int j = tid; j < T1 + (int)B; j += kBlock) s[j] = j < T1 ? hist_in[f * T1 + j] : src[f * B + (j - T1)];
  __syncthreads();
  for (int n = tid; n < (int)B; n += kBlock) {
    float acc = 0.0f;
    for (int k = 0; k < T; ++k) acc = acc + s[n + k] * coeffs[k];
    dst[f * B + n] = acc;
  }
  for (int j = tid; j < T1; j += kBlock) hist[f * T1 + j] = s[B + j];
  if (done) signal_done(done, seq);               // the drop-in's one filter: its completion word
}

// One f32 FIR pass over `batch` filters, outputs on the lattice `fo`.
template <int R, bool F>
static void fir_f32_launch(const float* coeffs, int T, const float* src, float* dst, uint32_t B, uint32_t batch,
                           const float* hist_in, FirIn in, FirOut fo, hipStream_t st) {
  const uint32_t nchunks = (B + kF32Chunk<R> - 1) / kF32Chunk<R>;
  const uint32_t items = nchunks * batch;
  const int kpre = fir_f32_kpre<R>(T < kFirSeg ? T : kFirSeg);
  constexpr int K0 = fir_f32_kpre<R>(1), KL = fir_f32_kpre<R>(kFirSeg);     // 9..13 (R = 8), 17..21 (R = 16)
  static_assert(KL - K0 == 4, "five window sizes");
  auto k = T > kFirSeg ? fir_f32_kernel<R, KL, true, F>
         : kpre <= K0 ? fir_f32_kernel<R, K0, false, F> : kpre == K0 + 1 ? fir_f32_kernel<R, K0 + 1, false, F>
         : kpre == K0 + 2 ? fir_f32_kernel<R, K0 + 2, false, F> : kpre == K0 + 3 ? fir_f32_kernel<R, K0 + 3, false, F>
         : fir_f32_kernel<R, KL, false, F>;
  uint32_t ipw = MI355X_FIR_IPW;
  if (T > kFirSeg) ipw = 1;                         // a long item is already many units
  // few items (short blocks of a small batch): one item per workgroup, or the ipw items of a
  // single workgroup would run one after the other (round 4: 16 filters x 32 samples took 63 us
  // in one workgroup, profiles/r04/probes/breakeven.json)
  if (ipw > 1 && items < 256u * 16u * ipw) ipw = max(1u, items / (256u * 16u));
  if (!ipw) {
    const uint32_t resident = (uint32_t)persistent_grid((const void*)k, kBlock, 0, items);
    ipw = (items + resident - 1) / resident;
  }
  hipLaunchKernelGGL(k, dim3((items + ipw - 1) / ipw), dim3(kBlock), 0, st, coeffs, T, src, dst, B, hist_in, nchunks,
                     items, ipw, in, fo);
}
static void fir_f32_pass(const float* coeffs, int T, const float* src, float* dst, uint32_t B, uint32_t batch,
                         const float* hist_in, FirIn in, FirOut fo, hipStream_t st, bool fma = false) {
  if (fma) return fir_f32_launch<16, true>(coeffs, T, src, dst, B, batch, hist_in, in, fo, st);
  // output slots per filter at 4096- and 2048-output items: R = 8 when R = 16 pads > 12 % more
  const uint64_t s16 = (uint64_t)((B + kF32Chunk<16> - 1) / kF32Chunk<16>) * kF32Chunk<16>;
  const uint64_t s8 = (uint64_t)((B + kF32Chunk<8> - 1) / kF32Chunk<8>) * kF32Chunk<8>;
  if (s16 * 100 > s8 * 112) return fir_f32_launch<8, false>(coeffs, T, src, dst, B, batch, hist_in, in, fo, st);
  fir_f32_launch<16, false>(coeffs, T, src, dst, B, batch, hist_in, in, fo, st);
}

// The f32 convolution family's windowed outputs as one FIR pass (conv.hip): taps c (row
// stride cstride), x rows of A samples (stride sx), outputs n = first .. first + num - 1 of
// v[n] = sum_t w[n + t] c[t], w[j] = x[j - (T-1)], stored at y[item sy + off + dir (n - first)].
hipError_t fir_f32_conv_pass(const float* c, uint64_t cstride, int T, const float* x, uint64_t sx, uint32_t A,
                             uint32_t first, float* y, uint64_t sy, int64_t off, int dir, uint32_t num, uint32_t batch,
                             hipStream_t st) {
  if (num == 0 || batch == 0) return hipSuccess;
  if (T < 1 || T > kFirMaxTaps || (uint64_t)((num + kF32ChunkMin - 1) / kF32ChunkMin) * batch > 0xFFFFFFFFull)
    return hipErrorInvalidValue;
  fir_f32_pass(c, T, x, y, num, batch, nullptr, FirIn{sx, A, (int)first, 0u, cstride},
               FirOut{1u, 1u, 0u, dir, off, sy}, st);
  return hipGetLastError();
}

template <typename T>
static hipError_t fir_launch(int kind, const T* coeffs, int T_, const T* src, T* dst, uint32_t B, uint32_t batch,
                             T* hist, hipStream_t st, uint32_t* done, uint32_t seq, bool* flagged) {
  if (batch == 0 || B == 0) return hipSuccess;
  if (T_ < 1) return hipErrorInvalidValue;        // numTaps > kFirMaxTaps: tap segments
  const int T1 = T_ - 1;
  if constexpr (sizeof(T) == 4) {
    if (kind == kFirF32 && batch <= 8 && (int64_t)T1 + B <= kFirSmallMax && (uint64_t)B * T_ <= (1u << 16)) {
      uint32_t* dn = batch == 1 ? done : nullptr;  // one workgroup: it can signal the completion
      hipLaunchKernelGGL(fir_f32_small_kernel, dim3(batch), dim3(kBlock), 0, st, (const float*)coeffs, T_,
                         (const float*)src, (float*)dst, B, (float*)hist, (const float*)hist, dn, seq);
      if (dn && flagged) *flagged = true;
      return hipGetLastError();
    }
  }
  const int chunk = kind == kFirF32 || kind == kFirF32Fma ? kF32ChunkMin : kFirChunk;
  const uint32_t nchunks = (B + chunk - 1) / chunk;
  const uint64_t items64 = (uint64_t)nchunks * batch;
  if (items64 > 0xFFFFFFFFull) return hipErrorInvalidValue;
  const uint32_t items = (uint32_t)items64;
  // The history is read by the filter pass and rewritten afterwards; if the new tail
  // depends on old history (B < T1) keep a copy of the old one.
  const T* hist_in = hist;
  T* tmp = nullptr;
  if (T1 > 0 && (int64_t)B < T1) {
    hipError_t e = hipMallocAsync((void**)&tmp, sizeof(T) * (size_t)batch * T1, st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(tmp, hist, sizeof(T) * (size_t)batch * T1, hipMemcpyDefault, st);
    if (e != hipSuccess) return e;
    hist_in = tmp;
  }
  // In place (src overlapping dst): chunk c+1 stages its look-back window from src while
  // chunk c may already be writing dst, and the new history is read from src after the
  // pass; filter from a stream-ordered copy of the input instead.
  T* src_copy = nullptr;
  {
    const size_t bytes = sizeof(T) * (size_t)batch * B;
    const uintptr_t s0 = (uintptr_t)src, d0 = (uintptr_t)dst;
    if (s0 < d0 + bytes && d0 < s0 + bytes) {
      hipError_t e = hipMallocAsync((void**)&src_copy, bytes, st);
      if (e != hipSuccess) return e;
      e = hipMemcpyAsync(src_copy, src, bytes, hipMemcpyDefault, st);
      if (e != hipSuccess) return e;
      src = src_copy;
    }
  }
  switch (kind) {
    case kFirF32:
    case kFirF32Fma: {
      fir_f32_pass((const float*)coeffs, T_, (const float*)src, (float*)dst, B, batch, (const float*)hist_in,
                   FirIn{B, B, 0, 1u, 0}, FirOut{1u, 1u, 0u, 1, 0, (uint64_t)B}, st, kind == kFirF32Fma);
      break;
    }
    case kFirQ15:
    case kFirFastQ15: {
      if (T_ <= kFirMaxTaps &&
          fir_q15_mfma_launch((const int16_t*)coeffs, T_, (const int16_t*)src, (int16_t*)dst, B, batch,
                              (const int16_t*)hist_in, st, kind == kFirFastQ15))
        break;
      auto k = kind == kFirQ15 ? (T_ > kFirMaxTaps ? fir_q15_kernel<false, true> : fir_q15_kernel<false, false>)
                               : (T_ > kFirMaxTaps ? fir_q15_kernel<true, true> : fir_q15_kernel<true, false>);
      hipLaunchKernelGGL(k, dim3(items), dim3(kBlock), 0, st, (const int16_t*)coeffs, T_, (const int16_t*)src,
                         (int16_t*)dst, B, (const int16_t*)hist_in, nchunks);
      break;
    }
    case kFirQ7: {
      if (fir_q7_mfma_launch((const int8_t*)coeffs, T_, (const int8_t*)src, (int8_t*)dst, B, batch,
                             (const int8_t*)hist_in, st))
        break;
      hipLaunchKernelGGL(T_ > kFirMaxTaps ? fir_q7_kernel<true> : fir_q7_kernel<false>, dim3(items), dim3(kBlock), 0, st, (const int8_t*)coeffs, T_,
                         (const int8_t*)src, (int8_t*)dst, B, (const int8_t*)hist_in, nchunks);
      break;
    }
    default: {
      if (kind == kFirQ31 && fir_q31_mfma_launch((const int32_t*)coeffs, T_, (const int32_t*)src, (int32_t*)dst, B,
                                                 batch, (const int32_t*)hist_in, st))
        break;
      auto k = kind == kFirQ31 ? (T_ > kFirMaxTaps ? fir_q31_kernel<false, true> : fir_q31_kernel<false, false>)
                               : (T_ > kFirMaxTaps ? fir_q31_kernel<true, true> : fir_q31_kernel<true, false>);
      hipLaunchKernelGGL(k, dim3(items), dim3(kBlock), 0, st, (const int32_t*)coeffs, T_, (const int32_t*)src,
                         (int32_t*)dst, B, (const int32_t*)hist_in, nchunks);
    }
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (T1 > 0) {
    const uint64_t n = (uint64_t)batch * T1;
    // stream order: the filter pass has read hist_in before it is overwritten here
    hipLaunchKernelGGL(fir_hist_kernel<T>, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                       src, hist, hist_in, B, T1, batch, B);
    e = hipGetLastError();
  }
  if (tmp) (void)hipFreeAsync(tmp, st);
  if (src_copy) (void)hipFreeAsync(src_copy, st);
  return e;
}

hipError_t fir_run(int kind, const void* coeffs, int num_taps, const void* src, void* dst, uint32_t block_size,
                   uint32_t batch, void* hist, hipStream_t st, uint32_t* done, uint32_t seq, bool* flagged) {
  if (flagged) *flagged = false;
  switch (kind) {
    case kFirF32:
    case kFirF32Fma:
      return fir_launch<float>(kind, (const float*)coeffs, num_taps, (const float*)src, (float*)dst, block_size,
                               batch, (float*)hist, st, done, seq, flagged);
    case kFirQ15:
    case kFirFastQ15:
      return fir_launch<int16_t>(kind, (const int16_t*)coeffs, num_taps, (const int16_t*)src, (int16_t*)dst,
                                 block_size, batch, (int16_t*)hist, st, done, seq, flagged);
    case kFirQ31:
    case kFirFastQ31:
      return fir_launch<int32_t>(kind, (const int32_t*)coeffs, num_taps, (const int32_t*)src, (int32_t*)dst,
                                 block_size, batch, (int32_t*)hist, st, done, seq, flagged);
    case kFirQ7:
      return fir_launch<int8_t>(kind, (const int8_t*)coeffs, num_taps, (const int8_t*)src, (int8_t*)dst,
                                block_size, batch, (int8_t*)hist, st, done, seq, flagged);
    default:
      return hipErrorInvalidValue;
  }
}

// ================================================================ multirate FIR
// Decimator (arm_fir_decimate_{f32,q15,q31,fast_q15,fast_q31}.c, generic C paths): with
// s = [history (numTaps-1) ; block], output j = sum_t s[M j + t] * h[t], t ascending from a
// zero accumulator; outBlockSize = blockSize / M.  Interpolator
// (arm_fir_interpolate_{f32,q15,q31}.c): s = [history (phaseLength-1) ; block], output
// n L + q = sum_i s[n + i] * h[(L-1-q) + i L], i ascending.  Accumulators per op:
//   f32: mul then add (bit-exact order);  q15: q63 sum of exact products, __SSAT(acc >> 15, 16);
//   q31: q63 sum, (q31)(acc >> 31);  fast q15 (decimator): q31_t wrapping sum, __SSAT(acc >> 15, 16);
//   fast q31 (decimator): acc = (q31)(((q63)acc << 32 + x*h) >> 32) = acc + floor(x*h / 2^32)
//   mod 2^32 (no rounding term, unlike arm_fir_fast_q31), output acc << 1.
// The integer sums are order-free, the f32 one is not.  One workgroup = one filter x a chunk of
// outputs; the window is staged in LDS (the decimator's as M phases X_p[m] = s[M (j0 + m) + p]
// so that lanes with consecutive outputs read consecutive words: bank-conflict free for any M);
// coefficients are wave-uniform scalar loads.
template <int OP> struct MrT;
template <> struct MrT<kMrF32> {
  using T = float; using Acc = float;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { const float p = w * c; return a + p; }
  static __device__ __forceinline__ T out(Acc a) { return a; }
};
template <> struct MrT<kMrQ15> {
  using T = int16_t; using Acc = int64_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (int32_t)w * (int32_t)c; }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat16((int32_t)(a >> 15)); }
};
template <> struct MrT<kMrQ31> {
  using T = int32_t; using Acc = uint64_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint64_t)((int64_t)w * c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)(int32_t)((int64_t)a >> 31); }
};
template <> struct MrT<kMrFastQ15> {
  using T = int16_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)((int32_t)w * (int32_t)c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat16((int32_t)a >> 15); }
};
template <> struct MrT<kMrFastQ31> {
  using T = int32_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc mac(Acc a, T w, T c) { return a + (uint32_t)mulhi(w, c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)(a << 1); }
};

constexpr int kMrWin = 8192;               // LDS window elements per workgroup

template <int OP>
__global__ __launch_bounds__(kBlock) void fir_decimate_kernel(const typename MrT<OP>::T* __restrict__ coeffs, int T,
                                                              int M, const typename MrT<OP>::T* __restrict__ src,
                                                              typename MrT<OP>::T* __restrict__ dst, uint32_t B,
                                                              const typename MrT<OP>::T* __restrict__ hist_in,
                                                              uint32_t nchunks, int J, int Wp) {
  using Op = MrT<OP>;
  using E = typename Op::T;
  __shared__ E win[kMrWin];
  const uint32_t f = blockIdx.x / nchunks;
  const int j0 = (int)(blockIdx.x - f * nchunks) * J;
  const int outs = (int)(B / (uint32_t)M);
  const int cnt = min(J, outs - j0);
  FirItem it;
  it.f = f; it.n0 = M * j0; it.count = cnt; it.total = M * (cnt - 1) + T;
  for (int idx = threadIdx.x; idx < M * Wp; idx += kBlock) {
    const int m = idx / M, p = idx - m * M;
    win[p * Wp + m] = fir_sample(hist_in, src, it, B, T - 1, idx);
  }
  __syncthreads();
  E* y = dst + (uint64_t)f * outs + j0;
  if constexpr (OP == kMrF32) {
    for (int jl = threadIdx.x; jl < cnt; jl += kBlock) {
      // t ascending: (i, p) = divmod(t, M), tap t reads X_p[jl + i]
      typename Op::Acc acc = 0;
      const E* w = win + jl;
      int t = 0;
      for (int i = 0; t < T; ++i, ++w)
        for (int p = 0; p < M && t < T; ++p, ++t) acc = Op::mac(acc, w[p * Wp], coeffs[t]);
      y[jl] = Op::out(acc);
    }
  } else {
    // order-free sums: phase by phase over the pre-permuted phase rows hp[p I + i] =
    // h[i M + p] (zero past numTaps), I = ceil(T / M): contiguous wave-uniform taps, each
    // applied to R = 4 outputs per lane (jl + 256 r) so one scalar-load wait covers 4R MACs
    // (R = 1 and 2 measured slower for every op)
    constexpr int R = 4;
    const int I = (T + M - 1) / M;
    for (int j0 = threadIdx.x; j0 < cnt; j0 += R * kBlock) {
      typename Op::Acc acc[R] = {};
      for (int p = 0; p < M && p < T; ++p) {
        const E* w = win + p * Wp + j0;
        const int32_t* hp = reinterpret_cast<const int32_t*>(coeffs) + p * I;   // dword rows
        for (int i = 0; i < I; ++i) {
          const E c = (E)hp[i];
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r] = Op::mac(acc[r], w[i + r * kBlock], c);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (j0 + r * kBlock < cnt) y[j0 + r * kBlock] = Op::out(acc[r]);
    }
  }
}

// Interpolator, LG phases per launch in registers: one input position n per lane, each window
// word s[n + i] read once and applied to the LG phases' accumulators (i ascending per output),
// phase coefficients h_q[i] = h[(L-1-q) + i L] pre-permuted into contiguous rows (wave-uniform
// scalar loads), the LG outputs y[n L + q0 .. q0 + LG - 1] stored together.
template <int OP, int LG>
__global__ __launch_bounds__(kBlock) void fir_interp_phases_kernel(const typename MrT<OP>::T* __restrict__ hq, int L,
                                                                   int q0, int P,
                                                                   const typename MrT<OP>::T* __restrict__ src,
                                                                   typename MrT<OP>::T* __restrict__ dst, uint32_t B,
                                                                   const typename MrT<OP>::T* __restrict__ hist_in,
                                                                   uint32_t nchunks, int N) {
  using Op = MrT<OP>;
  using E = typename Op::T;
  __shared__ E win[kMrWin];
  const uint32_t f = blockIdx.x / nchunks;
  const int n0 = (int)(blockIdx.x - f * nchunks) * N;
  const int cnt = min(N, (int)B - n0);
  FirItem it;
  it.f = f; it.n0 = n0; it.count = cnt; it.total = cnt + P - 1;
  for (int idx = threadIdx.x; idx < it.total; idx += kBlock) win[idx] = fir_sample(hist_in, src, it, B, P - 1, idx);
  __syncthreads();
  E* y = dst + ((uint64_t)f * B + n0) * (uint32_t)L + q0;
  const E* h = hq + (size_t)q0 * P;
  for (int nl = threadIdx.x; nl < cnt; nl += kBlock) {
    const E* w = win + nl;
    typename Op::Acc acc[LG];
#pragma unroll
    for (int q = 0; q < LG; ++q) acc[q] = 0;
    int i = 0;
    for (; i + 4 <= P; i += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const E x = w[i + u];
#pragma unroll
        for (int q = 0; q < LG; ++q) acc[q] = Op::mac(acc[q], x, h[q * P + i + u]);
      }
    }
    for (; i < P; ++i) {
      const E x = w[i];
#pragma unroll
      for (int q = 0; q < LG; ++q) acc[q] = Op::mac(acc[q], x, h[q * P + i]);
    }
    E* o = y + (uint64_t)nl * L;
#pragma unroll
    for (int q = 0; q < LG; ++q) o[q] = Op::out(acc[q]);
  }
}

// Four consecutive inputs per lane: the window rides in registers (one 16-B LDS read per lane
// per 4 taps) and each scalar coefficient feeds 4 outputs, so a tap block of 4 costs 4·4·LG
// MACs against one LDS read and LG·4 coefficient loads (the one-input-per-lane kernel above
// waited on a scalar load every 4·LG MACs).  Per output the taps still run i = 0, 1, ... in
// order.  Needs N % 4 == 0 (outputs per chunk) and a 16-B aligned window.
// consecutive inputs per lane: f32 8 (2048-output chunks: 110 vs 106 G input samples/s at 4),
// the int64-accumulator types 4 (chunks of R x 256 outputs keep every lane busy)
template <int OP> constexpr int interp_r() { return OP == kMrF32 ? 8 : 4; }
template <int OP, int LG, int R = interp_r<OP>()>
__global__ __launch_bounds__(kBlock) void fir_interp_phases4_kernel(const typename MrT<OP>::T* __restrict__ hq, int L,
                                                                    int q0, int P,
                                                                    const typename MrT<OP>::T* __restrict__ src,
                                                                    typename MrT<OP>::T* __restrict__ dst, uint32_t B,
                                                                    const typename MrT<OP>::T* __restrict__ hist_in,
                                                                    uint32_t nchunks, int N) {
  using Op = MrT<OP>;
  using E = typename Op::T;
  __shared__ __attribute__((aligned(16))) E win[kMrWin + 8];
  const uint32_t f = blockIdx.x / nchunks;
  const int n0 = (int)(blockIdx.x - f * nchunks) * N;
  const int cnt = min(N, (int)B - n0);
  FirItem it;
  it.f = f; it.n0 = n0; it.count = cnt; it.total = cnt + P - 1;
  const int padded = (it.total + 8 + 3) & ~3;           // zero tail: the last block reads past
  for (int idx = threadIdx.x; idx < padded; idx += kBlock)
    win[idx] = idx < it.total ? fir_sample(hist_in, src, it, B, P - 1, idx) : (E)0;
  __syncthreads();
  E* y = dst + ((uint64_t)f * B + n0) * (uint32_t)L + q0;
  const E* h = hq + (size_t)q0 * P;
  for (int nl = R * threadIdx.x; nl < cnt; nl += R * kBlock) {
    const E* w = win + nl;
    typename Op::Acc acc[R][LG];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int q = 0; q < LG; ++q) acc[r][q] = 0;
    E a[R + 4];
#pragma unroll
    for (int u = 0; u < R; ++u) a[u] = w[u];
    int i = 0;
    for (; i + 4 <= P; i += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[R + u] = w[i + R + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        E c[LG];
#pragma unroll
        for (int q = 0; q < LG; ++q) c[q] = h[q * P + i + u];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int q = 0; q < LG; ++q) acc[r][q] = Op::mac(acc[r][q], a[u + r], c[q]);
      }
#pragma unroll
      for (int u = 0; u < R; ++u) a[u] = a[u + 4];
    }
    for (; i < P; ++i) {                                // P % 4 tail taps
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const E x = w[i + r];
#pragma unroll
        for (int q = 0; q < LG; ++q) acc[r][q] = Op::mac(acc[r][q], x, h[q * P + i]);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (nl + r >= cnt) break;
      E* o = y + (uint64_t)(nl + r) * L;
#pragma unroll
      for (int q = 0; q < LG; ++q) o[q] = Op::out(acc[r][q]);
    }
  }
}

// Windows that do not fit the LDS image (decimator M (ceil(T / M) + 2) > kMrWin, interpolator
// phaseLength > kMrWin - 256): one thread per output reading its window straight from HBM/L2,
// taps ascending from a zero accumulator (the reference's order, arm_fir_decimate_f32.c /
// arm_fir_interpolate_f32.c generic paths).  Decimator: output j of filter f = sum_t s[M j + t]
// h[t]; interpolator (M = 1, phase stride L): output n L + q = sum_i s[n + i] h[(L-1-q) + i L].
template <int OP>
__global__ __launch_bounds__(kBlock) void fir_mr_direct_kernel(const typename MrT<OP>::T* __restrict__ h, int taps,
                                                               int M, int L, const typename MrT<OP>::T* __restrict__ src,
                                                               typename MrT<OP>::T* __restrict__ dst, uint32_t B,
                                                               const typename MrT<OP>::T* __restrict__ hist_in, int H,
                                                               uint32_t outs, uint32_t batch) {
  using Op = MrT<OP>;
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= (uint64_t)batch * outs) return;
  const uint32_t f = (uint32_t)(g / outs), o = (uint32_t)(g - (uint64_t)f * outs);
  const uint32_t n = o / (uint32_t)L, q = o - n * (uint32_t)L;   // decimator: L = 1, q = 0
  FirItem it;
  it.f = f; it.n0 = (int)(M * n); it.count = 1; it.total = taps;
  typename Op::Acc acc = 0;
  const typename MrT<OP>::T* hq = h + (L - 1 - (int)q);
  for (int i = 0; i < taps; ++i) acc = Op::mac(acc, fir_sample(hist_in, src, it, B, H, i), hq[(size_t)i * L]);
  dst[g] = Op::out(acc);
}

// h_q[i] = h[(L-1-q) + i L]: the interpolator's phases as contiguous coefficient rows
template <typename E>
__global__ void mr_phase_coeffs_kernel(const E* __restrict__ h, E* __restrict__ hq, int L, int P) {
  const int g = blockIdx.x * kBlock + threadIdx.x;
  if (g >= L * P) return;
  const int q = g / P, i = g - q * P;
  hq[g] = h[(L - 1 - q) + i * L];
}

// Shared host part: history copy when the new history depends on the old one (the pass reads
// hist_in, the history kernel rewrites hist), input copy when src overlaps dst, the filter
// launch, then the history update from `start`.
template <typename E, typename Launch>
static hipError_t mr_launch(const E* src, E* dst, size_t out_words, uint32_t B, uint32_t batch, E* hist, int H,
                            uint32_t start, hipStream_t st, Launch&& launch) {
  const E* hist_in = hist;
  E* tmp = nullptr;
  if (H > 0 && (int64_t)start < H) {
    hipError_t e = hipMallocAsync((void**)&tmp, sizeof(E) * (size_t)batch * H, st);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(tmp, hist, sizeof(E) * (size_t)batch * H, hipMemcpyDefault, st);
    if (e != hipSuccess) return e;
    hist_in = tmp;
  }
  E* src_copy = nullptr;
  {
    const size_t ib = sizeof(E) * (size_t)batch * B, ob = sizeof(E) * out_words;
    const uintptr_t s0 = (uintptr_t)src, d0 = (uintptr_t)dst;
    if (s0 < d0 + ob && d0 < s0 + ib) {
      hipError_t e = hipMallocAsync((void**)&src_copy, ib, st);
      if (e != hipSuccess) return e;
      e = hipMemcpyAsync(src_copy, src, ib, hipMemcpyDefault, st);
      if (e != hipSuccess) return e;
      src = src_copy;
    }
  }
  hipError_t e = launch(src, hist_in);
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess && H > 0) {
    const uint64_t n = (uint64_t)batch * H;
    hipLaunchKernelGGL(fir_hist_kernel<E>, dim3((uint32_t)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, src, hist,
                       hist_in, B, H, batch, start);
    e = hipGetLastError();
  }
  if (tmp) (void)hipFreeAsync(tmp, st);
  if (src_copy) (void)hipFreeAsync(src_copy, st);
  return e;
}

// hp[p I + i] = h[i M + p] (0 past numTaps), widened to dwords: the decimator's taps as M
// contiguous phase rows that scalar loads fetch four at a time
template <typename E>
__global__ void mr_decim_rows_kernel(const E* __restrict__ h, int32_t* __restrict__ hp, int T, int M, int I) {
  const int g = blockIdx.x * kBlock + threadIdx.x;
  if (g >= M * I) return;
  const int p = g / I, i = g - p * I, t = i * M + p;
  hp[g] = t < T ? (int32_t)h[t] : 0;
}

template <int OP>
static hipError_t decimate_launch(const void* coeffs, int T, int M, const void* src, void* dst, uint32_t B,
                                  uint32_t batch, void* hist, hipStream_t st) {
  using E = typename MrT<OP>::T;
  if (batch == 0 || B == 0) return hipSuccess;
  if (T < 1 || M < 1) return hipErrorInvalidValue;
  const int outs = (int)(B / (uint32_t)M);
  const int per_phase = (T + M - 1) / M;
  int J = kMrWin / M - per_phase - 1;               // M * (J + per_phase + 1) <= kMrWin
  if (J < 1) {                                      // window past the LDS image: direct kernel
    const uint64_t n = (uint64_t)batch * outs;
    if (n == 0) return mr_launch<E>((const E*)src, (E*)dst, 0, B, batch, (E*)hist, T - 1, (uint32_t)(outs * M), st,
                                    [&](const E*, const E*) { return hipSuccess; });
    if ((n + kBlock - 1) / kBlock > 0x7FFFFFFFull) return hipErrorInvalidValue;
    return mr_launch<E>((const E*)src, (E*)dst, (size_t)n, B, batch, (E*)hist, T - 1, (uint32_t)(outs * M), st,
                        [&](const E* s, const E* h) {
                          hipLaunchKernelGGL(fir_mr_direct_kernel<OP>, dim3((uint32_t)((n + kBlock - 1) / kBlock)),
                                             dim3(kBlock), 0, st, (const E*)coeffs, T, M, 1, s, (E*)dst, B, h, T - 1,
                                             (uint32_t)outs, batch);
                          return hipSuccess;
                        });
  }
  J = J >= 2 * kBlock ? 4 * kBlock < J ? 4 * kBlock : (J / kBlock) * kBlock : J;
  const int Wp = J + per_phase + 1;
  const uint32_t nchunks = outs > 0 ? (uint32_t)((outs + J - 1) / J) : 0;
  const uint64_t blocks = (uint64_t)nchunks * batch;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  // f32 with M <= 4 and T within the FIR window: the register-window FIR pass over every
  // input position, storing the outputs with n % M == 0 (M x the MACs at the FIR kernel's
  // issue efficiency beats the one-output-per-lane kernel up to M = 4: tools/bench_filters.py)
  const bool via_fir = OP == kMrF32 && M <= 4 && B % (uint32_t)M == 0 && T <= kFirMaxTaps &&
                       (uint64_t)((B + kF32ChunkMin - 1) / kF32ChunkMin) * batch <= 0xFFFFFFFFull;
  return mr_launch<E>((const E*)src, (E*)dst, (size_t)batch * outs, B, batch, (E*)hist, T - 1, (uint32_t)(outs * M),
                      st, [&](const E* s, const E* h) {
                        if (blocks == 0) return hipSuccess;
                        if constexpr (OP == kMrF32) {
                          if (via_fir) {
                            fir_f32_pass((const float*)coeffs, T, (const float*)s, (float*)dst, B, batch,
                                         (const float*)h, FirIn{B, B, 0, 1u, 0},
                                         FirOut{(uint32_t)M, 1u, 0u, 1, 0, (uint64_t)outs}, st);
                            return hipSuccess;
                          }
                        }
                        int32_t* hp = nullptr;
                        if constexpr (OP != kMrF32) {     // phase rows for the order-free sums
                          const int I = (T + M - 1) / M;
                          hipError_t e = hipMallocAsync((void**)&hp, sizeof(int32_t) * (size_t)M * I, st);
                          if (e != hipSuccess) return e;
                          const uint32_t n = (uint32_t)(M * I);
                          hipLaunchKernelGGL(mr_decim_rows_kernel<E>, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0,
                                             st, (const E*)coeffs, hp, T, M, I);
                        }
                        hipLaunchKernelGGL(fir_decimate_kernel<OP>, dim3((uint32_t)blocks), dim3(kBlock), 0, st,
                                           hp ? (const E*)hp : (const E*)coeffs, T, M, s, (E*)dst, B, h, nchunks, J,
                                           Wp);
                        if (hp) (void)hipFreeAsync(hp, st);
                        return hipSuccess;
                      });
}

template <int OP>
static hipError_t interpolate_launch(const void* coeffs, int L, int P, const void* src, void* dst, uint32_t B,
                                     uint32_t batch, void* hist, hipStream_t st) {
  using E = typename MrT<OP>::T;
  if (batch == 0 || B == 0) return hipSuccess;
  if (L < 1 || P < 1) return hipErrorInvalidValue;
  if (P > kMrWin - kBlock) {                        // window past the LDS image: direct kernel
    const uint64_t n = (uint64_t)batch * B * (uint32_t)L;
    if ((n + kBlock - 1) / kBlock > 0x7FFFFFFFull || (uint64_t)B * (uint32_t)L > 0xFFFFFFFFull)
      return hipErrorInvalidValue;
    return mr_launch<E>((const E*)src, (E*)dst, (size_t)n, B, batch, (E*)hist, P - 1, B, st,
                        [&](const E* s, const E* h) {
                          hipLaunchKernelGGL(fir_mr_direct_kernel<OP>, dim3((uint32_t)((n + kBlock - 1) / kBlock)),
                                             dim3(kBlock), 0, st, (const E*)coeffs, P, 1, L, s, (E*)dst, B, h, P - 1,
                                             (uint32_t)(B * (uint32_t)L), batch);
                          return hipSuccess;
                        });
  }
  int N = kMrWin - (P - 1);
  constexpr int kR = interp_r<OP>();
  N = N >= kR * kBlock ? kR * kBlock : (N >= kBlock ? (N / kBlock) * kBlock : N);
  const uint32_t nchunks = (B + N - 1) / N;
  const uint64_t blocks = (uint64_t)nchunks * batch;
  if (blocks > 0x7FFFFFFFull) return hipErrorInvalidValue;
  return mr_launch<E>((const E*)src, (E*)dst, (size_t)batch * B * L, B, batch, (E*)hist, P - 1, B, st,
                      [&](const E* s, const E* h) {
                        E* hq = nullptr;
                        hipError_t e = hipMallocAsync((void**)&hq, sizeof(E) * (size_t)L * P, st);
                        if (e != hipSuccess) return e;
                        const uint32_t nq = (uint32_t)L * P;
                        hipLaunchKernelGGL(mr_phase_coeffs_kernel<E>, dim3((nq + kBlock - 1) / kBlock), dim3(kBlock), 0,
                                           st, (const E*)coeffs, hq, L, P);
                        for (int q0 = 0; q0 < L; q0 += 8) {
                          const int lg = L - q0 < 8 ? L - q0 : 8;
                          auto k = lg == 1 ? fir_interp_phases_kernel<OP, 1> : lg == 2 ? fir_interp_phases_kernel<OP, 2>
                                 : lg == 3 ? fir_interp_phases_kernel<OP, 3> : lg == 4 ? fir_interp_phases_kernel<OP, 4>
                                 : lg == 5 ? fir_interp_phases_kernel<OP, 5> : lg == 6 ? fir_interp_phases_kernel<OP, 6>
                                 : lg == 7 ? fir_interp_phases_kernel<OP, 7> : fir_interp_phases_kernel<OP, 8>;
                          if (N % kR == 0 && lg <= 4)
                            k = lg == 1 ? fir_interp_phases4_kernel<OP, 1> : lg == 2 ? fir_interp_phases4_kernel<OP, 2>
                              : lg == 3 ? fir_interp_phases4_kernel<OP, 3> : fir_interp_phases4_kernel<OP, 4>;
                          hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(kBlock), 0, st, (const E*)hq, L, q0, P, s,
                                             (E*)dst, B, h, nchunks, N);
                        }
                        (void)hipFreeAsync(hq, st);
                        return hipSuccess;
                      });
}

hipError_t fir_decimate_run(int op, const void* coeffs, int num_taps, int M, const void* src, void* dst,
                            uint32_t block_size, uint32_t batch, void* hist, hipStream_t st) {
  switch (op) {
    case kMrF32: return decimate_launch<kMrF32>(coeffs, num_taps, M, src, dst, block_size, batch, hist, st);
    case kMrQ15: return decimate_launch<kMrQ15>(coeffs, num_taps, M, src, dst, block_size, batch, hist, st);
    case kMrQ31: return decimate_launch<kMrQ31>(coeffs, num_taps, M, src, dst, block_size, batch, hist, st);
    case kMrFastQ15: return decimate_launch<kMrFastQ15>(coeffs, num_taps, M, src, dst, block_size, batch, hist, st);
    case kMrFastQ31: return decimate_launch<kMrFastQ31>(coeffs, num_taps, M, src, dst, block_size, batch, hist, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t fir_interpolate_run(int op, const void* coeffs, int L, int phase_len, const void* src, void* dst,
                               uint32_t block_size, uint32_t batch, void* hist, hipStream_t st) {
  switch (op) {
    case kMrF32: return interpolate_launch<kMrF32>(coeffs, L, phase_len, src, dst, block_size, batch, hist, st);
    case kMrQ15: return interpolate_launch<kMrQ15>(coeffs, L, phase_len, src, dst, block_size, batch, hist, st);
    case kMrQ31: return interpolate_launch<kMrQ31>(coeffs, L, phase_len, src, dst, block_size, batch, hist, st);
    default: return hipErrorInvalidValue;
  }
}

// ---- sparse FIR: arm_fir_sparse_{f32,q31,q15,q7} -------------------------------------------
// y[n] = sum over k ascending of x[n - D_k] c_k (arm_fir_sparse_f32.c: the first tap stores
// x c_0, every later tap adds x c_k to the output, mul then add; q31 (q31)((q63 x c) >> 32)
// terms summed with wrap-around, output << 1 (arm_fir_sparse_q31.c); q15 / q7 q31 products
// summed with wrap-around in the q31 scratch, __SSAT(acc >> 15, 16) / __SSAT(acc >> 7, 8)
// (arm_fir_sparse_q15.c, _q7.c)).  Three sample sources:
//   kSpLds:  batched streams, history [batch][maxDelay] (oldest first) + block; a workgroup
//            stages x[n0 - maxDelay, n0 + kSpLOut) of its stream in LDS (delays outside
//            [0, maxDelay] read 0; fir_sparse_lds_kernel);
//   kSpGlob: the same addressing read straight from HBM/L2 (windows too large for LDS);
//   kSpCirc: the drop-in call: the reference's circular state buffer of L = maxDelay +
//            blockSize words after the block is written, tap k read from (r0 - D_k) (+ L if
//            negative), advancing with wrap at L, exactly as arm_circularRead_f32 does.
template <int OP> struct SpT;
template <> struct SpT<kSpF32> {
  using T = float; using Acc = float;
  static __device__ __forceinline__ Acc first(T x, T c) { return x * c; }
  static __device__ __forceinline__ Acc mac(Acc a, T x, T c) { const float p = x * c; return a + p; }
  static __device__ __forceinline__ T out(Acc a) { return a; }
};
template <> struct SpT<kSpQ31> {
  using T = int32_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc first(T x, T c) { return (uint32_t)mulhi(x, c); }
  static __device__ __forceinline__ Acc mac(Acc a, T x, T c) { return a + (uint32_t)mulhi(x, c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)(a << 1); }
};
template <> struct SpT<kSpQ15> {
  using T = int16_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc first(T x, T c) { return (uint32_t)((int32_t)x * (int32_t)c); }
  static __device__ __forceinline__ Acc mac(Acc a, T x, T c) { return a + first(x, c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat16((int32_t)a >> 15); }
};
template <> struct SpT<kSpQ7> {
  using T = int8_t; using Acc = uint32_t;
  static __device__ __forceinline__ Acc first(T x, T c) { return (uint32_t)((int32_t)x * (int32_t)c); }
  static __device__ __forceinline__ Acc mac(Acc a, T x, T c) { return a + first(x, c); }
  static __device__ __forceinline__ T out(Acc a) { return (T)ssat8((int32_t)a >> 7); }
};

enum SpSrc { kSpLds = 0, kSpGlob = 1, kSpCirc = 2 };
constexpr int kSpR = 4;                        // outputs per lane (direct-read kernel)
constexpr int kSpOut = kSpR * kBlock;          // outputs per workgroup (direct-read kernel)
constexpr int kSpLR = 16;                      // outputs per lane (LDS kernel)
constexpr int kSpLOut = kSpLR * kBlock;        // outputs per workgroup (LDS kernel)
constexpr int kSpLdsBytes = 64 * 1024;         // largest staged window

struct SpIn {
  const void* src;      // kSpLds / kSpGlob: [batch][B];  kSpCirc: the circular state
  const void* hist;     // [batch][maxD]
  uint32_t B, nchunks;
  int maxD;
  int L, r0;            // kSpCirc
};

// LDS kernel: win[j] = x[n0 - maxD + j], j < maxD + kSpLOut (zero past the block), lane t's
// outputs n0 + t + 256 r read win[maxD - D + t + 256 r]: one LDS base per tap and immediate
// offsets, no per-sample bounds checks (a tap with D outside [0, maxD] reads zeros, decided
// per tap); the taps' scalar loads are issued four at a time.
template <int OP>
__global__ __launch_bounds__(kBlock) void fir_sparse_lds_kernel(const typename SpT<OP>::T* __restrict__ coeffs,
                                                                const int32_t* __restrict__ delays, int T, SpIn in,
                                                                typename SpT<OP>::T* __restrict__ dst) {
  using Op = SpT<OP>;
  using E = typename Op::T;
  extern __shared__ __align__(16) unsigned char sp_lds[];
  E* win = reinterpret_cast<E*>(sp_lds);
  const uint64_t f = blockIdx.x / in.nchunks;
  const int n0 = (int)(blockIdx.x - f * in.nchunks) * kSpLOut;
  const int cnt = min(kSpLOut, (int)in.B - n0);
  const int maxD = in.maxD;
  const E* src = reinterpret_cast<const E*>(in.src) + f * in.B;
  const E* hist = reinterpret_cast<const E*>(in.hist) + f * (uint64_t)maxD;
  for (int j = threadIdx.x; j < maxD + kSpLOut; j += kBlock) {
    const int p = n0 - maxD + j;
    win[j] = p < 0 ? hist[maxD + p] : (p < n0 + cnt ? src[p] : (E)0);
  }
  __syncthreads();
  const E* wt = win + maxD + threadIdx.x;
  typename Op::Acc acc[kSpLR];
  auto tap = [&](E c, int D) {
    if (D >= 0 && D <= maxD) {                             // wave-uniform
      const E* w = wt - D;
#pragma unroll
      for (int r = 0; r < kSpLR; ++r) acc[r] = Op::mac(acc[r], w[r * kBlock], c);
    } else {
#pragma unroll
      for (int r = 0; r < kSpLR; ++r) acc[r] = Op::mac(acc[r], (E)0, c);
    }
  };
  {
    const E c = coeffs[0];
    const int D = delays[0];
    const E* w = wt - ((D >= 0 && D <= maxD) ? D : 0);
    const bool z = !(D >= 0 && D <= maxD);
#pragma unroll
    for (int r = 0; r < kSpLR; ++r) acc[r] = Op::first(z ? (E)0 : w[r * kBlock], c);
  }
  int k = 1;
  for (; k + 4 <= T; k += 4) {
    E c[4];
    int D[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { c[u] = coeffs[k + u]; D[u] = delays[k + u]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) tap(c[u], D[u]);
  }
  for (; k < T; ++k) tap(coeffs[k], delays[k]);
  E* y = dst + f * in.B + n0 + threadIdx.x;
#pragma unroll
  for (int r = 0; r < kSpLR; ++r)
    if ((int)threadIdx.x + r * kBlock < cnt) y[r * kBlock] = Op::out(acc[r]);
}

template <int OP, int SRC>
__global__ __launch_bounds__(kBlock) void fir_sparse_kernel(const typename SpT<OP>::T* __restrict__ coeffs,
                                                            const int32_t* __restrict__ delays, int T, SpIn in,
                                                            typename SpT<OP>::T* __restrict__ dst) {
  using Op = SpT<OP>;
  using E = typename Op::T;
  const uint64_t f = blockIdx.x / in.nchunks;
  const int n0 = (int)(blockIdx.x - f * in.nchunks) * kSpOut;
  const int cnt = min(kSpOut, (int)in.B - n0);
  const E* src = reinterpret_cast<const E*>(in.src) + (SRC == kSpCirc ? 0 : f * in.B);
  const E* hist = reinterpret_cast<const E*>(in.hist) + f * (uint64_t)in.maxD;
  auto fetch = [&](int n, int D, int idx) -> E {
    if constexpr (SRC == kSpGlob) {
      const int p = n - D;
      return p >= 0 ? (p < (int)in.B ? src[p] : (E)0) : (p >= -in.maxD ? hist[in.maxD + p] : (E)0);
    } else {
      int q = idx + n;
      if (q >= in.L) q -= in.L;
      if ((unsigned)q >= (unsigned)in.L) q = ((q % in.L) + in.L) % in.L;
      return src[q];
    }
  };
  typename Op::Acc acc[kSpR];
  for (int k = 0; k < T; ++k) {
    const E c = coeffs[k];
    const int D = delays[k];
    int idx = 0;
    if constexpr (SRC == kSpCirc) {
      idx = in.r0 - D;
      if (idx < 0) idx += in.L;
    }
#pragma unroll
    for (int r = 0; r < kSpR; ++r) {
      const int n = n0 + (int)threadIdx.x + r * kBlock;
      const E x = n < n0 + cnt ? fetch(n, D, idx) : (E)0;
      acc[r] = k == 0 ? Op::first(x, c) : Op::mac(acc[r], x, c);
    }
  }
  E* y = dst + f * in.B;
#pragma unroll
  for (int r = 0; r < kSpR; ++r) {
    const int n = n0 + (int)threadIdx.x + r * kBlock;
    if (n < n0 + cnt) y[n] = Op::out(acc[r]);
  }
}

template <int OP>
static hipError_t sparse_launch(const void* coeffs, const int32_t* delays, int T, int maxD, const void* src,
                                void* dst, uint32_t B, uint32_t batch, void* hist, int L, int r0, hipStream_t st) {
  using E = typename SpT<OP>::T;
  if (batch == 0 || B == 0) return hipSuccess;
  if (T < 1 || maxD < 0) return hipErrorInvalidValue;
  SpIn in{src, hist, B, (B + kSpOut - 1) / kSpOut, maxD, L, r0};
  const uint64_t blocks = (uint64_t)in.nchunks * batch;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  if (L > 0) {                                 // drop-in: one stream, circular state
    hipLaunchKernelGGL((fir_sparse_kernel<OP, kSpCirc>), dim3((uint32_t)blocks), dim3(kBlock), 0, st,
                       (const E*)coeffs, delays, T, in, (E*)dst);
    return hipGetLastError();
  }
  const size_t lds = sizeof(E) * ((size_t)maxD + kSpLOut);
  const SpIn lin{src, hist, B, (B + kSpLOut - 1) / kSpLOut, maxD, 0, 0};
  const uint64_t lblocks = (uint64_t)lin.nchunks * batch;
  return mr_launch<E>((const E*)src, (E*)dst, (size_t)batch * B, B, batch, (E*)hist, maxD, B, st,
                      [&](const E* s, const E* h) {
                        if (lds <= (size_t)kSpLdsBytes) {
                          SpIn l = lin;
                          l.src = s;
                          l.hist = h;
                          hipLaunchKernelGGL(fir_sparse_lds_kernel<OP>, dim3((uint32_t)lblocks), dim3(kBlock), lds, st,
                                             (const E*)coeffs, delays, T, l, (E*)dst);
                        } else {
                          in.src = s;
                          in.hist = h;
                          hipLaunchKernelGGL((fir_sparse_kernel<OP, kSpGlob>), dim3((uint32_t)blocks), dim3(kBlock),
                                             0, st, (const E*)coeffs, delays, T, in, (E*)dst);
                        }
                        return hipSuccess;
                      });
}

hipError_t fir_sparse_run(int op, const void* coeffs, const int32_t* delays, int num_taps, int max_delay,
                          const void* src, void* dst, uint32_t block_size, uint32_t batch, void* hist, int circ_len,
                          int circ_r0, hipStream_t st) {
  switch (op) {
    case kSpF32: return sparse_launch<kSpF32>(coeffs, delays, num_taps, max_delay, src, dst, block_size, batch, hist,
                                              circ_len, circ_r0, st);
    case kSpQ31: return sparse_launch<kSpQ31>(coeffs, delays, num_taps, max_delay, src, dst, block_size, batch, hist,
                                              circ_len, circ_r0, st);
    case kSpQ15: return sparse_launch<kSpQ15>(coeffs, delays, num_taps, max_delay, src, dst, block_size, batch, hist,
                                              circ_len, circ_r0, st);
    case kSpQ7: return sparse_launch<kSpQ7>(coeffs, delays, num_taps, max_delay, src, dst, block_size, batch, hist,
                                            circ_len, circ_r0, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mi355x
