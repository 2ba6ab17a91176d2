// FIR lattice filters: arm_fir_lattice_f32 / _q31 / _q15, `batch` independent streams.
//
// Reference (Source/FilteringFunctions/arm_fir_lattice_f32.c, _q31.c, _q15.c): per sample n,
// f_0 = g_0 = x(n); stage m = 1..M with coefficient k_m:
//   f_m(n) = g_{m-1}(n-1) k_m + f_{m-1}(n),   g_m(n) = f_{m-1}(n) k_m + g_{m-1}(n-1),
// y(n) = f_M(n); the state holds g_m(n-1) for m = 0..M-1 (state[0] = the previous input).
// Arithmetic per type: f32 mul then add (no FMA); q31 ((q31)((q63 a k) >> 32) << 1) + b with
// wrap-around; q15 __SSAT(((a k) >> 15) + b, 16).
//
// The recursion runs over stages, not over time: g_m(n) depends on x(n-m .. n) only.  So a
// wave owns 64 x kLatS consecutive samples (lane l: samples a + l kLatS + j, in registers) and
// runs all M stages on them; per stage the only cross-lane value is g_{m-1} of the previous
// lane's last sample (one DPP wave_shr:1 move).  Lane 0 of the first segment of a block takes it from
// the stream's state; other segments start M - 1 samples early (x(a - 1) is exact for stage
// 1, later stages' left edge is unknown) and store only the samples whose cone lies inside
// the segment, so segments are independent waves with no barriers.  The new state (g_m at the
// block's last sample, before stage m + 1) is written by the wave that owns that sample.
// Stage counts M > kLatWS / 2 fall back to one sequential thread per stream.
#include "common.hpp"
#include "kernels.hpp"

namespace mi355x {

template <int OP> struct LatT;
template <> struct LatT<kLatF32> {
  using T = float; using V = float;
  static __device__ __forceinline__ V in(T v) { return v; }
  static __device__ __forceinline__ T out(V v) { return v; }
  // f_m = g k + f ; g_m = f k + g   (arm_fir_lattice_f32.c: (gcurr0 * k) + fcurr0)
  static __device__ __forceinline__ V step(V a, V k, V b) { const float p = a * k; return p + b; }
};
template <> struct LatT<kLatQ31> {
  using T = int32_t; using V = int32_t;
  static __device__ __forceinline__ V in(T v) { return v; }
  static __device__ __forceinline__ T out(V v) { return v; }
  static __device__ __forceinline__ V step(V a, V k, V b) {     // arm_fir_lattice_q31.c
    return (int32_t)(((uint32_t)mulhi(a, k) << 1) + (uint32_t)b);
  }
};
template <> struct LatT<kLatQ15> {
  using T = int16_t; using V = int32_t;
  static __device__ __forceinline__ V in(T v) { return v; }
  static __device__ __forceinline__ T out(V v) { return (T)v; }
  static __device__ __forceinline__ V step(V a, V k, V b) {     // arm_fir_lattice_q15.c
    return ssat16((__mul24(a, k) >> 15) + b);      // |a|, |k| <= 2^15: the 24-bit product is exact
  }
};

constexpr int kLatS = 16;                  // samples per lane
constexpr int kLatWS = 64 * kLatS;         // samples per wave

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename V>
__device__ __forceinline__ V shift_up1(V v) {
  const int r = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
  return __builtin_bit_cast(V, r);
}

struct LatIn {
  uint32_t B;
  int M;
  uint32_t V;        // valid outputs of segments 1.. (segment 0: kLatWS)
  uint32_t nseg;
};

constexpr int kLatIpw = MI355X_LAT_IPW;    // consecutive segments per wave, next one prefetched

template <int OP>
__global__ __launch_bounds__(kBlock) void fir_lattice_kernel(const typename LatT<OP>::T* __restrict__ coeffs,
                                                             const typename LatT<OP>::T* __restrict__ src,
                                                             typename LatT<OP>::T* __restrict__ dst,
                                                             const typename LatT<OP>::T* __restrict__ st_in,
                                                             typename LatT<OP>::T* __restrict__ st_out,
                                                             uint64_t waves, LatIn in) {
  using Op = LatT<OP>;
  using T = typename Op::T;
  using V = typename Op::V;
  // coefficients (and, for a block's first segment, the stream's state) staged in LDS: the
  // per-stage loads are then LDS reads instead of scalar / lane-0 global loads whose latency
  // each stage would expose
  __shared__ V kc[kLatWS / 2];
  __shared__ V st_all[kBlock / 64][kLatWS / 2];
  // coalesced global I/O through a per-wave LDS tile (lane row pitch kLatS + 1: conflict-free
  // row reads): element e = 64 i + lane <-> tile[(e / kLatS) (kLatS + 1) + e % kLatS]
  __shared__ V tile_all[kBlock / 64][64 * (kLatS + 1)];
  for (int m = threadIdx.x; m < in.M; m += kBlock) kc[m] = Op::in(coeffs[m]);
  __syncthreads();
  const uint64_t w0 = ((uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * kLatIpw;
  if (w0 >= waves) return;                 // whole waves
  const int lane = threadIdx.x & 63;
  V* tile = tile_all[threadIdx.x >> 6];
  V* stl = st_all[threadIdx.x >> 6];
  struct Seg { uint64_t f; uint32_t s; int64_t lo, a, hi; };
  auto seg = [&](uint64_t w) {
    Seg g;
    g.f = w / in.nseg;
    g.s = (uint32_t)(w - g.f * in.nseg);
    g.lo = g.s == 0 ? 0 : (int64_t)kLatWS + (int64_t)(g.s - 1) * in.V;     // first stored output
    g.a = g.s == 0 ? 0 : g.lo - (in.M - 1);                                // first processed sample
    g.hi = min((int64_t)in.B, g.s == 0 ? (int64_t)kLatWS : g.lo + in.V);
    return g;
  };
  V xv[kLatS];
  auto load = [&](const Seg& g) {          // clamped addresses, no branch per load
    const T* x = src + g.f * in.B;
#pragma unroll
    for (int i = 0; i < kLatS; ++i) {
      const int64_t p = g.a + i * 64 + lane;
      xv[i] = Op::in(x[p < (int64_t)in.B ? p : (int64_t)in.B - 1]);
    }
  };
  Seg cur = seg(w0);
  load(cur);
  const uint64_t wend = min(waves, w0 + kLatIpw);
  for (uint64_t w = w0; w < wend; ++w) {
    const uint32_t s = cur.s;
    const T* x = src + cur.f * in.B;
    wave_sync();                           // previous segment's tile reads are done
#pragma unroll
    for (int i = 0; i < kLatS; ++i) {
      const int e = i * 64 + lane;
      tile[(e / kLatS) * (kLatS + 1) + e % kLatS] = cur.a + e < (int64_t)in.B ? xv[i] : (V)0;
    }
    const V xa = s != 0 ? Op::in(x[cur.a - 1]) : (V)0;   // a >= 1 when s != 0
    if (s == 0) {
      const T* sin = st_in + cur.f * (uint64_t)in.M;
      for (int m = lane; m < in.M; m += 64) stl[m] = Op::in(sin[m]);
    }
    wave_sync();
    V fv[kLatS], gv[kLatS];
#pragma unroll
    for (int j = 0; j < kLatS; ++j) fv[j] = gv[j] = tile[lane * (kLatS + 1) + j];
    const Seg nxt = seg(w + 1 < wend ? w + 1 : w);
    if (w + 1 < wend) load(nxt);           // in flight under this segment's stages
    T* sout = st_out + cur.f * (uint64_t)in.M;
    const bool last_seg = s == in.nseg - 1;
    const int64_t off_last = (int64_t)in.B - 1 - cur.a;
    const bool own_last = last_seg && lane == (int)(off_last / kLatS);
    const int jl = (int)(off_last % kLatS);
    // the next stage's coefficient and state word are read one stage ahead (same address in
    // every lane: LDS broadcast), so the loop's only cross-lane step is the DPP shift
    V k_nx = kc[0], s_nx = s == 0 ? stl[0] : (V)0;
    for (int m = 1; m <= in.M; ++m) {
      const V k = k_nx, sv = s_nx;
      if (m < in.M) {
        k_nx = kc[m];
        s_nx = s == 0 ? stl[m] : (V)0;
      }
      if (last_seg) {                      // new state[m-1] = g_{m-1}(B - 1)
        V gl = gv[0];
#pragma unroll
        for (int j = 1; j < kLatS; ++j) gl = j == jl ? gv[j] : gl;
        if (own_last) sout[m - 1] = Op::out(gl);
      }
      V left = shift_up1(gv[kLatS - 1]);   // lane l <- lane l - 1 (wave_shr:1)
      if (lane == 0) left = s == 0 ? sv : (m == 1 ? xa : (V)0);
#pragma unroll
      for (int j = kLatS - 1; j >= 0; --j) {
        const V gp = j ? gv[j - 1] : left;
        const V fo = fv[j];
        fv[j] = Op::step(gp, k, fo);
        gv[j] = Op::step(fo, k, gp);
      }
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < kLatS; ++j) tile[lane * (kLatS + 1) + j] = fv[j];
    wave_sync();
    T* y = dst + cur.f * in.B;
    V ov[kLatS];
#pragma unroll
    for (int i = 0; i < kLatS; ++i) {
      const int e = i * 64 + lane;
      ov[i] = tile[(e / kLatS) * (kLatS + 1) + e % kLatS];
    }
#pragma unroll
    for (int i = 0; i < kLatS; ++i) {
      const int64_t p = cur.a + i * 64 + lane;
      if (p >= cur.lo && p < cur.hi) y[p] = Op::out(ov[i]);
    }
    cur = nxt;
  }
}

// M > kLatWS / 2: one thread per stream walks the samples in order with the state in memory
// (st_out, initialised from st_in by the host), exactly the reference's loop.
template <int OP>
__global__ __launch_bounds__(kBlock) void fir_lattice_seq_kernel(const typename LatT<OP>::T* __restrict__ coeffs,
                                                                 const typename LatT<OP>::T* __restrict__ src,
                                                                 typename LatT<OP>::T* __restrict__ dst,
                                                                 typename LatT<OP>::T* __restrict__ st, uint32_t batch,
                                                                 uint32_t B, int M) {
  using Op = LatT<OP>;
  using V = typename Op::V;
  const uint64_t f = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (f >= batch) return;
  const auto* x = src + f * B;
  auto* y = dst + f * B;
  auto* g = st + f * (uint64_t)M;
  for (uint32_t n = 0; n < B; ++n) {
    V fc = Op::in(x[n]);
    V gc = fc;                             // g_0(n)
    for (int m = 1; m <= M; ++m) {
      const V k = Op::in(coeffs[m - 1]);
      const V gp = Op::in(g[m - 1]);       // g_{m-1}(n-1)
      g[m - 1] = Op::out(gc);              // becomes g_{m-1}(n)
      const V fo = fc;
      fc = Op::step(gp, k, fo);
      gc = Op::step(fo, k, gp);
    }
    y[n] = Op::out(fc);
  }
}

template <int OP>
static hipError_t lattice_launch(const void* coeffs, int M, const void* src, void* dst, uint32_t B, uint32_t batch,
                                 void* state, hipStream_t st) {
  using T = typename LatT<OP>::T;
  if (batch == 0 || B == 0) return hipSuccess;
  if (M < 1 || !state) return hipErrorInvalidValue;
  const size_t sbytes = sizeof(T) * (size_t)batch * M, ib = sizeof(T) * (size_t)batch * B;
  T* tmp = nullptr;                        // old state (segment 0 reads it while the last writes)
  hipError_t e = hipMallocAsync((void**)&tmp, sbytes, st);
  if (e == hipSuccess) e = hipMemcpyAsync(tmp, state, sbytes, hipMemcpyDeviceToDevice, st);
  T* src_copy = nullptr;                   // in place: segments read inputs other waves overwrite
  const uintptr_t s0 = (uintptr_t)src, d0 = (uintptr_t)dst;
  if (e == hipSuccess && s0 < d0 + ib && d0 < s0 + ib) {
    e = hipMallocAsync((void**)&src_copy, ib, st);
    if (e == hipSuccess) e = hipMemcpyAsync(src_copy, src, ib, hipMemcpyDeviceToDevice, st);
    src = src_copy;
  }
  if (e == hipSuccess) {
    if (M <= kLatWS / 2) {
      const uint32_t V = kLatWS - (uint32_t)(M - 1);
      LatIn in{B, M, V, 1 + (B > (uint32_t)kLatWS ? (B - kLatWS + V - 1) / V : 0)};
      const uint64_t waves = (uint64_t)batch * in.nseg;
      const uint64_t wpb = (uint64_t)(kBlock / 64) * kLatIpw;
      const uint64_t blocks = (waves + wpb - 1) / wpb;
      if (blocks > 0x7fffffffu) {
        e = hipErrorInvalidValue;
      } else {
        hipLaunchKernelGGL(fir_lattice_kernel<OP>, dim3((uint32_t)blocks), dim3(kBlock), 0, st, (const T*)coeffs,
                           (const T*)src, (T*)dst, (const T*)tmp, (T*)state, waves, in);
        e = hipGetLastError();
      }
    } else {
      hipLaunchKernelGGL(fir_lattice_seq_kernel<OP>, dim3((batch + kBlock - 1) / kBlock), dim3(kBlock), 0, st,
                         (const T*)coeffs, (const T*)src, (T*)dst, (T*)state, batch, B, M);
      e = hipGetLastError();
    }
  }
  if (tmp) (void)hipFreeAsync(tmp, st);
  if (src_copy) (void)hipFreeAsync(src_copy, st);
  return e;
}

hipError_t fir_lattice_run(int op, const void* coeffs, int num_stages, const void* src, void* dst,
                           uint32_t block_size, uint32_t batch, void* state, hipStream_t st) {
  switch (op) {
    case kLatF32: return lattice_launch<kLatF32>(coeffs, num_stages, src, dst, block_size, batch, state, st);
    case kLatQ31: return lattice_launch<kLatQ31>(coeffs, num_stages, src, dst, block_size, batch, state, st);
    case kLatQ15: return lattice_launch<kLatQ15>(coeffs, num_stages, src, dst, block_size, batch, state, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mi355x
