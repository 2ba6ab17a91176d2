// Batched complex FFT, f32 — MI355X (gfx950) kernels.
//
// Replaces the scalar path of Source/TransformFunctions/arm_cfft_f32.c:1243-1298
// (radix8by2 :846-958, radix8by4 :960-1201) and arm_cfft_radix8_f32.c:51-291, plus the
// table-driven arm_bitreversal_32 (arm_bitreversal2.c:84-108).
//
// Design: one workgroup = 256 threads = TPB transforms, 32 KiB of
// LDS.  Each transform is read from HBM once (16-B coalesced loads) and written once;
// every butterfly pass runs LDS -> registers -> LDS.  Every floating-point operation is
// the reference's, in the reference's association order, with contraction disabled —
// the output is bit-identical to the host scalar C path, not merely within tolerance.
// The bit-reversal table is applied as the permutation it induces (folded into the
// store), computed analytically for the reference tables and taken from a device copy
// for any other table.
#include "common.hpp"
#include "kernels.hpp"
#include "cfft_f32_core.hpp"

#pragma clang fp contract(off)

namespace mi355x {

template <int N>
__global__ __launch_bounds__(kBlock) void cfft_f32_kernel(float2* __restrict__ data, uint32_t batch,
                                                          const float2* __restrict__ tw,
                                                          const uint16_t* __restrict__ perm,
                                                          uint32_t flags) {
  using P = PlanF32<N>;
  // transforms sit SP complex apart in LDS: for N <= 64 (LPT <= 4: many transforms per
  // 32-lane group, all at the same offset) one pad element keeps their lanes on distinct
  // banks; larger N pay more in occupancy (LDS > 32 KiB) than they would gain (measured)
  constexpr int SP = N + (P::LPT <= 4 ? 1 : 0);
  __shared__ __attribute__((aligned(16))) float2 lds[P::TPB * SP];
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * P::TPB;
  const int valid = (int)min<uint64_t>((uint64_t)P::TPB, batch - t0);
  const bool ifft = flags & kIfft;

  // ---- load: 16-B coalesced, conj on the fly (arm_cfft_f32.c:1252-1261)
  {
    const float4* src = reinterpret_cast<const float4*>(data + t0 * N);
    const int n4 = valid * N / 2;
#pragma unroll 4
    for (int i = tid; i < n4; i += kBlock) {
      float4 v = src[i];
      if (ifft) { v.y = -v.y; v.w = -v.w; }
      const int e = 2 * i, t = e / N, k = e % N;
      lds[t * SP + swz<N>(k)] = make_float2(v.x, v.y);
      lds[t * SP + swz<N>(k + 1)] = make_float2(v.z, v.w);
    }
  }
  __syncthreads();

  const int tr = tid / P::LPT, lane = tid % P::LPT;
  float2* x = lds + tr * SP;

  cfft_f32_lds_fwd<N>(x, lane, tw);

  // ---- store: bit reversal as a gather from LDS, conj + 1/N scale (arm_cfft_f32.c:1282-1297)
  {
    float4* dst = reinterpret_cast<float4*>(data + t0 * N);
    const bool brev = flags & kBitrev;
    const float invL = 1.0f / (float)N;
    const int n4 = valid * N / 2;
#pragma unroll 4
    for (int i = tid; i < n4; i += kBlock) {
      const int e = 2 * i, t = e / N, k = e % N;   // outputs k, k+1 of transform t
      float2 a, b;
      if (brev) {
        const int sa = perm ? perm[k] : f32_src<N>(k);
        const int sb = perm ? perm[k + 1] : f32_src<N>(k + 1);
        a = lds[t * SP + swz<N>(sa)]; b = lds[t * SP + swz<N>(sb)];
      } else {
        a = lds[t * SP + swz<N>(k)]; b = lds[t * SP + swz<N>(k + 1)];
      }
      if (ifft) {
        a.x = a.x * invL; a.y = -a.y * invL;
        b.x = b.x * invL; b.y = -b.y * invL;
      }
      dst[i] = make_float4(a.x, a.y, b.x, b.y);
    }
  }
}

// ============================================================================================
// N = 1024 specialist (the BASELINE headline).  One wave per transform, persistent over the
// batch.  Reference pass order: radix-2 pre-pass (radix8by2), then 3 radix-8 stages on each
// 512-half, then the mixed-radix [2,8,8,8] digit reversal.
//   phase A (registers): lane l loads x[l+64m] and x[512+l+64m] (m = 0..7, 512-B coalesced
//            loads), runs the radix-2 pass on those 8 pairs and stage 0 of both halves
//            (its butterflies are exactly {l+64m} and {512+l+64m});
//   phase B (LDS exchange): stage 1, lane l = (q, j) = (l/8, l%8), both halves;
//   phase C (LDS exchange): stage 2, butterflies p = l and p = l+64.  Frequency of output
//            (p, m) is k = (p>>6) + 2*((p>>3)&7) + 16*(p&7) + 128*m, so lane l holds bins k
//            (from p=l) and k+1 (from p=l+64): each output row m is one 16-B store per lane,
//            the 64 lanes covering one contiguous 1 KiB — the bit reversal costs nothing.
// Twiddles are lane-constant across transforms and live in 36 VGPRs for the kernel's life.
// LDS: 16 blocks of 64 complex padded to 72, low 3 index bits XOR-swizzled with the next 3:
// every exchange access pattern above is bank-conflict free (a row-of-9 padding variant
// used 32 fewer VGPRs but measured 1% slower).
typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float2 ldnt(const float2* p) {
  const v2f v = __builtin_nontemporal_load(reinterpret_cast<const v2f*>(p));
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ void stnt(float4* p, float4 v) {
  __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
}

__device__ __forceinline__ int s1024(int e) {
  return (e >> 6) * 72 + (((e >> 3) & 7) << 3) + ((e & 7) ^ ((e >> 3) & 7));
}

#ifndef MI355X_N1024_WAVES
#define MI355X_N1024_WAVES 1
#endif
// Work mapping.  N1024_T = 0: persistent grid, wave g takes transforms g, g + G, g + 2G, ...
// N1024_T = T > 0: grid = batch / (T * WPB) waves, wave g takes the T CONSECUTIVE transforms
// gT .. gT+T-1 (the live HBM footprint stays a compact sliding window; measured by
// tools/probes/hbm_inplace.hip).  N1024_WPB waves per workgroup, each with its own LDS image.
// Default T = 4, WPB = 8, no software prefetch: 76 % of HBM peak against 66 % for the
// persistent prefetching walk (profiles/r01/variants_n1024_mapping.txt).
#ifndef MI355X_N1024_T
#define MI355X_N1024_T 4
#endif
#ifndef MI355X_N1024_WPB
#define MI355X_N1024_WPB 8
#endif
constexpr int kN1024T = MI355X_N1024_T, kN1024Wpb = MI355X_N1024_WPB;
// Each wave owns its LDS image, so the exchanges need only a wave-level barrier: one
// wave's LDS operations complete in issue order; the fences stop the compiler from moving
// accesses across the exchange.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ __launch_bounds__(64 * kN1024Wpb, MI355X_N1024_WAVES) void cfft_f32_n1024_kernel(float2* __restrict__ data, uint32_t batch,
                                                           const float2* __restrict__ tw, uint32_t flags) {
  __shared__ __attribute__((aligned(16))) float2 lds_all[kN1024Wpb][16 * 72];
  const int l = threadIdx.x & 63;
  float2* lds = lds_all[threadIdx.x >> 6];
  const uint32_t wave = blockIdx.x * kN1024Wpb + (threadIdx.x >> 6);
  const uint32_t t_begin = kN1024T ? wave * kN1024T : wave;
  const uint32_t t_end = kN1024T ? min(batch, t_begin + kN1024T) : batch;
  const uint32_t t_step = kN1024T ? 1u : gridDim.x * kN1024Wpb;
  const bool ifft = flags & kIfft;
  const bool brev = flags & kBitrev;
  const float invL = 1.0f / 1024.0f;

  // lane-constant twiddles (arm_cfft_f32.c:909-933; arm_cfft_radix8_f32.c:152-174)
  float2 wb[4], w0[7], w1[7];
#pragma unroll
  for (int i = 0; i < 4; ++i) wb[i] = tw[l + 64 * i];
#pragma unroll
  for (int m = 0; m < 7; ++m) w0[m] = tw[2 * (m + 1) * l];          // stage 0: j = l, modifier 2
  const int j1 = l & 7;
#pragma unroll
  for (int m = 0; m < 7; ++m) w1[m] = tw[16 * (m + 1) * j1];        // stage 1: j = l%8, modifier 16

// MI355X_PF: software-pipelined loads (the next transform's 16 loads are issued right
// after phase A, in flight during phases B/C).  MI355X_NT: non-temporal loads/stores (the
// batch is streamed once).  Both on: +4% over neither under the persistent walk
// (profiles/r01/variants_n1024.txt); with T = 4 consecutive transforms per wave the prefetch
// measured 1% slower and is off, NT stays (-13% without it).
#ifndef MI355X_PF
#define MI355X_PF 0
#endif
#ifndef MI355X_NT
#define MI355X_NT 1
#endif
#if MI355X_NT
#define LD(p) ldnt(p)
#else
#define LD(p) (*(p))
#endif
  float2 a[8], b[8];
#if MI355X_PF
  float2 na[8], nb[8];
  if (t_begin < t_end) {
    const float2* X0 = data + (size_t)t_begin * 1024;
#pragma unroll
    for (int m = 0; m < 8; ++m) { na[m] = LD(&X0[l + 64 * m]); nb[m] = LD(&X0[512 + l + 64 * m]); }
  }
#endif
  for (uint32_t t = t_begin; t < t_end; t += t_step) {
    float2* X = data + (size_t)t * 1024;
    // ---------------- phase A
#if MI355X_PF
#pragma unroll
    for (int m = 0; m < 8; ++m) { a[m] = na[m]; b[m] = nb[m]; }
#else
#pragma unroll
    for (int m = 0; m < 8; ++m) { a[m] = LD(&X[l + 64 * m]); b[m] = LD(&X[512 + l + 64 * m]); }
#endif
    if (ifft) {
#pragma unroll
      for (int m = 0; m < 8; ++m) { a[m].y = -a[m].y; b[m].y = -b[m].y; }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m) {       // radix8by2 pre-pass, arm_cfft_f32.c:867-951
      const float2 w = wb[m];
      const float2 p = a[m], q = b[m];
      a[m] = make_float2(p.x + q.x, p.y + q.y);
      const float2 t2 = make_float2(p.x - q.x, p.y - q.y);
      b[m] = make_float2(t2.x * w.x + t2.y * w.y, t2.y * w.x - t2.x * w.y);
      const float2 c = a[m + 4], d = b[m + 4];
      a[m + 4] = make_float2(c.x + d.x, c.y + d.y);
      const float2 t4 = make_float2(d.x - c.x, d.y - c.y);
      b[m + 4] = make_float2(t4.x * w.y - t4.y * w.x, t4.y * w.y + t4.x * w.x);
    }
    r8_sel(a, w0, l != 0);
    r8_sel(b, w0, l != 0);
    wave_sync();                    // previous transform's phase C reads are done
#pragma unroll
    for (int m = 0; m < 8; ++m) { lds[s1024(l + 64 * m)] = a[m]; lds[s1024(512 + l + 64 * m)] = b[m]; }
#if MI355X_PF
    if (t + t_step < t_end) {          // next transform's loads fly under phases B and C
      const float2* XN = data + (size_t)(t + t_step) * 1024;
#pragma unroll
      for (int m = 0; m < 8; ++m) { na[m] = LD(&XN[l + 64 * m]); nb[m] = LD(&XN[512 + l + 64 * m]); }
    }
#endif
    wave_sync();
    // ---------------- phase B: stage 1
    {
      const int base = 64 * (l >> 3) + j1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float2 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = lds[s1024(h * 512 + base + 8 * m)];
        r8_sel(v, w1, j1 != 0);
#pragma unroll
        for (int m = 0; m < 8; ++m) lds[s1024(h * 512 + base + 8 * m)] = v[m];
      }
    }
    wave_sync();
    // ---------------- phase C: stage 2 + digit reversal folded into the store
#pragma unroll
    for (int m = 0; m < 8; ++m) { a[m] = lds[s1024(8 * l + m)]; b[m] = lds[s1024(8 * (l + 64) + m)]; }
    r8_core(a);
    r8_core(b);
    if (ifft) {                          // arm_cfft_f32.c:1285-1297
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        a[m] = make_float2(a[m].x * invL, -a[m].y * invL);
        b[m] = make_float2(b[m].x * invL, -b[m].y * invL);
      }
    }
    float4* Y = reinterpret_cast<float4*>(X);
    if (brev) {
      const int kl = 2 * (l >> 3) + 16 * (l & 7);    // bin of (p = l, m = 0)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
#if MI355X_NT
        stnt(&Y[(kl + 128 * m) >> 1], make_float4(a[m].x, a[m].y, b[m].x, b[m].y));
#else
        Y[(kl + 128 * m) >> 1] = make_float4(a[m].x, a[m].y, b[m].x, b[m].y);
#endif
      }
    } else {
#pragma unroll
      for (int m = 0; m < 8; m += 2) {
        Y[(8 * l + m) >> 1] = make_float4(a[m].x, a[m].y, a[m + 1].x, a[m + 1].y);
        Y[(8 * (l + 64) + m) >> 1] = make_float4(b[m].x, b[m].y, b[m + 1].x, b[m + 1].y);
      }
    }
  }
}

template <int N>
static hipError_t launch_f32(float2* data, uint32_t batch, const float2* tw, const uint16_t* perm,
                             uint32_t flags, hipStream_t st) {
  using P = PlanF32<N>;
  const uint32_t grid = (uint32_t)((batch + P::TPB - 1) / P::TPB);
  hipLaunchKernelGGL(cfft_f32_kernel<N>, dim3(grid), dim3(kBlock), 0, st, data, batch, tw, perm, flags);
  return hipGetLastError();
}

hipError_t cfft_f32_launch(int n, float* data, uint32_t batch, const float* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st) {
  float2* d = reinterpret_cast<float2*>(data);
  const float2* w = reinterpret_cast<const float2*>(tw);
  if (batch == 0) return hipSuccess;
  switch (n) {
    case 16:   return launch_f32<16>(d, batch, w, perm, flags, st);
    case 32:   return launch_f32<32>(d, batch, w, perm, flags, st);
    case 64:   return launch_f32<64>(d, batch, w, perm, flags, st);
    case 128:  return launch_f32<128>(d, batch, w, perm, flags, st);
    case 256:  return launch_f32<256>(d, batch, w, perm, flags, st);
    case 512:  return launch_f32<512>(d, batch, w, perm, flags, st);
    case 1024:
      if (!perm) {   // the reference's own table (or no reversal): the specialist kernel
        const int per_block = (kN1024T ? kN1024T : 1) * kN1024Wpb;
        int grid = (int)((batch + per_block - 1) / per_block);
        if (!kN1024T) grid = persistent_grid((const void*)cfft_f32_n1024_kernel, 64 * kN1024Wpb, 0, grid, 8);
        hipLaunchKernelGGL(cfft_f32_n1024_kernel, dim3(grid), dim3(64 * kN1024Wpb), 0, st, d, batch, w, flags);
        return hipGetLastError();
      }
      return launch_f32<1024>(d, batch, w, perm, flags, st);
    case 2048: return launch_f32<2048>(d, batch, w, perm, flags, st);
    case 4096: return launch_f32<4096>(d, batch, w, perm, flags, st);
    default:   return hipSuccess;  // reference: unsupported length is a silent no-op
  }
}

}  // namespace mi355x
