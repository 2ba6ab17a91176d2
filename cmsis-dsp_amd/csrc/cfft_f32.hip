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

// Work mapping.  N1024_T = 0: persistent grid, wave g takes transforms g, g + G, g + 2G, ...
// N1024_T = T > 0: grid = batch / (T * WPB) waves, wave g takes the T CONSECUTIVE transforms
// gT .. gT+T-1 (the live HBM footprint stays a compact sliding window; measured by
// tools/probes/hbm_inplace.hip).  N1024_WPB waves per workgroup, each with its own LDS image.
// Default T = 4, WPB = 8, no software prefetch: 76 % of HBM peak against 66 % for the
// persistent prefetching walk (profiles/r01/variants_n1024_mapping.txt).
// N1024_SPLIT = S > 1: workgroup b works in region b % S of the batch (S contiguous regions,
// each S-th dispatched workgroup in the same region), so S address streams far apart are
// live at once instead of one sliding window (grid % S != 0 falls back to S = 1).
constexpr int kN1024T = MI355X_N1024_T, kN1024Wpb = MI355X_N1024_WPB, kN1024Split = MI355X_N1024_SPLIT;
// Each wave owns its LDS image, so the exchanges need only a wave-level barrier: one
// wave's LDS operations complete in issue order; the fences stop the compiler from moving
// accesses across the exchange.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// DONE (the synchronous drop-in, one workgroup): after its stores the workgroup writes `seq` into
// the caller's coherent host word `done` (runtime.cpp done_slot), so the call needs no second
// launch for its completion signal.
template <bool DONE>
__global__ __launch_bounds__(64 * kN1024Wpb, MI355X_N1024_WAVES) void cfft_f32_n1024_kernel(float2* __restrict__ data, uint32_t batch,
                                                           const float2* __restrict__ tw, uint32_t flags,
                                                           uint32_t* done, uint32_t seq) {
  __shared__ __attribute__((aligned(16))) float2 lds_all[kN1024Wpb][16 * 72];
  const int l = threadIdx.x & 63;
  float2* lds = lds_all[threadIdx.x >> 6];
  uint32_t vb = blockIdx.x;
  if (kN1024Split > 1 && gridDim.x % kN1024Split == 0)
    vb = (blockIdx.x % kN1024Split) * (gridDim.x / kN1024Split) + blockIdx.x / kN1024Split;
  const uint32_t wave = vb * kN1024Wpb + (threadIdx.x >> 6);
  const uint32_t t_begin = kN1024T ? wave * kN1024T : wave;
  const uint32_t t_end = kN1024T ? min(batch, t_begin + kN1024T) : batch;
  const uint32_t t_step = kN1024T ? 1u : gridDim.x * kN1024Wpb;
  const bool ifft = flags & kIfft;
  const bool brev = flags & kBitrev;
  const float invL = 1.0f / 1024.0f;

  // lane-constant twiddles (arm_cfft_f32.c:909-933; arm_cfft_radix8_f32.c:152-174)
  const int j1 = l & 7;
#if MI355X_N1024_TWLDS
  // read from a workgroup LDS copy of tw[0, 883) at each use instead of 36 registers held across
  // the loop (the rfft1024 measurement: fewer VGPRs -> more resident waves -> more records in flight).
  // Here it does not pay (round 6, one box, Gsamples/s / HBM frac): registers 8 waves x T4 381 / 0.764;
  // LDS 16 x T1 368, 16 x T2 375, 16 x T4 355, 4 x T1 360, 4 x T4 351 -- the 9 KiB per-wave image
  // already bounds residency (125 VGPRs: 16 waves per CU either way)
  __shared__ float2 tw_l[896];
  for (int i = threadIdx.x; i < 896; i += 64 * kN1024Wpb) tw_l[i] = tw[i];
  __syncthreads();
#else
  float2 wb[4], w0[7], w1[7];
#pragma unroll
  for (int i = 0; i < 4; ++i) wb[i] = tw[l + 64 * i];
#pragma unroll
  for (int m = 0; m < 7; ++m) w0[m] = tw[2 * (m + 1) * l];          // stage 0: j = l, modifier 2
#pragma unroll
  for (int m = 0; m < 7; ++m) w1[m] = tw[16 * (m + 1) * j1];        // stage 1: j = l%8, modifier 16
#endif

// MI355X_NT: non-temporal loads/stores (the batch is streamed once; -13% without).  A
// software-pipelined variant (the next transform's loads under phases B/C) was +4% under the
// persistent walk (profiles/r01/variants_n1024.txt) and 1% slower with T = 4 consecutive
// transforms per wave; it was removed in round 3.
#if MI355X_NT
#define LD(p) ldnt(p)
#else
#define LD(p) (*(p))
#endif
  float2 a[8], b[8];
  for (uint32_t t = t_begin; t < t_end; t += t_step) {
    float2* X = data + (size_t)t * 1024;
#if MI355X_N1024_TWLDS
    int lo = l;                          // opaque per transform: the table reads stay in the loop
    asm volatile("" : "+v"(lo));
    float2 wb[4], w0[7], w1[7];
#pragma unroll
    for (int i = 0; i < 4; ++i) wb[i] = tw_l[lo + 64 * i];
#pragma unroll
    for (int m = 0; m < 7; ++m) w0[m] = tw_l[2 * (m + 1) * lo];
#pragma unroll
    for (int m = 0; m < 7; ++m) w1[m] = tw_l[16 * (m + 1) * (lo & 7)];
#endif
    // ---------------- phase A
#pragma unroll
    for (int m = 0; m < 8; ++m) { a[m] = LD(&X[l + 64 * m]); b[m] = LD(&X[512 + l + 64 * m]); }
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
  if constexpr (DONE) signal_done(done, seq);
}

// ============================================================================================
// N = 4096 specialist.  The reference runs four radix-8 DIF stages (arm_cfft_f32.c:1278,
// arm_radix8_butterfly_f32 with modifier 1: strides 512, 64, 8, 1) and the base-8 digit
// reversal.  One 256-thread workgroup per transform (T consecutive transforms per
// workgroup), the next transform's 16 loads in flight under passes 2-4; every thread runs
// two radix-8 butterflies per stage:
//   pass 1 (registers, from HBM): butterflies j = t + 256a of stage 0, elements j + 512m
//          (each load instruction covers 512 consecutive bytes per wave);
//   pass 2: stage 1, butterfly (block (t>>6) + 4a, j = t & 63), elements 512blk + j + 64m;
//   pass 3: stage 2, butterfly (block (t>>3) + 32a, j = t & 7),  elements 64blk + j + 8m;
//   pass 4: stage 3, butterfly q = rev3(t + 256a) (octal digit reversal), elements 8q + m:
//          output m of that butterfly is frequency 512m + t + 256a, so each store
//          instruction writes 512 consecutive bytes per wave -- the reversal costs nothing.
// Stage twiddles depend only on the lane (j) and stay in 56 VGPRs for the kernel's life;
// the j == 0 groups (no twiddle multiply in the reference) are selected, not branched.
// LDS image s(e) = e + 8(e>>6) + (e>>9): every access pattern above is bank-conflict free
// (modelled with the ds_read_b64 / ds_write_b64 banking of MI355X_MICROARCH.md §LDS) and
// additive, so the eight accesses of a butterfly are one base + immediate offsets.
__device__ __forceinline__ int s4096f(int e) { return e + 8 * (e >> 6) + (e >> 9); }
__device__ __forceinline__ int rev3o(int t) { return ((t & 7) << 6) | (((t >> 3) & 7) << 3) | (t >> 6); }

// Work mapping: T = 0 persistent grid-stride walk; T > 0: workgroup b takes the T consecutive
// transforms bT .. bT+T-1 (as the fixed-point N = 4096 kernels, cfft_fixed.hip).
constexpr uint32_t kN4096T = MI355X_N4096_T;
// IFFT / BREV (ifftFlag, bitReverseFlag) are template parameters so that no output word or
// address goes through a run-time select.
template <bool IFFT, bool BREV>
__global__ __launch_bounds__(256, MI355X_N4096_WAVES) void cfft_f32_n4096_kernel(float2* __restrict__ data, uint32_t batch,
                                                             const float2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) float2 lds[4607];
  const int t = threadIdx.x;
  const float invL = 1.0f / 4096.0f;
  const int j1 = t & 63, j2 = t & 7;
  float2 w0[2][7], w1[7], w2[7];
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    w0[0][m] = tw[(m + 1) * t];
    w0[1][m] = tw[(m + 1) * (t + 256)];
    w1[m] = tw[(m + 1) * j1 * 8];
    w2[m] = tw[(m + 1) * j2 * 64];
  }
  const uint32_t tr_begin = kN4096T ? blockIdx.x * kN4096T : blockIdx.x;
  const uint32_t tr_end = kN4096T ? min(batch, tr_begin + kN4096T) : batch;
  const uint32_t tr_step = kN4096T ? 1u : gridDim.x;
  if (tr_begin >= tr_end) return;
  float2 v[2][8], nv[2][8];
  const int vin = t * 8;               // byte offset of element t (buffer I/O, SGPR soffsets)
  auto fetch = [&](uint32_t tr) {
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(data + (size_t)tr * 4096, 4096 * 8);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int m = 0; m < 8; ++m) nv[a][m] = buf_ld_f2(r, vin, (256 * a + 512 * m) * 8);
  };
  // pass 1: stage 0 (modifier 1) from the prefetched words, then the next transform's loads,
  // which fly under passes 2-4.  The loop is entered after pass 1 (cfft_fx4096_kernel): the
  // wait for the prefetched words then leaves the previous transform's stores in flight.
  auto pass1 = [&](uint32_t tr) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        v[a][m] = nv[a][m];
        // conj (arm_cfft_f32.c:1252-1261) as a sign-bit flip on the copy: written as a float
        // negation the compiler split the prefetch registers and re-copied them at the back edge
        if constexpr (IFFT) asm("v_xor_b32 %0, 0x80000000, %0" : "+v"(v[a][m].y));
      }
      r8_sel(v[a], w0[a], t + 256 * a != 0);
    }
    __syncthreads();                    // the previous transform's pass-4 reads are done
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s4096f(t + 256 * a + 512 * m)] = v[a][m];
    if (tr + tr_step < tr_end) fetch(tr + tr_step);
    __syncthreads();
  };
  fetch(tr_begin);
  pass1(tr_begin);
  for (uint32_t tr = tr_begin;;) {
    float2* X = data + (size_t)tr * 4096;
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(X, 4096 * 8);
    // ---------------- pass 2: stage 1 (modifier 8)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int base = 512 * ((t >> 6) + 4 * a) + j1;
#pragma unroll
      for (int m = 0; m < 8; ++m) v[a][m] = lds[s4096f(base + 64 * m)];
      r8_sel(v[a], w1, j1 != 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s4096f(base + 64 * m)] = v[a][m];
    }
    __syncthreads();
    // ---------------- pass 3: stage 2 (modifier 64)
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int base = 64 * ((t >> 3) + 32 * a) + j2;
#pragma unroll
      for (int m = 0; m < 8; ++m) v[a][m] = lds[s4096f(base + 8 * m)];
      r8_sel(v[a], w2, j2 != 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s4096f(base + 8 * m)] = v[a][m];
    }
    __syncthreads();
    // ---------------- pass 4: stage 3 (no twiddles) + digit reversal folded into the store
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int q = rev3o(t + 256 * a);
#pragma unroll
      for (int m = 0; m < 8; ++m) v[a][m] = lds[s4096f(8 * q + m)];
      r8_core(v[a]);
      if constexpr (IFFT) {             // arm_cfft_f32.c:1285-1297
#pragma unroll
        for (int m = 0; m < 8; ++m) v[a][m] = make_float2(v[a][m].x * invL, -v[a][m].y * invL);
      }
      if constexpr (BREV) {
#pragma unroll
        for (int m = 0; m < 8; ++m) buf_st_f2(rx, vin, (512 * m + 256 * a) * 8, v[a][m]);
      } else {
        float4* Y = reinterpret_cast<float4*>(X + 8 * q);
#pragma unroll
        for (int m = 0; m < 8; m += 2) Y[m >> 1] = make_float4(v[a][m].x, v[a][m].y, v[a][m + 1].x, v[a][m + 1].y);
      }
    }
    tr += tr_step;
    if (tr >= tr_end) return;
    pass1(tr);
  }
}


// ============================================================================================
// N = 512 specialist (arm_cfft_f32.c:1270: arm_radix8_butterfly_f32 with modifier 1, 512 = 8^3,
// then the base-8 digit reversal): one wave per transform, the N = 1024 kernel's structure for
// one 512-point half.  Lane l loads x[l + 64m] and runs stage 0 (butterfly j = l) in
// registers; stage 1 through LDS (butterfly (l >> 3, j = l & 7)); stage 2 on elements
// 8l + m, whose output m is bin 64m + 8(l & 7) + (l >> 3): with bitReverseFlag each store
// instruction writes a permutation of 64 consecutive bins (512 B), without it the lane's 8
// consecutive elements (two 16-B stores).  LDS image: s1024 (conflict free for these patterns).
constexpr int kN512T = MI355X_N512_T, kN512Wpb = MI355X_N512_WPB;
template <bool IFFT, bool BREV>
__global__ __launch_bounds__(64 * kN512Wpb) void cfft_f32_n512_kernel(float2* __restrict__ data, uint32_t batch,
                                                                     const float2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) float2 lds_all[kN512Wpb][8 * 72];
  const int l = threadIdx.x & 63;
  float2* lds = lds_all[threadIdx.x >> 6];
  const uint32_t wave = blockIdx.x * kN512Wpb + (threadIdx.x >> 6);
  const uint32_t t_begin = wave * kN512T, t_end = min(batch, t_begin + kN512T);
  const float invL = 1.0f / 512.0f;
  float2 w0[7], w1[7];
  const int j1 = l & 7;
#pragma unroll
  for (int m = 0; m < 7; ++m) { w0[m] = tw[(m + 1) * l]; w1[m] = tw[8 * (m + 1) * j1]; }
  const int kbin = 8 * (l & 7) + (l >> 3);
  for (uint32_t t = t_begin; t < t_end; ++t) {
    float2* X = data + (size_t)t * 512;
    float2 a[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      a[m] = ldnt(&X[l + 64 * m]);
      if (IFFT) a[m].y = -a[m].y;                      // arm_cfft_f32.c:1252-1261
    }
    r8_sel(a, w0, l != 0);
    wave_sync();                                       // the previous transform's stage-2 reads are done
#pragma unroll
    for (int m = 0; m < 8; ++m) lds[s1024(l + 64 * m)] = a[m];
    wave_sync();
    {
      const int base = 64 * (l >> 3) + j1;
#pragma unroll
      for (int m = 0; m < 8; ++m) a[m] = lds[s1024(base + 8 * m)];
      r8_sel(a, w1, j1 != 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s1024(base + 8 * m)] = a[m];
    }
    wave_sync();
#pragma unroll
    for (int m = 0; m < 8; ++m) a[m] = lds[s1024(8 * l + m)];
    r8_core(a);
    if (IFFT) {                                        // arm_cfft_f32.c:1285-1297
#pragma unroll
      for (int m = 0; m < 8; ++m) a[m] = make_float2(a[m].x * invL, -a[m].y * invL);
    }
    if (BREV) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const v2f o = {a[m].x, a[m].y};
        __builtin_nontemporal_store(o, reinterpret_cast<v2f*>(&X[kbin + 64 * m]));
      }
    } else {
      float4* Y = reinterpret_cast<float4*>(X + 8 * l);
#pragma unroll
      for (int m = 0; m < 8; m += 2) stnt(&Y[m >> 1], make_float4(a[m].x, a[m].y, a[m + 1].x, a[m + 1].y));
    }
  }
}

// ============================================================================================
// N = 2048 specialist.  Reference: arm_cfft_radix8by4_f32 (arm_cfft_f32.c:992-1188; rows
// k <= N/8 "top", the others "bottom" with the mirrored twiddle index i = N/4 - k), then
// 3 radix-8 stages on each 512-point quarter (modifier 4: strides 64, 8, 1), then the
// mixed-radix [4, 8, 8, 8] digit reversal.  One wave per transform, as the N = 1024
// kernel, with 32 complex per lane:
//   phase A (registers): lane l loads x[l + 64m + 512c] (m, c: 32 loads of 512 B per
//            wave), runs the radix-4 pass on its eight rows k = l + 64m, then stage 0 of
//            all four quarters, whose butterflies are exactly {512c + l + 64m};
//   phase B (LDS): stage 1, quarter c, butterfly (l >> 3, j = l & 7);
//   phase C (LDS): stage 2, butterfly r = 0..3 of lane l is (c, p) = (l & 3,
//            8((l >> 2) & 7) + (l >> 5) + 2r), whose output m is frequency
//            c + 4(p >> 3) + 32(p & 7) + 256m = l + 64r + 256m: 512 consecutive bytes per
//            store instruction, the reversal costs nothing.
// LDS image (per wave) s(e) = e + 8(e >> 6) + (e >> 8): conflict free and additive for all
// three patterns (same banking model as the N = 4096 kernel).
__device__ __forceinline__ int s2048(int e) { return e + 8 * (e >> 6) + (e >> 8); }

// radix8by4 top row (k <= N/8; k == 0 leaves the three products out), :1005-1060
__device__ __forceinline__ void by4_top(float2& A, float2& B, float2& C, float2& D, float2 w2, float2 w3, float2 w4,
                                        bool tw) {
  const float ap0 = A.x + C.x, as0 = A.x - C.x, ap1 = A.y + C.y, as1 = A.y - C.y;
  const float2 t2 = make_float2(as0 + B.y - D.y, as1 - B.x + D.x);
  const float2 t3 = make_float2(ap0 - B.x - D.x, ap1 - B.y - D.y);
  const float2 t4 = make_float2(as0 - B.y + D.y, as1 + B.x - D.x);
  A = make_float2(ap0 + B.x + D.x, ap1 + B.y + D.y);
  const float2 m2 = make_float2(t2.x * w2.x + t2.y * w2.y, t2.y * w2.x - t2.x * w2.y);
  const float2 m3 = make_float2(t3.x * w3.x + t3.y * w3.y, t3.y * w3.x - t3.x * w3.y);
  const float2 m4 = make_float2(t4.x * w4.x + t4.y * w4.y, t4.y * w4.x - t4.x * w4.y);
  B = tw ? m2 : t2; C = tw ? m3 : t3; D = tw ? m4 : t4;
}
// radix8by4 bottom row kb = N/4 - i (twiddles tw[i], tw[2i], tw[3i]), :1061-1110
__device__ __forceinline__ void by4_bot(float2& A, float2& B, float2& C, float2& D, float2 w2, float2 w3, float2 w4) {
  const float ap1 = A.x + C.x, as1 = A.x - C.x, ap0 = A.y + C.y, as0 = A.y - C.y;
  const float t22 = B.y - D.y + as1;
  const float t23 = A.y - C.y - B.x + D.x;
  const float t32 = ap1 - B.x - D.x;
  const float t33 = ap0 - B.y - D.y;
  const float t42 = B.y - D.y - as1;
  const float t43 = D.x - B.x - as0;
  A = make_float2(ap1 + B.x + D.x, ap0 + B.y + D.y);
  B = make_float2(t22 * w2.y + t23 * w2.x, t23 * w2.y - t22 * w2.x);
  C = make_float2(t33 * w3.y - t32 * w3.x, -t33 * w3.x - t32 * w3.y);
  D = make_float2(t42 * w4.y + t43 * w4.x, t43 * w4.y - t42 * w4.x);
}

constexpr int kN2048T = MI355X_N2048_T, kN2048Wpb = MI355X_N2048_WPB;

__global__ __launch_bounds__(64 * kN2048Wpb) void cfft_f32_n2048_kernel(float2* __restrict__ data, uint32_t batch,
                                                                       const float2* __restrict__ tw,
                                                                       uint32_t flags) {
  __shared__ __attribute__((aligned(16))) float2 lds_all[kN2048Wpb][2303];
  const int l = threadIdx.x & 63;
  float2* lds = lds_all[threadIdx.x >> 6];
  const uint32_t wave = blockIdx.x * kN2048Wpb + (threadIdx.x >> 6);
  const uint32_t t_begin = wave * kN2048T;
  const uint32_t t_end = min(batch, t_begin + kN2048T);
  const bool ifft = flags & kIfft;
  const bool brev = flags & kBitrev;
  const float invL = 1.0f / 2048.0f;
  // lane-constant twiddles: radix8by4 rows k = l + 64m (index k for top rows, 512 - k for
  // bottom rows), stage 0 (j = l, modifier 4), stage 1 (j = l & 7, modifier 32)
  float2 wq[8][3], w0[7], w1[7];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int k = l + 64 * m, i = k <= 256 ? k : 512 - k;
#pragma unroll
    for (int u = 0; u < 3; ++u) wq[m][u] = tw[(u + 1) * i];
  }
  const int j1 = l & 7;
#pragma unroll
  for (int m = 0; m < 7; ++m) { w0[m] = tw[4 * (m + 1) * l]; w1[m] = tw[32 * (m + 1) * j1]; }

  float2 R[4][8];
  for (uint32_t t = t_begin; t < t_end; ++t) {
    float2* X = data + (size_t)t * 2048;
    // ---------------- phase A: radix-4 pass on rows l + 64m, stage 0 of the four quarters
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const float2 x = ldnt(&X[l + 64 * m + 512 * c]);
        R[c][m] = ifft ? make_float2(x.x, -x.y) : x;
      }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      if (m < 4) {
        by4_top(R[0][m], R[1][m], R[2][m], R[3][m], wq[m][0], wq[m][1], wq[m][2], m != 0 || l != 0);
      } else if (m > 4) {
        by4_bot(R[0][m], R[1][m], R[2][m], R[3][m], wq[m][0], wq[m][1], wq[m][2]);
      } else {                          // k = 256 + l: top for l == 0 (the middle row), else bottom
        float2 a = R[0][m], b = R[1][m], c = R[2][m], d = R[3][m];
        by4_top(a, b, c, d, wq[m][0], wq[m][1], wq[m][2], true);
        by4_bot(R[0][m], R[1][m], R[2][m], R[3][m], wq[m][0], wq[m][1], wq[m][2]);
        if (l == 0) { R[0][m] = a; R[1][m] = b; R[2][m] = c; R[3][m] = d; }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) r8_sel(R[c], w0, l != 0);
    wave_sync();                        // previous transform's phase C reads are done
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s2048(512 * c + l + 64 * m)] = R[c][m];
    wave_sync();
    // ---------------- phase B: stage 1
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int base = 512 * c + 64 * (l >> 3) + j1;
      float2 v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = lds[s2048(base + 8 * m)];
      r8_sel(v, w1, j1 != 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[s2048(base + 8 * m)] = v[m];
    }
    wave_sync();
    // ---------------- phase C: stage 2 + digit reversal folded into the store
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = l & 3, p = 8 * ((l >> 2) & 7) + (l >> 5) + 2 * r;
      float2 v[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = lds[s2048(512 * c + 8 * p + m)];
      r8_core(v);
      if (ifft) {                       // arm_cfft_f32.c:1285-1297
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = make_float2(v[m].x * invL, -v[m].y * invL);
      }
      if (brev) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
          const v2f o = {v[m].x, v[m].y};
          __builtin_nontemporal_store(o, reinterpret_cast<v2f*>(&X[l + 64 * r + 256 * m]));
        }
      } else {
        float4* Y = reinterpret_cast<float4*>(X + 512 * c + 8 * p);
#pragma unroll
        for (int m = 0; m < 8; m += 2) Y[m >> 1] = make_float4(v[m].x, v[m].y, v[m + 1].x, v[m + 1].y);
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

// ============================================================================================
// N = 1024, ONE transform, latency-shaped (the synchronous drop-in's batch-1 call; MI355X_N1024_LAT).
// The batched kernel gives a transform one wave, so a lone call waits for that wave to run both
// 512-point halves.  After the radix8by2 pre-pass the halves are independent (stages 0-2 of the
// radix-8 core work inside a half), so here wave h of a 2-wave workgroup runs half h alone: both
// waves load the same 16 words per lane (the pre-pass pairs x[k] with x[k + 512]), wave 0 keeps the
// sums (half 0), wave 1 the twiddled differences (half 1), and from there each wave runs the
// batched kernel's phases A-C on its own half of the LDS image with wave-level ordering only —
// the same operations in the same order, so the words are the batched kernel's (bit-exact to the
// reference).  Half 0's outputs are the even bins, half 1's the odd ones (phase C's mapping), so
// each lane stores 8-byte words.  Then the workgroup writes the caller's completion word.
__global__ __launch_bounds__(128) void cfft_f32_n1024_lat_kernel(float2* __restrict__ X, const float2* __restrict__ tw,
                                                                 uint32_t flags, uint32_t* done, uint32_t seq) {
  __shared__ __attribute__((aligned(16))) float2 lds[16 * 72];
  const int l = threadIdx.x & 63, h = threadIdx.x >> 6;    // lane, half
  const bool ifft = flags & kIfft;
  const bool brev = flags & kBitrev;
  const float invL = 1.0f / 1024.0f;
  float2 wb[4], w0[7], w1[7];
  if (h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) wb[i] = tw[l + 64 * i];
  }
#pragma unroll
  for (int m = 0; m < 7; ++m) w0[m] = tw[2 * (m + 1) * l];
  const int j1 = l & 7;
#pragma unroll
  for (int m = 0; m < 7; ++m) w1[m] = tw[16 * (m + 1) * j1];

  float2 p[8], q[8], v[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) { p[m] = X[l + 64 * m]; q[m] = X[512 + l + 64 * m]; }
  if (ifft) {
#pragma unroll
    for (int m = 0; m < 8; ++m) { p[m].y = -p[m].y; q[m].y = -q[m].y; }
  }
  if (h == 0) {                                        // radix8by2 sums (arm_cfft_f32.c:867-951)
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = make_float2(p[m].x + q[m].x, p[m].y + q[m].y);
  } else {                                             // ... and twiddled differences
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const float2 w = wb[m];
      const float2 t2 = make_float2(p[m].x - q[m].x, p[m].y - q[m].y);
      v[m] = make_float2(t2.x * w.x + t2.y * w.y, t2.y * w.x - t2.x * w.y);
      const float2 t4 = make_float2(q[m + 4].x - p[m + 4].x, q[m + 4].y - p[m + 4].y);
      v[m + 4] = make_float2(t4.x * w.y - t4.y * w.x, t4.y * w.y + t4.x * w.x);
    }
  }
  // Both waves read all of X above and each writes half of it back below: every wave's loads must
  // have returned before either wave stores (the pre-pass already waited for its own loads, so the
  // barrier costs only the other wave's skew).
  __syncthreads();
  const int hb = 512 * h;
  r8_sel(v, w0, l != 0);                               // stage 0
#pragma unroll
  for (int m = 0; m < 8; ++m) lds[s1024(hb + l + 64 * m)] = v[m];
  wave_sync();
  {                                                    // stage 1
    const int base = hb + 64 * (l >> 3) + j1;
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = lds[s1024(base + 8 * m)];
    r8_sel(v, w1, j1 != 0);
#pragma unroll
    for (int m = 0; m < 8; ++m) lds[s1024(base + 8 * m)] = v[m];
  }
  wave_sync();
#pragma unroll
  for (int m = 0; m < 8; ++m) v[m] = lds[s1024(hb + 8 * l + m)];   // stage 2
  r8_core(v);
  if (ifft) {
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = make_float2(v[m].x * invL, -v[m].y * invL);
  }
  if (brev) {
    const int kl = 2 * (l >> 3) + 16 * (l & 7) + h;    // bin of (p = l + 64 h, m = 0)
#pragma unroll
    for (int m = 0; m < 8; ++m) X[kl + 128 * m] = v[m];
  } else {
    float4* Y = reinterpret_cast<float4*>(X + hb + 8 * l);
#pragma unroll
    for (int m = 0; m < 8; m += 2) Y[m >> 1] = make_float4(v[m].x, v[m].y, v[m + 1].x, v[m + 1].y);
  }
  signal_done(done, seq);
}

// The drop-in's one N = 1024 transform (the reference's own table) with its completion word
// written by the transform's workgroup; false: not this case (the caller launches the usual way).
bool cfft_f32_n1024_done_launch(float* data, uint32_t batch, const float* tw, const uint16_t* perm, uint32_t flags,
                                uint32_t* done, uint32_t seq, hipStream_t st) {
  if (perm || batch == 0 || batch > (uint32_t)((kN1024T ? kN1024T : 1) * kN1024Wpb)) return false;
  if (MI355X_N1024_LAT && batch == 1) {
    hipLaunchKernelGGL(cfft_f32_n1024_lat_kernel, dim3(1), dim3(128), 0, st, reinterpret_cast<float2*>(data),
                       reinterpret_cast<const float2*>(tw), flags, done, seq);
    return true;
  }
  hipLaunchKernelGGL(cfft_f32_n1024_kernel<true>, dim3(1), dim3(64 * kN1024Wpb), 0, st, reinterpret_cast<float2*>(data),
                     batch, reinterpret_cast<const float2*>(tw), flags, done, seq);
  return true;
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
    case 512:
      if (!perm && MI355X_F32_N512) {   // the reference's own table: the specialist kernel
        const bool inv = flags & kIfft, brev = flags & kBitrev;
        auto k = inv ? (brev ? cfft_f32_n512_kernel<true, true> : cfft_f32_n512_kernel<true, false>)
                     : (brev ? cfft_f32_n512_kernel<false, true> : cfft_f32_n512_kernel<false, false>);
        const int per_block = kN512T * kN512Wpb;
        hipLaunchKernelGGL(k, dim3((batch + per_block - 1) / per_block), dim3(64 * kN512Wpb), 0, st, d, batch, w);
        return hipGetLastError();
      }
      return launch_f32<512>(d, batch, w, perm, flags, st);
    case 1024:
      if (!perm) {   // the reference's own table (or no reversal): the specialist kernel
        const int per_block = (kN1024T ? kN1024T : 1) * kN1024Wpb;
        int grid = (int)((batch + per_block - 1) / per_block);
        if (!kN1024T) grid = persistent_grid((const void*)cfft_f32_n1024_kernel<false>, 64 * kN1024Wpb, 0, grid, 8);
        hipLaunchKernelGGL(cfft_f32_n1024_kernel<false>, dim3(grid), dim3(64 * kN1024Wpb), 0, st, d, batch, w, flags,
                           nullptr, 0u);
        return hipGetLastError();
      }
      return launch_f32<1024>(d, batch, w, perm, flags, st);
    case 2048:
      if (!perm && MI355X_F32_N2048) {
        const int per_block = kN2048T * kN2048Wpb;
        const int grid = (int)((batch + per_block - 1) / per_block);
        hipLaunchKernelGGL(cfft_f32_n2048_kernel, dim3(grid), dim3(64 * kN2048Wpb), 0, st, d, batch, w, flags);
        return hipGetLastError();
      }
      return launch_f32<2048>(d, batch, w, perm, flags, st);
    case 4096:
      if (!perm && MI355X_F32_N4096) {   // the reference's own table: the specialist kernel
        const bool inv = flags & kIfft, brev = flags & kBitrev;
        auto k = inv ? (brev ? cfft_f32_n4096_kernel<true, true> : cfft_f32_n4096_kernel<true, false>)
                     : (brev ? cfft_f32_n4096_kernel<false, true> : cfft_f32_n4096_kernel<false, false>);
        const int grid = kN4096T ? (int)((batch + kN4096T - 1) / kN4096T) : persistent_grid((const void*)k, 256, 0, batch);
        hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, st, d, batch, w);
        return hipGetLastError();
      }
      return launch_f32<4096>(d, batch, w, perm, flags, st);
    default:   return hipSuccess;  // reference: unsupported length is a silent no-op
  }
}

}  // namespace mi355x
