// Real FFT (fast) f32 split / merge passes — MI355X kernels, bit-exact.
//
// arm_rfft_fast_f32 (Source/TransformFunctions/arm_rfft_fast_f32.c:675-699) is
//   forward: arm_cfft_f32(Sint, p, 0, 1) then stage_rfft_f32 (:316-402)
//   inverse: merge_rfft_f32 (:405-462) then arm_cfft_f32(Sint, pOut, 1, 1).
// Fused path (rfft_fused_kernel<H, INV>, the reference's own CFFT tables): one launch per
// batch.  Forward: frames -> LDS, the shared bit-exact CFFT(H) core (cfft_f32_core.hpp),
// then the split evaluated straight from the digit-reversed CFFT image and stored with the
// CFFT output itself (the reference leaves it in p) -- 12 B moved per real sample instead
// of 16.  Inverse: the merge evaluated while loading, the inverse CFFT core, the reversal,
// conjugate and 1/H scaling on the store -- 8 B per sample instead of 16.
// Unfused path (custom CFFT tables): cfft_f32_launch plus the O(N) passes below, one
// thread per output complex bin, with the reference's expression trees kept verbatim.
#include "common.hpp"
#include "kernels.hpp"
#include "cfft_f32_core.hpp"

#pragma clang fp contract(off)

namespace mi355x {

// forward split: X = CFFT(p) of length H = N/2 (interleaved), output N floats
__global__ __launch_bounds__(kBlock) void rfft_stage_kernel(const float2* __restrict__ X, float2* __restrict__ out,
                                                            uint64_t total, int H, const float2* __restrict__ tw) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= total) return;
  const uint64_t t = g / H;
  const int i = (int)(g % H);
  const float2* x = X + t * H;
  if (i == 0) {
    // arm_rfft_fast_f32.c:335-353: first and last bins packed into out[0], out[1]
    const float2 a = x[0];
    const float t1a = a.x + a.x, t1b = a.y + a.y;
    out[t * H] = make_float2(0.5f * (t1a + t1b), 0.5f * (t1a - t1b));
    return;
  }
  const float2 A = x[i], B = x[H - i], w = tw[i];
  const float t1a = B.x - A.x, t1b = B.y + A.y;
  const float p0 = w.x * t1a, p1 = w.y * t1a, p2 = w.x * t1b, p3 = w.y * t1b;
  out[t * H + i] = make_float2(0.5f * (A.x + B.x + p0 + p3), 0.5f * (A.y - B.y + p1 - p2));
}

// inverse merge: p holds the packed half spectrum (N floats), output feeds the inverse CFFT
__global__ __launch_bounds__(kBlock) void rfft_merge_kernel(const float2* __restrict__ X, float2* __restrict__ out,
                                                            uint64_t total, int H, const float2* __restrict__ tw) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (g >= total) return;
  const uint64_t t = g / H;
  const int i = (int)(g % H);
  const float2* x = X + t * H;
  if (i == 0) {
    const float2 a = x[0];   // arm_rfft_fast_f32.c:420-429
    out[t * H] = make_float2(0.5f * (a.x + a.y), 0.5f * (a.x - a.y));
    return;
  }
  const float2 A = x[i], B = x[H - i], w = tw[i];
  const float t1a = A.x - B.x, t1b = A.y + B.y;
  const float r = w.x * t1a, s = w.y * t1b, tt = w.y * t1a, u = w.x * t1b;
  out[t * H + i] = make_float2(0.5f * (A.x + B.x - r - s), 0.5f * (A.y - B.y + tt - u));
}

// forward split of bin i from the CFFT image x (frequency k at x[f32_src<H>(k)])
template <int H>
__device__ __forceinline__ float2 split_bin(const float2* x, int i, const float2* __restrict__ tw) {
  if (i == 0) {                                       // arm_rfft_fast_f32.c:335-353
    const float2 a = x[swz<H>(f32_src<H>(0))];
    const float t1a = a.x + a.x, t1b = a.y + a.y;
    return make_float2(0.5f * (t1a + t1b), 0.5f * (t1a - t1b));
  }
  const float2 A = x[swz<H>(f32_src<H>(i))], B = x[swz<H>(f32_src<H>(H - i))], w = tw[i];
  const float t1a = B.x - A.x, t1b = B.y + A.y;
  const float p0 = w.x * t1a, p1 = w.y * t1a, p2 = w.x * t1b, p3 = w.y * t1b;
  return make_float2(0.5f * (A.x + B.x + p0 + p3), 0.5f * (A.y - B.y + p1 - p2));
}

// inverse merge of bin i from the packed half spectrum p (arm_rfft_fast_f32.c:405-462)
__device__ __forceinline__ float2 merge_bin(const float2* __restrict__ x, int i, int H, const float2* __restrict__ tw) {
  if (i == 0) {
    const float2 a = x[0];
    return make_float2(0.5f * (a.x + a.y), 0.5f * (a.x - a.y));
  }
  const float2 A = x[i], B = x[H - i], w = tw[i];
  const float t1a = A.x - B.x, t1b = A.y + B.y;
  const float r = w.x * t1a, s = w.y * t1b, tt = w.y * t1a, u = w.x * t1b;
  return make_float2(0.5f * (A.x + B.x - r - s), 0.5f * (A.y - B.y + tt - u));
}

template <int H, bool INV>
// src and pcopy may alias (forward: the CFFT output goes back to p): every frame is read
// into LDS before the barrier and written after it, by the same workgroup.
__global__ __launch_bounds__(kBlock) void rfft_fused_kernel(const float2* src, float2* pcopy,
                                                            float2* __restrict__ dst, uint32_t batch,
                                                            const float2* __restrict__ tw,
                                                            const float2* __restrict__ twr) {
  using P = PlanF32<H>;
  constexpr int SP = H + (P::LPT <= 4 ? 1 : 0);      // as the batched CFFT's LDS image
  __shared__ __attribute__((aligned(16))) float2 lds[P::TPB * SP];
  const int tid = threadIdx.x;
  const uint64_t t0 = (uint64_t)blockIdx.x * P::TPB;
  const int valid = (int)min<uint64_t>((uint64_t)P::TPB, batch - t0);
  const int n4 = valid * H / 2;                      // float4 (two bins) per item
  {
    const float4* s4 = reinterpret_cast<const float4*>(src + t0 * H);
#pragma unroll 4
    for (int i = tid; i < n4; i += kBlock) {
      const int e = 2 * i, t = e / H, k = e % H;
      float2 a, b;
      if (INV) {                                      // merge, then conj for the inverse CFFT
        const float2* x = src + (t0 + t) * H;
        a = merge_bin(x, k, H, twr);
        b = merge_bin(x, k + 1, H, twr);
        a.y = -a.y; b.y = -b.y;
      } else {
        const float4 v = s4[i];
        a = make_float2(v.x, v.y); b = make_float2(v.z, v.w);
      }
      lds[t * SP + swz<H>(k)] = a;
      lds[t * SP + swz<H>(k + 1)] = b;
    }
  }
  __syncthreads();
  const int tr = tid / P::LPT, lane = tid % P::LPT;
  cfft_f32_lds_fwd<H>(lds + tr * SP, lane, tw);
  float4* d4 = reinterpret_cast<float4*>(dst + t0 * H);
  float4* p4 = pcopy ? reinterpret_cast<float4*>(pcopy + t0 * H) : nullptr;
  const float invL = 1.0f / (float)H;
#pragma unroll 4
  for (int i = tid; i < n4; i += kBlock) {
    const int e = 2 * i, t = e / H, k = e % H;
    const float2* x = lds + t * SP;
    if (INV) {                                        // reversal, conj, 1/H (arm_cfft_f32.c:1282-1297)
      float2 a = x[swz<H>(f32_src<H>(k))], b = x[swz<H>(f32_src<H>(k + 1))];
      a.x = a.x * invL; a.y = -a.y * invL;
      b.x = b.x * invL; b.y = -b.y * invL;
      d4[i] = make_float4(a.x, a.y, b.x, b.y);
    } else {
      const float2 a = split_bin<H>(x, k, twr), b = split_bin<H>(x, k + 1, twr);
      d4[i] = make_float4(a.x, a.y, b.x, b.y);
      if (p4) {                                       // the reference leaves the CFFT output in p
        const float2 ca = x[swz<H>(f32_src<H>(k))], cb = x[swz<H>(f32_src<H>(k + 1))];
        p4[i] = make_float4(ca.x, ca.y, cb.x, cb.y);
      }
    }
  }
}

// ============================================================================================
// Forward N = 1024 specialist (inner CFFT H = 512 = 8^3: arm_radix8_butterfly_f32 with modifier
// 1, then the base-8 digit reversal, then stage_rfft_f32): one wave per transform, as
// cfft_f32_n1024_kernel (cfft_f32.hip) with one 512-point half.  Lane l loads x[l + 64m]
// (512 B per load instruction) and runs radix-8 stage 0 (butterfly j = l) in registers;
// stage 1 through LDS (butterfly (l >> 3, j = l & 7)); stage 2 on elements 8l + m, whose
// output m is bin 64m + 8(l & 7) + (l >> 3): stored to p per m as a permutation of 64
// consecutive bins and written to LDS in natural order; the split then reads bins k and
// H - k for k = l + 64m and stores out[k] (512 B per store instruction).  LDS image: the
// N = 1024 kernel's s1024 layout (blocks of 64 padded to 72, XOR-swizzled low bits: every
// pattern above conflict free).  Twiddles are lane-constant (stage 0: 7, stage 1: 7, split: 8).
// Mapping sweep (2^20 transforms, Gsamples/s): T consecutive transforms per wave x WPB waves per
// workgroup: T1 433, T2 473, T4 460, T8 462, T2 x 4 waves 442; the generic fused kernel 441.
// T: MI355X_RF1024_T when p receives the inner CFFT output (12 B per sample), MI355X_RF1024_TS with
// ARM_MI355X_RFFT_P_SCRATCH (8 B per sample): round-5 sweep on one box, Gsamples/s with p as
// scratch: T1 545, T2 606, T4 632, T8 644 (twiddles in 44 registers: 110-128 VGPRs, 4 waves per SIMD).
// Round 6: an out-of-place 4 KiB-record stream runs 6.0 TB/s with ONE transform per wave and 5.1 with
// eight (tools/probes/hbm_oop.hip, profiles/r06/probe_hbm_oop.txt); with the twiddles read from a
// workgroup LDS copy at each use (MI355X_RF1024_TWLDS: 77-88 VGPRs, 5 waves per SIMD) short waves pay
// no per-wave register preload.  Sweep on one box (Gsamples/s, P_SCRATCH / p kept), WPB x TS/T:
// registers 8 x 8/2 650/469; LDS 8 x 8/2 640/458, 4 x 8/2 650/469, 2 x 8/2 651/484, 8 x 1/1 727/426,
// 4 x 1/1 727/477, 4 x 2/2 744/461, 4 x 2/2 strided 737/467, 2 x 1/1 645/489, 16 x 1/1 644/440.
constexpr int kRfWpb = MI355X_RF1024_WPB;
__device__ __forceinline__ int rf_s(int e) { return (e >> 6) * 72 + (((e >> 3) & 7) << 3) + ((e & 7) ^ ((e >> 3) & 7)); }
__device__ __forceinline__ void rf_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
typedef float rf_v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void rf_st(float2* p, float2 v) {
  __builtin_nontemporal_store(rf_v2f{v.x, v.y}, reinterpret_cast<rf_v2f*>(p));
}

template <int kRfT, bool KEEP_P>
#if MI355X_RF1024_WPE
#define MI355X_RF1024_ATTR __attribute__((amdgpu_waves_per_eu(MI355X_RF1024_WPE)))
#else
#define MI355X_RF1024_ATTR
#endif
__global__ __launch_bounds__(64 * kRfWpb) MI355X_RF1024_ATTR void rfft1024_fwd_kernel(float2* p, float2* __restrict__ out,
                                                                   uint32_t batch, const float2* __restrict__ tw,
                                                                   const float2* __restrict__ twr) {
  __shared__ __attribute__((aligned(16))) float2 lds_all[kRfWpb][8 * 72];
  const int l = threadIdx.x & 63;
  float2* lds = lds_all[threadIdx.x >> 6];
  const uint32_t wave = blockIdx.x * kRfWpb + (threadIdx.x >> 6), n_waves = gridDim.x * kRfWpb;
  const int j1 = l & 7;
#if MI355X_RF1024_TWLDS
  // twiddles read from a per-workgroup LDS copy at each use (tw[0, 448): stage 0 and 1, twr[0, 512):
  // the split) instead of 44 lane-constant registers held across the loop: 110-128 -> fewer VGPRs,
  // more resident waves and more 4 KiB records in flight per CU
  __shared__ float2 tw_l[448 + 512];
  for (int i = threadIdx.x; i < 448 + 512; i += 64 * kRfWpb) tw_l[i] = i < 448 ? tw[i] : twr[i - 448];
  __syncthreads();
#else
  float2 w0[7], w1[7], ws[8];
#pragma unroll
  for (int m = 0; m < 7; ++m) { w0[m] = tw[(m + 1) * l]; w1[m] = tw[8 * (m + 1) * j1]; }
#pragma unroll
  for (int m = 0; m < 8; ++m) ws[m] = twr[l + 64 * m];
#endif
  const int kbin = 8 * (l & 7) + (l >> 3);            // stage-2 output m of lane l is bin kbin + 64 m
  for (uint32_t k = 0; k < (uint32_t)kRfT; ++k) {
    // MI355X_RF1024_STRIDE: wave w takes transforms w, w + W, w + 2W ... (W waves in the grid), so
    // the waves resident at one time stream neighbouring 4 KiB records (tools/probes/hbm_oop.hip);
    // else kRfT consecutive transforms per wave
    const uint32_t t = MI355X_RF1024_STRIDE ? wave + k * n_waves : wave * kRfT + k;
    if (t >= batch) break;
    float2* X = p + (size_t)t * 512;
    float2 a[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const rf_v2f v = __builtin_nontemporal_load(reinterpret_cast<const rf_v2f*>(&X[l + 64 * m]));
      a[m] = make_float2(v.x, v.y);
    }
#if MI355X_RF1024_TWLDS
    int lo = l;                                        // opaque per transform: the reads stay in the loop
    asm volatile("" : "+v"(lo));
    float2 w0[7], w1[7];
#pragma unroll
    for (int m = 0; m < 7; ++m) { w0[m] = tw_l[(m + 1) * lo]; w1[m] = tw_l[8 * (m + 1) * (lo & 7)]; }
#endif
    r8_sel(a, w0, l != 0);                             // stage 0, arm_cfft_radix8_f32.c:152-174
    rf_wave_sync();                                    // the previous transform's split reads are done
#pragma unroll
    for (int m = 0; m < 8; ++m) lds[rf_s(l + 64 * m)] = a[m];
    rf_wave_sync();
    {                                                  // stage 1
      const int base = 64 * (l >> 3) + j1;
#pragma unroll
      for (int m = 0; m < 8; ++m) a[m] = lds[rf_s(base + 8 * m)];
      r8_sel(a, w1, j1 != 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) lds[rf_s(base + 8 * m)] = a[m];
    }
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 8; ++m) a[m] = lds[rf_s(8 * l + m)];
    r8_core(a);                                        // stage 2 (no twiddles)
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      lds[rf_s(kbin + 64 * m)] = a[m];                 // natural order for the split
      if (KEEP_P) rf_st(&X[kbin + 64 * m], a[m]);      // the reference leaves the CFFT output in p
    }
    rf_wave_sync();
    float2* Y = out + (size_t)t * 512;
#pragma unroll
    for (int m = 0; m < 8; ++m) {                      // stage_rfft_f32, arm_rfft_fast_f32.c:316-402
      const int k = l + 64 * m;
      float2 o;
      if (k == 0) {
        const float2 x0 = lds[rf_s(0)];
        const float t1a = x0.x + x0.x, t1b = x0.y + x0.y;
        o = make_float2(0.5f * (t1a + t1b), 0.5f * (t1a - t1b));
      } else {
#if MI355X_RF1024_TWLDS
        const float2 A = lds[rf_s(k)], B = lds[rf_s(512 - k)], w = tw_l[448 + (lo + 64 * m)];
#else
        const float2 A = lds[rf_s(k)], B = lds[rf_s(512 - k)], w = ws[m];
#endif
        const float t1a = B.x - A.x, t1b = B.y + A.y;
        const float p0 = w.x * t1a, p1 = w.y * t1a, p2 = w.x * t1b, p3 = w.y * t1b;
        o = make_float2(0.5f * (A.x + B.x + p0 + p3), 0.5f * (A.y - B.y + p1 - p2));
      }
      rf_st(&Y[k], o);
    }
  }
}

template <int H>
static hipError_t launch_fused(bool inv, const float* p, float* pcopy, float* out, uint32_t batch, const float* tw,
                               const float* twr, hipStream_t st) {
  using P = PlanF32<H>;
  const uint32_t grid = (uint32_t)((batch + P::TPB - 1) / P::TPB);
  auto k = inv ? rfft_fused_kernel<H, true> : rfft_fused_kernel<H, false>;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, st, (const float2*)p, (float2*)pcopy, (float2*)out, batch,
                     (const float2*)tw, (const float2*)twr);
  return hipGetLastError();
}

hipError_t rfft_f32_fused_launch(int n_real, bool inverse, const float* p, float* pcopy, float* out, uint32_t batch,
                                 const float* tw, const float* tw_rfft, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  if (MI355X_RF1024 && n_real == 1024 && !inverse && (!pcopy || pcopy == p)) {
    if (pcopy) {
      constexpr int per_block = MI355X_RF1024_T * kRfWpb;
      hipLaunchKernelGGL((rfft1024_fwd_kernel<MI355X_RF1024_T, true>), dim3((batch + per_block - 1) / per_block),
                         dim3(64 * kRfWpb), 0, st, (float2*)p, (float2*)out, batch, (const float2*)tw,
                         (const float2*)tw_rfft);
    } else {
      constexpr int per_block = MI355X_RF1024_TS * kRfWpb;
      hipLaunchKernelGGL((rfft1024_fwd_kernel<MI355X_RF1024_TS, false>), dim3((batch + per_block - 1) / per_block),
                         dim3(64 * kRfWpb), 0, st, (float2*)p, (float2*)out, batch, (const float2*)tw,
                         (const float2*)tw_rfft);
    }
    return hipGetLastError();
  }
  switch (n_real) {
#define MI_RF(N) case N: return launch_fused<N / 2>(inverse, p, pcopy, out, batch, tw, tw_rfft, st);
    MI_RF(32) MI_RF(64) MI_RF(128) MI_RF(256) MI_RF(512) MI_RF(1024) MI_RF(2048) MI_RF(4096)
#undef MI_RF
    default: return hipErrorInvalidValue;
  }
}

static hipError_t launch_pass(bool merge, int n_real, const float* p, float* out, uint32_t batch,
                              const float* tw, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const int H = n_real / 2;
  const uint64_t total = (uint64_t)batch * H;
  const uint32_t grid = (uint32_t)((total + kBlock - 1) / kBlock);
  auto k = merge ? rfft_merge_kernel : rfft_stage_kernel;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kBlock), 0, st, (const float2*)p, (float2*)out, total, H,
                     (const float2*)tw);
  return hipGetLastError();
}

hipError_t rfft_f32_stage_launch(int n_real, const float* p, float* out, uint32_t batch, const float* tw,
                                 hipStream_t st) {
  return launch_pass(false, n_real, p, out, batch, tw, st);
}
hipError_t rfft_f32_merge_launch(int n_real, const float* p, float* out, uint32_t batch, const float* tw,
                                 hipStream_t st) {
  return launch_pass(true, n_real, p, out, batch, tw, st);
}

}  // namespace mi355x
