// Batched MFCC f32 — MI355X kernels around the batched real FFT.
//
// Replaces Source/TransformFunctions/arm_mfcc_f32.c:83-160 (RFFT-based default path) for
// `batch` frames.
//
// Fused path (mfcc_fused_kernel<H>, H = fftLen/2, the default for the reference's own
// bit-reversal tables): one launch, each frame read from HBM once and only the DCT
// outputs written.  A 256-thread workgroup holds TPB = 256/(H/16) frames in 32 KiB of LDS;
// the H/16 lanes of a frame normalise + window it in LDS, run the shared bit-exact CFFT
// core (cfft_f32_core.hpp), form the split spectrum (stage_rfft_f32) directly from the
// digit-reversed CFFT output, and continue with magnitudes, Mel, log and DCT in LDS.
//
// Unfused path (custom CFFT bit-reversal tables, or more Mel filters than fftLen/2): three
// stream-ordered launches per batch:
//   mfcc_pre   frame max |x| (arm_absmax_f32), x*(1/max) (arm_scale_f32), x*window
//              (arm_mult_f32) -> X, max -> M            [one wave per frame]
//   rfft       arm_rfft_fast_f32 forward on X -> Y      [the bit-exact batched RFFT]
//   mfcc_post  |Y_k| for k < fftLen/2 (arm_cmplx_mag_f32, bin 0 imaginary zeroed as in
//              :124-125), *max (arm_scale_f32), Mel dot products (arm_dot_prod_f32),
//              logf(. + 1e-6f) (arm_offset_f32, arm_vlog_f32), DCT rows (arm_mat_vec_mult_f32)
//                                                       [one wave per frame, spectrum in LDS]
// Every sum is k-ordered mul-then-add as in the reference (contract off), and the log is the
// host libm's logf restated for the device (host_logf.hpp, proven equal on all 2^32 inputs):
// every stage is bit-identical to the reference build.
#include "common.hpp"
#include "host_logf.hpp"
#include "kernels.hpp"
#include "cfft_f32_core.hpp"

#pragma clang fp contract(off)

namespace mi355x {

constexpr int kMfccWaves = 4;   // frames (waves) per 256-thread workgroup


__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// src and x may alias (in place): each lane rewrites only the words it read
__global__ __launch_bounds__(256) void mfcc_pre_kernel(const float* src, const float* __restrict__ win,
                                                       float* x, float* maxv, int maxv_stride, int n,
                                                       uint32_t batch) {
  const int lane = threadIdx.x & 63;
  const uint32_t frame = blockIdx.x * kMfccWaves + (threadIdx.x >> 6);
  if (frame >= batch) return;
  const float4* s = reinterpret_cast<const float4*>(src + (size_t)frame * n);
  const float4* w = reinterpret_cast<const float4*>(win);
  float4* o = reinterpret_cast<float4*>(x + (size_t)frame * n);
  const int n4 = n >> 2;
  // max |x|: the reference scans with a strict '>' from |x[0]|; the maximum of the same
  // non-negative values in any order is the same value
  float m = 0.0f;
  for (int i = lane; i < n4; i += 64) {
    const float4 v = s[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  m = wave_max(m);
  const bool scale = m != 0.0f;
  const float inv = scale ? 1.0f / m : 1.0f;   // arm_mfcc_f32.c:102-105
  for (int i = lane; i < n4; i += 64) {
    float4 v = s[i];
    if (scale) { v.x = v.x * inv; v.y = v.y * inv; v.z = v.z * inv; v.w = v.w * inv; }
    const float4 c = w[i];
    o[i] = make_float4(v.x * c.x, v.y * c.y, v.z * c.z, v.w * c.w);
  }
  if (lane == 0) maxv[(size_t)frame * maxv_stride] = m;
}

// maxv may alias dst (frame maxima carried in dst[frame][0]): read before any output store
__global__ __launch_bounds__(256) void mfcc_post_kernel(const float* __restrict__ y, const float* maxv, int maxv_stride,
                                                        int n, int nb_mel, const uint32_t* __restrict__ pos,
                                                        const uint32_t* __restrict__ len,
                                                        const uint32_t* __restrict__ off,
                                                        const float* __restrict__ coefs, int nb_dct,
                                                        const float* __restrict__ dct, float* dst,
                                                        uint32_t batch) {
  extern __shared__ float sh[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int half = n >> 1;
  float* mag = sh + wave * (half + nb_mel);
  float* mel = mag + half;
  const uint32_t frame = blockIdx.x * kMfccWaves + wave;
  const bool live = frame < batch;
  const float m = live ? maxv[(size_t)frame * maxv_stride] : 0.0f;
  if (live) {
    const float2* Y = reinterpret_cast<const float2*>(y + (size_t)frame * n);
    for (int k = lane; k < half; k += 64) {
      float2 c = Y[k];
      if (k == 0) c.y = 0.0f;                          // pTmp[1] = 0 (Nyquist packed there)
      const float rr = c.x * c.x, ii = c.y * c.y;
      const float s = rr + ii;
      float v = s >= 0.0f ? sqrtf(s) : 0.0f;           // arm_sqrt_f32
      if (m != 0.0f) v = v * m;
      mag[k] = v;
    }
  }
  __syncthreads();
  if (live) {
    for (int i = lane; i < nb_mel; i += 64) {
      const uint32_t p = pos[i], l = len[i];
      const float* c = coefs + off[i];
      float sum = 0.0f;
      for (uint32_t j = 0; j < l; ++j) {
        const uint32_t k = p + j;
        const float prod = (k < (uint32_t)half ? mag[k] : 0.0f) * c[j];
        sum = sum + prod;
      }
      mel[i] = host_logf(sum + 1.0e-6f);
    }
  }
  __syncthreads();
  if (live) {
    float* o = dst + (size_t)frame * nb_dct;
    for (int r = lane; r < nb_dct; r += 64) {
      const float* d = dct + (size_t)r * nb_mel;
      float sum = 0.0f;
#pragma unroll MI355X_MFCC_UNROLL
      for (int i = 0; i < nb_mel; ++i) {
        const float prod = d[i] * mel[i];
        sum = sum + prod;
      }
      o[r] = sum;
    }
  }
}

template <int H>
__global__ __launch_bounds__(kBlock) void mfcc_fused_kernel(const float* __restrict__ src, const float* __restrict__ win,
                                                            const float2* __restrict__ tw,
                                                            const float2* __restrict__ twr, int nb_mel,
                                                            const uint32_t* __restrict__ pos,
                                                            const uint32_t* __restrict__ len,
                                                            const uint32_t* __restrict__ off,
                                                            const float* __restrict__ coefs, int nb_dct,
                                                            const float* __restrict__ dct, float* __restrict__ dst,
                                                            uint32_t batch, int total, int stage) {
  using P = PlanF32<H>;
  constexpr int NF = 2 * H, LPT = P::LPT, TPB = P::TPB;
  __shared__ __attribute__((aligned(16))) float2 lds[TPB * H];
  // the CFFT(H) and split twiddles, staged once per workgroup: every butterfly of every
  // frame reads them from LDS instead of through the vector memory path
  __shared__ __attribute__((aligned(16))) float2 tws[H], twrs[H];
  __shared__ float wmax[kBlock / 64];
  const int tid = threadIdx.x;
  for (int i = tid; i < H; i += kBlock) { tws[i] = tw[i]; twrs[i] = twr[i]; }
  // the Mel coefficients and DCT rows too, when they fit beside the frames (dynamic LDS):
  // the sequential per-filter sums then wait on LDS instead of L2
  extern __shared__ float mtab[];
  if (stage) {
    for (int i = tid; i < total; i += kBlock) mtab[i] = coefs[i];
    for (int i = tid; i < nb_mel * nb_dct; i += kBlock) mtab[total + i] = dct[i];
  }
  const float* cbase = stage ? mtab : coefs;
  const float* dbase = stage ? mtab + total : dct;
  const uint64_t f0 = (uint64_t)blockIdx.x * TPB;
  const int valid = (int)min<uint64_t>((uint64_t)TPB, batch - f0);
  {  // frames -> LDS (swizzled image), 16-B coalesced; frames past the batch end are zero-filled
    const float4* s4 = reinterpret_cast<const float4*>(src + f0 * NF);
    const int n_valid = valid * (NF / 4);
#pragma unroll 4
    for (int i = tid; i < TPB * (NF / 4); i += kBlock) {
      const float4 v = i < n_valid ? s4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      const int e = 2 * i, t = e / H, k = e % H;
      lds[t * H + swz<H>(k)] = make_float2(v.x, v.y);
      lds[t * H + swz<H>(k + 1)] = make_float2(v.z, v.w);
    }
  }
  __syncthreads();
  const int tr = tid / LPT, lane = tid % LPT;
  float2* x = lds + tr * H;
  float* xf = reinterpret_cast<float*>(x);

  // ---- max |x| over the frame's LPT lanes (arm_absmax_f32; order-free for the max value)
  float m = 0.0f;
#pragma unroll 4
  for (int j = lane; j < H; j += LPT) {
    const float2 v = x[swz<H>(j)];
    m = fmaxf(m, fmaxf(fabsf(v.x), fabsf(v.y)));
  }
  if constexpr (LPT <= 64) {
#pragma unroll
    for (int o = LPT / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  } else {
    m = wave_max(m);
    if ((tid & 63) == 0) wmax[tid >> 6] = m;
    __syncthreads();
    m = 0.0f;
#pragma unroll
    for (int w = 0; w < LPT / 64; ++w) m = fmaxf(m, wmax[tr * (LPT / 64) + w]);
  }
  const bool scale = m != 0.0f;
  const float inv = scale ? 1.0f / m : 1.0f;          // arm_mfcc_f32.c:102-105
#pragma unroll 4
  for (int j = lane; j < H; j += LPT) {
    float2 v = x[swz<H>(j)];
    if (scale) { v.x = v.x * inv; v.y = v.y * inv; }
    const float2 w = reinterpret_cast<const float2*>(win)[j];
    x[swz<H>(j)] = make_float2(v.x * w.x, v.y * w.y);  // arm_mult_f32
  }
  __syncthreads();

  cfft_f32_lds_fwd<H>(x, lane, tws);                  // arm_rfft_fast_f32.c:689 (bitrev folded below)

  // ---- stage_rfft_f32 (arm_rfft_fast_f32.c:316-402) + |.| (arm_cmplx_mag_f32) + *max
  constexpr int KPL = H / LPT;                        // bins per lane (16)
  float mg[KPL];
#pragma unroll
  for (int i = 0; i < KPL; ++i) {
    const int k = lane + i * LPT;
    float re, im;
    if (k == 0) {
      const float2 a = x[swz<H>(f32_src<H>(0))];
      const float t1a = a.x + a.x, t1b = a.y + a.y;
      re = 0.5f * (t1a + t1b);
      im = 0.0f;                                      // pTmp[1] = 0 (arm_mfcc_f32.c:125)
    } else {
      const float2 A = x[swz<H>(f32_src<H>(k))], B = x[swz<H>(f32_src<H>(H - k))], w = twrs[k];
      const float t1a = B.x - A.x, t1b = B.y + A.y;
      const float p0 = w.x * t1a, p1 = w.y * t1a, p2 = w.x * t1b, p3 = w.y * t1b;
      re = 0.5f * (A.x + B.x + p0 + p3);
      im = 0.5f * (A.y - B.y + p1 - p2);
    }
    const float rr = re * re, ii = im * im;
    const float sq = rr + ii;
    float v = sq >= 0.0f ? sqrtf(sq) : 0.0f;
    if (scale) v = v * m;
    mg[i] = v;
  }
  __syncthreads();                                    // every spectrum read is done
  // Magnitudes then log-Mel values in the frame's own LDS rows.  The Mel stage runs one thread
  // per (filter, frame) pair, frame fastest (thread t: frame t % TPB, filter t / TPB), so a wave
  // holds a few CONSECUTIVE filters -- similar lengths (the suite's run 12 .. 115 taps) -- and its
  // loop runs to their longest instead of to the longest of all filters (one lane per filter:
  // ~26 % of the lanes' iterations did work).  Each sum keeps its sequential order.  A per-frame
  // skew of the magnitude rows puts the same bin of up to 8 frames on different banks.
  const bool skewed = nb_mel <= H - 8;
  const int skew = skewed ? (tr & 7) : 0, melo = skewed ? H + 8 : H;
  {
    float* mag = xf + skew;
#pragma unroll
    for (int i = 0; i < KPL; ++i) mag[lane + i * LPT] = mg[i];
  }
  __syncthreads();
  for (int q = tid; q < TPB * nb_mel; q += kBlock) {
    const int f = q % TPB, i = q / TPB;
    const float* mag = reinterpret_cast<const float*>(lds + f * H) + (skewed ? (f & 7) : 0);
    const uint32_t p = pos[i], l = len[i];
    const float* c = cbase + off[i];
    float sum = 0.0f;
#pragma unroll MI355X_MFCC_UNROLL
    for (uint32_t j = 0; j < l; ++j) {
      const uint32_t k = p + j;
      const float prod = (k < (uint32_t)H ? mag[k] : 0.0f) * c[j];
      sum = sum + prod;
    }
    reinterpret_cast<float*>(lds + f * H)[melo + i] = host_logf(sum + 1.0e-6f);
  }
  __syncthreads();
  const float* mel = xf + melo;
  if (tr < valid) {
    float* o = dst + (f0 + tr) * (uint64_t)nb_dct;
    for (int r = lane; r < nb_dct; r += LPT) {
      const float* d = dbase + (size_t)r * nb_mel;
      float sum = 0.0f;
#pragma unroll MI355X_MFCC_UNROLL
      for (int i = 0; i < nb_mel; ++i) {
        const float prod = d[i] * mel[i];
        sum = sum + prod;
      }
      o[r] = sum;
    }
  }
}

template <int H>
static hipError_t launch_fused(const float* src, const float* win, const float* tw, const float* twr, int nb_mel,
                               const uint32_t* pos, const uint32_t* len, const uint32_t* off, const float* coefs,
                               int nb_dct, const float* dct, float* dst, uint32_t batch, int total, hipStream_t st) {
  constexpr int TPB = PlanF32<H>::TPB;
  const uint32_t grid = (uint32_t)((batch + TPB - 1) / TPB);
  static size_t static_lds = 0;
  if (!static_lds) {
    hipFuncAttributes a;
    static_lds = hipFuncGetAttributes(&a, (const void*)mfcc_fused_kernel<H>) == hipSuccess ? a.sharedSizeBytes : 65536;
  }
  const size_t dyn = sizeof(float) * ((size_t)total + (size_t)nb_mel * nb_dct);
  const int stage = total > 0 && static_lds + dyn <= 65536 ? 1 : 0;
  hipLaunchKernelGGL(mfcc_fused_kernel<H>, dim3(grid), dim3(kBlock), stage ? dyn : 0, st, src, win, (const float2*)tw,
                     (const float2*)twr, nb_mel, pos, len, off, coefs, nb_dct, dct, dst, batch, total, stage);
  return hipGetLastError();
}

hipError_t mfcc_f32_fused_launch(int n, const float* src, const float* win, const float* tw, const float* twr,
                                 int nb_mel, const uint32_t* pos, const uint32_t* len, const uint32_t* off,
                                 const float* coefs, int nb_dct, const float* dct, float* dst, uint32_t batch,
                                 int total, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  if (nb_mel > n / 2) return hipErrorInvalidValue;
  switch (n) {
#define MI_FUSED(NF) \
    case NF: return launch_fused<NF / 2>(src, win, tw, twr, nb_mel, pos, len, off, coefs, nb_dct, dct, dst, batch, \
                                         total, st);
    MI_FUSED(32) MI_FUSED(64) MI_FUSED(128) MI_FUSED(256) MI_FUSED(512) MI_FUSED(1024) MI_FUSED(2048) MI_FUSED(4096)
#undef MI_FUSED
    default: return hipErrorInvalidValue;
  }
}

hipError_t mfcc_f32_pre_launch(int n, const float* src, const float* win, float* x, float* maxv, uint32_t batch,
                               int maxv_stride, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMfccWaves - 1) / kMfccWaves;
  hipLaunchKernelGGL(mfcc_pre_kernel, dim3(grid), dim3(64 * kMfccWaves), 0, st, src, win, x, maxv, maxv_stride, n,
                     batch);
  return hipGetLastError();
}

size_t mfcc_f32_post_lds(int n, int nb_mel) { return sizeof(float) * kMfccWaves * (size_t)(n / 2 + nb_mel); }

hipError_t mfcc_f32_post_launch(int n, const float* y, const float* maxv, int maxv_stride, int nb_mel,
                                const uint32_t* pos,
                                const uint32_t* len, const uint32_t* off, const float* coefs, int nb_dct,
                                const float* dct, float* dst, uint32_t batch, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const uint32_t grid = (batch + kMfccWaves - 1) / kMfccWaves;
  hipLaunchKernelGGL(mfcc_post_kernel, dim3(grid), dim3(64 * kMfccWaves), mfcc_f32_post_lds(n, nb_mel), st, y, maxv,
                     maxv_stride, n, nb_mel, pos, len, off, coefs, nb_dct, dct, dst, batch);
  return hipGetLastError();
}

}  // namespace mi355x
