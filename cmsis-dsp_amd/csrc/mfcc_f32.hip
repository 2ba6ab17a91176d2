// Batched MFCC f32 — MI355X kernels around the batched real FFT.
//
// Replaces Source/TransformFunctions/arm_mfcc_f32.c:83-160 (RFFT-based default path) for
// `batch` frames.  Three stream-ordered launches per batch:
//   mfcc_pre   frame max |x| (arm_absmax_f32), x*(1/max) (arm_scale_f32), x*window
//              (arm_mult_f32) -> X, max -> M            [one wave per frame]
//   rfft       arm_rfft_fast_f32 forward on X -> Y      [the bit-exact batched RFFT]
//   mfcc_post  |Y_k| for k < fftLen/2 (arm_cmplx_mag_f32, bin 0 imaginary zeroed as in
//              :124-125), *max (arm_scale_f32), Mel dot products (arm_dot_prod_f32),
//              logf(. + 1e-6f) (arm_offset_f32, arm_vlog_f32), DCT rows (arm_mat_vec_mult_f32)
//                                                       [one wave per frame, spectrum in LDS]
// Every sum is k-ordered mul-then-add as in the reference (contract off): the stages are
// bit-identical to the reference up to logf, whose device implementation may differ from
// the host libm's by an ulp.
#include "common.hpp"
#include "kernels.hpp"

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
      mel[i] = logf(sum + 1.0e-6f);
    }
  }
  __syncthreads();
  if (live) {
    float* o = dst + (size_t)frame * nb_dct;
    for (int r = lane; r < nb_dct; r += 64) {
      const float* d = dct + (size_t)r * nb_mel;
      float sum = 0.0f;
      for (int i = 0; i < nb_mel; ++i) {
        const float prod = d[i] * mel[i];
        sum = sum + prod;
      }
      o[r] = sum;
    }
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
