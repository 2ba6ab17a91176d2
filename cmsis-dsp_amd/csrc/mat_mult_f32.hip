// Batched f32 matrix multiply on the f32-input MFMA (v_mfma_f32_32x32x2_f32) — MI355X.
//
// Replaces Source/MatrixFunctions/arm_mat_mult_f32.c:600-730 (row-major C = A*B with a
// k-ordered sum per element).  v_mfma_f32_32x32x2_f32 accumulates as a k-ordered fmaf
// chain (exact f32 products summed with one rounding each): the same k order as the
// reference, one rounding fewer per term, so the result is within the normwise bound
// stated in DESIGN.md rather than bit-identical (the reference rounds a*b before the add).
//
// Tile: 128x128 per 256-thread workgroup (2x2 waves, 64x64 per wave = 2x2 MFMA 32x32
// tiles), BK = 16, LDS double buffer, A stored k-major in LDS so lanes read A[i][k] for
// consecutive i.  Workgroup ids are remapped so that the 8 column tiles of one row band
// share an XCD (L2 reuse of the A band).
#include "common.hpp"
#include "kernels.hpp"

namespace mi355x {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBM = 128, kBN = 128, kBK = 16;
constexpr int kLdA = kBM + 4;   // padded k-major rows of A (avoid write conflicts on the transpose)

__global__ __launch_bounds__(256) void mat_mult_f32_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                           float* __restrict__ C, int M, int K, int N) {
  __shared__ __attribute__((aligned(16))) float As[2][kBK][kLdA];
  __shared__ __attribute__((aligned(16))) float Bs[2][kBK][kBN];

  const int tilesN = (N + kBN - 1) / kBN, tilesM = (M + kBM - 1) / kBM;
  const int ntiles = tilesN * tilesM;
  // XCD-aware bijective remap of the linear tile id (cdna_hip_programming.md §5 'XCD swizzle')
  const int orig = blockIdx.x;
  const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tm = tile / tilesN, tn = tile % tilesN;
  const size_t bz = blockIdx.z;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int row0 = tm * kBM, col0 = tn * kBN;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // global -> register staging of one K tile: A 128x16 (8 floats/thread), B 16x128 (8 floats/thread)
  float ra[8], rb[8];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + u * 256;              // A element: row e/16, k e%16
      const int ar = e >> 4, ak = e & 15;
      const int gr = row0 + ar, gk = k0 + ak;
      ra[u] = (gr < M && gk < K) ? A[(size_t)gr * K + gk] : 0.0f;
      const int bk = e >> 7, bc = e & 127;       // B element: k e/128, col e%128
      const int gk2 = k0 + bk, gc = col0 + bc;
      rb[u] = (gk2 < K && gc < N) ? B[(size_t)gk2 * N + gc] : 0.0f;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + u * 256;
      As[buf][e & 15][e >> 4] = ra[u];
      Bs[buf][e >> 7][e & 127] = rb[u];
    }
  };

  const int nk = (K + kBK - 1) / kBK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * kBK);
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const int ka = kk + (lane >> 5);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][ka][wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[cur][ka][wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rr = row0 + wm * 64 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        const int cc = col0 + wn * 64 + j * 32 + (lane & 31);
        if (rr < M && cc < N) C[(size_t)rr * N + cc] = acc[i][j][reg];
      }
}

// Full-tile fast path (M, N multiples of 128, K a multiple of 16, 16-byte aligned rows):
// float4 global loads (2 of A and 2 of B per thread per K tile, no bounds checks), A written
// transposed into a k-major LDS tile whose row pitch of 130 words puts each 32-lane group of
// the transposing ds_write_b32 on 32 distinct banks, B written with ds_write_b128.  Half the
// registers of the general kernel, so four workgroups fit per CU (LDS- and VGPR-wise).
// Tile order (MI355X_MATF32_XCD): 0 = the 8 column tiles of one row band on one XCD (grid z =
// matrix); 1 = each XCD takes a contiguous run of (matrix, tile) pairs (1-D grid), so the 64 tiles
// of a 1024^2 matrix run together on one XCD and read its A / B panels through that XCD's L2.
#ifndef MI355X_MATF32_XCD
#define MI355X_MATF32_XCD 1
#endif
constexpr int kLdA4 = kBM + 2;

__global__ __launch_bounds__(256) void mat_mult_f32_full_kernel(const float* __restrict__ A,
                                                                const float* __restrict__ B,
                                                                float* __restrict__ C, int M, int K, int N) {
  __shared__ __attribute__((aligned(16))) float As[2][kBK][kLdA4];
  __shared__ __attribute__((aligned(16))) float Bs[2][kBK][kBN];

  const int tilesN = N / kBN, ntiles = tilesN * (M / kBM);
#if MI355X_MATF32_XCD
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int tile = (int)(lin % (uint32_t)ntiles);
  const size_t bz = lin / (uint32_t)ntiles;
#else
  const int orig = blockIdx.x;
  const int q = ntiles / 8, r = ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const size_t bz = blockIdx.z;
#endif
  const int tm = tile / tilesN, tn = tile % tilesN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int row0 = tm * kBM, col0 = tn * kBN;

  // this thread's float4 slots: A rows (tid>>2) and 64 + (tid>>2), k quad (tid&3);
  // B rows k = tid>>5 and 8 + (tid>>5), column quad (tid&31)
  const int a_row = tid >> 2, a_kq = (tid & 3) * 4;
  const int b_k = tid >> 5, b_c = (tid & 31) * 4;
  const float* pa = A + bz * (size_t)M * K + (size_t)(row0 + a_row) * K + a_kq;
  const float* pb = B + bz * (size_t)K * N + (size_t)b_k * N + col0 + b_c;
  const size_t a_step2 = (size_t)64 * K, b_step2 = (size_t)8 * N, b_tile = (size_t)kBK * N;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  float4 ra0, ra1, rb0, rb1;
#define MM_LOAD(kt)                                                              \
  do {                                                                           \
    const float* a_ = pa + (size_t)(kt) * kBK;                                   \
    const float* b_ = pb + (size_t)(kt) * b_tile;                                \
    ra0 = *reinterpret_cast<const float4*>(a_);                                  \
    ra1 = *reinterpret_cast<const float4*>(a_ + a_step2);                        \
    rb0 = *reinterpret_cast<const float4*>(b_);                                  \
    rb1 = *reinterpret_cast<const float4*>(b_ + b_step2);                        \
  } while (0)
#define MM_STORE(buf)                                                            \
  do {                                                                           \
    As[buf][a_kq + 0][a_row] = ra0.x; As[buf][a_kq + 0][a_row + 64] = ra1.x;      \
    As[buf][a_kq + 1][a_row] = ra0.y; As[buf][a_kq + 1][a_row + 64] = ra1.y;      \
    As[buf][a_kq + 2][a_row] = ra0.z; As[buf][a_kq + 2][a_row + 64] = ra1.z;      \
    As[buf][a_kq + 3][a_row] = ra0.w; As[buf][a_kq + 3][a_row + 64] = ra1.w;      \
    *reinterpret_cast<float4*>(&Bs[buf][b_k][b_c]) = rb0;                        \
    *reinterpret_cast<float4*>(&Bs[buf][b_k + 8][b_c]) = rb1;                    \
  } while (0)

  const int nk = K / kBK;
  MM_LOAD(0);
  MM_STORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) MM_LOAD(kt + 1);
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const int ka = kk + (lane >> 5);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][ka][wm * 64 + i * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[cur][ka][wn * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) MM_STORE(cur ^ 1);
    __syncthreads();
  }
#undef MM_LOAD
#undef MM_STORE

  float* c = C + bz * (size_t)M * N;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rr = row0 + wm * 64 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        const int cc = col0 + wn * 64 + j * 32 + (lane & 31);
        c[(size_t)rr * N + cc] = acc[i][j][reg];
      }
}

hipError_t mat_mult_f32_launch(int m, int k, int n, const float* a, const float* b, float* c, uint32_t batch,
                               hipStream_t st) {
  if (batch == 0 || m == 0 || n == 0) return hipSuccess;
  if (k == 0) return hipMemsetAsync(c, 0, sizeof(float) * (size_t)m * n * batch, st);
  const int tiles = ((m + kBM - 1) / kBM) * ((n + kBN - 1) / kBN);
  const bool full = m % kBM == 0 && n % kBN == 0 && k % kBK == 0 &&
                    ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0;
  if (full && (!MI355X_MATF32_XCD || (uint64_t)tiles * batch <= 0x7fffffffull)) {
    const dim3 grid = MI355X_MATF32_XCD ? dim3((uint32_t)((uint64_t)tiles * batch)) : dim3(tiles, 1, batch);
    hipLaunchKernelGGL(mat_mult_f32_full_kernel, grid, dim3(256), 0, st, a, b, c, m, k, n);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(mat_mult_f32_kernel, dim3(tiles, 1, batch), dim3(256), 0, st, a, b, c, m, k, n);
  return hipGetLastError();
}

}  // namespace mi355x
