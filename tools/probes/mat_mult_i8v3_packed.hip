// Batched q15 / q31 matrix multiply on the i8 matrix cores — MI355X, bit-exact.
//
// Replaces the host scalar paths of Source/MatrixFunctions/arm_mat_mult_q15.c (:741-912,
// !ARM_MATH_DSP branch: q63 sum of exact q15 products, __SSAT((sum >> 15), 16)) and
// arm_mat_mult_q31.c (:53-163: q63 sum of exact q31 products, wrapping as gcc's adds do,
// (q31)(sum >> 31)).  Both are plain integer sums, so any evaluation order gives the
// reference's bits.
//
// Byte slicing: a value v of P bytes is v = sum_p 256^p t_p + c0 with every t_p a SIGNED
// byte (the top byte as is, lower bytes offset by -128) and c0 = 128 * sum_{p<P-1} 256^p.
// Then, for C = A*B over K terms,
//   C_ij = sum_{p,q} 256^(p+q) (T^A_p T^B_q)_ij + c0 (rowsum(A)_i + colsum(B)_j) - K c0^2,
// where the P^2 plane products run on v_mfma_i32_32x32x32_i8 (exact int32 accumulation)
// into 2P-1 accumulators by weight class p+q, and the row / column sums are exact integer
// sums gathered while staging.  The result is formed in int64 (mod 2^64, as the reference
// wraps).  Accumulator bound: a class holds at most P pairs of |t t'| <= 2^14 per k, so
// K <= kMatI8MaxK keeps every int32 accumulator exact; longer K uses the VALU kernel.
// Operand maps (verified with exact data, tools/probes/mfma_i8_layout.hip): lane l holds
// A[row l&31][k = 16(l>>5) + j] and B[k = 16(l>>5) + j][col l&31] in byte j.
#include "common.hpp"
#include "kernels.hpp"

namespace mi355x {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef short s2x __attribute__((ext_vector_type(2)));

constexpr int kMatI8MaxK = 32704;

template <typename T> struct Slices;
template <> struct Slices<int16_t> { static constexpr int P = 2; static constexpr int64_t C0 = 128; };
template <> struct Slices<int32_t> { static constexpr int P = 4; static constexpr int64_t C0 = 128LL * (1 + 256 + 65536); };

// Plane p of four values given as the low bytes p of four dwords: signed bytes, the lower
// planes offset by -128 (x - 128 = x ^ 0x80 on a byte).
template <int P>
__device__ __forceinline__ uint32_t plane4(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, int p) {
  const uint32_t sel = 0x0c0c0400u + 0x0101u * (uint32_t)p;     // [v_lo.byte p, v_hi.byte p, 0, 0]
  const uint32_t lo = __builtin_amdgcn_perm(v1, v0, sel), hi = __builtin_amdgcn_perm(v3, v2, sel);
  const uint32_t w = lo | (hi << 16);
  return p == P - 1 ? w : w ^ 0x80808080u;
}

// ---- packed-plane pipeline: the byte planes are cut once per call by two HBM-bound pack
// kernels, so the GEMM itself is a plain NT i8 GEMM whose K loop is LDS-DMA staging,
// fragment reads and MFMAs only (round 2's kernel split the planes and transposed B in its
// K loop: 9.75 VALU per MFMA, MFMA busy 26 % / 44 %, profiles/r03/mat_mult_q15|q31).
//  * i8_pack_rows_kernel: A [M][K] -> plane rows p * Mp + m (t_p, 64 k-bytes per K step) and
//    rcorr[bz][Mp] = C0 * rowsum(A);
//  * i8_pack_cols_kernel: B [K][N] -> plane rows P * Mp + p * Np + n (transposed through LDS)
//    and ccorr[bz][Np] = C0 * colsum(B) - K * C0^2;
//    both into one K-step-tiled workspace [bz][K step][P (Mp + Np) rows][64 B];
//  * mat_mult_i8v3_kernel: C = sum_s 256^s (sum_{p+q=s} Ap_p Bp_q^T) + rcorr + ccorr (mod 2^64).
// Padding (rows to the tile, k to 64) is written as all-zero planes (t = 0, i.e. the value
// C0, not 0), which adds nothing to any plane product; the sums and the K * C0^2 term use
// the real values and the real K, so the identity above is exact without padded terms.
constexpr int kI8KT = 64;                      // K step (bytes of one plane row)
template <typename T> struct V3Cfg;
// Tile shapes: WM x WN waves, each owning (32 WBM) x (32 WBN) outputs with S = 2P-1 class
// accumulators per 32 x 32 subtile; D = LDS ring depth (K steps resident).  4-wave workgroups
// with a 64 KiB ring, so two independent workgroups share a CU and one's prologue, barrier
// waits and epilogue overlap the other's MFMAs.
#ifndef MI355X_I8_RING
#define MI355X_I8_RING 2
#endif
template <> struct V3Cfg<int16_t> {
  static constexpr int WM = 2, WN = 2, WBM = 2, WBN = 2, D = MI355X_I8_RING;
  static constexpr int BM = 32 * WM * WBM, BN = 32 * WN * WBN, NT = 64 * WM * WN;
};
template <> struct V3Cfg<int32_t> {
  static constexpr int WM = 2, WN = 2, WBM = 1, WBN = 1, D = MI355X_I8_RING;
  static constexpr int BM = 32 * WM * WBM, BN = 32 * WN * WBN, NT = 64 * WM * WN;
};

// plane p of the two q15 values in each of d0, d1: [d0.lo, d0.hi, d1.lo, d1.hi] byte p
template <int P>
__device__ __forceinline__ uint32_t plane_q15(uint32_t d0, uint32_t d1, int p) {
  const uint32_t sel = (uint32_t)p | (uint32_t)(2 + p) << 8 | (uint32_t)(4 + p) << 16 | (uint32_t)(6 + p) << 24;
  const uint32_t w = __builtin_amdgcn_perm(d1, d0, sel);
  return p == P - 1 ? w : w ^ 0x80808080u;
}

// plane byte t_p of one value (top plane signed as is, lower planes offset by -128)
template <int P>
__device__ __forceinline__ uint32_t tbyte(uint32_t u, int p) {
  const uint32_t b = (u >> (8 * p)) & 0xffu;
  return p == P - 1 ? b : b ^ 0x80u;
}

template <typename T>
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
#pragma unroll
  for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// One wave per row, 16 k per lane and pass (1024 k per pass); grid = (Mp / 4) * batch.
// Output: plane row prow0 + p * Mp + m of the K-step-tiled workspace (see launch_fixed).
template <typename T>
__global__ __launch_bounds__(256) void i8_pack_rows_kernel(const T* __restrict__ src, int M, int K, int Mp, int Kp,
                                                           int8_t* __restrict__ ws, int R, int64_t* __restrict__ corr,
                                                           int64_t bias) {
  constexpr int P = Slices<T>::P;
  constexpr int64_t C0 = Slices<T>::C0;
  constexpr int D = 16 * (int)sizeof(T) / 4;     // dwords of 16 values
  const int per = Mp / 4, nk = Kp / kI8KT;
  const size_t bz = blockIdx.x / (uint32_t)per;
  const int m = (int)(blockIdx.x % (uint32_t)per) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  const T* row = src + (bz * (size_t)M + (size_t)(m < M ? m : 0)) * (size_t)K;
  int8_t* out = ws + (bz * nk * (size_t)R + m) * kI8KT;
  const bool vec = ((K * (int)sizeof(T)) % 16) == 0 && (((uintptr_t)src) & 15) == 0;
  int64_t sum = 0;
  for (int k0 = 16 * lane; k0 < Kp; k0 += 1024) {
    uint32_t w[P][4];
    if (vec && m < M && k0 + 16 <= K) {
      uint32_t d[D];
      const uint4* q = reinterpret_cast<const uint4*>(row + k0);
#pragma unroll
      for (int i = 0; i < D / 4; ++i) {
        const uint4 v = q[i];
        d[4 * i] = v.x; d[4 * i + 1] = v.y; d[4 * i + 2] = v.z; d[4 * i + 3] = v.w;
      }
      if constexpr (sizeof(T) == 2) {
        int32_t s = 0;
#pragma unroll
        for (int i = 0; i < D; ++i) s = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, d[i]), s2x{1, 1}, s, false);
        sum += s;
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) w[p][q4] = plane_q15<P>(d[2 * q4], d[2 * q4 + 1], p);
      } else {
#pragma unroll
        for (int i = 0; i < D; ++i) sum += (int32_t)d[i];
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) w[p][q4] = plane4<P>(d[4 * q4], d[4 * q4 + 1], d[4 * q4 + 2], d[4 * q4 + 3], p);
      }
    } else {
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) w[p][q4] = 0;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int k = k0 + e;
        if (m < M && k < K) {
          const int32_t v = (int32_t)row[k];
          sum += v;
#pragma unroll
          for (int p = 0; p < P; ++p) w[p][e >> 2] |= tbyte<P>((uint32_t)v, p) << (8 * (e & 3));
        }
      }
    }
    int8_t* o = out + ((size_t)(k0 / kI8KT) * R) * kI8KT + (k0 % kI8KT);
#pragma unroll
    for (int p = 0; p < P; ++p)
      *reinterpret_cast<uint4*>(o + (size_t)p * Mp * kI8KT) = make_uint4(w[p][0], w[p][1], w[p][2], w[p][3]);
  }
  sum = wave_sum64<T>(sum);
  if (lane == 0) corr[bz * (size_t)Mp + m] = (int64_t)((uint64_t)C0 * (uint64_t)sum + (uint64_t)bias);
}

// 64 columns per workgroup, all of K in 128-row tiles through LDS; thread (column n =
// tid & 63, chunk c = tid >> 6) emits k = 32 c .. 32 c + 31 of its column per tile (lanes of
// a wave read 64 consecutive LDS elements of one row: no bank conflict); grid = (Np/64) * batch.
// Output: plane row prow0 + p * Np + n of the K-step-tiled workspace.
template <typename T>
__global__ __launch_bounds__(256) void i8_pack_cols_kernel(const T* __restrict__ src, int K, int N, int Np, int Kp,
                                                           int8_t* __restrict__ ws, int R, int prow0,
                                                           int64_t* __restrict__ corr, int64_t bias) {
  constexpr int P = Slices<T>::P;
  constexpr int64_t C0 = Slices<T>::C0;
  constexpr int TK = 128, PITCH = 64 + 16 / (int)sizeof(T);
  constexpr int LD = 32 * (int)sizeof(T) / 16;   // uint4 per 32-element row segment
  __shared__ __attribute__((aligned(16))) T tile[TK][PITCH];
  __shared__ int64_t red[4][64];
  const int per = Np / 64, nk = Kp / kI8KT;
  const size_t bz = blockIdx.x / (uint32_t)per;
  const int n0 = (int)(blockIdx.x % (uint32_t)per) * 64;
  const int tid = threadIdx.x, n = tid & 63, c = tid >> 6;
  const int kr = tid >> 1, cs = (tid & 1) * 32;
  const T* b = src + bz * (size_t)K * N;
  int8_t* out = ws + (bz * nk * (size_t)R + prow0 + n0 + n) * kI8KT;
  const bool vec = ((N * (int)sizeof(T)) % 16) == 0 && (((uintptr_t)src) & 15) == 0;
  const bool nval = n0 + n < N;
  int64_t sum = 0;
  for (int k0 = 0; k0 < Kp; k0 += TK) {
    const int k = k0 + kr;
    if (vec && k < K && n0 + cs + 32 <= N) {
      const uint4* q = reinterpret_cast<const uint4*>(b + (size_t)k * N + n0 + cs);
#pragma unroll
      for (int i = 0; i < LD; ++i) *reinterpret_cast<uint4*>(&tile[kr][cs + i * (16 / (int)sizeof(T))]) = q[i];
    } else {
#pragma unroll 4
      for (int e = 0; e < 32; ++e) {
        const int col = n0 + cs + e;
        tile[kr][cs + e] = (k < K && col < N) ? b[(size_t)k * N + col] : (T)0;
      }
    }
    __syncthreads();
    const int kc = k0 + 32 * c;
    if (kc < Kp) {
      uint32_t w[P][8];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int q = 0; q < 8; ++q) w[p][q] = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) {
        const int32_t v = (int32_t)tile[32 * c + i][n];
        if (nval && kc + i < K) {
          sum += v;
#pragma unroll
          for (int p = 0; p < P; ++p) w[p][i >> 2] |= tbyte<P>((uint32_t)v, p) << (8 * (i & 3));
        }
      }
      int8_t* o = out + ((size_t)(kc / kI8KT) * R) * kI8KT + (kc % kI8KT);
#pragma unroll
      for (int p = 0; p < P; ++p) {
        uint4* q = reinterpret_cast<uint4*>(o + (size_t)p * Np * kI8KT);
        q[0] = make_uint4(w[p][0], w[p][1], w[p][2], w[p][3]);
        q[1] = make_uint4(w[p][4], w[p][5], w[p][6], w[p][7]);
      }
    }
    __syncthreads();
  }
  red[c][n] = sum;
  __syncthreads();
  if (c == 0) {
    const int64_t s = red[0][n] + red[1][n] + red[2][n] + red[3][n];
    corr[bz * (size_t)Np + n0 + n] = (int64_t)((uint64_t)C0 * (uint64_t)s + (uint64_t)bias);
  }
}

// LDS image per K step: P A-plane images [BM][64 B] then P B-plane images [BN][64 B], every
// row unpadded with chunk c of row r at c ^ ((r >> 2) & 3) (conflict-free ds_read_b128
// fragment reads, tools/i8_lds_model.py).  One global_load_lds_dwordx4 fills 16 rows (1 KiB,
// lane-linear destination), so the swizzle is applied to the per-lane SOURCE address.
// Two buffers: step kt+1's LDS-DMA is issued before step kt's fragment reads and MFMAs and
// waited for (vmcnt(0)) at the step's closing barrier.
template <typename T>
__global__ __launch_bounds__(V3Cfg<T>::NT, 2) void mat_mult_i8v3_kernel(const int8_t* __restrict__ ws, int R,
                                                                     const int64_t* __restrict__ rcorr,
                                                                     const int64_t* __restrict__ ccorr,
                                                                     T* __restrict__ C, int M, int N, int Mp, int Np,
                                                                     int Kp, int fast) {
  using G = V3Cfg<T>;
  constexpr int P = Slices<T>::P, S = 2 * P - 1;
  constexpr int BM = G::BM, BN = G::BN, WBM = G::WBM, WBN = G::WBN, WN = G::WN, NW = G::WM * G::WN, D = G::D;
  constexpr int ROWS = P * (BM + BN), BUFB = ROWS * kI8KT, NG = ROWS / 16, GPW = NG / NW;
  static_assert(NG % NW == 0 && BM % 16 == 0 && BN % 16 == 0, "whole glds pieces per wave");
  static_assert(D >= 2 && D <= 4, "ring depth");
  __shared__ __attribute__((aligned(16))) int8_t lds[D * BUFB];

  // XCD-aware order: each XCD takes a contiguous run of (matrix, tile) pairs, so the tiles of a
  // matrix share its A row bands / B column bands in one L2.
  const int tilesN = Np / BN, tiles = tilesN * (Mp / BM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int t = (int)(lin % (uint32_t)tiles);
  const int row0 = (t / tilesN) * BM, col0 = (t % tilesN) * BN;
  const size_t bz = lin / (uint32_t)tiles;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // K-step-tiled workspace: step kt of matrix bz is R contiguous 64-B plane rows (A planes
  // p * Mp + m, then B planes P * Mp + p * Np + n), so one LDS-DMA piece (16 rows of a tile)
  // is 1 KiB of consecutive bytes: whole 128-B lines, each read once.
  const int nk = Kp / kI8KT;
  const int8_t* src[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int rs = (wid + NW * i) * 16 + (lane >> 2), ch = lane & 3;
    int prow, r;
    if (rs < P * BM) {
      r = rs % BM;
      prow = (rs / BM) * Mp + row0 + r;
    } else {
      r = (rs - P * BM) % BN;
      prow = P * Mp + ((rs - P * BM) / BN) * Np + col0 + r;
    }
    src[i] = ws + (bz * nk * (size_t)R + prow) * kI8KT + 16 * (ch ^ ((r >> 2) & 3));
  }
  auto issue = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < GPW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + (size_t)kt * R * kI8KT),
                                       (__attribute__((address_space(3))) void*)(lds + buf * BUFB + (wid + NW * i) * 1024),
                                       16, 0, 0);
  };

  i32x16 acc[S][WBM][WBN];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int i = 0; i < WBM; ++i)
#pragma unroll
      for (int j = 0; j < WBN; ++j) acc[s][i][j] = i32x16{};
  const int wm = wid / WN, wn = wid % WN, r = lane & 31, h = lane >> 5;
  auto step = [&](int buf) {
    const int8_t* base = lds + buf * BUFB;
#pragma unroll
    for (int kk = 0; kk < kI8KT / 32; ++kk) {
      i32x4 fa[P][WBM], fb[P][WBN];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int i = 0; i < WBM; ++i) {
          const int arow = wm * 32 * WBM + i * 32 + r;
          fa[p][i] = *reinterpret_cast<const i32x4*>(base + (p * BM + arow) * kI8KT +
                                                      16 * ((2 * kk + h) ^ ((arow >> 2) & 3)));
        }
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int j = 0; j < WBN; ++j) {
          const int brow = wn * 32 * WBN + j * 32 + r;
          fb[q][j] = *reinterpret_cast<const i32x4*>(base + (P * BM + q * BN + brow) * kI8KT +
                                                      16 * ((2 * kk + h) ^ ((brow >> 2) & 3)));
        }
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int q = 0; q < P; ++q)
#pragma unroll
          for (int i = 0; i < WBM; ++i)
#pragma unroll
            for (int j = 0; j < WBN; ++j)
              acc[p + q][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[p][i], fb[q][j], acc[p + q][i][j], 0, 0, 0);
    }
  };

  // Ring of D LDS buffers: step kt is read from buffer kt % D while steps kt+1 .. kt+D-1 are in
  // flight.  Each wave waits for its own LDS-DMA of step kt with a COUNTED vmcnt (the later
  // steps stay in flight) and the raw barrier then makes every wave's pieces visible; the same
  // barrier orders step kt-1's fragment reads (lgkmcnt(0)) before buffer (kt-1) % D is refilled.
  // __syncthreads() would drain every DMA in flight (vmcnt(0)).
#pragma unroll
  for (int i = 0; i < D - 1; ++i)
    if (i < nk) issue(i, i);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;               // steps issued after kt that may still be in flight
    if (D >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GPW) : "memory");
    else if (D >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + D - 1 < nk) issue(kt + D - 1, (kt + D - 1) % D);
    step(kt % D);
  }

  // epilogue (C/D map: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h), int64 combine
  C += bz * (size_t)M * N;
  const int64_t* rc = rcorr + bz * (size_t)Mp + row0;
  const int64_t* cc = ccorr + bz * (size_t)Np + col0;
#pragma unroll
  for (int i = 0; i < WBM; ++i) {
    int64_t rterm[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) rterm[reg] = rc[wm * 32 * WBM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h];
#pragma unroll
    for (int j = 0; j < WBN; ++j) {
      const int ccol = wn * 32 * WBN + j * 32 + r, gcol = col0 + ccol;
      const uint64_t cterm = (uint64_t)cc[ccol];
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int grow = row0 + wm * 32 * WBM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        uint64_t v = (uint64_t)rterm[reg] + cterm;
#pragma unroll
        for (int s = 0; s < S; ++s) v += (uint64_t)(int64_t)acc[s][i][j][reg] << (8 * s);
        if (grow < M && gcol < N) {
          const int64_t sum = (int64_t)v;
          // fast q15 (arm_mat_mult_fast_q15.c:356-401 host branch): q31_t modular sum, (q15)(sum >> 15)
          if constexpr (sizeof(T) == 2)
            C[(size_t)grow * N + gcol] = fast ? (T)((int32_t)(uint32_t)v >> 15) : (T)ssat16((int32_t)(sum >> 15));
          else C[(size_t)grow * N + gcol] = (T)(int32_t)(sum >> 31);
        }
      }
    }
  }
}

// K beyond the i8 accumulators' exact range: one thread per output, int64 sum.
template <typename T>
__global__ __launch_bounds__(256) void mat_mult_fixed_valu_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                                  T* __restrict__ C, int M, int K, int N,
                                                                  int fast) {
  const size_t bz = blockIdx.z;
  const int i = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j >= N) return;
  const T* a = A + bz * (size_t)M * K + (size_t)i * K;
  const T* b = B + bz * (size_t)K * N + j;
  uint64_t sum = 0;
  for (int k = 0; k < K; ++k) sum += (uint64_t)((int64_t)a[k] * b[(size_t)k * N]);
  const int64_t s = (int64_t)sum;
  if constexpr (sizeof(T) == 2)
    C[bz * (size_t)M * N + (size_t)i * N + j] = fast ? (T)((int32_t)(uint32_t)sum >> 15) : (T)ssat16((int32_t)(s >> 15));
  else C[bz * (size_t)M * N + (size_t)i * N + j] = (T)(int32_t)(s >> 31);
}

template <typename T>
static hipError_t launch_fixed(int m, int k, int n, const T* a, const T* b, T* c, uint32_t batch, hipStream_t st,
                               int fast = 0) {
  if (batch == 0 || m == 0 || n == 0) return hipSuccess;
  if (k == 0) return hipMemsetAsync(c, 0, sizeof(T) * (size_t)m * n * batch, st);
  if (k > kMatI8MaxK) {
    hipLaunchKernelGGL(mat_mult_fixed_valu_kernel<T>, dim3((n + 255) / 256, m, batch), dim3(256), 0, st, a, b, c,
                       m, k, n, fast);
    return hipGetLastError();
  }
  using G = V3Cfg<T>;
  constexpr int P = Slices<T>::P;
  constexpr int64_t C0 = Slices<T>::C0;
  const int Mp = (m + G::BM - 1) / G::BM * G::BM, Np = (n + G::BN - 1) / G::BN * G::BN;
  const int Kp = (k + kI8KT - 1) / kI8KT * kI8KT;
  // Workspace: [batch][K step][R = P (Mp + Np) plane rows][64 B] (A planes, then B planes), then
  // rcorr[batch][Mp] and ccorr[batch][Np]; stream-ordered, freed after the GEMM on the same stream
  // (the pool keeps it warm).
  const int R = P * (Mp + Np);
  const size_t planes = (size_t)batch * (size_t)R * Kp;
  const size_t bytes = planes + 8 * (size_t)batch * (Mp + Np);
  void* ws = nullptr;
  hipError_t e = hipMallocAsync(&ws, bytes, st);
  if (e != hipSuccess) return e;
  int8_t* W = static_cast<int8_t*>(ws);
  int64_t* rc = reinterpret_cast<int64_t*>(W + planes);   // Kp % 64 == 0: 8-B aligned
  int64_t* cc = rc + (size_t)batch * Mp;
  const uint64_t kc2 = (uint64_t)k * (uint64_t)C0 * (uint64_t)C0;
  hipLaunchKernelGGL(i8_pack_rows_kernel<T>, dim3((uint32_t)(Mp / 4) * batch), dim3(256), 0, st, a, m, k, Mp, Kp,
                     W, R, rc, (int64_t)0);
  hipLaunchKernelGGL(i8_pack_cols_kernel<T>, dim3((uint32_t)(Np / 64) * batch), dim3(256), 0, st, b, k, n, Np, Kp,
                     W, R, P * Mp, cc, (int64_t)(0 - kc2));
  const uint32_t tiles = (uint32_t)(Mp / G::BM) * (uint32_t)(Np / G::BN);
  hipLaunchKernelGGL(mat_mult_i8v3_kernel<T>, dim3(tiles * batch), dim3(G::NT), 0, st, W, R, rc, cc, c, m, n,
                     Mp, Np, Kp, fast);
  e = hipGetLastError();
  const hipError_t f = hipFreeAsync(ws, st);
  return e != hipSuccess ? e : f;
}

// ============================================================================================
// arm_mat_mult_fast_q31 (arm_mat_mult_fast_q31.c:152-166 / :215-266, !ARM_MATH_DSP):
// sum = (q31)(((q63)sum << 32 + a*b) >> 32) per product, i.e. sum += (a*b) >> 32 mod 2^32,
// output sum << 1.  Not an exact-product GEMM (every product is floored on its own), so it
// runs on the VALU: one v_mul_hi_i32 + one v_add per MAC, 64 x 64 tiles of 256 threads
// (4 x 4 outputs per thread), 16-deep K steps staged in LDS (A k-major so each thread reads
// its 4 rows as one 16-B word).
constexpr int kFQ_T = 64, kFQ_K = 16;
__global__ __launch_bounds__(256) void mat_mult_fast_q31_kernel(const int32_t* __restrict__ A,
                                                                const int32_t* __restrict__ B,
                                                                int32_t* __restrict__ C, int M, int K, int N,
                                                                int tiles_n) {
  __shared__ __attribute__((aligned(16))) int32_t As[kFQ_K][kFQ_T + 4];
  __shared__ __attribute__((aligned(16))) int32_t Bs[kFQ_K][kFQ_T + 4];
  const int tid = threadIdx.x;
  const size_t bz = blockIdx.y;
  const int row0 = (blockIdx.x / tiles_n) * kFQ_T, col0 = (blockIdx.x % tiles_n) * kFQ_T;
  const int32_t* a = A + bz * (size_t)M * K;
  const int32_t* b = B + bz * (size_t)K * N;
  const int tr = (tid / 16) * 4, tc = (tid % 16) * 4;
  uint32_t acc[4][4] = {};
  // loaders: A tile 64 x 16 (thread -> row tid/4, k 4*(tid%4) .. +3), B tile 16 x 64
  const int ar = tid / 4, ak = (tid % 4) * 4;
  const int bk = tid / 16, bc = (tid % 16) * 4;
  for (int k0 = 0; k0 < K; k0 += kFQ_K) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gr = row0 + ar, gk = k0 + ak + u;
      As[ak + u][ar] = (gr < M && gk < K) ? a[(size_t)gr * K + gk] : 0;
      const int gk2 = k0 + bk, gc = col0 + bc + u;
      Bs[bk][bc + u] = (gk2 < K && gc < N) ? b[(size_t)gk2 * N + gc] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kFQ_K; ++kk) {
      const int4 av = *reinterpret_cast<const int4*>(&As[kk][tr]);
      const int4 bv = *reinterpret_cast<const int4*>(&Bs[kk][tc]);
      const int32_t ar4[4] = {av.x, av.y, av.z, av.w}, bc4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += (uint32_t)mulhi(ar4[i], bc4[j]);
    }
    __syncthreads();
  }
  int32_t* c = C + bz * (size_t)M * N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gr = row0 + tr + i, gc = col0 + tc + j;
      if (gr < M && gc < N) c[(size_t)gr * N + gc] = (int32_t)(acc[i][j] << 1);
    }
}

hipError_t mat_mult_fast_q31_launch(int m, int k, int n, const int32_t* a, const int32_t* b, int32_t* c,
                                    uint32_t batch, hipStream_t st) {
  if (batch == 0 || m == 0 || n == 0) return hipSuccess;
  const int tn = (n + kFQ_T - 1) / kFQ_T, tm = (m + kFQ_T - 1) / kFQ_T;
  if (batch > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mat_mult_fast_q31_kernel, dim3(tm * tn, batch), dim3(256), 0, st, a, b, c, m, k, n, tn);
  return hipGetLastError();
}
hipError_t mat_mult_fast_q15_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c,
                                    uint32_t batch, hipStream_t st) {
  return launch_fixed<int16_t>(m, k, n, a, b, c, batch, st, 1);
}

hipError_t mat_mult_q15_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c, uint32_t batch,
                               hipStream_t st) {
  return launch_fixed<int16_t>(m, k, n, a, b, c, batch, st);
}
hipError_t mat_mult_q31_launch(int m, int k, int n, const int32_t* a, const int32_t* b, int32_t* c, uint32_t batch,
                               hipStream_t st) {
  return launch_fixed<int32_t>(m, k, n, a, b, c, batch, st);
}

}  // namespace mi355x
