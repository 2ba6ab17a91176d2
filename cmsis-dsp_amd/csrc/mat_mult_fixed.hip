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
#include <type_traits>

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

// ---- v2 kernel: 128 x 128 (q15) / 128 x 64 (q31) workgroup tiles of 8 waves (4 x 2), wave
// tiles 32 x 64 / 32 x 32 (accumulators fit two waves per SIMD, so one wave's MFMAs overlap
// the other's staging), double-buffered LDS planes (one barrier per K step), step kt+2's
// global loads in flight under step kt's MFMAs.  B arrives row-major [k][n]; the MFMA wants
// 16 k-consecutive bytes per column, so staging transposes 4 k-rows x CW columns per thread
// into k-contiguous dwords (v_perm) before the LDS write.
template <typename T> struct I8Cfg;
template <> struct I8Cfg<int16_t> { static constexpr int BM = 128, BN = 128, WBM = 1, WBN = 2, KT = 64; };
template <> struct I8Cfg<int32_t> { static constexpr int BM = 128, BN = 64, WBM = 1, WBN = 1, KT = 64; };
constexpr int kNT2 = 512, kWavesM = 4, kWavesN = 2;

// LDS plane layout: rows of 64 k-bytes (4 chunks of 16 B) with no padding; chunk c of row
// `row` sits at chunk c ^ ((row >> 2) & 3), and B's column `col` at row col ^ ((col >> CWL) & 1)
// (CWL = log2 of the columns one staging thread owns).  Conflict free for every access
// (MI355X_MICROARCH.md §LDS):
//  * fragment reads (ds_read_b128, 16-lane groups {0-3,12-15,20-27}, ..., banks mod 64): the 16
//    rows of a group hold (row mod 4, swizzled chunk) pairs that are all distinct, i.e. 16
//    distinct 4-bank sets (B's row permutation only swaps rows within such groups);
//  * A staging (ds_write_b128, 8 contiguous lanes, banks mod 32): two consecutive rows x 4
//    chunks -- the rows' parities differ, so the 16-dword halves do;
//  * B staging (ds_write_b32, 32-lane groups, banks mod 32): lanes 0-15 and 16-31 write 16
//    k-dwords of columns CW apart, whose rows the column permutation gives opposite parities.
// (Round 2's 80-byte pitch left both staging writes two-way conflicted: 12.5 M / 54.8 M conflict
// cycles per launch for q15 / q31, profiles/r02/mat_mult_q15|q31/pmc.json.)
__device__ __forceinline__ int i8_chunk(int row, int c) { return (c ^ (row >> 2)) & 3; }
template <int CW> __device__ __forceinline__ int i8_brow(int col) {
  constexpr int L = CW == 8 ? 3 : CW == 4 ? 2 : CW == 2 ? 1 : 0;
  return col ^ ((col >> L) & 1);
}
// B8 staging (ds_write_b64 of 8 k-bytes, 16-lane groups on consecutive column pairs, banks mod 32):
// flipping the row parity on bit 1 of the column spreads a group over both row parities, the
// most any 16 writes of 8 bytes into 64-byte rows can use (2-way); fragment reads keep each
// aligned row quad, so they stay conflict free.
__device__ __forceinline__ int i8_brow8(int col) { return col ^ ((col >> 1) & 1); }

// plane p of the two q15 values in each of d0, d1: [d0.lo, d0.hi, d1.lo, d1.hi] byte p
template <int P>
__device__ __forceinline__ uint32_t plane_q15(uint32_t d0, uint32_t d1, int p) {
  const uint32_t sel = (uint32_t)p | (uint32_t)(2 + p) << 8 | (uint32_t)(4 + p) << 16 | (uint32_t)(6 + p) << 24;
  const uint32_t w = __builtin_amdgcn_perm(d1, d0, sel);
  return p == P - 1 ? w : w ^ 0x80808080u;
}
// byte o of r0, r1, r2, r3 -> one dword (k-consecutive bytes of one column)
__device__ __forceinline__ uint32_t gather4(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, int o) {
  const uint32_t sel = (uint32_t)o | (uint32_t)(4 + o) << 8 | 0x0c0c0000u;
  return __builtin_amdgcn_perm(r1, r0, sel) | (__builtin_amdgcn_perm(r3, r2, sel) << 16);
}

// Diagnostic build only (MI355X_I8_STAMPS, tools/probes/i8_phases.py): thread 0 of each
// workgroup records s_memtime after the tile decode, the prologue, the K loop, the epilogue
// arithmetic and the copy-out, plus s_memrealtime and its HW_ID / XCC_ID, into a device buffer.
#if MI355X_I8_STAMPS
constexpr int kI8Stamps = 1 << 16;
__device__ uint64_t g_i8_stamps[kI8Stamps][8];
#define I8_STAMP(i)                                                                       \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.x < (uint32_t)kI8Stamps) {                           \
      g_i8_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memtime();                          \
      if ((i) == 0) {                                                                     \
        g_i8_stamps[blockIdx.x][5] = __builtin_amdgcn_s_memrealtime();                    \
        g_i8_stamps[blockIdx.x][7] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | \
                                     ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32); \
      }                                                                                   \
      if ((i) == 4) g_i8_stamps[blockIdx.x][6] = __builtin_amdgcn_s_memrealtime();        \
    }                                                                                     \
  } while (0)
#else
#define I8_STAMP(i) do { } while (0)
#endif

// FULL: M % BM == 0, N % BN == 0, K % 64 == 0 and 16-B / 8-B aligned rows -- no bounds
// checks, so the K loop is one basic block the scheduler can interleave (loads, staging,
// MFMAs); otherwise every load is guarded and zero-filled.
template <typename T, bool FULL>
__global__ __launch_bounds__(kNT2) void mat_mult_i8v2_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                             T* __restrict__ C, int M, int K, int N, int fast) {
  using G = I8Cfg<T>;
  constexpr int P = Slices<T>::P, S = 2 * P - 1;
  constexpr int64_t C0 = Slices<T>::C0;
  constexpr int BM = G::BM, BN = G::BN, WBM = G::WBM, WBN = G::WBN, kKT2 = G::KT, kPitch2 = kKT2;
  static_assert(kKT2 == 64, "the LDS swizzle assumes 4 chunks of 16 k-bytes per row");
  static_assert(BM == kWavesM * 32 * WBM && BN == kWavesN * 32 * WBN, "wave grid covers the tile");
  constexpr int EPD = 4 / sizeof(T);             // elements per dword
  constexpr int AK = BM * kKT2 / kNT2;           // A elements per staging thread (16)
  constexpr int AKD = AK / EPD;                  // ... as dwords
  constexpr int AQ = kKT2 / AK;                  // threads per A row (4)
  constexpr int NQ = kKT2 / 4;                   // k-quads per K step
  constexpr int CW = BN / (kNT2 / NQ);           // B columns per staging thread (8 q15 / 2 q31)
  constexpr int BD = CW / EPD;                   // dwords per B k-row segment (4 / 2)
  constexpr int BUF = P * (BM + BN) * kPitch2;   // one K step's planes; two buffers
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * BUF];

  // XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so the linear id is
  // permuted to give each XCD a contiguous run of (matrix, tile) pairs -- the tiles of one
  // matrix then share their A row bands / B column bands in that XCD's L2.
  const int tilesN = (N + BN - 1) / BN, tiles = tilesN * ((M + BM - 1) / BM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int t = (int)(lin % (uint32_t)tiles);
  const int tm = t / tilesN, tn = t % tilesN;
  const size_t bz = lin / (uint32_t)tiles;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row0 = tm * BM, col0 = tn * BN;
  I8_STAMP(0);

  // staging roles: A row ar, AK k from ak0; B k-quad bq (rows 4bq..4bq+3), columns bg*CW..+CW-1
  const int ar = tid / AQ, ak0 = AK * (tid % AQ);
  const int bq = tid % NQ, bg = tid / NQ;
  const int gr = row0 + ar, gc = col0 + bg * CW;
  // B8 (q15): thread (cp, kb8) stages columns 2cp, 2cp + 1 over k-rows 8 kb8 .. 8 kb8 + 7 (eight
  // coalesced dword loads), i.e. 8 k-bytes per column and plane: one ds_write_b64 each (4 per
  // thread instead of v2's 16 ds_write_b32) and half the transposing v_perm work
  constexpr bool B8 = MI355X_I8_B8 && sizeof(T) == 2;
  constexpr int NQB = B8 ? 8 : NQ;               // column-sum partials per column
  const int cp = tid % 64, kb8 = tid / 64;
  const int gcp = col0 + 2 * cp;
  const bool vecA = FULL || (((K * (int)sizeof(T)) % 16) == 0 && (((uintptr_t)A) & 15) == 0);
  const bool vecB = FULL || (((N * (int)sizeof(T)) % (4 * BD)) == 0 && (((uintptr_t)B) & (4 * BD - 1)) == 0);
  const bool vecB8 = FULL || ((N % 2) == 0 && (((uintptr_t)B) & 3) == 0);

  uint32_t ad[AKD], bd[4][BD], b8[8];
  auto load = [&](int k0) {
    const int ka = k0 + ak0;
    if (FULL || (vecA && gr < M && ka + AK <= K)) {
      const uint4* p = reinterpret_cast<const uint4*>(A + (size_t)gr * K + ka);
#pragma unroll
      for (int i = 0; i < AKD / 4; ++i) {
        const uint4 v = p[i];
        ad[4 * i] = v.x; ad[4 * i + 1] = v.y; ad[4 * i + 2] = v.z; ad[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < AKD; ++d) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < EPD; ++e) {
          const int k = ka + d * EPD + e;
          const uint32_t v = (gr < M && k < K) ? (uint32_t)A[(size_t)gr * K + k] : 0u;
          w |= (EPD == 2 ? (v & 0xffffu) : v) << (16 * e);
        }
        ad[d] = w;
      }
    }
    if constexpr (B8) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int kb = k0 + 8 * kb8 + i;
        if (FULL || (vecB8 && kb < K && gcp + 2 <= N)) {
          b8[i] = *reinterpret_cast<const uint32_t*>(B + (size_t)kb * N + gcp);
        } else {
          const uint32_t lo = (kb < K && gcp < N) ? (uint32_t)(uint16_t)B[(size_t)kb * N + gcp] : 0u;
          const uint32_t hi = (kb < K && gcp + 1 < N) ? (uint32_t)(uint16_t)B[(size_t)kb * N + gcp + 1] : 0u;
          b8[i] = lo | (hi << 16);
        }
      }
    } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kb = k0 + 4 * bq + i;
      if (FULL || (vecB && kb < K && gc + CW <= N)) {
        if constexpr (BD == 4) {
          const uint4 v = *reinterpret_cast<const uint4*>(B + (size_t)kb * N + gc);
          bd[i][0] = v.x; bd[i][1] = v.y; bd[i][2] = v.z; bd[i][3] = v.w;
        } else {
          const uint2 v = *reinterpret_cast<const uint2*>(B + (size_t)kb * N + gc);
          bd[i][0] = v.x; bd[i][1] = v.y;
        }
      } else {
#pragma unroll
        for (int d = 0; d < BD; ++d) {
          uint32_t w = 0;
#pragma unroll
          for (int e = 0; e < EPD; ++e) {
            const int c = gc + d * EPD + e;
            const uint32_t v = (kb < K && c < N) ? (uint32_t)B[(size_t)kb * N + c] : 0u;
            w |= (EPD == 2 ? (v & 0xffffu) : v) << (16 * e);
          }
          bd[i][d] = w;
        }
      }
    }
    }
  };

  // this thread's partial row / column sums over the K steps: int32 is exact for q15 (at most
  // 16 x 511 values of |v| <= 2^15 per partial), int64 for q31
  using PS = typename std::conditional<sizeof(T) == 2, int32_t, int64_t>::type;
  PS my_rsum = 0, my_csum[CW];
#pragma unroll
  for (int c = 0; c < CW; ++c) my_csum[c] = 0;
  int32_t bcs[2] = {0, 0};                       // B8: columns 2cp, 2cp + 1 (exact: <= 8 x 511 x 2^15)
  i32x16 acc[S][WBM][WBN];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int i = 0; i < WBM; ++i)
#pragma unroll
      for (int j = 0; j < WBN; ++j) acc[s][i][j] = i32x16{};
  const int wm = wid / kWavesN, wn = wid % kWavesN;
  const int r = lane & 31, h = lane >> 5;

  auto stage = [&](int buf) {
    auto As = reinterpret_cast<int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    auto Bs = reinterpret_cast<int8_t (*)[BN][kPitch2]>(lds + buf * BUF + P * BM * kPitch2);
    // exact row / column sums of the original values
    if constexpr (sizeof(T) == 2) {
      int32_t ra = 0;
#pragma unroll
      for (int d = 0; d < AKD; ++d) ra = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, ad[d]), s2x{1, 1}, ra, false);
      my_rsum += ra;
      if constexpr (B8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          bcs[0] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, b8[i]), s2x{1, 0}, bcs[0], false);
          bcs[1] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, b8[i]), s2x{0, 1}, bcs[1], false);
        }
      } else {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          const s2x sel = (c & 1) ? s2x{0, 1} : s2x{1, 0};
          int32_t cs = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) cs = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, bd[i][c >> 1]), sel, cs, false);
          my_csum[c] += cs;
        }
      }
    } else {
#pragma unroll
      for (int d = 0; d < AKD; ++d) my_rsum += (int32_t)ad[d];
#pragma unroll
      for (int c = 0; c < CW; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) my_csum[c] += (int32_t)bd[i][c];
    }
    // byte planes -> LDS
#pragma unroll
    for (int p = 0; p < P; ++p) {
      uint32_t w[AK / 4];
#pragma unroll
      for (int q = 0; q < AK / 4; ++q) {
        if constexpr (sizeof(T) == 2) w[q] = plane_q15<P>(ad[2 * q], ad[2 * q + 1], p);
        else w[q] = plane4<P>(ad[4 * q], ad[4 * q + 1], ad[4 * q + 2], ad[4 * q + 3], p);
      }
#pragma unroll
      for (int q = 0; q < AK / 16; ++q)
        *reinterpret_cast<uint4*>(&As[p][ar][16 * i8_chunk(ar, ak0 / 16 + q)]) =
            make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
      if constexpr (B8) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int o = 2 * c + p;                // byte of column 2cp + c, plane p, in a dword
          uint32_t g0 = gather4(b8[0], b8[1], b8[2], b8[3], o), g1 = gather4(b8[4], b8[5], b8[6], b8[7], o);
          if (p != P - 1) { g0 ^= 0x80808080u; g1 ^= 0x80808080u; }
          const int row = i8_brow8(2 * cp + c);
          *reinterpret_cast<uint2*>(&Bs[p][row][16 * i8_chunk(row, kb8 >> 1) + 8 * (kb8 & 1)]) = make_uint2(g0, g1);
        }
      } else {
#pragma unroll
        for (int c = 0; c < CW; ++c) {
          const int d = c / EPD, o = (c % EPD) * (int)sizeof(T) + p;
          uint32_t g = gather4(bd[0][d], bd[1][d], bd[2][d], bd[3][d], o);
          if (p != P - 1) g ^= 0x80808080u;
          const int row = i8_brow<CW>(bg * CW + c);
          *reinterpret_cast<uint32_t*>(&Bs[p][row][16 * i8_chunk(row, bq >> 2) + 4 * (bq & 3)]) = g;
        }
      }
    }
  };
  constexpr int KS = kKT2 / 32;                  // MFMA k-steps per K step
  i32x4 fa[KS][P][WBM], fb[KS][P][WBN];
  auto frags = [&](int buf) {
    auto As = reinterpret_cast<const int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    auto Bs = reinterpret_cast<const int8_t (*)[BN][kPitch2]>(lds + buf * BUF + P * BM * kPitch2);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int i = 0; i < WBM; ++i) {
          const int row = wm * 32 * WBM + i * 32 + r;
          fa[kk][p][i] = *reinterpret_cast<const i32x4*>(&As[p][row][16 * i8_chunk(row, 2 * kk + h)]);
        }
#pragma unroll
        for (int j = 0; j < WBN; ++j) {
          const int n = wn * 32 * WBN + j * 32 + r;
          const int row = B8 ? i8_brow8(n) : i8_brow<CW>(n);
          fb[kk][p][j] = *reinterpret_cast<const i32x4*>(&Bs[p][row][16 * i8_chunk(row, 2 * kk + h)]);
        }
      }
  };
  auto mma = [&]() {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int q = 0; q < P; ++q)
#pragma unroll
          for (int i = 0; i < WBM; ++i)
#pragma unroll
            for (int j = 0; j < WBN; ++j)
              acc[p + q][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[kk][p][i], fb[kk][q][j], acc[p + q][i][j], 0, 0, 0);
  };

  // SPLIT: the second MFMA k-step (kk = 1) of K step kt runs at the head of step kt + 1, from
  // registers, while that step's first fragment reads are in flight (the barrier only orders the
  // LDS; register fragments may cross it)
  constexpr bool SPLIT = MI355X_I8_SPLIT && KS == 2;
  i32x4 ga[P][WBM], gb[P][WBN], ha[P][WBM], hb[P][WBN];   // SPLIT: kk = 0 / kk = 1 fragments
  auto frags_kk = [&](int buf, int kk, i32x4 (&FA)[P][WBM], i32x4 (&FB)[P][WBN]) {
    auto As = reinterpret_cast<const int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    auto Bs = reinterpret_cast<const int8_t (*)[BN][kPitch2]>(lds + buf * BUF + P * BM * kPitch2);
#pragma unroll
    for (int p = 0; p < P; ++p) {
#pragma unroll
      for (int i = 0; i < WBM; ++i) {
        const int row = wm * 32 * WBM + i * 32 + r;
        FA[p][i] = *reinterpret_cast<const i32x4*>(&As[p][row][16 * i8_chunk(row, 2 * kk + h)]);
      }
#pragma unroll
      for (int j = 0; j < WBN; ++j) {
        const int n = wn * 32 * WBN + j * 32 + r;
        const int row = B8 ? i8_brow8(n) : i8_brow<CW>(n);
        FB[p][j] = *reinterpret_cast<const i32x4*>(&Bs[p][row][16 * i8_chunk(row, 2 * kk + h)]);
      }
    }
  };
  auto mma_kk = [&](const i32x4 (&FA)[P][WBM], const i32x4 (&FB)[P][WBN]) {
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int i = 0; i < WBM; ++i)
#pragma unroll
          for (int j = 0; j < WBN; ++j)
            acc[p + q][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[p][i], FB[q][j], acc[p + q][i][j], 0, 0, 0);
  };

  // Double-buffered K loop: step kt's fragments are read from buffer kt&1 first, then step
  // kt+1's planes are staged into the other buffer and step kt+2's global loads issued, and
  // the MFMAs (register-only) can interleave with that staging work; one barrier per step.
  const int nk = (K + kKT2 - 1) / kKT2;
  load(0);
  stage(0);
  if (nk > 1) load(kKT2);
  __syncthreads();
  I8_STAMP(1);
  int kt = 0;
  if constexpr (SPLIT) {
    frags_kk(0, 0, ga, gb);                      // step 0: nothing outstanding yet
    frags_kk(0, 1, ha, hb);
    if (nk > 1) stage(1);
    if (nk > 2) load(2 * kKT2);
    mma_kk(ga, gb);
    __syncthreads();
    kt = 1;
    for (; kt + 2 < nk; ++kt) {                  // steady state: one basic block when FULL
      const int cur = kt & 1;
      frags_kk(cur, 0, ga, gb);
      mma_kk(ha, hb);                            // step kt - 1, kk = 1
      frags_kk(cur, 1, ha, hb);
      stage(cur ^ 1);
      load((kt + 2) * kKT2);
      mma_kk(ga, gb);
#if MI355X_I8_SCHED
#pragma unroll
      for (int i = 0; i < 2 * P * P * WBM * WBN; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, MI355X_I8_SCHED, 0);
      }
#endif
      __syncthreads();
    }
    for (; kt < nk; ++kt) {
      const int cur = kt & 1;
      frags_kk(cur, 0, ga, gb);
      mma_kk(ha, hb);
      frags_kk(cur, 1, ha, hb);
      if (kt + 1 < nk) stage(cur ^ 1);
      mma_kk(ga, gb);
      __syncthreads();
    }
    mma_kk(ha, hb);                              // the last step's kk = 1
  }
  for (; !SPLIT && kt + 2 < nk; ++kt) {           // steady state: one basic block when FULL
    const int cur = kt & 1;
    frags(cur);
    stage(cur ^ 1);
    load((kt + 2) * kKT2);
    mma();
#if MI355X_I8_SCHED
#pragma unroll
    for (int i = 0; i < KS * P * P * WBM * WBN; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                 // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, MI355X_I8_SCHED, 0);   // then VALU
    }
#endif
    __syncthreads();
  }
  for (; !SPLIT && kt < nk; ++kt) {
    const int cur = kt & 1;
    frags(cur);
    if (kt + 1 < nk) stage(cur ^ 1);
    mma();
    __syncthreads();
  }
  I8_STAMP(2);

  // ---- epilogue: exact sums through LDS (reusing the plane buffers), int64 combine.  The
  // partial row / column sums are reduced once (one thread per row, one per column), then every
  // output reads its two final sums; whole tiles are staged as T in LDS and leave as 16-B
  // stores, 16 threads per 256-B row (the per-element stores issued one 2- / 4-byte store per
  // output, 32 lanes covering 64 / 128 B).
  int64_t* rs = reinterpret_cast<int64_t*>(lds);            // [AQ][BM] partials
  int64_t* cs = rs + AQ * BM;                               // [NQ][BN]
  int64_t* rfin = cs + NQ * BN;                             // [BM] final row sums
  int64_t* cfin = rfin + BM;                                // [BN] final column sums
  T* ct = reinterpret_cast<T*>(cfin + BN);                  // [BM][BN] output tile (FULL)
  static_assert((AQ * BM + NQ * BN + BM + BN) * 8 + BM * BN * sizeof(T) <= 2 * BUF, "epilogue fits the planes");
  rs[(tid % AQ) * BM + ar] = (int64_t)my_rsum;
  if constexpr (B8) {
    cs[kb8 * BN + 2 * cp] = (int64_t)bcs[0];
    cs[kb8 * BN + 2 * cp + 1] = (int64_t)bcs[1];
  } else {
#pragma unroll
    for (int c = 0; c < CW; ++c) cs[bq * BN + bg * CW + c] = (int64_t)my_csum[c];
  }
  __syncthreads();
  for (int i = tid; i < BM + BN; i += kNT2) {
    int64_t sum = 0;
    if (i < BM) {
#pragma unroll
      for (int q = 0; q < AQ; ++q) sum += rs[q * BM + i];
      rfin[i] = sum;
    } else {
#pragma unroll
      for (int q = 0; q < NQB; ++q) sum += cs[q * BN + (i - BM)];
      cfin[i - BM] = sum;
    }
  }
  __syncthreads();
  const int64_t kpad = (int64_t)nk * kKT2;   // padded k terms are zeros: the identity holds over kpad
#pragma unroll
  for (int j = 0; j < WBN; ++j) {
    const int cc = wn * 32 * WBN + j * 32 + r;
    const int64_t csum = cfin[cc];
    const int gcol = col0 + cc;
#pragma unroll
    for (int i = 0; i < WBM; ++i) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rr = wm * 32 * WBM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int grow = row0 + rr;
        uint64_t v = (uint64_t)(C0 * (rfin[rr] + csum)) - (uint64_t)kpad * (uint64_t)(C0 * C0);
#pragma unroll
        for (int s = 0; s < S; ++s) v += (uint64_t)(int64_t)acc[s][i][j][reg] << (8 * s);
        const int64_t sum = (int64_t)v;
        // fast q15 (arm_mat_mult_fast_q15.c:356-401 host branch): q31_t modular sum, (q15)(sum >> 15)
        T o;
        if constexpr (sizeof(T) == 2) o = fast ? (T)((int32_t)(uint32_t)v >> 15) : (T)ssat16((int32_t)(sum >> 15));
        else o = (T)(int32_t)(sum >> 31);
        if constexpr (FULL) ct[rr * BN + cc] = o;
        else if (grow < M && gcol < N) C[(size_t)grow * N + gcol] = o;
      }
    }
  }
  I8_STAMP(3);
  if constexpr (FULL) {
    __syncthreads();
    constexpr int VPR = BN * (int)sizeof(T) / 16;            // 16-B words per tile row
    static_assert(VPR * 16 == BN * (int)sizeof(T), "whole 16-B words per row");
#pragma unroll
    for (int w = tid; w < BM * VPR; w += kNT2) {
      const int rr = w / VPR, cw = w % VPR;
      *reinterpret_cast<uint4*>(C + (size_t)(row0 + rr) * N + col0 + cw * (16 / (int)sizeof(T))) =
          *reinterpret_cast<const uint4*>(ct + rr * BN + cw * (16 / (int)sizeof(T)));
    }
  }
  I8_STAMP(4);
}

// ---- v3 kernel (round 4): the v2 tiling with B staged ROW-major.  B's
// planes are stored as [k][n] byte rows (the global layout) and the MFMA's k-contiguous
// operand is read with ds_read_b64_tr_b8 (gfx950's 8-bit transposed LDS read: per 16-lane group
// an 8-row x 16-column byte block, lane i receiving column i, row q in byte q;
// tools/probes/tr_b8.hip), so the v_perm transpose of v2's staging disappears: a thread stages
// one k-row segment of B (32 bytes) with two 16-B loads and splits it into planes with one
// v_perm per 4 values.  Column sums accumulate per thread over the k-rows it stages (its
// columns are fixed for the whole K loop).  Selected by MI355X_I8_V3.
template <typename T> struct I8B3 {               // B staging geometry
  static constexpr int BN = I8Cfg<T>::BN, EB = 64 * BN / kNT2;   // elements per thread (16 q15 / 8 q31)
  static constexpr int TPR = BN / EB;                            // threads per k-row (8)
  // bytes per plane row: a multiple of 32 that is an odd multiple of 8 dwords mod 64, so the
  // 8 rows x 8 dwords a 32-lane group of ds_read_b64_tr_b8 touches cover the 64 banks once
  // (MI355X_I8_V3P overrides; BN + 16 measured 8x the v2 conflicts)
#ifdef MI355X_I8_V3P
  static constexpr int PITCH = MI355X_I8_V3P;
#else
  static constexpr int PITCH = BN == 128 ? 160 : 96;
#endif
};
typedef int v2i32_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2i32_t tr_b8(const int8_t* p) {   // p: a generic pointer into LDS
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i32_t*)p);
}

template <typename T, bool FULL>
__global__ __launch_bounds__(kNT2) void mat_mult_i8v3_kernel(const T* __restrict__ A, const T* __restrict__ B,
                                                             T* __restrict__ C, int M, int K, int N, int fast) {
  using G = I8Cfg<T>;
  using GB = I8B3<T>;
  constexpr int P = Slices<T>::P, S = 2 * P - 1;
  constexpr int64_t C0 = Slices<T>::C0;
  constexpr int BM = G::BM, BN = G::BN, WBM = G::WBM, WBN = G::WBN, kKT2 = G::KT, kPitch2 = kKT2;
  constexpr int EPD = 4 / sizeof(T);
  constexpr int AK = BM * kKT2 / kNT2, AKD = AK / EPD, AQ = kKT2 / AK;
  constexpr int EB = GB::EB, EBD = EB / EPD, TPR = GB::TPR, BP = GB::PITCH;
  constexpr int ABUF = P * BM * kPitch2, BBUF = P * kKT2 * BP;
  constexpr int BUF = ABUF + BBUF;
  // the epilogue reuses the plane buffers: partial sums (one column partial per staged k-row),
  // final sums and the output tile
  constexpr int EPI = (AQ * BM + kKT2 * BN + BM + BN) * 8 + BM * BN * (int)sizeof(T);
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * BUF > EPI ? 2 * BUF : EPI];

  const int tilesN = (N + BN - 1) / BN, tiles = tilesN * ((M + BM - 1) / BM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int t = (int)(lin % (uint32_t)tiles);
  const int tm = t / tilesN, tn = t % tilesN;
  const size_t bz = lin / (uint32_t)tiles;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int row0 = tm * BM, col0 = tn * BN;

  // staging roles: A row ar, AK k from ak0 (as v2); B k-row bk, columns bc .. bc + EB - 1
  const int ar = tid / AQ, ak0 = AK * (tid % AQ);
  const int bk = tid / TPR, bc = EB * (tid % TPR);
  const int gr = row0 + ar, gc = col0 + bc;
  const bool vecA = FULL || (((K * (int)sizeof(T)) % 16) == 0 && (((uintptr_t)A) & 15) == 0);
  const bool vecB = FULL || (((N * (int)sizeof(T)) % 16) == 0 && (((uintptr_t)B) & 15) == 0);

  uint32_t ad[AKD], bd[EBD];
  auto load = [&](int k0) {
    const int ka = k0 + ak0;
    if (FULL || (vecA && gr < M && ka + AK <= K)) {
      const uint4* p = reinterpret_cast<const uint4*>(A + (size_t)gr * K + ka);
#pragma unroll
      for (int i = 0; i < AKD / 4; ++i) {
        const uint4 v = p[i];
        ad[4 * i] = v.x; ad[4 * i + 1] = v.y; ad[4 * i + 2] = v.z; ad[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < AKD; ++d) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < EPD; ++e) {
          const int k = ka + d * EPD + e;
          const uint32_t v = (gr < M && k < K) ? (uint32_t)A[(size_t)gr * K + k] : 0u;
          w |= (EPD == 2 ? (v & 0xffffu) : v) << (16 * e);
        }
        ad[d] = w;
      }
    }
    const int kb = k0 + bk;
    if (FULL || (vecB && kb < K && gc + EB <= N)) {
      const uint4* p = reinterpret_cast<const uint4*>(B + (size_t)kb * N + gc);
#pragma unroll
      for (int i = 0; i < EBD / 4; ++i) {
        const uint4 v = p[i];
        bd[4 * i] = v.x; bd[4 * i + 1] = v.y; bd[4 * i + 2] = v.z; bd[4 * i + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int d = 0; d < EBD; ++d) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < EPD; ++e) {
          const int c = gc + d * EPD + e;
          const uint32_t v = (kb < K && c < N) ? (uint32_t)B[(size_t)kb * N + c] : 0u;
          w |= (EPD == 2 ? (v & 0xffffu) : v) << (16 * e);
        }
        bd[d] = w;
      }
    }
  };

  int64_t my_rsum = 0;
  // column sums of the k-rows this thread stages (at most K / 64 <= 511 of them): exact in int32
  // for q15 (|v| <= 2^15), int64 for q31
  using CS = typename std::conditional<sizeof(T) == 2, int32_t, int64_t>::type;
  CS my_csum[EB];
#pragma unroll
  for (int c = 0; c < EB; ++c) my_csum[c] = 0;
  i32x16 acc[S][WBM][WBN];
#pragma unroll
  for (int s2 = 0; s2 < S; ++s2)
#pragma unroll
    for (int i = 0; i < WBM; ++i)
#pragma unroll
      for (int j = 0; j < WBN; ++j) acc[s2][i][j] = i32x16{};
  const int wm = wid / kWavesN, wn = wid % kWavesN;
  const int r = lane & 31, h = lane >> 5;

  auto stage = [&](int buf) {
    auto As = reinterpret_cast<int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    int8_t* Bs = lds + buf * BUF + ABUF;           // [P][kKT2][BP]
    if constexpr (sizeof(T) == 2) {
      int32_t ra = 0;
#pragma unroll
      for (int d = 0; d < AKD; ++d) ra = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, ad[d]), s2x{1, 1}, ra, false);
      my_rsum += ra;
#pragma unroll
      for (int d = 0; d < EBD; ++d) {
        my_csum[2 * d] += (int16_t)(bd[d] & 0xffffu);
        my_csum[2 * d + 1] += (int16_t)(bd[d] >> 16);
      }
    } else {
#pragma unroll
      for (int d = 0; d < AKD; ++d) my_rsum += (int32_t)ad[d];
#pragma unroll
      for (int d = 0; d < EBD; ++d) my_csum[d] += (int32_t)bd[d];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      uint32_t w[AK / 4];
#pragma unroll
      for (int q = 0; q < AK / 4; ++q) {
        if constexpr (sizeof(T) == 2) w[q] = plane_q15<P>(ad[2 * q], ad[2 * q + 1], p);
        else w[q] = plane4<P>(ad[4 * q], ad[4 * q + 1], ad[4 * q + 2], ad[4 * q + 3], p);
      }
#pragma unroll
      for (int q = 0; q < AK / 16; ++q)
        *reinterpret_cast<uint4*>(&As[p][ar][16 * i8_chunk(ar, ak0 / 16 + q)]) =
            make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
      // B: plane p of this thread's EB values, EB contiguous bytes of plane row bk
      uint32_t wb[EB / 4];
#pragma unroll
      for (int q = 0; q < EB / 4; ++q) {
        if constexpr (sizeof(T) == 2) wb[q] = plane_q15<P>(bd[2 * q], bd[2 * q + 1], p);
        else wb[q] = plane4<P>(bd[4 * q], bd[4 * q + 1], bd[4 * q + 2], bd[4 * q + 3], p);
      }
      int8_t* dstb = Bs + (size_t)p * kKT2 * BP + bk * BP + bc;
      if constexpr (EB == 16) *reinterpret_cast<uint4*>(dstb) = make_uint4(wb[0], wb[1], wb[2], wb[3]);
      else *reinterpret_cast<uint2*>(dstb) = make_uint2(wb[0], wb[1]);
    }
  };
  constexpr int KS = kKT2 / 32;
  i32x4 fa[KS][P][WBM], fb[KS][P][WBN];
  // B fragment of column block j, k-step kk: lane l of 16-lane group g = l >> 4 supplies row
  // 16 h + 8 rr + (li >> 1), columns 16 (g & 1) + 8 (li & 1) of the block (li = l & 15), for the
  // two 8-row reads rr = 0, 1 (k bytes 16h .. 16h + 7 and 16h + 8 .. 16h + 15 of its column)
  const int li = lane & 15, gq = (lane >> 4) & 1;
  auto frags = [&](int buf) {
    auto As = reinterpret_cast<const int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    const int8_t* Bs = lds + buf * BUF + ABUF;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int i = 0; i < WBM; ++i) {
          const int row = wm * 32 * WBM + i * 32 + r;
          fa[kk][p][i] = *reinterpret_cast<const i32x4*>(&As[p][row][16 * i8_chunk(row, 2 * kk + h)]);
        }
#pragma unroll
        for (int j = 0; j < WBN; ++j) {
          const int col = wn * 32 * WBN + j * 32 + 16 * gq + 8 * (li & 1);
          const int8_t* b0 = Bs + (size_t)p * kKT2 * BP + (32 * kk + 16 * h + (li >> 1)) * BP + col;
          const v2i32_t lo = tr_b8(b0), hi = tr_b8(b0 + 8 * BP);
          fb[kk][p][j] = i32x4{lo.x, lo.y, hi.x, hi.y};
        }
      }
  };
  auto mma = [&]() {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int q = 0; q < P; ++q)
#pragma unroll
          for (int i = 0; i < WBM; ++i)
#pragma unroll
            for (int j = 0; j < WBN; ++j)
              acc[p + q][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[kk][p][i], fb[kk][q][j], acc[p + q][i][j], 0, 0, 0);
  };

  // as v2 (kk = 1 MFMAs under the next step's reads) for q15 only: with q31's four planes the two
  // fragment sets spill
  constexpr bool SPLIT = MI355X_I8_SPLIT && KS == 2 && sizeof(T) == 2;
  i32x4 ga[P][WBM], gb[P][WBN], ha[P][WBM], hb[P][WBN];
  auto frags_kk = [&](int buf, int kk, i32x4 (&FA)[P][WBM], i32x4 (&FB)[P][WBN]) {
    auto As = reinterpret_cast<const int8_t (*)[BM][kPitch2]>(lds + buf * BUF);
    const int8_t* Bs = lds + buf * BUF + ABUF;
#pragma unroll
    for (int p = 0; p < P; ++p) {
#pragma unroll
      for (int i = 0; i < WBM; ++i) {
        const int row = wm * 32 * WBM + i * 32 + r;
        FA[p][i] = *reinterpret_cast<const i32x4*>(&As[p][row][16 * i8_chunk(row, 2 * kk + h)]);
      }
#pragma unroll
      for (int j = 0; j < WBN; ++j) {
        const int col = wn * 32 * WBN + j * 32 + 16 * gq + 8 * (li & 1);
        const int8_t* b0 = Bs + (size_t)p * kKT2 * BP + (32 * kk + 16 * h + (li >> 1)) * BP + col;
        const v2i32_t lo = tr_b8(b0), hi = tr_b8(b0 + 8 * BP);
        FB[p][j] = i32x4{lo.x, lo.y, hi.x, hi.y};
      }
    }
  };
  auto mma_kk = [&](const i32x4 (&FA)[P][WBM], const i32x4 (&FB)[P][WBN]) {
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int q = 0; q < P; ++q)
#pragma unroll
        for (int i = 0; i < WBM; ++i)
#pragma unroll
          for (int j = 0; j < WBN; ++j)
            acc[p + q][i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[p][i], FB[q][j], acc[p + q][i][j], 0, 0, 0);
  };

  const int nk = (K + kKT2 - 1) / kKT2;
  load(0);
  stage(0);
  if (nk > 1) load(kKT2);
  __syncthreads();
  int kt = 0;
  if constexpr (SPLIT) {
    frags_kk(0, 0, ga, gb);
    frags_kk(0, 1, ha, hb);
    if (nk > 1) stage(1);
    if (nk > 2) load(2 * kKT2);
    mma_kk(ga, gb);
    __syncthreads();
    kt = 1;
    for (; kt + 2 < nk; ++kt) {
      const int cur = kt & 1;
      frags_kk(cur, 0, ga, gb);
      mma_kk(ha, hb);
      frags_kk(cur, 1, ha, hb);
      stage(cur ^ 1);
      load((kt + 2) * kKT2);
      mma_kk(ga, gb);
#if MI355X_I8_SCHED_V3
#pragma unroll
      for (int i = 0; i < 2 * P * P * WBM * WBN; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, MI355X_I8_SCHED_V3, 0);
      }
#endif
      __syncthreads();
    }
    for (; kt < nk; ++kt) {
      const int cur = kt & 1;
      frags_kk(cur, 0, ga, gb);
      mma_kk(ha, hb);
      frags_kk(cur, 1, ha, hb);
      if (kt + 1 < nk) stage(cur ^ 1);
      mma_kk(ga, gb);
      __syncthreads();
    }
    mma_kk(ha, hb);
  }
  for (; !SPLIT && kt + 2 < nk; ++kt) {
    const int cur = kt & 1;
    frags(cur);
    stage(cur ^ 1);
    load((kt + 2) * kKT2);
    mma();
#if MI355X_I8_SCHED_V3
#pragma unroll
    for (int i = 0; i < KS * P * P * WBM * WBN; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                 // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, MI355X_I8_SCHED_V3, 0);   // then VALU
    }
#endif
    __syncthreads();
  }
  for (; !SPLIT && kt < nk; ++kt) {
    const int cur = kt & 1;
    frags(cur);
    if (kt + 1 < nk) stage(cur ^ 1);
    mma();
    __syncthreads();
  }

  // ---- epilogue (as v2): partial sums reduced once, the output tile staged in LDS, 16-B stores
  constexpr int NQB = kKT2;                                 // one column partial per staged k-row
  int64_t* rs = reinterpret_cast<int64_t*>(lds);            // [AQ][BM]
  int64_t* cs = rs + AQ * BM;                               // [64 k-rows][BN]
  int64_t* rfin = cs + NQB * BN;
  int64_t* cfin = rfin + BM;
  T* ct = reinterpret_cast<T*>(cfin + BN);
  rs[(tid % AQ) * BM + ar] = my_rsum;
#pragma unroll
  for (int c = 0; c < EB; ++c) cs[bk * BN + bc + c] = (int64_t)my_csum[c];
  __syncthreads();
  for (int i = tid; i < BM + BN; i += kNT2) {
    int64_t sum = 0;
    if (i < BM) {
#pragma unroll
      for (int q = 0; q < AQ; ++q) sum += rs[q * BM + i];
      rfin[i] = sum;
    } else {
      for (int q = 0; q < NQB; ++q) sum += cs[q * BN + (i - BM)];
      cfin[i - BM] = sum;
    }
  }
  __syncthreads();
  const int64_t kpad = (int64_t)nk * kKT2;
#pragma unroll
  for (int j = 0; j < WBN; ++j) {
    const int cc = wn * 32 * WBN + j * 32 + r;
    const int64_t csum = cfin[cc];
    const int gcol = col0 + cc;
#pragma unroll
    for (int i = 0; i < WBM; ++i) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rr = wm * 32 * WBM + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const int grow = row0 + rr;
        uint64_t v = (uint64_t)(C0 * (rfin[rr] + csum)) - (uint64_t)kpad * (uint64_t)(C0 * C0);
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) v += (uint64_t)(int64_t)acc[s2][i][j][reg] << (8 * s2);
        const int64_t sum = (int64_t)v;
        T o;
        if constexpr (sizeof(T) == 2) o = fast ? (T)((int32_t)(uint32_t)v >> 15) : (T)ssat16((int32_t)(sum >> 15));
        else o = (T)(int32_t)(sum >> 31);
        if constexpr (FULL) ct[rr * BN + cc] = o;
        else if (grow < M && gcol < N) C[(size_t)grow * N + gcol] = o;
      }
    }
  }
  if constexpr (FULL) {
    __syncthreads();
    constexpr int VPR = BN * (int)sizeof(T) / 16;
#pragma unroll
    for (int w = tid; w < BM * VPR; w += kNT2) {
      const int rr = w / VPR, cw = w % VPR;
      *reinterpret_cast<uint4*>(C + (size_t)(row0 + rr) * N + col0 + cw * (16 / (int)sizeof(T))) =
          *reinterpret_cast<const uint4*>(ct + rr * BN + cw * (16 / (int)sizeof(T)));
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
  if (k <= kMatI8MaxK) {
    using G = I8Cfg<T>;
    const int tiles = ((m + G::BM - 1) / G::BM) * ((n + G::BN - 1) / G::BN);
    const bool full = m % G::BM == 0 && n % G::BN == 0 && k % G::KT == 0 &&
                      ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0 && (k * sizeof(T)) % 16 == 0 &&
                      (n * sizeof(T)) % 16 == 0 && ((uintptr_t)c & 15) == 0;
    if (MI355X_I8_V3 == 1 || (MI355X_I8_V3 == 2 && sizeof(T) == 4)) {   // 2: q31 only
      if (full)
        hipLaunchKernelGGL((mat_mult_i8v3_kernel<T, true>), dim3(tiles * batch), dim3(kNT2), 0, st, a, b, c, m, k, n,
                           fast);
      else
        hipLaunchKernelGGL((mat_mult_i8v3_kernel<T, false>), dim3(tiles * batch), dim3(kNT2), 0, st, a, b, c, m, k,
                           n, fast);
    } else if (full)
      hipLaunchKernelGGL((mat_mult_i8v2_kernel<T, true>), dim3(tiles * batch), dim3(kNT2), 0, st, a, b, c, m, k, n,
                         fast);
    else
      hipLaunchKernelGGL((mat_mult_i8v2_kernel<T, false>), dim3(tiles * batch), dim3(kNT2), 0, st, a, b, c, m, k, n,
                         fast);
  } else {
    hipLaunchKernelGGL(mat_mult_fixed_valu_kernel<T>, dim3((n + 255) / 256, m, batch), dim3(256), 0, st, a, b, c,
                       m, k, n, fast);
  }
  return hipGetLastError();
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

#if MI355X_I8_STAMPS
extern "C" int arm_mi355x_i8_stamps(uint64_t* out, size_t rows) {   // diagnostic builds only
  const size_t n = rows < (size_t)kI8Stamps ? rows : (size_t)kI8Stamps;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_i8_stamps), n * 8 * sizeof(uint64_t), 0, hipMemcpyDeviceToHost);
}
#endif

}  // namespace mi355x
