// Batched q7 matrix multiply on ONE i8 matrix-core plane — MI355X, bit-exact.
//
// Replaces the host scalar path of Source/MatrixFunctions/arm_mat_mult_q7.c:689-790 (the
// non-Helium, non-Neon branch): sum = sum_k (q31)a[i][k] * b[k][j] in q31_t, then
// (q7)__SSAT(sum >> 7, 8).  With uint16_t dimensions |sum| <= 65535 * 2^14 < 2^30, so the sum
// never wraps and an int32 accumulation of exact products in ANY order is the reference's value:
// the whole product is one v_mfma_i32_32x32x32_i8 GEMM with no byte planes, offsets or row /
// column corrections (the q15 / q31 kernels of mat_mult_fixed.hip need P^2 plane products).
//
// Tiling (1024^3 per matrix is balanced between HBM (3 MiB per GEMM) and the i8 MFMA rate, so
// the tile is sized for L2 traffic): 256 x 256 workgroup tiles of 8 waves (2 x 4), wave tiles of
// 128 x 64 (4 x 2 blocks of 32 x 32, 128 accumulator registers, two waves per SIMD), 64-deep K
// steps in a double-buffered LDS image, one barrier per step, step kt + 2's global loads in
// flight under step kt's MFMAs.  Per K step a workgroup moves 32 KiB from L2 for 4.2 M MACs.
//  * A stays row-major in LDS (rows of 64 k-bytes, chunk c of row r at c ^ ((r >> 2) & 3)): the
//    MFMA's A operand (16 k-consecutive bytes of one row per lane) is one ds_read_b128;
//  * B stays row-major too ([k][n] rows of 256 bytes, pitch 288), and the operand (16
//    k-consecutive bytes of one column) is read with two ds_read_b64_tr_b8 (gfx950's transposing
//    LDS read, tools/probes/tr_b8.hip) -- no VALU transpose anywhere in the K loop;
//  * staging is register pass-through: 2 + 2 global 16-B loads and 2 + 2 ds_write_b128 per
//    thread and K step (A: 4 threads per 64-B row; B: 16 threads per 256-B row, so every 8-lane
//    write group covers 32 distinct banks).
// The accumulators are C^T blocks (operands swapped in the MFMA), so the epilogue packs four
// saturated (acc >> 7) bytes per dword into the LDS output tile and writes it as 16-B rows.  Ragged shapes take the guarded instance (zero-filled loads: a zero term adds
// nothing, there is no offset algebra to keep).
#include "common.hpp"
#include "kernels.hpp"

#ifndef MI355X_Q7_SCHED     // pinned fragment-read / MFMA / staging order in the steady K step
#define MI355X_Q7_SCHED 1
#endif
#ifndef MI355X_Q7_KT        // K bytes per LDS step: 64 or 128
#define MI355X_Q7_KT 64
#endif
#ifndef MI355X_Q7_BN        // tile columns: 256 (8 waves, one workgroup per CU) or 128 (4 waves, two per CU)
#define MI355X_Q7_BN 256
#endif

namespace mi355x {

namespace {
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int v2i32 __attribute__((ext_vector_type(2)));

constexpr int kQ7BM = 256, kQ7BN = MI355X_Q7_BN, kQ7KT = MI355X_Q7_KT, kQ7NT = 2 * kQ7BN;
static_assert(kQ7BN == 256 || kQ7BN == 128, "tile columns 256 or 128");
static_assert(kQ7KT == 64 || kQ7KT == 128, "K step of 64 or 128 bytes");
constexpr int kQ7KC = kQ7KT / 16;                     // 16-B chunks per A row
constexpr int kQ7KS = kQ7KT / 32;                     // MFMA k-steps per K step
constexpr int kQ7NA = kQ7BM * kQ7KC / kQ7NT;          // A chunks staged per thread (2 | 4)
constexpr int kQ7NB = kQ7KT * (kQ7BN / 16) / kQ7NT;   // B chunks staged per thread (2 | 4)
constexpr int kQ7WM = 2, kQ7WN = kQ7BN / 64;         // wave grid (wave tiles of 128 x 64)
constexpr int kQ7BTR = kQ7BN / 16;                    // staging threads per B row
constexpr int kQ7WBM = kQ7BM / (32 * kQ7WM);          // 4 row blocks of 32 per wave
constexpr int kQ7WBN = kQ7BN / (32 * kQ7WN);          // 2 column blocks of 32 per wave
constexpr int kQ7BP = kQ7BN + 32;                     // B row pitch: 72 dwords = 8 x odd mod 64
constexpr int kQ7ABUF = kQ7BM * kQ7KT, kQ7BBUF = kQ7KT * kQ7BP, kQ7BUF = kQ7ABUF + kQ7BBUF;

// A row swizzle: chunk c of row r at c ^ f(r).  64-B rows: f = r >> 2 (mod 4); 128-B rows (two
// per 64-bank line): f = r >> 1 (mod 8).  Either way every 16-lane group of the fragments'
// ds_read_b128 covers the 64 banks once and every 8-lane group of the staging ds_write_b128 the
// 32 banks once.
__device__ __forceinline__ int q7_chunk(int row, int c) {
  return kQ7KC == 4 ? ((c ^ (row >> 2)) & 3) : ((c ^ (row >> 1)) & 7);
}
__device__ __forceinline__ v2i32 q7_tr8(const int8_t* p) {   // p: generic pointer into LDS
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i32*)p);
}
}  // namespace

// ---- epilogue: (q7)__SSAT(sum >> 7, 8) into an LDS output tile, then 16-B row stores.  The
// accumulator blocks are C^T (the K loop passes B's fragment as the MFMA's A operand): lane l,
// register g holds row l & 31, column (g & 3) + 8 (g >> 2) + 4 h.  The caller has passed a barrier
// after its last LDS read.
template <bool FULL>
__device__ __forceinline__ void q7_epilogue(const i32x16 (&acc)[kQ7WBM][kQ7WBN], int8_t* lds, int8_t* __restrict__ C,
                                            int M, int N, int row0, int col0, int wm, int wn, bool vecB) {
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  int8_t* ct = lds;
  // Transposed accumulators (the K loop swaps the MFMA operands): lane l holds output row l & 31
  // of a block and, in registers 4q .. 4q + 3, the four consecutive columns 8q + 4h .. + 3, so the
  // saturated bytes pack into one dword per 4 outputs -- 32 ds_write_b32 per lane instead of 128
  // byte stores.  Rows sit 264 B apart (66 dwords: the 32 rows of a store group fall on 16 banks,
  // 2-way, which costs nothing for ds_write_b32) and are read back as 8-B pieces.
  constexpr int CPT = kQ7BN + 8;
  static_assert(kQ7BM * CPT <= 2 * kQ7BUF, "the output tile fits the plane buffers");
#pragma unroll
  for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
    for (int j = 0; j < kQ7WBN; ++j) {
      const int rr = wm * 32 * kQ7WBM + 32 * i + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cc = wn * 32 * kQ7WBN + 32 * j + 8 * q + 4 * h;
        const uint32_t w = (uint32_t)(uint8_t)ssat8(acc[i][j][4 * q] >> 7) |
                           (uint32_t)(uint8_t)ssat8(acc[i][j][4 * q + 1] >> 7) << 8 |
                           (uint32_t)(uint8_t)ssat8(acc[i][j][4 * q + 2] >> 7) << 16 |
                           (uint32_t)(uint8_t)ssat8(acc[i][j][4 * q + 3] >> 7) << 24;
        *reinterpret_cast<uint32_t*>(ct + rr * CPT + cc) = w;
      }
    }
  __syncthreads();
  constexpr int VPRT = kQ7BN / 16;
  for (int w = tid; w < kQ7BM * VPRT; w += kQ7NT) {
    const int rr = w / VPRT, cw = 16 * (w % VPRT);
    const int grow = row0 + rr, gcol = col0 + cw;
    const uint2 lo = *reinterpret_cast<const uint2*>(ct + rr * CPT + cw);
    const uint2 hi = *reinterpret_cast<const uint2*>(ct + rr * CPT + cw + 8);
    const uint4 v = make_uint4(lo.x, lo.y, hi.x, hi.y);
    if (FULL) {
      *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = v;
    } else if (grow < M) {
      const int8_t* vb = ct + rr * CPT + cw;
      if (vecB && (((uintptr_t)C) & 15) == 0 && gcol + 16 <= N)
        *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = v;
      else
        for (int e = 0; e < 16 && gcol + e < N; ++e) C[(size_t)grow * N + gcol + e] = vb[e];
    }
  }
}

template <bool FULL>
__global__ __launch_bounds__(kQ7NT, kQ7BN == 128 ? 2 : 1) void mat_mult_q7_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                            int8_t* __restrict__ C, int M, int K, int N) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2 * kQ7BUF];

  // XCD-aware order (as mat_mult_fixed.hip): each XCD takes a contiguous run of (matrix, tile)
  // pairs, so the tiles of one matrix share its A row bands and B column bands in one L2
  const int tilesN = (N + kQ7BN - 1) / kQ7BN, tiles = tilesN * ((M + kQ7BM - 1) / kQ7BM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int t = (int)(lin % (uint32_t)tiles);
  const int row0 = (t / tilesN) * kQ7BM, col0 = (t % tilesN) * kQ7BN;
  const size_t bz = lin / (uint32_t)tiles;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // staging roles: A rows ar + (NT / KC) q, 16-B chunk ac; B k-rows bk + 32 q, 16 columns at bc
  const int ar = tid / kQ7KC, ac = tid % kQ7KC;
  const int bk = tid / kQ7BTR, bc = 16 * (tid % kQ7BTR);
  constexpr int kBRs = kQ7NT / kQ7BTR;                 // B k-rows per staging pass
  constexpr int kARs = kQ7NT / kQ7KC;                  // A rows per staging pass
  const bool vecA = FULL || ((K % 16) == 0 && (((uintptr_t)A) & 15) == 0);
  const bool vecB = FULL || ((N % 16) == 0 && (((uintptr_t)B) & 15) == 0);

  uint4 ra[kQ7NA], rb[kQ7NB];
  auto load16 = [&](const int8_t* base, size_t rowoff, int colg, int collim, bool rowok, bool vec) -> uint4 {
    if (FULL || (vec && rowok && colg + 16 <= collim)) return *reinterpret_cast<const uint4*>(base + rowoff + colg);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (rowok)
      for (int e = 0; e < 16; ++e)
        if (colg + e < collim) w[e >> 2] |= (uint32_t)(uint8_t)base[rowoff + colg + e] << (8 * (e & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < kQ7NA; ++q) {
      const int r = row0 + ar + kARs * q;
      ra[q] = load16(A, (size_t)r * K, k0 + 16 * ac, K, r < M, vecA);
    }
#pragma unroll
    for (int q = 0; q < kQ7NB; ++q) {
      const int kb = k0 + bk + kBRs * q;
      rb[q] = load16(B, (size_t)kb * N, col0 + bc, N, kb < K, vecB);
    }
  };
  auto stage = [&](int buf) {
    int8_t* As = lds + buf * kQ7BUF;
    int8_t* Bs = As + kQ7ABUF;
#pragma unroll
    for (int q = 0; q < kQ7NA; ++q) {
      const int r = ar + kARs * q;
      *reinterpret_cast<uint4*>(As + r * kQ7KT + 16 * q7_chunk(r, ac)) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < kQ7NB; ++q) *reinterpret_cast<uint4*>(Bs + (bk + kBRs * q) * kQ7BP + bc) = rb[q];
  };

  i32x16 acc[kQ7WBM][kQ7WBN];
#pragma unroll
  for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
    for (int j = 0; j < kQ7WBN; ++j) acc[i][j] = i32x16{};
  const int wm = wid / kQ7WN, wn = wid % kQ7WN;
  const int r = lane & 31, h = lane >> 5, li = lane & 15, gq = (lane >> 4) & 1;

  // fragments: A block i -> row wm*128 + 32 i + r, k-bytes 32 kk + 16 h .. +15 (one ds_read_b128);
  // B block j -> column of lane l inside the block, the same 16 k-bytes (two 8-row tr_b8 reads:
  // lane li of a 16-lane group supplies row li >> 1, columns 8 (li & 1) .. +7 of its 8 x 16 block)
  i32x4 fa[2][kQ7WBM], fb[2][kQ7WBN];
  auto frags = [&](int buf, int pair) {           // MFMA k-steps 2 pair, 2 pair + 1
    const int8_t* As = lds + buf * kQ7BUF;
    const int8_t* Bs = As + kQ7ABUF;
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      const int kk = 2 * pair + kq;
#pragma unroll
      for (int i = 0; i < kQ7WBM; ++i) {
        const int row = wm * 32 * kQ7WBM + 32 * i + r;
        fa[kq][i] = *reinterpret_cast<const i32x4*>(As + row * kQ7KT + 16 * q7_chunk(row, 2 * kk + h));
      }
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j) {
        const int col = wn * 32 * kQ7WBN + 32 * j + 16 * gq + 8 * (li & 1);
        const int8_t* b0 = Bs + (32 * kk + 16 * h + (li >> 1)) * kQ7BP + col;
        const v2i32 lo = q7_tr8(b0), hi = q7_tr8(b0 + 8 * kQ7BP);
        fb[kq][j] = i32x4{lo.x, lo.y, hi.x, hi.y};
      }
    }
  };
  auto mma = [&]() {
#pragma unroll
    for (int kq = 0; kq < 2; ++kq)
#pragma unroll
      for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
        for (int j = 0; j < kQ7WBN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb[kq][j], fa[kq][i], acc[i][j], 0, 0, 0);   // C^T blocks
  };
  // MI355X_Q7_SCHED: pin the steady-state order -- every fragment read of kk = 0 first, then the
  // 16 MFMAs with kk = 1's reads, the next step's LDS writes and global loads threaded between
  // them (one per MFMA), so LDS latency hides under the matrix core instead of being waited out
  // two MFMAs at a time (what the default schedule does to save registers).
  auto pin_schedule = [&]() {
#if MI355X_Q7_SCHED
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);          // kk = 0 fragment reads
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);        // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);        // one kk = 1 fragment read
    }
    if constexpr (kQ7NA + kQ7NB == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);      // one staging LDS write
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);      // one global load
      }
    } else {                                                    // BN = 128: 6 writes, 6 loads
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i < kQ7NA + kQ7NB) {
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
      }
    }
#endif
  };

  const int nk = (K + kQ7KT - 1) / kQ7KT;
  load(0);
  stage(0);
  if (nk > 1) load(kQ7KT);
  __syncthreads();
  int kt = 0;
  for (; kt + 2 < nk; ++kt) {                   // steady state: one basic block when FULL
    const int cur = kt & 1;
    frags(cur, 0);
    stage(cur ^ 1);
    load((kt + 2) * kQ7KT);
    mma();
    pin_schedule();
#pragma unroll
    for (int pr = 1; pr < kQ7KS / 2; ++pr) {
      frags(cur, pr);
      mma();
    }
    __syncthreads();
  }
  for (; kt < nk; ++kt) {
    const int cur = kt & 1;
    frags(cur, 0);
    if (kt + 1 < nk) stage(cur ^ 1);
    mma();
#pragma unroll
    for (int pr = 1; pr < kQ7KS / 2; ++pr) {
      frags(cur, pr);
      mma();
    }
    __syncthreads();
  }

  q7_epilogue<FULL>(acc, lds, C, M, N, row0, col0, wm, wn, vecB);
}

hipError_t mat_mult_q7_launch(int m, int k, int n, const int8_t* a, const int8_t* b, int8_t* c, uint32_t batch,
                              hipStream_t st) {
  if (batch == 0 || m == 0 || n == 0) return hipSuccess;
  if (k == 0) return hipMemsetAsync(c, 0, (size_t)m * n * batch, st);   // __SSAT(0 >> 7, 8) = 0
  const uint64_t tiles = (uint64_t)((m + kQ7BM - 1) / kQ7BM) * ((n + kQ7BN - 1) / kQ7BN);
  if (tiles * batch > 0x7fffffffull) return hipErrorInvalidValue;
  const bool full = m % kQ7BM == 0 && n % kQ7BN == 0 && k % kQ7KT == 0 && ((uintptr_t)a & 15) == 0 &&
                    ((uintptr_t)b & 15) == 0 && ((uintptr_t)c & 15) == 0;
  const dim3 grid((uint32_t)(tiles * batch));
  if (full)
    hipLaunchKernelGGL(mat_mult_q7_kernel<true>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  else
    hipLaunchKernelGGL(mat_mult_q7_kernel<false>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  return hipGetLastError();
}

}  // namespace mi355x
