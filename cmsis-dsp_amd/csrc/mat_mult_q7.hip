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
// The epilogue saturates (acc >> 7) to a byte, stages the 64 KiB output tile in LDS and writes it
// as 16-B rows.  Ragged shapes take the guarded instance (zero-filled loads: a zero term adds
// nothing, there is no offset algebra to keep).
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

#ifndef MI355X_Q7_SCHED
#define MI355X_Q7_SCHED 0
#endif
#ifndef MI355X_Q7_DMA       // whole tiles through the LDS-DMA kernel
#define MI355X_Q7_DMA 0
#endif
#ifndef MI355X_Q7_PIPE      // DMA kernel: fragments of step kt + 1 read under step kt's MFMAs
#define MI355X_Q7_PIPE 0
#endif
#ifndef MI355X_Q7_TEPI      // transposed accumulators: the epilogue packs 4 outputs per LDS dword
#define MI355X_Q7_TEPI 1
#endif
#ifndef MI355X_Q7_NOEPI
#define MI355X_Q7_NOEPI 0
#endif
#ifndef MI355X_Q7_KT        // K bytes per LDS step: 64 or 128
#define MI355X_Q7_KT 64
#endif

namespace mi355x {

namespace {
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int v2i32 __attribute__((ext_vector_type(2)));

constexpr int kQ7BM = 256, kQ7BN = 256, kQ7KT = MI355X_Q7_KT, kQ7NT = 512;
static_assert(kQ7KT == 64 || kQ7KT == 128, "K step of 64 or 128 bytes");
constexpr int kQ7KC = kQ7KT / 16;                     // 16-B chunks per A row
constexpr int kQ7KS = kQ7KT / 32;                     // MFMA k-steps per K step
constexpr int kQ7NA = kQ7BM * kQ7KC / kQ7NT;          // A chunks staged per thread (2 | 4)
constexpr int kQ7NB = kQ7KT * (kQ7BN / 16) / kQ7NT;   // B chunks staged per thread (2 | 4)
constexpr int kQ7WM = 2, kQ7WN = 4;                   // wave grid
constexpr int kQ7WBM = kQ7BM / (32 * kQ7WM);          // 4 row blocks of 32 per wave
constexpr int kQ7WBN = kQ7BN / (32 * kQ7WN);          // 2 column blocks of 32 per wave
constexpr int kQ7BP = kQ7BN + 32;                     // B row pitch: 72 dwords = 8 x odd mod 64
constexpr int kQ7ABUF = kQ7BM * kQ7KT, kQ7BBUF = kQ7KT * kQ7BP, kQ7BUF = kQ7ABUF + kQ7BBUF;
constexpr int kQ7CP = kQ7BN + 16;                     // output tile pitch in LDS (bytes)
static_assert(kQ7BM * kQ7CP <= 2 * kQ7BUF, "the output tile fits the plane buffers");

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

// ---- epilogue (both kernels): (q7)__SSAT(sum >> 7, 8) into an LDS output tile, then 16-B row
// stores.  Accumulator layout of a 32 x 32 block: lane l, register g holds row (g & 3) + 8 (g >> 2)
// + 4 h, column l & 31.  The caller has passed a barrier after its last LDS read.
template <bool FULL>
__device__ __forceinline__ void q7_epilogue(const i32x16 (&acc)[kQ7WBM][kQ7WBN], int8_t* lds, int8_t* __restrict__ C,
                                            int M, int N, int row0, int col0, int wm, int wn, bool vecB) {
  const int tid = threadIdx.x, lane = tid & 63, r = lane & 31, h = lane >> 5;
  int8_t* ct = lds;
#if MI355X_Q7_NOEPI     // diagnostic only: no output (times the K loop alone)
  if (acc[0][0][0] != 0x7fffffff) return;
#endif
#if MI355X_Q7_TEPI
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
  return;
#endif
#pragma unroll
  for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
    for (int j = 0; j < kQ7WBN; ++j) {
      const int cc = wn * 32 * kQ7WBN + 32 * j + r;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int rr = wm * 32 * kQ7WBM + 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
        ct[rr * kQ7CP + cc] = (int8_t)ssat8(acc[i][j][g] >> 7);
      }
    }
  __syncthreads();
  constexpr int VPR = kQ7BN / 16;                          // 16-B words per tile row
  for (int w = tid; w < kQ7BM * VPR; w += kQ7NT) {
    const int rr = w / VPR, cw = 16 * (w % VPR);
    const int grow = row0 + rr, gcol = col0 + cw;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + rr * kQ7CP + cw);
    if (FULL) {
      *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = v;
    } else if (grow < M) {
      const int8_t* vb = ct + rr * kQ7CP + cw;
      if (vecB && (((uintptr_t)C) & 15) == 0 && gcol + 16 <= N)
        *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = v;
      else
        for (int e = 0; e < 16 && gcol + e < N; ++e) C[(size_t)grow * N + gcol + e] = vb[e];
    }
  }
}

template <bool FULL>
__global__ __launch_bounds__(kQ7NT) void mat_mult_q7_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
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

  // staging roles: A rows ar + (512 / KC) q, 16-B chunk ac; B k-rows bk + 32 q, 16 columns at bc
  const int ar = tid / kQ7KC, ac = tid % kQ7KC;
  const int bk = tid >> 4, bc = 16 * (tid & 15);
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
      const int kb = k0 + bk + 32 * q;
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
    for (int q = 0; q < kQ7NB; ++q) *reinterpret_cast<uint4*>(Bs + (bk + 32 * q) * kQ7BP + bc) = rb[q];
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
          acc[i][j] = MI355X_Q7_TEPI ? __builtin_amdgcn_mfma_i32_32x32x32_i8(fb[kq][j], fa[kq][i], acc[i][j], 0, 0, 0)
                                     : __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[kq][i], fb[kq][j], acc[i][j], 0, 0, 0);
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
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);        // one staging LDS write
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);        // one global load
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

// ---- LDS-DMA kernel for whole tiles (MI355X_Q7_DMA): the same fragments, but every K step is
// moved global -> LDS by global_load_lds_dwordx4 (no staging registers, no ds_write), two steps in
// flight in a ring of three LDS buffers, one barrier per step.  A piece (one instruction) fills
// 1 KiB of LDS lane-linearly, so the LDS swizzles are applied to the per-lane SOURCE address: A
// rows of 64 B (16 rows per piece), chunk c of row r at c ^ ((r >> 2) & 3); B rows unpadded.
// WN wave columns: MI355X_Q7_DMA = 1 -> 8 waves (2 x 4), 256 x 256 tiles, one workgroup per CU
// (96 KiB ring); = 2 -> 4 waves (2 x 2), 256 x 128 tiles, a 72 KiB ring and TWO workgroups per CU,
// so the two waves of a SIMD belong to different workgroups and one's barrier / fragment-read wait
// is covered by the other's MFMAs.
template <int WN> struct Q7D {
  static constexpr int BN = 64 * WN, NT = 128 * WN, WAVES = 2 * WN;
  static constexpr int DA = kQ7BM * 64, DBUF = DA + 64 * BN;     // 16 KiB A + 64 BN B per step
  static constexpr int APW = 16 / WAVES;                           // A pieces per wave and step
  static constexpr int BROWS = 1024 / BN;                          // k-rows per B piece
  static constexpr int PIECES = APW + 2;
};
// B slot of 16-B chunk c in k-row k: 256-B rows c ^ 2 (k & 7); 128-B rows c ^ 2 ((k >> 1) & 3).  The
// 32-lane half of a transposing read takes 8 k-rows x 2 chunks: 16 distinct 16-B slots, the 64 banks
// once; +8 / +16 / +32 k-rows keep the slot, so the reads' immediates stay valid.
template <int WN> __device__ __forceinline__ int q7_bslot(int k, int c) {
  return WN == 4 ? (c ^ (2 * (k & 7))) : (c ^ (2 * ((k >> 1) & 3)));
}

// s_waitcnt vmcnt(n), n < 16 (the other counters untouched)
template <int N> __device__ __forceinline__ void q7_wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0xF70 | N);
}

// The ring is three separate LDS objects and the K loop is unrolled by three, so every access names
// its buffer statically: the compiler's wait insertion can then tell that a fragment read of buffer
// j does not alias the DMA pieces in flight into buffer j + 2 (with one array and a dynamic buffer
// index it waits vmcnt(0) before every LDS read, i.e. for the just-issued prefetch).
template <int WN>
__global__ __launch_bounds__(Q7D<WN>::NT, WN == 2 ? 2 : 1) void mat_mult_q7_dma_kernel(const int8_t* __restrict__ A,
                                                                const int8_t* __restrict__ B,
                                                                int8_t* __restrict__ C, int M, int K, int N) {
  using D = Q7D<WN>;
  constexpr int BN = D::BN, NT = D::NT, DA = D::DA, APW = D::APW;
  __shared__ __attribute__((aligned(16))) int8_t ring0[D::DBUF];
  __shared__ __attribute__((aligned(16))) int8_t ring1[D::DBUF];
  __shared__ __attribute__((aligned(16))) int8_t ring2[D::DBUF];
  const int tilesN = N / BN, tiles = tilesN * (M / kQ7BM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;
  const int t = (int)(lin % (uint32_t)tiles);
  const int row0 = (t / tilesN) * kQ7BM, col0 = (t % tilesN) * BN;
  const size_t bz = lin / (uint32_t)tiles;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // this wave's pieces: A pieces APW wid + i (rows 16 g .. 16 g + 15), B pieces 2 wid + i (k-rows
  // BROWS g ..)
  constexpr int BCH = BN / 16;                         // 16-B chunks per B k-row
  // A piece i of this wave starts 16 i rows after piece 0, with the same swizzle ((ra >> 2) & 3 =
  // (lane >> 4) & 3 for every piece): one per-lane pointer plus a uniform offset
  const int8_t* asrc0;
  const int8_t* bsrc[2];
  {
    const int ra = 16 * APW * wid + (lane >> 2);
    asrc0 = A + (size_t)(row0 + ra) * K + 16 * ((lane & 3) ^ ((ra >> 2) & 3));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int kb = D::BROWS * g + lane / BCH;
    bsrc[i] = B + (size_t)kb * N + col0 + 16 * q7_bslot<WN>(kb, lane % BCH);
  }
  auto issue = [&](int kt, int8_t* base) {
#pragma unroll
    for (int i = 0; i < APW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc0 + ((size_t)(16 * i) * K + (size_t)kt * 64)),
                                       (__attribute__((address_space(3))) void*)(base + (APW * wid + i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (size_t)kt * 64 * N),
                                       (__attribute__((address_space(3))) void*)(base + DA + (2 * wid + i) * 1024),
                                       16, 0, 0);
  };

  i32x16 acc[kQ7WBM][kQ7WBN];
#pragma unroll
  for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
    for (int j = 0; j < kQ7WBN; ++j) acc[i][j] = i32x16{};
  const int wm = wid / WN, wn = wid % WN;
  const int r = lane & 31, h = lane >> 5, li = lane & 15, gq = (lane >> 4) & 1;
  // Fragment reads are inline asm: the compiler's wait insertion cannot separate LDS reads from
  // the LDS-DMA pieces in flight when the read is a transposing ds_read (no memory operand), and
  // would wait vmcnt(0) -- for the prefetch just issued -- before every step.  The asm reads are
  // ordered by hand: each K step issues all 12 reads of its first MFMA k-step and then of its second,
  // and waits lgkmcnt(8) / lgkmcnt(0) before the two MFMA groups; the waits take the fragment
  // registers as operands so no MFMA can be scheduled above its wait.  The step's closing barrier is a
  // bare s_barrier after explicit waits: __syncthreads()'s fence would wait vmcnt(0), i.e. for the
  // prefetch too.
  auto lds_addr = [](const int8_t* p) { return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const int8_t*)p; };
  auto step = [&](const int8_t* As) {
    const int8_t* Bs = As + DA;
    i32x4 fa[2][kQ7WBM], fb[2][kQ7WBN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < kQ7WBM; ++i) {
        const int row = wm * 32 * kQ7WBM + 32 * i + r;
        const uint32_t a = lds_addr(As + row * 64 + 16 * ((2 * kk + h) ^ ((row >> 2) & 3)));
        asm volatile("ds_read_b128 %0, %1" : "=v"(fa[kk][i]) : "v"(a));
      }
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j) {
        const int kr = 32 * kk + 16 * h + (li >> 1);
        const uint32_t b = lds_addr(Bs + kr * BN + 16 * q7_bslot<WN>(kr, 4 * wn + 2 * j + gq) + 8 * (li & 1));
        v2i32 lo, hi;
        asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(lo) : "v"(b));
        asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(hi) : "v"(b), "i"(8 * BN));
        fb[kk][j] = i32x4{lo.x, lo.y, hi.x, hi.y};
      }
    }
    asm volatile("s_waitcnt lgkmcnt(8)"
                 : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]), "+v"(fa[0][3]), "+v"(fb[0][0]), "+v"(fb[0][1]));
#pragma unroll
    for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fa[1][2]), "+v"(fa[1][3]), "+v"(fb[1][0]), "+v"(fb[1][1]));
#pragma unroll
    for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
  };

  const int nk = K / 64;
#if MI355X_Q7_PIPE
  // Software-pipelined K loop: the fragments of step kt + 1 are read into the other register set
  // between step kt's two MFMA groups, so the first group covers the barrier and the second the
  // reads' latency; every step's fragments are in registers before its MFMAs, so the DMA distance
  // is three steps (ring slot kt % 3 is refilled with step kt + 3 right after the barrier that
  // follows every wave's last read of it).  The reads take four per-lane base VGPRs plus immediate
  // offsets (slot, block, k-step), and sched_barrier(0) fences keep the compiler from moving MFMAs
  // across the phases.  The loop is unrolled by 6 (3 slots x 2 register sets) through a generic
  // lambda, so every slot / set index is a constant expression.
  static_assert(kQ7WBM == 4 && kQ7WBN == 2, "the reads below are written out for 4 x 2 blocks");
  i32x4 fs[2][2][kQ7WBM], gs[2][2][kQ7WBN];           // [set][kk][block]
  const uint32_t lb = lds_addr(ring0);
  // ring1 / ring2 follow ring0 at DBUF strides (checked below: else the loop is not used)
  const bool contiguous = lds_addr(ring1) == lb + D::DBUF && lds_addr(ring2) == lb + 2 * D::DBUF;
  const int row0l = wm * 32 * kQ7WBM + r;             // block i adds 32 rows = 2048 B
  const uint32_t aA0 = lb + row0l * 64 + 16 * ((0 + h) ^ ((r >> 2) & 3));
  const uint32_t aA1 = lb + row0l * 64 + 16 * ((2 + h) ^ ((r >> 2) & 3));
  const int kr0 = 16 * h + (li >> 1);                 // kk adds 32 k-rows
  const uint32_t bB0 = lb + DA + kr0 * BN + 16 * q7_bslot<WN>(kr0, 4 * wn + 0 + gq) + 8 * (li & 1);
  const uint32_t bB1 = lb + DA + kr0 * BN + 16 * q7_bslot<WN>(kr0, 4 * wn + 2 + gq) + 8 * (li & 1);
  // immediates are 16 bits: when slot 2's largest offset does not fit, slot 2 reads from bases
  // moved up by one slot (four more VGPRs)
  constexpr bool kHi = 2 * D::DBUF + 40 * BN + 8 > 65535 || 2 * D::DBUF + 6144 + 16 > 65535;
  static_assert(D::DBUF + 40 * BN + 8 <= 65535 && D::DBUF + 6144 + 16 <= 65535, "ds_read immediate offsets");
  const uint32_t aA0h = aA0 + (kHi ? D::DBUF : 0), aA1h = aA1 + (kHi ? D::DBUF : 0);
  const uint32_t bB0h = bB0 + (kHi ? D::DBUF : 0), bB1h = bB1 + (kHi ? D::DBUF : 0);
#define Q7A(dst, base, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define Q7B(dst, base, off) asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
  const uint32_t aA0l = aA0, aA1l = aA1, bB0l = bB0, bB1l = bB1;
  auto rd = [&](auto SLOT, i32x4 (&fa)[2][kQ7WBM], i32x4 (&fb)[2][kQ7WBN]) {
    constexpr bool hi = kHi && decltype(SLOT)::value == 2;
    constexpr int so = (hi ? 1 : decltype(SLOT)::value) * D::DBUF;
    const uint32_t aA0 = hi ? aA0h : aA0l, aA1 = hi ? aA1h : aA1l, bB0 = hi ? bB0h : bB0l, bB1 = hi ? bB1h : bB1l;
    Q7A(fa[0][0], aA0, so + 0); Q7A(fa[0][1], aA0, so + 2048); Q7A(fa[0][2], aA0, so + 4096); Q7A(fa[0][3], aA0, so + 6144);
    v2i32 l0, h0, l1, h1;
    Q7B(l0, bB0, so); Q7B(h0, bB0, so + 8 * BN); Q7B(l1, bB1, so); Q7B(h1, bB1, so + 8 * BN);
    fb[0][0] = i32x4{l0.x, l0.y, h0.x, h0.y};
    fb[0][1] = i32x4{l1.x, l1.y, h1.x, h1.y};
    Q7A(fa[1][0], aA1, so + 0); Q7A(fa[1][1], aA1, so + 2048); Q7A(fa[1][2], aA1, so + 4096); Q7A(fa[1][3], aA1, so + 6144);
    v2i32 l2, h2, l3, h3;
    Q7B(l2, bB0, so + 32 * BN); Q7B(h2, bB0, so + 40 * BN); Q7B(l3, bB1, so + 32 * BN); Q7B(h3, bB1, so + 40 * BN);
    fb[1][0] = i32x4{l2.x, l2.y, h2.x, h2.y};
    fb[1][1] = i32x4{l3.x, l3.y, h3.x, h3.y};
  };
#undef Q7A
#undef Q7B
  auto wait_set = [&](i32x4 (&fa)[2][kQ7WBM], i32x4 (&fb)[2][kQ7WBN]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]), "+v"(fa[0][3]),
                 "+v"(fb[0][0]), "+v"(fb[0][1]));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fa[1][2]), "+v"(fa[1][3]),
                 "+v"(fb[1][0]), "+v"(fb[1][1]));
  };
  auto mma = [&](const i32x4 (&fa)[kQ7WBM], const i32x4 (&fb)[kQ7WBN]) {
#pragma unroll
    for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  auto ring = [&](auto SLOT) -> int8_t* { return SLOT.value == 0 ? ring0 : (SLOT.value == 1 ? ring1 : ring2); };
  if (!contiguous) __builtin_trap();                    // layout assumption (never taken: one kernel, 3 objects)
  issue(0, ring0);
  if (nk > 1) issue(1, ring1);
  if (nk > 2) issue(2, ring2);
  if (nk > 2) q7_wait_vm<2 * D::PIECES>(); else if (nk > 1) q7_wait_vm<D::PIECES>(); else q7_wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  rd(I0{}, fs[0], gs[0]);
  // one step: U = kt mod 6 (slot U mod 3, register set U mod 2)
  auto body = [&](int kt, auto CUR, auto NXT, auto SET) {
    constexpr int cs = decltype(SET)::value;
    wait_set(fs[cs], gs[cs]);
    __builtin_amdgcn_sched_barrier(0);
    mma(fs[cs][0], gs[cs][0]);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) {
      if (kt + 2 < nk) q7_wait_vm<D::PIECES>(); else q7_wait_vm<0>();   // step kt + 1 landed
      __builtin_amdgcn_s_barrier();                   // ... for every wave; slot CUR read by all
      if (kt + 3 < nk) issue(kt + 3, ring(CUR));
      rd(NXT, fs[cs ^ 1], gs[cs ^ 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    mma(fs[cs][1], gs[cs][1]);
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int k0 = 0; k0 < nk; k0 += 6) {
    body(k0, I0{}, I1{}, I0{});
    if (k0 + 1 < nk) body(k0 + 1, I1{}, I2{}, I1{});
    if (k0 + 2 < nk) body(k0 + 2, I2{}, I0{}, I0{});
    if (k0 + 3 < nk) body(k0 + 3, I0{}, I1{}, I1{});
    if (k0 + 4 < nk) body(k0 + 4, I1{}, I2{}, I0{});
    if (k0 + 5 < nk) body(k0 + 5, I2{}, I0{}, I1{});
  }
  __syncthreads();                                     // every wave's reads done before the staging
#else
  issue(0, ring0);
  if (nk > 1) issue(1, ring1);
  if (nk > 1) q7_wait_vm<D::PIECES>(); else q7_wait_vm<0>();   // step 0 landed; step 1 may fly
  __builtin_amdgcn_s_barrier();
  // iteration kt computes ring kt % 3 and issues step kt + 2 into ring (kt + 2) % 3, which was read
  // in iteration kt - 1 (its reads completed -- lgkmcnt(0) -- before its closing barrier)
  auto body = [&](int kt, const int8_t* cur, int8_t* nxt) {
    const bool more = kt + 2 < nk;
    if (more) issue(kt + 2, nxt);
    step(cur);
    if (more) q7_wait_vm<D::PIECES>(); else q7_wait_vm<0>();   // step kt + 1 landed; kt + 2 may fly
    __builtin_amdgcn_s_barrier();
  };
  for (int kt = 0; kt < nk; kt += 3) {
    body(kt, ring0, ring2);
    if (kt + 1 < nk) body(kt + 1, ring1, ring0);
    if (kt + 2 < nk) body(kt + 2, ring2, ring1);
  }
#endif
  // epilogue: rows of wave-row group wm staged in ring wm (128 rows x BN bytes each)
  {
#if MI355X_Q7_NOEPI
    if (acc[0][0][0] != 0x7fffffff) return;
#endif
    int8_t* ct = wm ? ring1 : ring0;
#pragma unroll
    for (int i = 0; i < kQ7WBM; ++i)
#pragma unroll
      for (int j = 0; j < kQ7WBN; ++j) {
        const int cc = wn * 32 * kQ7WBN + 32 * j + r;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int rr = 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;          // row within the group
          ct[rr * BN + cc] = (int8_t)ssat8(acc[i][j][g] >> 7);
        }
      }
    __syncthreads();
    for (int w = tid; w < kQ7BM * (BN / 16); w += NT) {
      const int rr = w / (BN / 16), cw = 16 * (w % (BN / 16));
      const int8_t* src = (rr < 128 ? ring0 : ring1) + (rr & 127) * BN + cw;
      *reinterpret_cast<uint4*>(C + (size_t)(row0 + rr) * N + col0 + cw) = *reinterpret_cast<const uint4*>(src);
    }
  }
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
  constexpr int kDWN = MI355X_Q7_DMA == 2 ? 2 : 4;
  if (MI355X_Q7_DMA && m % kQ7BM == 0 && n % Q7D<kDWN>::BN == 0 && k % 64 == 0 && ((uintptr_t)a & 15) == 0 &&
      ((uintptr_t)b & 15) == 0 && ((uintptr_t)c & 15) == 0) {
    const uint64_t dt = (uint64_t)(m / kQ7BM) * (n / Q7D<kDWN>::BN) * batch;
    if (dt <= 0x7fffffffull) {
      hipLaunchKernelGGL(mat_mult_q7_dma_kernel<kDWN>, dim3((uint32_t)dt), dim3(Q7D<kDWN>::NT), 0, st, a, b, c, m, k, n);
      return hipGetLastError();
    }
  }
  if (full)
    hipLaunchKernelGGL(mat_mult_q7_kernel<true>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  else
    hipLaunchKernelGGL(mat_mult_q7_kernel<false>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  return hipGetLastError();
}

}  // namespace mi355x
