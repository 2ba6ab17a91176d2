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

// ============================================================================================
// Whole tiles (M, N multiples of 256, K of 64, 16-B aligned): the ping-pong K loop.
//
// The kernel above keeps all 8 waves in lockstep -- every wave reads its fragments, then every wave
// issues its MFMAs, then all meet at the barrier -- so on each SIMD the two waves wait for LDS at
// the same time and the matrix core idles while they do (MFMA busy 0.37-0.39).  Here the
// waves form two groups (waves 0-3 and 4-7: one of each on every SIMD, cdna_hip_programming.md
// "The 256² 8-phase template") that run one barrier apart: between two consecutive workgroup
// barriers one group issues the 16 MFMAs of its current K chunk while the other reads the next
// chunk's fragments and issues the LDS-DMA of a later chunk, then they swap.  So each SIMD always
// has one wave feeding its matrix core while the other waits on LDS, and the barrier never drains
// the DMA in flight (raw s_barrier; vmcnt counted by hand, never 0 inside the loop).
//
// Data: K in chunks of 64 bytes; a ring of FOUR chunk slots (4 x 32 KiB = the whole 128 KiB LDS
// array), slot = A (256 rows x 64 B, 16-B chunk c of row r at c ^ ((r >> 2) & 3), as above) + B (64
// k-rows x 256 B, chunk c of k-row k at c ^ 2 (k & 7): every 32-lane half of a transposing read
// takes 8 k-rows x 2 chunks = the 64 banks once).  global_load_lds_dwordx4 fills 1 KiB of LDS
// lane-linearly per wave instruction, so both swizzles are applied to the per-lane SOURCE address
// (16 rows x 64 B per A piece, 4 k-rows x 256 B per B piece; 2 + 2 pieces per wave and chunk).
//
// Phase p (chunk p, slot p & 3), per group: L_p = 16 fragment reads of chunk p (inline asm: the
// compiler neither sees nor waits for them) + the DMA of chunk p + 2 into slot (p + 2) & 3 + a wait
// until chunk p + 1 has landed (vmcnt(4): chunk p + 2's four pieces may still fly) + barrier;
// M_p = lgkmcnt(0) (tied to the fragment registers, so no MFMA moves above it) + 16 MFMAs at
// priority 1 + barrier.  Group 1 starts one barrier late, so barrier-interval 2p + 1 holds group 0's
// M_p and group 1's L_p, and interval 2p + 2 group 0's L_{p+1} and group 1's M_p.  Ordering:
//  * RAW: chunk p + 1 is read in L_{p+1} (intervals 2p + 2 / 2p + 3); every wave that loaded a piece
//    of it waited for it in L_p (intervals 2p / 2p + 1), before barrier 2p + 1, which both readers
//    pass afterwards -- the wait-then-barrier the LDS-DMA needs (MI355X_MICROARCH.md item 7);
//  * WAR: slot (p + 2) & 3 last held chunk p - 2, whose reads were issued by interval 2p - 3 and
//    retired by each reader's lgkmcnt(0) at the start of its M_{p-2} (interval 2p - 2 at the latest);
//    the refill is issued in L_p, after barrier 2p - 1.
// Group 0 adds one closing barrier, so both groups have passed the same number when the epilogue
// reuses the array (every read retired, vmcnt(0) after the last chunk).
#ifndef MI355X_Q7_PP
#define MI355X_Q7_PP 1
#endif
#ifndef MI355X_Q7_DIAG      // diagnostics (wrong results): 1 = no DMA in the loop, 2 = no fragment reads, 3 = neither
#define MI355X_Q7_DIAG 0
#endif
#ifndef MI355X_Q7_STAMP     // diagnostic: s_memtime stamps (q7_stamp_buf, tools/probes/q7_stamps.hip)
#define MI355X_Q7_STAMP 0
#endif
#ifndef MI355X_Q7_NOEPI
#define MI355X_Q7_NOEPI 0
#endif
#ifndef MI355X_Q7_WGPC      // persistent workgroups per CU (1: the LDS ring takes the whole array)
#define MI355X_Q7_WGPC 1
#endif

namespace {
constexpr int kPPSlot = 32768, kPPB = 16384;           // slot bytes; B region offset in a slot
__device__ __forceinline__ uint32_t q7_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
template <int N> __device__ __forceinline__ void q7_wait_vm() {   // s_waitcnt vmcnt(N), N < 64
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0xF70 | (N & 15) | ((N >> 4) << 14));
}
}  // namespace

#if MI355X_Q7_STAMP   // diagnostic: s_memtime at every barrier of waves 0 and 4 of workgroups 0-63
__device__ unsigned long long q7_stamp_buf[64][2][160];
__device__ unsigned long long q7_stamp_real[64][2][2];   // s_memrealtime (100 MHz) at start / end
#endif

// Persistent: gridDim.x workgroups (a multiple of 8, at most one per CU) walk the tiles, and the
// chunk stream runs on across tile boundaries -- the DMA of the next tile's first chunks is in
// flight under the current tile's last MFMAs, and a tile's output leaves from registers (below)
// while the other group computes -- so no workgroup start, prologue burst or LDS epilogue sits
// between two tiles.  Tile order: XCD x (= workgroup % 8) takes the contiguous tile run
// [x T / 8, (x + 1) T / 8) (T % 8 == 0; else round robin), its G / 8 workgroups striding through it,
// so the tiles of one matrix run together in one L2 (as the kernel above).
//
// Epilogue from registers: block (i, j) of the C^T accumulators leaves lane (r, h) with rows r,
// columns 8q + 4h .. + 3 in register group q; four saturated bytes pack into one dword D_q, and two
// v_permlane32_swap (D0 <-> D2, D1 <-> D3: lanes 32-63 of the first with lanes 0-31 of the
// second) leave lane (r, h) with columns 16h .. 16h + 15 of row r, one 16-B store.  The stores count
// in vmcnt: every counted wait below names the LOADS allowed in flight, which stays correct with
// stores outstanding (they only add to the count).
__global__ __launch_bounds__(512, 1) void mat_mult_q7_pp_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                                int8_t* __restrict__ C, int M, int K, int N,
                                                                uint32_t T) {
  __shared__ __attribute__((aligned(1024))) int8_t lds[4 * kPPSlot];
  const int tilesN = N / 256, tpm = tilesN * (M / 256);
  const uint32_t G = gridDim.x, b = blockIdx.x;
  // this workgroup's tiles: first, stride, count
  uint32_t t_first, t_stride, n_t;
  if (T % 8 == 0 && G % 8 == 0) {
    const uint32_t per = T / 8, j = b / 8, gx = G / 8;
    t_first = (b % 8) * per + j;
    t_stride = gx;
    n_t = j < per ? (per - j + gx - 1) / gx : 0;
  } else {
    t_first = b;
    t_stride = G;
    n_t = b < T ? (T - b + G - 1) / G : 0;
  }
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: SGPR arithmetic, scalar branches
  const int wm = wid >> 2, wn = wid & 3;                // wave tile: rows 128 wm .., cols 64 wn ..
  const int r = L & 31, h = L >> 5, li = L & 15, gq = (L >> 4) & 1;
#if MI355X_Q7_STAMP
  const bool stamp = b < 64 && (wid == 0 || wid == 4) && L == 0;
  int ns = 0;
  auto STAMP = [&]() {
    if (stamp && ns < 160) q7_stamp_buf[b][wid >> 2][ns] = __builtin_amdgcn_s_memtime();
    ++ns;
  };
#else
  auto STAMP = [&]() {};
#endif

  // ---- per-lane DMA offsets (the tile base is added per issue) and LDS destinations
  const size_t aLane = (size_t)(32 * wid + (L >> 2)) * K + 16 * ((L & 3) ^ ((L >> 4) & 3));
  const size_t aPiece = (size_t)16 * K;                 // piece 2w + 1: 16 rows further, same swizzle
  const size_t bLane0 = (size_t)(8 * wid + (L >> 4)) * N + 16 * ((L & 15) ^ (2 * (L >> 4)));
  const size_t bLane1 = (size_t)(8 * wid + 4 + (L >> 4)) * N + 16 * ((L & 15) ^ (2 * (4 + (L >> 4))));
  const int nc = K / 64;
  const uint32_t total = n_t * (uint32_t)nc;            // chunks this workgroup streams
  // issue cursor: chunk `ic` of tile number `it` (0-based within this workgroup's list)
  uint32_t it = 0;
  int ic = 0;
  const int8_t* aTile = nullptr;
  const int8_t* bTile = nullptr;
  auto tile_bases = [&](uint32_t k) {                    // k-th tile of this workgroup
    const uint32_t t = t_first + k * t_stride;
    const uint32_t bz = t / (uint32_t)tpm, tt = t % (uint32_t)tpm;
    const int row0 = (int)(tt / (uint32_t)tilesN) * 256, col0 = (int)(tt % (uint32_t)tilesN) * 256;
    aTile = A + (size_t)bz * M * K + (size_t)row0 * K;
    bTile = B + (size_t)bz * K * N + col0;
  };
  auto piece = [&](uint32_t g, int q) {                 // DMA piece q (A 0, A 1, B 0, B 1) of chunk g
#if MI355X_Q7_DIAG == 1 || MI355X_Q7_DIAG >= 3          // diagnostic only: no DMA past the prologue
    if (g > 2) return;
#endif
    if (ic == 0 && q == 0) tile_bases(it);
    int8_t* sl = lds + (g & 3) * kPPSlot + (q < 2 ? 0 : kPPB) + 2048 * wid + 1024 * (q & 1);
    const int8_t* src = q < 2 ? aTile + (size_t)64 * ic + aLane + (q ? aPiece : 0)
                              : bTile + (size_t)64 * ic * N + (q == 2 ? bLane0 : bLane1);
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)sl, 16, 0, 0);
    if (q == 3 && ++ic == nc) { ic = 0; ++it; }
  };
  auto issue_next = [&](uint32_t g) {                   // chunk g of the stream into slot g & 3
    piece(g, 0); piece(g, 1); piece(g, 2); piece(g, 3);
  };

  // ---- fragment read bases (slot 0): A block i adds 2048 i, B k-step kk adds 8192 kk, the hi
  // 8 k-rows of a transposing read 2048
  const uint32_t lb = q7_lds_addr(lds);
  const int arow = 128 * wm + r;
  const uint32_t aK0 = lb + arow * 64 + 16 * ((0 + h) ^ ((r >> 2) & 3));
  const uint32_t aK1 = lb + arow * 64 + 16 * ((2 + h) ^ ((r >> 2) & 3));
  const int bkr = 16 * h + (li >> 1);
  const uint32_t bJ0 = lb + kPPB + bkr * 256 + 16 * ((4 * wn + 0 + gq) ^ (2 * (bkr & 7))) + 8 * (li & 1);
  const uint32_t bJ1 = lb + kPPB + bkr * 256 + 16 * ((4 * wn + 2 + gq) ^ (2 * (bkr & 7))) + 8 * (li & 1);

  i32x16 acc[4][2];
  i32x4 fa[2][4] = {};
  v2i32 fl[2][2] = {}, fh[2][2] = {};                   // B fragments: [kk][j] lo / hi 8 k-rows

#define Q7A(dst, base, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define Q7B(dst, base, off) asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
  auto read_frags = [&](uint32_t so) {
#if MI355X_Q7_DIAG >= 2                                 // diagnostic only: no fragment reads
    return;
#endif
    const uint32_t a0 = aK0 + so, a1 = aK1 + so, b0 = bJ0 + so, b1 = bJ1 + so;
    Q7A(fa[0][0], a0, 0); Q7A(fa[0][1], a0, 2048); Q7A(fa[0][2], a0, 4096); Q7A(fa[0][3], a0, 6144);
    Q7B(fl[0][0], b0, 0); Q7B(fh[0][0], b0, 2048); Q7B(fl[0][1], b1, 0); Q7B(fh[0][1], b1, 2048);
    Q7A(fa[1][0], a1, 0); Q7A(fa[1][1], a1, 2048); Q7A(fa[1][2], a1, 4096); Q7A(fa[1][3], a1, 6144);
    Q7B(fl[1][0], b0, 8192); Q7B(fh[1][0], b0, 10240); Q7B(fl[1][1], b1, 8192); Q7B(fh[1][1], b1, 10240);
  };
#undef Q7A
#undef Q7B
  auto wait_frags = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]), "+v"(fa[0][3]), "+v"(fa[1][0]), "+v"(fa[1][1]),
                   "+v"(fa[1][2]), "+v"(fa[1][3]), "+v"(fl[0][0]), "+v"(fh[0][0]), "+v"(fl[0][1]), "+v"(fh[0][1]),
                   "+v"(fl[1][0]), "+v"(fh[1][0]), "+v"(fl[1][1]), "+v"(fh[1][1]));
  };
  auto fb = [&](int kk, int j) { return i32x4{fl[kk][j].x, fl[kk][j].y, fh[kk][j].x, fh[kk][j].y}; };
  auto mma = [&](bool first) {
    if (first) {                                        // a tile's first chunk: C operand 0
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(0, j), fa[0][i], i32x16{}, 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(0, j), fa[0][i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(1, j), fa[1][i], acc[i][j], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP();
  };
  auto store_tile = [&](uint32_t k) {                   // (q7)__SSAT(acc >> 7, 8), from registers
#if MI355X_Q7_NOEPI                                     // diagnostic only: no output stores
    if (acc[0][0][0] != 0x7fffffff) return;
#endif
    const uint32_t t = t_first + k * t_stride;
    const uint32_t bz = t / (uint32_t)tpm, tt = t % (uint32_t)tpm;
    const int row0 = (int)(tt / (uint32_t)tilesN) * 256, col0 = (int)(tt % (uint32_t)tilesN) * 256;
    int8_t* c = C + (size_t)bz * M * N + (size_t)(row0 + 128 * wm + r) * N + col0 + 64 * wn + 16 * h;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        // (q7)__SSAT(x >> 7, 8) = high byte of sat16(2x): |x| < 2^30 (K <= 65535), so 2x does not
        // wrap; in [-2^14, 2^14) the high byte of 2x is x >> 7, above / below it sat16 gives 0x7fff /
        // 0x8000.  v_cvt_pk_i16_i32 saturates two words, one v_perm_b32 takes the four high bytes.
        uint32_t d[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const auto lo = __builtin_amdgcn_cvt_pk_i16(acc[i][j][4 * q] << 1, acc[i][j][4 * q + 1] << 1);
          const auto hi = __builtin_amdgcn_cvt_pk_i16(acc[i][j][4 * q + 2] << 1, acc[i][j][4 * q + 3] << 1);
          d[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07050301u);
        }
        const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
        const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
        *reinterpret_cast<uint4*>(c + (size_t)(32 * i) * N + 32 * j) = make_uint4(s02[0], s02[1], s13[0], s13[1]);
      }
  };

  if (total == 0) return;                               // (uniform per workgroup: no barrier skipped)
#if MI355X_Q7_STAMP
  if (stamp) q7_stamp_real[b][wid >> 2][0] = __builtin_amdgcn_s_memrealtime();
#endif
  STAMP();
  issue_next(0);
  if (total > 1) { issue_next(1); q7_wait_vm<4>(); } else q7_wait_vm<0>();
  barrier();                                            // chunk 0 landed for every wave
  if (wm) barrier();                                    // group 1 runs one barrier behind
  uint32_t k = 0;                                       // tile being computed
  int p = 0;                                            // its chunk
  for (uint32_t g = 0; g < total; ++g) {
    read_frags((uint32_t)((g & 3) * kPPSlot));
    if (g + 2 < total) {
      issue_next(g + 2);
      q7_wait_vm<4>();                                  // chunk g + 1 landed (g + 2 may fly)
    } else {
      q7_wait_vm<0>();
    }
    barrier();
    wait_frags();
    __builtin_amdgcn_s_setprio(1);
    mma(p == 0);
#if MI355X_Q7_DIAG == 4                                 // diagnostic only: 32 MFMAs per segment
    mma(false);
#endif
    __builtin_amdgcn_s_setprio(0);
    barrier();
    if (++p == nc) {                                    // the tile's last chunk: its output leaves
      store_tile(k);
      p = 0;
      ++k;
    }
  }
  if (!wm) barrier();                                   // both groups: the same barrier count
#if MI355X_Q7_STAMP
  if (stamp) q7_stamp_real[b][wid >> 2][1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ============================================================================================
// K a multiple of 128: the same ping-pong with 128-deep chunks (round 6, second pass).
//
// The stamps of the kernel above put a floor of ≈ 660 cycles under an interval of 16 MFMAs (512
// cycles of matrix core): ≈ 148 cycles of every barrier interval are the hand-over between the
// groups, whatever the interval holds (32 MFMAs per interval: 1,172 cycles, MI355X_Q7_DIAG=4).
// So here a chunk is 128 k-bytes and an interval holds 32 MFMAs per wave (4 k-steps x 4 x 2
// blocks; 96 fragment VGPRs, 128 accumulators).  A 128-deep chunk is 64 KiB (A 2 x 16 KiB, one
// half per group, + B 32 KiB) and the whole 160 KiB array is the ring:
//   A0 (group 0's 128 rows) 2 slots [0, 32K), A1 2 slots [32K, 64K), B 3 slots [64K, 160K); chunk
//   s in A slot s & 1 and B slot s % 3.  A rows of 128 B, 16-B chunk c of row r at c ^ ((r >> 1) & 7)
//   (every 16-lane group of a ds_read_b128 covers the 64 banks once); B k-rows of 256 B, chunk c of
//   k-row k at c ^ 2 (k & 7) (as above).
// Barrier interval 2s: group 0 reads chunk s (L_s) while group 1 runs M_{s-1}; interval 2s + 1:
// group 1 reads chunk s, group 0 runs M_s.  L segments retire their fragment reads (lgkmcnt(0))
// before their closing barrier, so a slot is free for a refill right after its last reader's
// barrier.  Refill placement (MI355X_Q7_MDMA; the stamps of DESIGN §4 price each):
//  * 2 (default): in L_s, after its reads retire, each group refills its own A half for chunk
//    s + 2 (the slot it has just read); in M_s, one piece after every 8 MFMAs, group 0 issues the
//    first half of B(s + 2), group 1 the second half of B(s + 3).  An M segment ends with
//    vmcnt(the pieces and stores issued since the group's previous M segment): everything issued
//    before that has landed.  RAW: A_g(s + 2) (L_s) and B(s + 2) (M_s / M_{s-1}) are waited at the
//    end of M_{s+1} / M_s, before their first reader two or more intervals later; WAR: A_g(s + 2)
//    refills the slot of A_g(s), read in L_s itself; B(s + 3) (group 1, M_s = interval 2s + 2) and
//    B(s + 2) (group 0, M_s = 2s + 1) refill B(s)'s / B(s - 1)'s slot, last read in 2s + 1 / 2s - 1.
//  * 1: all eight pieces between the MFMAs (group 0: A0(s + 2), B(s + 2) first half; group 1:
//    A1(s + 2), B(s + 3) second half), the same waits.
//  * 0: all pieces in the L segment after the reads (group 0: A1(s + 1), B(s + 2) first half; group
//    1: A0(s + 2), B(s + 2) second half), each L segment ending with vmcnt(its own pieces).
// Epilogue: a tile's output leaves in the group's NEXT L segment, after its reads retire (the first
// MFMAs of the next tile take C = 0 and come after it), through the A slot it has just read; vmcnt
// counts loads, stores and LDS-DMA in issue order, so the counted waits stay exact with stores in
// flight (each counts the stores issued after the pieces it waits for).
#ifndef MI355X_Q7_PP2
#define MI355X_Q7_PP2 1
#endif
#ifndef MI355X_Q7_CSTORE
#define MI355X_Q7_CSTORE 0
#endif
#ifndef MI355X_Q7_LDSEPI    // epilogue stores through a wave's LDS scratch (16 rows x 64 B per store)
#define MI355X_Q7_LDSEPI 1
#endif
#ifndef MI355X_Q7_MDMA      // DMA pieces issued between the MFMAs of the M segments (not in the L segments)
#define MI355X_Q7_MDMA 2
#endif
#ifndef MI355X_Q7_DMA_FIRST // L segment order: the DMA pieces before the fragment reads
#define MI355X_Q7_DMA_FIRST 0
#endif
#if MI355X_Q7_DIAG == 5                                 // diagnostic only: no counted waits in the loop
#define PP2_WAIT(n) ((void)0)
#else
#define PP2_WAIT(n) q7_wait_vm<n>()
#endif

// (q7)__SSAT(acc >> 7, 8) of a wave's 128 x 64 C^T accumulator tile, from registers (see the
// comment above mat_mult_q7_pp_kernel); c = the lane's first output byte (block i = 0, j = 0).
// The doubling is one 64-bit shift per register pair: the high word gains the low word's sign bit
// as its bit 0, which never moves the high byte of sat16 (2 x_hi is even: 2 x_hi + 1 stays inside
// the int16 range exactly when 2 x_hi does, and saturates the same way outside it).
__device__ __forceinline__ void q7_store_regs(const i32x16 (&acc)[4][2], int8_t* c, int N) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint32_t d[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint64_t w0, w1;
        asm("v_lshlrev_b64 %0, 1, %1" : "=v"(w0) : "v"(__builtin_bit_cast(uint64_t, v2i32{acc[i][j][4 * q], acc[i][j][4 * q + 1]})));
        asm("v_lshlrev_b64 %0, 1, %1" : "=v"(w1) : "v"(__builtin_bit_cast(uint64_t, v2i32{acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]})));
        const auto lo = __builtin_amdgcn_cvt_pk_i16((int)(uint32_t)w0, (int)(uint32_t)(w0 >> 32));
        const auto hi = __builtin_amdgcn_cvt_pk_i16((int)(uint32_t)w1, (int)(uint32_t)(w1 >> 32));
        d[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07050301u);
      }
      const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
      const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
#if MI355X_Q7_CSTORE                                    // diagnostic only (wrong places): 1 KiB contiguous per store
      *reinterpret_cast<uint4*>(c - (size_t)(threadIdx.x & 31) * N - 16 * ((threadIdx.x >> 5) & 1) - 64 * ((threadIdx.x >> 6) & 3) +
                                8192 * ((threadIdx.x >> 6) & 3) + 1024 * (2 * i + j) + 16 * (threadIdx.x & 63)) =
          make_uint4(s02[0], s02[1], s13[0], s13[1]);
#else
      *reinterpret_cast<uint4*>(c + (size_t)(32 * i) * N + 32 * j) = make_uint4(s02[0], s02[1], s13[0], s13[1]);
#endif
    }
}

__global__ __launch_bounds__(512, 1) void mat_mult_q7_pp2_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                                 int8_t* __restrict__ C, int M, int K, int N,
                                                                 uint32_t T) {
  constexpr uint32_t kGrpA = 32768, kSlotA = 16384, kB0 = 65536, kSlotB = 32768;
  __shared__ __attribute__((aligned(1024))) int8_t lds[163840];
  const int tilesN = N / 256, tpm = tilesN * (M / 256);
  const uint32_t G = gridDim.x, b = blockIdx.x;
  uint32_t t_first, t_stride, n_t;                      // this workgroup's tiles (as above)
  if (T % 8 == 0 && G % 8 == 0) {
    const uint32_t per = T / 8, j = b / 8, gx = G / 8;
    t_first = (b % 8) * per + j;
    t_stride = gx;
    n_t = j < per ? (per - j + gx - 1) / gx : 0;
  } else {
    t_first = b;
    t_stride = G;
    n_t = b < T ? (T - b + G - 1) / G : 0;
  }
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3, wq = wid & 3;
  const int r = L & 31, h = L >> 5, li = L & 15, gq = (L >> 4) & 1;
#if MI355X_Q7_STAMP == 1
  const bool stamp = b < 64 && (wid == 0 || wid == 4) && L == 0;
  int ns = 0;
  auto STAMP = [&]() {
    if (stamp && ns < 160) q7_stamp_buf[b][wid >> 2][ns] = __builtin_amdgcn_s_memtime();
    ++ns;
  };
#else
  auto STAMP = [&]() {};
#endif
#if MI355X_Q7_STAMP == 2    // diagnostic: s_memtime ticks per loop phase, written once at the end
  uint32_t ph[8] = {};
  auto cyc = [&]() -> uint32_t {
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t v = (uint32_t)__builtin_amdgcn_s_memtime();   // (SMEM: only at points with no LDS read in flight)
    __builtin_amdgcn_sched_barrier(0);
    return v;
  };
  uint32_t tc = cyc();
  auto PH = [&](int k) { const uint32_t t = cyc(); ph[k] += t - tc; tc = t; };
#else
  auto PH = [&](int) {};
#endif
  const int nc = K / 128;
  const uint32_t total = n_t * (uint32_t)nc;

  auto tile_origin = [&](uint32_t k, int& row0, int& col0) -> uint32_t {   // k-th tile: matrix index
    const uint32_t t = t_first + k * t_stride;
    const uint32_t bz = t / (uint32_t)tpm, tt = t % (uint32_t)tpm;
    row0 = (int)(tt / (uint32_t)tilesN) * 256;
    col0 = (int)(tt % (uint32_t)tilesN) * 256;
    return bz;
  };
  auto chunk_src = [&](uint32_t g, const int8_t*& aT, const int8_t*& bT) {   // stream chunk g
    const uint32_t kt = g / (uint32_t)nc;
    const int ic = (int)(g - kt * (uint32_t)nc);
    int row0, col0;
    const uint32_t bz = tile_origin(kt, row0, col0);
    aT = A + (size_t)bz * M * K + (size_t)row0 * K + 128 * ic;
    bT = B + (size_t)bz * K * N + (size_t)(128 * ic) * N + col0;
  };
  // per-lane DMA sources (the swizzles applied to the source address; LDS lane-linear)
  // (32-bit: < 16 rows of at most 65535 bytes)
  const uint32_t aLane0 = (uint32_t)((L >> 3) * K + 16 * ((L & 7) ^ (L >> 4)));
  const uint32_t aLane1 = (uint32_t)((8 + (L >> 3)) * K + 16 * ((L & 7) ^ (4 + (L >> 4))));
  const uint32_t bLane0 = (uint32_t)((L >> 4) * N + 16 * ((L & 15) ^ (2 * (L >> 4))));
  const uint32_t bLane1 = (uint32_t)((4 + (L >> 4)) * N + 16 * ((L & 15) ^ (2 * (4 + (L >> 4)))));
  auto dma = [&](const int8_t* src, int8_t* dst) {
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };
  auto issue_B = [&](uint32_t g, int half, int slot) {  // B(g) k-rows 64 half + 16 wq .. + 15: 4 pieces
    const int8_t *aT, *bT;
    chunk_src(g, aT, bT);
    int8_t* d = lds + kB0 + slot * kSlotB + 16384 * half + 4096 * wq;
    const int8_t* s = bT + (size_t)(64 * half + 16 * wq) * N;
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(s + (size_t)(8 * (q >> 1)) * N + (q & 1 ? bLane1 : bLane0), d + 1024 * q);
  };
  auto issue_A = [&](uint32_t g, int grp) {             // A(g) rows 128 grp + 32 wq .. + 31: 4 pieces
    const int8_t *aT, *bT;
    chunk_src(g, aT, bT);
    int8_t* d = lds + grp * kGrpA + (g & 1) * kSlotA + 4096 * wq;
    const int8_t* s = aT + (size_t)(128 * grp + 32 * wq) * K;
#pragma unroll
    for (int q = 0; q < 4; ++q) dma(s + (size_t)(16 * (q >> 1)) * K + (q & 1 ? aLane1 : aLane0), d + 1024 * q);
  };

  // single pieces (MI355X_Q7_MDMA: issued between the MFMAs): q-th piece of a 4-piece A or B group
  auto src_A = [&](uint32_t g, int grp, const int8_t*& s, int8_t*& d) {
    const int8_t *aT, *bT;
    chunk_src(g, aT, bT);
    d = lds + grp * kGrpA + (g & 1) * kSlotA + 4096 * wq;
    s = aT + (size_t)(128 * grp + 32 * wq) * K;
  };
  auto src_B = [&](uint32_t g, int half, int slot, const int8_t*& s, int8_t*& d) {
    const int8_t *aT, *bT;
    chunk_src(g, aT, bT);
    d = lds + kB0 + slot * kSlotB + 16384 * half + 4096 * wq;
    s = bT + (size_t)(64 * half + 16 * wq) * N;
  };
  auto piece_A = [&](const int8_t* s, int8_t* d, int q) { dma(s + (size_t)(16 * (q >> 1)) * K + (q & 1 ? aLane1 : aLane0), d + 1024 * q); };
  auto piece_B = [&](const int8_t* s, int8_t* d, int q) { dma(s + (size_t)(8 * (q >> 1)) * N + (q & 1 ? bLane1 : bLane0), d + 1024 * q); };

  // fragment bases (slot 0): A k-step kk of block i at aK[kk] + 4096 i; B as the kernel above
  const uint32_t lb = q7_lds_addr(lds);
  const uint32_t aRow = lb + wm * kGrpA + r * 128;
  const int fr = (r >> 1) & 7;
  const uint32_t aK0 = aRow + 16 * ((0 + h) ^ fr), aK1 = aRow + 16 * ((2 + h) ^ fr);
  const uint32_t aK2 = aRow + 16 * ((4 + h) ^ fr), aK3 = aRow + 16 * ((6 + h) ^ fr);
  const int bkr = 16 * h + (li >> 1);
  const uint32_t bJ0 = lb + kB0 + bkr * 256 + 16 * ((4 * wn + 0 + gq) ^ (2 * (bkr & 7))) + 8 * (li & 1);
  const uint32_t bJ1 = lb + kB0 + bkr * 256 + 16 * ((4 * wn + 2 + gq) ^ (2 * (bkr & 7))) + 8 * (li & 1);

  i32x16 acc[4][2];
  i32x4 fa[4][4] = {};
  v2i32 fl[4][2] = {}, fh[4][2] = {};                   // B fragments: [kk][j] lo / hi 8 k-rows
#define Q7A(dst, base, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define Q7B(dst, base, off) asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define Q7KK(kk, aK)                                                                                  \
  {                                                                                                   \
    const uint32_t a_ = aK + sa;                                                                      \
    Q7A(fa[kk][0], a_, 0); Q7A(fa[kk][1], a_, 4096); Q7A(fa[kk][2], a_, 8192); Q7A(fa[kk][3], a_, 12288); \
    Q7B(fl[kk][0], b0, 8192 * kk); Q7B(fh[kk][0], b0, 8192 * kk + 2048);                              \
    Q7B(fl[kk][1], b1, 8192 * kk); Q7B(fh[kk][1], b1, 8192 * kk + 2048);                              \
  }
  auto read_frags = [&](uint32_t sa, uint32_t sb) {     // slot offsets of A and B
#if MI355X_Q7_DIAG == 2 || MI355X_Q7_DIAG == 3         // diagnostic only: no fragment reads
    return;
#endif
    const uint32_t b0 = bJ0 + sb, b1 = bJ1 + sb;
    Q7KK(0, aK0) Q7KK(1, aK1) Q7KK(2, aK2) Q7KK(3, aK3)
  };
#undef Q7KK
#undef Q7A
#undef Q7B
  auto wait_frags = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]), "+v"(fa[0][3]), "+v"(fa[1][0]), "+v"(fa[1][1]),
                   "+v"(fa[1][2]), "+v"(fa[1][3]), "+v"(fa[2][0]), "+v"(fa[2][1]), "+v"(fa[2][2]), "+v"(fa[2][3]),
                   "+v"(fa[3][0]), "+v"(fa[3][1]), "+v"(fa[3][2]), "+v"(fa[3][3]));
    asm volatile(""
                 : "+v"(fl[0][0]), "+v"(fh[0][0]), "+v"(fl[0][1]), "+v"(fh[0][1]), "+v"(fl[1][0]), "+v"(fh[1][0]),
                   "+v"(fl[1][1]), "+v"(fh[1][1]), "+v"(fl[2][0]), "+v"(fh[2][0]), "+v"(fl[2][1]), "+v"(fh[2][1]),
                   "+v"(fl[3][0]), "+v"(fh[3][0]), "+v"(fl[3][1]), "+v"(fh[3][1]));
  };
  auto fb = [&](int kk, int j) { return i32x4{fl[kk][j].x, fl[kk][j].y, fh[kk][j].x, fh[kk][j].y}; };
  auto mma = [&](bool first) {
    if (first) {                                        // a tile's first chunk: C operand 0
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(0, j), fa[0][i], i32x16{}, 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(0, j), fa[0][i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int kk = 1; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(kk, j), fa[kk][i], acc[i][j], 0, 0, 0);
  };
  auto mma4 = [&](int kk, int i0, bool first) {         // 4 of the 32 MFMAs: k-step kk, blocks i0, i0 + 1
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = first ? __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(kk, j), fa[kk][i], i32x16{}, 0, 0, 0)
                          : __builtin_amdgcn_mfma_i32_32x32x32_i8(fb(kk, j), fa[kk][i], acc[i][j], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    STAMP();
  };
  // sc: the wave's 4 KiB of scratch (its share of the group's A slot that this L segment has just
  // read and retired, refilled only after the next barrier)
  auto store_tile = [&](uint32_t k, int8_t* sc) {
#if MI355X_Q7_NOEPI                                     // diagnostic only: no output stores
    if (acc[0][0][0] != 0x7fffffff) return;
#endif
    int row0, col0;
    const uint32_t bz = tile_origin(k, row0, col0);
#if MI355X_Q7_LDSEPI
    // through LDS: each store covers 16 rows x 64 B (four lanes per row) instead of 32 rows x 32 B.
    // Scratch rows of 64 B, 16-B chunk c of row rho at c ^ ((rho >> 1) & 3): conflict-free for the
    // 8-lane groups of ds_write_b128 and the 16-lane groups of ds_read_b128.  The scratch accesses
    // are inline asm: the compiler would otherwise order them behind the LDS-DMA in flight
    // (vmcnt(0)), which targets other slots.  Buffer stores: the wave's output rows as a buffer
    // resource (SGPRs) + a 32-bit lane offset, the uniform row offset in soffset.
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t cb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(C + (size_t)bz * M * N + (size_t)(row0 + 128 * wm) * N + col0 + 64 * wn), (short)0, 0x7fffffff, 0x00020000);
    const int wr = L >> 2, wc = (L & 3) ^ ((wr >> 1) & 3);
    const uint32_t co = (uint32_t)(wr * N + 16 * (L & 3));
    const uint32_t sb = q7_lds_addr(sc), rda = sb + wr * 64 + 16 * wc;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * half + ii;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          uint32_t d[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint64_t w0, w1;
            asm("v_lshlrev_b64 %0, 1, %1" : "=v"(w0) : "v"(__builtin_bit_cast(uint64_t, v2i32{acc[i][j][4 * q], acc[i][j][4 * q + 1]})));
            asm("v_lshlrev_b64 %0, 1, %1" : "=v"(w1) : "v"(__builtin_bit_cast(uint64_t, v2i32{acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]})));
            const auto lo = __builtin_amdgcn_cvt_pk_i16((int)(uint32_t)w0, (int)(uint32_t)(w0 >> 32));
            const auto hi = __builtin_amdgcn_cvt_pk_i16((int)(uint32_t)w1, (int)(uint32_t)(w1 >> 32));
            d[q] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07050301u);
          }
          const auto s02 = __builtin_amdgcn_permlane32_swap(d[0], d[2], false, false);
          const auto s13 = __builtin_amdgcn_permlane32_swap(d[1], d[3], false, false);
          const int rho = 32 * ii + r, c = 2 * j + h;                  // scratch row, 16-B chunk
          const uint32_t wa = sb + rho * 64 + 16 * (c ^ ((rho >> 1) & 3));
          asm volatile("ds_write_b128 %0, %1" ::"v"(wa), "v"(u32x4{s02[0], s02[1], s13[0], s13[1]}) : "memory");
        }
      }
#pragma unroll
      for (int t = 0; t < 4; t += 2) {                                 // rows 16 t + (L >> 2) of this half
        u32x4 v0, v1;
        asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(v0), "=v"(v1) : "v"(rda), "i"(1024 * t), "i"(1024 * (t + 1)) : "memory");
        __builtin_amdgcn_raw_buffer_store_b128(v0, cb, (int)co, (64 * half + 16 * t) * N, 0);
        __builtin_amdgcn_raw_buffer_store_b128(v1, cb, (int)co, (64 * half + 16 * t + 16) * N, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#else
    (void)sc;
    q7_store_regs(acc, C + (size_t)bz * M * N + (size_t)(row0 + 128 * wm + r) * N + col0 + 64 * wn + 16 * h, N);
#endif
  };

  if (total == 0) return;                               // (uniform per workgroup)
#if MI355X_Q7_STAMP == 1
  if (stamp) q7_stamp_real[b][wid >> 2][0] = __builtin_amdgcn_s_memrealtime();
#endif
  STAMP();
#if MI355X_Q7_MDMA
  // prologue: B(0), B(1), B(2) second half, A0(0), A0(1), A1(0), A1(1)
  if (wm == 0) {
    issue_B(0, 0, 0);
    issue_B(0, 1, 0);
    issue_A(0, 0);
    if (total > 1) issue_A(1, 0);
  } else {
    issue_A(0, 1);
    if (total > 1) {
      issue_B(1, 0, 1);
      issue_B(1, 1, 1);
      issue_A(1, 1);
    }
    if (total > 2) issue_B(2, 1, 2);
  }
#else
  if (wm == 0) {
    issue_B(0, 0, 0);
    issue_B(0, 1, 0);
    issue_A(0, 0);
    if (total > 1) issue_A(1, 0);
  } else {
    issue_A(0, 1);
    if (total > 1) {
      issue_B(1, 0, 1);
      issue_B(1, 1, 1);
    }
  }
#endif
  // vmcnt(0) lgkmcnt(0): also retires the kernel-argument loads here, so that the waitcnt pass
  // does not leave an lgkmcnt(0) on the argument pointers inside the loop (where it would wait for
  // the inline-asm fragment reads too)
  __builtin_amdgcn_s_waitcnt(0x0070);
  barrier();
  if (wm) barrier();                                    // group 1 runs one barrier behind
  uint32_t k = 0;                                       // tile being computed
  int p = 0;                                            // its chunk
  bool pend = false;                                    // tile k - 1's output still in acc
  int rs = 0, is = 2;                                   // B slots of chunk g and of chunk g + 2
#if MI355X_Q7_MDMA
  // DMA in the M segments: group 0 in M_g issues A0(g + 2) and B(g + 2)'s first half, group 1 in
  // M_g A1(g + 2) and B(g + 3)'s second half, one piece after every 4 MFMAs; an M segment ends with
  // vmcnt(its own pieces + the stores of the L segment before it): everything the group issued in
  // its previous M segment has landed (vmcnt counts loads, stores and LDS-DMA in issue order).
  for (uint32_t g = 0; g < total; ++g) {
    PH(7);
    read_frags((g & 1) * kSlotA, rs * kSlotB);
    const int8_t *pa = nullptr, *pb = nullptr;
    int8_t *da = nullptr, *db = nullptr;
    const bool ha = g + 2 < total, hb = wm == 0 ? g + 2 < total : g + 3 < total;
    if (ha) src_A(g + 2, wm, pa, da);
    if (hb) src_B(wm == 0 ? g + 2 : g + 3, wm, wm == 0 ? is : rs, pb, db);
    wait_frags();
    PH(3);
    const bool st = pend;
    if (pend) {
      store_tile(k - 1, lds + wm * kGrpA + (g & 1) * kSlotA + 4096 * wq);
      pend = false;
    }
#if MI355X_Q7_MDMA == 2                                 // the A pieces here (this slot's reads have retired)
    if (ha) {
#pragma unroll
      for (int q = 0; q < 4; ++q) piece_A(pa, da, q);
    }
#endif
    PH(4);
    barrier();
    PH(5);
    __builtin_amdgcn_s_setprio(1);
    const bool first = p == 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {                       // 8 x (4 MFMAs, one piece)
      if (e < 2 && first)                               // a tile's first chunk: C operand 0 (a branch, not selects)
        mma4(0, 2 * e, true);
      else
        mma4(e >> 1, 2 * (e & 1), false);
      __builtin_amdgcn_sched_barrier(0);
#if MI355X_Q7_MDMA == 2                                 // the B pieces: one after every 8 MFMAs
      if ((e & 1) && hb) piece_B(pb, db, e >> 1);
#else
      if (e < 4) {
        if (ha) piece_A(pa, da, e);
      } else {
        if (hb) piece_B(pb, db, e - 4);
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
    const int nv = (ha ? 4 : 0) + (hb ? 4 : 0) + (st ? 8 : 0);
    if (nv == 16) PP2_WAIT(16); else if (nv == 12) PP2_WAIT(12); else if (nv == 8) PP2_WAIT(8);
    else if (nv == 4) PP2_WAIT(4); else PP2_WAIT(0);
    PH(6);
    barrier();
    if (++p == nc) {
      p = 0;
      ++k;
      pend = true;
    }
    rs = rs == 2 ? 0 : rs + 1;
    is = is == 2 ? 0 : is + 1;
  }
#else
  for (uint32_t g = 0; g < total; ++g) {
    PH(7);
#if !MI355X_Q7_DMA_FIRST
    read_frags((g & 1) * kSlotA, rs * kSlotB);          // (aRow holds the group's region)
#endif
    uint32_t nvm = 0;                                   // pieces issued in this L segment
#if MI355X_Q7_DIAG == 1 || MI355X_Q7_DIAG == 3         // diagnostic only: no DMA past the prologue
    if (false) {
#else
    if (true) {
#endif
      if (wm == 0) {
        if (g + 1 < total) { issue_A(g + 1, 1); nvm += 4; }
        if (g + 2 < total) { issue_B(g + 2, 0, is); nvm += 4; }
      } else if (g + 2 < total) {
        issue_A(g + 2, 0);
        issue_B(g + 2, 1, is);
        nvm = 8;
      }
    }
#if MI355X_Q7_DMA_FIRST
    read_frags((g & 1) * kSlotA, rs * kSlotB);          // (aRow holds the group's region)
#endif
    // everything this group issued one L segment earlier has landed (nvm is wave-uniform)
    if (nvm == 8) PP2_WAIT(8); else if (nvm == 4) PP2_WAIT(4); else PP2_WAIT(0);
    wait_frags();                                       // this slot's reads retired before the barrier
    PH(3);
    if (pend) {                                         // the previous tile's output, after the waits
      store_tile(k - 1, lds + wm * kGrpA + (g & 1) * kSlotA + 4096 * wq);
      pend = false;
    }
    PH(4);
    barrier();
    PH(5);
    __builtin_amdgcn_s_setprio(1);
#if MI355X_Q7_DIAG != 6                                 // diagnostic only: no MFMAs (data movement alone)
    mma(p == 0);
#endif
    __builtin_amdgcn_s_setprio(0);
    PH(6);
    barrier();
    if (++p == nc) {
      p = 0;
      ++k;
      pend = true;
    }
    rs = rs == 2 ? 0 : rs + 1;
    is = is == 2 ? 0 : is + 1;
  }
#endif
  if (pend) {                                           // (no DMA in flight any more)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7");       // the last MFMAs' results (the asm reads hide them from the hazard pass)
    store_tile(k - 1, lds + wm * kGrpA + 4096 * wq);
  }
  if (!wm) barrier();                                   // both groups: the same barrier count
#if MI355X_Q7_STAMP == 1
  if (stamp) q7_stamp_real[b][wid >> 2][1] = __builtin_amdgcn_s_memrealtime();
#elif MI355X_Q7_STAMP == 2
  if (b < 64 && (wid == 0 || wid == 4) && L == 0)
    for (int e = 0; e < 8; ++e) q7_stamp_buf[b][wid >> 2][e] = ph[e];
#endif
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
  const bool pp2 = MI355X_Q7_PP2 && k % 128 == 0;
  if (MI355X_Q7_PP && kQ7BN == 256 && m % 256 == 0 && n % 256 == 0 && k % 64 == 0 && ((uintptr_t)a & 15) == 0 &&
      ((uintptr_t)b & 15) == 0 && ((uintptr_t)c & 15) == 0 && ((size_t)n & 15) == 0) {
    // one persistent workgroup per CU (128 KiB of LDS each), a multiple of 8 so every XCD gets
    // the same number; never more than the tiles
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      int v = 0;
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
    }
    const uint64_t T = tiles * batch;
    uint32_t g = (uint32_t)std::min<uint64_t>(T, (uint64_t)(cus / 8) * 8 * MI355X_Q7_WGPC);
    if (g >= 8) g -= g % 8;
    if (pp2)
      hipLaunchKernelGGL(mat_mult_q7_pp2_kernel, dim3(g), dim3(512), 0, st, a, b, c, m, k, n, (uint32_t)T);
    else
      hipLaunchKernelGGL(mat_mult_q7_pp_kernel, dim3(g), dim3(512), 0, st, a, b, c, m, k, n, (uint32_t)T);
    return hipGetLastError();
  }
  if (full)
    hipLaunchKernelGGL(mat_mult_q7_kernel<true>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  else
    hipLaunchKernelGGL(mat_mult_q7_kernel<false>, grid, dim3(kQ7NT), 0, st, a, b, c, m, k, n);
  return hipGetLastError();
}

}  // namespace mi355x
