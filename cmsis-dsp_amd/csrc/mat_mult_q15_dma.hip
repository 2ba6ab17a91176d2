// Batched q15 matrix multiply, whole tiles: raw q15 tiles moved by LDS-DMA, byte planes cut from
// the fragments in registers — MI355X, bit-exact.
//
// Same arithmetic as mat_mult_fixed.hip's byte-plane kernels (arm_mat_mult_q15.c:741-912 and the
// fast form arm_mat_mult_fast_q15.c:351-401): v = 256 t_hi + t_lo + 128 with t_hi the signed top
// byte and t_lo = low byte - 128, the four plane products on v_mfma_i32_32x32x32_i8 into three
// int32 class accumulators (exact for K <= 32704), and
//   C_ij = acc0 + 256 acc1 + 65536 acc2 + 128 (rowsum(A)_i + colsum(B)_j) - 128^2 K   (mod 2^64).
// What changes is where the plane split happens.  The register-staged kernel (v2) loads, splits,
// transposes and sums in its staging phase, with every wave of the workgroup in lockstep at one
// barrier per K step, so its MFMA and staging phases alternate (MFMA busy 34 %).  Here
//  * the K step's RAW q15 tiles go global -> LDS by global_load_lds_dwordx4 (no staging registers,
//    no ds_write), three steps in a ring of three LDS objects, one bare s_barrier per step;
//  * A fragments are two ds_read_b128 of 16 k-consecutive q15 values per lane; B fragments are four
//    ds_read_b64_tr_b16 (gfx950's 16-bit transposing read: per 16-lane group 4 k-rows x 16 columns,
//    lane i receiving column i), i.e. 16 k-consecutive values of one column per lane: no transpose
//    pass at all;
//  * each raw fragment is cut into its two byte planes with one v_perm per 4 values and plane
//    (plus one xor for the low plane), right before its MFMAs;
//  * the exact row / column sums come from the same raw fragments (v_dot2 with {1, 1}), summed only
//    by the waves of one wave column (rows) / one wave row (columns).
// LDS images (per ring slot, 32 KiB): A [128 rows][64 q15] with 16-B chunk c of row r at
// c ^ ((r >> 1) & 7) (conflict-free ds_read_b128: every 16-lane group meets (r & 1, slot) pairs
// that are all distinct); B [64 k-rows][128 q15] with chunk c of k-row k at c ^ 4 (k & 3) (each
// 32-lane half of a transposing read takes 4 rows x 4 chunks: 16 distinct slots, the 64 banks
// once).  A piece (one DMA instruction) fills 1 KiB lane-linearly, so the swizzles are applied to
// the per-lane source addresses.  LDS reads are inline asm with hand-counted lgkmcnt waits: the
// compiler cannot tell a transposing read from the DMA writes in flight and would otherwise wait
// for every outstanding piece before each read (see mat_mult_q7.hip).
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

#ifndef MI355X_Q15_PIPE      // fragments of step kt + 1 read under step kt's MFMAs
#define MI355X_Q15_PIPE 0
#endif

namespace mi355x {

namespace {
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int v2i32 __attribute__((ext_vector_type(2)));
typedef short s2x __attribute__((ext_vector_type(2)));

// WN wave columns: WN = 2 -> 8 waves, 128 x 128 tiles, one workgroup per CU (96 KiB ring);
// WN = 1 -> 4 waves, 128 x 64 tiles, a 72 KiB ring and TWO workgroups per CU, so the two waves
// of a SIMD belong to different workgroups and one's barrier / fragment-read wait is covered by
// the other's MFMAs (MI355X_Q15_DMA = 2).
constexpr int kQdBM = 128, kQdKT = 64;
template <int WN> struct QdCfg {
  static constexpr int BN = 64 * WN, NT = 256 * WN, WAVES = 4 * WN;
  static constexpr int A = kQdBM * kQdKT * 2, BUF = A + kQdKT * BN * 2;   // 16 + 8 WN KiB
  static constexpr int APW = 16 / WAVES;                 // A pieces (1 KiB) per wave and K step
  static constexpr int BROWS = 1024 / (2 * BN);          // k-rows per B piece
  static constexpr int PIECES = APW + 2;                 // DMA instructions per wave and K step
};
constexpr int kQdMaxK = 32704;

__device__ __forceinline__ uint32_t qd_lds(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p;
}
__device__ __forceinline__ int qd_aslot(int r, int c) { return c ^ ((r >> 1) & 7); }
// B rows of 256 B (WN = 2): chunk c of k-row k at c ^ 4 (k & 3); rows of 128 B (WN = 1): at
// c ^ 4 ((k >> 1) & 1).  Either way a 32-lane half of a transposing read (4 k-rows x 4 chunks)
// meets the 64 banks once, and +4 / +32 k-rows keep the slot, so the reads' immediates stay valid.
template <int WN> __device__ __forceinline__ int qd_bslot(int k, int c) {
  return WN == 2 ? (c ^ (4 * (k & 3))) : (c ^ (4 * ((k >> 1) & 1)));
}
// plane p of the four q15 values in d0, d1 (k order): signed top byte (p = 1) or low byte - 128
__device__ __forceinline__ int qd_plane(uint32_t d0, uint32_t d1, int p) {
  const uint32_t sel = (uint32_t)p | (uint32_t)(2 + p) << 8 | (uint32_t)(4 + p) << 16 | (uint32_t)(6 + p) << 24;
  const uint32_t w = __builtin_amdgcn_perm(d1, d0, sel);
  return (int)(p ? w : w ^ 0x80808080u);
}
template <int N> __device__ __forceinline__ void qd_wait_vm() {   // s_waitcnt vmcnt(N), N < 16
  static_assert(N >= 0 && N < 16, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0xF70 | N);
}
}  // namespace

template <bool FAST, int WN>
__global__ __launch_bounds__(QdCfg<WN>::NT, WN == 1 ? 2 : 1) void mat_mult_q15_dma_kernel(const int16_t* __restrict__ A,
                                                                 const int16_t* __restrict__ B,
                                                                 int16_t* __restrict__ C, int M, int K, int N) {
  using Cf = QdCfg<WN>;
  constexpr int kQdBN = Cf::BN, kQdNT = Cf::NT, kQdWN = WN, kQdA = Cf::A, kQdBUF = Cf::BUF;
  __shared__ __attribute__((aligned(16))) int8_t ring0[kQdBUF];
  __shared__ __attribute__((aligned(16))) int8_t ring1[kQdBUF];
  __shared__ __attribute__((aligned(16))) int8_t ring2[kQdBUF];

  const int tilesN = N / kQdBN, tiles = tilesN * (M / kQdBM);
  const uint32_t total = gridDim.x;
  uint32_t lin = blockIdx.x;
  if (total % 8 == 0) lin = (lin % 8) * (total / 8) + lin / 8;   // XCD-aware (as the other GEMMs)
  const int t = (int)(lin % (uint32_t)tiles);
  const int row0 = (t / tilesN) * kQdBM, col0 = (t % tilesN) * kQdBN;
  const size_t bz = lin / (uint32_t)tiles;
  A += bz * (size_t)M * K;
  B += bz * (size_t)K * N;
  C += bz * (size_t)M * N;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // DMA pieces of this wave: A pieces APW wid + i (rows 8 g .. 8 g + 7), B pieces 2 wid + i (k-rows
  // BROWS g ..); source addresses carry the LDS swizzle
  constexpr int APW = Cf::APW, BCH = kQdBN / 8;            // B 16-B chunks per k-row
  const int16_t* asrc[APW];
  const int16_t* bsrc[2];
#pragma unroll
  for (int i = 0; i < APW; ++i) {
    const int g = APW * wid + i;
    const int ra = 8 * g + (lane >> 3);
    asrc[i] = A + (size_t)(row0 + ra) * K + 8 * qd_aslot(ra, lane & 7);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int g = 2 * wid + i;
    const int kb = Cf::BROWS * g + lane / BCH;
    bsrc[i] = B + (size_t)kb * N + col0 + 8 * qd_bslot<WN>(kb, lane % BCH);
  }
  auto issue = [&](int kt, int8_t* base) {
#pragma unroll
    for (int i = 0; i < APW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (size_t)kt * kQdKT),
                                       (__attribute__((address_space(3))) void*)(base + (APW * wid + i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + (size_t)kt * kQdKT * N),
                                       (__attribute__((address_space(3))) void*)(base + kQdA + (2 * wid + i) * 1024),
                                       16, 0, 0);
  };

  const int wm = wid / kQdWN, wn = wid % kQdWN;
  const int r = lane & 31, h = lane >> 5, li = lane & 15, gq = (lane >> 4) & 1;
  const int arow = wm * 32 + r;
  // per-lane LDS byte offsets inside a ring slot: A chunks (kk, e) of this lane's row; B block j's
  // first tr_b16 address (the four reads of a k-step are +1024 B apart, the second k-step +8192)
  uint32_t aoff[2][2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int e = 0; e < 2; ++e) aoff[kk][e] = (uint32_t)(arow * 128 + 16 * qd_aslot(arow, 4 * kk + 2 * h + e));
  {
    const int q = li >> 2, p = li & 3;
    const int kr = 16 * h + q;                            // k-row of read 0 in k-step 0
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = 8 * wn + 4 * j + 2 * gq + (p >> 1);   // 16-B chunk of columns 4p .. 4p + 3
      boff[j] = (uint32_t)(kQdA + kr * (2 * kQdBN) + 16 * qd_bslot<WN>(kr, c) + 8 * (p & 1));
    }
  }
  const bool do_rows = wn == 0, do_cols = wm == 0;        // wave-uniform
  int32_t rsum = 0, csum[2] = {0, 0};

  i32x16 acc[3][2];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[s][j] = i32x16{};

  // one K step from ring slot `base`
  auto step = [&](const int8_t* base) {
    const uint32_t b0 = qd_lds(base);
    i32x4 ra[2][2], rb[2][2][2];          // raw dwords: A [kk][e], B [kk][j][t pair]
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int e = 0; e < 2; ++e) asm volatile("ds_read_b128 %0, %1" : "=v"(ra[kk][e]) : "v"(b0 + aoff[kk][e]));
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        v2i32 x0, x1, x2, x3;
        const uint32_t ba = b0 + boff[j];
        constexpr int R4 = 4 * 2 * kQdBN;                 // 4 k-rows in bytes
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x0) : "v"(ba), "i"(8 * R4 * kk));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x1) : "v"(ba), "i"(8 * R4 * kk + R4));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x2) : "v"(ba), "i"(8 * R4 * kk + 2 * R4));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x3) : "v"(ba), "i"(8 * R4 * kk + 3 * R4));
        rb[kk][j][0] = i32x4{x0.x, x0.y, x1.x, x1.y};
        rb[kk][j][1] = i32x4{x2.x, x2.y, x3.x, x3.y};
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk == 0)
        asm volatile("s_waitcnt lgkmcnt(10)"
                     : "+v"(ra[0][0]), "+v"(ra[0][1]), "+v"(rb[0][0][0]), "+v"(rb[0][0][1]), "+v"(rb[0][1][0]),
                       "+v"(rb[0][1][1]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(ra[1][0]), "+v"(ra[1][1]), "+v"(rb[1][0][0]), "+v"(rb[1][0][1]), "+v"(rb[1][1][0]),
                       "+v"(rb[1][1][1]));
      // raw dwords in k order: A d[0..7] = ra[kk][0].xyzw, ra[kk][1].xyzw; B likewise per block
      uint32_t ad[8], bd[2][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ad[u] = (uint32_t)ra[kk][0][u];
        ad[4 + u] = (uint32_t)ra[kk][1][u];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          bd[j][u] = (uint32_t)rb[kk][j][0][u];
          bd[j][4 + u] = (uint32_t)rb[kk][j][1][u];
        }
      }
      if (do_rows) {
#pragma unroll
        for (int u = 0; u < 8; ++u) rsum = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, ad[u]), s2x{1, 1}, rsum, false);
      }
      if (do_cols) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            csum[j] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, bd[j][u]), s2x{1, 1}, csum[j], false);
      }
      i32x4 fa[2], fb[2][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        fa[p] = i32x4{qd_plane(ad[0], ad[1], p), qd_plane(ad[2], ad[3], p), qd_plane(ad[4], ad[5], p),
                      qd_plane(ad[6], ad[7], p)};
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[p][j] = i32x4{qd_plane(bd[j][0], bd[j][1], p), qd_plane(bd[j][2], bd[j][3], p),
                           qd_plane(bd[j][4], bd[j][5], p), qd_plane(bd[j][6], bd[j][7], p)};
      }
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[p + q][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[p], fb[q][j], acc[p + q][j], 0, 0, 0);
    }
  };

  const int nk = K / kQdKT;
#if MI355X_Q15_PIPE
  // Software-pipelined K loop (as mat_mult_q7.hip MI355X_Q7_PIPE): the raw fragments of step kt + 1
  // are read into the other register set between step kt's two k-steps, so the first k-step's
  // plane split and MFMAs cover the barrier and the second the reads' latency; ring slot kt % 3 is
  // refilled with step kt + 3 right after the barrier that follows every wave's last read of it.
  // Reads: six per-lane base VGPRs (A chunk (kk, e), B block j) plus immediates (slot, k-rows).
  i32x4 pra[2][2][2], prb[2][2][2][2];                   // [set][kk][e], [set][kk][j][t pair]
  const uint32_t lb = qd_lds(ring0);
  const bool contiguous = qd_lds(ring1) == lb + kQdBUF && qd_lds(ring2) == lb + 2 * kQdBUF;
  constexpr int R4 = 4 * 2 * kQdBN;                     // 4 k-rows in bytes
  constexpr bool kHi = 2 * kQdBUF + kQdA + 8 * R4 + 3 * R4 + 8 > 65535;   // slot 2 from raised bases
  static_assert(kQdBUF + kQdA + 8 * R4 + 3 * R4 + 8 <= 65535, "ds_read immediate offsets");
  uint32_t aB[2][2][2], bB[2][2];                       // [lo/hi][kk][e], [lo/hi][j]
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    const uint32_t add = (hb && kHi) ? (uint32_t)kQdBUF : 0u;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int e = 0; e < 2; ++e) aB[hb][kk][e] = lb + aoff[kk][e] + add;
#pragma unroll
    for (int j = 0; j < 2; ++j) bB[hb][j] = lb + boff[j] + add;
  }
#define QDA(dst, base, off) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
#define QDB(dst, base, off) asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(off))
  auto rd = [&](auto SLOT, i32x4 (&ra)[2][2], i32x4 (&rb)[2][2][2]) {
    constexpr bool hi = kHi && decltype(SLOT)::value == 2;
    constexpr int so = (hi ? 1 : decltype(SLOT)::value) * kQdBUF;
    constexpr int hb = hi ? 1 : 0;
    QDA(ra[0][0], aB[hb][0][0], so); QDA(ra[0][1], aB[hb][0][1], so);
    v2i32 x0, x1, x2, x3, y0, y1, y2, y3;
    QDB(x0, bB[hb][0], so); QDB(x1, bB[hb][0], so + R4); QDB(x2, bB[hb][0], so + 2 * R4); QDB(x3, bB[hb][0], so + 3 * R4);
    QDB(y0, bB[hb][1], so); QDB(y1, bB[hb][1], so + R4); QDB(y2, bB[hb][1], so + 2 * R4); QDB(y3, bB[hb][1], so + 3 * R4);
    rb[0][0][0] = i32x4{x0.x, x0.y, x1.x, x1.y}; rb[0][0][1] = i32x4{x2.x, x2.y, x3.x, x3.y};
    rb[0][1][0] = i32x4{y0.x, y0.y, y1.x, y1.y}; rb[0][1][1] = i32x4{y2.x, y2.y, y3.x, y3.y};
    QDA(ra[1][0], aB[hb][1][0], so); QDA(ra[1][1], aB[hb][1][1], so);
    v2i32 z0, z1, z2, z3, w0, w1, w2, w3;
    QDB(z0, bB[hb][0], so + 8 * R4); QDB(z1, bB[hb][0], so + 9 * R4); QDB(z2, bB[hb][0], so + 10 * R4); QDB(z3, bB[hb][0], so + 11 * R4);
    QDB(w0, bB[hb][1], so + 8 * R4); QDB(w1, bB[hb][1], so + 9 * R4); QDB(w2, bB[hb][1], so + 10 * R4); QDB(w3, bB[hb][1], so + 11 * R4);
    rb[1][0][0] = i32x4{z0.x, z0.y, z1.x, z1.y}; rb[1][0][1] = i32x4{z2.x, z2.y, z3.x, z3.y};
    rb[1][1][0] = i32x4{w0.x, w0.y, w1.x, w1.y}; rb[1][1][1] = i32x4{w2.x, w2.y, w3.x, w3.y};
  };
#undef QDA
#undef QDB
  auto wait_set = [&](i32x4 (&ra)[2][2], i32x4 (&rb)[2][2][2]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra[0][0]), "+v"(ra[0][1]), "+v"(rb[0][0][0]), "+v"(rb[0][0][1]),
                 "+v"(rb[0][1][0]), "+v"(rb[0][1][1]));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ra[1][0]), "+v"(ra[1][1]), "+v"(rb[1][0][0]), "+v"(rb[1][0][1]),
                 "+v"(rb[1][1][0]), "+v"(rb[1][1][1]));
  };
  // one k-step from raw fragments: the exact row / column sums, the byte planes, 8 MFMAs
  auto kstep = [&](const i32x4 (&ra)[2], const i32x4 (&rb)[2][2]) {
    uint32_t ad[8], bd[2][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      ad[u] = (uint32_t)ra[0][u];
      ad[4 + u] = (uint32_t)ra[1][u];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bd[j][u] = (uint32_t)rb[j][0][u];
        bd[j][4 + u] = (uint32_t)rb[j][1][u];
      }
    }
    if (do_rows) {
#pragma unroll
      for (int u = 0; u < 8; ++u) rsum = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, ad[u]), s2x{1, 1}, rsum, false);
    }
    if (do_cols) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          csum[j] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2x, bd[j][u]), s2x{1, 1}, csum[j], false);
    }
    i32x4 fa[2], fb[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      fa[p] = i32x4{qd_plane(ad[0], ad[1], p), qd_plane(ad[2], ad[3], p), qd_plane(ad[4], ad[5], p),
                    qd_plane(ad[6], ad[7], p)};
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[p][j] = i32x4{qd_plane(bd[j][0], bd[j][1], p), qd_plane(bd[j][2], bd[j][3], p),
                         qd_plane(bd[j][4], bd[j][5], p), qd_plane(bd[j][6], bd[j][7], p)};
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[p + q][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[p], fb[q][j], acc[p + q][j], 0, 0, 0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  auto ring = [&](auto SLOT) -> int8_t* { return SLOT.value == 0 ? ring0 : (SLOT.value == 1 ? ring1 : ring2); };
  if (!contiguous) __builtin_trap();                    // layout assumption
  issue(0, ring0);
  if (nk > 1) issue(1, ring1);
  if (nk > 2) issue(2, ring2);
  if (nk > 2) qd_wait_vm<2 * Cf::PIECES>(); else if (nk > 1) qd_wait_vm<Cf::PIECES>(); else qd_wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  rd(I0{}, pra[0], prb[0]);
  auto body = [&](int kt, auto CUR, auto NXT, auto SET) {
    constexpr int cs = decltype(SET)::value;
    wait_set(pra[cs], prb[cs]);
    __builtin_amdgcn_sched_barrier(0);
    kstep(pra[cs][0], prb[cs][0]);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) {
      if (kt + 2 < nk) qd_wait_vm<Cf::PIECES>(); else qd_wait_vm<0>();   // step kt + 1 landed
      __builtin_amdgcn_s_barrier();                   // ... for every wave; slot CUR read by all
      if (kt + 3 < nk) issue(kt + 3, ring(CUR));
      rd(NXT, pra[cs ^ 1], prb[cs ^ 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    kstep(pra[cs][1], prb[cs][1]);
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
  __syncthreads();                                       // every wave's reads done before the epilogue
#else
  issue(0, ring0);
  if (nk > 1) issue(1, ring1);
  if (nk > 1) qd_wait_vm<Cf::PIECES>(); else qd_wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  auto body = [&](int kt, const int8_t* cur, int8_t* nxt) {
    const bool more = kt + 2 < nk;
    if (more) issue(kt + 2, nxt);
    step(cur);
    if (more) qd_wait_vm<Cf::PIECES>(); else qd_wait_vm<0>();   // step kt + 1 landed (kt + 2 may fly)
    __builtin_amdgcn_s_barrier();
  };
  for (int kt = 0; kt < nk; kt += 3) {
    body(kt, ring0, ring2);
    if (kt + 1 < nk) body(kt + 1, ring1, ring0);
    if (kt + 2 < nk) body(kt + 2, ring2, ring1);
  }

#endif

  // ---- epilogue: the two k-halves of the row / column sums meet in LDS (ring1), the int64 combine,
  // the output tile staged in ring0 as q15 and written as 16-B rows
  int32_t* rsp = reinterpret_cast<int32_t*>(ring1);          // [2][128] row partials (h)
  int32_t* csp = rsp + 2 * kQdBM;                            // [2][128] column partials (h)
  if (do_rows) rsp[h * kQdBM + arow] = rsum;
  if (do_cols) {
#pragma unroll
    for (int j = 0; j < 2; ++j) csp[h * kQdBN + wn * 64 + 32 * j + r] = csum[j];
  }
  __syncthreads();
  int16_t* ct = reinterpret_cast<int16_t*>(ring0);          // [128][BN]
  const int64_t C0 = 128;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cc = wn * 64 + 32 * j + r;
    const int64_t cs = (int64_t)csp[cc] + csp[kQdBN + cc];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int rr = wm * 32 + (g & 3) + 8 * (g >> 2) + 4 * h;
      const int64_t rs = (int64_t)rsp[rr] + rsp[kQdBM + rr];
      uint64_t v = (uint64_t)(C0 * (rs + cs)) - (uint64_t)K * (uint64_t)(C0 * C0);
      v += (uint64_t)(int64_t)acc[0][j][g];
      v += (uint64_t)(int64_t)acc[1][j][g] << 8;
      v += (uint64_t)(int64_t)acc[2][j][g] << 16;
      const int64_t sum = (int64_t)v;
      ct[rr * kQdBN + cc] = FAST ? (int16_t)((int32_t)(uint32_t)v >> 15) : (int16_t)ssat16((int32_t)(sum >> 15));
    }
  }
  __syncthreads();
  for (int w = tid; w < kQdBM * (kQdBN / 8); w += kQdNT) {  // 8 q15 outputs per 16-B word
    const int rr = w / (kQdBN / 8), cw = 8 * (w % (kQdBN / 8));
    *reinterpret_cast<uint4*>(C + (size_t)(row0 + rr) * N + col0 + cw) =
        *reinterpret_cast<const uint4*>(ct + rr * kQdBN + cw);
  }
}

// Whole tiles only (M multiple of 128, N of 128 / 64, K of 64, 16-B aligned operands, K <= 32704);
// returns false when the shape is not one (the caller takes the general kernels).
template <int WN>
static void qd_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c, uint32_t grid, hipStream_t st,
                      int fast) {
  if (fast)
    hipLaunchKernelGGL((mat_mult_q15_dma_kernel<true, WN>), dim3(grid), dim3(QdCfg<WN>::NT), 0, st, a, b, c, m, k, n);
  else
    hipLaunchKernelGGL((mat_mult_q15_dma_kernel<false, WN>), dim3(grid), dim3(QdCfg<WN>::NT), 0, st, a, b, c, m, k, n);
}
bool mat_mult_q15_dma_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c, uint32_t batch,
                             hipStream_t st, int fast, hipError_t* err) {
  if (!MI355X_Q15_DMA) return false;
  constexpr int WN = MI355X_Q15_DMA == 2 ? 1 : 2;
  constexpr int BN = QdCfg<WN>::BN;
  if (m % kQdBM || n % BN || k % kQdKT || k > kQdMaxK || k == 0) return false;
  if (((uintptr_t)a & 15) || ((uintptr_t)b & 15) || ((uintptr_t)c & 15)) return false;
  const uint64_t tiles = (uint64_t)(m / kQdBM) * (n / BN);
  if (tiles * batch > 0x7fffffffull || batch == 0) return false;
  qd_launch<WN>(m, k, n, a, b, c, (uint32_t)(tiles * batch), st, fast);
  *err = hipGetLastError();
  return true;
}

}  // namespace mi355x
