// Batched arm_fir_q15 on the i8 matrix cores — MI355X, bit-exact.
//
// Replaces the host scalar path of Source/FilteringFunctions/arm_fir_q15.c:458-726 (the
// ARM_MATH_LOOPUNROLL, !ARM_MATH_DSP branch): with s = [history (T - 1) ; block] and the taps in
// the reference's order, y[n] = __SSAT(acc >> 15, 16) where acc is a q63 sum over tap PAIRS of the
// __SMLALD pair sums (int32-wrapped, none.h:497-506) for the unrolled outputs and of exact products
// for the blockSize % 4 tail (:649-681).  A pair sum wraps only for a coefficient pair (-32768,
// -32768) times a sample pair (-32768, -32768); for any other taps both branches are the exact sum
// of products, an integer GEMM, which this kernel runs on v_mfma_i32_32x32x32_i8.  Taps holding
// such a pair take the exact pair-wise VALU path of the same kernel (it needs two consecutive
// coefficients of -32768).
//
// FIR as a GEMM: a block of 32 consecutive outputs n0 .. n0 + 31 is y[n0 + i] = sum_k Tc[i][k]
// w[k] over a window w of the state, with the banded Toeplitz matrix Tc[i][k] = c[k - d - i]
// (0 <= k - d - i < T; d in {0, 1} is the window's start one sample early, so that its source
// words are 4-byte aligned).  32 such blocks (1024 outputs) are one 32 x 32 MFMA tile: MFMA A
// operand = Tc (32 outputs x K), B operand = the 32 blocks' windows (K x 32 blocks, column j =
// w[32 j + k]: consecutive blocks' windows overlap, all read from one staged window in LDS),
// D[i][j] = y[n0 + 32 j + i] -- the accumulator layout gives a lane four consecutive outputs per
// register quad.  K = 32 KS >= T + 32.
//
// Exact i8 planes: samples x = 256 xh + xl' + 128 (xh = x >> 8, xl' = (x & 255) - 128, signed
// bytes); coefficients WITHOUT an offset, c = 2^14 a + 2^7 b + c0 (b, c0 in 0 .. 127, a = c >> 14
// in -2 .. 1, carried as a' = 64 a), so the only correction is the constant 128 sum(c):
//   sum x c = 2^16 (xh.a') + 2^15 (xh.b) + 2^8 (xh.c0 + xl'.a') + 2^7 (xl'.b) + (xl'.c0) + 128 sum c
// six plane products per K step into five int32 accumulators (each exact: |class sum| < 2^24 for
// K <= 192), formed in int64 for the output.  The three coefficient planes of Tc, as the MFMA's A
// operand wants them lane by lane, are built once per call by fir_q15_coef_image_kernel (for both
// window shifts d) and read by every workgroup from L2.
//
// Geometry: persistent workgroups of 4 waves walk the items = (filter, chunk of 4096 outputs); wave
// w takes the 32 blocks of outputs 1024 w .. + 1023.  The window (count + T samples) is staged into
// two LDS byte planes (xh, xl') in 256-B rows whose 16-B slots are XOR-swizzled by the row's parity
// (slot ^ (row & 1)), so the B-operand reads (ds_read_b128, lane j at byte 32 j + 32 ks + 16 h) hit
// 16 distinct slots in every 16-lane group.  The next item's window words are loaded into
// registers while the current item is multiplied.  Round 6: the window is loaded in word pairs
// (one v_perm + one 4-byte LDS write per plane and pair; only the words outside the block input
// take the per-sample path) and the output is formed in int32 (W >> 8 below): 580 -> 601-616
// Gsamples/s.  Measured and not kept (round 6): the window fed by LDS DMA two items
// ahead (625-634, i.e. the register prefetch is not the limit once the diagnostics below are
// summed: without MFMAs 859, without window loads 821, without staging 682), and the K steps'
// operands read one step ahead with inline asm (register spills at three workgroups per CU).
#include "common.hpp"
#include "kernels.hpp"

#ifndef MI355X_FIR_Q15_MFMA_WG     // workgroups per CU the register allocation must allow
#define MI355X_FIR_Q15_MFMA_WG 3
#endif

#ifndef MI355X_FIR_Q15_ALN        // fir_q15 / fast_q15: the 16-B aligned window mode when the shapes allow it
#define MI355X_FIR_Q15_ALN 1
#endif
#ifndef MI355X_FIR_Q7_ALN         // fir_q7: the 16-B aligned window mode when the shapes allow it
#define MI355X_FIR_Q7_ALN 1
#endif
#ifndef MI355X_FIR_Q31_ALN        // fir_q31: the 16-B aligned window mode when the shapes allow it
#define MI355X_FIR_Q31_ALN 1
#endif
#ifndef MI355X_FIR_STAMP
#define MI355X_FIR_STAMP 0
#endif
#ifndef MI355X_FIR_Q15_DIAG        // 1: diagnostic only -- no window loads after the first item (wrong output)
#define MI355X_FIR_Q15_DIAG 0
#endif

namespace mi355x {

#if MI355X_FIR_STAMP   // diagnostic: s_memtime per phase of the first 64 items of workgroups 0-63 (wave 0)
__device__ unsigned long long fir_stamp_buf[64][64][8];
#define FM_STAMP(k, e)                                                                              \
  do {                                                                                              \
    if (blockIdx.x < 64 && tid == 0 && (k) < 64) fir_stamp_buf[blockIdx.x][(k)][(e)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FM_STAMP(k, e) do { } while (0)
#endif

namespace {
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kFmChunk = 4096;                 // outputs per item (4 waves x 32 blocks x 32)
constexpr int kFmMaxKS = 6;                    // K steps: T + 32 <= 192 -> T <= 160
constexpr int kFmWords = (kFmChunk + 32 * kFmMaxKS) / 2;   // window words staged per item (>= count + T + 1 samples)
constexpr int kFmPer2 = kFmWords / 512;                    // word pairs per thread (words 0 .. 512 kFmPer2 - 1)
constexpr int kFmPer1 = (kFmWords - 512 * kFmPer2 + 255) / 256;   // then single words (9 registers in all)
constexpr int kFmPlane = 2 * kFmWords + 256;               // plane bytes (whole rows + look-ahead)

__device__ __forceinline__ int fm_swz(int m) {  // byte m of a plane -> LDS byte (16-B slots XORed by row parity)
  return (m & ~255) | ((((m >> 4) & 15) ^ ((m >> 8) & 1)) << 4) | (m & 15);
}
}  // namespace

// Coefficient planes of Tc for both window shifts d, lane by lane: image[d][ks][plane][lane] = the
// 16 bytes lane L = (i = L & 31, h = L >> 5) passes as the MFMA A operand at K step ks, i.e. the
// plane bytes of c[32 ks + 16 h + e - d - i], e = 0 .. 15 (0 outside the taps).  Also [2] words:
// sum(c) and whether a (-32768, -32768) tap pair is present.
__global__ __launch_bounds__(256) void fir_q15_coef_image_kernel(const int16_t* __restrict__ coeffs, int T, int KS,
                                                                 int d_base, uint4* __restrict__ image, int* __restrict__ info) {
  // one thread per (d, ks, lane): 2 KS x 64 threads, each the three planes' 16 bytes; the last
  // workgroup's first wave also reduces sum(c) and the wrap flag
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < 2 * KS * 64) {
    const int L = g & 63, ks = (g >> 6) % KS, d = (g >> 6) / KS, i = L & 31, h = L >> 5;
    uint32_t w[3][4] = {};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ci = 32 * ks + 16 * h + e - (d_base + d) - i;   // slot d holds window shift d_base + d
      const int32_t c = (ci >= 0 && ci < T) ? coeffs[ci] : 0;
      w[0][e >> 2] |= (uint32_t)(uint8_t)(int8_t)(64 * (c >> 14)) << (8 * (e & 3));
      w[1][e >> 2] |= (uint32_t)((c >> 7) & 127) << (8 * (e & 3));
      w[2][e >> 2] |= (uint32_t)(c & 127) << (8 * (e & 3));
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) image[((d * KS + ks) * 3 + p) * 64 + L] = make_uint4(w[p][0], w[p][1], w[p][2], w[p][3]);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x < 64) {
    int sum = 0, wrap = 0;
    for (int k = threadIdx.x; k < T; k += 64) sum += coeffs[k];
    for (int m = 2 * threadIdx.x; m + 1 < T; m += 128) wrap |= coeffs[m] == -32768 && coeffs[m + 1] == -32768;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      sum += __shfl_xor(sum, o);
      wrap |= __shfl_xor(wrap, o);
    }
    if (threadIdx.x == 0) {
      info[0] = sum;
      info[1] = wrap;
    }
  }
}

// Exact pair-wise path for taps holding a (-32768, -32768) pair (arm_fir_q15.c:482-640 unrolled
// outputs with the __SMLALD pair wrap, :649-681 tail outputs with exact products), from the planes.
__device__ __forceinline__ void fm_wrap_item(const uint8_t* ph, const uint8_t* pl, const int16_t* __restrict__ coeffs, int T,
                                          uint32_t B, int n0, int d, int count, int tid, int16_t* __restrict__ yf) {
  const int unrolled_end = (int)(B - (B & 3u));
  auto xs = [&](int m) -> int32_t {
    const int a = fm_swz(m);
    return (int32_t)(int16_t)(uint16_t)(((uint32_t)ph[a] << 8) | (uint32_t)(pl[a] ^ 0x80u));
  };
  for (int o = tid; o < count; o += 256) {
    const int n = n0 + o, m0 = o + d;                  // y[n] = sum_t s[n + t] c[t] = sum_t w[o + d + t] c[t]
    int64_t acc = 0;
    for (int m = 0; m < T / 2; ++m) {
      const int64_t p0 = (int64_t)xs(m0 + 2 * m) * coeffs[2 * m], p1 = (int64_t)xs(m0 + 2 * m + 1) * coeffs[2 * m + 1];
      acc += n < unrolled_end ? (int64_t)(int32_t)(uint32_t)(uint64_t)(p0 + p1) : p0 + p1;
    }
    yf[n] = (int16_t)ssat16((int32_t)(acc >> 15));
  }
}

template <int KS, bool FAST>
__device__ __forceinline__ void fm_tile_y(const uint4* __restrict__ imgd, const uint8_t* ph, const uint8_t* pl, int wid,
                                          int L, int32_t sumc, uint32_t (&y)[8]) {
  const int i = L & 31, h = L >> 5;
  const uint4* img = imgd + L;
  i32x16 a16 = {}, a15 = {}, a8 = {}, a7 = {}, a0 = {};
  const int mb = 1024 * wid + 32 * i + 16 * h;        // window byte of this lane at ks = 0 (column j = i)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const uint4 ua = img[(ks * 3 + 0) * 64], ub = img[(ks * 3 + 1) * 64], uc = img[(ks * 3 + 2) * 64];
    const i32x4 ca = i32x4{(int)ua.x, (int)ua.y, (int)ua.z, (int)ua.w};
    const i32x4 cb = i32x4{(int)ub.x, (int)ub.y, (int)ub.z, (int)ub.w};
    const i32x4 cc = i32x4{(int)uc.x, (int)uc.y, (int)uc.z, (int)uc.w};
    const int a = fm_swz(mb + 32 * ks);
    const i32x4 xh = *reinterpret_cast<const i32x4*>(ph + a);
    const i32x4 xl = *reinterpret_cast<const i32x4*>(pl + a);
    a16 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ca, xh, a16, 0, 0, 0);
    a15 = __builtin_amdgcn_mfma_i32_32x32x32_i8(cb, xh, a15, 0, 0, 0);
    a8 = __builtin_amdgcn_mfma_i32_32x32x32_i8(cc, xh, a8, 0, 0, 0);
    a8 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ca, xl, a8, 0, 0, 0);
    a7 = __builtin_amdgcn_mfma_i32_32x32x32_i8(cb, xl, a7, 0, 0, 0);
    a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(cc, xl, a0, 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    // S = 2^15 X + R, X = 2 a16 + a15, R = 2^7 Y + a0 + 2^7 sum c, Y = 2 a8 + a7; with
    // W = Y + sum c + (a0 >> 7): R = 2^7 W + (a0 & 127), so R >> 15 = W >> 8 (floor division),
    // every term int32 (|Y| < 2^26, |sum c| < 2^23)
    const int32_t X = 2 * a16[g] + a15[g];
    uint32_t v;
    if constexpr (FAST) {
      // arm_fir_fast_q15: the q31_t accumulator wraps mod 2^32 (every __SMLAD and tail product),
      // so the exact sum's low word is the reference's accumulator: S mod 2^32 in uint32 arithmetic
      const uint32_t S = ((uint32_t)X << 15) + ((uint32_t)(2 * a8[g] + a7[g]) << 7) + (uint32_t)a0[g] +
                         ((uint32_t)sumc << 7);
      v = (uint16_t)(int16_t)ssat16((int32_t)S >> 15);
    } else {
      const int32_t W = 2 * a8[g] + a7[g] + sumc + (a0[g] >> 7);
      v = (uint16_t)(int16_t)ssat16(X + (W >> 8));
    }
    y[g >> 1] = (g & 1) ? (y[g >> 1] | (v << 16)) : v;
  }
}

// lane (j = L & 31, h), register 4q + e -> output 8q + 4h + e of block j.  A whole tile goes out
// through the wave's 2 KiB LDS slot otw: each lane writes its four 8-B pieces (16-B chunk c = 4 j + q
// of the tile, half h), then reads chunks L and 64 + L back, so each global store instruction
// writes 1 KiB of consecutive outputs -- stored straight from the accumulator layout, every lane
// wrote 8 B into its own 64-B segment and the store phase took ~1,100 of an item's ~6,900 ticks
// (tools/probes/fir_stamps.hip).  Chunks are XOR-swizzled (c ^ ((c >> 4) & 3)) so that the writes
// spread over the 16 four-bank groups.
__device__ __forceinline__ int fm_ochunk(int c) { return c ^ ((c >> 4) & 3); }
__device__ __forceinline__ void fm_tile_store(const uint32_t (&y)[8], int wid, int L, int count,
                                              int16_t* __restrict__ yrow, uint4* otw) {
  const int j = L & 31, h = L >> 5;
  if (count == kFmChunk && ((((uintptr_t)yrow) & 15) == 0)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) reinterpret_cast<uint2*>(otw + fm_ochunk(4 * j + q))[h] = make_uint2(y[2 * q], y[2 * q + 1]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = 64 * r + L;
      *reinterpret_cast<uint4*>(yrow + 1024 * wid + 8 * c) = otw[fm_ochunk(c)];
    }
  } else {
    int16_t* yb = yrow + 1024 * wid + 32 * j + 4 * h;
    const int ob = 1024 * wid + 32 * j + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (ob + 8 * q + e < count) yb[8 * q + e] = (int16_t)(y[2 * q + (e >> 1)] >> (16 * (e & 1)));
  }
}

// FAST: arm_fir_fast_q15 (arm_fir_fast_q15.c: the same products summed in a wrapping q31_t, no
// pair-wrap special case since everything is mod 2^32)
// ALN: blockSize % 8 == 0 and 16-B aligned data -- every window starts d_base = (-T1) mod 8 samples early,
// so its history / block regions begin on 16-B boundaries and it is loaded as three dwordx4 per
// thread instead of nine dword loads (the image's slot 0 is that shift).
template <int KS, bool FAST, bool ALN>
__global__ __launch_bounds__(256, MI355X_FIR_Q15_MFMA_WG) void fir_q15_mfma_kernel(const int16_t* __restrict__ coeffs, int T, int d_base,
                                                              const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                              uint32_t B, const int16_t* __restrict__ hist,
                                                              uint32_t nchunks, uint32_t items,
                                                              const uint4* __restrict__ image,
                                                              const int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) uint8_t ph[kFmPlane];
  __shared__ __attribute__((aligned(16))) uint8_t pl[kFmPlane];
  __shared__ __attribute__((aligned(16))) uint4 imgl[2 * KS * 3 * 64];   // the coefficient image, once per workgroup
  __shared__ uint32_t hd[256];                           // head samples (and [192]: the tail sample) of the next window
  __shared__ __attribute__((aligned(16))) uint4 ot[4][128];   // per wave: the output tile on its way out
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T1 = T - 1;
  const bool wrap = !FAST && info[1] != 0;
  const int32_t sumc = info[0];                          // |sum c| <= 160 * 2^15
  for (int u = tid; u < 2 * KS * 3 * 64; u += 256) imgl[u] = image[u];   // visible after the loop's first barrier

  // window word u (samples 2u, 2u + 1 of w) of item `it`, w[m] = s[n0 - d + m], d = parity of the
  // block-input offset so that the words of the block input are 4-byte aligned
  struct Item { uint32_t f; int n0, count, d; };
  auto item_of = [&](uint32_t it) {
    Item x;
    x.f = it / nchunks;
    x.n0 = (int)(it - x.f * nchunks) * kFmChunk;
    x.count = min((int)B - x.n0, kFmChunk);
    x.d = ALN ? d_base : (int)(((uint64_t)x.f * B + (uint32_t)x.n0 - (uint32_t)T1) & 1u);   // s index n0 - d + m -> src f B + n0 - d + m - T1
    return x;
  };
  // Window words in PAIRS: thread tid takes words 2 (tid + 256 q) and + 1 (4 samples, one 4-byte
  // write per plane), then single words 512 kFmPer2 + tid + 256 q.
  // Window words: every word is loaded as one aligned dword from a CLAMPED block-input address with no
  // branch and no select, so nothing in the load phase waits for a load (a per-lane "block word or
  // per-sample path" select put the wave behind its own loads -- the result register's join made
  // the compiler wait there; phase stamps, tools/probes/fir_stamps.hip, had the load phase at 53 % of
  // an item).  The words before u_lo (a filter's first item: the history) come from per-sample head
  // samples and a block ending mid-word (odd blockSize) from the tail sample, both landed in LDS by
  // DMA; they are combined when the window is staged.
  struct Win { int u_lo, u_hi; bool straddle; };
  auto win_of = [&](const Item& x) {
    Win w;
    const int lo_num = T1 - x.n0 + x.d, hi_num = T1 + (int)B - 2 - x.n0 + x.d;
    w.u_lo = lo_num > 0 ? (lo_num + 1) >> 1 : 0;
    w.u_hi = hi_num >= 0 ? (hi_num >> 1) + 1 : 0;
    w.straddle = x.n0 - x.d + 2 * w.u_hi == T1 + (int)B - 1 && w.u_hi < kFmWords;   // word u_hi = (last sample, 0)
    return w;
  };
  uint32_t wv[ALN ? 12 : 2 * kFmPer2 + kFmPer1];
  auto aln_bounds = [&](const Item& x, int& m_lo, int& m_hi) {   // block samples of the window (multiples of 8)
    m_lo = max(T1 - x.n0 + x.d, 0);
    m_hi = min(T1 + (int)B - x.n0 + x.d, 2 * kFmWords);
  };
  auto load_window = [&](const Item& x) {
    const Win w = win_of(x);
    const int64_t base = (int64_t)x.f * B + x.n0 - x.d - T1;               // src index of w[0] (even)
    if constexpr (ALN) {
      int m_lo, m_hi;
      aln_bounds(x, m_lo, m_hi);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int m = min(max(8 * (tid + 256 * q), m_lo), m_hi - 8);
        const uint4 v = *reinterpret_cast<const uint4*>(src + base + m);
        wv[4 * q] = v.x;
        wv[4 * q + 1] = v.y;
        wv[4 * q + 2] = v.z;
        wv[4 * q + 3] = v.w;
      }
    } else {
    auto word = [&](int u) -> uint32_t {
      const int uc = min(max(u, w.u_lo), w.u_hi - 1);
      return *reinterpret_cast<const uint32_t*>(src + base + 2 * uc);
    };
#pragma unroll
    for (int q = 0; q < kFmPer2; ++q) {
#pragma unroll
      for (int e = 0; e < 2; ++e) wv[2 * q + e] = word(2 * (tid + 256 * q) + e);
    }
#pragma unroll
    for (int q = 0; q < kFmPer1; ++q) wv[2 * kFmPer2 + q] = word(min(512 * kFmPer2 + tid + 256 * q, kFmWords - 1));
    }
    // The head samples and the tail sample go to LDS by DMA (one zero-extended dword per lane,
    // tools/probes/lds_dma_sub.hip): waves 0-2 samples 64 w + lane, wave 3 the block's last sample.
    // No register receives them, so nothing here waits; barrier A's vmcnt(0) lands them.
    {
      const int j = x.n0 - x.d + 64 * wid + L;            // state index (2 u_lo <= T1 + 2 <= 161 samples)
      const bool in_h = j >= 0 && j < T1;
      const uint64_t ph_ = (uint64_t)(uintptr_t)(hist + (uint64_t)x.f * T1 + (in_h ? j : 0));
      const uint64_t pb_ = (uint64_t)(uintptr_t)(src + (uint64_t)x.f * B + (wid == 3 ? (int)B - 1 : min(max(j - T1, 0), (int)B - 1)));
      const uint64_t pa = (wid < 3 && in_h) ? ph_ : pb_;
      __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)pa, (__attribute__((address_space(3))) void*)(hd + 64 * wid),
                                       2, 0, 0);
    }
  };
  auto stage_window_aln = [&](const Item& x) {           // ALN: 8 samples -> 8 bytes per plane
    int m_lo, m_hi;
    aln_bounds(x, m_lo, m_hi);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int m0 = 8 * (tid + 256 * q);
      if (m0 >= 2 * kFmWords) continue;
      uint32_t w4[4];
      if (m0 < m_lo) {                                   // history head (wave 0): the DMA'd samples, 0 before the state
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int m = m0 + 2 * k;
          const uint32_t s0 = x.n0 - x.d + m >= 0 ? hd[m] : 0u, s1 = x.n0 - x.d + m + 1 >= 0 ? hd[m + 1] : 0u;
          w4[k] = s0 | (s1 << 16);
        }
      } else if (m0 < m_hi) {
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = wv[4 * q + k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = 0u;
      }
      const uint32_t h0 = __builtin_amdgcn_perm(w4[1], w4[0], 0x07050301u), h1 = __builtin_amdgcn_perm(w4[3], w4[2], 0x07050301u);
      const uint32_t l0 = __builtin_amdgcn_perm(w4[1], w4[0], 0x06040200u) ^ 0x80808080u;
      const uint32_t l1 = __builtin_amdgcn_perm(w4[3], w4[2], 0x06040200u) ^ 0x80808080u;
      const int a = fm_swz(m0);
      *reinterpret_cast<uint2*>(ph + a) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(pl + a) = make_uint2(l0, l1);
    }
  };
  auto stage_window = [&](const Item& x) {               // registers -> the two byte planes
    const Win w = win_of(x);
    auto val = [&](int u, uint32_t v) -> uint32_t {      // word u from its block load, the tail, or 0
      return u < w.u_hi ? v : (u == w.u_hi && w.straddle ? hd[192] : 0u);
    };
#pragma unroll
    for (int q = 0; q < kFmPer1; ++q) {
      const int u = 512 * kFmPer2 + tid + 256 * q;
      if (u >= kFmWords) continue;
      const uint32_t v = val(u, wv[2 * kFmPer2 + q]);
      const int a = fm_swz(2 * u);
      *reinterpret_cast<uint16_t*>(ph + a) = (uint16_t)(((v >> 8) & 0xFFu) | ((v >> 16) & 0xFF00u));
      *reinterpret_cast<uint16_t*>(pl + a) = (uint16_t)(((v & 0xFFu) | ((v >> 8) & 0xFF00u)) ^ 0x8080u);
    }
#pragma unroll
    for (int q = 0; q < kFmPer2; ++q) {
      const int u = 2 * (tid + 256 * q);
      uint32_t v0 = val(u, wv[2 * q]), v1 = val(u + 1, wv[2 * q + 1]);
      if (q == 0 && u < w.u_lo) {                        // head words: the per-sample loads (0 before the state)
        uint32_t hs[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) hs[e] = x.n0 - x.d + 4 * tid + e >= 0 ? hd[4 * tid + e] : 0u;   // j < T1 + B here
        v0 = hs[0] | (hs[1] << 16);
        if (u + 1 < w.u_lo) v1 = hs[2] | (hs[3] << 16);
      }
      const uint32_t hi = __builtin_amdgcn_perm(v1, v0, 0x07050301u);               // x >> 8 per sample
      const uint32_t lo = __builtin_amdgcn_perm(v1, v0, 0x06040200u) ^ 0x80808080u;  // (x & 255) - 128
      const int a = fm_swz(2 * u);
      *reinterpret_cast<uint32_t*>(ph + a) = hi;
      *reinterpret_cast<uint32_t*>(pl + a) = lo;
    }
  };

  uint32_t it = blockIdx.x;
  if (it >= items) return;
  Item cur = item_of(it);
  load_window(cur);
  for (int kk = 0;; ++kk) {
    FM_STAMP(kk, 0);
    __syncthreads();                                     // the previous item's reads are done
    FM_STAMP(kk, 1);
    if constexpr (ALN) stage_window_aln(cur); else stage_window(cur);
    FM_STAMP(kk, 2);
    __syncthreads();
    FM_STAMP(kk, 3);
    const uint32_t nxt = it + gridDim.x;
    const Item next = item_of(nxt < items ? nxt : it);
    if (nxt < items && !MI355X_FIR_Q15_DIAG) load_window(next);   // in flight under this item's MFMAs
    FM_STAMP(kk, 4);

    if (wrap) {
      fm_wrap_item(ph, pl, coeffs, T, B, cur.n0, cur.d, cur.count, tid, dst + (uint64_t)cur.f * B);
    } else if (1024 * wid < cur.count) {
      uint32_t y[8];
      fm_tile_y<KS, FAST>(imgl + (cur.d - d_base) * KS * 3 * 64, ph, pl, wid, L, sumc, y);
      FM_STAMP(kk, 5);
      fm_tile_store(y, wid, L, cur.count, dst + (uint64_t)cur.f * B + cur.n0, ot[wid]);
      FM_STAMP(kk, 6);
    }
    if (nxt >= items) break;
    it = nxt;
    cur = next;
  }
}

// true: launched (numTaps even, 2 .. 160, enough work to fill the chip); false: not this path
bool fir_q15_mfma_launch(const int16_t* coeffs, int T, const int16_t* src, int16_t* dst, uint32_t B,
                         uint32_t batch, const int16_t* hist_in, hipStream_t st, bool fast) {
  if (!(fast ? MI355X_FIR_FAST_Q15_MFMA : MI355X_FIR_Q15_MFMA) || T < 2 || (T & 1) || T > 32 * kFmMaxKS - 32 || B < 64 ||
      batch == 0)
    return false;
  const uint32_t nchunks = (B + kFmChunk - 1) / kFmChunk;
  const uint64_t items = (uint64_t)nchunks * batch;
  if (items < 256 || items > 0x7fffffffull) return false;
  const int ks = (T + 32 + 31) / 32;
  // aligned mode: shift d8 = (-T1) mod 8 when blockSize % 8 == 0, the data is 16-B aligned and the
  // shift costs no K step (K >= numTaps - 1 + d8 + 31 + 1)
  const int d8 = (8 - (T - 1) % 8) % 8;
  const bool aln = MI355X_FIR_Q15_ALN && B % 8 == 0 && ((uintptr_t)src & 15) == 0 && (T + d8 + 31 + 31) / 32 <= ks;
  const int d_base = aln ? d8 : 0;
  // the coefficient image (2 shifts x KS steps x 3 planes x 64 lanes x 16 B) and [sum, wrap]
  const size_t img_bytes = (size_t)2 * ks * 3 * 64 * 16;
  void* buf = nullptr;
  if (hipMallocAsync(&buf, img_bytes + 16, st) != hipSuccess) return false;
  uint4* img = (uint4*)buf;
  int* info = (int*)((char*)buf + img_bytes);
  hipLaunchKernelGGL(fir_q15_coef_image_kernel, dim3((2 * ks * 64 + 255) / 256), dim3(256), 0, st, coeffs, T, ks, d_base,
                     img, info);
#define FM_CASE(K)                                                                                              \
  case K: {                                                                                                     \
    auto kern = fast ? (aln ? fir_q15_mfma_kernel<K, true, true> : fir_q15_mfma_kernel<K, true, false>)          \
                     : (aln ? fir_q15_mfma_kernel<K, false, true> : fir_q15_mfma_kernel<K, false, false>);      \
    const int g = persistent_grid((const void*)kern, 256, 0, items);                                            \
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, st, coeffs, T, d_base, src, dst, B, hist_in, nchunks,      \
                       (uint32_t)items, (const uint4*)img, (const int*)info);                                   \
    break;                                                                                                      \
  }
  switch (ks) {
    FM_CASE(2)
    FM_CASE(3)
    FM_CASE(4)
    FM_CASE(5)
    FM_CASE(6)
    default:
      (void)hipFreeAsync(buf, st);
      return false;
  }
#undef FM_CASE
  (void)hipFreeAsync(buf, st);
  return true;
}

// =============================================================================================
// Batched arm_fir_q31 on the i8 matrix cores (round 6), bit-exact.  Replaces the scalar path of
// Source/FilteringFunctions/arm_fir_q31.c (the q63 accumulator of exact q31 x q31 products,
// y = (q31)(acc >> 31), :880-1000 LOOPUNROLL and tail alike): acc wraps mod 2^64 in the reference
// build and y keeps its bits 31 .. 62, so any exact sum order gives the reference's words.
//
// Same banded-Toeplitz GEMM as the q15 kernel (d = 0: q31 samples are 4-byte words), with four
// byte planes per operand:
//   samples  x = 2^24 x3 + 2^16 x2' + 2^8 x1' + x0' + beta, xi' = byte i - 128 (i < 3), x3 the
//            signed top byte, beta = 128 (2^16 + 2^8 + 1);
//   taps     c' = 2^24 d3 + 2^16 d2 + 2^8 d1 + d0, balanced signed digits (each -128 .. 127), which
//            covers c' in [-2^31, 0x7F7F7F7F]; a tap above that ("big", within 2^-7.98 of +1.0) is
//            carried as c' = c - 2^31, and 2^31 x (the difference) adds exactly x to y = S >> 31.
// sum_t x c = sum_{i,j} 2^{8 (i + j)} (x_i' . d_j) + beta sum c'  (+ 2^31 sum over big taps of x):
// 16 plane products per K step into seven int32 accumulators by shift class i + j (each exact:
// at most 4 products of |.| <= 128 x 128 x 192), combined in int64 mod 2^64 for the output.
// Up to kQ31MaxBig big taps are corrected per output from the planes; more take an exact
// per-output VALU path in the same kernel.
constexpr int kQ31Words = kFmChunk + 32 * kFmMaxKS;            // window samples staged per item (4288)
constexpr int kQ31Groups = (kQ31Words + 1023) / 1024;          // 4-sample groups per thread
constexpr int kQ31Plane = kQ31Words + 256;                     // plane bytes (whole rows + look-ahead)
constexpr int kQ31MaxBig = 4;
constexpr int64_t kQ31Beta = 128 * (65536 + 256 + 1);

__device__ __forceinline__ int64_t q31_tap_carried(int32_t c) {   // c' of the tap
  return c > 0x7F7F7F7F ? (int64_t)c - (int64_t)0x80000000LL : (int64_t)c;
}

// image[ks][digit][lane]: the 16 digit bytes lane L = (i = L & 31, h = L >> 5) passes as the A operand
// at K step ks (taps c'[32 ks + 16 h + e - i]); info: [0, 1] sum c' (int64), [2] number of big taps,
// [3 ..] their indices (first kQ31MaxBig)
__global__ __launch_bounds__(256) void fir_q31_coef_image_kernel(const int32_t* __restrict__ coeffs, int T, int KS, int d,
                                                                 uint4* __restrict__ image, int* __restrict__ info) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < KS * 64) {
    const int L = g & 63, ks = g >> 6, i = L & 31, h = L >> 5;
    uint32_t w[4][4] = {};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ci = 32 * ks + 16 * h + e - d - i;      // window shifted d samples early (aligned mode)
      int64_t v = (ci >= 0 && ci < T) ? q31_tap_carried(coeffs[ci]) : 0;
#pragma unroll
      for (int dgt = 0; dgt < 4; ++dgt) {
        const int64_t dd = dgt < 3 ? ((v + 128) & 255) - 128 : v;   // balanced digit
        v = (v - dd) >> 8;
        w[dgt][e >> 2] |= (uint32_t)(uint8_t)(int8_t)dd << (8 * (e & 3));
      }
    }
#pragma unroll
    for (int dgt = 0; dgt < 4; ++dgt) image[(ks * 4 + dgt) * 64 + L] = make_uint4(w[dgt][0], w[dgt][1], w[dgt][2], w[dgt][3]);
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x < 64) {   // one wave: sum c' and the big taps in order
    const int l = threadIdx.x;
    int64_t sum = 0;
    int nbig = 0;
    for (int k0 = 0; k0 < T; k0 += 64) {
      const int k = k0 + l;
      const int32_t c = k < T ? coeffs[k] : 0;
      sum += q31_tap_carried(c);
      const bool big = c > 0x7F7F7F7F;
      const uint64_t mask = __ballot(big);
      if (big) {
        const int r = nbig + __popcll(mask & ((1ull << l) - 1));
        if (r < kQ31MaxBig) info[3 + r] = k;
      }
      nbig += __popcll(mask);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if (l == 0) {
      info[0] = (int)(uint32_t)(uint64_t)sum;
      info[1] = (int)(uint32_t)((uint64_t)sum >> 32);
      info[2] = nbig;
    }
  }
}

// ALN: blockSize % 4 == 0 and 16-B aligned data -- the window starts d = (-T1) mod 4 samples early so
// that its history / block / tail regions all begin on 16-B boundaries, and it is loaded as dwordx4
// (five instructions per thread and item instead of twenty dword loads: vector-memory instruction
// issue, ~40-100 cycles each under this load, was a large share of an item; MI355X_MICROARCH.md).
template <int KS, bool ALN>
__global__ __launch_bounds__(256, 2) void fir_q31_mfma_kernel(const int32_t* __restrict__ coeffs, int T, int d,
                                                              const int32_t* __restrict__ src, int32_t* __restrict__ dst,
                                                              uint32_t B, const int32_t* __restrict__ hist,
                                                              uint32_t nchunks, uint32_t items,
                                                              const uint4* __restrict__ image,
                                                              const int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) uint8_t pq[4][kQ31Plane];
  __shared__ __attribute__((aligned(16))) uint4 imgl[KS * 4 * 64];
  __shared__ uint32_t hd[192];                           // the next window's history head (DMA)
  __shared__ __attribute__((aligned(16))) uint4 ot[4][256];   // per wave: the output tile on its way out
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T1 = T - 1;
  const uint64_t k0 = (uint64_t)kQ31Beta * ((uint64_t)(uint32_t)info[0] | ((uint64_t)(uint32_t)info[1] << 32));
  const int nbig = info[2];
  int big[kQ31MaxBig];
#pragma unroll
  for (int b = 0; b < kQ31MaxBig; ++b) big[b] = b < nbig ? info[3 + b] : 0;
  for (int u = tid; u < KS * 4 * 64; u += 256) imgl[u] = image[u];   // visible after the loop's first barrier

  struct Item { uint32_t f; int n0, count; };
  auto item_of = [&](uint32_t it) {
    Item x;
    x.f = it / nchunks;
    x.n0 = (int)(it - x.f * nchunks) * kFmChunk;
    x.count = min((int)B - x.n0, kFmChunk);
    return x;
  };
  // window sample m = s[n0 + m] (state = [history T1 ; block B], 0 past it): thread tid takes the
  // four samples 4 (tid + 256 q) + e, each one aligned dword from a clamped, always-valid address
  // Window samples m = 4 (tid + 256 q) + e: one dword each from a CLAMPED block-input index with no
  // branch (as in the q15 kernel: a per-lane select between the block load and a per-sample path
  // made the wave wait for its own loads); the history head of a filter's first item (m < T1 - n0 <=
  // 160, wave 0's first group) lands in LDS by DMA from waves 0-2 and is merged at staging.
  uint32_t wv[4 * kQ31Groups];
  auto load_window = [&](const Item& x) {
    const int m_lo = max(T1 - x.n0 + d, 0), m_hi = min(T1 + (int)B - x.n0 + d, kQ31Words);   // block samples [m_lo, m_hi)
    const int32_t* blk = src + ((int64_t)x.f * B + x.n0 - d - T1);  // window sample m of the block input: blk[m]
#pragma unroll
    for (int q = 0; q < kQ31Groups; ++q) {
      if constexpr (ALN) {                                 // m_lo, m_hi, blk: multiples of 4 samples / 16 B
        const int m = min(max(4 * (tid + 256 * q), m_lo), m_hi - 4);
        const uint4 v = *reinterpret_cast<const uint4*>(blk + m);
        wv[4 * q] = v.x;
        wv[4 * q + 1] = v.y;
        wv[4 * q + 2] = v.z;
        wv[4 * q + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = min(max(4 * (tid + 256 * q) + e, m_lo), m_hi - 1);
          wv[4 * q + e] = (uint32_t)blk[m];
        }
      }
    }
    const int j = x.n0 - d + 64 * wid + L;                 // head sample 64 w + lane (waves 0-2)
    // (numTaps 1: no history at all -- any valid address, never read)
    const int32_t* hp = T1 > 0 ? hist + (uint64_t)x.f * T1 + min(max(j, 0), T1 - 1) : src + (uint64_t)x.f * B;
    if (wid < 3)
      __builtin_amdgcn_global_load_lds((const void*)hp, (__attribute__((address_space(3))) void*)(hd + 64 * wid), 4, 0, 0);
  };
  auto stage_window = [&](const Item& x) {               // 4 samples -> one 4-byte word per plane
    const int m_lo = max(T1 - x.n0 + d, 0), m_hi = min(T1 + (int)B - x.n0 + d, kQ31Words);
#pragma unroll
    for (int q = 0; q < kQ31Groups; ++q) {
      const int m = 4 * (tid + 256 * q);
      if (m >= kQ31Words) continue;
      uint32_t sv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int me = m + e;                            // head: 0 before the state (j < 0)
        sv[e] = me < m_lo ? (q == 0 && me >= d - x.n0 ? hd[me] : 0u) : (me < m_hi ? wv[4 * q + e] : 0u);
      }
      const uint32_t s0 = sv[0], s1 = sv[1], s2 = sv[2], s3 = sv[3];
      const uint32_t u01 = __builtin_amdgcn_perm(s1, s0, 0x05010400u), u23 = __builtin_amdgcn_perm(s3, s2, 0x05010400u);
      const uint32_t v01 = __builtin_amdgcn_perm(s1, s0, 0x07030602u), v23 = __builtin_amdgcn_perm(s3, s2, 0x07030602u);
      const int a = fm_swz(m);
      *reinterpret_cast<uint32_t*>(&pq[0][a]) = __builtin_amdgcn_perm(u23, u01, 0x05040100u) ^ 0x80808080u;
      *reinterpret_cast<uint32_t*>(&pq[1][a]) = __builtin_amdgcn_perm(u23, u01, 0x07060302u) ^ 0x80808080u;
      *reinterpret_cast<uint32_t*>(&pq[2][a]) = __builtin_amdgcn_perm(v23, v01, 0x05040100u) ^ 0x80808080u;
      *reinterpret_cast<uint32_t*>(&pq[3][a]) = __builtin_amdgcn_perm(v23, v01, 0x07060302u);
    }
  };
  auto xs = [&](int m) -> int32_t {                      // window sample m from the planes
    const int a = fm_swz(m);
    return (int32_t)(((uint32_t)pq[3][a] << 24) | ((uint32_t)(pq[2][a] ^ 0x80u) << 16) |
                     ((uint32_t)(pq[1][a] ^ 0x80u) << 8) | (uint32_t)(pq[0][a] ^ 0x80u));
  };

  uint32_t it = blockIdx.x;
  if (it >= items) return;
  Item cur = item_of(it);
  load_window(cur);
  for (;;) {
    __syncthreads();                                     // the previous item's reads (and the head DMA's landing)
    stage_window(cur);
    __syncthreads();
    const uint32_t nxt = it + gridDim.x;
    const Item next = item_of(nxt < items ? nxt : it);
    if (nxt < items) load_window(next);                  // in flight under this item's MFMAs
    int32_t* yf = dst + (uint64_t)cur.f * B + cur.n0;
    if (nbig > kQ31MaxBig) {
      // exact per-output path (arm_fir_q31.c: q63 sum of exact products, y = acc >> 31)
      for (int o = tid; o < cur.count; o += 256) {
        uint64_t acc = 0;
        for (int t = 0; t < T; ++t) acc += (uint64_t)((int64_t)xs(o + d + t) * coeffs[t]);
        yf[o] = (int32_t)(uint32_t)(acc >> 31);
      }
    } else if (1024 * wid < cur.count) {
      const int i = L & 31, h = L >> 5;
      const uint4* img = imgl + L;
      i32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {};
      const int mb = 1024 * wid + 32 * i + 16 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        i32x4 D[4], P[4];
        const int a = fm_swz(mb + 32 * ks);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint4 u = img[(ks * 4 + r) * 64];
          D[r] = i32x4{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
          P[r] = *reinterpret_cast<const i32x4*>(&pq[r][a]);
        }
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[0], P[3], c3, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[0], P[2], c2, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[1], P[3], c4, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[0], P[1], c1, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[1], P[2], c3, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[2], P[3], c5, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[1], P[1], c2, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[0], P[0], c0, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[2], P[2], c4, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[2], P[1], c3, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[1], P[0], c1, 0, 0, 0);
        c6 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[3], P[3], c6, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[2], P[0], c2, 0, 0, 0);
        c5 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[3], P[2], c5, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[3], P[1], c4, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(D[3], P[0], c3, 0, 0, 0);
      }
      // lane (j = L & 31, h), register 4q + e -> output 8q + 4h + e of block j
      const int j = L & 31;
      const int ob = 1024 * wid + 32 * j + 4 * h;
      int32_t y[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        // S = sum_s 2^{8 s} c_s + beta sum c' (mod 2^64, Horner in int64); y = bits 31 .. 62
        uint64_t S = (uint64_t)(int64_t)c6[g];
        S = (S << 8) + (uint64_t)(int64_t)c5[g];
        S = (S << 8) + (uint64_t)(int64_t)c4[g];
        S = (S << 8) + (uint64_t)(int64_t)c3[g];
        S = (S << 8) + (uint64_t)(int64_t)c2[g];
        S = (S << 8) + (uint64_t)(int64_t)c1[g];
        S = (S << 8) + (uint64_t)(int64_t)c0[g];
        y[g] = (int32_t)(uint32_t)((S + k0) >> 31);
      }
      if (nbig) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int o = ob + 8 * (g >> 2) + (g & 3);
          for (int b = 0; b < nbig; ++b) y[g] += xs(o + d + big[b]);   // mod 2^32, as the reference's (q31_t) cast
        }
      }
      int32_t* yb = yf + ob;
      if (cur.count == kFmChunk && ((((uintptr_t)yf) & 15) == 0)) {
        // through the wave's 4 KiB LDS slot (16-B chunk c = 8 j + 2 q + h, XOR-swizzled), then four
        // coalesced 1 KiB stores
        uint4* otw = ot[wid];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 8 * j + 2 * q + h;
          otw[c ^ ((c >> 4) & 7)] = make_uint4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 64 * r + L;
          *reinterpret_cast<uint4*>(yf + 1024 * wid + 4 * c) = otw[c ^ ((c >> 4) & 7)];
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ob + 8 * q + e < cur.count) yb[8 * q + e] = y[4 * q + e];
      }
    }
    if (nxt >= items) break;
    it = nxt;
    cur = next;
  }
}

// true: launched (numTaps 1 .. 161, enough work to fill the chip); false: not this path
bool fir_q31_mfma_launch(const int32_t* coeffs, int T, const int32_t* src, int32_t* dst, uint32_t B,
                         uint32_t batch, const int32_t* hist_in, hipStream_t st) {
  if (!MI355X_FIR_Q31_MFMA || T < 1 || T > 32 * kFmMaxKS - 31 || B == 0 || batch == 0) return false;
  const uint32_t nchunks = (B + kFmChunk - 1) / kFmChunk;
  const uint64_t items = (uint64_t)nchunks * batch;
  if (items < 256 || items > 0x7fffffffull) return false;
  const int ks = (T + 31 + 31) / 32;
  // aligned mode: the shift d = (-T1) mod 4 puts every region of every window on a 16-B boundary;
  // taken when blockSize % 4 == 0, the pointers are 16-B aligned and the shift costs no K step
  const int d4 = (4 - (T - 1) % 4) % 4;
  const bool aln = MI355X_FIR_Q31_ALN && B % 4 == 0 && ((uintptr_t)src & 15) == 0 && (T + 31 + d4 + 31) / 32 == ks;
  const int d = aln ? d4 : 0;
  const size_t img_bytes = (size_t)ks * 4 * 64 * 16;
  void* buf = nullptr;
  if (hipMallocAsync(&buf, img_bytes + 32, st) != hipSuccess) return false;
  uint4* img = (uint4*)buf;
  int* info = (int*)((char*)buf + img_bytes);
  hipLaunchKernelGGL(fir_q31_coef_image_kernel, dim3((ks * 64 + 255) / 256), dim3(256), 0, st, coeffs, T, ks, d, img, info);
#define FQ_CASE(K)                                                                                              \
  case K: {                                                                                                     \
    auto kern = aln ? fir_q31_mfma_kernel<K, true> : fir_q31_mfma_kernel<K, false>;                             \
    const int g = persistent_grid((const void*)kern, 256, 0, items);                                            \
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, st, coeffs, T, d, src, dst, B, hist_in, nchunks,            \
                       (uint32_t)items, (const uint4*)img, (const int*)info);                                   \
    break;                                                                                                      \
  }
  switch (ks) {
    FQ_CASE(1)
    FQ_CASE(2)
    FQ_CASE(3)
    FQ_CASE(4)
    FQ_CASE(5)
    FQ_CASE(6)
    default:
      (void)hipFreeAsync(buf, st);
      return false;
  }
#undef FQ_CASE
  (void)hipFreeAsync(buf, st);
  return true;
}

// =============================================================================================
// Batched arm_fir_q7 on the i8 matrix cores (round 6), bit-exact.  The reference
// (Source/FilteringFunctions/arm_fir_q7.c:446-560 and the tail) sums (q15_t)(x * c) -- exact, |x c|
// <= 2^14 -- in a q31_t and stores (q7_t)__SSAT(acc >> 7, 8); with numTaps <= 161 the sum is exact
// in int32, so the whole filter is ONE i8 plane product per K step: the samples and the taps are
// already the MFMA's i8 operands.  Same Toeplitz tiling as above; the window starts d = 0 .. 3
// samples early so that its block-input words are 4-byte aligned (one coefficient image per d).
constexpr int kQ7Words = (kFmChunk + 32 * kFmMaxKS) / 4;      // window words (4 samples) per item: 1072
constexpr int kQ7Per = (kQ7Words + 255) / 256;                // words per thread
constexpr int kQ7Plane = 4 * kQ7Words + 256;

// image[d][ks][lane]: taps c[32 ks + 16 h + e - d - i] as the A operand (lane L: i = L & 31, h = L >> 5)
__global__ __launch_bounds__(256) void fir_q7_coef_image_kernel(const int8_t* __restrict__ coeffs, int T, int KS,
                                                                int d_base, uint4* __restrict__ image) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g >= 4 * KS * 64) return;
  const int L = g & 63, ks = (g >> 6) % KS, d = (g >> 6) / KS, i = L & 31, h = L >> 5;
  uint32_t w[4] = {};
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int ci = 32 * ks + 16 * h + e - (d_base + d) - i;   // slot d holds window shift d_base + d
    w[e >> 2] |= (uint32_t)(uint8_t)((ci >= 0 && ci < T) ? coeffs[ci] : 0) << (8 * (e & 3));
  }
  image[(d * KS + ks) * 64 + L] = make_uint4(w[0], w[1], w[2], w[3]);
}

// ALN: blockSize % 16 == 0 and 16-B aligned data -- the window starts d_base = (-T1) mod 16 samples
// early (image slot 0), every region begins on a 16-B boundary, two dwordx4 loads per thread.
template <int KS, bool ALN>
__global__ __launch_bounds__(256) void fir_q7_mfma_kernel(int T, int d_base, const int8_t* __restrict__ src, int8_t* __restrict__ dst,
                                                          uint32_t B, const int8_t* __restrict__ hist, uint32_t nchunks,
                                                          uint32_t items, const uint4* __restrict__ image) {
  __shared__ __attribute__((aligned(16))) uint8_t pw[kQ7Plane];
  __shared__ __attribute__((aligned(16))) uint4 imgl[4 * KS * 64];
  __shared__ uint32_t hd[256];                           // the next window's head samples [0, 192) and tail word samples [192, 196)
  __shared__ __attribute__((aligned(16))) uint32_t ot[4][256];   // per wave: the output tile on its way out
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T1 = T - 1;
  for (int u = tid; u < 4 * KS * 64; u += 256) imgl[u] = image[u];   // visible after the loop's first barrier

  struct Item { uint32_t f; int n0, count, d; };
  auto item_of = [&](uint32_t it) {
    Item x;
    x.f = it / nchunks;
    x.n0 = (int)(it - x.f * nchunks) * kFmChunk;
    x.count = min((int)B - x.n0, kFmChunk);
    x.d = ALN ? d_base : (int)(((uint64_t)x.f * B + (uint32_t)x.n0 - (uint32_t)T1) & 3u);   // w[m] = s[n0 - d + m]
    return x;
  };
  // Window words (4 samples) from CLAMPED aligned block-input words, no branch; the words not wholly
  // in the block input -- the history head of a filter's first item and the block's last partial
  // word -- from per-sample LDS DMA (ubyte, zero-extended to a dword per lane): waves 0-2 head samples
  // 64 w + lane, wave 3 (lanes 0-3) the four samples of word u_hi.  As in the q15 kernel.
  struct Win { int u_lo, u_hi; };
  auto win_of = [&](const Item& x) {
    Win w;
    const int lo_num = T1 - x.n0 + x.d, hi_num = T1 + (int)B - 4 - x.n0 + x.d;
    w.u_lo = lo_num > 0 ? (lo_num + 3) >> 2 : 0;
    w.u_hi = hi_num >= 0 ? (hi_num >> 2) + 1 : 0;
    return w;
  };
  uint32_t wv[ALN ? 8 : kQ7Per];
  auto aln_bounds = [&](const Item& x, int& m_lo, int& m_hi) {   // block samples of the window (multiples of 16)
    m_lo = max(T1 - x.n0 + x.d, 0);
    m_hi = min(T1 + (int)B - x.n0 + x.d, 4 * kQ7Words);
  };
  auto load_window = [&](const Item& x) {
    const Win w = win_of(x);
    const int8_t* blk = src + ((int64_t)x.f * B + x.n0 - x.d - T1);      // w[m] of the block input: blk[m] (aligned)
    if constexpr (ALN) {
      int m_lo, m_hi;
      aln_bounds(x, m_lo, m_hi);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int m = min(max(16 * (tid + 256 * q), m_lo), m_hi - 16);
        const uint4 v = *reinterpret_cast<const uint4*>(blk + m);
        wv[4 * q] = v.x;
        wv[4 * q + 1] = v.y;
        wv[4 * q + 2] = v.z;
        wv[4 * q + 3] = v.w;
      }
    } else {
    // clamped to the aligned dwords inside this filter's block (never empty: blockSize >= 64)
    const uintptr_t lo_a = ((uintptr_t)(src + (uint64_t)x.f * B) + 3) & ~(uintptr_t)3;
    const uintptr_t hi_a = ((uintptr_t)(src + (uint64_t)(x.f + 1) * B) & ~(uintptr_t)3) - 4;
#pragma unroll
    for (int q = 0; q < kQ7Per; ++q) {
      const uintptr_t ad = (uintptr_t)(blk + 4 * (tid + 256 * q));
      wv[q] = *reinterpret_cast<const uint32_t*>(ad < lo_a ? lo_a : (ad > hi_a ? hi_a : ad));
    }
    }
    const int m = wid < 3 ? 64 * wid + L : 4 * w.u_hi + min(L, 3);
    const int j = x.n0 - x.d + m;                          // state index of window sample m
    const bool in_h = j >= 0 && j < T1;
    const int8_t* p = in_h ? hist + (uint64_t)x.f * T1 + j : src + (uint64_t)x.f * B + min(max(j - T1, 0), (int)B - 1);
    __builtin_amdgcn_global_load_lds((const void*)p, (__attribute__((address_space(3))) void*)(hd + 64 * wid), 1, 0, 0);
  };
  auto stage_window_aln = [&](const Item& x) {           // ALN: 16 samples -> one 16-B slot
    int m_lo, m_hi;
    aln_bounds(x, m_lo, m_hi);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int m0 = 16 * (tid + 256 * q);
      if (m0 >= 4 * kQ7Words) continue;
      uint32_t w4[4];
      if (m0 < m_lo) {                                   // history head (wave 0): the DMA'd samples, 0 before the state
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          uint32_t v = 0u;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int m = m0 + 4 * k + e;
            v |= (x.n0 - x.d + m >= 0 ? (hd[m] & 255u) : 0u) << (8 * e);
          }
          w4[k] = v;
        }
      } else if (m0 < m_hi) {
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = wv[4 * q + k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = 0u;
      }
      *reinterpret_cast<uint4*>(pw + fm_swz(m0)) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  };
  auto stage_window = [&](const Item& x) {
    const Win w = win_of(x);
#pragma unroll
    for (int q = 0; q < kQ7Per; ++q) {
      const int u = tid + 256 * q;
      if (u >= kQ7Words) continue;
      uint32_t v = wv[q];
      if (u < w.u_lo || u >= w.u_hi) {                   // per-sample: head (hd[m]) or the tail word (hd[192 + e])
        v = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = x.n0 - x.d + 4 * u + e;
          const bool valid = j >= 0 && j - T1 < (int)B;
          const uint32_t sm = u < w.u_lo ? hd[min(4 * u + e, 191)] : (u == w.u_hi ? hd[192 + e] : 0u);
          v |= (valid ? (sm & 255u) : 0u) << (8 * e);
        }
      }
      *reinterpret_cast<uint32_t*>(pw + fm_swz(4 * u)) = v;
    }
  };

  uint32_t it = blockIdx.x;
  if (it >= items) return;
  Item cur = item_of(it);
  load_window(cur);
  for (;;) {
    __syncthreads();                                     // the previous item's reads (and the DMA's landing)
    if constexpr (ALN) stage_window_aln(cur); else stage_window(cur);
    __syncthreads();
    const uint32_t nxt = it + gridDim.x;
    const Item next = item_of(nxt < items ? nxt : it);
    if (nxt < items) load_window(next);                  // in flight under this item's MFMAs
    if (1024 * wid < cur.count) {
      const int i = L & 31, h = L >> 5;
      const uint4* img = imgl + (cur.d - d_base) * KS * 64 + L;
      i32x16 acc = {};
      const int mb = 1024 * wid + 32 * i + 16 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint4 u = img[ks * 64];
        const i32x4 c = i32x4{(int)u.x, (int)u.y, (int)u.z, (int)u.w};
        const i32x4 x = *reinterpret_cast<const i32x4*>(pw + fm_swz(mb + 32 * ks));
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(c, x, acc, 0, 0, 0);
      }
      // lane (j = L & 31, h), register 4q + e -> output 8q + 4h + e of block j
      const int j = L & 31, ob = 1024 * wid + 32 * j + 4 * h;
      int8_t* yf = dst + (uint64_t)cur.f * B + cur.n0;
      uint32_t y[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) v |= (uint32_t)(uint8_t)(int8_t)ssat8(acc[4 * q + e] >> 7) << (8 * e);
        y[q] = v;
      }
      if (cur.count == kFmChunk && ((((uintptr_t)yf) & 15) == 0)) {
        // through the wave's 1 KiB LDS slot (dword 8 j + 2 q + h), then one coalesced 1 KiB store
        uint32_t* otw = ot[wid];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 8 * j + 2 * q + h;
          otw[c ^ (((c >> 5) & 7) << 2)] = y[q];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t r[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = 4 * L + e;
          r[e] = otw[c ^ (((c >> 5) & 7) << 2)];
        }
        *reinterpret_cast<uint4*>(yf + 1024 * wid + 16 * L) = make_uint4(r[0], r[1], r[2], r[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ob + 8 * q + e < cur.count) yf[ob + 8 * q + e] = (int8_t)(y[q] >> (8 * e));
      }
    }
    if (nxt >= items) break;
    it = nxt;
    cur = next;
  }
}

// true: launched (numTaps 1 .. 157, enough work to fill the chip); false: not this path
bool fir_q7_mfma_launch(const int8_t* coeffs, int T, const int8_t* src, int8_t* dst, uint32_t B, uint32_t batch,
                        const int8_t* hist_in, hipStream_t st) {
  if (!MI355X_FIR_Q7_MFMA || T < 1 || T > 32 * kFmMaxKS - 35 || B < 64 || batch == 0) return false;
  const uint32_t nchunks = (B + kFmChunk - 1) / kFmChunk;
  const uint64_t items = (uint64_t)nchunks * batch;
  if (items < 256 || items > 0x7fffffffull) return false;
  // aligned mode: shift d16 = (-T1) mod 16 (blockSize % 16 == 0, 16-B aligned data), K >= numTaps + d16 + 31;
  // otherwise the window shift d <= 3 per item, K >= numTaps + 34
  const int d16 = (16 - (T - 1) % 16) % 16;
  const int ks_aln = (T + d16 + 31 + 31) / 32;
  const bool aln = MI355X_FIR_Q7_ALN && B % 16 == 0 && ((uintptr_t)src & 15) == 0 && ks_aln <= kFmMaxKS;
  const int ks = aln ? ks_aln : (T + 34 + 31) / 32;
  const int d_base = aln ? d16 : 0;
  const size_t img_bytes = (size_t)4 * ks * 64 * 16;
  void* buf = nullptr;
  if (hipMallocAsync(&buf, img_bytes, st) != hipSuccess) return false;
  uint4* img = (uint4*)buf;
  hipLaunchKernelGGL(fir_q7_coef_image_kernel, dim3((4 * ks * 64 + 255) / 256), dim3(256), 0, st, coeffs, T, ks, d_base, img);
#define F7_CASE(K)                                                                                              \
  case K: {                                                                                                     \
    auto kern = aln ? fir_q7_mfma_kernel<K, true> : fir_q7_mfma_kernel<K, false>;                               \
    const int g = persistent_grid((const void*)kern, 256, 0, items);                                            \
    hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, st, T, d_base, src, dst, B, hist_in, nchunks,               \
                       (uint32_t)items, (const uint4*)img);                                                     \
    break;                                                                                                      \
  }
  switch (ks) {
    F7_CASE(2)
    F7_CASE(3)
    F7_CASE(4)
    F7_CASE(5)
    F7_CASE(6)
    default:
      (void)hipFreeAsync(buf, st);
      return false;
  }
#undef F7_CASE
  (void)hipFreeAsync(buf, st);
  return true;
}

}  // namespace mi355x
