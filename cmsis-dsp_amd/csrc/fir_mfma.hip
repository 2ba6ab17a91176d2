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

#ifndef MI355X_FIR_Q15_DIAG        // 1: diagnostic only -- no window loads after the first item (wrong output)
#define MI355X_FIR_Q15_DIAG 0
#endif

namespace mi355x {

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
                                                                 uint4* __restrict__ image, int* __restrict__ info) {
  // one thread per (d, ks, lane): 2 KS x 64 threads, each the three planes' 16 bytes; the last
  // workgroup's first wave also reduces sum(c) and the wrap flag
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < 2 * KS * 64) {
    const int L = g & 63, ks = (g >> 6) % KS, d = (g >> 6) / KS, i = L & 31, h = L >> 5;
    uint32_t w[3][4] = {};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ci = 32 * ks + 16 * h + e - d - i;
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

template <int KS>
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
    const int32_t W = 2 * a8[g] + a7[g] + sumc + (a0[g] >> 7);
    const uint32_t v = (uint16_t)(int16_t)ssat16(X + (W >> 8));
    y[g >> 1] = (g & 1) ? (y[g >> 1] | (v << 16)) : v;
  }
}

// lane (j = L & 31, h), register 4q + e -> output 8q + 4h + e of block j
__device__ __forceinline__ void fm_tile_store(const uint32_t (&y)[8], int wid, int L, int count,
                                              int16_t* __restrict__ yrow) {
  const int j = L & 31, h = L >> 5;
  int16_t* yb = yrow + 1024 * wid + 32 * j + 4 * h;
  const int ob = 1024 * wid + 32 * j + 4 * h;
  if (count == kFmChunk && ((((uintptr_t)yrow) & 7) == 0)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<uint2*>(yb + 8 * q) = make_uint2(y[2 * q], y[2 * q + 1]);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (ob + 8 * q + e < count) yb[8 * q + e] = (int16_t)(y[2 * q + (e >> 1)] >> (16 * (e & 1)));
  }
}

// One wave's 32 x 32 output tile of an item (outputs 1024 wid .. + 1023) from the staged planes:
// 6 plane products per K step into five int32 accumulators, then the exact output.
template <int KS>
__device__ __forceinline__ void fm_tile(const uint4* __restrict__ imgd, const uint8_t* ph, const uint8_t* pl, int wid,
                                        int L, int count, int16_t* __restrict__ yrow, int32_t sumc) {
  uint32_t y[8];
  fm_tile_y<KS>(imgd, ph, pl, wid, L, sumc, y);
  fm_tile_store(y, wid, L, count, yrow);
}

template <int KS>
__global__ __launch_bounds__(256, MI355X_FIR_Q15_MFMA_WG) void fir_q15_mfma_kernel(const int16_t* __restrict__ coeffs, int T,
                                                              const int16_t* __restrict__ src, int16_t* __restrict__ dst,
                                                              uint32_t B, const int16_t* __restrict__ hist,
                                                              uint32_t nchunks, uint32_t items,
                                                              const uint4* __restrict__ image,
                                                              const int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) uint8_t ph[kFmPlane];
  __shared__ __attribute__((aligned(16))) uint8_t pl[kFmPlane];
  __shared__ __attribute__((aligned(16))) uint4 imgl[2 * KS * 3 * 64];   // the coefficient image, once per workgroup
  const int tid = threadIdx.x, L = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T1 = T - 1;
  const bool wrap = info[1] != 0;
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
    x.d = (int)(((uint64_t)x.f * B + (uint32_t)x.n0 - (uint32_t)T1) & 1u);   // s index n0 - d + m -> src f B + n0 - d + m - T1
    return x;
  };
  // Window words in PAIRS: thread tid takes words 2 (tid + 256 q) and + 1 (4 samples, one 4-byte
  // write per plane), then single words 512 kFmPer2 + tid + 256 q.  Words whose two samples both lie in the block input (u_lo <= u < u_hi, wave-
  // uniform bounds) are aligned dword loads; the rest (history of a filter's first item, the
  // zero tail past the block) sample by sample from a clamped, always-valid address.
  uint32_t wv[2 * kFmPer2 + kFmPer1];
  auto word_slow = [&](const Item& x, int u) -> uint32_t {
    uint32_t r = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = x.n0 - x.d + 2 * u + e;              // state index
      const bool in_h = j >= 0 && j < T1, in_b = j >= T1 && j - T1 < (int)B;
      const int16_t* p = in_h ? hist + (uint64_t)x.f * T1 + j : (in_b ? src + (uint64_t)x.f * B + (j - T1) : src);
      const uint32_t v = (uint16_t)*p;
      r |= ((in_h || in_b) ? v : 0u) << (16 * e);
    }
    return r;
  };
  auto load_window = [&](const Item& x) {
    const int64_t base = (int64_t)x.f * B + x.n0 - x.d - T1;               // src index of w[0] (even)
    const int lo_num = T1 - x.n0 + x.d, hi_num = T1 + (int)B - 2 - x.n0 + x.d;
    const int u_lo = lo_num > 0 ? (lo_num + 1) >> 1 : 0, u_hi = hi_num >= 0 ? (hi_num >> 1) + 1 : 0;
    auto word = [&](int u) -> uint32_t {
      return (u >= u_lo && u < u_hi) ? *reinterpret_cast<const uint32_t*>(src + base + 2 * u) : word_slow(x, u);
    };
#pragma unroll
    for (int q = 0; q < kFmPer2; ++q) {
#pragma unroll
      for (int e = 0; e < 2; ++e) wv[2 * q + e] = word(2 * (tid + 256 * q) + e);
    }
#pragma unroll
    for (int q = 0; q < kFmPer1; ++q) {
      const int u = 512 * kFmPer2 + tid + 256 * q;
      wv[2 * kFmPer2 + q] = u < kFmWords ? word(u) : 0u;
    }
  };
  auto stage_window = [&]() {                            // registers -> the two byte planes
#pragma unroll
    for (int q = 0; q < kFmPer1; ++q) {
      const int u = 512 * kFmPer2 + tid + 256 * q;
      if (u >= kFmWords) continue;
      const uint32_t v = wv[2 * kFmPer2 + q];
      const int a = fm_swz(2 * u);
      *reinterpret_cast<uint16_t*>(ph + a) = (uint16_t)(((v >> 8) & 0xFFu) | ((v >> 16) & 0xFF00u));
      *reinterpret_cast<uint16_t*>(pl + a) = (uint16_t)(((v & 0xFFu) | ((v >> 8) & 0xFF00u)) ^ 0x8080u);
    }
#pragma unroll
    for (int q = 0; q < kFmPer2; ++q) {
      const int u = 2 * (tid + 256 * q);
      const uint32_t v0 = wv[2 * q], v1 = wv[2 * q + 1];
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
  for (;;) {
    __syncthreads();                                     // the previous item's reads are done
    stage_window();
    __syncthreads();
    const uint32_t nxt = it + gridDim.x;
    const Item next = item_of(nxt < items ? nxt : it);
    if (nxt < items && !MI355X_FIR_Q15_DIAG) load_window(next);   // in flight under this item's MFMAs

    if (wrap) {
      fm_wrap_item(ph, pl, coeffs, T, B, cur.n0, cur.d, cur.count, tid, dst + (uint64_t)cur.f * B);
    } else if (1024 * wid < cur.count) {
      fm_tile<KS>(imgl + cur.d * KS * 3 * 64, ph, pl, wid, L, cur.count, dst + (uint64_t)cur.f * B + cur.n0, sumc);
    }
    if (nxt >= items) break;
    it = nxt;
    cur = next;
  }
}

// true: launched (numTaps even, 2 .. 160, enough work to fill the chip); false: not this path
bool fir_q15_mfma_launch(const int16_t* coeffs, int T, const int16_t* src, int16_t* dst, uint32_t B,
                         uint32_t batch, const int16_t* hist_in, hipStream_t st) {
  if (!MI355X_FIR_Q15_MFMA || T < 2 || (T & 1) || T > 32 * kFmMaxKS - 32 || B == 0 || batch == 0) return false;
  const uint32_t nchunks = (B + kFmChunk - 1) / kFmChunk;
  const uint64_t items = (uint64_t)nchunks * batch;
  if (items < 256 || items > 0x7fffffffull) return false;
  const int ks = (T + 32 + 31) / 32;
  // the coefficient image (2 shifts x KS steps x 3 planes x 64 lanes x 16 B) and [sum, wrap]
  const size_t img_bytes = (size_t)2 * ks * 3 * 64 * 16;
  void* buf = nullptr;
  if (hipMallocAsync(&buf, img_bytes + 16, st) != hipSuccess) return false;
  uint4* img = (uint4*)buf;
  int* info = (int*)((char*)buf + img_bytes);
  hipLaunchKernelGGL(fir_q15_coef_image_kernel, dim3((2 * ks * 64 + 255) / 256), dim3(256), 0, st, coeffs, T, ks, img, info);
#define FM_CASE(K)                                                                                              \
  case K: {                                                                                                     \
    const int g = persistent_grid((const void*)fir_q15_mfma_kernel<K>, 256, 0, items);                         \
    hipLaunchKernelGGL(fir_q15_mfma_kernel<K>, dim3(g), dim3(256), 0, st, coeffs, T, src, dst, B, hist_in,       \
                       nchunks, (uint32_t)items, (const uint4*)img, (const int*)info);                          \
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

}  // namespace mi355x
