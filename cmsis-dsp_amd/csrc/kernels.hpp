// Internal launch entry points of the HIP kernels (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi355x {

// Grid of a persistent kernel: every CU filled to the occupancy the compiled kernel allows
// (hipOccupancyMaxActiveBlocksPerMultiprocessor x CU count), never more blocks than items.
// The CU count is per device (cached for the first 16 ordinals).
inline int persistent_grid(const void* kernel, int block, size_t lds, uint64_t items, int fallback_per_cu = 2) {
  static int cus_cache[16] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  int cus = (dev >= 0 && dev < 16) ? cus_cache[dev] : 0;
  if (!cus) {
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    if (dev >= 0 && dev < 16) cus_cache[dev] = cus;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds) != hipSuccess || per_cu <= 0)
    per_cu = fallback_per_cu;
  const uint64_t g = (uint64_t)cus * per_cu;
  return (int)(g < items ? g : items);
}

// In-place batched CFFT over `batch` contiguous transforms of n complex samples.
// tw: device copy of the instance's twiddle table.  perm: optional device permutation
// (nullptr = the reference tables' canonical digit reversal).  flags: kIfft | kBitrev
// (| kSatShl1 for q31 / q15).
hipError_t cfft_f32_launch(int n, float* data, uint32_t batch, const float* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st);
// N = 256 / 512 / 1024 / 2048 with the reference's own bit-reversal table (cfft_fixed_r16.hip);
// false if N is not one of those lengths.
bool cfft_q31_r16_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, uint32_t flags, hipStream_t st);
bool cfft_q15_r16_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, uint32_t flags, hipStream_t st);
// The same kernels with the MFCC front end fused into their load phase (PRE): forward, frame
// maxima to maxv[frame * mstride]; false when n is not 256..2048.
// Stores v into *dflag (a device-mapped coherent host word) after the stream's earlier work
// (sync.hip): the drop-in calls' completion signal.
hipError_t done_flag_launch(uint32_t* dflag, uint32_t v, hipStream_t st);
// One arm_cfft_f32 N = 1024 call of the drop-in (the reference's table, batch within one
// workgroup) whose workgroup stores seq into done when its stores are visible; false: not this
// case, nothing launched.
bool cfft_f32_n1024_done_launch(float* data, uint32_t batch, const float* tw, const uint16_t* perm, uint32_t flags,
                                uint32_t* done, uint32_t seq, hipStream_t st);

// The whole MFCC q31 / q15 in one launch (front end + CFFT + back end, cfft_fixed_r16.hip);
// n = fftLen / 2.  hipErrorNotSupported: not handled (take the two-launch schedule).
hipError_t mfcc_q31_fused_launch(int n, const int32_t* frames, uint32_t batch, const int32_t* tw, const int32_t* win,
                                 bool brev, const int4* stw, int nb_mel, const int32_t* coefs, const uint32_t* bf,
                                 int total, int kmin, int kcnt, int nb_dct, const int32_t* dct, const int32_t* lut,
                                 int32_t* dst, hipStream_t st);
hipError_t mfcc_q15_fused_launch(int n, const int16_t* frames, uint32_t batch, const int16_t* tw, const int16_t* win,
                                 bool brev, const int4* stw, int nb_mel, const int16_t* coefs, const uint32_t* bf,
                                 int total, int kmin, int kcnt, int nb_dct, const int16_t* dct, const int32_t* lut,
                                 int16_t* dst, hipStream_t st);
bool cfft_q31_r16_mfcc_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, const int32_t* win,
                              int32_t* maxv, int mstride, bool brev, hipStream_t st);
bool cfft_q15_r16_mfcc_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, const int16_t* win,
                              int16_t* maxv, int mstride, bool brev, hipStream_t st);
hipError_t cfft_q31_launch(int n, int32_t* data, uint32_t batch, const int32_t* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st);
hipError_t cfft_q15_launch(int n, int16_t* data, uint32_t batch, const int16_t* tw, const uint16_t* perm,
                           uint32_t flags, hipStream_t st);

// Real FFT split (forward, after the N/2 CFFT) / merge (inverse, before it) passes.
hipError_t rfft_f32_stage_launch(int n_real, const float* p, float* out, uint32_t batch,
                                 const float* tw_rfft, hipStream_t st);
// Single-launch RFFT for the reference's canonical CFFT tables: tw = CFFT(n/2) twiddles,
// tw_rfft = twiddleCoef_rfft_n.  Forward writes the spectrum to `out` and, when pcopy is
// non-null, the inner CFFT output to pcopy (the reference leaves it in p).
hipError_t rfft_f32_fused_launch(int n_real, bool inverse, const float* p, float* pcopy, float* out, uint32_t batch,
                                 const float* tw, const float* tw_rfft, hipStream_t st);
hipError_t rfft_f32_merge_launch(int n_real, const float* p, float* out, uint32_t batch,
                                 const float* tw_rfft, hipStream_t st);

// RFFT q31 / q15 split (forward: src = [batch][N] CFFT(N/2) output -> dst [batch][2N]
// spectrum) or merge (inverse: src = [batch][2N] spectrum rows -> dst [batch][N] inverse
// CFFT input) pass.  ta / tb: device realCoef{A,B}; mod = the instance's modifier.
// forward arm_rfft_q31, N = 8192 (reference tables), inner CFFT + split in one launch (cfft_fixed.hip)
// forward arm_rfft_q31 / _q15 of fftLenReal = 2n, n = 256 .. 2048, in one launch (false: other n);
// rec = device_split_records(A, B, mod, n, sizeof word)
bool rfft_q31_r16_fused_launch(int n, int32_t* src, int32_t* dst, uint32_t batch, const int32_t* tw, const void* rec,
                               hipStream_t st);
bool rfft_q15_r16_fused_launch(int n, int16_t* src, int16_t* dst, uint32_t batch, const int16_t* tw, const void* rec,
                               hipStream_t st);
// inverse arm_rfft_q31 / _q15 of fftLenReal = 2n, n = 256 .. 2048, in one launch (merge fused into
// the radix-16 CFFT's first pass; false: other n); spec [batch][4n], dst [batch][2n]
bool rfft_q31_r16_inv_fused_launch(int n, const int32_t* spec, int32_t* dst, uint32_t batch, const int32_t* tw,
                                   const void* rec, hipStream_t st);
bool rfft_q15_r16_inv_fused_launch(int n, const int16_t* spec, int16_t* dst, uint32_t batch, const int16_t* tw,
                                   const void* rec, hipStream_t st);
// ... and fftLenReal = 8192 (the CFFT-4096 specialists), from the instance's realCoefA / B
hipError_t rfft_q31_8192_fused_launch(int32_t* src, int32_t* dst, uint32_t batch, const int32_t* tw, const int32_t* ta,
                                      const int32_t* tb, uint32_t mod, hipStream_t st);
hipError_t rfft_q31_8192_inv_fused_launch(const int32_t* spec, int32_t* dst, uint32_t batch, const int32_t* tw,
                                          const void* rec, hipStream_t st);
hipError_t rfft_q15_8192_inv_fused_launch(const int16_t* spec, int16_t* dst, uint32_t batch, const int16_t* tw,
                                          const void* rec, hipStream_t st);
hipError_t rfft_q15_8192_fused_launch(int16_t* src, int16_t* dst, uint32_t batch, const int16_t* tw, const int16_t* ta,
                                      const int16_t* tb, uint32_t mod, hipStream_t st);
hipError_t rfft_q31_pass_launch(bool inverse, int n, const int32_t* src, int32_t* dst, uint32_t batch,
                                const int32_t* ta, const int32_t* tb, uint32_t mod, hipStream_t st);
hipError_t rfft_q15_pass_launch(bool inverse, int n, const int16_t* src, int16_t* dst, uint32_t batch,
                                const int16_t* ta, const int16_t* tb, uint32_t mod, hipStream_t st);

// FIR: `batch` independent filters sharing one coefficient set, any of the five reference
// variants (kind).  hist: [batch][numTaps-1] streaming state (read, then overwritten with
// the new tail).  Element type: f32 float, q15/fast_q15 int16, q31/fast_q31 int32, q7 int8.
enum FirKind { kFirF32 = 0, kFirQ15 = 1, kFirQ31 = 2, kFirFastQ15 = 3, kFirFastQ31 = 4, kFirQ7 = 5,
               kFirF32Fma = 6 };   // kFirF32Fma: the opt-in fused-multiply-add f32 path (tolerance)
// done / seq (the synchronous drop-in): when the pass ends in one workgroup it also stores seq into
// the completion word done (runtime.cpp done_slot) and sets *flagged.
// arm_fir_q15 on the i8 matrix cores (fir_mfma.hip): false when the shape is not its (the caller
// then runs fir_q15_kernel)
bool fir_q15_mfma_launch(const int16_t* coeffs, int T, const int16_t* src, int16_t* dst, uint32_t B, uint32_t batch,
                         const int16_t* hist_in, hipStream_t st, bool fast = false);   // fast: arm_fir_fast_q15
// arm_fir_q7 likewise (numTaps <= 157)
bool fir_q7_mfma_launch(const int8_t* coeffs, int T, const int8_t* src, int8_t* dst, uint32_t B, uint32_t batch,
                        const int8_t* hist_in, hipStream_t st);
// arm_fir_q31 likewise (numTaps <= 161)
bool fir_q31_mfma_launch(const int32_t* coeffs, int T, const int32_t* src, int32_t* dst, uint32_t B, uint32_t batch,
                         const int32_t* hist_in, hipStream_t st);
hipError_t fir_run(int kind, const void* coeffs, int num_taps, const void* src, void* dst, uint32_t block_size,
                   uint32_t batch, void* hist, hipStream_t st, uint32_t* done = nullptr, uint32_t seq = 0,
                   bool* flagged = nullptr);

// Multirate FIR (fir.hip): `batch` independent decimators / interpolators sharing one
// coefficient set.  Decimator: outputs [batch][blockSize / M], hist [batch][numTaps - 1].
// Interpolator (phase_len = numTaps / L): outputs [batch][blockSize * L], hist
// [batch][phase_len - 1].  The interpolator takes kMrF32 / kMrQ15 / kMrQ31.
enum MrOp { kMrF32 = 0, kMrQ15 = 1, kMrQ31 = 2, kMrFastQ15 = 3, kMrFastQ31 = 4 };
hipError_t fir_decimate_run(int op, const void* coeffs, int num_taps, int M, const void* src, void* dst,
                            uint32_t block_size, uint32_t batch, void* hist, hipStream_t st);
hipError_t fir_interpolate_run(int op, const void* coeffs, int L, int phase_len, const void* src, void* dst,
                               uint32_t block_size, uint32_t batch, void* hist, hipStream_t st);
// Sparse FIR (fir.hip): `batch` streams sharing taps c[k] at delays D[k] (device arrays).
// circ_len == 0: block [batch][B] + history [batch][max_delay] (oldest first, updated);
// circ_len = L > 0: one stream whose samples are the reference's circular state buffer `src`
// of L words (block already written), tap k starting at circ_r0 - D[k] (wrapped), hist unused.
enum SpOp { kSpF32 = 0, kSpQ31 = 1, kSpQ15 = 2, kSpQ7 = 3 };
hipError_t fir_sparse_run(int op, const void* coeffs, const int32_t* delays, int num_taps, int max_delay,
                          const void* src, void* dst, uint32_t block_size, uint32_t batch, void* hist, int circ_len,
                          int circ_r0, hipStream_t st);
// FIR lattice (fir_lattice.hip): `batch` streams sharing numStages reflection coefficients;
// state [batch][numStages] = g_m at each stream's previous sample (updated in place).
enum LatOp { kLatF32 = 0, kLatQ31 = 1, kLatQ15 = 2 };
hipError_t fir_lattice_run(int op, const void* coeffs, int num_stages, const void* src, void* dst,
                           uint32_t block_size, uint32_t batch, void* state, hipStream_t st);

// MFCC f32 around the batched RFFT (mfcc_f32.hip): frame normalisation + window, then the
// spectrum -> Mel -> log -> DCT tail.  post needs mfcc_f32_post_lds(n, nb_mel) bytes of LDS.
// Fused single-launch MFCC for the reference's canonical CFFT tables (nb_mel <= n/2):
// tw = the inner CFFT(n/2) twiddles, twr = the RFFT split twiddles (twiddleCoef_rfft_n).
hipError_t mfcc_f32_fused_launch(int n, const float* src, const float* win, const float* tw, const float* twr,
                                 int nb_mel, const uint32_t* pos, const uint32_t* len, const uint32_t* off,
                                 const float* coefs, int nb_dct, const float* dct, float* dst, uint32_t batch,
                                 int total, hipStream_t st);
// The frame maximum of frame f is written to / read from maxv[f * maxv_stride].
hipError_t mfcc_f32_pre_launch(int n, const float* src, const float* win, float* x, float* maxv, uint32_t batch,
                               int maxv_stride, hipStream_t st);
// MFCC q31 around the batched q31 RFFT (mfcc_q31.hip); post needs mfcc_q31_post_lds bytes.
hipError_t mfcc_q31_pre_launch(int n, const int32_t* src, const int32_t* win, int32_t* x, int32_t* maxv,
                               uint32_t batch, int maxv_stride, hipStream_t st);
size_t mfcc_q31_post_lds(int n, int nb_mel);
hipError_t mfcc_q15_pre_launch(int n, const int16_t* src, const int16_t* win, int16_t* x, int16_t* maxv,
                               uint32_t batch, int maxv_stride, hipStream_t st);
hipError_t mfcc_q15_post_launch(int n, const int16_t* y, const int4* tw, const int16_t* maxv, int maxv_stride, int nb_mel,
                                int kmin, int kcnt, const int16_t* coefs,
                                const uint32_t* bf, int total, int nb_dct, const int16_t* dct, const int32_t* lut, int16_t* dst, uint32_t batch,
                                hipStream_t st);

hipError_t mfcc_q31_post_launch(int n, const int32_t* y, const int4* tw, const int32_t* maxv, int maxv_stride, int nb_mel,
                                int kmin, int kcnt, const int32_t* coefs,
                                const uint32_t* bf, int total, int nb_dct, const int32_t* dct, const int32_t* lut, int32_t* dst, uint32_t batch,
                                hipStream_t st);
size_t mfcc_f32_post_lds(int n, int nb_mel);
hipError_t mfcc_f32_post_launch(int n, const float* y, const float* maxv, int maxv_stride, int nb_mel,
                                const uint32_t* pos,
                                const uint32_t* len, const uint32_t* off, const float* coefs, int nb_dct,
                                const float* dct, float* dst, uint32_t batch, hipStream_t st);

// Row-major C[b] = A[b] (m x k) * B[b] (k x n), contiguous batch.
hipError_t mat_mult_f32_launch(int m, int k, int n, const float* a, const float* b, float* c,
                               uint32_t batch, hipStream_t st);

// Convolution / correlation family (conv.hip), bit-exact per op:
//   v[n] = sum_k x[k] * g[n-k], k ascending, g = h (convolution) or h time-reversed
//   (corr: correlation), for n in [first, first + num), stored at
//   y[item * sy + yoff + ydir * n].  x / h item strides sx / sh (0 = shared).
// kConvFastQ15 requires A >= B (the reference's x is the longer input).
enum ConvOp { kConvF32 = 0, kConvQ15 = 1, kConvQ31 = 2, kConvFastQ15 = 3, kConvFastQ31 = 4, kConvQ7 = 5,
              kConvFastOptQ15 = 6 };
struct ConvJob {
  int op;
  bool corr;
  const void* x; uint32_t A; uint64_t sx;
  const void* h; uint32_t B; uint64_t sh;
  void* y; uint64_t sy; int64_t yoff; int ydir;
  uint32_t first, num, batch;
};
hipError_t conv_family_run(const ConvJob& job, hipStream_t st);
// f32 windowed outputs through the FIR kernel (fir.hip): v[n] = sum_t w[n + t] c[t],
// w[j] = x[j - (T-1)], n = first .. first + num - 1, stored at y[item sy + off + dir (n - first)].
hipError_t fir_f32_conv_pass(const float* c, uint64_t cstride, int T, const float* x, uint64_t sx, uint32_t A,
                             uint32_t first, float* y, uint64_t sy, int64_t off, int dir, uint32_t num, uint32_t batch,
                             hipStream_t st);

// Row-major q15 / q31 C[b] = A[b] * B[b] (arm_mat_mult_q15 / _q31 semantics, bit-exact):
// byte-sliced planes on the i8 matrix cores (mat_mult_fixed.hip).
hipError_t mat_mult_q15_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c, uint32_t batch,
                               hipStream_t st);
hipError_t mat_mult_q31_launch(int m, int k, int n, const int32_t* a, const int32_t* b, int32_t* c, uint32_t batch,
                               hipStream_t st);
// Row-major q7 C[b] = A[b] * B[b] (arm_mat_mult_q7 semantics, bit-exact): one i8 MFMA plane
// (mat_mult_q7.hip).
hipError_t mat_mult_q7_launch(int m, int k, int n, const int8_t* a, const int8_t* b, int8_t* c, uint32_t batch,
                              hipStream_t st);
// arm_mat_mult_fast_q15 (exact i8-plane GEMM, modular q31 sum, (q15)(sum >> 15)) and
// arm_mat_mult_fast_q31 (VALU: sum of per-product (a*b) >> 32, output << 1).
hipError_t mat_mult_fast_q15_launch(int m, int k, int n, const int16_t* a, const int16_t* b, int16_t* c,
                                    uint32_t batch, hipStream_t st);
hipError_t mat_mult_fast_q31_launch(int m, int k, int n, const int32_t* a, const int32_t* b, int32_t* c,
                                    uint32_t batch, hipStream_t st);

}  // namespace mi355x
