/*
 * arm_math_mi355x.h — additive batched API of the MI355X CMSIS-DSP backend.
 *
 * The drop-in functions of arm_math.h process one transform / block / matrix per call,
 * synchronously.  These entry points are the path that can reach the HBM roofline:
 *   - all data pointers are DEVICE pointers (hipMalloc'd, or managed memory);
 *   - `batch` items are contiguous (stride = one item), processed in one launch;
 *   - work is enqueued on `stream` (a hipStream_t passed as void*, NULL = legacy default
 *     stream) and the call returns without synchronising;
 *   - results are bit-identical to calling the reference scalar function on each item in
 *     turn (f32 CFFT/RFFT/FIR and all fixed-point functions), or within the stated
 *     tolerance (arm_mat_mult_f32_batch, MFMA accumulation — DESIGN.md §mat_mult);
 *   - return ARM_MATH_SUCCESS, ARM_MATH_ARGUMENT_ERROR (unsupported length, NULL pointer,
 *     launch failure; details in arm_mi355x_last_error_string()).
 * Instance structs are the reference's own (arm_math.h).  Tables and coefficients they point
 * to: a device pointer is used in place; the library's own CommonTables are uploaded once per
 * device and cached by address; any other host table is cached by CONTENT (hash + compare) in
 * an LRU bounded in bytes (arm_mi355x_set_table_cache_limit), so changing coefficients
 * between calls is always seen and never grows device memory without bound.
 * Multi-GPU: either one process (or host thread) per device, each calling these on its
 * own shard with that device current (the library's caches, scratch and internal streams
 * are per device and per thread), or one call of the *_batch_multi entry points below,
 * which enqueue every shard on its device before waiting for any.
 */
#ifndef ARM_MATH_MI355X_BATCH_H
#define ARM_MATH_MI355X_BATCH_H

#include "arm_math.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Complex FFT over `batch` contiguous transforms of 2*fftLen words each, in place.
 * Per-item semantics: arm_cfft_f32 / _q31 / _q15 (arm_cfft_f32.c:1243, arm_cfft_q31.c:704,
 * arm_cfft_q15.c:671). */
arm_status arm_cfft_f32_batch(const arm_cfft_instance_f32 *S, float32_t *d_p1, uint32_t batch,
                              uint8_t ifftFlag, uint8_t bitReverseFlag, void *stream);
arm_status arm_cfft_q31_batch(const arm_cfft_instance_q31 *S, q31_t *d_p1, uint32_t batch,
                              uint8_t ifftFlag, uint8_t bitReverseFlag, void *stream);
arm_status arm_cfft_q15_batch(const arm_cfft_instance_q15 *S, q15_t *d_p1, uint32_t batch,
                              uint8_t ifftFlag, uint8_t bitReverseFlag, void *stream);

/* Real FFT (fast) over `batch` contiguous signals of fftLenRFFT floats.
 * Per-item semantics: arm_rfft_fast_f32 (arm_rfft_fast_f32.c:675-699), including the
 * reference's overwrite of d_p on the forward transform. */
arm_status arm_rfft_fast_f32_batch(const arm_rfft_fast_instance_f32 *S, float32_t *d_p,
                                   float32_t *d_out, uint32_t batch, uint8_t ifftFlag, void *stream);
/* The same with flags.  ARM_MI355X_RFFT_P_SCRATCH: d_p is scratch, as the reference documents
 * pIn of arm_rfft_fast_f32 ("the input buffer is modified by this function"): the forward
 * transform may leave it with any contents, which lets the batched kernels skip writing the
 * inner CFFT's output back (8 instead of 12 bytes of HBM traffic per real sample).  d_out is
 * bit-identical either way; the inverse never writes d_p.  Other flag bits: ARM_MATH_ARGUMENT_ERROR. */
#define ARM_MI355X_RFFT_P_SCRATCH 1u
arm_status arm_rfft_fast_f32_batch_ex(const arm_rfft_fast_instance_f32 *S, float32_t *d_p,
                                      float32_t *d_out, uint32_t batch, uint8_t ifftFlag, uint32_t flags,
                                      void *stream);

/* Real FFT, q31 / q15, over `batch` signals (per item: arm_rfft_q31 / arm_rfft_q15,
 * arm_rfft_q31.c:148-183).  Forward (S->ifftFlagR != 1): d_src [batch][N] is overwritten
 * by the inner CFFT as in the reference, d_dst [batch][2N] receives the spectra.
 * Inverse: d_src [batch][2N] spectrum rows (words 0 .. N+1 of each row are read; the
 * layout of the forward output), d_dst [batch][N]. */
arm_status arm_rfft_q31_batch(const arm_rfft_instance_q31 *S, q31_t *d_src, q31_t *d_dst, uint32_t batch,
                              void *stream);
arm_status arm_rfft_q15_batch(const arm_rfft_instance_q15 *S, q15_t *d_src, q15_t *d_dst, uint32_t batch,
                              void *stream);

/* MFCC over `batch` contiguous frames of S->fftLen samples (arm_mfcc_f32.c:83-160 per
 * frame).  d_src: [batch][fftLen] input frames (used as work space: overwritten);
 * d_tmp: [batch][fftLen] work space; d_dst: [batch][nbDctOutputs].  The instance's
 * coefficient tables may be host or device pointers (host tables are uploaded on each
 * call through the calling thread's staging buffers, in stream order). */
arm_status arm_mfcc_f32_batch(const arm_mfcc_instance_f32 *S, float32_t *d_src, float32_t *d_dst,
                              float32_t *d_tmp, uint32_t batch, void *stream);
/* MFCC q31 over `batch` contiguous frames (arm_mfcc_q31.c:88-225 per frame, bit-exact):
 * d_src [batch][fftLen] (overwritten), d_tmp [batch][2*fftLen] work, d_dst [batch][nbDct]. */
arm_status arm_mfcc_q31_batch(const arm_mfcc_instance_q31 *S, q31_t *d_src, q31_t *d_dst, q31_t *d_tmp,
                              uint32_t batch, void *stream);
/* MFCC q15 over `batch` contiguous frames (arm_mfcc_q15.c:96-228 per frame, bit-exact):
 * d_src [batch][fftLen] (overwritten), d_tmp [batch][2*fftLen] q15 work, d_dst [batch][nbDct]. */
arm_status arm_mfcc_q15_batch(const arm_mfcc_instance_q15 *S, q15_t *d_src, q15_t *d_dst, q15_t *d_tmp,
                              uint32_t batch, void *stream);

/* FIR over `batch` independent filters sharing S->numTaps / S->pCoeffs (host or device
 * pointer; S->pState is not used).  d_src/d_dst: [batch][blockSize].  d_hist:
 * [batch][numTaps-1] streaming state, read as the history before the block and
 * overwritten with the history after it, so consecutive calls equal one long call
 * (arm_fir_f32.c:1242-1278).  Zero it to start a stream (arm_fir_init_f32). */
arm_status arm_fir_f32_batch(const arm_fir_instance_f32 *S, const float32_t *d_src, float32_t *d_dst,
                             uint32_t blockSize, uint32_t batch, float32_t *d_hist, void *stream);
/* Opt-in TOLERANCE path of arm_fir_f32_batch (same arguments and state contract): every
 * output still sums its taps in the reference's order, but each MAC is one fused multiply-add
 * (v_fma_f32: the product is not rounded before the add), so results differ from the reference
 * in the last bits: |y - y_exact| <= numTaps * 2^-24 * sum_k |x b| (checked against float64 in
 * tests/test_fir_fma.py, with the reference suite's thresholds, FIRF32.cpp).  About twice the
 * bit-exact kernel's throughput (one VALU instruction per MAC instead of two). */
arm_status arm_fir_f32_batch_fma(const arm_fir_instance_f32 *S, const float32_t *d_src, float32_t *d_dst,
                                 uint32_t blockSize, uint32_t batch, float32_t *d_hist, void *stream);
arm_status arm_fir_q15_batch(const arm_fir_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                             uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_fast_q15_batch(const arm_fir_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                  uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_q31_batch(const arm_fir_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                             uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);
arm_status arm_fir_fast_q31_batch(const arm_fir_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                  uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);
arm_status arm_fir_q7_batch(const arm_fir_instance_q7 *S, const q7_t *d_src, q7_t *d_dst,
                            uint32_t blockSize, uint32_t batch, q7_t *d_hist, void *stream);

/* Multirate FIR over `batch` independent streams sharing one instance's coefficients (the
 * instance's pState is not used): d_src [batch][blockSize]; decimators write
 * d_dst [batch][blockSize / M] with d_hist [batch][numTaps - 1]; interpolators write
 * d_dst [batch][blockSize * L] with d_hist [batch][phaseLength - 1].  Per-stream semantics:
 * arm_fir_decimate_* / arm_fir_interpolate_*. */
arm_status arm_fir_decimate_f32_batch(const arm_fir_decimate_instance_f32 *S, const float32_t *d_src,
                                      float32_t *d_dst, uint32_t blockSize, uint32_t batch, float32_t *d_hist,
                                      void *stream);
arm_status arm_fir_decimate_q15_batch(const arm_fir_decimate_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                      uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_decimate_fast_q15_batch(const arm_fir_decimate_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                           uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_decimate_q31_batch(const arm_fir_decimate_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                      uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);
arm_status arm_fir_decimate_fast_q31_batch(const arm_fir_decimate_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                           uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);
arm_status arm_fir_interpolate_f32_batch(const arm_fir_interpolate_instance_f32 *S, const float32_t *d_src,
                                         float32_t *d_dst, uint32_t blockSize, uint32_t batch, float32_t *d_hist,
                                         void *stream);
arm_status arm_fir_interpolate_q15_batch(const arm_fir_interpolate_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                         uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_interpolate_q31_batch(const arm_fir_interpolate_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                         uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);

/* Sparse FIR over `batch` independent streams sharing S's taps and delays (host or device
 * arrays): d_src / d_dst [batch][blockSize], d_hist [batch][maxDelay] = each stream's last
 * maxDelay input samples, oldest first (zero-initialise, updated in place; the linear form of
 * the reference's circular state, which the batched call does not use).  Delays outside
 * [0, maxDelay] read zero.  Per-stream semantics: arm_fir_sparse_f32 / _q31 / _q15 / _q7. */
arm_status arm_fir_sparse_f32_batch(const arm_fir_sparse_instance_f32 *S, const float32_t *d_src, float32_t *d_dst,
                                    uint32_t blockSize, uint32_t batch, float32_t *d_hist, void *stream);
arm_status arm_fir_sparse_q31_batch(const arm_fir_sparse_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                    uint32_t blockSize, uint32_t batch, q31_t *d_hist, void *stream);
arm_status arm_fir_sparse_q15_batch(const arm_fir_sparse_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                    uint32_t blockSize, uint32_t batch, q15_t *d_hist, void *stream);
arm_status arm_fir_sparse_q7_batch(const arm_fir_sparse_instance_q7 *S, const q7_t *d_src, q7_t *d_dst,
                                   uint32_t blockSize, uint32_t batch, q7_t *d_hist, void *stream);

/* FIR lattice over `batch` independent streams sharing S's coefficients: d_src / d_dst
 * [batch][blockSize], d_state [batch][numStages] (each stream's state in the reference's
 * layout, zero-initialise; updated in place).  Per-stream semantics: arm_fir_lattice_*. */
arm_status arm_fir_lattice_f32_batch(const arm_fir_lattice_instance_f32 *S, const float32_t *d_src, float32_t *d_dst,
                                     uint32_t blockSize, uint32_t batch, float32_t *d_state, void *stream);
arm_status arm_fir_lattice_q31_batch(const arm_fir_lattice_instance_q31 *S, const q31_t *d_src, q31_t *d_dst,
                                     uint32_t blockSize, uint32_t batch, q31_t *d_state, void *stream);
arm_status arm_fir_lattice_q15_batch(const arm_fir_lattice_instance_q15 *S, const q15_t *d_src, q15_t *d_dst,
                                     uint32_t blockSize, uint32_t batch, q15_t *d_state, void *stream);

/* Convolution of `batch` pairs: item i convolves d_a + i*strideA (srcALen samples) with
 * d_b + i*strideB (srcBLen samples; strideB = 0 shares one kernel) into
 * d_dst + i*(srcALen + srcBLen - 1).  Per-item semantics: arm_conv_f32 / _q15 / _q31. */
arm_status arm_conv_f32_batch(const float32_t *d_a, uint32_t srcALen, uint32_t strideA, const float32_t *d_b,
                              uint32_t srcBLen, uint32_t strideB, float32_t *d_dst, uint32_t batch, void *stream);
arm_status arm_conv_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                              uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t batch, void *stream);
arm_status arm_conv_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                              uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t batch, void *stream);
arm_status arm_conv_fast_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                                   uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t batch, void *stream);
arm_status arm_conv_fast_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                                   uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t batch, void *stream);
arm_status arm_conv_q7_batch(const q7_t *d_a, uint32_t srcALen, uint32_t strideA, const q7_t *d_b,
                             uint32_t srcBLen, uint32_t strideB, q7_t *d_dst, uint32_t batch, void *stream);

/* Partial convolution of `batch` pairs (strides as arm_conv_*_batch): item i's numPoints
 * outputs firstIndex .. firstIndex + numPoints - 1 go COMPACTLY to d_dst + i*numPoints.
 * ARM_MATH_ARGUMENT_ERROR when firstIndex + numPoints > srcALen + srcBLen - 1. */
arm_status arm_conv_partial_f32_batch(const float32_t *d_a, uint32_t srcALen, uint32_t strideA,
                                      const float32_t *d_b, uint32_t srcBLen, uint32_t strideB, float32_t *d_dst,
                                      uint32_t firstIndex, uint32_t numPoints, uint32_t batch, void *stream);
arm_status arm_conv_partial_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                                      uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t firstIndex,
                                      uint32_t numPoints, uint32_t batch, void *stream);
arm_status arm_conv_partial_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                                      uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t firstIndex,
                                      uint32_t numPoints, uint32_t batch, void *stream);
arm_status arm_conv_partial_fast_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                                           uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t firstIndex,
                                           uint32_t numPoints, uint32_t batch, void *stream);
arm_status arm_conv_partial_fast_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                                           uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t firstIndex,
                                           uint32_t numPoints, uint32_t batch, void *stream);
arm_status arm_conv_partial_q7_batch(const q7_t *d_a, uint32_t srcALen, uint32_t strideA, const q7_t *d_b,
                                     uint32_t srcBLen, uint32_t strideB, q7_t *d_dst, uint32_t firstIndex,
                                     uint32_t numPoints, uint32_t batch, void *stream);

/* Correlation of `batch` pairs: item i writes d_dst + i*(2*max(srcALen, srcBLen) - 1) at the
 * positions arm_correlate_* writes (the others are left untouched). */
arm_status arm_correlate_f32_batch(const float32_t *d_a, uint32_t srcALen, uint32_t strideA, const float32_t *d_b,
                                   uint32_t srcBLen, uint32_t strideB, float32_t *d_dst, uint32_t batch,
                                   void *stream);
arm_status arm_correlate_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                                   uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t batch, void *stream);
arm_status arm_correlate_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                                   uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t batch, void *stream);
arm_status arm_correlate_fast_q15_batch(const q15_t *d_a, uint32_t srcALen, uint32_t strideA, const q15_t *d_b,
                                        uint32_t srcBLen, uint32_t strideB, q15_t *d_dst, uint32_t batch,
                                        void *stream);
arm_status arm_correlate_fast_q31_batch(const q31_t *d_a, uint32_t srcALen, uint32_t strideA, const q31_t *d_b,
                                        uint32_t srcBLen, uint32_t strideB, q31_t *d_dst, uint32_t batch,
                                        void *stream);
arm_status arm_correlate_q7_batch(const q7_t *d_a, uint32_t srcALen, uint32_t strideA, const q7_t *d_b,
                                  uint32_t srcBLen, uint32_t strideB, q7_t *d_dst, uint32_t batch, void *stream);

/* Row-major C[b] = A[b] * B[b] for `batch` contiguous (numRows x numCols) matrices with
 * the shapes of the three instances (their pData must be device pointers to the first
 * item).  Returns ARM_MATH_SIZE_MISMATCH on incompatible shapes (arm_mat_mult_f32.c:618-630). */
arm_status arm_mat_mult_f32_batch(const arm_matrix_instance_f32 *pSrcA, const arm_matrix_instance_f32 *pSrcB,
                                  arm_matrix_instance_f32 *pDst, uint32_t batch, void *stream);
/* q7 / q15 / q31 analogues (bit-exact; q7 on one i8 matrix-core plane, q15 / q31 byte-sliced
 * planes on the i8 matrix cores). */
arm_status arm_mat_mult_q7_batch(const arm_matrix_instance_q7 *pSrcA, const arm_matrix_instance_q7 *pSrcB,
                                 arm_matrix_instance_q7 *pDst, uint32_t batch, void *stream);
arm_status arm_mat_mult_q15_batch(const arm_matrix_instance_q15 *pSrcA, const arm_matrix_instance_q15 *pSrcB,
                                  arm_matrix_instance_q15 *pDst, uint32_t batch, void *stream);
arm_status arm_mat_mult_q31_batch(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                                  arm_matrix_instance_q31 *pDst, uint32_t batch, void *stream);
arm_status arm_mat_mult_fast_q15_batch(const arm_matrix_instance_q15 *pSrcA, const arm_matrix_instance_q15 *pSrcB,
                                       arm_matrix_instance_q15 *pDst, uint32_t batch, void *stream);
arm_status arm_mat_mult_fast_q31_batch(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                                       arm_matrix_instance_q31 *pDst, uint32_t batch, void *stream);

/* Multi-GPU complex FFT (SURVEY §8b "a multi-GPU entry point"; per item: arm_cfft_f32 /
 * _q31 / _q15, transform_functions.h:456-460).  Shard s of `nshards` is batch[s] contiguous
 * transforms at DEVICE pointer d_p1[s] on HIP device devices[s] (a device may appear in
 * several shards).  Every shard is launched on an internal stream of its device before any
 * is waited for, so the devices run concurrently; the call returns when all shards are
 * done (synchronous, like the drop-in API).  Input written on other streams must be
 * complete before the call.  Arguments are validated before anything is launched:
 * ARM_MATH_ARGUMENT_ERROR for a bad device index, NULL pointer or unsupported length.
 * The calling thread's current device is restored. */
arm_status arm_cfft_f32_batch_multi(const arm_cfft_instance_f32 *S, uint32_t nshards, const int *devices,
                                    float32_t *const *d_p1, const uint32_t *batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag);
arm_status arm_cfft_q31_batch_multi(const arm_cfft_instance_q31 *S, uint32_t nshards, const int *devices,
                                    q31_t *const *d_p1, const uint32_t *batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag);
arm_status arm_cfft_q15_batch_multi(const arm_cfft_instance_q15 *S, uint32_t nshards, const int *devices,
                                    q15_t *const *d_p1, const uint32_t *batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag);

/* Multi-GPU FIR (the batch is sliced by filter, so each filter's history stays on
 * its device; per filter: arm_fir_f32.c:911-1280, arm_fir_q15.c:458-726, ...).  Shard s of
 * `nshards` is batch[s] filters of blockSize samples on HIP device devices[s]: DEVICE pointers
 * d_src[s] / d_dst[s] [batch[s]][blockSize] and d_hist[s] [batch[s]][numTaps-1] with the
 * arm_fir_*_batch state contract.  S->pCoeffs: a host pointer (uploaded once per device), or a
 * device pointer every shard's device can read.  Launch/validate/wait semantics as
 * arm_cfft_f32_batch_multi. */
arm_status arm_fir_f32_batch_multi(const arm_fir_instance_f32 *S, uint32_t nshards, const int *devices,
                                   const float32_t *const *d_src, float32_t *const *d_dst, float32_t *const *d_hist,
                                   uint32_t blockSize, const uint32_t *batch);
arm_status arm_fir_q15_batch_multi(const arm_fir_instance_q15 *S, uint32_t nshards, const int *devices,
                                   const q15_t *const *d_src, q15_t *const *d_dst, q15_t *const *d_hist,
                                   uint32_t blockSize, const uint32_t *batch);
arm_status arm_fir_fast_q15_batch_multi(const arm_fir_instance_q15 *S, uint32_t nshards, const int *devices,
                                        const q15_t *const *d_src, q15_t *const *d_dst, q15_t *const *d_hist,
                                        uint32_t blockSize, const uint32_t *batch);
arm_status arm_fir_q31_batch_multi(const arm_fir_instance_q31 *S, uint32_t nshards, const int *devices,
                                   const q31_t *const *d_src, q31_t *const *d_dst, q31_t *const *d_hist,
                                   uint32_t blockSize, const uint32_t *batch);
arm_status arm_fir_fast_q31_batch_multi(const arm_fir_instance_q31 *S, uint32_t nshards, const int *devices,
                                        const q31_t *const *d_src, q31_t *const *d_dst, q31_t *const *d_hist,
                                        uint32_t blockSize, const uint32_t *batch);
arm_status arm_fir_q7_batch_multi(const arm_fir_instance_q7 *S, uint32_t nshards, const int *devices,
                                  const q7_t *const *d_src, q7_t *const *d_dst, q7_t *const *d_hist,
                                  uint32_t blockSize, const uint32_t *batch);

/* Multi-GPU matrix multiply (per matrix: arm_mat_mult_f32.c:600-730 / _q15 / _q31): shard s is
 * batch[s] contiguous matrices with the instances' shapes (their pData are not used) at DEVICE
 * pointers d_a[s], d_b[s], d_c[s] on devices[s].  ARM_MATH_SIZE_MISMATCH on incompatible
 * shapes; otherwise as arm_cfft_f32_batch_multi. */
arm_status arm_mat_mult_f32_batch_multi(const arm_matrix_instance_f32 *pSrcA, const arm_matrix_instance_f32 *pSrcB,
                                        arm_matrix_instance_f32 *pDst, uint32_t nshards, const int *devices,
                                        const float32_t *const *d_a, const float32_t *const *d_b,
                                        float32_t *const *d_c, const uint32_t *batch);
arm_status arm_mat_mult_q7_batch_multi(const arm_matrix_instance_q7 *pSrcA, const arm_matrix_instance_q7 *pSrcB,
                                       arm_matrix_instance_q7 *pDst, uint32_t nshards, const int *devices,
                                       const q7_t *const *d_a, const q7_t *const *d_b, q7_t *const *d_c,
                                       const uint32_t *batch);
arm_status arm_mat_mult_q15_batch_multi(const arm_matrix_instance_q15 *pSrcA, const arm_matrix_instance_q15 *pSrcB,
                                        arm_matrix_instance_q15 *pDst, uint32_t nshards, const int *devices,
                                        const q15_t *const *d_a, const q15_t *const *d_b, q15_t *const *d_c,
                                        const uint32_t *batch);
arm_status arm_mat_mult_q31_batch_multi(const arm_matrix_instance_q31 *pSrcA, const arm_matrix_instance_q31 *pSrcB,
                                        arm_matrix_instance_q31 *pDst, uint32_t nshards, const int *devices,
                                        const q31_t *const *d_a, const q31_t *const *d_b, q31_t *const *d_c,
                                        const uint32_t *batch);

/* Number of HIP devices visible to the process (0 when none). */
int arm_mi355x_device_count(void);

/* Error channel for the void-returning drop-in functions: 0 = no error, otherwise the
 * hipError_t of the last failure on this thread. */
int arm_mi355x_last_error(void);
const char *arm_mi355x_last_error_string(void);
void arm_mi355x_clear_error(void);

/* Device bytes held by the content-keyed cache of host tables / coefficients (all devices),
 * and its limit PER DEVICE (default 256 MiB).  Lowering it evicts least-recently-used entries
 * now.  An entry in use by a call that is still being enqueued is never evicted, and an
 * evicted entry's memory is released in stream order after the work that read it (an event
 * recorded after each call's launches; no device synchronize, no lock held while waiting). */
size_t arm_mi355x_table_cache_bytes(void);
void arm_mi355x_set_table_cache_limit(size_t bytes);

/* Per-thread runtime resources.  A thread that calls the synchronous (drop-in) functions gets a
 * stream per device, device scratch, pinned staging buffers and a completion word, grown on
 * demand (the reference allocates nothing: this is the backend's cost of being a drop-in).
 * They are released automatically when a thread other than the process's main thread exits;
 * arm_mi355x_release_thread_resources() releases the calling thread's set now (call it between
 * calls, e.g. before a pool retires a worker, or on the main thread; the next call re-creates
 * what it needs).  arm_mi355x_thread_resource_owners() counts the threads holding a set. */
void arm_mi355x_release_thread_resources(void);
int arm_mi355x_thread_resource_owners(void);

/* Library identification: "cmsisdsp-mi355x <version> gfx950 src:<id>", where <id> is a hash of
 * the sources the library was built from (cmsis-dsp_amd/Makefile SRC_ID), followed by
 * " [macros]" when the library was built with any non-default tuning macro (bench lines print
 * it). */
const char *arm_mi355x_version(void);

#ifdef __cplusplus
}
#endif
#endif
