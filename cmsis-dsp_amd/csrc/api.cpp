// C ABI of libcmsisdsp_mi355x.so: the drop-in processing functions of arm_math.h and the
// batched device API of arm_math_mi355x.h.  Every GPU failure is caught here and mapped
// to the reference's status values (or the thread-local error channel for void functions);
// nothing aborts.  There is no CPU fallback: all compute runs in the HIP kernels.
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/arm_math.h"
#include "../../include/arm_math_mi355x.h"
#include "common.hpp"
#include "kernels.hpp"
#include "runtime.hpp"

using namespace mi355x;

namespace {

bool cfft_len_ok(uint32_t n) {
  return n == 16 || n == 32 || n == 64 || n == 128 || n == 256 || n == 512 || n == 1024 || n == 2048 || n == 4096;
}

#define MI_CHECK(expr, where)                        \
  do {                                               \
    hipError_t e_ = (expr);                          \
    if (e_ != hipSuccess) { set_error(e_, where); return false; } \
  } while (0)

struct CfftPrep {
  const void* tw = nullptr;
  const uint16_t* perm = nullptr;
  uint32_t flags = 0;
};

// kind: 0 f32, 1 q31, 2 q15
bool cfft_prepare(uint32_t n, const void* pTwiddle, const uint16_t* pBitRev, uint16_t bitRevLen, int kind,
                  uint8_t ifftFlag, uint8_t bitReverseFlag, CfftPrep& out) {
  // twiddle words: f32 N complex (twiddleCoef_N[2N]); fixed-point 3N/4 complex
  // (twiddleCoef_N_q31[3N/2], arm_common_tables.h:61-116)
  const size_t twb = kind == 0 ? 8u * n : (kind == 1 ? 4u * 3u * n / 2u : 2u * 3u * n / 2u);
  out.tw = device_table(pTwiddle, twb);
  if (!out.tw) return false;   // device_table recorded the cause
  out.flags = (ifftFlag == 1u ? kIfft : 0u) | (bitReverseFlag ? kBitrev : 0u);   // arm_cfft_f32.c:1252,1282
  if (bitReverseFlag) {
    bool canon = true, ok = true;
    out.perm = device_perm((int)n, pBitRev, bitRevLen, kind == 0 ? 0 : 1, &canon, &ok);
    if (!ok) { set_error(hipErrorInvalidValue, "bit-reversal table"); return false; }
  }
  return true;
}

hipError_t cfft_launch(int kind, uint32_t n, void* d, uint32_t batch, const CfftPrep& pr, hipStream_t st) {
  switch (kind) {
    case 0: return cfft_f32_launch((int)n, (float*)d, batch, (const float*)pr.tw, pr.perm, pr.flags, st);
    case 1: return cfft_q31_launch((int)n, (int32_t*)d, batch, (const int32_t*)pr.tw, pr.perm, pr.flags, st);
    default: return cfft_q15_launch((int)n, (int16_t*)d, batch, (const int16_t*)pr.tw, pr.perm, pr.flags, st);
  }
}

// synchronous single-transform drop-in path (host or device buffer)
template <typename Inst>
void cfft_sync(const Inst* S, void* p1, uint8_t ifftFlag, uint8_t bitReverseFlag, int kind, size_t word) {
  if (!S || !p1 || !cfft_len_ok(S->fftLen)) return;       // reference: silent no-op
  const uint32_t n = S->fftLen;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  CfftPrep pr;
  if (!cfft_prepare(n, S->pTwiddle, S->pBitRevTable, S->bitRevLength, kind, ifftFlag, bitReverseFlag, pr)) return;
  const size_t bytes = 2 * word * n;
  if (is_device_ptr(p1)) {
    hipError_t e = cfft_launch(kind, n, p1, 1, pr, st);
    if (e == hipSuccess) e = wait_stream(st);
    if (e != hipSuccess) set_error(e, "arm_cfft");
    return;
  }
  if (bytes <= kZeroCopyMax) {               // one launch on the coherent pinned copy, no DMA
    HostIO io(st);
    void* z = io.zinout(p1, bytes);
    if (!z) { set_error(hipErrorOutOfMemory, "arm_cfft staging"); return; }
    // N = 1024 f32 (the reference example's shape): the transform's workgroup also writes the
    // completion word, so the call is one launch (runtime.hpp done_slot)
    uint32_t* done = nullptr;
    uint32_t seq = 0;
    if (kind == 0 && n == 1024 && !pr.perm && done_slot(&done, &seq) &&
        cfft_f32_n1024_done_launch((float*)z, 1, (const float*)pr.tw, pr.perm, pr.flags, done, seq, st)) {
      hipError_t e = hipGetLastError();
      if (e == hipSuccess) e = io.finish(seq);
      if (e != hipSuccess) set_error(e, "arm_cfft");
      return;
    }
    hipError_t e = cfft_launch(kind, n, z, 1, pr, st);
    if (e == hipSuccess) e = io.finish();
    if (e != hipSuccess) set_error(e, "arm_cfft");
    return;
  }
  void* d = scratch(bytes, 0);
  if (!d) { set_error(hipErrorOutOfMemory, "arm_cfft scratch"); return; }
  HostIO io(st);
  hipError_t e = io.in(d, p1, bytes);
  if (e == hipSuccess) e = cfft_launch(kind, n, d, 1, pr, st);
  if (e == hipSuccess) e = io.out(p1, d, bytes);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, "arm_cfft");
}

template <typename Inst>
arm_status cfft_batch(const Inst* S, void* d_p1, uint32_t batch, uint8_t ifftFlag, uint8_t bitReverseFlag,
                      void* stream, int kind) {
  if (!S || (!d_p1 && batch) || !cfft_len_ok(S->fftLen)) return ARM_MATH_ARGUMENT_ERROR;
  BlobScope hold((hipStream_t)stream);
  CfftPrep pr;
  if (!cfft_prepare(S->fftLen, S->pTwiddle, S->pBitRevTable, S->bitRevLength, kind, ifftFlag, bitReverseFlag, pr))
    return ARM_MATH_ARGUMENT_ERROR;
  hipError_t e = cfft_launch(kind, S->fftLen, d_p1, batch, pr, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_cfft_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// multi-GPU: validate every shard, launch each on its device's internal stream (one BlobScope per
// shard, so the tables a shard uses stay held until its launches are enqueued), then wait for
// every device that received work.  launch(s, st) enqueues shard s on st (its device current).
template <typename Launch>
arm_status run_multi(uint32_t nshards, const int* devices, const uint32_t* batch, const char* what, Launch&& launch) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) { (void)hipGetLastError(); ndev = 0; }
  for (uint32_t s = 0; s < nshards; ++s)
    if (devices[s] < 0 || devices[s] >= ndev) return ARM_MATH_ARGUMENT_ERROR;
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::vector<int> used;
  arm_status status = ARM_MATH_SUCCESS;
  for (uint32_t s = 0; s < nshards && status == ARM_MATH_SUCCESS; ++s) {
    if (!batch[s]) continue;
    hipError_t e = hipSetDevice(devices[s]);
    if (e != hipSuccess) { set_error(e, what); status = ARM_MATH_ARGUMENT_ERROR; break; }
    if (std::find(used.begin(), used.end(), devices[s]) == used.end()) used.push_back(devices[s]);
    hipStream_t st = sync_stream();
    if (!st) { set_error(hipErrorOutOfMemory, what); status = ARM_MATH_ARGUMENT_ERROR; break; }
    BlobScope hold(st);
    if (!launch(s, st)) status = ARM_MATH_ARGUMENT_ERROR;
  }
  for (int d : used) {   // drain every device that received work, also after a failure
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) e = hipStreamSynchronize(sync_stream());
    if (e != hipSuccess) { set_error(e, what); status = ARM_MATH_ARGUMENT_ERROR; }
  }
  (void)hipSetDevice(prev);
  return status;
}

template <typename Inst>
arm_status cfft_batch_multi(const Inst* S, uint32_t nshards, const int* devices, void* const* d_p1,
                            const uint32_t* batch, uint8_t ifftFlag, uint8_t bitReverseFlag, int kind) {
  if (!S || !cfft_len_ok(S->fftLen) || (nshards && (!devices || !d_p1 || !batch))) return ARM_MATH_ARGUMENT_ERROR;
  for (uint32_t s = 0; s < nshards; ++s)
    if (batch[s] && !d_p1[s]) return ARM_MATH_ARGUMENT_ERROR;
  return run_multi(nshards, devices, batch, "arm_cfft_batch_multi", [&](uint32_t s, hipStream_t st) {
    CfftPrep pr;
    if (!cfft_prepare(S->fftLen, S->pTwiddle, S->pBitRevTable, S->bitRevLength, kind, ifftFlag, bitReverseFlag, pr))
      return false;
    hipError_t e = cfft_launch(kind, S->fftLen, d_p1[s], batch[s], pr, st);
    if (e != hipSuccess) { set_error(e, "arm_cfft_batch_multi"); return false; }
    return true;
  });
}

bool rfft_len_ok(uint32_t n) { return n >= 32 && n <= 4096 && (n & (n - 1)) == 0; }

// arm_rfft_fast_f32.c:675-699 on `batch` signals; d_p / d_out device pointers
// p_scratch (ARM_MI355X_RFFT_P_SCRATCH): the forward fused kernels skip writing the inner CFFT's
// output back into p (the reference documents p as scratch; the drop-in always writes it).
bool rfft_run(const arm_rfft_fast_instance_f32* S, float* d_p, float* d_out, uint32_t batch, uint8_t ifftFlag,
              hipStream_t st, bool p_scratch = false) {
  const uint32_t n = S->fftLenRFFT, h = S->Sint.fftLen;
  if (h != n / 2 || !cfft_len_ok(h)) { set_error(hipErrorInvalidValue, "rfft instance"); return false; }
  BlobScope hold(st);
  const void* twr = device_table(S->pTwiddleRFFT, sizeof(float) * n);
  if (!twr) return false;
  CfftPrep pr;
  // the inner CFFT receives ifftFlag unchanged and bitReverseFlag = 1 (:689, :694)
  if (!cfft_prepare(h, S->Sint.pTwiddle, S->Sint.pBitRevTable, S->Sint.bitRevLength, 0, ifftFlag, 1, pr))
    return false;
  if (!pr.perm && ifftFlag <= 1) {   // the reference's own tables: one fused launch
    // (ifftFlag > 1: merge + a FORWARD inner CFFT, arm_cfft_f32.c:1252 -- unfused path)
    MI_CHECK(rfft_f32_fused_launch((int)n, ifftFlag != 0, d_p, (ifftFlag || p_scratch) ? nullptr : d_p, d_out, batch,
                                   (const float*)pr.tw, (const float*)twr, st),
             "rfft fused");
    return true;
  }
  if (ifftFlag) {
    MI_CHECK(rfft_f32_merge_launch((int)n, d_p, d_out, batch, (const float*)twr, st), "rfft merge");
    MI_CHECK(cfft_f32_launch((int)h, d_out, batch, (const float*)pr.tw, pr.perm, pr.flags, st), "rfft cfft");
  } else {
    MI_CHECK(cfft_f32_launch((int)h, d_p, batch, (const float*)pr.tw, pr.perm, pr.flags, st), "rfft cfft");
    MI_CHECK(rfft_f32_stage_launch((int)n, d_p, d_out, batch, (const float*)twr, st), "rfft stage");
  }
  return true;
}

// ---- RFFT q31 / q15 (arm_rfft_q31.c:148-183, arm_rfft_q15.c): `batch` signals.
// Forward: d_src [batch][N] (overwritten by the inner CFFT, as the reference leaves pSrc),
// d_dst [batch][2N].  Inverse: d_src [batch][2N] spectrum rows (words 0 .. N+1 read),
// d_dst [batch][N]; the final arm_shift(+1) is folded into the inverse CFFT's store.
template <typename T, typename RInst>
bool rfft_fixed_run(const RInst* S, T* d_src, T* d_dst, uint32_t batch, hipStream_t st) {
  constexpr int kind = sizeof(T) == 4 ? 1 : 2;
  const uint32_t n = S->fftLenReal, L = n / 2;
  const auto* in = S->pCfft;
  if (!in || in->fftLen != L || !cfft_len_ok(L) || n > 8192) { set_error(hipErrorInvalidValue, "rfft instance"); return false; }
  BlobScope hold(st);
  const bool inv = S->ifftFlagR == 1u;
  CfftPrep pr;
  if (!cfft_prepare(L, in->pTwiddle, in->pBitRevTable, in->bitRevLength, kind, inv ? 1 : 0, S->bitReverseFlagR, pr))
    return false;
  // forward, the reference's own bit reversal, bitReverseFlag 1: the split runs inside the CFFT
  // launch (cfft_fixed.hip L = 4096 from the tables as they are; cfft_fixed_r16.hip L = 256 .. 2048
  // from packed per-bin records)
  const bool fuse = !inv && !pr.perm && (pr.flags & kBitrev) &&
                    (L == 4096 ? (kind == 1 ? MI355X_RFFT_Q31_FUSED : MI355X_RFFT_Q15_FUSED && MI355X_FX_Q15_PACKED)
                               : L >= 256 && L <= 2048 && MI355X_RFFT_FX_R16_FUSED);
  // inverse, same conditions: the merge runs in the CFFT's first pass (cfft_fixed_r16.hip L = 256 ..
  // 2048, cfft_fixed.hip L = 4096 -- q31 there stages half the records, so only for tables whose
  // records are symmetric, as the reference's realCoefAQ31 / BQ31 are)
  bool ifuse = inv && !pr.perm && (pr.flags & kBitrev) &&
               (L == 4096 ? (kind == 1 ? MI355X_RFFT_Q31_INV_FUSED : MI355X_RFFT_Q15_INV_FUSED && MI355X_FX_Q15_PACKED)
                          : L >= 256 && L <= 2048 && MI355X_RFFT_FX_R16_INV_FUSED);
  const void* irec = nullptr;
  if (ifuse) {
    bool sym = false;
    irec = device_split_records(S->pTwiddleAReal, S->pTwiddleBReal, S->twidCoefRModifier, L, (int)sizeof(T), st, &sym);
    if (!irec) return false;
    if (kind == 1 && L == 4096 && !sym) ifuse = false;
  }
  // the split / merge pass reads realCoef[2*mod*k + 1] for k < L: mod * N words cover it
  const T *ta = nullptr, *tb = nullptr;
  if ((!fuse && !ifuse) || (fuse && L == 4096)) {
    const size_t words = std::max<size_t>(2, (size_t)S->twidCoefRModifier * n);
    ta = (const T*)device_table(S->pTwiddleAReal, sizeof(T) * words);
    tb = (const T*)device_table(S->pTwiddleBReal, sizeof(T) * words);
    if (!ta || !tb) return false;
  }
  auto pass = [&](const T* a, T* b) {
    if constexpr (kind == 1)
      return rfft_q31_pass_launch(inv, (int)n, a, b, batch, ta, tb, S->twidCoefRModifier, st);
    else
      return rfft_q15_pass_launch(inv, (int)n, a, b, batch, ta, tb, S->twidCoefRModifier, st);
  };
  if (ifuse) {
    if (L == 4096) {
      MI_CHECK(kind == 1 ? rfft_q31_8192_inv_fused_launch((const int32_t*)d_src, (int32_t*)d_dst, batch, (const int32_t*)pr.tw, irec, st)
                         : rfft_q15_8192_inv_fused_launch((const int16_t*)d_src, (int16_t*)d_dst, batch, (const int16_t*)pr.tw, irec, st),
               "rfft inverse fused 8192");
      return true;
    }
    const bool done = kind == 1
        ? rfft_q31_r16_inv_fused_launch((int)L, (const int32_t*)d_src, (int32_t*)d_dst, batch, (const int32_t*)pr.tw, irec, st)
        : rfft_q15_r16_inv_fused_launch((int)L, (const int16_t*)d_src, (int16_t*)d_dst, batch, (const int16_t*)pr.tw, irec, st);
    if (!done) { set_error(hipErrorInvalidValue, "rfft inverse fused length"); return false; }
    MI_CHECK(hipGetLastError(), "rfft inverse fused");
  } else if (inv) {
    MI_CHECK(pass(d_src, d_dst), "rfft merge");
    pr.flags |= kSatShl1;
    MI_CHECK(cfft_launch(kind, L, d_dst, batch, pr, st), "rfft cfft");
  } else if (fuse) {
    if (L == 4096) {
      MI_CHECK(kind == 1 ? rfft_q31_8192_fused_launch((int32_t*)d_src, (int32_t*)d_dst, batch, (const int32_t*)pr.tw,
                                                      (const int32_t*)ta, (const int32_t*)tb, S->twidCoefRModifier, st)
                         : rfft_q15_8192_fused_launch((int16_t*)d_src, (int16_t*)d_dst, batch, (const int16_t*)pr.tw,
                                                      (const int16_t*)ta, (const int16_t*)tb, S->twidCoefRModifier, st),
               "rfft fused");
    } else {
      const void* rec = device_split_records(S->pTwiddleAReal, S->pTwiddleBReal, S->twidCoefRModifier, L, (int)sizeof(T), st);
      if (!rec) return false;
      const bool done = kind == 1
          ? rfft_q31_r16_fused_launch((int)L, (int32_t*)d_src, (int32_t*)d_dst, batch, (const int32_t*)pr.tw, rec, st)
          : rfft_q15_r16_fused_launch((int)L, (int16_t*)d_src, (int16_t*)d_dst, batch, (const int16_t*)pr.tw, rec, st);
      if (!done) { set_error(hipErrorInvalidValue, "rfft fused length"); return false; }
      MI_CHECK(hipGetLastError(), "rfft fused");
    }
  } else {
    MI_CHECK(cfft_launch(kind, L, d_src, batch, pr, st), "rfft cfft");
    MI_CHECK(pass(d_src, d_dst), "rfft split");
  }
  return true;
}

// drop-in arm_rfft_q31 / _q15: host or device buffers, synchronous
template <typename T, typename RInst>
void rfft_fixed_sync(const RInst* S, T* pSrc, T* pDst) {
  if (!S || !pSrc || !pDst) return;
  const uint32_t n = S->fftLenReal;
  if (n < 32 || n > 8192 || (n & (n - 1))) return;   // reference: lengths of the init switch only
  const bool inv = S->ifftFlagR == 1u;
  // forward: src N words in/out, dst 2N out; inverse: src words 0..N+1 in, dst N out
  const size_t sb = sizeof(T) * (inv ? (size_t)n + 2 : n), db = sizeof(T) * (inv ? n : 2 * (size_t)n);
  hipStream_t st = sync_stream();
  const bool ds = is_device_ptr(pSrc), dd = is_device_ptr(pDst);
  // the batched inverse reads spectrum rows of 2N words: a host row is staged that wide
  T* s = ds ? pSrc : (T*)scratch(sizeof(T) * 2 * (size_t)n, 0);
  T* d = dd ? pDst : (T*)scratch(db, 1);
  if (!s || !d) { set_error(hipErrorOutOfMemory, "arm_rfft scratch"); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!ds) e = io.in(s, pSrc, sb);
  if (e != hipSuccess) { set_error(e, "arm_rfft"); return; }
  if (!rfft_fixed_run<T>(S, s, d, 1, st)) { (void)hipStreamSynchronize(st); return; }
  if (!ds && !inv) e = io.out(pSrc, s, sb);   // forward overwrites pSrc
  if (e == hipSuccess && !dd) e = io.out(pDst, d, db);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, "arm_rfft");
}

template <typename T, typename RInst>
arm_status rfft_fixed_batch(const RInst* S, T* d_src, T* d_dst, uint32_t batch, void* stream) {
  if (!S || (batch && (!d_src || !d_dst))) return ARM_MATH_ARGUMENT_ERROR;
  const uint32_t n = S->fftLenReal;
  if (n < 32 || n > 8192 || (n & (n - 1))) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0) return ARM_MATH_SUCCESS;
  return rfft_fixed_run<T>(S, d_src, d_dst, batch, (hipStream_t)stream) ? ARM_MATH_SUCCESS : ARM_MATH_ARGUMENT_ERROR;
}

// ---- MFCC (arm_mfcc_f32.c:83-160): the instance's user tables packed into one
// content-cached device blob: [dct | filter coefs | window | pos | len | coef offsets]
struct MfccDev {
  int total = 0;                   // Mel coefficients (sum of filterLengths)
  const float* dct = nullptr;
  const float* coefs = nullptr;
  const float* win = nullptr;
  const uint32_t* pos = nullptr;
  const uint32_t* len = nullptr;
  const uint32_t* off = nullptr;
};

template <typename T>
bool host_copy(const T* p, size_t count, std::vector<T>& out) {
  out.resize(count);
  if (!count) return true;
  if (!p) return false;
  if (is_device_ptr(p)) return hipMemcpy(out.data(), p, sizeof(T) * count, hipMemcpyDeviceToHost) == hipSuccess;
  memcpy(out.data(), p, sizeof(T) * count);
  return true;
}

bool mfcc_prepare(const arm_mfcc_instance_f32* S, MfccDev& d) {
  const uint32_t n = S->fftLen, nm = S->nbMelFilters, nd = S->nbDctOutputs;
  if (!rfft_len_ok(n) || S->rfft.fftLenRFFT != n) { set_error(hipErrorInvalidValue, "mfcc instance"); return false; }
  if (mfcc_f32_post_lds((int)n, (int)nm) > 65536) { set_error(hipErrorInvalidValue, "mfcc: too many Mel filters"); return false; }
  std::vector<uint32_t> pos, len;
  if (!host_copy(S->filterPos, nm, pos) || !host_copy(S->filterLengths, nm, len)) {
    set_error(hipErrorInvalidValue, "mfcc filter tables");
    return false;
  }
  std::vector<uint32_t> off(nm);
  uint64_t total = 0;
  for (uint32_t i = 0; i < nm; ++i) {
    if ((uint64_t)pos[i] + len[i] > n) { set_error(hipErrorInvalidValue, "mfcc filter beyond fftLen"); return false; }
    off[i] = (uint32_t)total;
    total += len[i];
  }
  auto up16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t b_dct = up16(sizeof(float) * nm * nd), b_cf = up16(sizeof(float) * total), b_win = up16(sizeof(float) * n);
  const size_t b_u = up16(sizeof(uint32_t) * nm);
  std::vector<uint8_t> blob(b_dct + b_cf + b_win + 3 * b_u + 16, 0);
  std::vector<float> tmp;
  if (!host_copy(S->dctCoefs, (size_t)nm * nd, tmp)) { set_error(hipErrorInvalidValue, "mfcc dct"); return false; }
  memcpy(blob.data(), tmp.data(), sizeof(float) * tmp.size());
  if (!host_copy(S->filterCoefs, (size_t)total, tmp)) { set_error(hipErrorInvalidValue, "mfcc coefs"); return false; }
  memcpy(blob.data() + b_dct, tmp.data(), sizeof(float) * tmp.size());
  if (!host_copy(S->windowCoefs, (size_t)n, tmp)) { set_error(hipErrorInvalidValue, "mfcc window"); return false; }
  memcpy(blob.data() + b_dct + b_cf, tmp.data(), sizeof(float) * tmp.size());
  uint8_t* u = blob.data() + b_dct + b_cf + b_win;
  memcpy(u, pos.data(), sizeof(uint32_t) * nm);
  memcpy(u + b_u, len.data(), sizeof(uint32_t) * nm);
  memcpy(u + 2 * b_u, off.data(), sizeof(uint32_t) * nm);
  const uint8_t* dev = (const uint8_t*)device_blob(blob.data(), blob.size());
  if (!dev) return false;
  d.total = (int)total;
  d.dct = (const float*)dev;
  d.coefs = (const float*)(dev + b_dct);
  d.win = (const float*)(dev + b_dct + b_cf);
  d.pos = (const uint32_t*)(dev + b_dct + b_cf + b_win);
  d.len = (const uint32_t*)(dev + b_dct + b_cf + b_win + b_u);
  d.off = (const uint32_t*)(dev + b_dct + b_cf + b_win + 2 * b_u);
  return true;
}

// x: [batch][n] frames, y: [batch][n] work, dst: [batch][nbDct].  The reference's own
// (canonical) CFFT tables take the fused single-launch kernel (x read once, y unused);
// otherwise three launches, x overwritten and the frame maxima carried in dst[frame][0]
// between the passes (read before the row is written).
bool mfcc_run(const arm_mfcc_instance_f32* S, const MfccDev& d, float* x, float* y, float* dst, uint32_t batch,
              hipStream_t st) {
  const int n = (int)S->fftLen, nd = (int)S->nbDctOutputs, nm = (int)S->nbMelFilters;
  const arm_cfft_instance_f32& in = S->rfft.Sint;
  BlobScope hold(st);
  bool canon = true, ok = true;
  if (in.pBitRevTable) (void)device_perm((int)in.fftLen, in.pBitRevTable, in.bitRevLength, 0, &canon, &ok);
  if (ok && canon && nm <= n / 2 && in.fftLen == (uint32_t)n / 2) {
    const void* tw = device_table(in.pTwiddle, 8u * in.fftLen);
    const void* twr = device_table(S->rfft.pTwiddleRFFT, sizeof(float) * n);
    if (!tw || !twr) return false;
    MI_CHECK(mfcc_f32_fused_launch(n, x, d.win, (const float*)tw, (const float*)twr, nm, d.pos, d.len, d.off,
                                   d.coefs, nd, d.dct, dst, batch, d.total, st),
             "mfcc fused");
    return true;
  }
  MI_CHECK(mfcc_f32_pre_launch(n, x, d.win, x, dst, batch, nd, st), "mfcc pre");
  if (!rfft_run(&S->rfft, x, y, batch, 0, st)) return false;
  MI_CHECK(mfcc_f32_post_launch(n, y, dst, nd, nm, d.pos, d.len, d.off, d.coefs, nd, d.dct, dst, batch, st),
           "mfcc post");
  return true;
}

// ---- MFCC q31 / q15 (arm_mfcc_q31.c:88-225, arm_mfcc_q15.c:96-228): the same content-cached
// blob layout as the f32 instance in q31 / q15 words; the inner RFFT is the bit-exact batched
// fixed-point RFFT.  Mel filters must
// stay within the fftLen/2 + 1 magnitudes (the reference would read its CFFT's leftovers).
template <typename T>
struct MfccFxDev {
  const T* dct = nullptr;
  const T* coefs = nullptr;
  const T* win = nullptr;
  const uint32_t* pos = nullptr;
  const uint32_t* len = nullptr;
  const uint32_t* off = nullptr;
  const uint32_t* bf = nullptr;    // flat Mel coefficient g -> bin << 16 | filter
  int total = 0;
  int kmin = 0, kcnt = 0;          // the bins some Mel filter reads: kmin .. kmin + kcnt - 1
  const int4* tw = nullptr;        // split twiddles per bin k <= fftLen/2: {A[2mk], A[2mk+1], B[2mk], B[2mk+1]}
  const int32_t* lut = nullptr;
};

template <typename T, typename Inst>
bool mfcc_fx_prepare(const Inst* S, MfccFxDev<T>& d) {
  const uint32_t n = S->fftLen, nm = S->nbMelFilters, nd = S->nbDctOutputs;
  if (!rfft_len_ok(n) || S->rfft.fftLenReal != n || S->rfft.ifftFlagR != 0) {
    set_error(hipErrorInvalidValue, "mfcc q31 instance");
    return false;
  }
  if (mfcc_q31_post_lds((int)n, (int)nm) > 65536) { set_error(hipErrorInvalidValue, "mfcc q31: too many Mel filters"); return false; }
  std::vector<uint32_t> pos, len;
  if (!host_copy(S->filterPos, nm, pos) || !host_copy(S->filterLengths, nm, len)) {
    set_error(hipErrorInvalidValue, "mfcc q31 filter tables");
    return false;
  }
  std::vector<uint32_t> off(nm);
  uint64_t total = 0;
  for (uint32_t i = 0; i < nm; ++i) {
    if ((uint64_t)pos[i] + len[i] > n / 2 + 1) { set_error(hipErrorInvalidValue, "mfcc q31 filter beyond fftLen/2"); return false; }
    off[i] = (uint32_t)total;
    total += len[i];
  }
  if (nm > 0xFFFFu || total > 0x7FFFFFFFull) { set_error(hipErrorInvalidValue, "mfcc: too many Mel coefficients"); return false; }
  {
    uint32_t lo = n, hi = 0;
    for (uint32_t i = 0; i < nm; ++i)
      if (len[i]) { lo = std::min(lo, pos[i]); hi = std::max(hi, pos[i] + len[i]); }
    d.kmin = lo < hi ? (int)lo : 0;
    d.kcnt = lo < hi ? (int)(hi - lo) : 0;
  }
  auto up16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
  const size_t b_dct = up16(sizeof(T) * nm * nd), b_cf = up16(sizeof(T) * total), b_win = up16(sizeof(T) * n);
  const size_t b_u = up16(sizeof(uint32_t) * nm), b_bf = up16(sizeof(uint32_t) * total);
  const size_t b_tw = up16(sizeof(int4) * (n / 2 + 1));
  std::vector<uint8_t> blob(b_dct + b_cf + b_win + 3 * b_u + b_bf + b_tw + 16, 0);
  std::vector<T> tmp;
  if (!host_copy(S->dctCoefs, (size_t)nm * nd, tmp)) { set_error(hipErrorInvalidValue, "mfcc dct"); return false; }
  memcpy(blob.data(), tmp.data(), sizeof(T) * tmp.size());
  if (!host_copy(S->filterCoefs, (size_t)total, tmp)) { set_error(hipErrorInvalidValue, "mfcc coefs"); return false; }
  memcpy(blob.data() + b_dct, tmp.data(), sizeof(T) * tmp.size());
  if (!host_copy(S->windowCoefs, (size_t)n, tmp)) { set_error(hipErrorInvalidValue, "mfcc window"); return false; }
  memcpy(blob.data() + b_dct + b_cf, tmp.data(), sizeof(T) * tmp.size());
  uint8_t* u = blob.data() + b_dct + b_cf + b_win;
  memcpy(u, pos.data(), sizeof(uint32_t) * nm);
  memcpy(u + b_u, len.data(), sizeof(uint32_t) * nm);
  memcpy(u + 2 * b_u, off.data(), sizeof(uint32_t) * nm);
  uint32_t* bfh = reinterpret_cast<uint32_t*>(u + 3 * b_u);
  for (uint32_t i = 0, g = 0; i < nm; ++i)
    for (uint32_t j = 0; j < len[i]; ++j) bfh[g++] = ((pos[i] + j) << 16) | i;
  {   // the split's twiddle records (arm_rfft_q31.c:293-326 index 2 * modifier * k)
    const uint32_t mod = S->rfft.twidCoefRModifier, words = mod * n;
    std::vector<T> ta, tb;
    if (!host_copy(S->rfft.pTwiddleAReal, words, ta) || !host_copy(S->rfft.pTwiddleBReal, words, tb)) {
      set_error(hipErrorInvalidValue, "mfcc rfft tables");
      return false;
    }
    int4* twh = reinterpret_cast<int4*>(u + 3 * b_u + b_bf);
    for (uint32_t k = 1; k < n / 2; ++k) {
      const uint32_t c = 2 * mod * k;
      if constexpr (sizeof(T) == 2) {   // q15: packed pairs for v_dot2 (mfcc_fixed_post.hpp mq_split_q15)
        auto p2 = [](int32_t lo, int32_t hi) { return (int32_t)((uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16)); };
        const int32_t a0 = ta[c], a1 = ta[c + 1], b0 = tb[c], b1 = tb[c + 1];
        twh[k] = make_int4(p2(a0, ~a1), p2(b0, b1), p2(b1, ~b0), p2(a1, a0));
      } else {
        twh[k] = make_int4(ta[c], ta[c + 1], tb[c], tb[c + 1]);
      }
    }
  }
  const uint8_t* dev = (const uint8_t*)device_blob(blob.data(), blob.size());
  d.lut = (const int32_t*)device_table(sqrt_initial_lut_q31, sizeof(int32_t) * 32);
  if (!dev || !d.lut) return false;
  d.dct = (const T*)dev;
  d.coefs = (const T*)(dev + b_dct);
  d.win = (const T*)(dev + b_dct + b_cf);
  d.pos = (const uint32_t*)(dev + b_dct + b_cf + b_win);
  d.len = (const uint32_t*)(dev + b_dct + b_cf + b_win + b_u);
  d.off = (const uint32_t*)(dev + b_dct + b_cf + b_win + 2 * b_u);
  d.bf = (const uint32_t*)(dev + b_dct + b_cf + b_win + 3 * b_u);
  d.total = (int)total;
  d.tw = (const int4*)(dev + b_dct + b_cf + b_win + 3 * b_u + b_bf);
  return true;
}

// x: [batch][n] frames (overwritten), y: [batch][2n] spectra, dst: [batch][nbDct]; the frame
// maxima ride in dst[frame][0] between the launches (read before the row is written)
// MFCC q31 / q15 schedule (MI355X_MFCC_FX_MODE, tuning.hpp; fftLen 512..4096 with the reference's
// own CFFT bit reversal): 1 = two launches (default: front end fused into the radix-16 CFFT's load
// phase, then the post kernel), 2 = one launch (round 4: front end, radix-16 CFFT and back end in
// one kernel, the spectra never leave LDS: traffic = the frames once, but 1.30 / 1.09 ms against
// 1.02 / 0.83 ms per 2^18 frames -- the CFFT and back-end phases of a workgroup serialise at two
// workgroups per CU), 0 = three launches (pre, CFFT, post: also every other length
// and custom bit-reversal tables).
template <typename T, typename Inst>
bool mfcc_fx_run(const Inst* S, const MfccFxDev<T>& d, T* x, T* y, T* dst, uint32_t batch, hipStream_t st) {
  const int n = (int)S->fftLen, nd = (int)S->nbDctOutputs, nm = (int)S->nbMelFilters;
  // the forward RFFT's inner CFFT (arm_rfft_q31.c:148-183: cfft(L, fwd, bitReverseFlagR), then
  // arm_split_rfft): its tables and bit-reversal mode
  const auto* in = S->rfft.pCfft;
  const uint32_t L = (uint32_t)n / 2;
  if (!in || in->fftLen != L || !cfft_len_ok(L)) { set_error(hipErrorInvalidValue, "mfcc rfft instance"); return false; }
  BlobScope hold(st);
  CfftPrep pr;
  if (!cfft_prepare(L, in->pTwiddle, in->pBitRevTable, in->bitRevLength, sizeof(T) == 4 ? 1 : 2, 0,
                    S->rfft.bitReverseFlagR, pr))
    return false;
  if (MI355X_MFCC_FX_MODE >= 2 && !pr.perm) {    // the whole MFCC in one launch
    hipError_t e;
    if constexpr (sizeof(T) == 4)
      e = mfcc_q31_fused_launch((int)L, x, batch, (const int32_t*)pr.tw, d.win, S->rfft.bitReverseFlagR != 0, d.tw,
                                nm, d.coefs, d.bf, d.total, d.kmin, d.kcnt, nd, d.dct, d.lut, dst, st);
    else
      e = mfcc_q15_fused_launch((int)L, x, batch, (const int16_t*)pr.tw, d.win, S->rfft.bitReverseFlagR != 0, d.tw,
                                nm, d.coefs, d.bf, d.total, d.kmin, d.kcnt, nd, d.dct, d.lut, dst, st);
    if (e != hipErrorNotSupported) {
      MI_CHECK(e, "mfcc fused");
      return true;
    }
  }
  bool front = false;                       // pre + CFFT done by one launch
  if (MI355X_MFCC_FX_MODE >= 1 && !pr.perm) {
    if constexpr (sizeof(T) == 4)
      front = cfft_q31_r16_mfcc_launch((int)L, x, batch, (const int32_t*)pr.tw, d.win, dst, nd,
                                       S->rfft.bitReverseFlagR != 0, st);
    else
      front = cfft_q15_r16_mfcc_launch((int)L, x, batch, (const int16_t*)pr.tw, d.win, dst, nd,
                                       S->rfft.bitReverseFlagR != 0, st);
    if (front) MI_CHECK(hipGetLastError(), "mfcc front");
  }
  if (!front) {
    if constexpr (sizeof(T) == 4) {
      MI_CHECK(mfcc_q31_pre_launch(n, x, d.win, x, dst, batch, nd, st), "mfcc q31 pre");
    } else {
      MI_CHECK(mfcc_q15_pre_launch(n, x, d.win, x, dst, batch, nd, st), "mfcc q15 pre");
    }
    MI_CHECK(cfft_launch(sizeof(T) == 4 ? 1 : 2, L, x, batch, pr, st), "mfcc cfft");
  }
  (void)y;
  if constexpr (sizeof(T) == 4) {
    MI_CHECK(mfcc_q31_post_launch(n, x, d.tw, dst, nd, nm, d.kmin, d.kcnt, d.coefs, d.bf, d.total, nd, d.dct, d.lut, dst,
                                  batch, st),
             "mfcc q31 post");
  } else {
    MI_CHECK(mfcc_q15_post_launch(n, x, d.tw, dst, nd, nm, d.kmin, d.kcnt, d.coefs, d.bf, d.total, nd, d.dct, d.lut, dst,
                                  batch, st),
             "mfcc q15 post");
  }
  return true;
}

// FIR coefficients: device pointers in place, host sets through the content-keyed cache
// (uploaded synchronously once per distinct set, so an asynchronous batch call never
// shares a staging buffer with a later call on another stream)
template <typename T>
const T* device_coeffs(const T* c, int n, bool* ok) {
  const T* d = (const T*)device_table(c, sizeof(T) * (size_t)n);
  *ok = d != nullptr;
  return d;
}

bool ranges_overlap(const void* a, const void* b, size_t bytes) {
  const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
  return bytes && x < y + bytes && y < x + bytes;
}

// drop-in FIR: state = [history(T-1) ; block(B)] on host or device (arm_fir_f32.c:911-1280).
// After the call the state holds [new history ; block input], as the reference leaves it.
template <typename T, typename Inst>
void fir_sync(const Inst* S, const T* pSrc, T* pDst, uint32_t B, int kind) {
  if (!S || !S->pState || !S->pCoeffs || S->numTaps == 0 || B == 0) return;
  const int taps = S->numTaps, T1 = taps - 1;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, taps, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, "arm_fir coeffs"); return; }
  const bool dstate = is_device_ptr(S->pState), dsrc = is_device_ptr(pSrc), ddst = is_device_ptr(pDst);
  const size_t sb = sizeof(T) * (size_t)B, hb = sizeof(T) * (size_t)T1;
  if (!dstate && !dsrc && !ddst && hb + sb <= kZeroCopyMax) {
    // all host, small: the caller's state buffer itself, [history ; block], staged as one
    // coherent pinned copy the kernels use in place (the filter reads it, the history kernel
    // rewrites its head), so after finish() it holds [new history ; block input] exactly as the
    // reference leaves pState; outputs likewise -- two launches, no DMA
    HostIO io(st);
    T* zs = (T*)io.zinout(S->pState, hb + sb);
    T* zd = (T*)io.zout(pDst, sb);
    if (!zs || !zd) { set_error(hipErrorOutOfMemory, "arm_fir staging"); return; }
    memmove(zs + T1, pSrc, sb);                   // pSrc may alias pDst: read before anything
    uint32_t* done = nullptr;
    uint32_t seq = 0;
    bool flagged = false;                         // the filter's workgroup wrote the completion word
    if (!done_slot(&done, &seq)) done = nullptr;
    hipError_t e = fir_run(kind, dc, taps, zs + T1, zd, B, 1, zs, st, done, seq, &flagged);
    if (e == hipSuccess) e = io.finish(flagged ? seq : 0);
    if (e == hipSuccess) hold.synced();
    if (e != hipSuccess) set_error(e, "arm_fir");
    return;
  }
  // in place on the device (pSrc overlapping pDst): filter from a copy of the input, which
  // also feeds the new history and the state tail (the reference copies each input into
  // pState before writing pDst, arm_fir_f32.c:947-975)
  const bool alias = dsrc && ddst && ranges_overlap(pSrc, pDst, sb);
  T* dhist = dstate ? S->pState : (T*)scratch(hb + 16, 2);
  const T* dsr = (dsrc && !alias) ? pSrc : (const T*)scratch(sb, 3);
  T* dds = ddst ? pDst : (T*)scratch(sb, 4);
  if (!dhist || !dsr || !dds) { set_error(hipErrorOutOfMemory, "arm_fir scratch"); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!dstate && T1 > 0) e = io.in(dhist, S->pState, hb);
  if (e == hipSuccess && alias) e = hipMemcpyAsync((void*)dsr, pSrc, sb, hipMemcpyDeviceToDevice, st);
  else if (e == hipSuccess && !dsrc) e = io.in((void*)dsr, pSrc, sb);
  if (e == hipSuccess) e = fir_run(kind, dc, taps, dsr, dds, B, 1, dhist, st);
  if (e == hipSuccess && !ddst) e = io.out(pDst, dds, sb);
  if (e == hipSuccess && !dstate && T1 > 0) e = io.out(S->pState, dhist, hb);
  // state tail keeps the block input (the reference copies it there, :947-975)
  if (e == hipSuccess) {
    if (dstate) e = hipMemcpyAsync(S->pState + T1, dsr, sb, hipMemcpyDeviceToDevice, st);
    else if (dsrc) e = io.out(S->pState + T1, dsr, sb);
    else memcpy(S->pState + T1, pSrc, sb);     // host input, host state: the caller's words
  }
  if (e == hipSuccess) e = io.finish();
  if (e == hipSuccess) hold.synced();
  if (e != hipSuccess) set_error(e, "arm_fir");
}

template <typename T, typename Inst>
arm_status fir_batch(const Inst* S, const T* d_src, T* d_dst, uint32_t B, uint32_t batch, T* d_hist, void* stream,
                     int kind) {
  if (!S || !S->pCoeffs || S->numTaps == 0 || (batch && B && (!d_src || !d_dst))) return ARM_MATH_ARGUMENT_ERROR;
  if (S->numTaps > 1 && batch && !d_hist) return ARM_MATH_ARGUMENT_ERROR;
  hipStream_t st = (hipStream_t)stream;
  BlobScope hold(st);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, S->numTaps, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, "arm_fir_batch coeffs"); return ARM_MATH_ARGUMENT_ERROR; }
  hipError_t e = fir_run(kind, dc, S->numTaps, d_src, d_dst, B, batch, d_hist, st);
  if (e != hipSuccess) { set_error(e, "arm_fir_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// multi-GPU FIR (the batch is sliced by filter, each shard's history rows stay on
// its device): shard s = batch[s] filters at d_src[s] / d_dst[s] / d_hist[s] on devices[s].
template <typename T, typename Inst>
arm_status fir_batch_multi(const Inst* S, uint32_t nshards, const int* devices, const T* const* d_src, T* const* d_dst,
                           T* const* d_hist, uint32_t B, const uint32_t* batch, int kind) {
  if (!S || !S->pCoeffs || S->numTaps == 0 || (nshards && (!devices || !batch || !d_src || !d_dst || !d_hist)))
    return ARM_MATH_ARGUMENT_ERROR;
  for (uint32_t s = 0; s < nshards; ++s)
    if (batch[s] && ((B && (!d_src[s] || !d_dst[s])) || (S->numTaps > 1 && !d_hist[s]))) return ARM_MATH_ARGUMENT_ERROR;
  return run_multi(nshards, devices, batch, "arm_fir_batch_multi", [&](uint32_t s, hipStream_t st) {
    bool ok = true;
    const T* dc = device_coeffs<T>(S->pCoeffs, S->numTaps, &ok);   // uploaded once per device
    if (!ok) return false;
    hipError_t e = fir_run(kind, dc, S->numTaps, d_src[s], d_dst[s], B, batch[s], d_hist[s], st);
    if (e != hipSuccess) { set_error(e, "arm_fir_batch_multi"); return false; }
    return true;
  });
}

// zero a host or device buffer (the init functions' memset)
void zero_words(void* p, size_t bytes, const char* what) {
  if (is_device_ptr(p)) {
    hipError_t e = hipMemset(p, 0, bytes);
    if (e != hipSuccess) set_error(e, what);
  } else {
    memset(p, 0, bytes);
  }
}

// ---- multirate FIR (decimator / interpolator) ----------------------------------------
// Drop-in: state = [history (H) ; block (B)] on host or device; after the call it holds
// [new history ; block input], as the reference leaves it (the block is copied into pState
// before the pass, arm_fir_decimate_f32.c / arm_fir_interpolate_f32.c).  run(dc, src, dst,
// hist, st) launches the batched pass for one stream.
template <typename T, typename Run>
void mr_sync(T* pState, const T* pCoeffs, int ncoef, int H, const T* pSrc, T* pDst, uint32_t B, size_t out_words,
             const char* what, Run&& run) {
  if (!pState || !pCoeffs || ncoef <= 0 || B == 0) return;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  bool ok = true;
  const T* dc = device_coeffs<T>(pCoeffs, ncoef, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, what); return; }
  const bool dstate = is_device_ptr(pState), dsrc = is_device_ptr(pSrc), ddst = is_device_ptr(pDst);
  const size_t sb = sizeof(T) * (size_t)B, hb = sizeof(T) * (size_t)H, ob = sizeof(T) * out_words;
  const bool alias = dsrc && ddst && ranges_overlap(pSrc, pDst, sb > ob ? sb : ob);
  T* dhist = dstate ? pState : (T*)scratch(hb + 16, 2);
  const T* dsr = (dsrc && !alias) ? pSrc : (const T*)scratch(sb, 3);
  T* dds = ddst ? pDst : (T*)scratch(ob + 16, 4);
  if (!dhist || !dsr || !dds) { set_error(hipErrorOutOfMemory, what); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!dstate && H > 0) e = io.in(dhist, pState, hb);
  if (e == hipSuccess && alias) e = hipMemcpyAsync((void*)dsr, pSrc, sb, hipMemcpyDeviceToDevice, st);
  else if (e == hipSuccess && !dsrc) e = io.in((void*)dsr, pSrc, sb);
  if (e == hipSuccess) e = run(dc, dsr, dds, dhist, st);
  if (e == hipSuccess && !ddst && ob) e = io.out(pDst, dds, ob);
  if (e == hipSuccess && !dstate && H > 0) e = io.out(pState, dhist, hb);
  if (e == hipSuccess) {
    if (dstate) e = hipMemcpyAsync(pState + H, dsr, sb, hipMemcpyDeviceToDevice, st);
    else if (dsrc) e = io.out(pState + H, dsr, sb);
    else memcpy(pState + H, pSrc, sb);
  }
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, what);
}

template <typename T, typename Inst>
arm_status decimate_init(Inst* S, uint16_t numTaps, uint8_t M, const T* pCoeffs, T* pState, uint32_t blockSize) {
  if (!S) return ARM_MATH_ARGUMENT_ERROR;
  if (M == 0 || blockSize % M) return ARM_MATH_LENGTH_ERROR;       // arm_fir_decimate_init_f32.c
  S->numTaps = numTaps; S->pCoeffs = pCoeffs; S->pState = pState; S->M = M;
  if (pState) zero_words(pState, sizeof(T) * ((size_t)numTaps + blockSize - 1), "arm_fir_decimate_init");
  return ARM_MATH_SUCCESS;
}
template <typename T, typename Inst>
arm_status interpolate_init(Inst* S, uint8_t L, uint16_t numTaps, const T* pCoeffs, T* pState, uint32_t blockSize) {
  if (!S) return ARM_MATH_ARGUMENT_ERROR;
  if (L == 0 || numTaps % L) return ARM_MATH_LENGTH_ERROR;         // arm_fir_interpolate_init_f32.c
  S->pCoeffs = pCoeffs; S->L = L; S->phaseLength = (uint16_t)(numTaps / L); S->pState = pState;
  if (pState) zero_words(pState, sizeof(T) * ((size_t)blockSize + S->phaseLength - 1), "arm_fir_interpolate_init");
  return ARM_MATH_SUCCESS;
}
template <typename T, typename Inst>
void decimate_sync(const Inst* S, const T* pSrc, T* pDst, uint32_t B, int op, const char* what) {
  if (!S || S->M == 0 || S->numTaps == 0) return;
  const int M = S->M, taps = S->numTaps;
  mr_sync<T>(S->pState, S->pCoeffs, taps, taps - 1, pSrc, pDst, B, B / M, what,
             [&](const T* dc, const T* src, T* dst, T* hist, hipStream_t st) {
               return fir_decimate_run(op, dc, taps, M, src, dst, B, 1, hist, st);
             });
}
template <typename T, typename Inst>
void interpolate_sync(const Inst* S, const T* pSrc, T* pDst, uint32_t B, int op, const char* what) {
  if (!S || S->L == 0 || S->phaseLength == 0) return;
  const int L = S->L, P = S->phaseLength;
  mr_sync<T>(S->pState, S->pCoeffs, L * P, P - 1, pSrc, pDst, B, (size_t)B * L, what,
             [&](const T* dc, const T* src, T* dst, T* hist, hipStream_t st) {
               return fir_interpolate_run(op, dc, L, P, src, dst, B, 1, hist, st);
             });
}
template <typename T, typename Inst>
arm_status decimate_batch(const Inst* S, const T* d_src, T* d_dst, uint32_t B, uint32_t batch, T* d_hist,
                          void* stream, int op, const char* what) {
  if (!S || !S->pCoeffs || S->numTaps == 0 || S->M == 0) return ARM_MATH_ARGUMENT_ERROR;
  if (batch && B && (!d_src || (B >= S->M && !d_dst) || (S->numTaps > 1 && !d_hist))) return ARM_MATH_ARGUMENT_ERROR;
  BlobScope hold((hipStream_t)stream);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, S->numTaps, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, what); return ARM_MATH_ARGUMENT_ERROR; }
  hipError_t e = fir_decimate_run(op, dc, S->numTaps, S->M, d_src, d_dst, B, batch, d_hist, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}
template <typename T, typename Inst>
arm_status interpolate_batch(const Inst* S, const T* d_src, T* d_dst, uint32_t B, uint32_t batch, T* d_hist,
                             void* stream, int op, const char* what) {
  if (!S || !S->pCoeffs || S->phaseLength == 0 || S->L == 0) return ARM_MATH_ARGUMENT_ERROR;
  if (batch && B && (!d_src || !d_dst || (S->phaseLength > 1 && !d_hist))) return ARM_MATH_ARGUMENT_ERROR;
  BlobScope hold((hipStream_t)stream);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, (int)S->L * S->phaseLength, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, what); return ARM_MATH_ARGUMENT_ERROR; }
  hipError_t e = fir_interpolate_run(op, dc, S->L, S->phaseLength, d_src, d_dst, B, batch, d_hist,
                                     (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// ---- sparse FIR ---------------------------------------------------------------------------
// Drop-in: the reference's circular state (L = maxDelay + blockSize words, host or device) gets
// the block at stateIndex (arm_circularWrite_f32), then one kernel reads every tap straight from
// it at the reference's read indices (arm_fir_sparse_f32.c); pScratchIn / pScratchOut are not
// needed.  Host state + host input: the block is written into the caller's state on the host and
// the state uploaded once (the kernel never modifies it).
template <typename T, typename Inst>
void sparse_init(Inst* S, uint16_t numTaps, const T* pCoeffs, T* pState, int32_t* pTapDelay, uint16_t maxDelay,
                 uint32_t blockSize) {
  if (!S) return;
  S->numTaps = numTaps; S->pCoeffs = pCoeffs; S->pTapDelay = pTapDelay; S->maxDelay = maxDelay;
  S->stateIndex = 0;                                                  // arm_fir_sparse_init_f32.c
  if (pState) zero_words(pState, sizeof(T) * ((size_t)maxDelay + blockSize), "arm_fir_sparse_init");
  S->pState = pState;
}

template <typename T, typename Inst>
void sparse_sync(Inst* S, const T* pSrc, T* pDst, uint32_t B, int op, const char* what) {
  if (!S || !S->pState || !S->pCoeffs || !S->pTapDelay || S->numTaps == 0 || B == 0) return;
  const int taps = S->numTaps;
  const uint32_t L = (uint32_t)S->maxDelay + B;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  bool ok = true, okd = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, taps, &ok);
  const int32_t* dd = device_coeffs<int32_t>(S->pTapDelay, taps, &okd);
  if (!ok || !okd) { set_error(hipErrorOutOfMemory, what); return; }
  const bool dstate = is_device_ptr(S->pState), dsrc = is_device_ptr(pSrc), ddst = is_device_ptr(pDst);
  // words moved: the circular length, or up to a stateIndex a larger earlier block left past it
  const size_t es = sizeof(T), sb = es * B, lb = es * std::max<size_t>(L, (size_t)S->stateIndex + 1);
  T* ds = dstate ? S->pState : (T*)scratch(lb + 16, 2);
  // a device output overlapping the state would be read by later taps: write to scratch
  const bool dalias = ddst && dstate && ranges_overlap(pDst, S->pState, lb > sb ? lb : sb);
  T* dds = (ddst && !dalias) ? pDst : (T*)scratch(sb + 16, 4);
  if (!ds || !dds) { set_error(hipErrorOutOfMemory, what); return; }
  // arm_circularWrite_f32 position by position: sample i at w, then w + 1 wrapped once at L
  // (a stateIndex left >= L by a larger earlier blockSize writes there first, as the reference
  // does), as contiguous segments
  auto circular_write = [&](auto&& copy) -> hipError_t {
    int64_t w = S->stateIndex;
    for (uint32_t i = 0; i < B;) {
      const uint32_t n = w >= (int64_t)L ? 1u : (B - i < L - (uint32_t)w ? B - i : L - (uint32_t)w);
      hipError_t e = copy((size_t)w, i, n);
      if (e != hipSuccess) return e;
      i += n;
      w += n;
      if (w >= (int64_t)L) w -= L;
    }
    S->stateIndex = (uint16_t)w;
    return hipSuccess;
  };
  const uint16_t prev = S->stateIndex;
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!dstate && !dsrc) {
    e = circular_write([&](size_t w, uint32_t i, uint32_t n) {
      memcpy(S->pState + w, pSrc + i, es * n);
      return hipSuccess;
    });
    if (e == hipSuccess) e = io.in(ds, S->pState, lb);
  } else {
    if (!dstate) e = io.in(ds, S->pState, lb);
    if (e == hipSuccess)
      e = circular_write([&](size_t w, uint32_t i, uint32_t n) {
        return dsrc ? hipMemcpyAsync(ds + w, pSrc + i, es * n, hipMemcpyDeviceToDevice, st) : io.in(ds + w, pSrc + i, es * n);
      });
  }
  const uint16_t next = S->stateIndex;
  S->stateIndex = prev;                                               // committed on success
  const int r0 = (int32_t)((uint32_t)next - B);                       // arm_fir_sparse_f32.c readIndex
  if (e == hipSuccess) e = fir_sparse_run(op, dc, dd, taps, S->maxDelay, ds, dds, B, 1, nullptr, (int)L, r0, st);
  if (e == hipSuccess && dalias) e = hipMemcpyAsync(pDst, dds, sb, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess && !ddst) e = io.out(pDst, dds, sb);
  if (e == hipSuccess && !dstate && dsrc) e = io.out(S->pState, ds, lb);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) { set_error(e, what); return; }
  S->stateIndex = next;
}

// Batched: `batch` streams with linear histories d_hist[batch][maxDelay] (oldest first,
// updated), delays in [0, maxDelay] (others read 0); stateIndex / pState are not used.
template <typename T, typename Inst>
arm_status sparse_batch(const Inst* S, const T* d_src, T* d_dst, uint32_t B, uint32_t batch, T* d_hist, void* stream,
                        int op, const char* what) {
  if (!S || !S->pCoeffs || !S->pTapDelay || S->numTaps == 0) return ARM_MATH_ARGUMENT_ERROR;
  if (batch && B && (!d_src || !d_dst || (S->maxDelay > 0 && !d_hist))) return ARM_MATH_ARGUMENT_ERROR;
  BlobScope hold((hipStream_t)stream);
  bool ok = true, okd = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, S->numTaps, &ok);
  const int32_t* dd = device_coeffs<int32_t>(S->pTapDelay, S->numTaps, &okd);
  if (!ok || !okd) { set_error(hipErrorOutOfMemory, what); return ARM_MATH_ARGUMENT_ERROR; }
  hipError_t e = fir_sparse_run(op, dc, dd, S->numTaps, S->maxDelay, d_src, d_dst, B, batch, d_hist, 0, 0,
                                (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// ---- FIR lattice ----------------------------------------------------------------------------
// Drop-in: state (numStages words, host or device) in, filter, state out (arm_fir_lattice_f32.c);
// the kernel reads the old state from its own copy, so in-place device state is fine.
template <typename T, typename Inst>
void lattice_init(Inst* S, uint16_t numStages, const T* pCoeffs, T* pState) {
  if (!S) return;
  S->numStages = numStages; S->pCoeffs = pCoeffs; S->pState = pState;     // arm_fir_lattice_init_f32.c
  if (pState && numStages) zero_words(pState, sizeof(T) * numStages, "arm_fir_lattice_init");
}

template <typename T, typename Inst>
void lattice_sync(const Inst* S, const T* pSrc, T* pDst, uint32_t B, int op, const char* what) {
  if (!S || !S->pState || !S->pCoeffs || S->numStages == 0 || B == 0) return;
  const int M = S->numStages;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, M, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, what); return; }
  const bool dstate = is_device_ptr(S->pState), dsrc = is_device_ptr(pSrc), ddst = is_device_ptr(pDst);
  const size_t sb = sizeof(T) * (size_t)B, hb = sizeof(T) * (size_t)M;
  T* dhist = dstate ? S->pState : (T*)scratch(hb + 16, 2);
  const T* dsr = dsrc ? pSrc : (const T*)scratch(sb, 3);
  T* dds = ddst ? pDst : (T*)scratch(sb + 16, 4);
  if (!dhist || !dsr || !dds) { set_error(hipErrorOutOfMemory, what); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!dstate) e = io.in(dhist, S->pState, hb);
  if (e == hipSuccess && !dsrc) e = io.in((void*)dsr, pSrc, sb);
  if (e == hipSuccess) e = fir_lattice_run(op, dc, M, dsr, dds, B, 1, dhist, st);
  if (e == hipSuccess && !ddst) e = io.out(pDst, dds, sb);
  if (e == hipSuccess && !dstate) e = io.out(S->pState, dhist, hb);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, what);
}

template <typename T, typename Inst>
arm_status lattice_batch(const Inst* S, const T* d_src, T* d_dst, uint32_t B, uint32_t batch, T* d_state,
                         void* stream, int op, const char* what) {
  if (!S || !S->pCoeffs || S->numStages == 0) return ARM_MATH_ARGUMENT_ERROR;
  if (batch && B && (!d_src || !d_dst || !d_state)) return ARM_MATH_ARGUMENT_ERROR;
  BlobScope hold((hipStream_t)stream);
  bool ok = true;
  const T* dc = device_coeffs<T>(S->pCoeffs, S->numStages, &ok);
  if (!ok) { set_error(hipErrorOutOfMemory, what); return ARM_MATH_ARGUMENT_ERROR; }
  hipError_t e = fir_lattice_run(op, dc, S->numStages, d_src, d_dst, B, batch, d_state, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// ---- convolution / correlation family ------------------------------------------------
// How each reference function maps onto one ConvJob (conv.hip):
//   conv (exact):      x = pSrcA, h = pSrcB, all srcALen + srcBLen - 1 outputs forward;
//   conv (fast q15/q31): x = the longer input (arm_conv_fast_q15.c:83-103);
//   conv_partial:      outputs [firstIndex, firstIndex + numPoints) at pDst[n];
//   correlate (all):   x = the longer input, h = the shorter reversed; forward at
//                      srcALen - srcBLen, or backward from srcALen + srcBLen - 2 when
//                      srcALen < srcBLen (arm_correlate_f32.c:1040-1070).
// Returns the job and the written output range [wlo, whi) of one item.
enum ConvVariant { kVarConv = 0, kVarPartial = 1, kVarCorr = 2 };
ConvJob conv_plan(int op, int variant, const void* a, uint32_t alen, const void* b, uint32_t blen, uint32_t first,
                  uint32_t num, uint64_t* wlo, uint64_t* whi, bool* swapped) {
  ConvJob j{};
  j.op = op;
  j.corr = variant == kVarCorr;
  const bool swap = (variant == kVarCorr || op == kConvFastQ15 || op == kConvFastQ31) && alen < blen;
  *swapped = swap;
  j.x = swap ? b : a; j.A = swap ? blen : alen;
  j.h = swap ? a : b; j.B = swap ? alen : blen;
  const uint32_t L = alen + blen - 1;
  j.ydir = 1; j.yoff = 0; j.first = 0; j.num = L;
  *wlo = 0; *whi = L;
  if (variant == kVarPartial) {
    j.first = first; j.num = num;
    *wlo = first; *whi = (uint64_t)first + num;
  } else if (variant == kVarCorr) {
    if (alen >= blen) { j.yoff = alen - blen; *wlo = alen - blen; *whi = (uint64_t)j.yoff + L; }
    else { j.yoff = L - 1; j.ydir = -1; }
  }
  return j;
}

// drop-in: host or device operands, synchronous
template <typename T>
void conv_family_sync(int op, int variant, const T* a, uint32_t alen, const T* b, uint32_t blen, T* dst,
                      uint32_t first, uint32_t num, const char* what) {
  if (!a || !b || !dst || alen == 0 || blen == 0) return;
  uint64_t wlo, whi;
  bool swapped = false;
  ConvJob j = conv_plan(op, variant, a, alen, b, blen, first, num, &wlo, &whi, &swapped);
  if (j.num == 0) return;
  const size_t ab = sizeof(T) * alen, bb = sizeof(T) * blen;
  hipStream_t st = sync_stream();
  const bool da = is_device_ptr(a), db = is_device_ptr(b), dd = is_device_ptr(dst);
  const T* A = da ? a : (const T*)scratch(ab, 0);
  const T* B = db ? b : (const T*)scratch(bb, 1);
  T* Y = dd ? dst : (T*)scratch(sizeof(T) * whi, 2);
  if (!A || !B || !Y) { set_error(hipErrorOutOfMemory, what); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!da) e = io.in((void*)A, a, ab);
  if (e == hipSuccess && !db) e = io.in((void*)B, b, bb);
  j.x = swapped ? (const void*)B : (const void*)A;
  j.h = swapped ? (const void*)A : (const void*)B;
  j.y = Y; j.sx = j.sh = j.sy = 0; j.batch = 1;
  if (e == hipSuccess) e = conv_family_run(j, st);
  // only the words the reference writes are copied back (partial / correlate leave the rest)
  if (e == hipSuccess && !dd) e = io.out(dst + wlo, Y + wlo, sizeof(T) * (whi - wlo));
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, what);
}

// batched device API: item i reads a + i*sa, b + i*sb (0 = shared) and writes y + i*sy at
// the drop-in positions, except conv_partial, which writes its numPoints outputs compactly.
template <typename T>
arm_status conv_family_batch(int op, int variant, const T* a, uint32_t alen, uint32_t sa, const T* b, uint32_t blen,
                             uint32_t sb, T* y, uint32_t first, uint32_t num, uint32_t batch, void* stream,
                             const char* what) {
  if (batch && (!a || !b || !y || alen == 0 || blen == 0)) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0) return ARM_MATH_SUCCESS;
  uint64_t wlo, whi;
  bool swapped = false;
  ConvJob j = conv_plan(op, variant, a, alen, b, blen, first, num, &wlo, &whi, &swapped);
  j.sx = swapped ? sb : sa;
  j.sh = swapped ? sa : sb;
  j.y = y; j.batch = batch;
  if (variant == kVarPartial) { j.sy = num; j.yoff = -(int64_t)first; }
  else if (variant == kVarCorr) j.sy = 2ull * (alen > blen ? alen : blen) - 1;
  else j.sy = (uint64_t)alen + blen - 1;
  hipError_t e = conv_family_run(j, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

bool partial_range_ok(uint32_t alen, uint32_t blen, uint32_t first, uint32_t num) {
  // arm_conv_partial_f32.c:644: (firstIndex + numPoints) > (srcALen + (srcBLen - 1))
  return (uint64_t)first + num <= (uint64_t)alen + blen - 1;
}

template <typename M>
bool mat_shapes_ok(const M* a, const M* b, const M* c) {
  return a->numCols == b->numRows && a->numRows == c->numRows && b->numCols == c->numCols;
}

// multi-GPU matrix multiply: shard s = batch[s] matrices (shapes of the instances) at d_a[s],
// d_b[s], d_c[s] on devices[s].  launch(m, k, n, a, b, c, batch, st) is the per-type launcher.
template <typename T, typename M, typename Launch>
arm_status mat_batch_multi(const M* pSrcA, const M* pSrcB, M* pDst, uint32_t nshards, const int* devices,
                           const T* const* d_a, const T* const* d_b, T* const* d_c, const uint32_t* batch,
                           const char* what, Launch&& launch) {
  if (!pSrcA || !pSrcB || !pDst || (nshards && (!devices || !batch || !d_a || !d_b || !d_c))) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  for (uint32_t s = 0; s < nshards; ++s)
    if (batch[s] && (!d_a[s] || !d_b[s] || !d_c[s])) return ARM_MATH_ARGUMENT_ERROR;
  return run_multi(nshards, devices, batch, what, [&](uint32_t s, hipStream_t st) {
    hipError_t e = launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, d_a[s], d_b[s], d_c[s], batch[s], st);
    if (e != hipSuccess) { set_error(e, what); return false; }
    return true;
  });
}

// drop-in fixed-point matrix multiply (host or device operands), synchronous
template <typename T, typename M>
arm_status mat_mult_fixed_sync(const M* pSrcA, const M* pSrcB, M* pDst, bool fast = false) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  const int m = pSrcA->numRows, k = pSrcA->numCols, n = pSrcB->numCols;
  const size_t ab = sizeof(T) * (size_t)m * k, bb = sizeof(T) * (size_t)k * n, cb = sizeof(T) * (size_t)m * n;
  hipStream_t st = sync_stream();
  const bool da = is_device_ptr(pSrcA->pData), db = is_device_ptr(pSrcB->pData), dc = is_device_ptr(pDst->pData);
  T* A = da ? pSrcA->pData : (T*)scratch(ab + 16, 0);
  T* B = db ? pSrcB->pData : (T*)scratch(bb + 16, 1);
  T* Cd = dc ? pDst->pData : (T*)scratch(cb + 16, 2);
  if (!A || !B || !Cd) { set_error(hipErrorOutOfMemory, "arm_mat_mult scratch"); return ARM_MATH_ARGUMENT_ERROR; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!da) e = io.in(A, pSrcA->pData, ab);
  if (e == hipSuccess && !db) e = io.in(B, pSrcB->pData, bb);
  if (e == hipSuccess) {
    if constexpr (sizeof(T) == 1)
      e = mat_mult_q7_launch(m, k, n, A, B, Cd, 1, st);
    else if constexpr (sizeof(T) == 2)
      e = fast ? mat_mult_fast_q15_launch(m, k, n, A, B, Cd, 1, st) : mat_mult_q15_launch(m, k, n, A, B, Cd, 1, st);
    else
      e = fast ? mat_mult_fast_q31_launch(m, k, n, A, B, Cd, 1, st) : mat_mult_q31_launch(m, k, n, A, B, Cd, 1, st);
  }
  if (e == hipSuccess && !dc) e = io.out(pDst->pData, Cd, cb);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) { set_error(e, "arm_mat_mult"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// FIR init: zero numTaps + blockSize - 1 state words (arm_fir_init_f32.c:74-95,
// arm_fir_init_q15.c:119-139, the !ARM_MATH_DSP branch: no even-numTaps check).
// The state buffer is caller memory, host or device.
template <typename T, typename Inst>
void fir_init(Inst* S, uint16_t numTaps, const T* pCoeffs, T* pState, uint32_t blockSize) {
  S->numTaps = numTaps;
  S->pCoeffs = pCoeffs;
  S->pState = pState;
  if (!pState) return;
  const size_t bytes = sizeof(T) * ((size_t)numTaps + blockSize - 1);
  if (is_device_ptr(pState)) {
    hipError_t e = hipMemset(pState, 0, bytes);
    if (e != hipSuccess) set_error(e, "arm_fir_init");
  } else {
    memset(pState, 0, bytes);
  }
}
}  // namespace

extern "C" {

#ifndef MI355X_BUILD_DEFS
#define MI355X_BUILD_DEFS ""
#endif
#ifndef MI355X_SRC_ID
#define MI355X_SRC_ID "unknown"
#endif
// "src:" is the sha256-based id of the sources the library was built from (Makefile SRC_ID);
// "[...]" lists the non-default tuning macros of the build (Makefile DEFS, build_variant.sh)
const char* arm_mi355x_version(void) {
  return sizeof(MI355X_BUILD_DEFS) > 1 ? "cmsisdsp-mi355x 0.3.0 gfx950 src:" MI355X_SRC_ID " [" MI355X_BUILD_DEFS "]"
                                       : "cmsisdsp-mi355x 0.3.0 gfx950 src:" MI355X_SRC_ID;
}

void arm_cfft_f32(const arm_cfft_instance_f32* S, float32_t* p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  cfft_sync(S, p1, ifftFlag, bitReverseFlag, 0, sizeof(float));
}
void arm_cfft_q31(const arm_cfft_instance_q31* S, q31_t* p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  cfft_sync(S, p1, ifftFlag, bitReverseFlag, 1, sizeof(int32_t));
}
void arm_cfft_q15(const arm_cfft_instance_q15* S, q15_t* p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  cfft_sync(S, p1, ifftFlag, bitReverseFlag, 2, sizeof(int16_t));
}

arm_status arm_cfft_f32_batch(const arm_cfft_instance_f32* S, float32_t* d_p1, uint32_t batch, uint8_t ifftFlag,
                              uint8_t bitReverseFlag, void* stream) {
  return cfft_batch(S, d_p1, batch, ifftFlag, bitReverseFlag, stream, 0);
}
arm_status arm_cfft_q31_batch(const arm_cfft_instance_q31* S, q31_t* d_p1, uint32_t batch, uint8_t ifftFlag,
                              uint8_t bitReverseFlag, void* stream) {
  return cfft_batch(S, d_p1, batch, ifftFlag, bitReverseFlag, stream, 1);
}
arm_status arm_cfft_q15_batch(const arm_cfft_instance_q15* S, q15_t* d_p1, uint32_t batch, uint8_t ifftFlag,
                              uint8_t bitReverseFlag, void* stream) {
  return cfft_batch(S, d_p1, batch, ifftFlag, bitReverseFlag, stream, 2);
}

arm_status arm_cfft_f32_batch_multi(const arm_cfft_instance_f32* S, uint32_t nshards, const int* devices,
                                    float32_t* const* d_p1, const uint32_t* batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag) {
  return cfft_batch_multi(S, nshards, devices, (void* const*)d_p1, batch, ifftFlag, bitReverseFlag, 0);
}
arm_status arm_cfft_q31_batch_multi(const arm_cfft_instance_q31* S, uint32_t nshards, const int* devices,
                                    q31_t* const* d_p1, const uint32_t* batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag) {
  return cfft_batch_multi(S, nshards, devices, (void* const*)d_p1, batch, ifftFlag, bitReverseFlag, 1);
}
arm_status arm_cfft_q15_batch_multi(const arm_cfft_instance_q15* S, uint32_t nshards, const int* devices,
                                    q15_t* const* d_p1, const uint32_t* batch, uint8_t ifftFlag,
                                    uint8_t bitReverseFlag) {
  return cfft_batch_multi(S, nshards, devices, (void* const*)d_p1, batch, ifftFlag, bitReverseFlag, 2);
}
int arm_mi355x_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return 0; }
  return n;
}

void arm_rfft_fast_f32(const arm_rfft_fast_instance_f32* S, float32_t* p, float32_t* pOut, uint8_t ifftFlag) {
  if (!S || !p || !pOut || !rfft_len_ok(S->fftLenRFFT)) return;
  const size_t bytes = sizeof(float) * S->fftLenRFFT;
  hipStream_t st = sync_stream();
  const bool dp = is_device_ptr(p), dout = is_device_ptr(pOut);
  float* d_p = dp ? p : (float*)scratch(bytes, 0);
  float* d_o = dout ? pOut : (float*)scratch(bytes, 1);
  if (!d_p || !d_o) { set_error(hipErrorOutOfMemory, "arm_rfft_fast scratch"); return; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!dp) e = io.in(d_p, p, bytes);
  if (e != hipSuccess) { set_error(e, "arm_rfft_fast"); return; }
  if (!rfft_run(S, d_p, d_o, 1, ifftFlag, st)) { (void)hipStreamSynchronize(st); return; }
  if (!dp && !ifftFlag) e = io.out(p, d_p, bytes);   // forward overwrites p
  if (e == hipSuccess && !dout) e = io.out(pOut, d_o, bytes);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, "arm_rfft_fast");
}

arm_status arm_rfft_fast_f32_batch(const arm_rfft_fast_instance_f32* S, float32_t* d_p, float32_t* d_out,
                                   uint32_t batch, uint8_t ifftFlag, void* stream) {
  if (!S || !rfft_len_ok(S->fftLenRFFT) || (batch && (!d_p || !d_out))) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0) return ARM_MATH_SUCCESS;
  return rfft_run(S, d_p, d_out, batch, ifftFlag, (hipStream_t)stream) ? ARM_MATH_SUCCESS : ARM_MATH_ARGUMENT_ERROR;
}
arm_status arm_rfft_fast_f32_batch_ex(const arm_rfft_fast_instance_f32* S, float32_t* d_p, float32_t* d_out,
                                      uint32_t batch, uint8_t ifftFlag, uint32_t flags, void* stream) {
  if (!S || !rfft_len_ok(S->fftLenRFFT) || (batch && (!d_p || !d_out))) return ARM_MATH_ARGUMENT_ERROR;
  if (flags & ~(uint32_t)ARM_MI355X_RFFT_P_SCRATCH) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0) return ARM_MATH_SUCCESS;
  return rfft_run(S, d_p, d_out, batch, ifftFlag, (hipStream_t)stream, (flags & ARM_MI355X_RFFT_P_SCRATCH) != 0)
             ? ARM_MATH_SUCCESS
             : ARM_MATH_ARGUMENT_ERROR;
}

void arm_rfft_q31(const arm_rfft_instance_q31* S, q31_t* pSrc, q31_t* pDst) { rfft_fixed_sync<int32_t>(S, pSrc, pDst); }
void arm_rfft_q15(const arm_rfft_instance_q15* S, q15_t* pSrc, q15_t* pDst) { rfft_fixed_sync<int16_t>(S, pSrc, pDst); }
arm_status arm_rfft_q31_batch(const arm_rfft_instance_q31* S, q31_t* d_src, q31_t* d_dst, uint32_t batch,
                              void* stream) {
  return rfft_fixed_batch<int32_t>(S, d_src, d_dst, batch, stream);
}
arm_status arm_rfft_q15_batch(const arm_rfft_instance_q15* S, q15_t* d_src, q15_t* d_dst, uint32_t batch,
                              void* stream) {
  return rfft_fixed_batch<int16_t>(S, d_src, d_dst, batch, stream);
}

void arm_fir_init_f32(arm_fir_instance_f32* S, uint16_t numTaps, const float32_t* pCoeffs, float32_t* pState,
                      uint32_t blockSize) {
  if (S) fir_init<float>(S, numTaps, pCoeffs, pState, blockSize);
}
arm_status arm_fir_init_q15(arm_fir_instance_q15* S, uint16_t numTaps, const q15_t* pCoeffs, q15_t* pState,
                            uint32_t blockSize) {
  if (!S) return ARM_MATH_ARGUMENT_ERROR;
  fir_init<int16_t>(S, numTaps, pCoeffs, pState, blockSize);
  return ARM_MATH_SUCCESS;
}

void arm_fir_init_q31(arm_fir_instance_q31* S, uint16_t numTaps, const q31_t* pCoeffs, q31_t* pState,
                      uint32_t blockSize) {
  if (S) fir_init<int32_t>(S, numTaps, pCoeffs, pState, blockSize);
}

void arm_fir_init_q7(arm_fir_instance_q7* S, uint16_t numTaps, const q7_t* pCoeffs, q7_t* pState,
                     uint32_t blockSize) {
  if (S) fir_init<int8_t>(S, numTaps, pCoeffs, pState, blockSize);
}

void arm_fir_f32(const arm_fir_instance_f32* S, const float32_t* pSrc, float32_t* pDst, uint32_t blockSize) {
  fir_sync<float>(S, pSrc, pDst, blockSize, kFirF32);
}
void arm_fir_q7(const arm_fir_instance_q7* S, const q7_t* pSrc, q7_t* pDst, uint32_t blockSize) {
  fir_sync<int8_t>(S, pSrc, pDst, blockSize, kFirQ7);
}
void arm_fir_q15(const arm_fir_instance_q15* S, const q15_t* pSrc, q15_t* pDst, uint32_t blockSize) {
  fir_sync<int16_t>(S, pSrc, pDst, blockSize, kFirQ15);
}
void arm_fir_fast_q15(const arm_fir_instance_q15* S, const q15_t* pSrc, q15_t* pDst, uint32_t blockSize) {
  fir_sync<int16_t>(S, pSrc, pDst, blockSize, kFirFastQ15);
}
void arm_fir_q31(const arm_fir_instance_q31* S, const q31_t* pSrc, q31_t* pDst, uint32_t blockSize) {
  fir_sync<int32_t>(S, pSrc, pDst, blockSize, kFirQ31);
}
void arm_fir_fast_q31(const arm_fir_instance_q31* S, const q31_t* pSrc, q31_t* pDst, uint32_t blockSize) {
  fir_sync<int32_t>(S, pSrc, pDst, blockSize, kFirFastQ31);
}
arm_status arm_fir_f32_batch(const arm_fir_instance_f32* S, const float32_t* d_src, float32_t* d_dst,
                             uint32_t blockSize, uint32_t batch, float32_t* d_hist, void* stream) {
  return fir_batch<float>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirF32);
}
arm_status arm_fir_f32_batch_fma(const arm_fir_instance_f32* S, const float32_t* d_src, float32_t* d_dst,
                                 uint32_t blockSize, uint32_t batch, float32_t* d_hist, void* stream) {
  return fir_batch<float>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirF32Fma);
}
arm_status arm_fir_q15_batch(const arm_fir_instance_q15* S, const q15_t* d_src, q15_t* d_dst, uint32_t blockSize,
                             uint32_t batch, q15_t* d_hist, void* stream) {
  return fir_batch<int16_t>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirQ15);
}
arm_status arm_fir_fast_q15_batch(const arm_fir_instance_q15* S, const q15_t* d_src, q15_t* d_dst, uint32_t blockSize,
                                  uint32_t batch, q15_t* d_hist, void* stream) {
  return fir_batch<int16_t>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirFastQ15);
}
arm_status arm_fir_q31_batch(const arm_fir_instance_q31* S, const q31_t* d_src, q31_t* d_dst, uint32_t blockSize,
                             uint32_t batch, q31_t* d_hist, void* stream) {
  return fir_batch<int32_t>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirQ31);
}
arm_status arm_fir_fast_q31_batch(const arm_fir_instance_q31* S, const q31_t* d_src, q31_t* d_dst, uint32_t blockSize,
                                  uint32_t batch, q31_t* d_hist, void* stream) {
  return fir_batch<int32_t>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirFastQ31);
}
arm_status arm_fir_q7_batch(const arm_fir_instance_q7* S, const q7_t* d_src, q7_t* d_dst, uint32_t blockSize,
                            uint32_t batch, q7_t* d_hist, void* stream) {
  return fir_batch<int8_t>(S, d_src, d_dst, blockSize, batch, d_hist, stream, kFirQ7);
}

#define MI355X_FIR_MULTI(NAME, INST, T, CT, KIND)                                                          \
  arm_status NAME##_batch_multi(const INST* S, uint32_t nshards, const int* devices, const T* const* d_src, \
                                T* const* d_dst, T* const* d_hist, uint32_t blockSize, const uint32_t* batch) { \
    return fir_batch_multi<CT>(S, nshards, devices, (const CT* const*)d_src, (CT* const*)d_dst,          \
                               (CT* const*)d_hist, blockSize, batch, KIND);                              \
  }
MI355X_FIR_MULTI(arm_fir_f32, arm_fir_instance_f32, float32_t, float, kFirF32)
MI355X_FIR_MULTI(arm_fir_q15, arm_fir_instance_q15, q15_t, int16_t, kFirQ15)
MI355X_FIR_MULTI(arm_fir_fast_q15, arm_fir_instance_q15, q15_t, int16_t, kFirFastQ15)
MI355X_FIR_MULTI(arm_fir_q31, arm_fir_instance_q31, q31_t, int32_t, kFirQ31)
MI355X_FIR_MULTI(arm_fir_fast_q31, arm_fir_instance_q31, q31_t, int32_t, kFirFastQ31)
MI355X_FIR_MULTI(arm_fir_q7, arm_fir_instance_q7, q7_t, int8_t, kFirQ7)
#undef MI355X_FIR_MULTI

arm_status arm_mat_mult_f32_batch_multi(const arm_matrix_instance_f32* pSrcA, const arm_matrix_instance_f32* pSrcB,
                                        arm_matrix_instance_f32* pDst, uint32_t nshards, const int* devices,
                                        const float32_t* const* d_a, const float32_t* const* d_b,
                                        float32_t* const* d_c, const uint32_t* batch) {
  return mat_batch_multi<float>(pSrcA, pSrcB, pDst, nshards, devices, d_a, d_b, d_c, batch,
                                "arm_mat_mult_f32_batch_multi", mat_mult_f32_launch);
}
arm_status arm_mat_mult_q7_batch_multi(const arm_matrix_instance_q7* pSrcA, const arm_matrix_instance_q7* pSrcB,
                                       arm_matrix_instance_q7* pDst, uint32_t nshards, const int* devices,
                                       const q7_t* const* d_a, const q7_t* const* d_b, q7_t* const* d_c,
                                       const uint32_t* batch) {
  return mat_batch_multi<int8_t>(pSrcA, pSrcB, pDst, nshards, devices, d_a, d_b, d_c, batch,
                                 "arm_mat_mult_q7_batch_multi", mat_mult_q7_launch);
}
arm_status arm_mat_mult_q15_batch_multi(const arm_matrix_instance_q15* pSrcA, const arm_matrix_instance_q15* pSrcB,
                                        arm_matrix_instance_q15* pDst, uint32_t nshards, const int* devices,
                                        const q15_t* const* d_a, const q15_t* const* d_b, q15_t* const* d_c,
                                        const uint32_t* batch) {
  return mat_batch_multi<int16_t>(pSrcA, pSrcB, pDst, nshards, devices, d_a, d_b, d_c, batch,
                                  "arm_mat_mult_q15_batch_multi", mat_mult_q15_launch);
}
arm_status arm_mat_mult_q31_batch_multi(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                                        arm_matrix_instance_q31* pDst, uint32_t nshards, const int* devices,
                                        const q31_t* const* d_a, const q31_t* const* d_b, q31_t* const* d_c,
                                        const uint32_t* batch) {
  return mat_batch_multi<int32_t>(pSrcA, pSrcB, pDst, nshards, devices, d_a, d_b, d_c, batch,
                                  "arm_mat_mult_q31_batch_multi", mat_mult_q31_launch);
}

arm_status arm_mat_mult_f32(const arm_matrix_instance_f32* pSrcA, const arm_matrix_instance_f32* pSrcB,
                            arm_matrix_instance_f32* pDst) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  const int m = pSrcA->numRows, k = pSrcA->numCols, n = pSrcB->numCols;
  const size_t ab = sizeof(float) * (size_t)m * k, bb = sizeof(float) * (size_t)k * n, cb = sizeof(float) * (size_t)m * n;
  hipStream_t st = sync_stream();
  const bool da = is_device_ptr(pSrcA->pData), db = is_device_ptr(pSrcB->pData), dc = is_device_ptr(pDst->pData);
  float* A = da ? pSrcA->pData : (float*)scratch(ab + 16, 0);
  float* B = db ? pSrcB->pData : (float*)scratch(bb + 16, 1);
  float* C = dc ? pDst->pData : (float*)scratch(cb + 16, 2);
  if (!A || !B || !C) { set_error(hipErrorOutOfMemory, "arm_mat_mult scratch"); return ARM_MATH_ARGUMENT_ERROR; }
  HostIO io(st);
  hipError_t e = hipSuccess;
  if (!da) e = io.in(A, pSrcA->pData, ab);
  if (e == hipSuccess && !db) e = io.in(B, pSrcB->pData, bb);
  if (e == hipSuccess) e = mat_mult_f32_launch(m, k, n, A, B, C, 1, st);
  if (e == hipSuccess && !dc) e = io.out(pDst->pData, C, cb);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_f32"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

arm_status arm_mat_mult_f32_batch(const arm_matrix_instance_f32* pSrcA, const arm_matrix_instance_f32* pSrcB,
                                  arm_matrix_instance_f32* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_f32_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData, pSrcB->pData,
                                     pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_f32_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// ---- MFCC f32 (drop-in + batched) ------------------------------------------------
void arm_mfcc_f32(const arm_mfcc_instance_f32* S, float32_t* pSrc, float32_t* pDst, float32_t* pTmp) {
  (void)pTmp;   // work space lives on the device; the reference's pTmp contents are not reproduced
  if (!S || !pSrc || !pDst || S->nbDctOutputs == 0) return;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  MfccDev d;
  if (!mfcc_prepare(S, d)) return;
  const uint32_t n = S->fftLen, nd = S->nbDctOutputs;
  float* x = (float*)scratch(sizeof(float) * n, 0);
  float* y = (float*)scratch(sizeof(float) * n, 1);
  const bool ddst = is_device_ptr(pDst);
  float* o = ddst ? pDst : (float*)scratch(sizeof(float) * nd, 2);
  if (!x || !y || !o) { set_error(hipErrorOutOfMemory, "arm_mfcc scratch"); return; }
  HostIO io(st);
  hipError_t e = is_device_ptr(pSrc) ? hipMemcpyAsync(x, pSrc, sizeof(float) * n, hipMemcpyDeviceToDevice, st)
                                     : io.in(x, pSrc, sizeof(float) * n);
  if (e != hipSuccess) { set_error(e, "arm_mfcc_f32"); return; }
  if (!mfcc_run(S, d, x, y, o, 1, st)) { (void)hipStreamSynchronize(st); return; }
  if (!ddst) e = io.out(pDst, o, sizeof(float) * nd);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) set_error(e, "arm_mfcc_f32");
}

arm_status arm_mfcc_f32_batch(const arm_mfcc_instance_f32* S, float32_t* d_src, float32_t* d_dst, float32_t* d_tmp,
                              uint32_t batch, void* stream) {
  if (!S || (batch && (!d_src || !d_dst || !d_tmp))) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0 || S->nbDctOutputs == 0) return ARM_MATH_SUCCESS;
  BlobScope hold((hipStream_t)stream);
  MfccDev d;
  if (!mfcc_prepare(S, d)) return ARM_MATH_ARGUMENT_ERROR;
  return mfcc_run(S, d, d_src, d_tmp, d_dst, batch, (hipStream_t)stream) ? ARM_MATH_SUCCESS : ARM_MATH_ARGUMENT_ERROR;
}

// ---- MFCC q31 / q15 (drop-in + batched) -----------------------------------------
// Drop-in: the reference's pSrc / pTmp work contents are not reproduced (device scratch).
}  // extern "C"
template <typename T, typename Inst>
static arm_status mfcc_fx_dropin(const Inst* S, T* pSrc, T* pDst, const char* what) {
  if (!S || !pSrc || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (S->nbDctOutputs == 0) return ARM_MATH_SUCCESS;
  hipStream_t st = sync_stream();
  BlobScope hold(st);
  MfccFxDev<T> d;
  if (!mfcc_fx_prepare<T>(S, d)) return ARM_MATH_ARGUMENT_ERROR;
  const uint32_t n = S->fftLen, nd = S->nbDctOutputs;
  T* x = (T*)scratch(sizeof(T) * n, 0);
  T* y = (T*)scratch(sizeof(T) * 2 * n, 1);
  const bool ddst = is_device_ptr(pDst);
  T* o = ddst ? pDst : (T*)scratch(sizeof(T) * nd, 2);
  if (!x || !y || !o) { set_error(hipErrorOutOfMemory, what); return ARM_MATH_ARGUMENT_ERROR; }
  HostIO io(st);
  hipError_t e = is_device_ptr(pSrc) ? hipMemcpyAsync(x, pSrc, sizeof(T) * n, hipMemcpyDeviceToDevice, st)
                                     : io.in(x, pSrc, sizeof(T) * n);
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  if (!mfcc_fx_run<T>(S, d, x, y, o, 1, st)) { (void)hipStreamSynchronize(st); return ARM_MATH_ARGUMENT_ERROR; }
  if (!ddst) e = io.out(pDst, o, sizeof(T) * nd);
  if (e == hipSuccess) e = io.finish();
  if (e != hipSuccess) { set_error(e, what); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

template <typename T, typename Inst>
static arm_status mfcc_fx_batch(const Inst* S, T* d_src, T* d_dst, T* d_tmp, uint32_t batch, void* stream) {
  if (!S || (batch && (!d_src || !d_dst || !d_tmp))) return ARM_MATH_ARGUMENT_ERROR;
  if (batch == 0 || S->nbDctOutputs == 0) return ARM_MATH_SUCCESS;
  BlobScope hold((hipStream_t)stream);
  MfccFxDev<T> d;
  if (!mfcc_fx_prepare<T>(S, d)) return ARM_MATH_ARGUMENT_ERROR;
  return mfcc_fx_run<T>(S, d, d_src, d_tmp, d_dst, batch, (hipStream_t)stream) ? ARM_MATH_SUCCESS
                                                                                : ARM_MATH_ARGUMENT_ERROR;
}
extern "C" {

arm_status arm_mfcc_q31(const arm_mfcc_instance_q31* S, q31_t* pSrc, q31_t* pDst, q31_t* pTmp) {
  (void)pTmp;
  return mfcc_fx_dropin<int32_t>(S, pSrc, pDst, "arm_mfcc_q31");
}
arm_status arm_mfcc_q31_batch(const arm_mfcc_instance_q31* S, q31_t* d_src, q31_t* d_dst, q31_t* d_tmp,
                              uint32_t batch, void* stream) {
  return mfcc_fx_batch<int32_t>(S, d_src, d_dst, d_tmp, batch, stream);
}
arm_status arm_mfcc_q15(const arm_mfcc_instance_q15* S, q15_t* pSrc, q15_t* pDst, q31_t* pTmp) {
  (void)pTmp;
  return mfcc_fx_dropin<int16_t>(S, pSrc, pDst, "arm_mfcc_q15");
}
arm_status arm_mfcc_q15_batch(const arm_mfcc_instance_q15* S, q15_t* d_src, q15_t* d_dst, q15_t* d_tmp,
                              uint32_t batch, void* stream) {
  return mfcc_fx_batch<int16_t>(S, d_src, d_dst, d_tmp, batch, stream);
}

// ---- matrix multiply q7 / q15 / q31 ---------------------------------------------
// arm_mat_mult_q7.c:689-790 (scalar branch): q31_t sum of exact q7 products (never wraps for
// uint16_t dimensions), (q7)__SSAT(sum >> 7, 8); pState (the Helium/Neon transpose buffer) unused.
arm_status arm_mat_mult_q7(const arm_matrix_instance_q7* pSrcA, const arm_matrix_instance_q7* pSrcB,
                           arm_matrix_instance_q7* pDst, q7_t* pState) {
  (void)pState;
  return mat_mult_fixed_sync<int8_t>(pSrcA, pSrcB, pDst);
}
arm_status arm_mat_mult_q7_batch(const arm_matrix_instance_q7* pSrcA, const arm_matrix_instance_q7* pSrcB,
                                 arm_matrix_instance_q7* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_q7_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData, pSrcB->pData,
                                    pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_q7_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}
arm_status arm_mat_mult_q15(const arm_matrix_instance_q15* pSrcA, const arm_matrix_instance_q15* pSrcB,
                            arm_matrix_instance_q15* pDst, q15_t* pState) {
  (void)pState;   // the reference's transpose buffer (ARM_MATH_DSP branch only)
  return mat_mult_fixed_sync<int16_t>(pSrcA, pSrcB, pDst);
}
arm_status arm_mat_mult_q31(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                            arm_matrix_instance_q31* pDst) {
  return mat_mult_fixed_sync<int32_t>(pSrcA, pSrcB, pDst);
}
// arm_mat_mult_opt_q31.c:648-780 (the host build's scalar branch): the q31 product above; pState
// (the Helium branch's transpose buffer) is unused there too.
arm_status arm_mat_mult_opt_q31(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                                arm_matrix_instance_q31* pDst, q31_t* pState) {
  (void)pState;
  return mat_mult_fixed_sync<int32_t>(pSrcA, pSrcB, pDst);
}
// arm_mat_mult_fast_q15.c:351-401 (!ARM_MATH_DSP: q31_t modular sum, (q15)(sum >> 15)),
// arm_mat_mult_fast_q31.c:152-166 (per-product high word, sum << 1); pState unused (the
// reference's transpose buffer).
arm_status arm_mat_mult_fast_q15(const arm_matrix_instance_q15* pSrcA, const arm_matrix_instance_q15* pSrcB,
                                 arm_matrix_instance_q15* pDst, q15_t* pState) {
  (void)pState;
  return mat_mult_fixed_sync<int16_t>(pSrcA, pSrcB, pDst, true);
}
arm_status arm_mat_mult_fast_q31(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                                 arm_matrix_instance_q31* pDst) {
  return mat_mult_fixed_sync<int32_t>(pSrcA, pSrcB, pDst, true);
}
arm_status arm_mat_mult_fast_q15_batch(const arm_matrix_instance_q15* pSrcA, const arm_matrix_instance_q15* pSrcB,
                                       arm_matrix_instance_q15* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_fast_q15_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData,
                                          pSrcB->pData, pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_fast_q15_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}
arm_status arm_mat_mult_fast_q31_batch(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                                       arm_matrix_instance_q31* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_fast_q31_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData,
                                          pSrcB->pData, pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_fast_q31_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}
arm_status arm_mat_mult_q15_batch(const arm_matrix_instance_q15* pSrcA, const arm_matrix_instance_q15* pSrcB,
                                  arm_matrix_instance_q15* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_q15_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData, pSrcB->pData,
                                     pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_q15_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}
arm_status arm_mat_mult_q31_batch(const arm_matrix_instance_q31* pSrcA, const arm_matrix_instance_q31* pSrcB,
                                  arm_matrix_instance_q31* pDst, uint32_t batch, void* stream) {
  if (!pSrcA || !pSrcB || !pDst) return ARM_MATH_ARGUMENT_ERROR;
  if (!mat_shapes_ok(pSrcA, pSrcB, pDst)) return ARM_MATH_SIZE_MISMATCH;
  hipError_t e = mat_mult_q31_launch(pSrcA->numRows, pSrcA->numCols, pSrcB->numCols, pSrcA->pData, pSrcB->pData,
                                     pDst->pData, batch, (hipStream_t)stream);
  if (e != hipSuccess) { set_error(e, "arm_mat_mult_q31_batch"); return ARM_MATH_ARGUMENT_ERROR; }
  return ARM_MATH_SUCCESS;
}

// ---- convolution ------------------------------------------------------------------
#define MI355X_CONV_FULL(NAME, T, CT, OP, VAR)                                                                  \
  void NAME(const T* pSrcA, uint32_t srcALen, const T* pSrcB, uint32_t srcBLen, T* pDst) {                      \
    conv_family_sync<CT>(OP, VAR, (const CT*)pSrcA, srcALen, (const CT*)pSrcB, srcBLen, (CT*)pDst, 0, 0, #NAME); \
  }                                                                                                             \
  arm_status NAME##_batch(const T* d_a, uint32_t srcALen, uint32_t strideA, const T* d_b, uint32_t srcBLen,     \
                          uint32_t strideB, T* d_dst, uint32_t batch, void* stream) {                           \
    return conv_family_batch<CT>(OP, VAR, (const CT*)d_a, srcALen, strideA, (const CT*)d_b, srcBLen, strideB,   \
                                 (CT*)d_dst, 0, 0, batch, stream, #NAME "_batch");                              \
  }
MI355X_CONV_FULL(arm_conv_f32, float32_t, float, kConvF32, kVarConv)
MI355X_CONV_FULL(arm_conv_q15, q15_t, int16_t, kConvQ15, kVarConv)
MI355X_CONV_FULL(arm_conv_q31, q31_t, int32_t, kConvQ31, kVarConv)
MI355X_CONV_FULL(arm_conv_fast_q15, q15_t, int16_t, kConvFastQ15, kVarConv)
MI355X_CONV_FULL(arm_conv_fast_q31, q31_t, int32_t, kConvFastQ31, kVarConv)
MI355X_CONV_FULL(arm_correlate_f32, float32_t, float, kConvF32, kVarCorr)
MI355X_CONV_FULL(arm_correlate_q15, q15_t, int16_t, kConvQ15, kVarCorr)
MI355X_CONV_FULL(arm_correlate_q31, q31_t, int32_t, kConvQ31, kVarCorr)
MI355X_CONV_FULL(arm_correlate_fast_q15, q15_t, int16_t, kConvFastQ15, kVarCorr)
MI355X_CONV_FULL(arm_correlate_fast_q31, q31_t, int32_t, kConvFastQ31, kVarCorr)
MI355X_CONV_FULL(arm_conv_q7, q7_t, int8_t, kConvQ7, kVarConv)
MI355X_CONV_FULL(arm_correlate_q7, q7_t, int8_t, kConvQ7, kVarCorr)
#undef MI355X_CONV_FULL

#define MI355X_CONV_PARTIAL(NAME, T, CT, OP)                                                                       \
  arm_status NAME(const T* pSrcA, uint32_t srcALen, const T* pSrcB, uint32_t srcBLen, T* pDst, uint32_t firstIndex, \
                  uint32_t numPoints) {                                                                            \
    if (!partial_range_ok(srcALen, srcBLen, firstIndex, numPoints)) return ARM_MATH_ARGUMENT_ERROR;                \
    conv_family_sync<CT>(OP, kVarPartial, (const CT*)pSrcA, srcALen, (const CT*)pSrcB, srcBLen, (CT*)pDst,         \
                         firstIndex, numPoints, #NAME);                                                            \
    return ARM_MATH_SUCCESS;                                                                                       \
  }                                                                                                                \
  arm_status NAME##_batch(const T* d_a, uint32_t srcALen, uint32_t strideA, const T* d_b, uint32_t srcBLen,        \
                          uint32_t strideB, T* d_dst, uint32_t firstIndex, uint32_t numPoints, uint32_t batch,     \
                          void* stream) {                                                                          \
    if (!partial_range_ok(srcALen, srcBLen, firstIndex, numPoints)) return ARM_MATH_ARGUMENT_ERROR;                \
    return conv_family_batch<CT>(OP, kVarPartial, (const CT*)d_a, srcALen, strideA, (const CT*)d_b, srcBLen,       \
                                 strideB, (CT*)d_dst, firstIndex, numPoints, batch, stream, #NAME "_batch");       \
  }
MI355X_CONV_PARTIAL(arm_conv_partial_f32, float32_t, float, kConvF32)
MI355X_CONV_PARTIAL(arm_conv_partial_q15, q15_t, int16_t, kConvQ15)
MI355X_CONV_PARTIAL(arm_conv_partial_q31, q31_t, int32_t, kConvQ31)
MI355X_CONV_PARTIAL(arm_conv_partial_q7, q7_t, int8_t, kConvQ7)
// arm_conv_partial_fast_q15 / _q31: outputs firstIndex .. of arm_conv_fast_q15 / _q31.  The
// reference's own bodies (arm_conv_partial_fast_q15.c:110-118 stage sizes) read outside the
// inputs for most ranges (the host build segfaults: tools/probes/conv_family_model.py), so
// the contract is the documented one: the fast convolution's words over the range.
MI355X_CONV_PARTIAL(arm_conv_partial_fast_q15, q15_t, int16_t, kConvFastQ15)
MI355X_CONV_PARTIAL(arm_conv_partial_fast_q31, q31_t, int32_t, kConvFastQ31)
#undef MI355X_CONV_PARTIAL

// The scratch-buffer ("_opt") forms (arm_conv_opt_q15.c, arm_conv_opt_q7.c,
// arm_correlate_opt_q15.c, arm_correlate_opt_q7.c, arm_conv_partial_opt_q15.c, _q7.c): the
// exact sums of the plain functions (tests/test_conv_opt.py pins that on the reference build),
// so they run the same kernels; the fast q15 ones are a modular sum with a saturating output
// (kConvFastOptQ15).  The scratch buffers are not needed.
void arm_conv_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen, q15_t* pDst,
                      q15_t* pScratch1, q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  arm_conv_q15(pSrcA, srcALen, pSrcB, srcBLen, pDst);
}
void arm_conv_opt_q7(const q7_t* pSrcA, uint32_t srcALen, const q7_t* pSrcB, uint32_t srcBLen, q7_t* pDst,
                     q15_t* pScratch1, q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  arm_conv_q7(pSrcA, srcALen, pSrcB, srcBLen, pDst);
}
void arm_correlate_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen, q15_t* pDst,
                           q15_t* pScratch) {
  (void)pScratch;
  arm_correlate_q15(pSrcA, srcALen, pSrcB, srcBLen, pDst);
}
void arm_correlate_opt_q7(const q7_t* pSrcA, uint32_t srcALen, const q7_t* pSrcB, uint32_t srcBLen, q7_t* pDst,
                          q15_t* pScratch1, q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  arm_correlate_q7(pSrcA, srcALen, pSrcB, srcBLen, pDst);
}
arm_status arm_conv_partial_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen,
                                    q15_t* pDst, uint32_t firstIndex, uint32_t numPoints, q15_t* pScratch1,
                                    q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  return arm_conv_partial_q15(pSrcA, srcALen, pSrcB, srcBLen, pDst, firstIndex, numPoints);
}
arm_status arm_conv_partial_opt_q7(const q7_t* pSrcA, uint32_t srcALen, const q7_t* pSrcB, uint32_t srcBLen,
                                   q7_t* pDst, uint32_t firstIndex, uint32_t numPoints, q15_t* pScratch1,
                                   q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  return arm_conv_partial_q7(pSrcA, srcALen, pSrcB, srcBLen, pDst, firstIndex, numPoints);
}
void arm_conv_fast_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen, q15_t* pDst,
                           q15_t* pScratch1, q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  conv_family_sync<int16_t>(kConvFastOptQ15, kVarConv, pSrcA, srcALen, pSrcB, srcBLen, pDst, 0, 0,
                            "arm_conv_fast_opt_q15");
}
void arm_correlate_fast_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen,
                                q15_t* pDst, q15_t* pScratch) {
  (void)pScratch;
  conv_family_sync<int16_t>(kConvFastOptQ15, kVarCorr, pSrcA, srcALen, pSrcB, srcBLen, pDst, 0, 0,
                            "arm_correlate_fast_opt_q15");
}
arm_status arm_conv_partial_fast_opt_q15(const q15_t* pSrcA, uint32_t srcALen, const q15_t* pSrcB, uint32_t srcBLen,
                                         q15_t* pDst, uint32_t firstIndex, uint32_t numPoints, q15_t* pScratch1,
                                         q15_t* pScratch2) {
  (void)pScratch1; (void)pScratch2;
  if (!partial_range_ok(srcALen, srcBLen, firstIndex, numPoints)) return ARM_MATH_ARGUMENT_ERROR;
  conv_family_sync<int16_t>(kConvFastOptQ15, kVarPartial, pSrcA, srcALen, pSrcB, srcBLen, pDst, firstIndex,
                            numPoints, "arm_conv_partial_fast_opt_q15");
  return ARM_MATH_SUCCESS;
}

// ---- multirate FIR ---------------------------------------------------------------------
arm_status arm_fir_decimate_init_f32(arm_fir_decimate_instance_f32* S, uint16_t numTaps, uint8_t M,
                                     const float32_t* pCoeffs, float32_t* pState, uint32_t blockSize) {
  return decimate_init<float>(S, numTaps, M, pCoeffs, pState, blockSize);
}
arm_status arm_fir_decimate_init_q15(arm_fir_decimate_instance_q15* S, uint16_t numTaps, uint8_t M,
                                     const q15_t* pCoeffs, q15_t* pState, uint32_t blockSize) {
  return decimate_init<int16_t>(S, numTaps, M, pCoeffs, pState, blockSize);
}
arm_status arm_fir_decimate_init_q31(arm_fir_decimate_instance_q31* S, uint16_t numTaps, uint8_t M,
                                     const q31_t* pCoeffs, q31_t* pState, uint32_t blockSize) {
  return decimate_init<int32_t>(S, numTaps, M, pCoeffs, pState, blockSize);
}
arm_status arm_fir_interpolate_init_f32(arm_fir_interpolate_instance_f32* S, uint8_t L, uint16_t numTaps,
                                        const float32_t* pCoeffs, float32_t* pState, uint32_t blockSize) {
  return interpolate_init<float>(S, L, numTaps, pCoeffs, pState, blockSize);
}
arm_status arm_fir_interpolate_init_q15(arm_fir_interpolate_instance_q15* S, uint8_t L, uint16_t numTaps,
                                        const q15_t* pCoeffs, q15_t* pState, uint32_t blockSize) {
  return interpolate_init<int16_t>(S, L, numTaps, pCoeffs, pState, blockSize);
}
arm_status arm_fir_interpolate_init_q31(arm_fir_interpolate_instance_q31* S, uint8_t L, uint16_t numTaps,
                                        const q31_t* pCoeffs, q31_t* pState, uint32_t blockSize) {
  return interpolate_init<int32_t>(S, L, numTaps, pCoeffs, pState, blockSize);
}
#define MI355X_DECIM(NAME, INST, T, CT, OP)                                                              \
  void NAME(const INST* S, const T* pSrc, T* pDst, uint32_t blockSize) {                                \
    decimate_sync<CT>(S, (const CT*)pSrc, (CT*)pDst, blockSize, OP, #NAME);                             \
  }                                                                                                     \
  arm_status NAME##_batch(const INST* S, const T* d_src, T* d_dst, uint32_t blockSize, uint32_t batch,  \
                          T* d_hist, void* stream) {                                                    \
    return decimate_batch<CT>(S, (const CT*)d_src, (CT*)d_dst, blockSize, batch, (CT*)d_hist, stream, OP, \
                              #NAME "_batch");                                                          \
  }
MI355X_DECIM(arm_fir_decimate_f32, arm_fir_decimate_instance_f32, float32_t, float, kMrF32)
MI355X_DECIM(arm_fir_decimate_q15, arm_fir_decimate_instance_q15, q15_t, int16_t, kMrQ15)
MI355X_DECIM(arm_fir_decimate_fast_q15, arm_fir_decimate_instance_q15, q15_t, int16_t, kMrFastQ15)
MI355X_DECIM(arm_fir_decimate_q31, arm_fir_decimate_instance_q31, q31_t, int32_t, kMrQ31)
MI355X_DECIM(arm_fir_decimate_fast_q31, arm_fir_decimate_instance_q31, q31_t, int32_t, kMrFastQ31)
#undef MI355X_DECIM
#define MI355X_INTERP(NAME, INST, T, CT, OP)                                                             \
  void NAME(const INST* S, const T* pSrc, T* pDst, uint32_t blockSize) {                                \
    interpolate_sync<CT>(S, (const CT*)pSrc, (CT*)pDst, blockSize, OP, #NAME);                          \
  }                                                                                                     \
  arm_status NAME##_batch(const INST* S, const T* d_src, T* d_dst, uint32_t blockSize, uint32_t batch,  \
                          T* d_hist, void* stream) {                                                    \
    return interpolate_batch<CT>(S, (const CT*)d_src, (CT*)d_dst, blockSize, batch, (CT*)d_hist, stream, OP, \
                                 #NAME "_batch");                                                       \
  }
MI355X_INTERP(arm_fir_interpolate_f32, arm_fir_interpolate_instance_f32, float32_t, float, kMrF32)
MI355X_INTERP(arm_fir_interpolate_q15, arm_fir_interpolate_instance_q15, q15_t, int16_t, kMrQ15)
MI355X_INTERP(arm_fir_interpolate_q31, arm_fir_interpolate_instance_q31, q31_t, int32_t, kMrQ31)
#undef MI355X_INTERP

#define MI355X_SPARSE(T, CT, OP)                                                                        \
  void arm_fir_sparse_init_##T(arm_fir_sparse_instance_##T* S, uint16_t numTaps, const CT* pCoeffs, CT* pState, \
                               int32_t* pTapDelay, uint16_t maxDelay, uint32_t blockSize) {            \
    sparse_init(S, numTaps, pCoeffs, pState, pTapDelay, maxDelay, blockSize);                           \
  }                                                                                                     \
  arm_status arm_fir_sparse_##T##_batch(const arm_fir_sparse_instance_##T* S, const CT* d_src, CT* d_dst, \
                                        uint32_t blockSize, uint32_t batch, CT* d_hist, void* stream) { \
    return sparse_batch(S, d_src, d_dst, blockSize, batch, d_hist, stream, OP, "arm_fir_sparse_" #T "_batch"); \
  }
MI355X_SPARSE(f32, float32_t, kSpF32)
MI355X_SPARSE(q31, q31_t, kSpQ31)
MI355X_SPARSE(q15, q15_t, kSpQ15)
MI355X_SPARSE(q7, q7_t, kSpQ7)
#undef MI355X_SPARSE
#define MI355X_LATTICE(T, CT, OP)                                                                       \
  void arm_fir_lattice_init_##T(arm_fir_lattice_instance_##T* S, uint16_t numStages, const CT* pCoeffs,  \
                                CT* pState) {                                                           \
    lattice_init(S, numStages, pCoeffs, pState);                                                        \
  }                                                                                                     \
  void arm_fir_lattice_##T(const arm_fir_lattice_instance_##T* S, const CT* pSrc, CT* pDst, uint32_t blockSize) { \
    lattice_sync(S, pSrc, pDst, blockSize, OP, "arm_fir_lattice_" #T);                                  \
  }                                                                                                     \
  arm_status arm_fir_lattice_##T##_batch(const arm_fir_lattice_instance_##T* S, const CT* d_src, CT* d_dst, \
                                         uint32_t blockSize, uint32_t batch, CT* d_state, void* stream) { \
    return lattice_batch(S, d_src, d_dst, blockSize, batch, d_state, stream, OP, "arm_fir_lattice_" #T "_batch"); \
  }
MI355X_LATTICE(f32, float32_t, kLatF32)
MI355X_LATTICE(q31, q31_t, kLatQ31)
MI355X_LATTICE(q15, q15_t, kLatQ15)
#undef MI355X_LATTICE
void arm_fir_sparse_f32(arm_fir_sparse_instance_f32* S, const float32_t* pSrc, float32_t* pDst, float32_t* pScratchIn,
                        uint32_t blockSize) {
  (void)pScratchIn;
  sparse_sync(S, pSrc, pDst, blockSize, kSpF32, "arm_fir_sparse_f32");
}
void arm_fir_sparse_q31(arm_fir_sparse_instance_q31* S, const q31_t* pSrc, q31_t* pDst, q31_t* pScratchIn,
                        uint32_t blockSize) {
  (void)pScratchIn;
  sparse_sync(S, pSrc, pDst, blockSize, kSpQ31, "arm_fir_sparse_q31");
}
void arm_fir_sparse_q15(arm_fir_sparse_instance_q15* S, const q15_t* pSrc, q15_t* pDst, q15_t* pScratchIn,
                        q31_t* pScratchOut, uint32_t blockSize) {
  (void)pScratchIn; (void)pScratchOut;
  sparse_sync(S, pSrc, pDst, blockSize, kSpQ15, "arm_fir_sparse_q15");
}
void arm_fir_sparse_q7(arm_fir_sparse_instance_q7* S, const q7_t* pSrc, q7_t* pDst, q7_t* pScratchIn,
                       q31_t* pScratchOut, uint32_t blockSize) {
  (void)pScratchIn; (void)pScratchOut;
  sparse_sync(S, pSrc, pDst, blockSize, kSpQ7, "arm_fir_sparse_q7");
}

}  // extern "C"
