// Shared device/host helpers for the MI355X CMSIS-DSP backend (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tuning.hpp"

namespace mi355x {

// Exact integer semantics of the reference's host scalar path (Include/dsp/none.h):
// int32 arithmetic wraps (gcc on x86-64), right shifts of signed values are arithmetic.
// Everything is done on uint32_t so the compiler cannot exploit signed-overflow UB.
__device__ __forceinline__ int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
__device__ __forceinline__ int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
__device__ __forceinline__ int32_t wshl(int32_t a, int s) { return (int32_t)((uint32_t)a << s); }
// (int32_t)(((q63_t)a * b) >> 32): arm_cfft_radix4_q31.c:235 — exactly v_mul_hi_i32.
// Emitted directly: from __mulhi LLVM sometimes rebuilds the product as a general 64-bit
// multiply of the sign-extended operands (v_mul_hi_u32 + v_mad_u64_u32 + v_mul_lo_u32 per
// product instead of one v_mul_hi_i32; 30 % of the q31 N=4096 kernel's VALU instructions).
__device__ __forceinline__ int32_t mulhi(int32_t a, int32_t b) {
  int32_t r;
  asm("v_mul_hi_i32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// none.h:184-206 rounding forms (SMMULR / SMMLAR / SMMLSR)
__device__ __forceinline__ int32_t mult_R(int32_t x, int32_t y) {
  return (int32_t)((uint64_t)((int64_t)x * y + 0x80000000LL) >> 32);
}
__device__ __forceinline__ int32_t multAcc_R(int32_t a, int32_t x, int32_t y) {
  uint64_t v = ((uint64_t)(int64_t)a << 32) + (uint64_t)((int64_t)x * y) + 0x80000000ULL;
  return (int32_t)(v >> 32);
}
__device__ __forceinline__ int32_t multSub_R(int32_t a, int32_t x, int32_t y) {
  uint64_t v = ((uint64_t)(int64_t)a << 32) - (uint64_t)((int64_t)x * y) + 0x80000000ULL;
  return (int32_t)(v >> 32);
}
// __SSAT(val, 16): none.h:78-94
__device__ __forceinline__ int32_t ssat16(int32_t v) { return v > 32767 ? 32767 : (v < -32768 ? -32768 : v); }
__device__ __forceinline__ int32_t ssat8(int32_t v) { return v > 127 ? 127 : (v < -128 ? -128 : v); }

constexpr int kBlock = 256;   // 4 wave64 per workgroup

// Raw buffer resource over [p, p + bytes) (gfx9 descriptor dword 3 = 0x00020000): buffer
// loads/stores take one VGPR byte offset plus an SGPR soffset, so the per-access 64-bit
// address arithmetic of global_load/global_store disappears.  aux 2 = nontemporal.
typedef int v2i __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
template <int AUX = 2>
__device__ __forceinline__ float2 buf_ld_f2(__amdgpu_buffer_rsrc_t r, int vo, int so) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, AUX));
}
template <int AUX = 2>
__device__ __forceinline__ void buf_st_f2(__amdgpu_buffer_rsrc_t r, int vo, int so, float2 x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2i, x), r, vo, so, AUX);
}

template <int N> struct Log2 { static constexpr int v = 1 + Log2<N / 2>::v; };
template <> struct Log2<1> { static constexpr int v = 0; };

// Binary bit reversal over B bits: the effective permutation of the fixed-point tables
// armBitRevIndexTable_fixed_N (verified against the table swaps on the host).
template <int B> __device__ __forceinline__ int bitrev(int k) { return (int)(__brev((uint32_t)k) >> (32 - B)); }

// Flags shared by every transform kernel.  kSatShl1 (fixed point only): every output word
// is shifted left by one with saturation on store -- arm_shift_q31 / arm_shift_q15 by +1
// (arm_shift_q31.c:143-146, arm_shift_q15.c:225), which the q31/q15 inverse RFFT applies
// after its inner CFFT (arm_rfft_q31.c:164).
enum : uint32_t { kIfft = 1u, kBitrev = 2u, kSatShl1 = 4u };

__device__ __forceinline__ int32_t sat_shl1_q31(int32_t v) {
  const int32_t o = (int32_t)((uint32_t)v << 1);
  return (o >> 1) != v ? (int32_t)(0x7FFFFFFF ^ (v >> 31)) : o;
}
__device__ __forceinline__ int32_t sat_shl1_q15(int32_t v) { return ssat16(v << 1); }

// End of a one-workgroup synchronous drop-in launch: every thread's stores are made visible
// system-wide, then one lane stores seq into the caller's coherent host word (the completion
// signal the host spins on, runtime.cpp done_slot; sync.hip does the same as its own launch).
__device__ __forceinline__ void signal_done(uint32_t* done, uint32_t seq) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace mi355x
