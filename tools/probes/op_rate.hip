// Single-instruction issue-rate probe (gfx950): for each VALU opcode the fixed-point FFT
// and FIR kernels are built from, 8 independent dependency chains per lane of ITER steps,
// one instruction per step (inline asm, so the opcode is exactly the one named), grid =
// 8 waves per SIMD on every CU.  Prints T lane-instructions/s per opcode: a full-rate wave64
// instruction issues every 2 cycles per SIMD (78.6 T at 2.4 GHz), a half-rate one every 4.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITER = 2048;

#define CHAIN8(BODY)                                                        \
  _Pragma("unroll 4") for (int it = 0; it < ITER; ++it) {                  \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) { BODY; }                 \
  }

template <int K>
__global__ __launch_bounds__(256) void probe(int* out, int seed) {
  int a[8];
  float f[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x * 7 + i; f[i] = (float)a[i]; }
  const int c = seed * 3 + 1, d = seed + 5;
  if constexpr (K == 0) CHAIN8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 1) CHAIN8(asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 2) CHAIN8(asm volatile("v_mul_hi_i32 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 3) CHAIN8(asm volatile("v_ashrrev_i32 %0, 1, %0" : "+v"(a[i])))
  if constexpr (K == 4) CHAIN8(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 5) CHAIN8(asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(d)))
  if constexpr (K == 6) CHAIN8(asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 7) CHAIN8(asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 8) CHAIN8(asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[i]) : "v"((float)c)))
  if constexpr (K == 9) CHAIN8(asm volatile("v_mul_f32 %0, %0, %1" : "+v"(f[i]) : "v"((float)c)))
  if constexpr (K == 10) CHAIN8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "s"(c)))
  if constexpr (K == 11) CHAIN8(asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 7])))
  if constexpr (K == 12) CHAIN8(asm volatile("v_dot2_i32_i16 %0, %0, %1, %0" : "+v"(a[i]) : "v"(c)))
  if constexpr (K == 13) CHAIN8(asm volatile("v_pk_ashrrev_i16 %0, 1, %0" : "+v"(a[i])))
  if constexpr (K == 14) CHAIN8(asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(c), "v"(d)))
  if constexpr (K == 15) CHAIN8(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(c)))
  // FIR-shaped FMAs: accumulator + window VGPR + coefficient (SGPR or VGPR)
  if constexpr (K == 16) CHAIN8(asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[i]) : "s"((float)c), "v"(f[(i + 1) & 7])))
  if constexpr (K == 17) CHAIN8(asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[i]) : "v"((float)d), "v"(f[(i + 1) & 7])))
  if constexpr (K == 18) CHAIN8(asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[i]) : "s"((float)c), "v"((float)d)))
  // 64-bit products (MFCC q31 split / sqrt): 64-bit accumulator chains, carry-out to an SGPR pair
  long long q[8];
  for (int i = 0; i < 8; ++i) q[i] = a[i];
  unsigned long long sc = 0;
  if constexpr (K == 19) CHAIN8(asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q[i]), "=s"(sc) : "v"(c), "v"(d)))
  if constexpr (K == 20) CHAIN8(asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[i]), "=s"(sc) : "v"(c), "v"(d)))
  if constexpr (K == 21) CHAIN8(asm volatile("v_alignbit_b32 %0, %0, %1, 28" : "+v"(a[i]) : "v"(c)))
  int s = (int)sc;
  for (int i = 0; i < 8; ++i) s += a[i] + (int)f[i] + (int)q[i] + (int)(q[i] >> 32);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int K>
static void run(int* out, const char* name) {
  const int grid = 256 * 8;    // 256-thread blocks: 8 per CU = 8 waves per SIMD
  hipLaunchKernelGGL(probe<K>, dim3(grid), dim3(256), 0, 0, out, 1);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<K>, dim3(grid), dim3(256), 0, 0, out, r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double lane_instr = 5.0 * grid * 256.0 * ITER * 8;
  printf("%-22s %8.2f T lane-instr/s\n", name, lane_instr / (ms * 1e-3) * 1e-12);
}

int main() {
  int* out;
  (void)hipMalloc(&out, sizeof(int) * 256 * 256 * 8);
  run<0>(out, "v_add_u32");
  run<1>(out, "v_sub_u32");
  run<2>(out, "v_mul_hi_i32");
  run<3>(out, "v_ashrrev_i32");
  run<4>(out, "v_xor_b32");
  run<5>(out, "v_add3_u32");
  run<6>(out, "v_pk_add_u16");
  run<7>(out, "v_lshl_add_u32");
  run<8>(out, "v_add_f32");
  run<9>(out, "v_mul_f32");
  run<10>(out, "v_add_u32 (sgpr)");
  run<11>(out, "v_mov_b32");
  run<12>(out, "v_dot2_i32_i16");
  run<13>(out, "v_pk_ashrrev_i16");
  run<14>(out, "v_perm_b32");
  run<15>(out, "v_mul_lo_u32");
  run<16>(out, "v_fmac_f32 s,v(acc'),acc");
  run<17>(out, "v_fmac_f32 v,v(acc'),acc");
  run<18>(out, "v_fmac_f32 s,v(const),acc");
  run<19>(out, "v_mad_i64_i32");
  run<20>(out, "v_mad_u64_u32");
  run<21>(out, "v_alignbit_b32");
  return 0;
}
