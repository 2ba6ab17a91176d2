// Integer VALU issue-rate probe (gfx950) for the q31 butterfly's instruction mix:
// v_mul_hi_i32, v_mul_lo_u32, v_add_u32, v_ashrrev_i32, v_mul_i32_i24.  Each lane runs 8
// independent chains; prints T lane-ops/s (one op = one VALU instruction per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void probe(int* out, int seed) {
  int a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed + threadIdx.x * 7 + i;
  const int c = seed * 3 + 0x12345;
#pragma unroll 4
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) a[i] = __mulhi(a[i], c) + it;            // v_mul_hi_i32 + v_add
      if constexpr (KIND == 1) a[i] = a[i] * c + it;                    // v_mul_lo_u32 + v_add (or mad)
      if constexpr (KIND == 2) a[i] = (a[i] + c) ^ it;                  // v_add + v_xor
      if constexpr (KIND == 3) a[i] = (a[i] >> 1) + c;                  // v_ashr + v_add (or lshl_add)
      if constexpr (KIND == 4) a[i] = __mul24(a[i], c) + it;            // v_mul_i32_i24 + v_add
    }
  }
  int s = 0;
  for (int i = 0; i < 8; ++i) s += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int* out; hipMalloc(&out, sizeof(int) * 256 * 256 * 16 * 4);
  const char* names[] = {"v_mul_hi_i32+v_add", "v_mul_lo_u32+v_add", "v_add+v_xor", "v_ashr+v_add", "v_mul_i32_i24+v_add"};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int kind = 0; kind < 5; ++kind) {
    for (int waves = 1; waves <= 8; waves *= 2) {
      const int grid = 256 * waves;
      auto k = kind == 0 ? probe<0> : kind == 1 ? probe<1> : kind == 2 ? probe<2> : kind == 3 ? probe<3> : probe<4>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1);
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, r);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double lane_ops = 5.0 * grid * 256.0 * ITER * 8 * 2;
      printf("%-22s waves/SIMD=%d  %8.2f T lane-instr/s (2 instr per chain step)\n", names[kind], waves,
             lane_ops / (ms * 1e-3) * 1e-12);
    }
  }
  return 0;
}
