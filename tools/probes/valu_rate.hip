// VALU issue-rate probe (gfx950): sustained wave-instructions per SIMD-cycle for the
// instructions the FIR kernels are built from.  Each lane runs 8 independent chains of
// ITER dependent ops; grid = 4 waves/SIMD x 256 CUs x 4.  Prints T lane-values/s per kind
// (a packed v_pk_*_f32 instruction produces two values per lane; a plain one, one).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void probe(int* out, int seed) {
  int a[8]; float f[8]; f2 p[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x + i; f[i] = (float)a[i]; p[i] = f2{f[i], f[i] + 1.0f}; }
  const f2 cp = f2{1.0001f + seed, 1.0002f + seed}, hp = f2{0.5f, 0.25f};
  const int c = seed * 3 + 1;
  const float cf = 1.0001f + seed;
#pragma unroll 4
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (KIND == 0) a[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a[i] ^ it), __builtin_bit_cast(s2, c), a[i], false);
      if constexpr (KIND == 1) f[i] = f[i] * cf + 0.5f;   // contract(off) below: mul + add
      if constexpr (KIND == 2) f[i] = __builtin_fmaf(f[i], cf, 0.5f);
      if constexpr (KIND == 3) a[i] = __mul24(a[i], c) + it;
      if constexpr (KIND == 4) p[i] = p[i] * cp + hp;      // v_pk_mul_f32 + v_pk_add_f32 (2 values each)
      if constexpr (KIND == 5) p[i] = __builtin_elementwise_fma(p[i], cp, hp);   // v_pk_fma_f32
    }
  }
  int s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + (int)f[i] + (int)(p[i].x + p[i].y);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int* out; hipMalloc(&out, sizeof(int) * 256 * 256 * 16 * 4);
  const char* names[] = {"v_dot2c_i32_i16 (xor+dot2)", "v_mul_f32+v_add_f32", "v_fma_f32", "v_mul_i32_i24+v_add",
                         "v_pk_mul_f32+v_pk_add_f32", "v_pk_fma_f32"};
  // lane-VALUES per lane per inner step (a packed op produces two values per lane)
  const int ops_per[] = {2, 2, 1, 2, 4, 2};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int kind = 0; kind < 6; ++kind) {
    for (int waves = 1; waves <= 8; waves *= 2) {
      const int grid = 256 * waves;   // 256-thread blocks: 4 waves = 1 per SIMD each
      auto k = kind == 0 ? probe<0> : kind == 1 ? probe<1> : kind == 2 ? probe<2> : kind == 3 ? probe<3>
             : kind == 4 ? probe<4> : probe<5>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1);
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, r);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double lane_ops = 5.0 * grid * 256.0 * ITER * 8 * ops_per[kind];
      printf("%-28s waves/SIMD=%d  %8.2f T lane-values/s\n", names[kind], waves, lane_ops / (ms * 1e-3) * 1e-12);
    }
  }
  return 0;
}
