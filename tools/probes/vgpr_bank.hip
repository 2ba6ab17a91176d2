// VGPR bank probe (gfx950): does a VOP2 v_add_f32 whose two VGPR sources sit in the same
// register bank (index mod 4) issue slower than one whose sources sit in different banks?
// Each kernel runs 64 independent v_add_f32 per asm block (dest v32..v47, sources v0..v31),
// 8 waves per SIMD; prints wave-instructions per SIMD-cycle (at 2 cycles/instr = 0.5).
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int ITER = 2048;

#define ADD16(D, A, B) \
  "v_add_f32 v" #D ", v" #A ", v" #B "\n"
template <int KIND>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0) {   // sources in different banks: (4i, 4i+1)
      asm volatile(
#define R(i) "v_add_f32 v" #i "0, v" #i "1, v" #i "2\n"
          "v_add_f32 v32, v0, v1\n v_add_f32 v33, v4, v5\n v_add_f32 v34, v8, v9\n v_add_f32 v35, v12, v13\n"
          "v_add_f32 v36, v16, v17\n v_add_f32 v37, v20, v21\n v_add_f32 v38, v24, v25\n v_add_f32 v39, v28, v29\n"
          "v_add_f32 v40, v2, v3\n v_add_f32 v41, v6, v7\n v_add_f32 v42, v10, v11\n v_add_f32 v43, v14, v15\n"
          "v_add_f32 v44, v18, v19\n v_add_f32 v45, v22, v23\n v_add_f32 v46, v26, v27\n v_add_f32 v47, v30, v31\n"
          ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    } else if constexpr (KIND == 1) {   // sources in the same bank: (i, i+4)
      asm volatile(
          "v_add_f32 v32, v0, v4\n v_add_f32 v33, v1, v5\n v_add_f32 v34, v2, v6\n v_add_f32 v35, v3, v7\n"
          "v_add_f32 v36, v8, v12\n v_add_f32 v37, v9, v13\n v_add_f32 v38, v10, v14\n v_add_f32 v39, v11, v15\n"
          "v_add_f32 v40, v16, v20\n v_add_f32 v41, v17, v21\n v_add_f32 v42, v18, v22\n v_add_f32 v43, v19, v23\n"
          "v_add_f32 v44, v24, v28\n v_add_f32 v45, v25, v29\n v_add_f32 v46, v26, v30\n v_add_f32 v47, v27, v31\n"
          ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    } else if constexpr (KIND == 2) {   // accumulate form d = d + s, d and s in different banks
      asm volatile(
          "v_add_f32 v32, v32, v1\n v_add_f32 v33, v33, v2\n v_add_f32 v34, v34, v3\n v_add_f32 v35, v35, v4\n"
          "v_add_f32 v36, v36, v5\n v_add_f32 v37, v37, v6\n v_add_f32 v38, v38, v7\n v_add_f32 v39, v39, v8\n"
          "v_add_f32 v40, v40, v9\n v_add_f32 v41, v41, v10\n v_add_f32 v42, v42, v11\n v_add_f32 v43, v43, v12\n"
          "v_add_f32 v44, v44, v13\n v_add_f32 v45, v45, v14\n v_add_f32 v46, v46, v15\n v_add_f32 v47, v47, v16\n"
          ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    } else {                            // accumulate form, d and s in the same bank
      asm volatile(
          "v_add_f32 v32, v32, v0\n v_add_f32 v33, v33, v1\n v_add_f32 v34, v34, v2\n v_add_f32 v35, v35, v3\n"
          "v_add_f32 v36, v36, v4\n v_add_f32 v37, v37, v5\n v_add_f32 v38, v38, v6\n v_add_f32 v39, v39, v7\n"
          "v_add_f32 v40, v40, v8\n v_add_f32 v41, v41, v9\n v_add_f32 v42, v42, v10\n v_add_f32 v43, v43, v11\n"
          "v_add_f32 v44, v44, v12\n v_add_f32 v45, v45, v13\n v_add_f32 v46, v46, v14\n v_add_f32 v47, v47, v15\n"
          ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
          "v46", "v47");
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = seed;
}

int main() {
  float* out; hipMalloc(&out, sizeof(float) * 256 * 256 * 8);
  const char* names[] = {"sources in different banks", "sources in the same bank",
                         "d = d + s, different banks", "d = d + s, same bank"};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  for (int kind = 0; kind < 4; ++kind) {
    for (int waves = 2; waves <= 8; waves *= 2) {
      const int grid = 256 * waves;
      auto k = kind == 0 ? probe<0> : kind == 1 ? probe<1> : kind == 2 ? probe<2> : probe<3>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.0f);
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.0f);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double winstr = 5.0 * grid * 4.0 * ITER * 16;   // wave-instructions
      printf("%-28s waves/SIMD=%d  %7.3f T wave-instr/s  (%.3f per SIMD-cycle at %d MHz)\n", names[kind], waves,
             winstr / (ms * 1e-3) * 1e-12, winstr / (ms * 1e-3) / 1024.0 / (clk * 1e3), clk / 1000);
    }
  }
  return 0;
}
