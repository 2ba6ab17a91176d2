// v_fmac_f32 issue rate vs VGPR bank of its operands (gfx950).  The FIR FMA loop
// (fir_f32_kernel<.., FMA = true>) issues acc[r] = fma(x[r + u], c[u], acc[r]): src1 = a window
// VGPR, src2 = the accumulator (also the destination), src0 = an SGPR coefficient.  VGPRs sit in
// 4 banks (v mod 4).  Each variant is one inline-asm block with explicit registers, repeated
// ITER times by 256-thread blocks at W waves per SIMD on every CU; prints T lane-FMA/s
// (78.6 T = one wave64 instruction every 2 cycles per SIMD at 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

constexpr int ITER = 512;

#define CLOB "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", \
  "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29",      \
  "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44",      \
  "v45", "v46", "v47", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27"


template <int K>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
  float acc = seed;
  asm volatile(
      "v_mov_b32 v0, %0\n" "v_mov_b32 v1, %0\n" "v_mov_b32 v2, %0\n" "v_mov_b32 v3, %0\n"
      "s_mov_b32 s20, 0x3f800001\n" "s_mov_b32 s21, 0x3f800002\n" "s_mov_b32 s22, 0x3f800003\n"
      "s_mov_b32 s23, 0x3f800004\n" "s_mov_b32 s24, 0x3f800005\n" "s_mov_b32 s25, 0x3f800006\n"
      "s_mov_b32 s26, 0x3f800007\n" "s_mov_b32 s27, 0x3f800008\n"
      :: "v"(seed) : CLOB);
  for (int it = 0; it < ITER; ++it) {
    if constexpr (K == 0) {          // same bank: v_fmac vR, s, v(R+16)   (R = 0..15) x 8
      asm volatile(
          ".rept 8\n"
          "v_fmac_f32 v0, s20, v16\n v_fmac_f32 v1, s20, v17\n v_fmac_f32 v2, s20, v18\n v_fmac_f32 v3, s20, v19\n"
          "v_fmac_f32 v4, s20, v20\n v_fmac_f32 v5, s20, v21\n v_fmac_f32 v6, s20, v22\n v_fmac_f32 v7, s20, v23\n"
          "v_fmac_f32 v8, s20, v24\n v_fmac_f32 v9, s20, v25\n v_fmac_f32 v10, s20, v26\n v_fmac_f32 v11, s20, v27\n"
          "v_fmac_f32 v12, s20, v28\n v_fmac_f32 v13, s20, v29\n v_fmac_f32 v14, s20, v30\n v_fmac_f32 v15, s20, v31\n"
          ".endr\n" ::: CLOB);
    } else if constexpr (K == 1) {   // different bank: x = v(R+17)
      asm volatile(
          ".rept 8\n"
          "v_fmac_f32 v0, s20, v17\n v_fmac_f32 v1, s20, v18\n v_fmac_f32 v2, s20, v19\n v_fmac_f32 v3, s20, v20\n"
          "v_fmac_f32 v4, s20, v21\n v_fmac_f32 v5, s20, v22\n v_fmac_f32 v6, s20, v23\n v_fmac_f32 v7, s20, v24\n"
          "v_fmac_f32 v8, s20, v25\n v_fmac_f32 v9, s20, v26\n v_fmac_f32 v10, s20, v27\n v_fmac_f32 v11, s20, v28\n"
          "v_fmac_f32 v12, s20, v29\n v_fmac_f32 v13, s20, v30\n v_fmac_f32 v14, s20, v31\n v_fmac_f32 v15, s20, v32\n"
          ".endr\n" ::: CLOB);
    } else if constexpr (K == 2) {   // bit-exact form: v_mul into a temp (rotating 4), v_add into acc
      asm volatile(
          ".rept 8\n"
          "v_mul_f32 v40, s20, v16\n v_add_f32 v0, v0, v40\n v_mul_f32 v41, s20, v17\n v_add_f32 v1, v1, v41\n"
          "v_mul_f32 v42, s20, v18\n v_add_f32 v2, v2, v42\n v_mul_f32 v43, s20, v19\n v_add_f32 v3, v3, v43\n"
          "v_mul_f32 v40, s20, v20\n v_add_f32 v4, v4, v40\n v_mul_f32 v41, s20, v21\n v_add_f32 v5, v5, v41\n"
          "v_mul_f32 v42, s20, v22\n v_add_f32 v6, v6, v42\n v_mul_f32 v43, s20, v23\n v_add_f32 v7, v7, v43\n"
          ".endr\n" ::: CLOB);
    } else if constexpr (K == 3) {   // fmac with a VGPR coefficient, different banks (x = R+17, c = v44)
      asm volatile(
          ".rept 8\n"
          "v_fmac_f32 v0, v44, v17\n v_fmac_f32 v1, v44, v18\n v_fmac_f32 v2, v44, v19\n v_fmac_f32 v3, v44, v20\n"
          "v_fmac_f32 v4, v44, v21\n v_fmac_f32 v5, v44, v22\n v_fmac_f32 v6, v44, v23\n v_fmac_f32 v7, v44, v24\n"
          "v_fmac_f32 v8, v44, v25\n v_fmac_f32 v9, v44, v26\n v_fmac_f32 v10, v44, v27\n v_fmac_f32 v11, v44, v28\n"
          "v_fmac_f32 v12, v44, v29\n v_fmac_f32 v13, v44, v30\n v_fmac_f32 v14, v44, v31\n v_fmac_f32 v15, v44, v32\n"
          ".endr\n" ::: CLOB);
    } else if constexpr (K == 4) {   // 8 accumulators only (dependency distance 8), different banks
      asm volatile(
          ".rept 16\n"
          "v_fmac_f32 v0, s20, v17\n v_fmac_f32 v1, s20, v18\n v_fmac_f32 v2, s20, v19\n v_fmac_f32 v3, s20, v20\n"
          "v_fmac_f32 v4, s20, v21\n v_fmac_f32 v5, s20, v22\n v_fmac_f32 v6, s20, v23\n v_fmac_f32 v7, s20, v24\n"
          ".endr\n" ::: CLOB);
    } else if constexpr (K == 5) {   // v_pk_fma_f32: 2 FMAs per lane-instruction, acc pairs, x pairs
      asm volatile(
          ".rept 8\n"
          "v_pk_fma_f32 v[0:1], v[18:19], s[20:21], v[0:1] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[2:3], v[20:21], s[20:21], v[2:3] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[4:5], v[22:23], s[20:21], v[4:5] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[6:7], v[24:25], s[20:21], v[6:7] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[8:9], v[26:27], s[20:21], v[8:9] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[10:11], v[28:29], s[20:21], v[10:11] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[12:13], v[30:31], s[20:21], v[12:13] op_sel_hi:[1,0,1]\n"
          "v_pk_fma_f32 v[14:15], v[32:33], s[20:21], v[14:15] op_sel_hi:[1,0,1]\n"
          ".endr\n" ::: CLOB);
    }
  }
  float r;
  asm volatile("v_mov_b32 %0, v0" : "=v"(r) :: CLOB);
  out[blockIdx.x * 256 + threadIdx.x] = r + acc;
}

template <int K>
static void run(float* out, const char* name, int fma_per_block, int cus) {
  for (int w : {1, 2, 4, 5, 8}) {
    const int grid = cus * w;               // 256-thread blocks: w per CU = w waves per SIMD
    hipLaunchKernelGGL(probe<K>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<K>, dim3(grid), dim3(256), 0, 0, out, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double lane_fma = 5.0 * grid * 256.0 * ITER * fma_per_block;
    printf("%-44s waves/SIMD=%d  %6.2f T lane-FMA/s\n", name, w, lane_fma / (ms * 1e-3) * 1e-12);
    fflush(stdout);
  }
}

int main() {
  float* out;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  if (hipMalloc(&out, sizeof(float) * 256 * cus * 8) != hipSuccess) return 1;
  run<0>(out, "fmac sgpr, acc/x same bank (16 acc)", 128, cus);
  run<1>(out, "fmac sgpr, acc/x different bank (16 acc)", 128, cus);
  run<2>(out, "mul+add (bit-exact form), 8 acc", 64, cus);
  run<3>(out, "fmac vgpr coef, different bank (16 acc)", 128, cus);
  run<4>(out, "fmac sgpr, different bank (8 acc)", 128, cus);
  run<5>(out, "pk_fma_f32 sgpr pair (16 acc = 8 pairs)", 128, cus);
  hipFree(out);
  return 0;
}
