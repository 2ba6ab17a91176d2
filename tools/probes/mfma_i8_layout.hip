// Checks the assumed operand map of v_mfma_i32_32x32x32_i8 with exact integer data:
// lane l holds A[row l&31][k = 16(l>>5) + j] and B[k = 16(l>>5) + j][col l&31] in byte j
// of its 128-bit operand; C/D: col = l&31, row = (reg&3) + 8(reg>>2) + 4(l>>5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const signed char* A, const signed char* B, int* C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  signed char a[16], b[16];
  for (int j = 0; j < 16; ++j) { a[j] = A[r * 32 + 16 * h + j]; b[j] = B[(16 * h + j) * 32 + r]; }
  i32x4 av = *reinterpret_cast<i32x4*>(a), bv = *reinterpret_cast<i32x4*>(b);
  i32x16 acc = {};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) C[((reg & 3) + 8 * (reg >> 2) + 4 * h) * 32 + r] = acc[reg];
}

int main() {
  signed char hA[1024], hB[1024];
  int hC[1024], ref[1024];
  srand(7);
  for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() & 255); hB[i] = (signed char)(rand() & 255); }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int q = 0; q < 32; ++q) s += hA[i * 32 + q] * hB[q * 32 + j];
      ref[i * 32 + j] = s;
    }
  signed char *dA, *dB; int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
  printf("mfma_i32_32x32x32_i8 layout check: %d / 1024 mismatches%s\n", bad, bad ? "" : " (map confirmed)");
  return bad != 0;
}
