// Semantics probe of gfx950's ds_read_b64_tr_b8 (the 8-bit transposed LDS read) for the i8-MFMA
// B operand of mat_mult_q15 / _q31.  The LDS holds a 16 x 32 byte tile
// T[r][c] = r * 32 + c (mod 256); every lane supplies the address `addr(lane)` below (the bf16
// form's rule scaled to bytes: lane 2q + p of a 16-lane group points at row q, columns 8p ..
// 8p + 7 of its block) and the 8 bytes it receives are printed, so the delivered layout can be
// read off directly (expected, by analogy with ds_read_b64_tr_b16: lane i of the group gets
// column i of the block's 8 rows, row q in byte q).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void probe(uint64_t* out, int mode) {
  __shared__ __attribute__((aligned(16))) uint8_t t[16 * 32];
  const int lane = threadIdx.x;
  for (int i = lane; i < 16 * 32; i += 64) t[i] = (uint8_t)((i / 32) * 32 + (i % 32));
  __syncthreads();
  const int g = lane >> 4, li = lane & 15;
  // block of group g: rows 8 * (g >> 1) .. + 7, columns 16 * (g & 1) .. + 15
  const int r0 = 8 * (g >> 1), c0 = 16 * (g & 1);
  int row, col;
  if (mode == 0) { row = r0 + (li >> 1); col = c0 + 8 * (li & 1); }      // lane 2q + p -> row q, cols 8p..
  else           { row = r0 + (li & 7);  col = c0 + 8 * (li >> 3); }     // lane q + 8p -> row q, cols 8p..
  typedef int v2i __attribute__((ext_vector_type(2)));
  const v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(t + row * 32 + col));
  out[mode * 64 + lane] = (uint64_t)(uint32_t)r.x | ((uint64_t)(uint32_t)r.y << 32);
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 2 * 64 * 8) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 0);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 1);
  uint64_t h[128];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int m = 0; m < 2; ++m) {
    printf("mode %d (byte = row*32 + col):\n", m);
    for (int l = 0; l < 64; ++l) {
      printf("  lane %2d:", l);
      for (int b = 0; b < 8; ++b) {
        const unsigned v = (unsigned)((h[m * 64 + l] >> (8 * b)) & 0xff);
        printf(" r%02u/c%02u", v / 32, v % 32);
      }
      printf("\n");
    }
  }
  return 0;
}
