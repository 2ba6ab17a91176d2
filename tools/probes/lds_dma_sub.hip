// Probe (gfx950): where global_load_lds with 1- and 2-byte elements puts each lane's data in LDS
// (the dword variant writes lane l at M0 + 4 l).  One wave; LDS pre-filled with 0xAA bytes;
// source bytes = their index; prints the first 64 LDS dwords after each DMA.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int SZ>
__global__ void probe(const unsigned char* src, unsigned* out) {
  __shared__ unsigned lds[256];
  const int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) lds[i] = 0xAAAAAAAAu;
  __syncthreads();
  if constexpr (SZ == 1)
    __builtin_amdgcn_global_load_lds((const void*)(src + l + 1), (__attribute__((address_space(3))) void*)lds, 1, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((const void*)(src + 2 * l + 2), (__attribute__((address_space(3))) void*)lds, 2, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = l; i < 256; i += 64) out[i] = lds[i];
}

int main() {
  unsigned char h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (unsigned char)i;
  unsigned char* s;
  unsigned* o;
  unsigned ho[256];
  if (hipMalloc(&s, 1024) != hipSuccess || hipMalloc(&o, 1024) != hipSuccess) return 1;
  (void)hipMemcpy(s, h, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, s, o);
  (void)hipMemcpy(ho, o, 1024, hipMemcpyDeviceToHost);
  printf("size 1 (src byte l+1 per lane):");
  for (int i = 0; i < 24; ++i) printf(" %08x", ho[i]);
  printf("\n");
  hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, s, o);
  (void)hipMemcpy(ho, o, 1024, hipMemcpyDeviceToHost);
  printf("size 2 (src bytes 2l+2, 2l+3 per lane):");
  for (int i = 0; i < 24; ++i) printf(" %08x", ho[i]);
  printf("\n");
  return 0;
}
