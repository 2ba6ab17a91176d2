// Access-pattern ceiling probe (gfx950) for the 256-thread-per-transform CFFT kernels
// (cfft_fx4096 q31/q15, cfft_f32_n4096): a workgroup of TH threads owns S-byte transforms,
// T consecutive ones per workgroup; per transform every thread loads S/(TH*VB) vectors of VB
// bytes (each instruction covers TH*VB contiguous bytes), writes them to LDS, barrier, reads
// a transposed slot back, barrier, stores in place.  PF = the next transform's loads are
// issued before the current one is stored (the kernels' register prefetch).  Extra dynamic
// LDS sets workgroups per CU.  Prints TB/s of read + write over 8 GiB.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

template <int VB> struct Vec;
template <> struct Vec<8> { using T = v2i; };
template <> struct Vec<16> { using T = v4i; };

template <int TH, int S, int VB, int T, bool PF, bool Q>
__global__ __launch_bounds__(TH) void tile_kernel(int* __restrict__ x, long nxf, int s) {
  using V = typename Vec<VB>::T;
  constexpr int PER = S / (TH * VB);
  extern __shared__ v4i lds_raw[];
  V* lds = reinterpret_cast<V*>(lds_raw);
  const int tid = threadIdx.x;
  // Q: wave w moves the contiguous (S / waves)-byte part w of the transform (lane-contiguous
  // VB-byte words), instead of every instruction covering TH * VB bytes across the waves.
  const int io = Q ? (tid >> 6) * (PER * 64) + (tid & 63) : tid;
  constexpr int IS = Q ? 64 : TH;
  const long t0 = (long)blockIdx.x * T;
  V r[PER];
  auto ld = [&](long t) {
    const V* p = reinterpret_cast<const V*>(reinterpret_cast<char*>(x) + t * S) + io;
#pragma unroll
    for (int m = 0; m < PER; ++m) r[m] = __builtin_nontemporal_load(p + IS * m);
  };
  ld(t0);
  for (int t = 0; t < T; ++t) {
    if (!PF && t > 0) ld(t0 + t);
#pragma unroll
    for (int m = 0; m < PER; ++m) lds[tid + TH * m] = r[m] + s;
    __syncthreads();
    V o[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) o[m] = lds[(TH - 1 - tid) + TH * m];
    __syncthreads();
    if (PF && t + 1 < T) ld(t0 + t + 1);
    V* q = reinterpret_cast<V*>(reinterpret_cast<char*>(x) + (t0 + t) * S) + io;
#pragma unroll
    for (int m = 0; m < PER; ++m) __builtin_nontemporal_store(o[m], q + IS * m);
  }
}


// One wave per transform (the one-wave f32 kernels' pattern): wave w of a WPB-wave workgroup
// owns T consecutive S-byte transforms; per transform it loads (VBL-byte words), round-trips
// them through its own LDS region (no barrier: a wave's LDS operations run in order) or, with
// BAR, through the region with a workgroup barrier after the write and after the read (the
// multi-wave kernels' coupling), and stores in place (VBS-byte words).
template <int S, int T, int VBL, int VBS, int WPB, int BAR>
__global__ __launch_bounds__(64 * WPB) void wave_kernel(int* __restrict__ x, int s) {
  using VL = typename Vec<VBL>::T;
  using VS = typename Vec<VBS>::T;
  constexpr int PL = S / (64 * VBL), PS = S / (64 * VBS);
  extern __shared__ v4i lds_raw[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* lw = reinterpret_cast<char*>(lds_raw) + w * (S + 256);
  const long t0 = ((long)blockIdx.x * WPB + w) * T;
  for (int t = 0; t < T; ++t) {
    const VL* p = reinterpret_cast<const VL*>(reinterpret_cast<char*>(x) + (t0 + t) * S) + lane;
    VL r[PL];
#pragma unroll
    for (int m = 0; m < PL; ++m) r[m] = __builtin_nontemporal_load(p + 64 * m);
#pragma unroll
    for (int m = 0; m < PL; ++m) reinterpret_cast<VL*>(lw)[lane + 64 * m] = r[m] + s;
    if (BAR) __syncthreads();
    VS o[PS];
#pragma unroll
    for (int m = 0; m < PS; ++m) o[m] = reinterpret_cast<VS*>(lw)[(63 - lane) + 64 * m];
    if (BAR) __syncthreads();
    VS* q = reinterpret_cast<VS*>(reinterpret_cast<char*>(x) + (t0 + t) * S) + lane;
#pragma unroll
    for (int m = 0; m < PS; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}
template <int S, int T, int VBL, int VBS, int WPB, int BAR>
void timew(int* x, long bytes, hipEvent_t e0, hipEvent_t e1) {
  const long nxf = bytes / S;
  const dim3 g(nxf / (T * WPB)), b(64 * WPB);
  const size_t lds = (size_t)WPB * (S + 256);
  auto k = wave_kernel<S, T, VBL, VBS, WPB, BAR>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, 1);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  printf("wave S=%5d T=%d VBL=%2d VBS=%2d WPB=%d BAR=%d lds=%6zu  %.3f ms  %.3f TB/s\n", S, T, VBL, VBS, WPB, BAR, lds, ms,
         2.0 * bytes / (ms * 1e-3) * 1e-12);
  fflush(stdout);
}

template <int TH, int S, int VB, int T, bool PF, bool Q = false>
void timeit(int* x, long bytes, int extra_lds, hipEvent_t e0, hipEvent_t e1) {
  const long nxf = bytes / S;
  const dim3 g(nxf / T), b(TH);
  const size_t lds = S + extra_lds;
  auto k = tile_kernel<TH, S, VB, T, PF, Q>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, nxf, 1);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, nxf, 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  printf("Q=%d TH=%4d S=%5d VB=%2d T=%2d PF=%d lds=%6zu (wg/CU<=%3zu)  %.3f ms  %.3f TB/s\n", (int)Q, TH, S, VB, T, PF,
         lds, (size_t)160 * 1024 / lds, ms, 2.0 * bytes / (ms * 1e-3) * 1e-12);
  fflush(stdout);
}

int main() {
  const long bytes = 8L << 30;
  int* x;
  if (hipMalloc(&x, bytes) != hipSuccess) return 1;
  hipMemset(x, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // one wave per transform: the f32 N=1024 kernel's pattern (8 KiB, T = 4, 8 waves, 8-B loads,
  // 16-B stores), then one property at a time toward the 256-thread fixed-point kernels
  timew<8192, 4, 8, 16, 8, 0>(x, bytes, e0, e1);
  timew<8192, 4, 8, 16, 8, 1>(x, bytes, e0, e1);
  timew<8192, 4, 16, 16, 8, 0>(x, bytes, e0, e1);
  timew<8192, 2, 8, 16, 8, 0>(x, bytes, e0, e1);
  timew<8192, 8, 8, 16, 8, 0>(x, bytes, e0, e1);
  timew<16384, 2, 8, 16, 4, 0>(x, bytes, e0, e1);
  timew<16384, 2, 16, 16, 4, 0>(x, bytes, e0, e1);
  timew<16384, 2, 16, 16, 4, 1>(x, bytes, e0, e1);
  timew<16384, 4, 16, 16, 4, 0>(x, bytes, e0, e1);
  timew<16384, 1, 16, 16, 4, 0>(x, bytes, e0, e1);
  timew<16384, 2, 16, 16, 2, 0>(x, bytes, e0, e1);
  timew<16384, 2, 16, 16, 8, 0>(x, bytes, e0, e1);
  timew<32768, 2, 16, 16, 2, 0>(x, bytes, e0, e1);
  timew<32768, 1, 16, 16, 4, 0>(x, bytes, e0, e1);
  timew<32768, 2, 16, 16, 4, 0>(x, bytes, e0, e1);
  hipFree(x);
  return 0;
}
