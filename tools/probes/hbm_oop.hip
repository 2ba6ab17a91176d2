// Access-pattern ceiling probe (gfx950), round 6: the arm_rfft_fast_f32
// P_SCRATCH shape -- one wave per 4 KiB transform read from one buffer and 4 KiB written to ANOTHER
// (rfft1024_fwd_kernel<TS, false>, csrc/rfft_f32.hip), against the in-place shape the CFFT class runs
// (profiles/r03/probe_hbm_wgtile.txt: 6.0-6.27 TB/s) and a flat copy.
//   wave : WPB waves per workgroup, each T consecutive transforms of S bytes; VB-byte lane vectors
//          (the kernel: 8); loads -> LDS -> reversed read (one wave-local round trip, like the
//          kernel's stage passes) -> stores to dst (OOP) or back to src; PF issues the next
//          transform's loads before this one's stores.
//   flat : grid-stride 16 B per lane copy src -> dst, GRID workgroups of 256.
// Every variant moves 4 GiB in + 4 GiB out (the bench workload: 2^20 transforms of 1024 floats);
// prints TB/s of read + write.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
template <int VB> struct Vec;
template <> struct Vec<8> { using T = v2i; };
template <> struct Vec<16> { using T = v4i; };

template <int WPB, int S, int VB, int T, bool PF, bool OOP, bool STRIDE = false>
__global__ __launch_bounds__(64 * WPB) void wave_kernel(const int* src, int* dst, int s) {
  using V = typename Vec<VB>::T;
  constexpr int PER = S / (64 * VB);
  __shared__ V lds_all[WPB][S / VB];
  V* lds = lds_all[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63;
  // STRIDE: wave i takes transforms i, i + W, i + 2W ... (W = waves in the grid), so the waves
  // resident at one time touch neighbouring transforms; else T consecutive transforms per wave
  const long wv = (long)blockIdx.x * WPB + (threadIdx.x >> 6), nw = (long)gridDim.x * WPB;
  auto tr = [&](int k) { return STRIDE ? wv + k * nw : wv * T + k; };
  V r[PER];
  auto ld = [&](long t) {
    const V* p = reinterpret_cast<const V*>(reinterpret_cast<const char*>(src) + t * S) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) r[m] = __builtin_nontemporal_load(p + 64 * m);
  };
  ld(tr(0));
  for (int t = 0; t < T; ++t) {
    if (!PF && t > 0) ld(tr(t));
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < PER; ++m) lds[lane + 64 * m] = r[m] + s;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    V o[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) o[m] = lds[(63 - lane) + 64 * (PER - 1 - m)];
    if (PF && t + 1 < T) ld(tr(t + 1));
    int* base = OOP ? dst : const_cast<int*>(src);
    V* q = reinterpret_cast<V*>(reinterpret_cast<char*>(base) + tr(t) * S) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}

__global__ __launch_bounds__(256) void flat_kernel(const v4i* __restrict__ src, v4i* __restrict__ dst, long n, int s) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i) + s, dst + i);
}

static float timed(void (*launch)(const int*, int*), const int* a, int* b, hipEvent_t e0, hipEvent_t e1) {
  for (int i = 0; i < 3; ++i) launch(a, b);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) launch(a, b);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

constexpr long kBytes = 4L << 30;
static void report(const char* what, float ms) {
  printf("%-58s %.3f ms  %.3f TB/s\n", what, ms, 2.0 * kBytes / (ms * 1e-3) * 1e-12);
  fflush(stdout);
}

template <int WPB, int S, int VB, int T, bool PF, bool OOP, bool STRIDE = false>
static void wave(const int* a, int* b, hipEvent_t e0, hipEvent_t e1) {
  auto launch = [](const int* x, int* y) {
    hipLaunchKernelGGL((wave_kernel<WPB, S, VB, T, PF, OOP, STRIDE>), dim3(kBytes / S / T / WPB), dim3(64 * WPB), 0, 0, x, y, 1);
  };
  const float ms = timed(launch, a, b, e0, e1);
  char w[160];
  snprintf(w, sizeof w, "wave %s WPB=%d S=%d VB=%2d T=%2d PF=%d %s", OOP ? "oop  " : "inpl ", WPB, S, VB, T, PF,
           STRIDE ? "strided" : "consecutive");
  report(w, ms);
}

template <int GRID>
static void flat(const int* a, int* b, hipEvent_t e0, hipEvent_t e1) {
  auto launch = [](const int* x, int* y) {
    hipLaunchKernelGGL(flat_kernel, dim3(GRID), dim3(256), 0, 0, (const v4i*)x, (v4i*)y, kBytes / 16, 1);
  };
  const float ms = timed(launch, a, b, e0, e1);
  char w[160];
  snprintf(w, sizeof w, "flat copy grid=%d", GRID);
  report(w, ms);
}

int main() {
  int *a, *b;
  if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&b, kBytes) != hipSuccess) return 1;
  hipMemset(a, 0, kBytes);
  hipMemset(b, 0, kBytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  flat<2048>(a, b, e0, e1);
  flat<8192>(a, b, e0, e1);
  flat<65536>(a, b, e0, e1);
  // in place (the CFFT class) vs out of place (P_SCRATCH), the kernel's shape: VB 8, WPB 1
  wave<1, 4096, 8, 8, false, false>(a, b, e0, e1);
  wave<1, 4096, 8, 8, false, true>(a, b, e0, e1);
  wave<1, 4096, 8, 1, false, true>(a, b, e0, e1);
  wave<1, 4096, 8, 2, false, true>(a, b, e0, e1);
  wave<1, 4096, 8, 4, false, true>(a, b, e0, e1);
  wave<1, 4096, 8, 16, false, true>(a, b, e0, e1);
  wave<1, 4096, 8, 8, true, true>(a, b, e0, e1);
  wave<1, 4096, 8, 16, true, true>(a, b, e0, e1);
  wave<1, 4096, 16, 8, false, true>(a, b, e0, e1);
  wave<1, 4096, 16, 8, true, true>(a, b, e0, e1);
  wave<4, 4096, 8, 8, false, true>(a, b, e0, e1);
  wave<4, 4096, 8, 2, false, true>(a, b, e0, e1);
  wave<4, 4096, 8, 8, true, true>(a, b, e0, e1);
  wave<1, 4096, 16, 8, true, false>(a, b, e0, e1);
  // round 6: the mapping -- resident waves on neighbouring transforms
  for (int rep = 0; rep < 2; ++rep) {
    wave<1, 4096, 8, 1, false, true>(a, b, e0, e1);
    wave<1, 4096, 8, 8, false, true>(a, b, e0, e1);
    wave<1, 4096, 8, 8, false, true, true>(a, b, e0, e1);
    wave<1, 4096, 8, 4, false, true, true>(a, b, e0, e1);
    wave<1, 4096, 8, 16, false, true, true>(a, b, e0, e1);
    wave<1, 4096, 8, 8, true, true, true>(a, b, e0, e1);
    wave<1, 4096, 8, 16, true, true, true>(a, b, e0, e1);
    wave<4, 4096, 8, 8, false, true, true>(a, b, e0, e1);
    wave<4, 4096, 8, 8, true, true, true>(a, b, e0, e1);
    wave<1, 4096, 8, 8, false, false, true>(a, b, e0, e1);
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
