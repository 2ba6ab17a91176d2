// Access-pattern ceiling probe (gfx950), round 4: the two shapes between
// "one wave per transform" (6.0-6.27 TB/s, profiles/r03/probe_hbm_wgtile.txt) and "256 threads
// per transform with workgroup barriers" (5.3-5.7 TB/s) that the configs[3] N = 4096 kernels
// (q31: 32 KiB, q15: 16 KiB per transform) could take:
//   tile  : TH-thread workgroups per transform (TH = 128: two waves), T consecutive transforms,
//           loads -> LDS -> __syncthreads -> transposed read -> __syncthreads -> stores, the next
//           transform's loads issued before the stores (PF);
//   pair  : a wave PAIR per transform, PAIRS pairs per workgroup and no s_barrier: wave h of a pair
//           loads half h, writes it to the pair's LDS image (double-buffered by transform parity),
//           publishes a flag, waits (s_sleep) for the partner's flag, reads the mirrored slot of the
//           whole transform and stores it; before overwriting a buffer it waits until the partner
//           has finished reading it.  EX = exchanges per transform (the kernels have 2-3).
// Every variant moves 8 GiB in place; prints TB/s of read + write.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
template <int VB> struct Vec;
template <> struct Vec<8> { using T = v2i; };
template <> struct Vec<16> { using T = v4i; };

template <int TH, int S, int VB, int T, bool PF>
__global__ __launch_bounds__(TH) void tile_kernel(int* __restrict__ x, int s) {
  using V = typename Vec<VB>::T;
  constexpr int PER = S / (TH * VB);
  extern __shared__ v4i lds_raw[];
  V* lds = reinterpret_cast<V*>(lds_raw);
  const int tid = threadIdx.x;
  const long t0 = (long)blockIdx.x * T;
  V r[PER];
  auto ld = [&](long t) {
    const V* p = reinterpret_cast<const V*>(reinterpret_cast<char*>(x) + t * S) + tid;
#pragma unroll
    for (int m = 0; m < PER; ++m) r[m] = __builtin_nontemporal_load(p + TH * m);
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
    V* q = reinterpret_cast<V*>(reinterpret_cast<char*>(x) + (t0 + t) * S) + tid;
#pragma unroll
    for (int m = 0; m < PER; ++m) __builtin_nontemporal_store(o[m], q + TH * m);
  }
}

template <int S, int VB, int T, int PAIRS, int EX>
__global__ __launch_bounds__(128 * PAIRS) void pair_kernel(int* __restrict__ x, int s) {
  using V = typename Vec<VB>::T;
  constexpr int H = S / 2;                 // bytes per wave
  constexpr int PER = H / (64 * VB);
  constexpr int NV = S / VB;               // vectors per transform
  extern __shared__ v4i lds_raw[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, p = w >> 1, h = w & 1;
  // layout: [PAIRS][2 buffers][NV vectors] then flags [PAIRS][2 waves][2: wrote, read]
  V* img = reinterpret_cast<V*>(lds_raw) + (size_t)p * 2 * NV;
  volatile int* flags = reinterpret_cast<volatile int*>(reinterpret_cast<V*>(lds_raw) + (size_t)PAIRS * 2 * NV);
  volatile int* mine = flags + (p * 2 + h) * 2;
  volatile int* other = flags + (p * 2 + (h ^ 1)) * 2;
  if (lane == 0) { mine[0] = 0; mine[1] = 0; }
  __syncthreads();                         // flags initialised (once per workgroup)
  const long t0 = ((long)blockIdx.x * PAIRS + p) * T;
  V r[PER];
  auto ld = [&](long t) {
    const V* q = reinterpret_cast<const V*>(reinterpret_cast<char*>(x) + t * S + h * H) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
  };
  auto wait_ge = [&](volatile int* f, int v) {
    while (*f < v) __builtin_amdgcn_s_sleep(1);
  };
  ld(t0);
  int gen = 0;                             // exchanges done so far by this wave
  for (int t = 0; t < T; ++t) {
    V o[PER];
#pragma unroll
    for (int e = 0; e < EX; ++e) {
      V* buf = img + (gen & 1) * NV;
      // the partner must have finished reading this buffer (exchange gen - 2)
      if (gen >= 2) wait_ge(other + 1, gen - 1);
#pragma unroll
      for (int m = 0; m < PER; ++m) buf[h * (NV / 2) + lane + 64 * m] = (e == 0 ? r[m] : o[m]) + s;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) mine[0] = gen + 1;
      wait_ge(other + 0, gen + 1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
      for (int m = 0; m < PER; ++m) o[m] = buf[(NV - 1) - (h * (NV / 2) + lane + 64 * m)];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) mine[1] = gen + 1;
      ++gen;
    }
    if (t + 1 < T) ld(t0 + t + 1);
    V* q = reinterpret_cast<V*>(reinterpret_cast<char*>(x) + (t0 + t) * S + h * H) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}

static void report(const char* what, float ms, long bytes) {
  printf("%s  %.3f ms  %.3f TB/s\n", what, ms, 2.0 * bytes / (ms * 1e-3) * 1e-12);
  fflush(stdout);
}

template <typename K>
static float run(K k, dim3 g, dim3 b, size_t lds, int* x, hipEvent_t e0, hipEvent_t e1) {
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, 1);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, g, b, lds, 0, x, 1);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

template <int TH, int S, int VB, int T, bool PF>
void tile(int* x, long bytes, int extra, hipEvent_t e0, hipEvent_t e1) {
  const size_t lds = S + extra;
  const float ms = run(tile_kernel<TH, S, VB, T, PF>, dim3(bytes / S / T), dim3(TH), lds, x, e0, e1);
  char w[160];
  snprintf(w, sizeof w, "tile TH=%4d S=%5d VB=%2d T=%2d PF=%d lds=%6zu (wg/CU<=%2zu)", TH, S, VB, T, PF, lds,
           (size_t)160 * 1024 / lds);
  report(w, ms, bytes);
}

template <int S, int VB, int T, int PAIRS, int EX>
void pair(int* x, long bytes, int extra, hipEvent_t e0, hipEvent_t e1) {
  const size_t lds = (size_t)PAIRS * 2 * S + PAIRS * 16 + extra;
  const float ms = run(pair_kernel<S, VB, T, PAIRS, EX>, dim3(bytes / S / T / PAIRS), dim3(128 * PAIRS), lds, x, e0, e1);
  char w[160];
  snprintf(w, sizeof w, "pair S=%5d VB=%2d T=%2d PAIRS=%d EX=%d lds=%6zu (wg/CU<=%2zu)", S, VB, T, PAIRS, EX, lds,
           (size_t)160 * 1024 / lds);
  report(w, ms, bytes);
}

int main() {
  const long bytes = 8L << 30;
  int* x;
  if (hipMalloc(&x, bytes) != hipSuccess) return 1;
  hipMemset(x, 0, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // two-wave workgroups per transform (q31: 32 KiB, q15: 16 KiB), occupancy by extra LDS
  tile<128, 32768, 16, 8, true>(x, bytes, 0, e0, e1);
  tile<128, 32768, 16, 4, true>(x, bytes, 0, e0, e1);
  tile<128, 32768, 8, 8, true>(x, bytes, 0, e0, e1);
  tile<128, 32768, 16, 8, true>(x, bytes, 20000, e0, e1);
  tile<128, 16384, 16, 8, true>(x, bytes, 0, e0, e1);
  tile<128, 16384, 16, 8, true>(x, bytes, 16000, e0, e1);
  // the 256-thread reference point
  tile<256, 32768, 16, 8, true>(x, bytes, 22528, e0, e1);
  // wave pairs with flag hand-offs, 1 and 3 exchanges per transform
  pair<32768, 16, 4, 1, 1>(x, bytes, 0, e0, e1);
  pair<32768, 16, 4, 2, 1>(x, bytes, 0, e0, e1);
  pair<32768, 16, 2, 1, 1>(x, bytes, 0, e0, e1);
  pair<32768, 16, 8, 1, 1>(x, bytes, 0, e0, e1);
  pair<32768, 16, 4, 1, 3>(x, bytes, 0, e0, e1);
  pair<32768, 8, 4, 1, 1>(x, bytes, 0, e0, e1);
  pair<16384, 16, 4, 1, 1>(x, bytes, 0, e0, e1);
  pair<16384, 16, 4, 2, 1>(x, bytes, 0, e0, e1);
  pair<16384, 16, 8, 2, 1>(x, bytes, 0, e0, e1);
  pair<16384, 16, 4, 2, 2>(x, bytes, 0, e0, e1);
  hipFree(x);
  return 0;
}
