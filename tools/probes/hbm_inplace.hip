// In-place streaming ceiling probe (gfx950) for the CFFT access pattern: every wave owns
// 8 KiB chunks (one N=1024 f32 transform), reads the whole chunk, writes it back (x*s),
// persistent grid walking the batch with stride = grid.  Variants: load width 8/16 B per
// lane, nontemporal loads/stores, waves per workgroup, resident waves per CU (grid size),
// and "pipelined" = the next chunk's loads issued before the current chunk is stored (as
// the FFT kernel does).  Prints TB/s of read+write for each variant over 8 GiB.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float v2f __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int W, bool NTL, bool NTS, bool PIPE>
__global__ void stream_kernel(float* __restrict__ x, long chunks, float s) {
  using V = typename std::conditional<W == 8, v2f, v4f>::type;
  constexpr int PER = 8192 / (64 * W);           // vector loads per lane per chunk
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * (blockDim.x >> 6);
  V r[PER];
  auto load = [&](long c) {
    const V* p = reinterpret_cast<const V*>(x + c * 2048) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) r[m] = NTL ? __builtin_nontemporal_load(p + 64 * m) : p[64 * m];
  };
  long c = wave;
  if (PIPE && c < chunks) load(c);
  for (; c < chunks; c += nw) {
    if (!PIPE) load(c);
    V o[PER];
#pragma unroll
    for (int m = 0; m < PER; ++m) o[m] = r[m] * s;
    if (PIPE && c + nw < chunks) load(c + nw);
    V* q = reinterpret_cast<V*>(x + c * 2048) + lane;
#pragma unroll
    for (int m = 0; m < PER; ++m) {
      if (NTS) __builtin_nontemporal_store(o[m], q + 64 * m); else q[64 * m] = o[m];
    }
  }
}

// One wave per chunk, no persistent loop (grid = chunks / waves per block).
template <bool NT>
__global__ void oneshot_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63;
  const long c = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  v4f* q = reinterpret_cast<v4f*>(x + c * 2048) + lane;
  v4f r[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) r[m] = NT ? __builtin_nontemporal_load(q + 64 * m) : q[64 * m];
#pragma unroll
  for (int m = 0; m < 8; ++m) { if (NT) __builtin_nontemporal_store(r[m] * s, q + 64 * m); else q[64 * m] = r[m] * s; }
}

// Each wave T consecutive chunks, next chunk prefetched before the current one is stored.
template <int T>
__global__ void tchunk_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63;
  const long c0 = ((long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * T;
  v4f r[8];
  {
    const v4f* q = reinterpret_cast<const v4f*>(x + c0 * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
  }
  for (int t = 0; t < T; ++t) {
    v4f o[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) o[m] = r[m] * s;
    if (t + 1 < T) {
      const v4f* q = reinterpret_cast<const v4f*>(x + (c0 + t + 1) * 2048) + lane;
#pragma unroll
      for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
    }
    v4f* q = reinterpret_cast<v4f*>(x + (c0 + t) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}

// tchunk with the N=1024 FFT kernel's widths: 8-B loads (16 per chunk, 512 B per wave
// instruction) and 16-B stores (8 per chunk), no prefetch.
template <int T>
__global__ void tchunk8_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63;
  const long c0 = ((long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * T;
  for (int t = 0; t < T; ++t) {
    const v2f* q = reinterpret_cast<const v2f*>(x + (c0 + t) * 2048) + lane;
    v2f r[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
    v4f* o = reinterpret_cast<v4f*>(x + (c0 + t) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      v4f w = {r[2 * m].x, r[2 * m].y, r[2 * m + 1].x, r[2 * m + 1].y};
      __builtin_nontemporal_store(w * s, o + 64 * m);
    }
  }
}

// Each wave T chunks interleaved by the grid (chunk = wave + t * waves), pipelined.
template <int T>
__global__ void tstride_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63;
  const long w = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long nw = (long)gridDim.x * (blockDim.x >> 6);
  v4f r[8];
  {
    const v4f* q = reinterpret_cast<const v4f*>(x + w * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
  }
  for (int t = 0; t < T; ++t) {
    v4f o[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) o[m] = r[m] * s;
    if (t + 1 < T) {
      const v4f* q = reinterpret_cast<const v4f*>(x + (w + (t + 1) * nw) * 2048) + lane;
#pragma unroll
      for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
    }
    v4f* q = reinterpret_cast<v4f*>(x + (w + t * nw) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}

// Each workgroup T x W chunks; at step t its W waves take W ADJACENT chunks
// ((b*T + t)*W + w), so the workgroup's live footprint is one contiguous W*8 KiB span.
template <int T, bool PF>
__global__ void wgil_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
  const long base = (long)blockIdx.x * T * W + w;
  v4f r[8];
  auto ld = [&](long c) {
    const v4f* q = reinterpret_cast<const v4f*>(x + c * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * m);
  };
  if (PF) ld(base);
  for (int t = 0; t < T; ++t) {
    if (!PF) ld(base + (long)t * W);
    v4f o[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) o[m] = r[m] * s;
    if (PF && t + 1 < T) ld(base + (long)(t + 1) * W);
    v4f* q = reinterpret_cast<v4f*>(x + (base + (long)t * W) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(o[m], q + 64 * m);
  }
}

// tchunk with the 8 row loads/stores of a chunk issued in a per-wave rotated order
// (row (m + R*wave) & 7), so concurrently issuing waves hit different 1 KiB rows.
template <int T, int R>
__global__ void trot_kernel(float* __restrict__ x, float s) {
  const int lane = threadIdx.x & 63;
  const long wv = (long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long c0 = wv * T;
  const int rot = (int)(wv * R) & 7;
  v4f r[8];
  for (int t = 0; t < T; ++t) {
    const v4f* q = reinterpret_cast<const v4f*>(x + (c0 + t) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + 64 * ((m + rot) & 7));
    v4f* o = reinterpret_cast<v4f*>(x + (c0 + t) * 2048) + lane;
#pragma unroll
    for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(r[m] * s, o + 64 * ((m + rot) & 7));
  }
}

// Cooperative flat access: a workgroup of W waves owns T x W consecutive chunks; at step t
// its instruction m of thread j moves float4 m*64W + j of the step's W*8 KiB span (every
// workgroup instruction covers W KiB contiguous).
template <int T, int W>
__global__ void coop_kernel(float* __restrict__ x, float s) {
  const int j = threadIdx.x;
  for (int t = 0; t < T; ++t) {
    v4f* q = reinterpret_cast<v4f*>(x + ((long)blockIdx.x * T + t) * W * 2048) + j;
    v4f r[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) r[m] = __builtin_nontemporal_load(q + m * 64 * W);
#pragma unroll
    for (int m = 0; m < 8; ++m) __builtin_nontemporal_store(r[m] * s, q + m * 64 * W);
  }
}

// torch-like flat elementwise: each thread U float4 at block-contiguous offsets.
template <int U, bool NT>
__global__ void flat_kernel(float* __restrict__ x, float s) {
  const long base = (long)blockIdx.x * blockDim.x * U + threadIdx.x;
  v4f* q = reinterpret_cast<v4f*>(x);
  v4f r[U];
#pragma unroll
  for (int m = 0; m < U; ++m) r[m] = NT ? __builtin_nontemporal_load(q + base + m * blockDim.x) : q[base + m * blockDim.x];
#pragma unroll
  for (int m = 0; m < U; ++m) {
    if (NT) __builtin_nontemporal_store(r[m] * s, q + base + m * blockDim.x); else q[base + m * blockDim.x] = r[m] * s;
  }
}

template <typename K>
void timeit(const char* name, K k, dim3 g, dim3 b, float* x, long bytes, hipEvent_t e0, hipEvent_t e1) {
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, g, b, 0, 0, x, 1.0000001f);
  hipEventRecord(e0);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k, g, b, 0, 0, x, 1.0000001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 10;
  printf("%-28s grid=%8u blk=%4u  %.3f ms  %.3f TB/s\n", name, g.x, b.x, ms, 2.0 * bytes / (ms * 1e-3) * 1e-12);
}

template <int W, bool NTL, bool NTS, bool PIPE>
void run(float* x, long chunks, int wpb, int wpc, int cus, hipEvent_t e0, hipEvent_t e1) {
  const int grid = cus * wpc / wpb;
  auto k = stream_kernel<W, NTL, NTS, PIPE>;
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * wpb), 0, 0, x, chunks, 1.0000001f);
  hipEventRecord(e0);
  const int it = 10;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k, dim3(grid), dim3(64 * wpb), 0, 0, x, chunks, 1.0000001f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= it;
  printf("W=%2d ntl=%d nts=%d pipe=%d wpb=%d wpc=%2d  %.3f ms  %.3f TB/s\n", W, NTL, NTS, PIPE, wpb, wpc, ms,
         2.0 * chunks * 8192 / (ms * 1e-3) * 1e-12);
}

int main() {
  const long chunks = 1L << 20;                      // 8 GiB
  float* x;
  if (hipMalloc(&x, chunks * 8192) != hipSuccess) return 1;
  hipMemset(x, 0, chunks * 8192);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long bytes = chunks * 8192;
  for (int rep = 0; rep < 2; ++rep) {
    char nm[64];
#define TCH(T, WPB) snprintf(nm, 64, "tchunk T%d wpb%d", T, WPB); \
    timeit(nm, tchunk_kernel<T>, dim3(chunks / (T * WPB)), dim3(64 * WPB), x, bytes, e0, e1);
#define COOP(T, WPB) snprintf(nm, 64, "coop T%d wpb%d", T, WPB); \
    timeit(nm, coop_kernel<T, WPB>, dim3(chunks / (T * WPB)), dim3(64 * WPB), x, bytes, e0, e1);
    TCH(4, 8)
    snprintf(nm, 64, "tchunk8 T4 wpb8");
    timeit(nm, tchunk8_kernel<4>, dim3(chunks / 32), dim3(512), x, bytes, e0, e1);
    snprintf(nm, 64, "tchunk8 T4 wpb4");
    timeit(nm, tchunk8_kernel<4>, dim3(chunks / 16), dim3(256), x, bytes, e0, e1);
    COOP(1, 1) COOP(1, 4) COOP(1, 8) COOP(2, 4) COOP(2, 8) COOP(4, 4) COOP(4, 8) COOP(8, 8) COOP(1, 16) COOP(2, 16)
    timeit("flat U1 nt", flat_kernel<1, true>, dim3(bytes / 16 / 1 / 256), dim3(256), x, bytes, e0, e1);
    timeit("flat U8 nt", flat_kernel<8, true>, dim3(bytes / 16 / 8 / 256), dim3(256), x, bytes, e0, e1);
  }
  hipFree(x);
  return 0;
}
