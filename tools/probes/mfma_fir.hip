// Probe for an MFMA-assisted bit-exact FIR f32 (gfx950):
//  1. lane layout of v_mfma_f32_4x4x1_16b_f32 (which lane's A / B value lands in which D register);
//  2. whether D = 0 + a*b equals the VALU product round(a*b) bit for bit (normal, denormal,
//     inf/nan operands) -- the reference rounds each product before its add (arm_fir_f32.c);
//  3. whether 4x4x1 MFMAs and the v_add_f32 that consume their products co-execute
//     (products/s and adds/s of MFMA-only, add-only and mixed loops).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const float* a, const float* b, float* d, int n_waves) {
  const int w = blockIdx.x, l = threadIdx.x;
  if (w >= n_waves) return;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[w * 64 + l], b[w * 64 + l], acc, 0, 0, 0);
  for (int i = 0; i < 4; ++i) d[(w * 4 + i) * 64 + l] = acc[i];
}

constexpr int ITER = 2048;
// KIND 0: MFMA only (2 per step); 1: adds only (8 per step); 2: both (adds consume the
// previous step's products).
template <int KIND>
__global__ __launch_bounds__(256) void rate_kernel(float* out, float seed) {
  const int l = threadIdx.x;
  float x = seed + l * 0.001f;
  float c0 = 1.0001f + l * 1e-6f, c1 = 0.9999f - l * 1e-6f;
  f4 p0 = {x, x, x, x}, p1 = p0, acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const f4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int it = 0; it < ITER; ++it) {
    if constexpr (KIND == 0 || KIND == 2) {
      f4 q0 = __builtin_amdgcn_mfma_f32_4x4x1f32(c0, x, z, 0, 0, 0);
      f4 q1 = __builtin_amdgcn_mfma_f32_4x4x1f32(c1, x, z, 0, 0, 0);
      if constexpr (KIND == 2) { acc0 += p0; acc1 += p1; }
      else { acc0 = q0 - acc0; acc1 = q1 - acc1; }   // keep the results live (one VALU pair)
      p0 = q0; p1 = q1;
      x += 1.0f;   // next step's sample (a VALU op the real kernel replaces by an LDS read)
    } else {
      acc0 += p0; acc1 += p1;
      p0 = p0 * 0.5f; p1 = p1 * 0.5f;  // new values (stand-in for products)
    }
  }
  f4 s = acc0 + acc1;
  out[blockIdx.x * 256 + l] = s[0] + s[1] + s[2] + s[3];
}

static uint32_t rng = 12345;
static uint32_t nxt() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }
static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main() {
  const int W = 4096;   // waves per category
  std::vector<float> a(W * 64), b(W * 64), d(W * 256);
  float *da, *db, *dd;
  hipMalloc(&da, a.size() * 4); hipMalloc(&db, b.size() * 4); hipMalloc(&dd, d.size() * 4);
  // 1. layout with distinct small integers (exact products)
  for (int l = 0; l < 64; ++l) { a[l] = (float)(l + 1); b[l] = (float)(1000 * (l + 1)); }
  hipMemcpy(da, a.data(), 256, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, da, db, dd, 1);
  hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
  int h1 = 0, h2 = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const float v = d[i * 64 + l];
      h1 += v != a[4 * (l >> 2) + i] * b[l];
      h2 += v != a[l] * b[4 * (l >> 2) + i];
    }
  printf("layout: H1 D_i[l]=A[4(l>>2)+i]*B[l] mismatches %d/256; H2 D_i[l]=A[l]*B[4(l>>2)+i] mismatches %d/256\n", h1, h2);
  printf("lane0..5 reg0..3:");
  for (int l = 0; l < 6; ++l) { printf(" |"); for (int i = 0; i < 4; ++i) printf(" %g", d[i * 64 + l]); }
  printf("\n");
  // 2. exactness under H1 indexing, per operand class
  const char* cls[] = {"normal (exp 100..154)", "products near/below 2^-126", "denormal operand", "any bit pattern"};
  for (int c = 0; c < 4; ++c) {
    for (int k = 0; k < W * 64; ++k) {
      uint32_t ua = nxt(), ub = nxt();
      if (c == 0) { ua = (ua & 0x807fffffu) | ((100u + nxt() % 55) << 23); ub = (ub & 0x807fffffu) | ((100u + nxt() % 55) << 23); }
      if (c == 1) { ua = (ua & 0x807fffffu) | ((40u + nxt() % 30) << 23); ub = (ub & 0x807fffffu) | ((40u + nxt() % 30) << 23); }
      if (c == 2) { ua = ua & 0x807fffffu; ub = (ub & 0x807fffffu) | ((120u + nxt() % 40) << 23); }
      a[k] = bits(ua); b[k] = bits(ub);
    }
    hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(layout_kernel, dim3(W), dim3(64), 0, 0, da, db, dd, W);
    hipMemcpy(d.data(), dd, d.size() * 4, hipMemcpyDeviceToHost);
    long mism = 0, nan_ok = 0, tot = 0; int shown = 0;
    for (int w = 0; w < W; ++w)
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) {
          const float ref = a[w * 64 + 4 * (l >> 2) + i] * b[w * 64 + l];
          const float got = d[(w * 4 + i) * 64 + l];
          ++tot;
          if (std::isnan(ref) && std::isnan(got)) { ++nan_ok; continue; }
          if (ubits(ref) != ubits(got)) {
            ++mism;
            if (shown++ < 4) printf("   a=%08x b=%08x ref=%08x got=%08x\n", ubits(a[w * 64 + 4 * (l >> 2) + i]), ubits(b[w * 64 + l]), ubits(ref), ubits(got));
          }
        }
    printf("exact: %-28s mismatches %ld / %ld (nan both %ld)\n", cls[c], mism, tot, nan_ok);
  }
  // 3. co-execution rates
  float* out; hipMalloc(&out, sizeof(float) * 256 * 256 * 8 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[] = {"mfma only (2x4x4x1/step)", "add only (8 v_add/step)", "mfma + add"};
  for (int kind = 0; kind < 3; ++kind)
    for (int waves = 1; waves <= 4; waves *= 2) {
      const int grid = 256 * waves;
      auto k = kind == 0 ? rate_kernel<0> : kind == 1 ? rate_kernel<1> : rate_kernel<2>;
      hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, 1.0f);
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, (float)r);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double steps = 5.0 * grid * 4.0 * ITER;   // wave-steps (4 waves per block)
      printf("%-26s waves/SIMD=%d  %7.2f T products/s (512 per wave-step)  %.3f ms\n", names[kind], waves,
             steps * 512 / (ms * 1e-3) * 1e-12, ms / 5);
    }
  return 0;
}
