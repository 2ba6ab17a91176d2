/*
 * ORACLE — test infrastructure: the CPU baseline timing driver (bench.py cpu_baseline).
 * Built twice from this one file:
 *   oracle/_ref/bench_ref   -DBENCH_AGAINST_REFERENCE: linked to the reference's own
 *                           objects (oracle/ref.mk) -> cpu_baseline.kind "reference";
 *   oracle/_build/bench_port -DBENCH_AGAINST_ORACLE: linked to the restatement -> "port".
 * Usage: bench_xxx <workload> <n> <threads> <seconds>
 *   workload: cfft_f32 | cfft_q31 | cfft_q15 (n = fftLen), fir_f32 | fir_q15 (n = numTaps, block 4096),
 *             rfft_f32 | rfft_q31 | rfft_q15 (n = real length, forward),
 *             mat_mult_f32 / mat_mult_q7 / mat_mult_q15 / mat_mult_q31 (n = square dimension), mfcc_f32 / mfcc_q31 / mfcc_q15 (n = fftLen; 20 triangular
 *             Mel filters, 13 DCT outputs, Hamming window -- the suite's shape)
 * Each thread owns its own buffers (the library is reentrant) and runs until the time
 * budget is spent; in-place transforms alternate forward / inverse to stay bounded.
 * Prints one JSON object: samples processed, seconds, threads, rate.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <time.h>

#ifdef BENCH_AGAINST_REFERENCE
#include "arm_math.h"
#include "arm_const_structs.h"
#define F(name) name
#else
#include "src/oracle.h"
#define F(name) oracle_##name
arm_status oracle_arm_cfft_init_f32(arm_cfft_instance_f32 *S, uint16_t n);
arm_status oracle_arm_cfft_init_q31(arm_cfft_instance_q31 *S, uint16_t n);
arm_status oracle_arm_cfft_init_q15(arm_cfft_instance_q15 *S, uint16_t n);
void oracle_arm_fir_init_f32(arm_fir_instance_f32 *S, uint16_t numTaps, const float *pCoeffs, float *pState,
                             uint32_t blockSize);
arm_status oracle_arm_rfft_fast_init_f32(arm_rfft_fast_instance_f32 *S, uint16_t n);
void oracle_arm_conv_f32(const float *pSrcA, uint32_t srcALen, const float *pSrcB, uint32_t srcBLen, float *pDst);
void oracle_arm_fir_init_q31(arm_fir_instance_q31 *S, uint16_t numTaps, const int32_t *pCoeffs, int32_t *pState,
                             uint32_t blockSize);
arm_status oracle_arm_fir_init_q15(arm_fir_instance_q15 *S, uint16_t numTaps, const int16_t *pCoeffs,
                                   int16_t *pState, uint32_t blockSize);
void oracle_arm_mat_init_q7(arm_matrix_instance_q7 *S, uint16_t r, uint16_t c, int8_t *p);
void oracle_arm_mat_init_q15(arm_matrix_instance_q15 *S, uint16_t r, uint16_t c, int16_t *p);
void oracle_arm_mat_init_q31(arm_matrix_instance_q31 *S, uint16_t r, uint16_t c, int32_t *p);
void oracle_arm_mat_init_f32(arm_matrix_instance_f32 *S, uint16_t r, uint16_t c, float *p);
#endif

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct { const char *wl; int n; double seconds; int tid; double samples; double flops; } job_t;

static uint64_t sm(uint64_t *s) {   /* splitmix64 */
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static float uni(uint64_t *s) { return (float)((sm(s) >> 40) * (1.0 / 16777216.0)) - 0.5f; }

static void *worker(void *arg) {
  job_t *j = (job_t *)arg;
  uint64_t seed = 0x5EEDull + 7919ull * (uint64_t)j->tid;
  const double t0 = now();
  double samples = 0;
  if (!strncmp(j->wl, "cfft_", 5)) {
    const int n = j->n;
    float *xf = malloc(sizeof(float) * 2 * n);
    int32_t *xi = malloc(sizeof(int32_t) * 2 * n);
    int16_t *xs = malloc(sizeof(int16_t) * 2 * n);
    for (int i = 0; i < 2 * n; ++i) { xf[i] = uni(&seed); xi[i] = (int32_t)sm(&seed); xs[i] = (int16_t)(sm(&seed) >> 7); }
    arm_cfft_instance_f32 Sf; arm_cfft_instance_q31 S31; arm_cfft_instance_q15 S15;
    F(arm_cfft_init_f32)(&Sf, n); F(arm_cfft_init_q31)(&S31, n); F(arm_cfft_init_q15)(&S15, n);
    uint64_t it = 0;
    do {
      for (int r = 0; r < 16; ++r, ++it) {
        if (!strcmp(j->wl, "cfft_f32")) F(arm_cfft_f32)(&Sf, xf, (uint8_t)(it & 1), 1);
        else if (!strcmp(j->wl, "cfft_q31")) F(arm_cfft_q31)(&S31, xi, 0, 1);
        else F(arm_cfft_q15)(&S15, xs, 0, 1);
      }
      samples += 16.0 * n;
    } while (now() - t0 < j->seconds);
    free(xf); free(xi); free(xs);
  } else if (!strcmp(j->wl, "fir_f32")) {
    const int taps = j->n, block = 4096;
    float *c = malloc(sizeof(float) * taps), *st = malloc(sizeof(float) * (taps + block - 1));
    float *in = malloc(sizeof(float) * block), *out = malloc(sizeof(float) * block);
    for (int i = 0; i < taps; ++i) c[i] = uni(&seed) * 0.1f;
    for (int i = 0; i < block; ++i) in[i] = uni(&seed);
    arm_fir_instance_f32 S;
    F(arm_fir_init_f32)(&S, (uint16_t)taps, c, st, block);
    do { F(arm_fir_f32)(&S, in, out, block); samples += block; } while (now() - t0 < j->seconds);
    free(c); free(st); free(in); free(out);
  } else if (!strcmp(j->wl, "fir_q31") || !strcmp(j->wl, "fir_fast_q31")) {
    const int taps = j->n, block = 4096, fast = !strcmp(j->wl, "fir_fast_q31");
    int32_t *c = malloc(sizeof(int32_t) * taps), *st = malloc(sizeof(int32_t) * (taps + block - 1));
    int32_t *in = malloc(sizeof(int32_t) * block), *out = malloc(sizeof(int32_t) * block);
    for (int i = 0; i < taps; ++i) c[i] = (int32_t)(sm(&seed) >> 36);
    for (int i = 0; i < block; ++i) in[i] = (int32_t)sm(&seed);
    arm_fir_instance_q31 S;
    F(arm_fir_init_q31)(&S, (uint16_t)taps, c, st, block);
    do {
      if (fast) F(arm_fir_fast_q31)(&S, in, out, block); else F(arm_fir_q31)(&S, in, out, block);
      samples += block;
    } while (now() - t0 < j->seconds);
    free(c); free(st); free(in); free(out);
  } else if (!strcmp(j->wl, "fir_q15") || !strcmp(j->wl, "fir_fast_q15")) {
    const int taps = j->n, block = 4096;
    int16_t *c = malloc(sizeof(int16_t) * taps), *st = malloc(sizeof(int16_t) * (taps + block - 1));
    int16_t *in = malloc(sizeof(int16_t) * block), *out = malloc(sizeof(int16_t) * block);
    for (int i = 0; i < taps; ++i) c[i] = (int16_t)(sm(&seed) >> 52);
    for (int i = 0; i < block; ++i) in[i] = (int16_t)(sm(&seed) >> 48);
    arm_fir_instance_q15 S;
    F(arm_fir_init_q15)(&S, (uint16_t)taps, c, st, block);
    const int fast = !strcmp(j->wl, "fir_fast_q15");
    do {
      if (fast) F(arm_fir_fast_q15)(&S, in, out, block); else F(arm_fir_q15)(&S, in, out, block);
      samples += block;
    } while (now() - t0 < j->seconds);
    free(c); free(st); free(in); free(out);
  } else if (!strcmp(j->wl, "conv_f32")) {
    const int taps = j->n, block = 4096;
    float *a = malloc(sizeof(float) * block), *b = malloc(sizeof(float) * taps), *y = malloc(sizeof(float) * (block + taps));
    for (int i = 0; i < block; ++i) a[i] = uni(&seed);
    for (int i = 0; i < taps; ++i) b[i] = uni(&seed);
    do { F(arm_conv_f32)(a, block, b, taps, y); samples += block + taps - 1; } while (now() - t0 < j->seconds);
    free(a); free(b); free(y);
  } else if (!strcmp(j->wl, "rfft_f32")) {
    const int n = j->n;
    float *x = malloc(sizeof(float) * n), *p = malloc(sizeof(float) * n), *o = malloc(sizeof(float) * n);
    for (int i = 0; i < n; ++i) x[i] = uni(&seed);
    arm_rfft_fast_instance_f32 S;
    F(arm_rfft_fast_init_f32)(&S, (uint16_t)n);
    do {
      for (int r = 0; r < 16; ++r) { memcpy(p, x, sizeof(float) * n); F(arm_rfft_fast_f32)(&S, p, o, 0); }
      samples += 16.0 * n;
    } while (now() - t0 < j->seconds);
    free(x); free(p); free(o);
  } else if (!strcmp(j->wl, "rfft_q31") || !strcmp(j->wl, "rfft_q15")) {
    const int n = j->n, q31 = !strcmp(j->wl, "rfft_q31");
    int32_t *x31 = malloc(sizeof(int32_t) * n), *p31 = malloc(sizeof(int32_t) * n), *o31 = malloc(sizeof(int32_t) * 2 * n);
    int16_t *x15 = malloc(sizeof(int16_t) * n), *p15 = malloc(sizeof(int16_t) * n), *o15 = malloc(sizeof(int16_t) * 2 * n);
    for (int i = 0; i < n; ++i) { x31[i] = (int32_t)sm(&seed); x15[i] = (int16_t)(sm(&seed) >> 7); }
    arm_rfft_instance_q31 S31; arm_rfft_instance_q15 S15;
    F(arm_rfft_init_q31)(&S31, (uint32_t)n, 0, 1); F(arm_rfft_init_q15)(&S15, (uint32_t)n, 0, 1);
    do {
      for (int r = 0; r < 16; ++r) {
        if (q31) { memcpy(p31, x31, sizeof(int32_t) * n); F(arm_rfft_q31)(&S31, p31, o31); }
        else { memcpy(p15, x15, sizeof(int16_t) * n); F(arm_rfft_q15)(&S15, p15, o15); }
      }
      samples += 16.0 * n;
    } while (now() - t0 < j->seconds);
    free(x31); free(p31); free(o31); free(x15); free(p15); free(o15);
  } else if (!strcmp(j->wl, "mfcc_f32")) {
    const int n = j->n, nm = 20, nd = 13;
    uint32_t pos[20], len[20], total = 0;
    float *coefs = malloc(sizeof(float) * n), dct[13 * 20];
    float *win = malloc(sizeof(float) * n), *x = malloc(sizeof(float) * n), *src = malloc(sizeof(float) * n);
    float *tmp = calloc(2 * n, sizeof(float)), out[13];
    for (int i = 0; i < nm; ++i) {                   /* evenly spaced triangles below n/2 */
      pos[i] = 1 + (uint32_t)i * (n / 2 - 2) / (nm + 1);
      len[i] = 2 * ((n / 2 - 2) / (nm + 1)) + 1;
      if (pos[i] + len[i] > (uint32_t)n / 2) len[i] = n / 2 - pos[i];
      for (uint32_t k = 0; k < len[i]; ++k) coefs[total + k] = 1.0f - fabsf((float)k - len[i] / 2.0f) / len[i];
      total += len[i];
    }
    for (int r = 0; r < nd; ++r)
      for (int c = 0; c < nm; ++c) dct[r * nm + c] = (float)cos(3.14159265358979 / nm * (c + 0.5) * r);
    for (int i = 0; i < n; ++i) { win[i] = 0.54f - 0.46f * (float)cos(6.283185307179586 * i / n); x[i] = uni(&seed); }
    arm_mfcc_instance_f32 S;
    F(arm_mfcc_init_f32)(&S, n, nm, nd, dct, pos, len, coefs, win);
    do {
      memcpy(src, x, sizeof(float) * n);
      F(arm_mfcc_f32)(&S, src, out, tmp);
      samples += n;
    } while (now() - t0 < j->seconds);
    free(coefs); free(win); free(x); free(src); free(tmp);
  } else if (!strcmp(j->wl, "mfcc_q31")) {           /* the same shape in q31 */
    const int n = j->n, nm = 20, nd = 13;
    uint32_t pos[20], len[20], total = 0;
    int32_t *coefs = malloc(sizeof(int32_t) * n), dct[13 * 20];
    int32_t *win = malloc(sizeof(int32_t) * n), *x = malloc(sizeof(int32_t) * n), *src = malloc(sizeof(int32_t) * n);
    int32_t *tmp = calloc(2 * n, sizeof(int32_t)), out[13];
    for (int i = 0; i < nm; ++i) {
      pos[i] = 1 + (uint32_t)i * (n / 2 - 2) / (nm + 1);
      len[i] = 2 * ((n / 2 - 2) / (nm + 1)) + 1;
      if (pos[i] + len[i] > (uint32_t)n / 2) len[i] = n / 2 - pos[i];
      for (uint32_t k = 0; k < len[i]; ++k)
        coefs[total + k] = (int32_t)(2147483647.0 * (1.0 - fabs((double)k - len[i] / 2.0) / len[i]));
      total += len[i];
    }
    for (int r = 0; r < nd; ++r)
      for (int c = 0; c < nm; ++c) dct[r * nm + c] = (int32_t)(0.3 * 2147483647.0 * cos(3.14159265358979 / nm * (c + 0.5) * r));
    for (int i = 0; i < n; ++i) {
      win[i] = (int32_t)(2147483647.0 * (0.54 - 0.46 * cos(6.283185307179586 * i / n)));
      x[i] = (int32_t)sm(&seed);
    }
    arm_mfcc_instance_q31 S;
    F(arm_mfcc_init_q31)(&S, n, nm, nd, dct, pos, len, coefs, win);
    do {
      memcpy(src, x, sizeof(int32_t) * n);
      F(arm_mfcc_q31)(&S, src, out, tmp);
      samples += n;
    } while (now() - t0 < j->seconds);
    free(coefs); free(win); free(x); free(src); free(tmp);
  } else if (!strcmp(j->wl, "mfcc_q15")) {           /* the same shape in q15 */
    const int n = j->n, nm = 20, nd = 13;
    uint32_t pos[20], len[20], total = 0;
    int16_t *coefs = malloc(sizeof(int16_t) * n), dct[13 * 20];
    int16_t *win = malloc(sizeof(int16_t) * n), *x = malloc(sizeof(int16_t) * n), *src = malloc(sizeof(int16_t) * n);
    int32_t *tmp = calloc(2 * n, sizeof(int32_t));
    int16_t out[13];
    for (int i = 0; i < nm; ++i) {
      pos[i] = 1 + (uint32_t)i * (n / 2 - 2) / (nm + 1);
      len[i] = 2 * ((n / 2 - 2) / (nm + 1)) + 1;
      if (pos[i] + len[i] > (uint32_t)n / 2) len[i] = n / 2 - pos[i];
      for (uint32_t k = 0; k < len[i]; ++k)
        coefs[total + k] = (int16_t)(32767.0 * (1.0 - fabs((double)k - len[i] / 2.0) / len[i]));
      total += len[i];
    }
    for (int r = 0; r < nd; ++r)
      for (int c = 0; c < nm; ++c) dct[r * nm + c] = (int16_t)(0.3 * 32767.0 * cos(3.14159265358979 / nm * (c + 0.5) * r));
    for (int i = 0; i < n; ++i) {
      win[i] = (int16_t)(32767.0 * (0.54 - 0.46 * cos(6.283185307179586 * i / n)));
      x[i] = (int16_t)sm(&seed);
    }
    arm_mfcc_instance_q15 S;
    F(arm_mfcc_init_q15)(&S, n, nm, nd, dct, pos, len, coefs, win);
    do {
      memcpy(src, x, sizeof(int16_t) * n);
      F(arm_mfcc_q15)(&S, src, out, tmp);
      samples += n;
    } while (now() - t0 < j->seconds);
    free(coefs); free(win); free(x); free(src); free(tmp);
  } else if (!strcmp(j->wl, "mat_mult_q15") || !strcmp(j->wl, "mat_mult_q31") || !strcmp(j->wl, "mat_mult_fast_q31")) {
    const int d = j->n, q15 = !strcmp(j->wl, "mat_mult_q15"), fast = !strcmp(j->wl, "mat_mult_fast_q31");
    int16_t *a16 = malloc(2 * d * d), *b16 = malloc(2 * d * d), *o16 = malloc(2 * d * d), *st16 = malloc(2 * d * d);
    int32_t *a32 = malloc(4 * d * d), *b32 = malloc(4 * d * d), *o32 = malloc(4 * d * d);
    for (int i = 0; i < d * d; ++i) { a16[i] = (int16_t)sm(&seed); b16[i] = (int16_t)sm(&seed); a32[i] = (int32_t)sm(&seed); b32[i] = (int32_t)sm(&seed); }
    arm_matrix_instance_q15 A15, B15, O15;
    arm_matrix_instance_q31 A31, B31, O31;
    F(arm_mat_init_q15)(&A15, d, d, a16); F(arm_mat_init_q15)(&B15, d, d, b16); F(arm_mat_init_q15)(&O15, d, d, o16);
    F(arm_mat_init_q31)(&A31, d, d, a32); F(arm_mat_init_q31)(&B31, d, d, b32); F(arm_mat_init_q31)(&O31, d, d, o32);
    do {
      if (q15) F(arm_mat_mult_q15)(&A15, &B15, &O15, st16);
      else if (fast) F(arm_mat_mult_fast_q31)(&A31, &B31, &O31);
      else F(arm_mat_mult_q31)(&A31, &B31, &O31);
      samples += (double)d * d; j->flops += 2.0 * d * d * d;
    } while (now() - t0 < j->seconds);
    free(a16); free(b16); free(o16); free(st16); free(a32); free(b32); free(o32);
  } else if (!strcmp(j->wl, "mat_mult_q7")) {
    const int d = j->n;
    int8_t *a = malloc((size_t)d * d), *b = malloc((size_t)d * d), *o = malloc((size_t)d * d), *st = malloc((size_t)d * d);
    for (int i = 0; i < d * d; ++i) { a[i] = (int8_t)sm(&seed); b[i] = (int8_t)sm(&seed); }
    arm_matrix_instance_q7 A, B, O;
    F(arm_mat_init_q7)(&A, d, d, a); F(arm_mat_init_q7)(&B, d, d, b); F(arm_mat_init_q7)(&O, d, d, o);
    do { F(arm_mat_mult_q7)(&A, &B, &O, st); samples += (double)d * d; j->flops += 2.0 * d * d * d; }
    while (now() - t0 < j->seconds);
    free(a); free(b); free(o); free(st);
  } else if (!strcmp(j->wl, "mat_mult_f32")) {
    const int d = j->n;
    float *a = malloc(sizeof(float) * d * d), *b = malloc(sizeof(float) * d * d), *o = malloc(sizeof(float) * d * d);
    for (int i = 0; i < d * d; ++i) { a[i] = uni(&seed); b[i] = uni(&seed); }
    arm_matrix_instance_f32 A, B, O;
    F(arm_mat_init_f32)(&A, d, d, a); F(arm_mat_init_f32)(&B, d, d, b); F(arm_mat_init_f32)(&O, d, d, o);
    do { F(arm_mat_mult_f32)(&A, &B, &O); samples += (double)d * d; j->flops += 2.0 * d * d * d; }
    while (now() - t0 < j->seconds);
    free(a); free(b); free(o);
  }
  j->samples = samples;
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 5) { fprintf(stderr, "usage: %s workload n threads seconds\n", argv[0]); return 2; }
  const char *wl = argv[1];
  const int n = atoi(argv[2]), threads = atoi(argv[3]);
  const double secs = atof(argv[4]);
  pthread_t th[512];
  job_t jobs[512];
  const double t0 = now();
  for (int t = 0; t < threads && t < 512; ++t) {
    jobs[t] = (job_t){wl, n, secs, t, 0, 0};
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  double samples = 0, flops = 0;
  for (int t = 0; t < threads && t < 512; ++t) { pthread_join(th[t], NULL); samples += jobs[t].samples; flops += jobs[t].flops; }
  const double el = now() - t0;
  printf("{\"workload\": \"%s\", \"n\": %d, \"threads\": %d, \"seconds\": %.4f, \"samples\": %.0f, "
         "\"gsamples_per_s\": %.6f, \"gflops\": %.4f}\n", wl, n, threads, el, samples, samples / el * 1e-9,
         flops / el * 1e-9);
  return 0;
}
