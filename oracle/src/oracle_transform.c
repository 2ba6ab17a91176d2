/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Never linked, loaded or called by the product library.
 *
 * Plain-C restatement of the reference's scalar transform path, written against the
 * arithmetic contract rather than the reference's code layout:
 *   CFFT f32  Source/TransformFunctions/arm_cfft_f32.c:1243-1298 (dispatch, conj/scale),
 *             :846-958 (radix8by2), :960-1201 (radix8by4), arm_cfft_radix8_f32.c:51-291
 *   CFFT q31  arm_cfft_q31.c:704-755, :763-881, arm_cfft_radix4_q31.c:153-473, :524-834
 *   CFFT q15  arm_cfft_q15.c:671-722, :782-827, :881-926 (scalar, !ARM_MATH_DSP),
 *             arm_cfft_radix4_q15.c:572-970, :1434-1813 (scalar branches)
 *   bit reversal  arm_bitreversal2.c:84-148 (sequential swaps of complex pairs)
 *   RFFT fast f32 arm_rfft_fast_f32.c:316-462, :675-699
 *   RFFT q31/q15  arm_rfft_q31.c:148-183, :256-476; arm_rfft_q15.c (scalar branches)
 * Pinned by tests/test_oracle.py against oracle/_ref (the reference compiled from its
 * own sources) bit for bit, and against the reference's Testing/Patterns fixtures.
 * Build: make -C oracle  (gcc, -O2, -ffp-contract=off).
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

/* ------------------------------------------------------------------ helpers */
typedef struct { float re, im; } cpx;

static int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static int32_t wshl1(int32_t a) { return (int32_t)((uint32_t)a << 1); }
static int32_t hi32(int32_t a, int32_t b) { return (int32_t)(((int64_t)a * b) >> 32); }
static int32_t sat16(int32_t v) { return v > 32767 ? 32767 : v < -32768 ? -32768 : v; }
static int32_t tr16(int32_t v) { return (int32_t)(int16_t)(uint16_t)(uint32_t)v; }

/* complex multiply by a table twiddle in the reference's form: (a*c + b*s, b*c - a*s) */
static cpx twmul(float a, float b, const float *w) {
  cpx r;
  r.re = w[0] * a + w[1] * b;
  r.im = w[0] * b - w[1] * a;
  return r;
}

/* ---- the table-driven permutation: swap complex pairs named by byte offset / 8 ---- */
static void swap_pairs_words(void *buf, size_t word, const uint16_t *tab, uint16_t len) {
  uint8_t tmp[8];
  uint8_t *b = (uint8_t *)buf;
  for (uint32_t i = 0; i + 1 < len; i += 2) {
    size_t x = (size_t)(tab[i] >> 2) * word, y = (size_t)(tab[i + 1] >> 2) * word;
    memcpy(tmp, b + x, 2 * word);
    memcpy(b + x, b + y, 2 * word);
    memcpy(b + y, tmp, 2 * word);
  }
}

/* ------------------------------------------------------------------ f32 radix-8 core */
static const float kSqrtHalf = 0.70710678118f;   /* arm_cfft_radix8_f32.c:68 */

/* One DIF radix-8 butterfly over z[0..7] (z[m] = element i1 + m*n2).  w: 7 twiddles
 * (w[m-1] = table[m*j*mod]) or NULL for the j == 0 group. */
static void oracle_r8(cpx z[8], const float *tw, uint32_t idx) {
  float a_p[4], a_m[4], b_p[4], b_m[4];      /* sums / differences of pairs (k, k+4) */
  for (int k = 0; k < 4; ++k) {
    a_p[k] = z[k].re + z[k + 4].re;  a_m[k] = z[k].re - z[k + 4].re;
    b_p[k] = z[k].im + z[k + 4].im;  b_m[k] = z[k].im - z[k + 4].im;
  }
  /* even half */
  float e0 = a_p[0] - a_p[2], e1 = a_p[0] + a_p[2], e2 = a_p[1] - a_p[3], e3 = a_p[1] + a_p[3];
  float f0 = b_p[0] - b_p[2], f1 = b_p[0] + b_p[2], f2 = b_p[1] - b_p[3], f3 = b_p[1] + b_p[3];
  cpx out[8];
  out[0].re = e1 + e3;  out[0].im = f1 + f3;
  cpx o4 = {e1 - e3, f1 - f3};
  cpx o2 = {e0 + f2, f0 - e2};
  cpx o6 = {e0 - f2, f0 + e2};
  /* odd half */
  float g0 = (a_m[1] - a_m[3]) * kSqrtHalf, g1 = (a_m[1] + a_m[3]) * kSqrtHalf;
  float h0 = (b_m[1] - b_m[3]) * kSqrtHalf, h1 = (b_m[1] + b_m[3]) * kSqrtHalf;
  float p0 = a_m[0] - g0, p1 = a_m[0] + g0, q0 = a_m[2] - g1, q1 = a_m[2] + g1;
  float u0 = b_m[0] - h0, u1 = b_m[0] + h0, v0 = b_m[2] - h1, v1 = b_m[2] + h1;
  cpx o1 = {p1 + v1, u1 - q1};
  cpx o7 = {p1 - v1, u1 + q1};
  cpx o5 = {p0 + v0, u0 - q0};
  cpx o3 = {p0 - v0, u0 + q0};
  if (tw) {
    o1 = twmul(o1.re, o1.im, tw + 2 * (1 * idx));
    o2 = twmul(o2.re, o2.im, tw + 2 * (2 * idx));
    o3 = twmul(o3.re, o3.im, tw + 2 * (3 * idx));
    o4 = twmul(o4.re, o4.im, tw + 2 * (4 * idx));
    o5 = twmul(o5.re, o5.im, tw + 2 * (5 * idx));
    o6 = twmul(o6.re, o6.im, tw + 2 * (6 * idx));
    o7 = twmul(o7.re, o7.im, tw + 2 * (7 * idx));
  }
  out[1] = o1; out[2] = o2; out[3] = o3; out[4] = o4; out[5] = o5; out[6] = o6; out[7] = o7;
  for (int m = 0; m < 8; ++m) z[m] = out[m];
}

static void oracle_radix8(cpx *x, uint32_t len, const float *tw, uint32_t mod) {
  for (uint32_t span = len; span >= 8; span >>= 3, mod <<= 3) {
    const uint32_t step = span >> 3;
    for (uint32_t j = 0; j < step; ++j)
      for (uint32_t base = j; base < len; base += span) {
        cpx z[8];
        for (int m = 0; m < 8; ++m) z[m] = x[base + m * step];
        oracle_r8(z, j ? tw : NULL, j * mod);
        for (int m = 0; m < 8; ++m) x[base + m * step] = z[m];
      }
  }
}

static void oracle_first_radix2(cpx *x, uint32_t n, const float *tw) {
  const uint32_t h = n / 2, q = n / 4;
  for (uint32_t k = 0; k < q; ++k) {
    const float *w = tw + 2 * k;
    cpx a = x[k], b = x[k + h], c = x[k + q], d = x[k + h + q];
    x[k].re = a.re + b.re;  x[k].im = a.im + b.im;
    x[k + q].re = c.re + d.re;  x[k + q].im = c.im + d.im;
    x[k + h] = twmul(a.re - b.re, a.im - b.im, w);
    float dr = d.re - c.re, di = d.im - c.im;   /* "vertical symmetry": W^(k+N/4) */
    x[k + h + q].re = dr * w[1] - di * w[0];
    x[k + h + q].im = di * w[1] + dr * w[0];
  }
}

static void oracle_first_radix4(cpx *x, uint32_t n, const float *tw) {
  const uint32_t q = n / 4, e = n / 8;
  /* rows k = 0 .. N/8 (k = 0 untwiddled) */
  for (uint32_t k = 0; k <= e; ++k) {
    cpx A = x[k], B = x[k + q], Cc = x[k + 2 * q], D = x[k + 3 * q];
    float sr = A.re + Cc.re, dr = A.re - Cc.re, si = A.im + Cc.im, di = A.im - Cc.im;
    cpx r2 = {dr + B.im - D.im, di - B.re + D.re};
    cpx r3 = {sr - B.re - D.re, si - B.im - D.im};
    cpx r4 = {dr - B.im + D.im, di + B.re - D.re};
    x[k].re = sr + B.re + D.re;  x[k].im = si + B.im + D.im;
    if (k == 0) { x[q] = r2; x[2 * q] = r3; x[3 * q] = r4; continue; }
    x[k + q] = twmul(r2.re, r2.im, tw + 2 * k);
    x[k + 2 * q] = twmul(r3.re, r3.im, tw + 4 * k);
    x[k + 3 * q] = twmul(r4.re, r4.im, tw + 6 * k);
  }
  /* mirrored rows kb = N/4 - i, i = 1 .. N/8-1, reusing the twiddles of row i */
  for (uint32_t i = 1; i < e; ++i) {
    const uint32_t kb = q - i;
    cpx A = x[kb], B = x[kb + q], Cc = x[kb + 2 * q], D = x[kb + 3 * q];
    float sr = A.re + Cc.re, dr = A.re - Cc.re, si = A.im + Cc.im, di = A.im - Cc.im;
    float c2a = B.im - D.im + dr, c2b = A.im - Cc.im - B.re + D.re;
    float c3a = sr - B.re - D.re, c3b = si - B.im - D.im;
    float c4a = B.im - D.im - dr, c4b = D.re - B.re - di;
    x[kb].re = sr + B.re + D.re;  x[kb].im = si + B.im + D.im;
    const float *w2 = tw + 2 * i, *w3 = tw + 4 * i, *w4 = tw + 6 * i;
    x[kb + q].im = c2b * w2[1] - c2a * w2[0];
    x[kb + q].re = c2a * w2[1] + c2b * w2[0];
    x[kb + 2 * q].im = -c3b * w3[0] - c3a * w3[1];
    x[kb + 2 * q].re = c3b * w3[1] - c3a * w3[0];
    x[kb + 3 * q].im = c4b * w4[1] - c4a * w4[0];
    x[kb + 3 * q].re = c4a * w4[1] + c4b * w4[0];
  }
}

void oracle_arm_cfft_f32(const arm_cfft_instance_f32 *S, float *p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  const uint32_t n = S->fftLen;
  cpx *x = (cpx *)p1;
  if (ifftFlag == 1u)
    for (uint32_t i = 0; i < n; ++i) x[i].im = -x[i].im;
  switch (n) {
    case 16: case 128: case 1024:
      oracle_first_radix2(x, n, S->pTwiddle);
      oracle_radix8(x, n / 2, S->pTwiddle, 2);
      oracle_radix8(x + n / 2, n / 2, S->pTwiddle, 2);
      break;
    case 32: case 256: case 2048:
      oracle_first_radix4(x, n, S->pTwiddle);
      for (int c = 0; c < 4; ++c) oracle_radix8(x + c * (n / 4), n / 4, S->pTwiddle, 4);
      break;
    case 64: case 512: case 4096:
      oracle_radix8(x, n, S->pTwiddle, 1);
      break;
    default:
      break;
  }
  if (bitReverseFlag) swap_pairs_words(p1, sizeof(float), S->pBitRevTable, S->bitRevLength);
  if (ifftFlag == 1u) {
    const float s = 1.0f / (float)n;
    for (uint32_t i = 0; i < n; ++i) { x[i].re = x[i].re * s; x[i].im = -x[i].im * s; }
  }
}

/* ------------------------------------------------------------------ q31 radix-4 core */
typedef struct { int32_t re, im; } icpx;

/* one radix-4 butterfly; stage: 0 first (>>4 in, <<1 out), 1 middle (>>2, >>1), 2 last */
static void q31_r4(icpx *a, icpx *b, icpx *c, icpx *d, const int32_t *tw, uint32_t ia, int stage, int inv) {
  const int sh = stage == 0 ? 4 : 0;
  const int32_t xa = a->re >> sh, ya = a->im >> sh, xb = b->re >> sh, yb = b->im >> sh;
  const int32_t xc = c->re >> sh, yc = c->im >> sh, xd = d->re >> sh, yd = d->im >> sh;
  if (stage == 2) {
    icpx A = {wadd(wadd(xa, xb), wadd(xc, xd)), wadd(wadd(ya, yb), wadd(yc, yd))};
    icpx B = {wsub(wadd(xa, xc), wadd(xb, xd)), wsub(wadd(ya, yc), wadd(yb, yd))};
    icpx P = {wsub(wadd(xa, yb), wadd(xc, yd)), wsub(wadd(ya, xd), wadd(xb, yc))};   /* a - jb - c + jd */
    icpx M = {wsub(wadd(xa, yd), wadd(xc, yb)), wsub(wadd(ya, xb), wadd(yc, xd))};   /* a + jb - c - jd */
    *a = A; *b = B;
    *c = inv ? M : P;
    *d = inv ? P : M;
    return;
  }
  const int32_t sP = wadd(xa, xc), sM = wsub(xa, xc), tP = wadd(ya, yc), tM = wsub(ya, yc);
  const int32_t uP = wadd(xb, xd), uM = wsub(xb, xd), vP = wadd(yb, yd), vM = wsub(yb, yd);
  int32_t A_re = wadd(sP, uP), A_im = wadd(tP, vP);
  const int32_t e_re = wsub(sP, uP), e_im = wsub(tP, vP);           /* a - b + c - d */
  /* fwd: a - jb - c + jd -> (sM + vM, tM - uM); inv: the conjugate rotation */
  const int32_t f_re = inv ? wsub(sM, vM) : wadd(sM, vM), f_im = inv ? wadd(tM, uM) : wsub(tM, uM);
  const int32_t g_re = inv ? wadd(sM, vM) : wsub(sM, vM), g_im = inv ? wsub(tM, uM) : wadd(tM, uM);
  const int32_t *w1 = tw + 2 * ia, *w2 = tw + 4 * ia, *w3 = tw + 6 * ia;
  int32_t out[6];
  const int32_t *src[3][2] = {{&e_re, &e_im}, {&f_re, &f_im}, {&g_re, &g_im}};
  const int32_t *ws[3] = {w2, w1, w3};
  for (int o = 0; o < 3; ++o) {
    const int32_t r = *src[o][0], s = *src[o][1], co = ws[o][0], si = ws[o][1];
    int32_t re = inv ? wsub(hi32(r, co), hi32(s, si)) : wadd(hi32(r, co), hi32(s, si));
    int32_t im = inv ? wadd(hi32(s, co), hi32(r, si)) : wsub(hi32(s, co), hi32(r, si));
    if (stage == 0) { re = wshl1(re); im = wshl1(im); } else { re >>= 1; im >>= 1; }
    out[2 * o] = re; out[2 * o + 1] = im;
  }
  if (stage == 1) { A_re >>= 2; A_im >>= 2; }
  a->re = A_re; a->im = A_im;
  b->re = out[0]; b->im = out[1];      /* (a-b+c-d)*W^2n lands on i1 */
  c->re = out[2]; c->im = out[3];
  d->re = out[4]; d->im = out[5];
}

static void q31_radix4(icpx *x, uint32_t len, const int32_t *tw, uint32_t mod, int inv) {
  int stage = 0;
  for (uint32_t span = len; span >= 4; span >>= 2, mod <<= 2) {
    const uint32_t step = span >> 2;
    const int kind = step == 1 ? 2 : stage;
    for (uint32_t j = 0; j < step; ++j)
      for (uint32_t base = j; base < len; base += span)
        q31_r4(&x[base], &x[base + step], &x[base + 2 * step], &x[base + 3 * step], tw, j * mod, kind, inv);
    stage = 1;
  }
}

void oracle_arm_cfft_q31(const arm_cfft_instance_q31 *S, int32_t *p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  const uint32_t n = S->fftLen;
  const int inv = ifftFlag == 1u;
  icpx *x = (icpx *)p1;
  switch (n) {
    case 16: case 64: case 256: case 1024: case 4096:
      q31_radix4(x, n, S->pTwiddle, 1, inv);
      break;
    case 32: case 128: case 512: case 2048: {
      const uint32_t h = n / 2;
      for (uint32_t i = 0; i < h; ++i) {
        const int32_t co = S->pTwiddle[2 * i], si = S->pTwiddle[2 * i + 1];
        const int32_t ar = x[i].re >> 2, ai = x[i].im >> 2, br = x[i + h].re >> 2, bi = x[i + h].im >> 2;
        const int32_t dx = wsub(ar, br), dy = wsub(ai, bi);
        x[i].re = wadd(ar, br);
        x[i].im = wadd(ai, bi);
        /* none.h:184-196 rounding multiplies */
        int64_t acc_re = ((int64_t)dx * co + 0x80000000LL) >> 32;
        int64_t acc_im = ((int64_t)dy * co + 0x80000000LL) >> 32;
        uint64_t t_re = ((uint64_t)acc_re << 32) + (uint64_t)(inv ? -((int64_t)dy * si) : ((int64_t)dy * si)) + 0x80000000ULL;
        uint64_t t_im = ((uint64_t)acc_im << 32) + (uint64_t)(inv ? ((int64_t)dx * si) : -((int64_t)dx * si)) + 0x80000000ULL;
        x[i + h].re = wshl1((int32_t)(t_re >> 32));
        x[i + h].im = wshl1((int32_t)(t_im >> 32));
      }
      q31_radix4(x, h, S->pTwiddle, 2, inv);
      q31_radix4(x + h, h, S->pTwiddle, 2, inv);
      for (uint32_t i = 0; i < 2 * n; ++i) p1[i] = wshl1(p1[i]);
      break;
    }
    default:
      break;
  }
  if (bitReverseFlag) swap_pairs_words(p1, sizeof(int32_t), S->pBitRevTable, S->bitRevLength);
}

/* ------------------------------------------------------------------ q15 radix-4 core */
/* (c*x + s*y) >> 16 as q15 with int32 wrap of the sum */
static int32_t q15dot(int32_t c, int32_t x, int32_t s, int32_t y, int sub) {
  uint32_t u = (uint32_t)(c * x), v = (uint32_t)(s * y);
  return tr16((int32_t)(sub ? u - v : u + v) >> 16);
}

static void q15_r4(icpx *a, icpx *b, icpx *c, icpx *d, const int16_t *tw, uint32_t ia, int stage, int inv) {
  const int sh = stage == 0 ? 2 : 0;
  const int32_t ar = a->re >> sh, ai = a->im >> sh, br = b->re >> sh, bi = b->im >> sh;
  const int32_t cr = c->re >> sh, ci = c->im >> sh, dr = d->re >> sh, di = d->im >> sh;
  const int32_t pr = sat16(ar + cr), pi = sat16(ai + ci), mr = sat16(ar - cr), mi = sat16(ai - ci);
  const int32_t qr = sat16(br + dr), qi = sat16(bi + di), nr = sat16(br - dr), ni = sat16(bi - di);
  icpx A, B, Cc, D;
  if (stage == 1) { A.re = tr16(((pr >> 1) + (qr >> 1)) >> 1); A.im = tr16(((pi >> 1) + (qi >> 1)) >> 1); }
  else            { A.re = tr16((pr >> 1) + (qr >> 1));        A.im = tr16((pi >> 1) + (qi >> 1)); }
  int32_t er, ei;
  if (stage == 0) { er = sat16(pr - qr); ei = sat16(pi - qi); }
  else            { er = tr16((pr >> 1) - (qr >> 1)); ei = tr16((pi >> 1) - (qi >> 1)); }
  /* the two odd outputs: fwd (m - j n), (m + j n); inv swapped */
  int32_t fr, fi, gr, gi;   /* f -> position 2 (xb'), g -> position 3 (xd') */
  if (stage == 0) {
    int32_t sr_ = sat16(mr + ni), si_ = sat16(mi - nr), rr_ = sat16(mr - ni), ri_ = sat16(mi + nr);
    if (!inv) { fr = sr_; fi = si_; gr = rr_; gi = ri_; } else { fr = rr_; fi = ri_; gr = sr_; gi = si_; }
  } else {
    int32_t sr_ = tr16((mr >> 1) + (ni >> 1)), si_ = tr16((mi >> 1) - (nr >> 1));
    int32_t rr_ = tr16((mr >> 1) - (ni >> 1)), ri_ = tr16((mi >> 1) + (nr >> 1));
    if (!inv) { fr = sr_; fi = si_; gr = rr_; gi = ri_; } else { fr = rr_; fi = ri_; gr = sr_; gi = si_; }
  }
  if (stage == 2) {
    B.re = er; B.im = ei;
    Cc.re = fr; Cc.im = fi;
    D.re = gr; D.im = gi;
  } else {
    const int16_t *w1 = tw + 2 * ia, *w2 = tw + 4 * ia, *w3 = tw + 6 * ia;
    if (!inv) {
      B.re = q15dot(w2[0], er, w2[1], ei, 0);  B.im = q15dot(w2[0], ei, w2[1], er, 1);
      Cc.re = q15dot(w1[0], fr, w1[1], fi, 0); Cc.im = q15dot(w1[0], fi, w1[1], fr, 1);
      D.re = q15dot(w3[0], gr, w3[1], gi, 0);  D.im = q15dot(w3[0], gi, w3[1], gr, 1);
    } else {
      B.re = q15dot(w2[0], er, w2[1], ei, 1);  B.im = q15dot(w2[1], er, w2[0], ei, 0);
      Cc.re = q15dot(w1[0], fr, w1[1], fi, 1); Cc.im = q15dot(w1[1], fr, w1[0], fi, 0);
      D.re = q15dot(w3[0], gr, w3[1], gi, 1);  D.im = q15dot(w3[1], gr, w3[0], gi, 0);
    }
  }
  *a = A; *b = B; *c = Cc; *d = D;
}

static void q15_radix4(icpx *x, uint32_t len, const int16_t *tw, uint32_t mod, int inv) {
  int stage = 0;
  for (uint32_t span = len; span >= 4; span >>= 2, mod <<= 2) {
    const uint32_t step = span >> 2;
    const int kind = step == 1 ? 2 : stage;
    for (uint32_t j = 0; j < step; ++j)
      for (uint32_t base = j; base < len; base += span)
        q15_r4(&x[base], &x[base + step], &x[base + 2 * step], &x[base + 3 * step], tw, j * mod, kind, inv);
    stage = 1;
  }
}

void oracle_arm_cfft_q15(const arm_cfft_instance_q15 *S, int16_t *p1, uint8_t ifftFlag, uint8_t bitReverseFlag) {
  const uint32_t n = S->fftLen;
  const int inv = ifftFlag == 1u;
  int known = 1;
  switch (n) {
    case 16: case 32: case 64: case 128: case 256: case 512: case 1024: case 2048: case 4096: break;
    default: known = 0;
  }
  if (known) {
    /* widen to int32 working words, run the int16-semantics butterflies, narrow back */
    static __thread icpx w[4096];
    for (uint32_t i = 0; i < n; ++i) { w[i].re = p1[2 * i]; w[i].im = p1[2 * i + 1]; }
    if (n == 32 || n == 128 || n == 512 || n == 2048) {
      const uint32_t h = n / 2;
      for (uint32_t i = 0; i < h; ++i) {
        const int32_t co = S->pTwiddle[2 * i], si = S->pTwiddle[2 * i + 1];
        const int32_t ar = w[i].re >> 1, ai = w[i].im >> 1, br = w[i + h].re >> 1, bi = w[i + h].im >> 1;
        const int32_t dx = tr16(ar - br), dy = tr16(ai - bi);
        w[i].re = tr16((ar + br) >> 1);
        w[i].im = tr16((bi + ai) >> 1);
        const int32_t xc = tr16((dx * co) >> 16), ys = tr16((dy * si) >> 16);
        const int32_t yc = tr16((dy * co) >> 16), xs = tr16((dx * si) >> 16);
        w[i + h].re = tr16(inv ? xc - ys : xc + ys);
        w[i + h].im = tr16(inv ? yc + xs : yc - xs);
      }
      q15_radix4(w, h, S->pTwiddle, 2, inv);
      q15_radix4(w + h, h, S->pTwiddle, 2, inv);
      for (uint32_t i = 0; i < n; ++i) { w[i].re = tr16(wshl1(w[i].re)); w[i].im = tr16(wshl1(w[i].im)); }
    } else {
      q15_radix4(w, n, S->pTwiddle, 1, inv);
    }
    for (uint32_t i = 0; i < n; ++i) { p1[2 * i] = (int16_t)w[i].re; p1[2 * i + 1] = (int16_t)w[i].im; }
  }
  if (bitReverseFlag) swap_pairs_words(p1, sizeof(int16_t), S->pBitRevTable, S->bitRevLength);
}

/* ------------------------------------------------------------------ RFFT fast f32 */
void oracle_arm_rfft_fast_f32(const arm_rfft_fast_instance_f32 *S, float *p, float *pOut, uint8_t ifftFlag) {
  const uint32_t h = S->Sint.fftLen;
  const float *t = S->pTwiddleRFFT;
  cpx *X = (cpx *)p, *Y = (cpx *)pOut;
  if (ifftFlag) {
    Y[0].re = 0.5f * (X[0].re + X[0].im);
    Y[0].im = 0.5f * (X[0].re - X[0].im);
    for (uint32_t i = 1; i < h; ++i) {
      const cpx A = X[i], B = X[h - i];
      const float d = A.re - B.re, s = A.im + B.im;
      Y[i].re = 0.5f * (A.re + B.re - t[2 * i] * d - t[2 * i + 1] * s);
      Y[i].im = 0.5f * (A.im - B.im + t[2 * i + 1] * d - t[2 * i] * s);
    }
    oracle_arm_cfft_f32(&S->Sint, pOut, ifftFlag, 1);
  } else {
    oracle_arm_cfft_f32(&S->Sint, p, ifftFlag, 1);
    const float s0 = X[0].re + X[0].re, s1 = X[0].im + X[0].im;
    Y[0].re = 0.5f * (s0 + s1);
    Y[0].im = 0.5f * (s0 - s1);
    for (uint32_t i = 1; i < h; ++i) {
      const cpx A = X[i], B = X[h - i];
      const float d = B.re - A.re, s = B.im + A.im;
      Y[i].re = 0.5f * (A.re + B.re + t[2 * i] * d + t[2 * i + 1] * s);
      Y[i].im = 0.5f * (A.im - B.im + t[2 * i + 1] * d - t[2 * i] * s);
    }
  }
}

/* ------------------------------------------------------------------ RFFT q31 / q15
 * arm_rfft_q31.c:148-183 (dispatch), arm_split_rfft_q31 :256-341, arm_split_rifft_q31
 * :397-476 (scalar branches); arm_rfft_q15.c (dispatch), arm_split_rfft_q15 / _rifft_q15
 * (!ARM_MATH_DSP branches); arm_shift_q31.c / arm_shift_q15.c (left shift by 1 with
 * saturation).  L = N/2 complex bins of the inner CFFT; table stride c = 2*modifier*k.
 * Forward: pSrc is transformed in place, pDst receives the full 2N-word spectrum (bins
 * L+1 .. N-1 mirrored as conjugates).  Inverse: pSrc words 0 .. N+1 are read. */
static int32_t rnd_mul(int32_t x, int32_t y) { return (int32_t)(((int64_t)x * y + 0x80000000LL) >> 32); }
static int32_t rnd_acc(int32_t a, int32_t x, int32_t y) {
  return (int32_t)((int64_t)(((uint64_t)(int64_t)a << 32) + (uint64_t)((int64_t)x * y) + 0x80000000ULL) >> 32);
}
static int32_t rnd_sub(int32_t a, int32_t x, int32_t y) {
  return (int32_t)((int64_t)(((uint64_t)(int64_t)a << 32) - (uint64_t)((int64_t)x * y) + 0x80000000ULL) >> 32);
}
static int32_t sat_shl1_q31(int32_t v) {
  const int32_t o = (int32_t)((uint32_t)v << 1);
  return (o >> 1) != v ? (int32_t)(0x7FFFFFFF ^ (v >> 31)) : o;
}

void oracle_arm_rfft_q31(const arm_rfft_instance_q31 *S, int32_t *pSrc, int32_t *pDst) {
  const uint32_t n = S->fftLenReal, L = n / 2, mod = S->twidCoefRModifier;
  const int32_t *A = S->pTwiddleAReal, *B = S->pTwiddleBReal;
  if (S->ifftFlagR == 1) {
    for (uint32_t k = 0; k < L; ++k) {
      const uint32_t c = 2 * mod * k;
      const int32_t a1 = A[c], a2 = A[c + 1], b1 = B[c];
      const int32_t xr = pSrc[2 * k], xi = pSrc[2 * k + 1], yr = pSrc[2 * (L - k)], yi = pSrc[2 * (L - k) + 1];
      int32_t re = rnd_mul(xr, a1), im = rnd_mul(xr, (int32_t)(0u - (uint32_t)a2));
      re = rnd_acc(re, xi, a2); im = rnd_acc(im, xi, a1);
      re = rnd_acc(re, yi, a2); im = rnd_sub(im, yi, b1);
      re = rnd_acc(re, yr, b1); im = rnd_acc(im, yr, a2);
      pDst[2 * k] = re; pDst[2 * k + 1] = im;
    }
    oracle_arm_cfft_q31(S->pCfft, pDst, 1, S->bitReverseFlagR);
    for (uint32_t i = 0; i < n; ++i) pDst[i] = sat_shl1_q31(pDst[i]);
  } else {
    oracle_arm_cfft_q31(S->pCfft, pSrc, S->ifftFlagR, S->bitReverseFlagR);
    for (uint32_t k = 1; k < L; ++k) {
      const uint32_t c = 2 * mod * k;
      const int32_t a1 = A[c], a2 = A[c + 1], b1 = B[c];
      const int32_t xr = pSrc[2 * k], xi = pSrc[2 * k + 1], yr = pSrc[2 * (L - k)], yi = pSrc[2 * (L - k) + 1];
      int32_t re = rnd_mul(xr, a1), im = rnd_mul(xr, a2);
      re = rnd_sub(re, xi, a2); im = rnd_acc(im, xi, a1);
      re = rnd_sub(re, yi, a2); im = rnd_sub(im, yi, b1);
      re = rnd_acc(re, yr, b1); im = rnd_sub(im, yr, a2);
      pDst[2 * k] = re; pDst[2 * k + 1] = im;
      pDst[2 * n - 2 * k] = re; pDst[2 * n - 2 * k + 1] = (int32_t)(0u - (uint32_t)im);
    }
    pDst[n] = wsub(pSrc[0], pSrc[1]) >> 1; pDst[n + 1] = 0;
    pDst[0] = wadd(pSrc[0], pSrc[1]) >> 1; pDst[1] = 0;
  }
}

void oracle_arm_rfft_q15(const arm_rfft_instance_q15 *S, int16_t *pSrc, int16_t *pDst) {
  const uint32_t n = S->fftLenReal, L = n / 2, mod = S->twidCoefRModifier;
  const int16_t *A = S->pTwiddleAReal, *B = S->pTwiddleBReal;
  /* q15 x q15 products in int, sums wrap mod 2^32 (done in uint32_t), >> 16 arithmetic */
#define P(a, b) ((uint32_t)((int32_t)(a) * (int32_t)(b)))
  if (S->ifftFlagR == 1) {
    for (uint32_t k = 0; k < L; ++k) {
      const uint32_t c = 2 * mod * k;
      const int16_t xr = pSrc[2 * k], xi = pSrc[2 * k + 1], yr = pSrc[2 * (L - k)], yi = pSrc[2 * (L - k) + 1];
      const int32_t re = (int32_t)(P(yr, B[c]) - P(yi, B[c + 1]) + P(xr, A[c]) + P(xi, A[c + 1])) >> 16;
      const int32_t im = (int32_t)(P(xi, A[c]) - P(xr, A[c + 1]) - P(yr, B[c + 1]) - P(yi, B[c]));
      pDst[2 * k] = (int16_t)re; pDst[2 * k + 1] = (int16_t)(im >> 16);
    }
    oracle_arm_cfft_q15(S->pCfft, pDst, 1, S->bitReverseFlagR);
    for (uint32_t i = 0; i < n; ++i) pDst[i] = (int16_t)sat16((int32_t)pDst[i] * 2);   /* << 1 without UB */
  } else {
    oracle_arm_cfft_q15(S->pCfft, pSrc, S->ifftFlagR, S->bitReverseFlagR);
    for (uint32_t k = 1; k < L; ++k) {
      const uint32_t c = 2 * mod * k;
      const int16_t xr = pSrc[2 * k], xi = pSrc[2 * k + 1], yr = pSrc[2 * (L - k)], yi = pSrc[2 * (L - k) + 1];
      const int32_t re = (int32_t)(P(xr, A[c]) - P(xi, A[c + 1]) + P(yr, B[c]) + P(yi, B[c + 1])) >> 16;
      const int32_t im = (int32_t)(P(yr, B[c + 1]) - P(yi, B[c]) + P(xi, A[c]) + P(xr, A[c + 1])) >> 16;
      pDst[2 * k] = (int16_t)re; pDst[2 * k + 1] = (int16_t)im;
      pDst[2 * n - 2 * k] = (int16_t)re; pDst[2 * n - 2 * k + 1] = (int16_t)(-im);
    }
    pDst[n] = (int16_t)((pSrc[0] - pSrc[1]) >> 1); pDst[n + 1] = 0;
    pDst[0] = (int16_t)((pSrc[0] + pSrc[1]) >> 1); pDst[1] = 0;
  }
#undef P
}
