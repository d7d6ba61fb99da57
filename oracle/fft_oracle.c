/*
 * fft_oracle.c — CPU restatement of the FFT64 external product (tfhe-rs's own arithmetic).
 *
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h): used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker; never linked into the product.
 *
 * tfhe-rs (npm tfhe / node-tfhe 0.8.7 — packages/pnpm-lock.yaml:1988-1995 — absent from the mount)
 * runs keyswitch_programmable_bootstrap (ml/biometrics/notebooks/main.rs:71) over the native 2^64
 * torus with the external product computed by an f64 negacyclic FFT (concrete-fft: fold the N real
 * coefficients into N/2 complex, twist by zeta^j, zeta = e^{i pi/N}, cyclic DFT; BSK stored in the
 * Fourier domain).  The exact product it approximates is the reference's wrapping negacyclic
 * product (ml/extensions/rust/src/computations.rs:50-54,101-105); or_poly_mul_torus_schoolbook below
 * computes that exactly and tests bound the FFT's deviation from it.
 *
 * This file fixes ONE operation sequence (every +, -, *, fma, in order) so the gfx950 kernels in
 * tfhe_amd/csrc/pbs_fft.hip reproduce every double bit-for-bit:
 *   cmul(z, w)       re = fma(z.re, w.re, -(z.im * w.im)),  im = fma(z.re, w.im, z.im * w.re)
 *                    (inverse transforms use w = (w.re, -w.im))
 *   dft8             radix-2 decimation in frequency, 3 stages, natural order in and out; the
 *                    internal rotations by e^{+-i pi/4 j} are the explicit forms in w8() below, the
 *                    sqrt(1/2) of the odd half folded into the last stage's fmas (round 5, see dft8)
 *   3 passes         M = 512 = 8 x 8 x 8 over a 64 x 8 grid (the device's lane x register grid),
 *                    w = e^{2 pi i / M}, n = n0 + 8 n1 + 64 n2, k = k0 + 8 k1 + 64 k2:
 *                    A: lane L = n0 + 8 n1 transforms n2, then x[k0] *= w^{L k0} (k0 > 0; with the twist
 *                       merged, see N = 1024 / N = 2048 below, every k0 by the merged table)
 *                    B: lane n0 + 8 k0 transforms n1, then x[k1] *= w^{8 n0 k1}            (k1 > 0)
 *                    C: lane k1 + 8 k0 transforms n0 -> Z[k] in slot k2
 *                    so spectra are kept in DEVICE ORDER: slot d = L + 64 e holds frequency
 *                    k(d) = (L >> 3) + 8 (L & 7) + 64 e (the BSK is converted by the same routine)
 *   inverse          the passes reversed (decimation in time), device order in, natural order out:
 *                    C': lane k1 + 8 k0 transforms k2 -> n0, x[n0] *= conj(w^{8 n0 k1})   (n0 > 0)
 *                    B': lane n0 + 8 k0 transforms k1 -> n1, x[n1] *= conj(w^{k0 (n0 + 8 n1)}) (all; the
 *                        merged tables also carry the lane part of the untwist)
 *                    A': lane n0 + 8 n1 transforms k0 -> n2 = z[L + 64 n2]
 *   N = 2048         (P-FHEVM, preset 3) one 1024-point transform per polynomial on the device's 64-lane x
 *                    16-slot grid (round 4; the section "N = 2048, one wave per polynomial" below has the stages)
 *   N = 1024         the twist is merged into the passes (see fft_tab.twAm / twIm): z = v * zeta^{64 e} for
 *                    slot e > 0 before pass A, whose table is zeta^{L (1 + 4 e)} for all 8 slots; inverse pass
 *                    B' uses zeta^{(n0 + 8 n1)(4 k0 + 1)} and the output slot e > 0 gets conj(zeta^{64 e})
 *   MAC              re = fma(D.re, K.re, re); re = fma(-D.im, K.im, re);
 *                    im = fma(D.re, K.im, im); im = fma(D.im, K.re, im)   from (0, 0) (N = 1024: the first
 *                    term of each component chain is re = D.re * K.re, im = D.re * K.im instead), over
 *                    c = 0..k and, within c, the levels least significant first (l = L-1 .. 0:
 *                    the order the device produces digits, carry chain upward)
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "tfhe_oracle.h"

#define FFT_M 512

/* ---- twiddles: fixed series in plain double (no libm), |x| <= pi/4 ------------------------ */
static double fs_sin(double x) {
  double x2 = x * x, term = x, sum = 0.0;
  for (int i = 1; i <= 21; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static double fs_cos(double x) {
  double x2 = x * x, term = 1.0, sum = 0.0;
  for (int i = 0; i <= 20; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static void tw_octant(uint32_t t, uint32_t M, double* c, double* s) { /* t <= M/8 */
  const double x = (double)t * (6.28318530717958647692 / (double)M);
  *c = fs_cos(x);
  *s = fs_sin(x);
}
static void tw_quarter(uint32_t t, uint32_t M, double* c, double* s) { /* t <= M/4 */
  if (8 * t > M) {
    double cu, su;
    tw_octant(M / 4 - t, M, &cu, &su);
    *c = su;
    *s = cu;
  } else {
    tw_octant(t, M, c, s);
  }
}
void or_fft_twiddle(uint32_t t, uint32_t M, double* c, double* s) {
  t %= M;
  int neg = 0;
  if (2 * t > M) { t = M - t; neg = 1; }
  double cc, ss;
  if (4 * t > M) { /* theta = pi/2 + phi */
    double cu, su;
    tw_quarter(t - M / 4, M, &cu, &su);
    cc = -su;
    ss = cu;
  } else {
    tw_quarter(t, M, &cc, &ss);
  }
  *c = cc;
  *s = neg ? -ss : ss;
}

typedef struct fft_tab {
  or_c64 twist[FFT_M];  /* zeta^j, zeta = e^{i pi / N} */
  or_c64 twB[8][64];    /* w^{8 (L & 7) k1}, w = e^{2 pi i / M} */
  /* N = 1024 merged twist (pbs_fft.hip / fft512.h): zeta^j = zeta^L zeta^{64 e} for j = L + 64 e; the slot
   * constant zeta^{64 e} multiplies before pass A, zeta^L rides in pass A's table (all 8 slots), and the
   * inverse carries zeta^{n0 + 8 n1} in pass B''s table and conj(zeta^{64 e}) after pass A' */
  or_c64 twAm[8][64];   /* zeta^{L (1 + 4 e)} */
  or_c64 twIm[8][64];   /* zeta^{(n0 + 8 e)(4 k0 + 1)}, L = n0 + 8 k0 */
} fft_tab;

static fft_tab g_tab;
static int g_tab_ready = 0;

static const fft_tab* tab(void) {
#pragma omp critical(or_fft_tab)
  {
    if (!g_tab_ready) {
      for (uint32_t j = 0; j < FFT_M; j++) or_fft_twiddle(j, 2 * FFT_M * 2, &g_tab.twist[j].re, &g_tab.twist[j].im);
      for (uint32_t e = 0; e < 8; e++)
        for (uint32_t L = 0; L < 64; L++) {
          or_fft_twiddle((8 * (L & 7) * e) % FFT_M, FFT_M, &g_tab.twB[e][L].re, &g_tab.twB[e][L].im);
          or_fft_twiddle((L * (1 + 4 * e)) % (4 * FFT_M), 4 * FFT_M, &g_tab.twAm[e][L].re, &g_tab.twAm[e][L].im);
          or_fft_twiddle((((L & 7) + 8 * e) * (4 * (L >> 3) + 1)) % (4 * FFT_M), 4 * FFT_M, &g_tab.twIm[e][L].re,
                         &g_tab.twIm[e][L].im);
        }
      __atomic_store_n(&g_tab_ready, 1, __ATOMIC_RELEASE);
    }
  }
  return &g_tab;
}

/* ---- complex pieces ------------------------------------------------------------------------ */
static inline or_c64 cadd(or_c64 a, or_c64 b) { or_c64 r = {a.re + b.re, a.im + b.im}; return r; }
static inline or_c64 csub(or_c64 a, or_c64 b) { or_c64 r = {a.re - b.re, a.im - b.im}; return r; }
static inline or_c64 cmul(or_c64 z, double wr, double wi) {
  or_c64 r = {fma(z.re, wr, -(z.im * wi)), fma(z.re, wi, z.im * wr)};
  return r;
}

#define SQRT1_2 0.70710678118654752440
/* t * e^{+-i pi j / 4}, j in 1..3, explicit forms (exact negations) */
static inline or_c64 w8(or_c64 t, int j, int inv) {
  const double p = t.re, q = t.im;
  or_c64 r;
  if (!inv) {
    if (j == 1) { r.re = (p - q) * SQRT1_2; r.im = (p + q) * SQRT1_2; }
    else if (j == 2) { r.re = -q; r.im = p; }
    else { r.re = -((p + q) * SQRT1_2); r.im = (p - q) * SQRT1_2; }
  } else {
    if (j == 1) { r.re = (p + q) * SQRT1_2; r.im = (q - p) * SQRT1_2; }
    else if (j == 2) { r.re = q; r.im = -p; }
    else { r.re = (q - p) * SQRT1_2; r.im = -((p + q) * SQRT1_2); }
  }
  return r;
}

/* dft8 (round 5, = fft512.h FFT_DFT8_FMA): the even half as below; the odd half keeps the w8 forms unscaled
 * (u5 = w8^1 t1 / s, u7 = w8^3 t3 / s, s = sqrt(1/2)) and folds s into the last stage:
 *   z5' = u5 + u7, z7' = u5 - u7, z4 = t0 + r t2, z6 = t0 - r t2   (r = +i forward, -i inverse)
 *   X1 = fma(s, z5', z4), X5 = fma(-s, z5', z4), X3 = z6 + r (s z7'), X7 = z6 - r (s z7') as fmas */
static void dft8(or_c64 x[8], int inv) {
  or_c64 y[4], t[4];
  for (int j = 0; j < 4; j++) {
    y[j] = cadd(x[j], x[j + 4]);
    t[j] = csub(x[j], x[j + 4]);
  }
  double ar, ai, cr, ci, z4r, z4i, z6r, z6i;
  if (!inv) {
    ar = t[1].re - t[1].im; ai = t[1].re + t[1].im;
    cr = -(t[3].re + t[3].im); ci = t[3].re - t[3].im;
    z4r = t[0].re - t[2].im; z4i = t[0].im + t[2].re;
    z6r = t[0].re + t[2].im; z6i = t[0].im - t[2].re;
  } else {
    ar = t[1].re + t[1].im; ai = t[1].im - t[1].re;
    cr = t[3].im - t[3].re; ci = -(t[3].re + t[3].im);
    z4r = t[0].re + t[2].im; z4i = t[0].im - t[2].re;
    z6r = t[0].re - t[2].im; z6i = t[0].im + t[2].re;
  }
  const double z5r = ar + cr, z5i = ai + ci, z7r = ar - cr, z7i = ai - ci;
  const or_c64 e0 = cadd(y[0], y[2]), e2 = csub(y[0], y[2]), e1 = cadd(y[1], y[3]);
  const or_c64 e3 = w8(csub(y[1], y[3]), 2, inv);
  x[0] = cadd(e0, e1);
  x[4] = csub(e0, e1);
  x[2] = cadd(e2, e3);
  x[6] = csub(e2, e3);
  x[1].re = fma(SQRT1_2, z5r, z4r); x[1].im = fma(SQRT1_2, z5i, z4i);
  x[5].re = fma(-SQRT1_2, z5r, z4r); x[5].im = fma(-SQRT1_2, z5i, z4i);
  if (!inv) {
    x[3].re = fma(-SQRT1_2, z7i, z6r); x[3].im = fma(SQRT1_2, z7r, z6i);
    x[7].re = fma(SQRT1_2, z7i, z6r); x[7].im = fma(-SQRT1_2, z7r, z6i);
  } else {
    x[3].re = fma(SQRT1_2, z7i, z6r); x[3].im = fma(-SQRT1_2, z7r, z6i);
    x[7].re = fma(-SQRT1_2, z7i, z6r); x[7].im = fma(SQRT1_2, z7r, z6i);
  }
}

/* the round-1..4 dft8 (56 f64 operations), kept for reference; unused */
__attribute__((unused)) static void dft8_r4(or_c64 x[8], int inv) {
  or_c64 y[8], z[8], u[8];
  for (int j = 0; j < 4; j++) {
    y[j] = cadd(x[j], x[j + 4]);
    const or_c64 t = csub(x[j], x[j + 4]);
    y[j + 4] = j ? w8(t, j, inv) : t;
  }
  for (int h = 0; h < 8; h += 4)
    for (int j = 0; j < 2; j++) {
      z[h + j] = cadd(y[h + j], y[h + j + 2]);
      const or_c64 t = csub(y[h + j], y[h + j + 2]);
      z[h + j + 2] = j ? w8(t, 2, inv) : t;
    }
  for (int g = 0; g < 8; g += 2) {
    u[g] = cadd(z[g], z[g + 1]);
    u[g + 1] = csub(z[g], z[g + 1]);
  }
  static const int brv3[8] = {0, 4, 2, 6, 1, 5, 3, 7};
  for (int k = 0; k < 8; k++) x[k] = u[brv3[k]];
}

/* FFT_TDFT8 (default 0, = fft512.h): measured slower on the device, kept for its A/B build (make FFT_TDFT8=1 ...) */
#ifndef FFT_TDFT8
#define FFT_TDFT8 0
#endif
/* the N = 1024 forward's slot twist + pass A's DFT8 as one twisted DFT8 (round 5, = fft512.h twist_dft8_fwd): x(X) =
 * sum_e x_e X^e at the roots X_k = e^{i pi (1 + 4k)/16} of X^8 = i by a radix-2 split (X^8 - i = (X^4 - w)(X^4 + w), ...),
 * 12 butterflies a +- e^{i th} b each with b through the tangent / cotangent form and cos / sin th in the output fmas */
#define TD_T8 0.41421356237309504880   /* tan(pi/8) */
#define TD_C8 0.92387953251128675613   /* cos(pi/8) */
#define TD_T16 0.19891236737965800691  /* tan(pi/16) */
#define TD_C16 0.98078528040323044913  /* cos(pi/16) */
#define TD_T316 0.66817863791929891999 /* tan(3pi/16) */
#define TD_C316 0.83146961230254523708 /* cos(3pi/16) */
static void tbfly(or_c64* a, or_c64* b, double t, double sc, int cot) {
  double ur, ui;
  if (!cot) { ur = fma(-t, b->im, b->re); ui = fma(t, b->re, b->im); }
  else { ur = fma(t, b->re, -b->im); ui = fma(t, b->im, b->re); }
  const or_c64 p = *a;
  a->re = fma(sc, ur, p.re); a->im = fma(sc, ui, p.im);
  b->re = fma(-sc, ur, p.re); b->im = fma(-sc, ui, p.im);
}
__attribute__((unused)) static void tdft8_fwd(or_c64 x[8]) {
  for (int e = 0; e < 4; e++) {
    const double ur = x[e + 4].re - x[e + 4].im, ui = x[e + 4].im + x[e + 4].re;
    const or_c64 p = x[e];
    x[e].re = fma(SQRT1_2, ur, p.re); x[e].im = fma(SQRT1_2, ui, p.im);
    x[e + 4].re = fma(-SQRT1_2, ur, p.re); x[e + 4].im = fma(-SQRT1_2, ui, p.im);
  }
  tbfly(&x[0], &x[2], TD_T8, TD_C8, 0);
  tbfly(&x[1], &x[3], TD_T8, TD_C8, 0);
  tbfly(&x[4], &x[6], -TD_T8, TD_C8, 1);
  tbfly(&x[5], &x[7], -TD_T8, TD_C8, 1);
  tbfly(&x[0], &x[1], TD_T16, TD_C16, 0);
  tbfly(&x[2], &x[3], -TD_T16, TD_C16, 1);
  tbfly(&x[4], &x[5], TD_T316, TD_C316, 1);
  tbfly(&x[6], &x[7], -TD_T316, -TD_C316, 0);
  const or_c64 y[8] = {x[0], x[4], x[2], x[6], x[1], x[5], x[3], x[7]}; /* positions -> X_k */
  memcpy(x, y, sizeof(y));
}

/* forward 3-pass DFT: natural order in, device order out; pass A multiplies slots merged ? 0..7 : 1..7 by twa
 * (the twist-merged tables multiply every slot); twin: the input is not yet twisted, pass A's DFT8 is tdft8_fwd */
static void dft512_fwd_tab(const or_c64* in, or_c64* out, const or_c64 (*twa)[64], int merged, int twin) {
  const fft_tab* T = tab();
  or_c64 A[64][8], Bv[64][8], x[8];
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = in[L + 64 * e];
    if (twin) tdft8_fwd(x);
    else dft8(x, 0);
    for (int e = merged ? 0 : 1; e < 8; e++) x[e] = cmul(x[e], twa[e][L].re, twa[e][L].im);
    memcpy(A[L], x, sizeof(x));
  }
  for (int L = 0; L < 64; L++) { /* lane n0 + 8 k0 */
    for (int e = 0; e < 8; e++) x[e] = A[(L & 7) + 8 * e][L >> 3];
    dft8(x, 0);
    for (int e = 1; e < 8; e++) x[e] = cmul(x[e], T->twB[e][L].re, T->twB[e][L].im);
    memcpy(Bv[L], x, sizeof(x));
  }
  for (int L = 0; L < 64; L++) { /* lane k1 + 8 k0 */
    for (int e = 0; e < 8; e++) x[e] = Bv[e + 8 * (L >> 3)][L & 7];
    dft8(x, 0);
    for (int e = 0; e < 8; e++) out[L + 64 * e] = x[e];
  }
}



/* inverse 3-pass DFT (no 1/M): device order in, natural order out (merged: pass B' uses twIm) */
static void dft512_inv_tab(const or_c64* in, or_c64* out, const or_c64 (*twi)[64]) {
  const fft_tab* T = tab();
  or_c64 S1[64][8], S2[64][8], x[8];
  for (int L = 0; L < 64; L++) { /* lane k1 + 8 k0: k2 -> n0 */
    for (int e = 0; e < 8; e++) x[e] = in[L + 64 * e];
    dft8(x, 1);
    for (int e = 1; e < 8; e++) x[e] = cmul(x[e], T->twB[e][L].re, -T->twB[e][L].im);
    memcpy(S1[L], x, sizeof(x));
  }
  for (int L = 0; L < 64; L++) { /* lane n0 + 8 k0: k1 -> n1 */
    for (int e = 0; e < 8; e++) x[e] = S1[e + 8 * (L >> 3)][L & 7];
    dft8(x, 1);
    for (int e = 0; e < 8; e++) x[e] = cmul(x[e], twi[e][L].re, -twi[e][L].im);
    memcpy(S2[L], x, sizeof(x));
  }
  for (int L = 0; L < 64; L++) { /* lane n0 + 8 n1: k0 -> n2 */
    for (int e = 0; e < 8; e++) x[e] = S2[(L & 7) + 8 * e][L >> 3];
    dft8(x, 1);
    for (int e = 0; e < 8; e++) out[L + 64 * e] = x[e];
  }
}



/* ---- N = 2048, one wave per polynomial (round 4, pbs_fft2k.hip / fft1k.h) ------------------------
 * M = 1024 = 16 x 4 x 16 over the device's 64-lane x 16-slot grid, natural input n = L + 64 e:
 *   z_n = (a_n + i a_{n+1024}) zeta^n, zeta = e^{2 pi i / 4096}: the slot part zeta^{64 e} multiplies slot e > 0,
 *   the lane part zeta^L rides in pass A's table
 *   A  lane L: DFT16 over e -> k1, then x[k1] *= ta[k1][L] = zeta^{L (1 + 4 k1)}        (every k1)
 *   X  register exchange (v_permlane32_swap / v_permlane16_swap): slot bit 3 <-> lane bit 5, slot bit 2 <->
 *      lane bit 4, so lane L' = l0 + 16 (k1 >> 2) holds slot s' = (k1 & 3) + 4 l1   (L = l0 + 16 l1)
 *   B  per g = k1 & 3: radix-4 over l1 (slots g + 4 l1) -> m0 (slots g + 4 m0), then x *= tb[m0][l0] =
 *      e^{2 pi i l0 m0 / 64}                                                          (m0 > 0)
 *   T  LDS transpose: lane L'' = s' + 16 (L' >> 4) holds slot l0
 *   C  DFT16 over l0 -> m1: slot m1 of lane L'' = Z[k], k = (L''&3) + 4 (L''>>4) + 16 ((L''>>2)&3) + 64 m1,
 *      stored at device index L'' + 64 m1
 *   inverse: C' (inverse DFT16), T back, conj tb + inverse radix-4, X back, conj ta, inverse DFT16 (A'),
 *      conj(zeta^{64 e}) for e > 0; no 1/M (2^-10 is folded into the BSK)
 * DFT16 (natural in and out): radix-4 over n1 for each n0 (positions n0 + 4 k0), x[n0 + 4 k0] *= W16^{n0 k0}
 * (n0, k0 > 0: W^1 = (C16, S16), W^3 = (S16, C16), W^9 = (-C16, -S16) as cmul; W^2, W^6 as the w8 forms; W^4 = i),
 * radix-4 over n0 for each k0 (positions 4 k0 + k1) -> X[k0 + 4 k1].  radix-4 (a, b, c, d): t0 = a + c,
 * t1 = a - c, t2 = b + d, t3 = b - d; X0 = t0 + t2, X2 = t0 - t2, X1 = t1 + i t3, X3 = t1 - i t3 (inverse:
 * X1 = t1 - i t3, X3 = t1 + i t3).  The inverse DFT16 is the same with conjugate twiddles. */
#define C16 0.92387953251128675613
#define S16 0.38268343236508977173
typedef struct fft1k_tab {
  or_c64 slot[16];    /* zeta^{64 e} */
  or_c64 ta[16][64];  /* zeta^{L (1 + 4 k)} */
  or_c64 tb[4][16];   /* zeta^{64 l0 m} = e^{2 pi i l0 m / 64} */
} fft1k_tab;
static fft1k_tab g_tab1k;
static int g_tab1k_ready = 0;

static const fft1k_tab* tab1k(void) {
#pragma omp critical(or_fft_tab1k)
  {
    if (!g_tab1k_ready) {
      for (uint32_t e = 0; e < 16; e++) or_fft_twiddle(64 * e, 4096, &g_tab1k.slot[e].re, &g_tab1k.slot[e].im);
      for (uint32_t k = 0; k < 16; k++)
        for (uint32_t L = 0; L < 64; L++)
          or_fft_twiddle((L * (1 + 4 * k)) % 4096, 4096, &g_tab1k.ta[k][L].re, &g_tab1k.ta[k][L].im);
      for (uint32_t m = 0; m < 4; m++)
        for (uint32_t l = 0; l < 16; l++)
          or_fft_twiddle((64 * l * m) % 4096, 4096, &g_tab1k.tb[m][l].re, &g_tab1k.tb[m][l].im);
      __atomic_store_n(&g_tab1k_ready, 1, __ATOMIC_RELEASE);
    }
  }
  return &g_tab1k;
}

static inline or_c64 cmulc(or_c64 z, or_c64 w) { return cmul(z, w.re, -w.im); }

static void radix4(or_c64* x, int i0, int st, int inv) {
  const or_c64 a = x[i0], b = x[i0 + st], c = x[i0 + 2 * st], d = x[i0 + 3 * st];
  const or_c64 t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
  x[i0] = cadd(t0, t2);
  x[i0 + 2 * st] = csub(t0, t2);
  const or_c64 p = {t1.re - t3.im, t1.im + t3.re}, q = {t1.re + t3.im, t1.im - t3.re}; /* t1 + i t3, t1 - i t3 */
  x[i0 + st] = inv ? q : p;
  x[i0 + 3 * st] = inv ? p : q;
}

/* t * W16^k (inv: conj), k in {1, 2, 3, 4, 6, 9} */
static inline or_c64 w16(or_c64 t, int k, int inv) {
  const double p = t.re, q = t.im;
  or_c64 r;
  switch (k) {
    case 1: return inv ? cmul(t, C16, -S16) : cmul(t, C16, S16);
    case 3: return inv ? cmul(t, S16, -C16) : cmul(t, S16, C16);
    case 9: return inv ? cmul(t, -C16, S16) : cmul(t, -C16, -S16);
    case 2: return w8(t, 1, inv);
    case 6: return w8(t, 3, inv);
    default: /* 4: i */
      if (!inv) { r.re = -q; r.im = p; } else { r.re = q; r.im = -p; }
      return r;
  }
}

/* w8^j (j = 1, 3) without its sqrt(1/2) (fft1k.h w8u) */
static inline or_c64 w8u(or_c64 t, int j, int inv) {
  const double p = t.re, q = t.im;
  or_c64 r;
  if (j == 1) {
    if (!inv) { r.re = p - q; r.im = p + q; } else { r.re = p + q; r.im = q - p; }
  } else {
    if (!inv) { r.re = -(p + q); r.im = p - q; } else { r.re = q - p; r.im = -(p + q); }
  }
  return r;
}
/* radix4 over (a, b, c, d) with c = s cu (cs = 1) or b = s bu, d = s du (cs = 0), s folded into fmas (fft1k.h r4_cs /
 * r4_bds) */
static void radix4_s(or_c64* x, int i0, int cs, int inv) {
  const or_c64 a = x[i0], b = x[i0 + 1], c = x[i0 + 2], d = x[i0 + 3];
  or_c64 t0, t1, A, C, p, q;
  if (cs) {
    t0.re = fma(SQRT1_2, c.re, a.re); t0.im = fma(SQRT1_2, c.im, a.im);
    t1.re = fma(-SQRT1_2, c.re, a.re); t1.im = fma(-SQRT1_2, c.im, a.im);
    const or_c64 t2 = cadd(b, d), t3 = csub(b, d);
    A = cadd(t0, t2);
    C = csub(t0, t2);
    p = (or_c64){t1.re - t3.im, t1.im + t3.re};
    q = (or_c64){t1.re + t3.im, t1.im - t3.re};
  } else {
    t0 = cadd(a, c);
    t1 = csub(a, c);
    const or_c64 t2 = cadd(b, d), t3 = csub(b, d); /* / s */
    A.re = fma(SQRT1_2, t2.re, t0.re); A.im = fma(SQRT1_2, t2.im, t0.im);
    C.re = fma(-SQRT1_2, t2.re, t0.re); C.im = fma(-SQRT1_2, t2.im, t0.im);
    p.re = fma(-SQRT1_2, t3.im, t1.re); p.im = fma(SQRT1_2, t3.re, t1.im);
    q.re = fma(SQRT1_2, t3.im, t1.re); q.im = fma(-SQRT1_2, t3.re, t1.im);
  }
  x[i0] = A;
  x[i0 + 2] = C;
  x[i0 + 1] = inv ? q : p;
  x[i0 + 3] = inv ? p : q;
}

/* dft16 (round 5, = fft1k.h F1_DFT16_FMA): the first radix-4 pass, then group k0 = 0 plain, groups 1 and 3 with
 * W^1 / W^3 / W^9 as cmul and the W^2 / W^6 element unscaled (radix4_s cs = 1), group 2 with W^4 = i and the W^2 / W^6
 * elements unscaled (radix4_s cs = 0) */
static void dft16(or_c64 x[16], int inv) {
  for (int n0 = 0; n0 < 4; n0++) radix4(x, n0, 4, inv);
  radix4(x, 0, 1, inv);
  x[5] = w16(x[5], 1, inv);
  x[6] = w8u(x[6], 1, inv);
  x[7] = w16(x[7], 3, inv);
  radix4_s(x, 4, 1, inv);
  x[9] = w8u(x[9], 1, inv);
  x[10] = w16(x[10], 4, inv);
  x[11] = w8u(x[11], 3, inv);
  radix4_s(x, 8, 0, inv);
  x[13] = w16(x[13], 3, inv);
  x[14] = w8u(x[14], 3, inv);
  x[15] = w16(x[15], 9, inv);
  radix4_s(x, 12, 1, inv);
  or_c64 y[16];
  for (int k0 = 0; k0 < 4; k0++)
    for (int k1 = 0; k1 < 4; k1++) y[k0 + 4 * k1] = x[4 * k0 + k1];
  memcpy(x, y, sizeof(y));
}

/* the round-4 dft16, kept for reference; unused */
__attribute__((unused)) static void dft16_r4(or_c64 x[16], int inv) {
  static const int K[16] = {0, 0, 0, 0, 0, 1, 2, 3, 0, 2, 4, 6, 0, 3, 6, 9}; /* n0 k0 at position n0 + 4 k0 */
  for (int n0 = 0; n0 < 4; n0++) radix4(x, n0, 4, inv);
  for (int pos = 5; pos < 16; pos++)
    if ((pos & 3) && (pos >> 2)) x[pos] = w16(x[pos], K[(pos >> 2) * 4 + (pos & 3)], inv);
  for (int k0 = 0; k0 < 4; k0++) radix4(x, 4 * k0, 1, inv);
  or_c64 y[16];
  for (int k0 = 0; k0 < 4; k0++)
    for (int k1 = 0; k1 < 4; k1++) y[k0 + 4 * k1] = x[4 * k0 + k1];
  memcpy(x, y, sizeof(y));
}

static void fft1k_fwd(const double* a, or_c64* out) {
  const fft1k_tab* T = tab1k();
  static _Thread_local or_c64 X[64][16], Y[64][16];
  for (int L = 0; L < 64; L++) {
    or_c64* x = X[L];
    for (int e = 0; e < 16; e++) {
      const or_c64 v = {a[L + 64 * e], a[L + 64 * e + 1024]};
      x[e] = e ? cmul(v, T->slot[e].re, T->slot[e].im) : v;
    }
    dft16(x, 0);
    for (int k = 0; k < 16; k++) x[k] = cmul(x[k], T->ta[k][L].re, T->ta[k][L].im);
  }
  for (int Lp = 0; Lp < 64; Lp++) /* register exchange */
    for (int sp = 0; sp < 16; sp++) Y[Lp][sp] = X[(Lp & 15) | ((sp >> 2) << 4)][(sp & 3) | ((Lp >> 4) << 2)];
  for (int Lp = 0; Lp < 64; Lp++) { /* pass B */
    or_c64* y = Y[Lp];
    for (int g = 0; g < 4; g++) {
      radix4(y, g, 4, 0);
      for (int m = 1; m < 4; m++) y[g + 4 * m] = cmul(y[g + 4 * m], T->tb[m][Lp & 15].re, T->tb[m][Lp & 15].im);
    }
  }
  for (int Lpp = 0; Lpp < 64; Lpp++) { /* transpose + pass C */
    or_c64 z[16];
    for (int r = 0; r < 16; r++) z[r] = Y[r + 16 * (Lpp >> 4)][Lpp & 15];
    dft16(z, 0);
    for (int m = 0; m < 16; m++) out[Lpp + 64 * m] = z[m];
  }
}

static void fft1k_inv(const or_c64* in, double* a) {
  const fft1k_tab* T = tab1k();
  static _Thread_local or_c64 X[64][16], Y[64][16], Z[64][16];
  for (int Lpp = 0; Lpp < 64; Lpp++) { /* pass C' */
    for (int m = 0; m < 16; m++) Z[Lpp][m] = in[Lpp + 64 * m];
    dft16(Z[Lpp], 1);
  }
  for (int Lp = 0; Lp < 64; Lp++) { /* transpose back, conj tb, inverse radix-4 */
    or_c64* y = Y[Lp];
    for (int sp = 0; sp < 16; sp++) y[sp] = Z[sp + 16 * (Lp >> 4)][Lp & 15];
    for (int g = 0; g < 4; g++) {
      for (int m = 1; m < 4; m++) y[g + 4 * m] = cmulc(y[g + 4 * m], T->tb[m][Lp & 15]);
      radix4(y, g, 4, 1);
    }
  }
  for (int L = 0; L < 64; L++) { /* exchange back, conj ta, pass A', untwist */
    or_c64* x = X[L];
    for (int k = 0; k < 16; k++) x[k] = cmulc(Y[(L & 15) | ((k >> 2) << 4)][(k & 3) | ((L >> 4) << 2)], T->ta[k][L]);
    dft16(x, 1);
    for (int e = 0; e < 16; e++) {
      const or_c64 v = e ? cmulc(x[e], T->slot[e]) : x[e];
      a[L + 64 * e] = v.re;
      a[L + 64 * e + 1024] = v.im;
    }
  }
}

void or_fft_fwd(const double* a, uint32_t N, or_c64* out) {
  if (N == 4 * FFT_M) { fft1k_fwd(a, out); return; }
  if (N != 2 * FFT_M) abort();
  const fft_tab* T = tab();
  or_c64 z[FFT_M];
#if FFT_TDFT8
  for (int j = 0; j < FFT_M; j++) z[j] = (or_c64){a[j], a[j + FFT_M]};
  /* j = L + 64 e: the slot part zeta^{64 e} of the twist inside pass A's twisted DFT8, zeta^L in pass A's table */
  dft512_fwd_tab(z, out, T->twAm, 1, 1);
#else
  for (int j = 0; j < FFT_M; j++) { /* j = L + 64 e: slot constant zeta^{64 e} (e > 0), zeta^L in pass A */
    const or_c64 v = {a[j], a[j + FFT_M]};
    const int e = j >> 6;
    z[j] = e ? cmul(v, T->twist[64 * e].re, T->twist[64 * e].im) : v;
  }
  dft512_fwd_tab(z, out, T->twAm, 1, 0);
#endif
}

void or_fft_inv(const or_c64* in, uint32_t N, double* out) {
  if (N == 4 * FFT_M) { fft1k_inv(in, out); return; }
  if (N != 2 * FFT_M) abort();
  const fft_tab* T = tab();
  or_c64 z[FFT_M];
  dft512_inv_tab(in, z, T->twIm);
  for (int j = 0; j < FFT_M; j++) { /* conj(zeta^{64 e}) after pass A' (e > 0); conj(zeta^L) rode in pass B' */
    const int e = j >> 6;
    const or_c64 v = e ? cmul(z[j], T->twist[64 * e].re, -T->twist[64 * e].im) : z[j];
    out[j] = v.re;
    out[j + FFT_M] = v.im;
  }
}

/* The device's accumulator update (fft512.h torus_acc_add / torus_acc_add_wide, FFT_TORUS_NORINT, round 5): h =
 * floor(x 2^-32), l = fma(-h, 2^32, x) (exact unless -2^32 < x < 0, where x + 2^32 rounds once), and the increment
 * h 2^32 + rint(l) mod 2^64 -- rint(x) mod 2^64 except for that double rounding of tiny negative x.  The device takes
 * rint(l) from the bits of l + 2^52 and h mod 2^32 from those of h + 1.5 2^52 (N = 1024) or of the exact split
 * h - 2^32 floor(h 2^-32) + 1.5 2^52 (N = 2048); both are h mod 2^32 exactly, as computed here. */
uint64_t or_f64_to_torus_dev(double x) {
  const double h = floor(x * 0x1p-32);
  const double l = fma(-h, 0x1p32, x);
  const double hh = floor(h * 0x1p-32);
  const double hm = fma(-hh, 0x1p32, h); /* exact, in [0, 2^32) */
  return ((uint64_t)hm << 32) + (uint64_t)rint(l); /* rint(l) in [0, 2^32], the same as the bits of l + 2^52 */
}

/* round(x) (ties to even) mod 2^64; every step after rint is exact */
uint64_t or_f64_to_torus(double x) {
  const double t = rint(x);
  const double h = floor(t * 0x1p-32);
  const double l = t - h * 0x1p32;
  const double hh = floor(h * 0x1p-32);
  const double hm = h - hh * 0x1p32;
  return ((uint64_t)hm << 32) | (uint64_t)l;
}

void or_bsk_to_fourier(const or_params* p, const uint64_t* bsk, or_c64* bsk_f) {
  const uint32_t N = p->N, M = N / 2;
  const size_t polys = or_bsk_len(p) / N;
#pragma omp parallel for schedule(static)
  for (size_t q = 0; q < polys; q++) {
    double a[4 * FFT_M];
    const double inv_m = 1.0 / (double)M; /* 2^-9 (N = 1024) or 2^-10 (N = 2048): exact */
    for (uint32_t j = 0; j < N; j++) a[j] = (double)(int64_t)bsk[q * N + j];
    or_c64* o = bsk_f + q * M;
    or_fft_fwd(a, N, o);
    for (uint32_t j = 0; j < M; j++) {
      o[j].re = o[j].re * inv_m;
      o[j].im = o[j].im * inv_m;
    }
  }
}

/* (X^t * in)[i] on native torus values, t in [0, 2N) */
static void monomial_torus(uint64_t* out, const uint64_t* in, uint32_t N, uint32_t t) {
  for (uint32_t i = 0; i < N; i++) {
    int64_t d = (int64_t)i - (int64_t)t;
    int neg = 0;
    while (d < 0) { d += N; neg ^= 1; }
    out[i] = neg ? 0 - in[d] : in[d];
  }
}

/* the N = 2048 MAC order: 0 = one fma chain over every (c, l) from zero (pbs_fft2k.hip's slot-owned MAC), 1 = the
 * split order of N = 1024 (per-component products, then one add: pbs_fft2k.hip F1_PAIRMAC).  A/B switch, set through
 * or_set_fft2k_mac_split (oracle.py: ORACLE_FFT2K_SPLIT=1) */
int or_fft2k_mac_split = 0;
void or_set_fft2k_mac_split(int v) { or_fft2k_mac_split = v != 0; }

/* trace (nullable): (n + 1) x (k+1)N words, the accumulator before CMUX 0 and after every CMUX i (skipped CMUXes
 * included), so tests can hand each state to the exact arbiter (exact_oracle.c) */
static void blind_rotate_fft_impl(const or_params* p, const or_c64* bsk_f, const uint64_t* lwe_in, const uint64_t* lut,
                                  uint64_t* acc, uint64_t* trace) {
  const uint32_t N = p->N, M = N / 2, k = p->k, L = p->pbs_level, n = p->n;
  if (k != 1 || (N != 2 * FFT_M && N != 4 * FFT_M) || L > 8) abort();
  const size_t per_i = (size_t)(k + 1) * L * (k + 1) * M;
  uint64_t lt[4 * FFT_M], rot[4 * FFT_M];
  for (uint32_t i = 0; i < N; i++) lt[i] = or_p_to_tor(lut[i]); /* convert, then rotate */
  memset(acc, 0, (size_t)N * 8);
  const uint32_t bt = or_mod_switch(lwe_in[n], 2 * N);
  monomial_torus(acc + N, lt, N, (2 * N - bt) % (2 * N));
  static _Thread_local double dig[8][4 * FFT_M];
  or_c64 D[2 * FFT_M], O[2][2 * FFT_M], Oc[2][2 * FFT_M];
  /* MAC order.  N = 1024 (pbs_fft.hip: component-pair and latency kernels): one fma chain per component,
   * O_j = O_j^0 + O_j^1 with O_j^c = chain over the levels of D_(c,l) (.) BSK_i[(c, l)][j] from zero.
   * N = 2048 (pbs_fft2k.hip): one chain over every (c, l) from zero. */
  const int split = N == 2 * FFT_M || or_fft2k_mac_split;
  double res[4 * FFT_M];
  int64_t d[64];
  const size_t row = (size_t)(k + 1) * N;
  if (trace) memcpy(trace, acc, row * 8);
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t a = or_mod_switch(lwe_in[i], 2 * N);
    if (a == 0) { /* (X^0 - 1) acc == 0: every double stays +-0, rounds to 0 */
      if (trace) memcpy(trace + (i + 1) * row, acc, row * 8);
      continue;
    }
    memset(O, 0, sizeof(O));
    for (uint32_t c = 0; c <= k; c++) {
      monomial_torus(rot, acc + (size_t)c * N, N, a);
      for (uint32_t j = 0; j < N; j++) {
        or_decompose(rot[j] - acc[(size_t)c * N + j], p->pbs_base_log, L, d);
        for (uint32_t l = 0; l < L; l++) dig[l][j] = (double)d[l];
      }
      or_c64 (*A)[2 * FFT_M] = split ? Oc : O; /* this component's chain (split) or the running one */
      if (split) memset(Oc, 0, sizeof(Oc));
      for (int l = (int)L - 1; l >= 0; l--) {
        or_fft_fwd(dig[l], N, D);
        const or_c64* row = bsk_f + per_i * i + (size_t)(c * L + l) * (k + 1) * M;
        /* N = 1024: each component chain's first term is a multiply (pbs_fft.hip mac_first: the chain does not
         * start from a zeroed sum; the two forms differ only in the sign of an exact zero) */
        const int first = split && l == (int)L - 1;
        for (uint32_t j = 0; j <= k; j++) {
          const or_c64* K = row + (size_t)j * M;
          if (first) {
            for (uint32_t f = 0; f < M; f++) {
              A[j][f].re = D[f].re * K[f].re;
              A[j][f].re = fma(-D[f].im, K[f].im, A[j][f].re);
              A[j][f].im = D[f].re * K[f].im;
              A[j][f].im = fma(D[f].im, K[f].re, A[j][f].im);
            }
            continue;
          }
          for (uint32_t f = 0; f < M; f++) {
            A[j][f].re = fma(D[f].re, K[f].re, A[j][f].re);
            A[j][f].re = fma(-D[f].im, K[f].im, A[j][f].re);
            A[j][f].im = fma(D[f].re, K[f].im, A[j][f].im);
            A[j][f].im = fma(D[f].im, K[f].re, A[j][f].im);
          }
        }
      }
      if (split)
        for (uint32_t j = 0; j <= k; j++)
          for (uint32_t f = 0; f < M; f++) {
            if (c == 0) O[j][f] = Oc[j][f];
            else {
              O[j][f].re = O[j][f].re + Oc[j][f].re;
              O[j][f].im = O[j][f].im + Oc[j][f].im;
            }
          }
    }
    for (uint32_t j = 0; j <= k; j++) {
      or_fft_inv(O[j], N, res);
      /* the device's rint-free update at both N (fft512.h torus_acc_add_y / torus_acc_add_wide_y, round 5) */
      for (uint32_t f = 0; f < N; f++) acc[(size_t)j * N + f] += or_f64_to_torus_dev(res[f]);
    }
    if (trace) memcpy(trace + (i + 1) * row, acc, row * 8);
  }
}

void or_blind_rotate_fft(const or_params* p, const or_c64* bsk_f, const uint64_t* lwe_in, const uint64_t* lut,
                         uint64_t* acc) {
  blind_rotate_fft_impl(p, bsk_f, lwe_in, lut, acc, NULL);
}

void or_blind_rotate_fft_trace(const or_params* p, const or_c64* bsk_f, const uint64_t* lwe_in, const uint64_t* lut,
                               uint64_t* trace) {
  uint64_t* acc = (uint64_t*)malloc((size_t)(p->k + 1) * p->N * 8);
  blind_rotate_fft_impl(p, bsk_f, lwe_in, lut, acc, trace);
  free(acc);
}

void or_sample_extract_torus(const or_params* p, const uint64_t* acc, uint64_t* out) {
  const uint32_t N = p->N, k = p->k;
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = acc + (size_t)c * N;
    out[(size_t)c * N] = A[0];
    for (uint32_t j = 1; j < N; j++) out[(size_t)c * N + j] = 0 - A[N - j];
  }
  out[(size_t)k * N] = acc[(size_t)k * N];
}

void or_pbs_batch_fft(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const uint64_t* lwe_in, size_t B,
                      const uint64_t* luts, size_t n_lut, const uint32_t* lut_index, uint64_t* lwe_out, int threads) {
  or_pbs_batch_fft_ex(p, bsk_f, ksk, NULL, lwe_in, B, luts, n_lut, lut_index, lwe_out, threads);
}

/* order 0 (P-GATE): BR -> SE -> KS; order 1 (P-FHEVM): KS -> MS noise reduction (ms, nullable) -> BR -> SE,
 * the same sequence as or_pbs_ex with the FFT64 blind rotation */
void or_pbs_batch_fft_ex(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const or_ms_key* ms,
                         const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                         const uint32_t* lut_index, uint64_t* lwe_out, int threads) {
  const size_t big = (size_t)p->k * p->N + 1, small = (size_t)p->n + 1, row = (size_t)(p->k + 1) * p->N;
  const size_t din = p->order == 0 ? small : big, dout = p->order == 0 ? small : big;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
  for (size_t q = 0; q < B; q++) {
    size_t li = lut_index ? lut_index[q] : 0;
    if (li >= n_lut) li = 0;
    uint64_t* acc = (uint64_t*)malloc(row * 8);
    if (p->order == 0) {
      uint64_t* ext = (uint64_t*)malloc(big * 8);
      or_blind_rotate_fft(p, bsk_f, lwe_in + q * din, luts + li * p->N, acc);
      or_sample_extract_torus(p, acc, ext);
      or_keyswitch(p, ksk, ext, lwe_out + q * dout);
      free(ext);
    } else {
      uint64_t* sm = (uint64_t*)malloc(small * 8);
      or_keyswitch(p, ksk, lwe_in + q * din, sm);
      or_ms_reduce(p, ms, sm);
      or_blind_rotate_fft(p, bsk_f, sm, luts + li * p->N, acc);
      or_sample_extract_torus(p, acc, lwe_out + q * dout);
      free(sm);
    }
    free(acc);
  }
  (void)threads;
}

void or_poly_mul_torus_schoolbook(uint64_t* out, const int64_t* a, const uint64_t* b, uint32_t N) {
  memset(out, 0, (size_t)N * 8);
  for (uint32_t i = 0; i < N; i++) {
    if (!a[i]) continue;
    const uint64_t ai = (uint64_t)a[i];
    for (uint32_t j = 0; j < N; j++) {
      const uint32_t d = i + j;
      if (d < N) out[d] += ai * b[j];
      else out[d - N] -= ai * b[j];
    }
  }
}
