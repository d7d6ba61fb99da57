/*
 * fft_batch_body.h — the width-generic part of fft_batch.c (TEST INFRASTRUCTURE ONLY, see tfhe_oracle.h): one
 * blind rotation of BW ciphertexts, lane q of every BW x f64 vector holding ciphertext q.  Included once per width
 * by fft_batch_w4.c (AVX2, the x86-64-v3 build) and fft_batch_w8.c (AVX-512F, compiled for that target and only
 * called when the CPU reports it); each defines BW, BR_SIMD, VF (fma, one rounding), VFLOOR and VRINT (round to
 * nearest even) before the include.  Every floating-point operation is fft_oracle.c's, in its order.
 */
#include <stdlib.h>
#include <string.h>

#include "tfhe_oracle.h"

#define M4 512 /* complex points per transform (N = 1024) */
#define N4 1024

/* the tables of fft_oracle.c's fft_tab (built once by fft_batch.c from the same or_fft_twiddle values) */
typedef struct {
  or_c64 tw64[8];      /* zeta^{64 e}, zeta = e^{i pi / 1024} */
  or_c64 twB[8][64];   /* w^{8 (L & 7) e}, w = e^{2 pi i / 512} */
  or_c64 twAm[8][64];  /* zeta^{L (1 + 4 e)} */
  or_c64 twIm[8][64];  /* zeta^{(n0 + 8 e)(4 k0 + 1)}, L = n0 + 8 k0 */
} or_fftb_tab;
const or_fftb_tab* or_fftb_tables(void);
/* fft_oracle.c's fft1k_tab (N = 2048) */
typedef struct {
  or_c64 slot[16];    /* zeta^{64 e}, zeta = e^{2 pi i / 4096} */
  or_c64 ta[16][64];  /* zeta^{L (1 + 4 k)} */
  or_c64 tb[4][16];   /* e^{2 pi i l0 m / 64} */
} or_fftb_tab1k;
const or_fftb_tab1k* or_fftb_tables1k(void);
/* or_mod_switch(x, 4096) */
static inline uint32_t ms4096(uint64_t x) { return (uint32_t)((((x >> 51) + 1) >> 1) & 4095u); }

/* or_mod_switch(x, 2048) */
static inline uint32_t ms2048(uint64_t x) { return (uint32_t)((((x >> 52) + 1) >> 1) & 2047u); }

#ifdef BW
typedef double VD __attribute__((vector_size(8 * BW)));
typedef unsigned long long VU __attribute__((vector_size(8 * BW)));
typedef struct { VD re, im; } CX;

/* exact broadcasts (a vector-plus-scalar form would turn -0.0 into +0.0) */
static inline VD BC(double x) {
  VD r;
  for (int q = 0; q < BW; q++) r[q] = x;
  return r;
}
static inline VU BCU(unsigned long long x) {
  VU r;
  for (int q = 0; q < BW; q++) r[q] = x;
  return r;
}
static inline CX cadd(CX a, CX b) { CX r = {a.re + b.re, a.im + b.im}; return r; }
static inline CX csub(CX a, CX b) { CX r = {a.re - b.re, a.im - b.im}; return r; }
/* fft_oracle.c cmul: re = fma(z.re, wr, -(z.im wi)), im = fma(z.re, wi, z.im wr) */
static inline CX cmul(CX z, double wr, double wi) {
  const VD r = BC(wr), i = BC(wi);
  CX o = {VF(z.re, r, -(z.im * i)), VF(z.re, i, z.im * r)};
  return o;
}

#define SQRT1_2 0.70710678118654752440
/* fft_oracle.c dft8 (round-5 form), operation for operation */
static inline void dft8(CX x[8], int inv) {
  CX y[4], t[4];
  for (int j = 0; j < 4; j++) {
    y[j] = cadd(x[j], x[j + 4]);
    t[j] = csub(x[j], x[j + 4]);
  }
  VD ar, ai, cr, ci, z4r, z4i, z6r, z6i;
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
  const VD z5r = ar + cr, z5i = ai + ci, z7r = ar - cr, z7i = ai - ci;
  const CX e0 = cadd(y[0], y[2]), e2 = csub(y[0], y[2]), e1 = cadd(y[1], y[3]);
  const CX d13 = csub(y[1], y[3]);
  CX e3;  /* w8(d13, 2, inv): forward (-q, p), inverse (q, -p) */
  if (!inv) { e3.re = -d13.im; e3.im = d13.re; }
  else { e3.re = d13.im; e3.im = -d13.re; }
  x[0] = cadd(e0, e1);
  x[4] = csub(e0, e1);
  x[2] = cadd(e2, e3);
  x[6] = csub(e2, e3);
  const VD s = BC(SQRT1_2), ns = BC(-SQRT1_2);
  x[1].re = VF(s, z5r, z4r); x[1].im = VF(s, z5i, z4i);
  x[5].re = VF(ns, z5r, z4r); x[5].im = VF(ns, z5i, z4i);
  if (!inv) {
    x[3].re = VF(ns, z7i, z6r); x[3].im = VF(s, z7r, z6i);
    x[7].re = VF(s, z7i, z6r); x[7].im = VF(ns, z7r, z6i);
  } else {
    x[3].re = VF(s, z7i, z6r); x[3].im = VF(ns, z7r, z6i);
    x[7].re = VF(ns, z7i, z6r); x[7].im = VF(s, z7r, z6i);
  }
}

/* or_fft_fwd at N = 1024 (FFT_TDFT8 = 0): slot twist, then passes A (merged table), B, C; device order out */
static void fwd(const VD* a, CX* out, const or_fftb_tab* T) {
  CX A[64][8], Bv[64][8], x[8];
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) {
      const CX v = {a[L + 64 * e], a[L + 64 * e + M4]};
      x[e] = e ? cmul(v, T->tw64[e].re, T->tw64[e].im) : v;
    }
    dft8(x, 0);
    for (int e = 0; e < 8; e++) A[L][e] = cmul(x[e], T->twAm[e][L].re, T->twAm[e][L].im);
  }
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = A[(L & 7) + 8 * e][L >> 3];
    dft8(x, 0);
    Bv[L][0] = x[0];
    for (int e = 1; e < 8; e++) Bv[L][e] = cmul(x[e], T->twB[e][L].re, T->twB[e][L].im);
  }
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = Bv[e + 8 * (L >> 3)][L & 7];
    dft8(x, 0);
    for (int e = 0; e < 8; e++) out[L + 64 * e] = x[e];
  }
}

/* or_fft_inv at N = 1024: passes C', B' (merged table), A', then conj(zeta^{64 e}); N doubles out (not rounded) */
static void inv(const CX* in, VD* out, const or_fftb_tab* T) {
  CX S1[64][8], S2[64][8], x[8];
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = in[L + 64 * e];
    dft8(x, 1);
    S1[L][0] = x[0];
    for (int e = 1; e < 8; e++) S1[L][e] = cmul(x[e], T->twB[e][L].re, -T->twB[e][L].im);
  }
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = S1[e + 8 * (L >> 3)][L & 7];
    dft8(x, 1);
    for (int e = 0; e < 8; e++) S2[L][e] = cmul(x[e], T->twIm[e][L].re, -T->twIm[e][L].im);
  }
  for (int L = 0; L < 64; L++) {
    for (int e = 0; e < 8; e++) x[e] = S2[(L & 7) + 8 * e][L >> 3];
    dft8(x, 1);
    for (int e = 0; e < 8; e++) {
      const CX v = e ? cmul(x[e], T->tw64[e].re, -T->tw64[e].im) : x[e];
      out[L + 64 * e] = v.re;
      out[L + 64 * e + M4] = v.im;
    }
  }
}

/* or_f64_to_torus_dev, BW lanes: h = floor(x 2^-32), l = fma(-h, 2^32, x), hm = h mod 2^32 (exact split),
 * increment = hm 2^32 + rint(l); hm and rint(l) are integers in [0, 2^32], read from the bits of v + 2^52 */
static inline VU torus_dev(VD x) {
  const VD two32 = BC(0x1p32), inv32 = BC(0x1p-32), m52 = BC(0x1p52);
  const VD h = VFLOOR(x * inv32);
  const VD l = VF(-h, two32, x);
  const VD hh = VFLOOR(h * inv32);
  const VD hm = VF(-hh, two32, h);
  const VD rl = VRINT(l);
  const VU mant = BCU((1ull << 52) - 1);
  return ((((VU)(hm + m52)) & mant) << 32) + (((VU)(rl + m52)) & mant);
}

/* or_decompose at base_log 7 x 3 levels on BW lanes: digits d[l] as exact doubles (|d| <= 64, through the
 * 2^52 + 2^51 bias: bits(2^52 + 2^51 + d) - (2^52 + 2^51) = d) */
static inline void decompose_7x3(VU x, VD d[3]) {
  const VU one = BCU(1), mask = BCU(127), m21 = BCU(0x1FFFFF);
  VU state = (((x >> 42) + one) >> 1) & m21;
  const VU bias = BCU(0x4338000000000000ull);
  const VD fbias = BC(0x1.8p52);
  for (int l = 2; l >= 0; l--) {
    const VU res = state & mask;
    state = state >> 7;
    const VU carry = ((((res - one) | state) & res) >> 6) & one;
    state = state + carry;
    const VU dig = res - (carry << 7); /* two's complement: bits(1.5 2^52 + d) = bias + d */
    d[l] = (VD)(dig + bias) - fbias;
  }
}

/* blind rotation of BW ciphertexts (fft_oracle.c blind_rotate_fft_impl, N = 1024 split MAC); acc_out[q]: 2N words */
void BR_SIMD(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe, const uint64_t* const* lut,
             uint64_t* const* acc_out) {
  const or_fftb_tab* T = or_fftb_tables();
  const uint32_t n = p->n, L = 3;
  const size_t per_i = (size_t)2 * L * 2 * M4;
  /* accumulators, lane-interleaved: acc[c][j] lane q */
  VU* acc = (VU*)aligned_alloc(64, sizeof(VU) * 2 * N4);
  VU* rot = (VU*)aligned_alloc(64, sizeof(VU) * N4);
  VD* dig = (VD*)aligned_alloc(64, sizeof(VD) * 3 * N4);
  VD* res = (VD*)aligned_alloc(64, sizeof(VD) * N4);
  CX* D = (CX*)aligned_alloc(64, sizeof(CX) * M4);
  CX* O = (CX*)aligned_alloc(64, sizeof(CX) * 2 * M4);
  CX* Oc = (CX*)aligned_alloc(64, sizeof(CX) * 2 * M4);
  for (int q = 0; q < BW; q++) {
    const uint32_t bt = ms2048(lwe[q][n]), t = (2 * N4 - bt) % (2 * N4);
    for (uint32_t j = 0; j < N4; j++) { /* acc_0 = 0, acc_1 = X^{-b~} lut (monomial_torus) */
      int64_t d = (int64_t)j - (int64_t)t;
      int neg = 0;
      while (d < 0) { d += N4; neg ^= 1; }
      const uint64_t v = or_p_to_tor(lut[q][d]);
      acc[j][q] = 0;
      acc[N4 + j][q] = neg ? 0 - v : v;
    }
  }
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a[BW];
    for (int q = 0; q < BW; q++) a[q] = ms2048(lwe[q][i]);
    /* a lane with a = 0 runs the CMUX on zero digits: every double is +-0 and the update adds 0, as the scalar
     * restatement's skip leaves the accumulator */
    const double* Kb = (const double*)(bsk_f + per_i * i);
    for (uint32_t c = 0; c < 2; c++) {
      const VU* ac = acc + (size_t)c * N4;
      for (int q = 0; q < BW; q++) { /* (X^a acc_c) lane q = monomial_torus: j < r from r' - ... (sign s1), rest s0 */
        const uint32_t r = a[q] & (N4 - 1);
        const uint64_t s0 = a[q] >= N4 ? ~0ull : 0, s1 = ~s0; /* all ones = negate: (v ^ s) - s */
        for (uint32_t j = 0; j < r; j++) rot[j][q] = (ac[j + N4 - r][q] ^ s1) - s1;
        for (uint32_t j = r; j < N4; j++) rot[j][q] = (ac[j - r][q] ^ s0) - s0;
      }
      for (uint32_t j = 0; j < N4; j++) {
        VD d3[3];
        decompose_7x3(rot[j] - ac[j], d3);
        dig[j] = d3[0];
        dig[N4 + j] = d3[1];
        dig[2 * N4 + j] = d3[2];
      }
      for (int l = 2; l >= 0; l--) {
        fwd(dig + (size_t)l * N4, D, T);
        const double* row = Kb + 2 * ((size_t)(c * L + l) * 2 * M4);
        for (uint32_t j = 0; j < 2; j++) {
          const double* K = row + 2 * (size_t)j * M4;
          CX* A = Oc + (size_t)j * M4;
          if (l == 2) {
            for (uint32_t f = 0; f < M4; f++) {
              const VD kr = BC(K[2 * f]), ki = BC(K[2 * f + 1]);
              A[f].re = D[f].re * kr;
              A[f].re = VF(-D[f].im, ki, A[f].re);
              A[f].im = D[f].re * ki;
              A[f].im = VF(D[f].im, kr, A[f].im);
            }
          } else {
            for (uint32_t f = 0; f < M4; f++) {
              const VD kr = BC(K[2 * f]), ki = BC(K[2 * f + 1]);
              A[f].re = VF(D[f].re, kr, A[f].re);
              A[f].re = VF(-D[f].im, ki, A[f].re);
              A[f].im = VF(D[f].re, ki, A[f].im);
              A[f].im = VF(D[f].im, kr, A[f].im);
            }
          }
        }
      }
      if (c == 0) memcpy(O, Oc, sizeof(CX) * 2 * M4);
      else
        for (uint32_t f = 0; f < 2 * M4; f++) O[f] = cadd(O[f], Oc[f]);
    }
    for (uint32_t j = 0; j < 2; j++) {
      inv(O + (size_t)j * M4, res, T);
      VU* aj = acc + (size_t)j * N4;
      for (uint32_t f = 0; f < N4; f++) aj[f] = aj[f] + torus_dev(res[f]);
    }
  }
  for (int q = 0; q < BW; q++)
    for (uint32_t j = 0; j < 2 * N4; j++) acc_out[q][j] = acc[j][q];
  free(acc); free(rot); free(dig); free(res); free(D); free(O); free(Oc);
}


/* ---- N = 2048 (P-FHEVM): fft_oracle.c fft1k_fwd / fft1k_inv, dft16, radix-4, operation for operation ---- */
#define C16 0.92387953251128675613
#define S16 0.38268343236508977173
static inline void radix4(CX* x, int i0, int st, int inv) {
  const CX a = x[i0], b = x[i0 + st], c = x[i0 + 2 * st], d = x[i0 + 3 * st];
  const CX t0 = cadd(a, c), t1 = csub(a, c), t2 = cadd(b, d), t3 = csub(b, d);
  x[i0] = cadd(t0, t2);
  x[i0 + 2 * st] = csub(t0, t2);
  const CX p = {t1.re - t3.im, t1.im + t3.re}, q = {t1.re + t3.im, t1.im - t3.re};
  x[i0 + st] = inv ? q : p;
  x[i0 + 3 * st] = inv ? p : q;
}
/* t * W16^k (inv: conj) for the k dft16 uses: 1, 3, 9 as cmul, 4 = i */
static inline CX w16(CX t, int k, int inv) {
  switch (k) {
    case 1: return inv ? cmul(t, C16, -S16) : cmul(t, C16, S16);
    case 3: return inv ? cmul(t, S16, -C16) : cmul(t, S16, C16);
    case 9: return inv ? cmul(t, -C16, S16) : cmul(t, -C16, -S16);
    default: {
      CX r;
      if (!inv) { r.re = -t.im; r.im = t.re; } else { r.re = t.im; r.im = -t.re; }
      return r;
    }
  }
}
static inline CX w8u(CX t, int j, int inv) {
  const VD p = t.re, q = t.im;
  CX r;
  if (j == 1) {
    if (!inv) { r.re = p - q; r.im = p + q; } else { r.re = p + q; r.im = q - p; }
  } else {
    if (!inv) { r.re = -(p + q); r.im = p - q; } else { r.re = q - p; r.im = -(p + q); }
  }
  return r;
}
static inline void radix4_s(CX* x, int i0, int cs, int inv) {
  const CX a = x[i0], b = x[i0 + 1], c = x[i0 + 2], d = x[i0 + 3];
  const VD s = BC(SQRT1_2), ns = BC(-SQRT1_2);
  CX t0, t1, A, C, p, q;
  if (cs) {
    t0.re = VF(s, c.re, a.re); t0.im = VF(s, c.im, a.im);
    t1.re = VF(ns, c.re, a.re); t1.im = VF(ns, c.im, a.im);
    const CX t2 = cadd(b, d), t3 = csub(b, d);
    A = cadd(t0, t2);
    C = csub(t0, t2);
    p.re = t1.re - t3.im; p.im = t1.im + t3.re;
    q.re = t1.re + t3.im; q.im = t1.im - t3.re;
  } else {
    t0 = cadd(a, c);
    t1 = csub(a, c);
    const CX t2 = cadd(b, d), t3 = csub(b, d);
    A.re = VF(s, t2.re, t0.re); A.im = VF(s, t2.im, t0.im);
    C.re = VF(ns, t2.re, t0.re); C.im = VF(ns, t2.im, t0.im);
    p.re = VF(ns, t3.im, t1.re); p.im = VF(s, t3.re, t1.im);
    q.re = VF(s, t3.im, t1.re); q.im = VF(ns, t3.re, t1.im);
  }
  x[i0] = A;
  x[i0 + 2] = C;
  x[i0 + 1] = inv ? q : p;
  x[i0 + 3] = inv ? p : q;
}
static inline void dft16(CX x[16], int inv) {
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
  CX y[16];
  for (int k0 = 0; k0 < 4; k0++)
    for (int k1 = 0; k1 < 4; k1++) y[k0 + 4 * k1] = x[4 * k0 + k1];
  memcpy(x, y, sizeof(y));
}
/* X, Y, Z: 64 x 16 workspaces each */
static void fwd2k(const VD* a, CX* out, const or_fftb_tab1k* T, CX (*X)[16], CX (*Y)[16]) {
  for (int L = 0; L < 64; L++) {
    CX* x = X[L];
    for (int e = 0; e < 16; e++) {
      const CX v = {a[L + 64 * e], a[L + 64 * e + 1024]};
      x[e] = e ? cmul(v, T->slot[e].re, T->slot[e].im) : v;
    }
    dft16(x, 0);
    for (int k = 0; k < 16; k++) x[k] = cmul(x[k], T->ta[k][L].re, T->ta[k][L].im);
  }
  for (int Lp = 0; Lp < 64; Lp++)
    for (int sp = 0; sp < 16; sp++) Y[Lp][sp] = X[(Lp & 15) | ((sp >> 2) << 4)][(sp & 3) | ((Lp >> 4) << 2)];
  for (int Lp = 0; Lp < 64; Lp++) {
    CX* y = Y[Lp];
    for (int g = 0; g < 4; g++) {
      radix4(y, g, 4, 0);
      for (int m = 1; m < 4; m++) y[g + 4 * m] = cmul(y[g + 4 * m], T->tb[m][Lp & 15].re, T->tb[m][Lp & 15].im);
    }
  }
  for (int Lpp = 0; Lpp < 64; Lpp++) {
    CX z[16];
    for (int r = 0; r < 16; r++) z[r] = Y[r + 16 * (Lpp >> 4)][Lpp & 15];
    dft16(z, 0);
    for (int m = 0; m < 16; m++) out[Lpp + 64 * m] = z[m];
  }
}
static void inv2k(const CX* in, VD* a, const or_fftb_tab1k* T, CX (*X)[16], CX (*Y)[16], CX (*Z)[16]) {
  for (int Lpp = 0; Lpp < 64; Lpp++) {
    for (int m = 0; m < 16; m++) Z[Lpp][m] = in[Lpp + 64 * m];
    dft16(Z[Lpp], 1);
  }
  for (int Lp = 0; Lp < 64; Lp++) {
    CX* y = Y[Lp];
    for (int sp = 0; sp < 16; sp++) y[sp] = Z[sp + 16 * (Lp >> 4)][Lp & 15];
    for (int g = 0; g < 4; g++) {
      for (int m = 1; m < 4; m++) y[g + 4 * m] = cmul(y[g + 4 * m], T->tb[m][Lp & 15].re, -T->tb[m][Lp & 15].im);
      radix4(y, g, 4, 1);
    }
  }
  for (int L = 0; L < 64; L++) {
    CX* x = X[L];
    for (int k = 0; k < 16; k++)
      x[k] = cmul(Y[(L & 15) | ((k >> 2) << 4)][(k & 3) | ((L >> 4) << 2)], T->ta[k][L].re, -T->ta[k][L].im);
    dft16(x, 1);
    for (int e = 0; e < 16; e++) {
      const CX v = e ? cmul(x[e], T->slot[e].re, -T->slot[e].im) : x[e];
      a[L + 64 * e] = v.re;
      a[L + 64 * e + 1024] = v.im;
    }
  }
}

/* or_decompose at base_log 23 x 1 level (digits up to 2^22: exact through the same 1.5 2^52 bias) */
static inline VD decompose_23x1(VU x) {
  const VU one = BCU(1), m23 = BCU(0x7FFFFF);
  const VU res = (((x >> 40) + one) >> 1) & m23;
  const VU carry = (((res - one) & res) >> 22) & one;
  return (VD)((res - (carry << 23)) + BCU(0x4338000000000000ull)) - BC(0x1.8p52);
}

/* blind rotation of BW ciphertexts at N = 2048, k = 1, 2^23 x 1 (fft_oracle.c blind_rotate_fft_impl: ONE fma chain
 * per output over (c, l) from zero) */
void BR_SIMD_2K(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe, const uint64_t* const* lut,
                uint64_t* const* acc_out) {
  enum { N2 = 2048, M2 = 1024 };
  const or_fftb_tab1k* T = or_fftb_tables1k();
  const uint32_t n = p->n;
  const size_t per_i = (size_t)2 * 1 * 2 * M2;
  VU* acc = (VU*)aligned_alloc(64, sizeof(VU) * 2 * N2);
  VU* rot = (VU*)aligned_alloc(64, sizeof(VU) * N2);
  VD* dig = (VD*)aligned_alloc(64, sizeof(VD) * N2);
  VD* res = (VD*)aligned_alloc(64, sizeof(VD) * N2);
  CX* D = (CX*)aligned_alloc(64, sizeof(CX) * M2);
  CX* O = (CX*)aligned_alloc(64, sizeof(CX) * 2 * M2);
  CX(*X)[16] = (CX(*)[16])aligned_alloc(64, sizeof(CX) * 64 * 16);
  CX(*Y)[16] = (CX(*)[16])aligned_alloc(64, sizeof(CX) * 64 * 16);
  CX(*Z)[16] = (CX(*)[16])aligned_alloc(64, sizeof(CX) * 64 * 16);
  for (int q = 0; q < BW; q++) {
    const uint32_t bt = ms4096(lwe[q][n]), t = (2 * N2 - bt) % (2 * N2);
    for (uint32_t j = 0; j < N2; j++) {
      int64_t d = (int64_t)j - (int64_t)t;
      int neg = 0;
      while (d < 0) { d += N2; neg ^= 1; }
      const uint64_t v = or_p_to_tor(lut[q][d]);
      acc[j][q] = 0;
      acc[N2 + j][q] = neg ? 0 - v : v;
    }
  }
  const VD zero = BC(0.0);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a[BW];
    for (int q = 0; q < BW; q++) a[q] = ms4096(lwe[q][i]);
    const double* Kb = (const double*)(bsk_f + per_i * i);
    for (uint32_t f = 0; f < 2 * M2; f++) { O[f].re = zero; O[f].im = zero; }
    for (uint32_t c = 0; c < 2; c++) {
      const VU* ac = acc + (size_t)c * N2;
      for (int q = 0; q < BW; q++) {
        const uint32_t r = a[q] & (N2 - 1);
        const uint64_t s0 = a[q] >= N2 ? ~0ull : 0, s1 = ~s0;
        for (uint32_t j = 0; j < r; j++) rot[j][q] = (ac[j + N2 - r][q] ^ s1) - s1;
        for (uint32_t j = r; j < N2; j++) rot[j][q] = (ac[j - r][q] ^ s0) - s0;
      }
      for (uint32_t j = 0; j < N2; j++) dig[j] = decompose_23x1(rot[j] - ac[j]);
      fwd2k(dig, D, T, X, Y);
      const double* row = Kb + 2 * ((size_t)c * 2 * M2);
      for (uint32_t j = 0; j < 2; j++) {
        const double* K = row + 2 * (size_t)j * M2;
        CX* A = O + (size_t)j * M2;
        for (uint32_t f = 0; f < M2; f++) {
          const VD kr = BC(K[2 * f]), ki = BC(K[2 * f + 1]);
          A[f].re = VF(D[f].re, kr, A[f].re);
          A[f].re = VF(-D[f].im, ki, A[f].re);
          A[f].im = VF(D[f].re, ki, A[f].im);
          A[f].im = VF(D[f].im, kr, A[f].im);
        }
      }
    }
    for (uint32_t j = 0; j < 2; j++) {
      inv2k(O + (size_t)j * M2, res, T, X, Y, Z);
      VU* aj = acc + (size_t)j * N2;
      for (uint32_t f = 0; f < N2; f++) aj[f] = aj[f] + torus_dev(res[f]);
    }
  }
  for (int q = 0; q < BW; q++)
    for (uint32_t j = 0; j < 2 * N2; j++) acc_out[q][j] = acc[j][q];
  free(acc); free(rot); free(dig); free(res); free(D); free(O); free(X); free(Y); free(Z);
}
#endif /* BW */
