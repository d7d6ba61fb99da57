/*
 * sns_oracle.c — CPU restatement of switch-and-squash / noise squashing (fhEVM's
 * sns-worker, coprocessor-docker-compose.yml:124-140).  TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h).
 *
 * tfhe-rs (absent from /root/reference) squashes a P-FHEVM ciphertext by keyswitching it to the small
 * key, reducing its modulus-switch noise, and bootstrapping it with a BSK encrypted under a 128-bit
 * GLWE key with the identity LUT: the output is an LWE over Z_2^128 (dim k*N) carrying the same
 * message with tiny noise, which threshold decryption can then flood.  Its parameter set
 * (NOISE_SQUASHING_PARAM_..._MESSAGE_2_CARRY_2_KS_PBS_TUNIFORM_2M128) is not in the mount; we use its
 * published shape: k = 2, N = 2048, base 2^24 x 3 levels, GLWE noise 2^30 (of 2^128).
 *
 * Arithmetic (round 3): the native 2^128 torus, as tfhe-rs has it.  GLWE / BSK / accumulator
 * coefficients are Z_2^128 words stored as two u64 planes (lo, hi); the decomposition reads the word
 * directly (tfhe-rs SignedDecomposer, 72 bits as 3 digits of 24, gadget 2^(128 - 24 (l + 1))).
 *
 * The external product restates the device's precision contract (tfhe_amd/csrc/sns.hip, sns_fft.h): at
 * load every key coefficient is rounded to the nearest multiple of 2^16 (or_sns_bsk_round), so a key word
 * is 2^16 x a 112-bit signed integer = 2^16 (l_0 + sum_(t=1..4) l_t 2^(48 + 16 (t - 1))) with l_0 the
 * balanced low 48 bits and l_1..l_4 balanced 16-bit limbs (round 4; seven 16-bit limbs before).  The
 * product digits x key is sum_t 2^(16 + w_t) (sum_r d_r (*) l_(r, t)) mod 2^128 (w_0 = 0,
 * w_t = 48 + 16 (t - 1)):
 *  * limbs 1..4: every convolution is an integer of magnitude <= 9 * 2048 * 2^23 * 2^15 = 2^52.2; the
 *    oracle computes it EXACTLY with the negacyclic NTT mod p = 2^64 - 2^32 + 1 (|value| < p / 2: the
 *    signed lift of the residue is the integer) -- an independent method from the device's f64 FFT, which
 *    must land on the same integers;
 *  * limb 0: its products reach 2^84 and the device's f64 values are not the exact integers (the error,
 *    <= 2^33.3 even for all-maximum operands, lands at weight 2^16 of a 2^128 torus whose output noise is
 *    ~2^64).  The oracle RESTATES the
 *    device's f64 computation for this limb operation by operation (sf_* below: the twisted fold, the
 *    radix-4 DIF / DIT stages, explicit fused multiply-adds, the 9-term MAC order, the untwist, rint and
 *    the conversion of the double's bits), as oracle/fft_oracle.c does for the FFT64 PBS; contraction is
 *    off (Makefile).
 *
 * Key generation: body = sum_j mask_j (*) S_j + e + s_i g_l (mod 2^128); the binary-key products are
 * computed here by rotated additions (the product library uses exact NTTs of 32-bit quarters: any exact
 * method gives the same words).
 *
 * Parity unpinned (no squashed ciphertext in the reference); message-level checks pin
 * decrypt(squash(ct)) == decrypt(ct).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "tfhe_oracle.h"

typedef unsigned __int128 u128;

static const uint64_t SP[2] = {0xFFFFFFFF00000001ull, 0xFFFFFFFC00000001ull};

/* x mod p1 (p1 = 2^64 - 2^32 + 1: 2^64 = 2^32 - 1, 2^96 = -1), canonical */
static inline uint64_t gl_red(u128 x) {
  const uint64_t E = 0xFFFFFFFFull, lo = (uint64_t)x, hi = (uint64_t)(x >> 64), hh = hi >> 32, hl = hi & E;
  uint64_t t0 = lo - hh;
  if (lo < hh) t0 -= E; /* borrow: + 2^64 - E = + p */
  const uint64_t t1 = hl * E;
  uint64_t r = t0 + t1;
  if (r < t1) r += E; /* carry: - 2^64 + E = - p */
  return r >= SP[0] ? r - SP[0] : r;
}
static inline uint64_t mmul(uint64_t a, uint64_t b, uint64_t p) {
  return p == SP[0] ? gl_red((u128)a * b) : (uint64_t)(((u128)a * b) % p);
}
static inline uint64_t madd(uint64_t a, uint64_t b, uint64_t p) {
  u128 s = (u128)a + b;
  return (uint64_t)(s >= p ? s - p : s);
}
static inline uint64_t msub(uint64_t a, uint64_t b, uint64_t p) { return a >= b ? a - b : a + (p - b); }
static uint64_t mpow(uint64_t a, uint64_t e, uint64_t p) {
  uint64_t r = 1;
  while (e) {
    if (e & 1) r = mmul(r, a, p);
    a = mmul(a, a, p);
    e >>= 1;
  }
  return r;
}
static inline uint64_t from_i64(int64_t v, uint64_t p) { return v >= 0 ? (uint64_t)v % p : p - ((uint64_t)(-v) % p); }

uint64_t or_sns_prime(int which) { return SP[which & 1]; }

/* psi: a^((p-1)/2N) for the smallest quadratic non-residue a (psi^N = -1: primitive 2N-th root) */
uint64_t or_sns_psi(int which, uint32_t N) {
  const uint64_t p = SP[which & 1];
  for (uint64_t a = 2;; a++)
    if (mpow(a, (p - 1) / 2, p) == p - 1) return mpow(a, (p - 1) / (2ull * N), p);
}

static void ntt_core(uint64_t* a, uint32_t N, uint64_t w, uint64_t p) {
  for (uint32_t i = 1, j = 0; i < N; i++) { /* bit reversal */
    uint32_t bit = N >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { uint64_t t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (uint32_t len = 2; len <= N; len <<= 1) {
    const uint64_t wl = mpow(w, N / len, p);
    for (uint32_t i = 0; i < N; i += len) {
      uint64_t wn = 1;
      for (uint32_t j = 0; j < len / 2; j++) {
        const uint64_t u = a[i + j], v = mmul(a[i + j + len / 2], wn, p);
        a[i + j] = madd(u, v, p);
        a[i + j + len / 2] = msub(u, v, p);
        wn = mmul(wn, wl, p);
      }
    }
  }
}

/* A[j] = a(psi^(2j+1)) mod p_which, natural order; inverse includes 1/N */
void or_sns_ntt_fwd(int which, uint64_t* a, uint32_t N) {
  const uint64_t p = SP[which & 1], psi = or_sns_psi(which, N);
  uint64_t t = 1;
  for (uint32_t i = 0; i < N; i++) { a[i] = mmul(a[i], t, p); t = mmul(t, psi, p); }
  ntt_core(a, N, mmul(psi, psi, p), p);
}
void or_sns_ntt_inv(int which, uint64_t* a, uint32_t N) {
  const uint64_t p = SP[which & 1], psi = or_sns_psi(which, N), ipsi = mpow(psi, p - 2, p);
  ntt_core(a, N, mmul(ipsi, ipsi, p), p);
  const uint64_t ninv = mpow(N, p - 2, p);
  uint64_t t = ninv;
  for (uint32_t i = 0; i < N; i++) { a[i] = mmul(a[i], t, p); t = mmul(t, ipsi, p); }
}

int or_sns_params_preset(int preset, or_sns_params* o) {
  if (preset != 0) return -1;
  o->n = 918; o->k = 2; o->N = 2048; o->base_log = 24; o->level = 3; o->noise_log2 = -34;
  return 0;
}

size_t or_sns_bsk_len(const or_sns_params* sp) {
  return (size_t)sp->n * (sp->k + 1) * sp->level * (sp->k + 1) * 2 * sp->N;
}

static inline u128 ld128(const uint64_t* plane_lo, size_t N, size_t t) { return ((u128)plane_lo[N + t] << 64) | plane_lo[t]; }
static inline void st128(uint64_t* plane_lo, size_t N, size_t t, u128 v) {
  plane_lo[t] = (uint64_t)v;
  plane_lo[N + t] = (uint64_t)(v >> 64);
}

/* tfhe-rs SignedDecomposer on a 128-bit word: digits[0] most significant (gadget 2^(128-B(l+1))) */
static void decompose128(u128 x, uint32_t base_log, uint32_t level, int64_t* digits) {
  const uint32_t prec = base_log * level, nonrep = 128 - prec;
  u128 state = ((x >> (nonrep - 1)) + 1) >> 1;
  state &= ((u128)1 << prec) - 1;
  const uint64_t B = 1ull << base_log, mask = B - 1;
  for (int l = (int)level - 1; l >= 0; l--) {
    const uint64_t res = (uint64_t)state & mask;
    state >>= base_log;
    const uint64_t carry = ((((res - 1) | (uint64_t)state) & res) >> (base_log - 1)) & 1;
    state += carry;
    digits[l] = (int64_t)res - (int64_t)(carry << base_log);
  }
}

/* ---- keys ---------------------------------------------------------------------------------- */
/* GLWE key: k*N bits from ChaCha stream 5.  BSK row (i, c, l) on stream 0x400000 + i: masks uniform over
 * Z_2^128 (per coefficient the lo word, then the hi word), one Gaussian integer of noise per body
 * coefficient, body = sum_j mask_j (*) S_j + e; s_i * 2^(128 - B (l + 1)) is added to coefficient 0 of
 * component c.  Layout [i][c*L + l][j][word: lo, hi][N]. */
void or_sns_keygen(const or_sns_params* sp, uint64_t seed, const uint64_t* lwe_key, uint64_t* glwe_key,
                   uint64_t* bsk) {
  const uint32_t k = sp->k, N = sp->N, L = sp->level;
  or_rng r;
  or_rng_init(&r, seed, 5);
  for (uint32_t i = 0; i < k * N; i++) glwe_key[i] = or_rng_u64(&r) & 1;
  if (!bsk) return;
  const size_t row = (size_t)(k + 1) * 2 * N, per_i = (size_t)(k + 1) * L * row;
#pragma omp parallel for schedule(dynamic, 1)
  for (uint32_t i = 0; i < sp->n; i++) {
    or_rng rr;
    or_rng_init(&rr, seed, 0x400000 + i);
    u128* body = (u128*)malloc((size_t)N * sizeof(u128));
    u128* mask = (u128*)malloc((size_t)N * sizeof(u128));
    for (uint32_t c = 0; c <= k; c++)
      for (uint32_t l = 0; l < L; l++) {
        uint64_t* out = bsk + per_i * i + row * (c * L + l); /* [j][w][N] */
        for (uint32_t j = 0; j < k; j++)
          for (uint32_t t = 0; t < N; t++) {
            const uint64_t lo = or_rng_u64(&rr), hi = or_rng_u64(&rr);
            st128(out + (size_t)j * 2 * N, N, t, ((u128)hi << 64) | lo);
          }
        for (uint32_t t = 0; t < N; t++) body[t] = (u128)(__int128)or_rng_gauss(&rr, sp->noise_log2);
        /* + mask_j (*) S_j: for each key bit u set, add X^u mask_j (negacyclic) */
        for (uint32_t j = 0; j < k; j++) {
          for (uint32_t t = 0; t < N; t++) mask[t] = ld128(out + (size_t)j * 2 * N, N, t);
          const uint64_t* S = glwe_key + (size_t)j * N;
          for (uint32_t u = 0; u < N; u++) {
            if (!S[u]) continue;
            for (uint32_t x = 0; x < u; x++) body[x] -= mask[x + N - u];
            for (uint32_t x = u; x < N; x++) body[x] += mask[x - u];
          }
        }
        for (uint32_t t = 0; t < N; t++) st128(out + (size_t)k * 2 * N, N, t, body[t]);
        if (lwe_key[i]) {
          const u128 g = (u128)1 << (128 - sp->base_log * (l + 1));
          uint64_t* dst = out + (size_t)c * 2 * N;
          st128(dst, N, 0, ld128(dst, N, 0) + g);
        }
      }
    free(body);
    free(mask);
  }
}

/* ---- the device's f64 transform for the low limb (tfhe_amd/csrc/sns_fft.h, restated) ---------------- */
#define SF_M 1024
typedef struct { double x, y; } sf_cd;
static inline sf_cd sf_add(sf_cd a, sf_cd b) { return (sf_cd){a.x + b.x, a.y + b.y}; }
static inline sf_cd sf_sub(sf_cd a, sf_cd b) { return (sf_cd){a.x - b.x, a.y - b.y}; }
static inline sf_cd sf_cmul(sf_cd a, sf_cd b) { return (sf_cd){fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x)}; }
static inline sf_cd sf_cmulc(sf_cd a, sf_cd b) { return (sf_cd){fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -(a.x * b.y))}; }
static inline sf_cd sf_cmac(sf_cd acc, sf_cd a, sf_cd b) {
  return (sf_cd){fma(-a.y, b.y, fma(a.x, b.x, acc.x)), fma(a.y, b.x, fma(a.x, b.y, acc.y))};
}
/* T[e] = e^{2 pi i e / M}, P[m] = e^{i pi m / N}: long-double cosl / sinl rounded once (make_sns_fft_const) */
static void sf_tables(sf_cd* T, sf_cd* P, uint32_t N) {
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int e = 0; e < SF_M; e++) {
    T[e] = (sf_cd){(double)cosl(2 * pi * e / SF_M), (double)sinl(2 * pi * e / SF_M)};
    P[e] = (sf_cd){(double)cosl(pi * e / (int)N), (double)sinl(pi * e / (int)N)};
  }
}
/* radix-4 DIF stage s over the whole array (positions in place), twiddles on the outputs */
static void sf_dif_stage(sf_cd* a, int s, const sf_cd* T) {
  const int lq = 8 - 2 * s, q = 1 << lq;
  for (int t = 0; t < SF_M / 4; t++) {
    const int j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j, e = j << (2 * s);
    sf_cd* x = a + base;
    const sf_cd x0 = x[0], x1 = x[q], x2 = x[2 * q], x3 = x[3 * q];
    const sf_cd a0 = sf_add(x0, x2), a1 = sf_sub(x0, x2), a2 = sf_add(x1, x3), d = sf_sub(x1, x3);
    const sf_cd a3 = {-d.y, d.x};
    x[0] = sf_add(a0, a2);
    x[q] = sf_cmul(sf_add(a1, a3), T[e]);
    x[2 * q] = sf_cmul(sf_sub(a0, a2), T[2 * e]);
    x[3 * q] = sf_cmul(sf_sub(a1, a3), T[3 * e]);
  }
}
/* its DIT inverse: conjugate twiddles on the inputs, then the butterfly with -i */
static void sf_dit_stage(sf_cd* a, int s, const sf_cd* T) {
  const int lq = 8 - 2 * s, q = 1 << lq;
  for (int t = 0; t < SF_M / 4; t++) {
    const int j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j, e = j << (2 * s);
    sf_cd* x = a + base;
    const sf_cd y0 = x[0], y1 = sf_cmulc(x[q], T[e]), y2 = sf_cmulc(x[2 * q], T[2 * e]), y3 = sf_cmulc(x[3 * q], T[3 * e]);
    const sf_cd b0 = sf_add(y0, y2), b1 = sf_sub(y0, y2), b2 = sf_add(y1, y3), d = sf_sub(y1, y3);
    const sf_cd b3 = {d.y, -d.x};
    x[0] = sf_add(b0, b2);
    x[q] = sf_add(b1, b3);
    x[2 * q] = sf_sub(b0, b2);
    x[3 * q] = sf_sub(b1, b3);
  }
}
/* N = 2048 integer coefficients -> spectrum: fold + twist by P, 5 DIF stages */
static void sf_forward(const double* v, sf_cd* z, const sf_cd* T, const sf_cd* P) {
  for (int m = 0; m < SF_M; m++) z[m] = sf_cmul((sf_cd){v[m], v[m + SF_M]}, P[m]);
  for (int s = 0; s < 5; s++) sf_dif_stage(z, s, T);
}
/* an integer-valued double (|v| < 2^127) as a word mod 2^128 (snsf::f64_int_to_w128) */
static u128 sf_to_w128(double v) {
  if (v < 0x1p62 && v > -0x1p62) return (u128)(__int128)(long long)v;
  uint64_t bits;
  memcpy(&bits, &v, 8);
  const int e = (int)((bits >> 52) & 0x7FF) - 1075;
  const u128 m = (u128)((bits & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull) << e;
  return (bits >> 63) ? (u128)0 - m : m;
}

/* Load-time rounding of the squashing key (the device's precision contract, tfhe_amd/csrc/sns.hip): every
 * coefficient, read as a signed 128-bit integer, is rounded to the nearest multiple of 2^16 (ties up).
 * The rounding error (< 2^15 per mask and body coefficient) adds ~2^20 of phase noise to a key whose own
 * noise is 2^30; the rounded key is 2^16 x a 112-bit integer: the five limbs above. */
void or_sns_bsk_round(const or_sns_params* sp, const uint64_t* bsk, uint64_t* out) {
  const size_t N = sp->N, planes = or_sns_bsk_len(sp) / (2 * N);
#pragma omp parallel for schedule(static)
  for (size_t pp = 0; pp < planes; pp++)
    for (size_t t = 0; t < N; t++) {
      /* the add wraps mod 2^128 (a word within 2^15 of 2^127 rounds to -2^127: the same torus point) */
      const __int128 rr = (__int128)(ld128(bsk + 2 * pp * N, N, t) + ((u128)1 << 15)) >> 16; /* floor: arithmetic shift */
      st128(out + 2 * pp * N, N, t, (u128)(rr * 65536));
    }
}

/* rounded key -> limb spectra: [i][r][j][t][N] words, t = limb 0..4.  Limb 0 (the balanced low 48 bits) is
 * stored as the device's f64 spectrum / M (1024 complex doubles, their bits in the N words); limbs 1..4 as
 * NTTs mod p1 of the signed 16-bit limb values. */
size_t or_sns_limb_ntt_len(const or_sns_params* sp) { return or_sns_bsk_len(sp) / 2 * OR_SNS_LIMBS; }
void or_sns_bsk_to_limb_ntt(const or_sns_params* sp, const uint64_t* rounded, uint64_t* out) {
  const size_t N = sp->N, planes = or_sns_bsk_len(sp) / (2 * N);
  sf_cd T[SF_M], P[SF_M];
  sf_tables(T, P, (uint32_t)N);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t pp = 0; pp < planes; pp++) {
    uint64_t* o = out + pp * OR_SNS_LIMBS * N;
    double* low = (double*)malloc(N * sizeof(double));
    sf_cd* z = (sf_cd*)malloc(SF_M * sizeof(sf_cd));
    for (size_t t = 0; t < N; t++) {
      __int128 rr = (__int128)ld128(rounded + 2 * pp * N, N, t) >> 16; /* exact: a multiple of 2^16 */
      for (int l = 0; l < OR_SNS_LIMBS; l++) {
        int64_t v;
        if (l == OR_SNS_LIMBS - 1) {
          v = (int64_t)rr; /* the top limb keeps the remainder (|.| <= 2^15) */
        } else {
          const int bits = l == 0 ? 48 : 16;
          const __int128 half = (__int128)1 << (bits - 1), mask = ((__int128)1 << bits) - 1;
          const __int128 lim = ((rr + half) & mask) - half;
          rr = (rr - lim) >> bits;
          v = (int64_t)lim;
        }
        if (l == 0) low[t] = (double)v; /* |v| <= 2^47: exact */
        else o[(size_t)l * N + t] = from_i64(v, SP[0]);
      }
    }
    sf_forward(low, z, T, P);
    for (int f = 0; f < SF_M; f++) {
      const double w[2] = {z[f].x * (1.0 / SF_M), z[f].y * (1.0 / SF_M)};
      memcpy(o + 2 * f, w, 16);
    }
    for (int l = 1; l < OR_SNS_LIMBS; l++) or_sns_ntt_fwd(0, o + (size_t)l * N, (uint32_t)N);
    free(low);
    free(z);
  }
}

/* identity LUT on msg_modulus values with one padding bit: delta = 2^127 / msg_modulus, half-box
 * rotation (the wrapped half negated); words [lo, hi][N] */
void or_sns_lut_identity(const or_sns_params* sp, uint32_t msg_modulus, uint64_t* lut) {
  const uint32_t N = sp->N, box = N / msg_modulus;
  const u128 delta = ((u128)1 << 127) / msg_modulus;
  for (uint32_t i = 0; i < N; i++) {
    const uint32_t src = i + box / 2;
    const u128 t = (u128)((src < N ? src : src - N) / box) * delta;
    st128(lut, N, i, src < N ? t : (u128)0 - t);
  }
}

/* one ciphertext: lwe_small (n+1, native 2^64) -> acc [(k+1)][lo, hi][N] */
void or_sns_blind_rotate(const or_sns_params* sp, const uint64_t* bsk_limb, const uint64_t* lwe, const uint64_t* lut,
                         uint64_t* acc) {
  const uint32_t k = sp->k, N = sp->N, L = sp->level, twoN = 2 * N, R = (k + 1) * L;
  const uint64_t p = SP[0];
  const size_t poly = (size_t)2 * N; /* both words */
  u128* a = (u128*)malloc((size_t)(k + 1) * N * sizeof(u128));
  u128* rot = (u128*)malloc((size_t)N * sizeof(u128));
  uint64_t* dig = (uint64_t*)malloc((size_t)R * N * 8);
  uint64_t* s = (uint64_t*)malloc((size_t)N * 8);
  double* dv = (double*)malloc((size_t)N * sizeof(double));
  sf_cd* Df = (sf_cd*)malloc((size_t)R * SF_M * sizeof(sf_cd)); /* the low limb's digit spectra (f64) */
  sf_cd* z = (sf_cd*)malloc(SF_M * sizeof(sf_cd));
  sf_cd T[SF_M], P[SF_M];
  sf_tables(T, P, N);
  int64_t d[8];
  /* acc = X^{-b~} * (0, .., 0, lut) */
  memset(a, 0, (size_t)(k + 1) * N * sizeof(u128));
  const uint32_t bt = or_mod_switch(lwe[sp->n], twoN);
  const uint32_t sh = (twoN - bt) % twoN;
  for (uint32_t t = 0; t < N; t++) {
    uint32_t dst = t + sh;
    int neg = 0;
    if (dst >= twoN) dst -= twoN;
    if (dst >= N) { dst -= N; neg = 1; }
    const u128 v = ld128(lut, N, t);
    a[(size_t)k * N + dst] = neg ? (u128)0 - v : v;
  }
  const size_t bsk_i = (size_t)R * (k + 1) * OR_SNS_LIMBS * N;
  for (uint32_t i = 0; i < sp->n; i++) {
    const uint32_t ai = or_mod_switch(lwe[i], twoN);
    if (!ai) continue; /* zero digits: every product is an exact zero, on the device too */
    /* digits of X^{ai} acc_c - acc_c: NTT mod p (limbs 1..4) and the device's f64 spectrum (limb 0) */
    for (uint32_t c = 0; c <= k; c++) {
      const u128* ac = a + (size_t)c * N;
      for (uint32_t t = 0; t < N; t++) {
        uint32_t dst = t + ai;
        int neg = 0;
        if (dst >= twoN) dst -= twoN;
        if (dst >= N) { dst -= N; neg = 1; }
        rot[dst] = neg ? (u128)0 - ac[t] : ac[t];
      }
      for (uint32_t t = 0; t < N; t++) {
        decompose128(rot[t] - ac[t], sp->base_log, L, d);
        for (uint32_t l = 0; l < L; l++) dig[(size_t)(c * L + l) * N + t] = from_i64(d[l], p);
      }
    }
    for (uint32_t r = 0; r < R; r++) {
      for (uint32_t t = 0; t < N; t++) {
        const uint64_t w = dig[(size_t)r * N + t];
        dv[t] = w > p / 2 ? -(double)(p - w) : (double)w;
      }
      sf_forward(dv, Df + (size_t)r * SF_M, T, P);
      or_sns_ntt_fwd(0, dig + (size_t)r * N, N);
    }
    const uint64_t* bi = bsk_limb + bsk_i * i;
    for (uint32_t j = 0; j <= k; j++) {
      u128* aj = a + (size_t)j * N;
      /* limbs 1..4: acc_j += 2^(64 + 16 (l - 1)) * (sum_r d_r (*) l_(r, j, l)), exact */
      for (int l = 1; l < OR_SNS_LIMBS; l++) {
        for (uint32_t t = 0; t < N; t++) {
          uint64_t acc_t = 0;
          for (uint32_t r = 0; r < R; r++)
            acc_t = madd(acc_t, mmul(dig[(size_t)r * N + t], bi[(((size_t)r * (k + 1) + j) * OR_SNS_LIMBS + l) * N + t], p), p);
          s[t] = acc_t;
        }
        or_sns_ntt_inv(0, s, N);
        const int shift = 64 + 16 * (l - 1);
        for (uint32_t t = 0; t < N; t++) {
          const __int128 v = s[t] > p / 2 ? -(__int128)(p - s[t]) : (__int128)s[t]; /* exact: |value| < 2^53 */
          aj[t] += (u128)v << shift;
        }
      }
      /* limb 0, the device's f64 order: 9-term MAC from zero, 5 DIT stages, untwist, rint; acc_j += v << 16 */
      for (int f = 0; f < SF_M; f++) {
        sf_cd o = {0.0, 0.0};
        for (uint32_t r = 0; r < R; r++) {
          sf_cd kk;
          memcpy(&kk, bi + (((size_t)r * (k + 1) + j) * OR_SNS_LIMBS) * N + 2 * f, 16);
          o = sf_cmac(o, Df[(size_t)r * SF_M + f], kk);
        }
        z[f] = o;
      }
      for (int st = 4; st >= 0; st--) sf_dit_stage(z, st, T);
      for (int m = 0; m < SF_M; m++) {
        const sf_cd y = sf_cmulc(z[m], P[m]);
        aj[m] += sf_to_w128(rint(y.x)) << 16;
        aj[m + SF_M] += sf_to_w128(rint(y.y)) << 16;
      }
    }
  }
  for (uint32_t j = 0; j <= k; j++)
    for (uint32_t t = 0; t < N; t++) st128(acc + (size_t)j * poly, N, t, a[(size_t)j * N + t]);
  free(a); free(rot); free(dig); free(s); free(dv); free(Df); free(z);
}

/* acc -> LWE over Z_2^128, dim k*N (+ body): (lo, hi) pairs; a'_(cN) = A_c[0], a'_(cN + t) = -A_c[N - t] */
void or_sns_sample_extract(const or_sns_params* sp, const uint64_t* acc, uint64_t* out) {
  const uint32_t k = sp->k, N = sp->N;
  const size_t poly = (size_t)2 * N;
  for (uint32_t c = 0; c < k; c++)
    for (uint32_t t = 0; t < N; t++) {
      const u128 v = ld128(acc + (size_t)c * poly, N, t == 0 ? 0 : N - t);
      const u128 y = t == 0 ? v : (u128)0 - v;
      out[2 * ((size_t)c * N + t)] = (uint64_t)y;
      out[2 * ((size_t)c * N + t) + 1] = (uint64_t)(y >> 64);
    }
  const u128 b = ld128(acc + (size_t)k * poly, N, 0);
  out[2 * ((size_t)k * N)] = (uint64_t)b;
  out[2 * ((size_t)k * N) + 1] = (uint64_t)(b >> 64);
}

void or_sns_squash(const or_sns_params* sp, const uint64_t* bsk_limb, const uint64_t* lwe_small, size_t B,
                   uint32_t msg_modulus, uint64_t* out, int threads) {
  const size_t acc_len = (size_t)(sp->k + 1) * 2 * sp->N, out_len = 2 * ((size_t)sp->k * sp->N + 1);
  uint64_t* lut = (uint64_t*)malloc((size_t)2 * sp->N * 8);
  or_sns_lut_identity(sp, msg_modulus, lut);
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 16)
  for (size_t q = 0; q < B; q++) {
    uint64_t* acc = (uint64_t*)malloc(acc_len * 8);
    or_sns_blind_rotate(sp, bsk_limb, lwe_small + q * (sp->n + 1), lut, acc);
    or_sns_sample_extract(sp, acc, out + q * out_len);
    free(acc);
  }
  free(lut);
}

/* phase b - <a, s> mod 2^128 of count LWE128s (dim = k*N) -> (lo, hi) pairs */
void or_sns_phase(const or_sns_params* sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count,
                  uint64_t* out) {
  const size_t dim = (size_t)sp->k * sp->N;
  for (size_t q = 0; q < count; q++) {
    const uint64_t* c = cts + q * 2 * (dim + 1);
    u128 s = 0;
    for (size_t i = 0; i < dim; i++)
      if (glwe_key[i]) s += ((u128)c[2 * i + 1] << 64) | c[2 * i];
    const u128 ph = (((u128)c[2 * dim + 1] << 64) | c[2 * dim]) - s;
    out[2 * q] = (uint64_t)ph;
    out[2 * q + 1] = (uint64_t)(ph >> 64);
  }
}
