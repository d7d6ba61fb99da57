/*
 * tfhe_oracle.c — CPU restatement of the TFHE PBS path.  TEST INFRASTRUCTURE ONLY
 * (see tfhe_oracle.h for scope, the reference file:line each piece follows, and the
 * "parity unpinned" statement).  Plain C11, no dependencies beyond libm / OpenMP.
 */
#include "tfhe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;
#define EPS 0xFFFFFFFFull

/* ======================================================================================
 * Parameters.  P-GATE = CGGI / TFHE-lib default gate set (literature constants; BASELINE.json
 * names "TFHE 128-bit default (N=1024)").  P-FHEVM = PARAM_MESSAGE_2_CARRY_2_KS_PBS_TUNIFORM_2M128
 * decoded from sdk/relayer/src/test/keys/privateKey.bin (selected by name at
 * sdk/relayer/src/tfhe.ts:14-19).  The oracle models TUniform noise of P-FHEVM with a Gaussian
 * of the same order (noise values are not part of any pinned vector).
 * ==================================================================================== */
int or_params_preset(int preset, or_params* o) {
  memset(o, 0, sizeof(*o));
  if (preset == 0) {
    o->n = 630; o->k = 1; o->N = 1024;
    o->pbs_base_log = 7; o->pbs_level = 3;
    o->ks_base_log = 2; o->ks_level = 8;
    o->lwe_noise_log2 = -15; o->glwe_noise_log2 = -25;
    o->order = 0;
    return 0;
  }
  if (preset == 2) { /* P-GATE, FFT64 transform (native torus BSK) */
    or_params_preset(0, o);
    o->transform = 1;
    return 0;
  }
  if (preset == 3) { /* P-FHEVM, FFT64 transform (native torus BSK, N = 2048 as two 512-point halves) */
    or_params_preset(1, o);
    o->transform = 1;
    return 0;
  }
  if (preset == 1) {
    o->n = 918; o->k = 1; o->N = 2048;
    o->pbs_base_log = 23; o->pbs_level = 1;
    o->ks_base_log = 4; o->ks_level = 4;
    o->lwe_noise_log2 = -19; o->glwe_noise_log2 = -47;
    o->order = 1;
    return 0;
  }
  return -1;
}

/* ======================================================================================
 * ChaCha20 block function (RFC 8439 §2.3).  Key = seed(8B LE) | stream(8B LE) | "tfhe-amd chacha!"
 * nonce = 0, 32-bit block counter from 0.  Each block yields 8 u64 (little-endian word pairs).
 * ==================================================================================== */
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define QR(a, b, c, d)                 \
  a += b; d ^= a; d = rotl32(d, 16);   \
  c += d; b ^= c; b = rotl32(b, 12);   \
  a += b; d ^= a; d = rotl32(d, 8);    \
  c += d; b ^= c; b = rotl32(b, 7);

static void chacha_block(const uint32_t key[8], uint32_t ctr, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    ctr, 0, 0, 0};
  uint32_t x[16];
  memcpy(x, s, sizeof(x));
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

void or_rng_init(or_rng* r, uint64_t seed, uint64_t stream) {
  static const char tag[16] = {'t', 'f', 'h', 'e', '-', 'a', 'm', 'd', ' ', 'c', 'h', 'a', 'c', 'h', 'a', '!'};
  r->key[0] = (uint32_t)seed; r->key[1] = (uint32_t)(seed >> 32);
  r->key[2] = (uint32_t)stream; r->key[3] = (uint32_t)(stream >> 32);
  for (int i = 0; i < 4; i++)
    r->key[4 + i] = (uint32_t)(uint8_t)tag[4 * i] | (uint32_t)(uint8_t)tag[4 * i + 1] << 8 |
                    (uint32_t)(uint8_t)tag[4 * i + 2] << 16 | (uint32_t)(uint8_t)tag[4 * i + 3] << 24;
  r->ctr = 0;
  r->pos = 16;
}

uint64_t or_rng_u64(or_rng* r) {
  if (r->pos >= 16) { chacha_block(r->key, r->ctr++, r->buf); r->pos = 0; }
  uint64_t v = (uint64_t)r->buf[r->pos] | ((uint64_t)r->buf[r->pos + 1] << 32);
  r->pos += 2;
  return v;
}

uint64_t or_rng_mod_p(or_rng* r) {
  for (;;) { uint64_t x = or_rng_u64(r); if (x < OR_P) return x; }
}

/* Box-Muller, cosine branch only.  u1 in (0,1], u2 in [0,1) from the top 53 bits.
 * log and cos are evaluated with fixed series in plain IEEE double arithmetic (+ - * / sqrt,
 * no FMA contraction, no libm), so the sampled noise -- and therefore every key and ciphertext --
 * is bit-identical on any IEEE-754 host. */
static double det_log(double u) { /* u in (0, 1] */
  int ex;
  double m = frexp(u, &ex); /* u = m * 2^ex, m in [0.5, 1) */
  if (m < 0.70710678118654752) { m *= 2.0; ex -= 1; }
  double s = (m - 1.0) / (m + 1.0), s2 = s * s, term = s, sum = 0.0;
  for (int i = 1; i <= 23; i += 2) { sum += term / (double)i; term *= s2; }
  return (double)ex * 6.93147180369123816490e-01 + ((double)ex * 1.90821492927058770002e-10 + 2.0 * sum);
}
static double det_sin_series(double x) { /* |x| <= pi/4 */
  double x2 = x * x, term = x, sum = 0.0;
  for (int i = 1; i <= 21; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static double det_cos_series(double x) {
  double x2 = x * x, term = 1.0, sum = 0.0;
  for (int i = 0; i <= 20; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static double det_cos2pi(double u) { /* u in [0, 1) */
  const double two_pi = 6.28318530717958647692;
  double v = u <= 0.5 ? u : 1.0 - u, sign = 1.0;
  if (v > 0.25) { sign = -1.0; v = 0.5 - v; }
  if (v > 0.125) return sign * det_sin_series(two_pi * (0.25 - v));
  return sign * det_cos_series(two_pi * v);
}

int64_t or_rng_gauss(or_rng* r, int32_t log2_sigma) {
  double u1 = (double)((or_rng_u64(r) >> 11) + 1) * 0x1.0p-53;
  double u2 = (double)(or_rng_u64(r) >> 11) * 0x1.0p-53;
  double z = sqrt(-2.0 * det_log(u1)) * det_cos2pi(u2);
  return (int64_t)llrint(ldexp(z, 64 + log2_sigma));
}

/* ======================================================================================
 * Z_p arithmetic, p = 2^64 - 2^32 + 1.  All results canonical in [0, p).
 * ==================================================================================== */
uint64_t or_add(uint64_t a, uint64_t b) {
  uint64_t s = a + b, t = s + EPS; /* s - p == s + EPS (mod 2^64) */
  return (s < a || s >= OR_P) ? t : s;
}
uint64_t or_sub(uint64_t a, uint64_t b) {
  uint64_t d = a - b;
  return a < b ? d + OR_P : d;
}
/* 128-bit product reduced with 2^64 == 2^32 - 1 and 2^96 == -1 (mod p). */
uint64_t or_mul(uint64_t a, uint64_t b) {
  u128 x = (u128)a * b;
  uint64_t lo = (uint64_t)x, hi = (uint64_t)(x >> 64);
  uint64_t hh = hi >> 32, hl = hi & EPS;
  uint64_t t0 = lo - hh;
  t0 = lo < hh ? t0 - EPS : t0;
  uint64_t t1 = (hl << 32) - hl;
  uint64_t t2 = t0 + t1;
  t2 = t2 < t1 ? t2 + EPS : t2;
  return t2 >= OR_P ? t2 - OR_P : t2;
}
uint64_t or_pow(uint64_t a, uint64_t e) {
  uint64_t r = 1;
  while (e) { if (e & 1) r = or_mul(r, a); a = or_mul(a, a); e >>= 1; }
  return r;
}
static uint64_t or_neg(uint64_t a) { return a ? OR_P - a : 0; }
static uint64_t or_from_i64(int64_t v) {
  if (v >= 0) return (uint64_t)v;
  return or_neg((0ull - (uint64_t)v) % OR_P);
}

uint64_t or_psi(uint32_t N) {
  /* generator 7; w = 7^((p-1)/2N); choose w^m with (w^m)^(2N/64) == 8 (needs 2N >= 64). */
  uint64_t w = or_pow(7, (OR_P - 1) / (2ull * N));
  uint64_t r = or_pow(w, 2ull * N / 64);
  uint64_t k = 0, t = 1;
  for (k = 0; k < 64; k++) { if (t == r) break; t = or_mul(t, 8); }
  uint64_t m = 1;
  while ((k * m) % 64 != 1) m += 2;
  return or_pow(w, m);
}

uint64_t or_tor_to_p(uint64_t v) { return v - ((v >> 32) + ((v >> 31) & 1)); }
uint64_t or_p_to_tor(uint64_t x) { return x + ((x + 0x80000000ull) >> 32); }

/* ======================================================================================
 * Polynomials mod X^N + 1 over Z_p.
 * The schoolbook product is the obviously-correct arbiter (computations.rs:50-54 semantics:
 * polynomial_wrapping_mul, here over Z_p instead of Z_2^64).
 * ==================================================================================== */
void or_poly_mul_schoolbook(uint64_t* out, const uint64_t* a, const uint64_t* b, uint32_t N) {
  uint64_t* t = (uint64_t*)calloc(N, 8);
  for (uint32_t i = 0; i < N; i++) {
    if (!a[i]) continue;
    for (uint32_t j = 0; j < N; j++) {
      uint64_t pr = or_mul(a[i], b[j]);
      uint32_t d = i + j;
      if (d < N) t[d] = or_add(t[d], pr);
      else t[d - N] = or_sub(t[d - N], pr);
    }
  }
  memcpy(out, t, (size_t)N * 8);
  free(t);
}

static uint32_t bitrev(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
  return r;
}

/* Textbook negacyclic NTT: twist by psi^i, cyclic radix-2 DIT NTT with omega = psi^2
 * (bit-reverse permutation first), natural output A[j] = a(psi^(2j+1)).
 * Tables are cached per N (sizes 2^5 .. 2^16). */
typedef struct ntt_tab {
  uint32_t N;
  uint64_t *twist, *untwist; /* psi^i ; psi^-i * N^-1 */
  uint64_t *wf, *wi;         /* per-stage roots, concatenated: stage len uses [len/2 - 1 + j] */
  uint32_t* rev;
} ntt_tab;
static ntt_tab g_tabs[17];

static const ntt_tab* get_tab(uint32_t N) {
  int lg = 0;
  while ((1u << lg) < N) lg++;
  ntt_tab* t = &g_tabs[lg];
  if (__atomic_load_n(&t->N, __ATOMIC_ACQUIRE) == N) return t;
#pragma omp critical(or_ntt_tab)
  {
    if (t->N != N) {
      uint64_t psi = or_psi(N), psi_inv = or_pow(psi, OR_P - 2), ninv = or_pow(N, OR_P - 2);
      t->twist = (uint64_t*)malloc((size_t)N * 8);
      t->untwist = (uint64_t*)malloc((size_t)N * 8);
      t->wf = (uint64_t*)malloc((size_t)N * 8);
      t->wi = (uint64_t*)malloc((size_t)N * 8);
      t->rev = (uint32_t*)malloc((size_t)N * 4);
      uint64_t a = 1, b = ninv;
      for (uint32_t i = 0; i < N; i++) {
        t->twist[i] = a; t->untwist[i] = b;
        a = or_mul(a, psi); b = or_mul(b, psi_inv);
        t->rev[i] = bitrev(i, lg);
      }
      uint64_t om = or_mul(psi, psi), omi = or_mul(psi_inv, psi_inv);
      for (uint32_t len = 2; len <= N; len <<= 1) {
        uint64_t wl = or_pow(om, N / len), wli = or_pow(omi, N / len), w = 1, wi = 1;
        for (uint32_t j = 0; j < len / 2; j++) {
          t->wf[len / 2 - 1 + j] = w; t->wi[len / 2 - 1 + j] = wi;
          w = or_mul(w, wl); wi = or_mul(wi, wli);
        }
      }
      __atomic_store_n(&t->N, N, __ATOMIC_RELEASE);
    }
  }
  return t;
}

static void cyclic_ntt(uint64_t* a, uint32_t N, const uint32_t* rev, const uint64_t* roots) {
  for (uint32_t i = 0; i < N; i++) {
    uint32_t j = rev[i];
    if (j > i) { uint64_t t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  for (uint32_t len = 2; len <= N; len <<= 1) {
    const uint64_t* w = roots + len / 2 - 1;
    for (uint32_t s = 0; s < N; s += len)
      for (uint32_t j = 0; j < len / 2; j++) {
        uint64_t u = a[s + j], v = or_mul(a[s + j + len / 2], w[j]);
        a[s + j] = or_add(u, v);
        a[s + j + len / 2] = or_sub(u, v);
      }
  }
}

void or_ntt_fwd(uint64_t* a, uint32_t N) {
  const ntt_tab* t = get_tab(N);
  for (uint32_t i = 0; i < N; i++) a[i] = or_mul(a[i], t->twist[i]);
  cyclic_ntt(a, N, t->rev, t->wf);
}

void or_ntt_inv(uint64_t* a, uint32_t N) {
  const ntt_tab* t = get_tab(N);
  cyclic_ntt(a, N, t->rev, t->wi);
  for (uint32_t i = 0; i < N; i++) a[i] = or_mul(a[i], t->untwist[i]);
}

void or_poly_mul_ntt(uint64_t* out, const uint64_t* a, const uint64_t* b, uint32_t N) {
  uint64_t* x = (uint64_t*)malloc((size_t)N * 8);
  uint64_t* y = (uint64_t*)malloc((size_t)N * 8);
  memcpy(x, a, (size_t)N * 8); memcpy(y, b, (size_t)N * 8);
  or_ntt_fwd(x, N); or_ntt_fwd(y, N);
  for (uint32_t i = 0; i < N; i++) x[i] = or_mul(x[i], y[i]);
  or_ntt_inv(x, N);
  memcpy(out, x, (size_t)N * 8);
  free(x); free(y);
}

void or_poly_monomial_mul(uint64_t* out, const uint64_t* in, uint32_t N, uint32_t t) {
  t %= 2 * N;
  for (uint32_t i = 0; i < N; i++) {
    uint32_t d = i + t; /* in[i] * X^t lands at i+t, negated per wrap past N */
    int neg = 0;
    if (d >= N) { d -= N; neg ^= 1; }
    if (d >= N) { d -= N; neg ^= 1; }
    out[d] = neg ? or_neg(in[i]) : in[i];
  }
}

/* ======================================================================================
 * Decomposition — tfhe-rs SignedDecomposer semantics (encryption.rs:152-166,191-201 use
 * SignedDecomposer::new + closest_representable):
 *   closest_representable: round to the top base_log*level bits, ties up.
 *   balanced digits, least significant first, with the tie-to-next-digit carry rule
 *   carry = (((res - 1) | state) & res) >> (base_log - 1).
 * ==================================================================================== */
void or_decompose(uint64_t x, uint32_t base_log, uint32_t level, int64_t* digits) {
  uint32_t prec = base_log * level;
  uint32_t nonrep = 64 - prec;
  uint64_t state = (x >> (nonrep - 1)) + 1; /* round at bit nonrep-1 */
  state >>= 1;
  if (prec < 64) state &= ((1ull << prec) - 1);
  uint64_t B = 1ull << base_log, mask = B - 1;
  for (int l = (int)level - 1; l >= 0; l--) {
    uint64_t res = state & mask;
    state >>= base_log;
    uint64_t carry = (((res - 1) | state) & res) >> (base_log - 1);
    carry &= 1;
    state += carry;
    digits[l] = (int64_t)res - (int64_t)(carry << base_log);
  }
}

uint32_t or_mod_switch(uint64_t x, uint32_t two_n) {
  int lg = 0;
  while ((1u << lg) < two_n) lg++;
  uint64_t v = ((x >> (64 - lg - 1)) + 1) >> 1;
  return (uint32_t)(v & (two_n - 1));
}

/* ======================================================================================
 * Sizes and key generation.
 * BSK_i = GGSW_S(s_i): row (c, lvl) (c = component receiving the message: c<k mask, c==k body)
 *   = GLWE_S(0) + s_i * g_lvl added to component c coefficient 0, g_lvl = 2^(64 - beta*(lvl+1)).
 * KSK[j][r] = LWE_s(s'_j * 2^(64 - gamma*(r+1))).
 * PRNG streams: LWE key 1, GLWE key 2, BSK_i 0x1000+i, KSK_j 0x100000+j.
 * ==================================================================================== */
size_t or_bsk_len(const or_params* p) {
  return (size_t)p->n * (p->k + 1) * p->pbs_level * (p->k + 1) * p->N;
}
size_t or_ksk_len(const or_params* p) {
  return (size_t)p->k * p->N * p->ks_level * (p->n + 1);
}

static void glwe_encrypt_zero_p(const or_params* p, const uint64_t* glwe_key, or_rng* r, uint64_t* out) {
  const uint32_t N = p->N, k = p->k;
  uint64_t* body = out + (size_t)k * N;
  for (uint32_t c = 0; c < k; c++)
    for (uint32_t i = 0; i < N; i++) out[(size_t)c * N + i] = or_rng_mod_p(r);
  for (uint32_t i = 0; i < N; i++) body[i] = or_from_i64(or_rng_gauss(r, p->glwe_noise_log2));
  /* body += sum_c A_c * S_c, S binary: add rotated copies (exact, no product needed) */
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = out + (size_t)c * N;
    const uint64_t* S = glwe_key + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!S[j]) continue;
      for (uint32_t i = 0; i < N; i++) {
        uint32_t d = i + j;
        if (d < N) body[d] = or_add(body[d], A[i]);
        else body[d - N] = or_sub(body[d - N], A[i]);
      }
    }
  }
}

static void glwe_encrypt_native(uint32_t k, uint32_t N, const uint64_t* key, int32_t noise_log2, or_rng* r,
                                const uint64_t* m, uint64_t* out);

static void lwe_encrypt_one(uint32_t dim, const uint64_t* key, int32_t noise_log2, or_rng* r, uint64_t m,
                            uint64_t* out) {
  uint64_t b = 0;
  for (uint32_t i = 0; i < dim; i++) {
    out[i] = or_rng_u64(r);
    b += out[i] * key[i];
  }
  b += (uint64_t)or_rng_gauss(r, noise_log2);
  out[dim] = b + m;
}

void or_keygen(const or_params* p, uint64_t seed, uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk,
               uint64_t* ksk) {
  or_rng r;
  or_rng_init(&r, seed, 1);
  for (uint32_t i = 0; i < p->n; i++) lwe_key[i] = or_rng_u64(&r) & 1;
  or_rng_init(&r, seed, 2);
  for (uint32_t i = 0; i < p->k * p->N; i++) glwe_key[i] = or_rng_u64(&r) & 1;
  or_server_keygen(p, seed, lwe_key, glwe_key, bsk, ksk);
}

/* server keys for given binary secret keys (ingested tfhe-rs ClientKey; same streams as or_keygen) */
void or_server_keygen(const or_params* p, uint64_t seed, const uint64_t* lwe_key, const uint64_t* glwe_key,
                      uint64_t* bsk, uint64_t* ksk) {
  const uint32_t n = p->n, k = p->k, N = p->N, L = p->pbs_level;
  if (bsk) {
    const size_t row = (size_t)(k + 1) * N, per_i = (size_t)(k + 1) * L * row;
#pragma omp parallel for schedule(dynamic, 4)
    for (uint32_t i = 0; i < n; i++) {
      or_rng rr;
      or_rng_init(&rr, seed, 0x1000 + i);
      for (uint32_t c = 0; c <= k; c++)
        for (uint32_t l = 0; l < L; l++) {
          uint64_t* out = bsk + per_i * i + row * (c * L + l);
          uint64_t g = 1ull << (64 - p->pbs_base_log * (l + 1));
          if (p->transform == 1) { /* native torus GGSW (FFT64) */
            glwe_encrypt_native(k, N, glwe_key, p->glwe_noise_log2, &rr, NULL, out);
            if (lwe_key[i]) out[(size_t)c * N] += g;
          } else {
            glwe_encrypt_zero_p(p, glwe_key, &rr, out);
            if (lwe_key[i]) out[(size_t)c * N] = or_add(out[(size_t)c * N], g);
          }
        }
    }
  }
  if (ksk) {
    const size_t per_j = (size_t)p->ks_level * (n + 1);
#pragma omp parallel for schedule(dynamic, 16)
    for (uint32_t j = 0; j < k * N; j++) {
      or_rng rr;
      or_rng_init(&rr, seed, 0x100000 + j);
      for (uint32_t l = 0; l < p->ks_level; l++) {
        uint64_t m = glwe_key[j] << (64 - p->ks_base_log * (l + 1));
        lwe_encrypt_one(n, lwe_key, p->lwe_noise_log2, &rr, m, ksk + per_j * j + (size_t)l * (n + 1));
      }
    }
  }
}

void or_lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, uint64_t seed, uint64_t stream0,
                    const uint64_t* msgs, size_t count, uint64_t* out) {
#pragma omp parallel for schedule(static) if (count > 64)
  for (size_t q = 0; q < count; q++) {
    or_rng r;
    or_rng_init(&r, seed, stream0 + q);
    lwe_encrypt_one(dim, key, noise_log2, &r, msgs[q], out + q * (dim + 1));
  }
}

void or_lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out) {
  for (size_t q = 0; q < count; q++) {
    const uint64_t* c = ct + q * (dim + 1);
    uint64_t s = 0;
    for (uint32_t i = 0; i < dim; i++) s += c[i] * key[i];
    out[q] = c[dim] - s;
  }
}

/* ======================================================================================
 * Blind rotation (CMUX loop), sample extraction, keyswitch.
 * ==================================================================================== */
void or_bsk_to_ntt(const or_params* p, const uint64_t* bsk, uint64_t* bsk_ntt) {
  const size_t polys = or_bsk_len(p) / p->N;
#pragma omp parallel for schedule(static)
  for (size_t q = 0; q < polys; q++) {
    memcpy(bsk_ntt + q * p->N, bsk + q * p->N, (size_t)p->N * 8);
    or_ntt_fwd(bsk_ntt + q * p->N, p->N);
  }
}

/* acc <- acc + ExtProd(BSK_i, (X^a - 1) * acc) */
static void cmux_step(const or_params* p, const uint64_t* bsk_i, int schoolbook, uint32_t a, uint64_t* acc,
                      uint64_t* tmp, uint64_t* dig, uint64_t* sum, uint64_t* prod) {
  const uint32_t N = p->N, k = p->k, L = p->pbs_level;
  const size_t row = (size_t)(k + 1) * N;
  for (uint32_t c = 0; c <= k; c++) {
    or_poly_monomial_mul(tmp + (size_t)c * N, acc + (size_t)c * N, N, a);
    for (uint32_t i = 0; i < N; i++) tmp[(size_t)c * N + i] = or_sub(tmp[(size_t)c * N + i], acc[(size_t)c * N + i]);
  }
  memset(sum, 0, row * 8);
  int64_t d[64];
  for (uint32_t c = 0; c <= k; c++) {
    /* digit polynomials for every level of component c */
    for (uint32_t i = 0; i < N; i++) {
      or_decompose(tmp[(size_t)c * N + i], p->pbs_base_log, L, d);
      for (uint32_t l = 0; l < L; l++) dig[(size_t)l * N + i] = or_from_i64(d[l]);
    }
    for (uint32_t l = 0; l < L; l++) {
      uint64_t* D = dig + (size_t)l * N;
      const uint64_t* rowp = bsk_i + row * (c * L + l);
      if (!schoolbook) {
        or_ntt_fwd(D, N);
        for (uint32_t j = 0; j <= k; j++)
          for (uint32_t i = 0; i < N; i++)
            sum[(size_t)j * N + i] = or_add(sum[(size_t)j * N + i], or_mul(D[i], rowp[(size_t)j * N + i]));
      } else {
        for (uint32_t j = 0; j <= k; j++) {
          or_poly_mul_schoolbook(prod, D, rowp + (size_t)j * N, N);
          for (uint32_t i = 0; i < N; i++) sum[(size_t)j * N + i] = or_add(sum[(size_t)j * N + i], prod[i]);
        }
      }
    }
  }
  for (uint32_t j = 0; j <= k; j++) {
    if (!schoolbook) or_ntt_inv(sum + (size_t)j * N, N);
    for (uint32_t i = 0; i < N; i++) acc[(size_t)j * N + i] = or_add(acc[(size_t)j * N + i], sum[(size_t)j * N + i]);
  }
}

void or_blind_rotate(const or_params* p, const uint64_t* bsk_any, int use_schoolbook, const uint64_t* lwe_in,
                     const uint64_t* lut, uint64_t* acc) {
  const uint32_t N = p->N, k = p->k, L = p->pbs_level, n = p->n;
  const size_t row = (size_t)(k + 1) * N, per_i = (size_t)(k + 1) * L * row;
  memset(acc, 0, row * 8);
  uint32_t bt = or_mod_switch(lwe_in[n], 2 * N);
  or_poly_monomial_mul(acc + (size_t)k * N, lut, N, (2 * N - bt) % (2 * N)); /* X^{-b~} * v */
  uint64_t* tmp = (uint64_t*)malloc(row * 8);
  uint64_t* dig = (uint64_t*)malloc((size_t)L * N * 8);
  uint64_t* sum = (uint64_t*)malloc(row * 8);
  uint64_t* prod = (uint64_t*)malloc((size_t)N * 8);
  for (uint32_t i = 0; i < n; i++) {
    uint32_t a = or_mod_switch(lwe_in[i], 2 * N);
    if (a == 0) continue; /* (X^0 - 1) acc == 0: the external product is exactly zero */
    cmux_step(p, bsk_any + per_i * i, use_schoolbook, a, acc, tmp, dig, sum, prod);
  }
  free(tmp); free(dig); free(sum); free(prod);
}

void or_sample_extract(const or_params* p, const uint64_t* acc, uint64_t* out) {
  const uint32_t N = p->N, k = p->k;
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = acc + (size_t)c * N;
    out[(size_t)c * N] = or_p_to_tor(A[0]);
    for (uint32_t j = 1; j < N; j++) out[(size_t)c * N + j] = or_p_to_tor(or_neg(A[N - j]));
  }
  out[(size_t)k * N] = or_p_to_tor(acc[(size_t)k * N]);
}

void or_keyswitch(const or_params* p, const uint64_t* ksk, const uint64_t* in, uint64_t* out) {
  const uint32_t n = p->n, big = p->k * p->N, L = p->ks_level;
  memset(out, 0, (size_t)(n + 1) * 8);
  out[n] = in[big];
  int64_t d[64];
  for (uint32_t j = 0; j < big; j++) {
    or_decompose(in[j], p->ks_base_log, L, d);
    for (uint32_t l = 0; l < L; l++) {
      if (!d[l]) continue;
      const uint64_t* kr = ksk + ((size_t)j * L + l) * (n + 1);
      uint64_t m = (uint64_t)d[l];
      for (uint32_t c = 0; c <= n; c++) out[c] -= m * kr[c];
    }
  }
}

/* ======================================================================================
 * Modulus-switch noise reduction (header: or_ms_key).
 * ==================================================================================== */
void or_ms_zeros_keygen(const or_params* p, uint64_t seed, const uint64_t* lwe_key, uint32_t count,
                        uint64_t* zeros) {
#pragma omp parallel for schedule(static)
  for (uint32_t z = 0; z < count; z++) {
    or_rng rr;
    or_rng_init(&rr, seed, 0x200000 + z);
    lwe_encrypt_one(p->n, lwe_key, p->lwe_noise_log2, &rr, 0, zeros + (size_t)z * (p->n + 1));
  }
}

static uint32_t log2u(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) l++;
  return l;
}

/* signed error of the switch to 2N (tfhe-rs modulus_switch: ((x >> (s-1)) + 1) >> 1) */
static inline int64_t ms_err(uint64_t x, uint32_t shift) {
  uint64_t r = ((x >> (shift - 1)) + 1) >> 1;
  return (int64_t)((r << shift) - x);
}

static double ms_measure_sums(const or_ms_key* ms, int64_t s1, unsigned __int128 s2, int64_t eb) {
  const double mean = (double)(2 * eb - s1) * 0.5;
  const double sq = (double)(uint64_t)(s2 >> 64) * 0x1p64 + (double)(uint64_t)s2;
  const double var = sq * 0.25 + ms->input_variance * 0x1p128;
  const double sd = sqrt(var);
  const double dev = ms->r_sigma * sd;
  return fabs(mean) + dev;
}

double or_ms_measure(const or_params* p, const or_ms_key* ms, const uint64_t* ct, const uint64_t* zero) {
  const uint32_t shift = 64 - log2u(2 * p->N);
  int64_t s1 = 0;
  unsigned __int128 s2 = 0;
  for (uint32_t i = 0; i < p->n; i++) {
    const int64_t e = ms_err(ct[i] + (zero ? zero[i] : 0), shift);
    s1 += e;
    s2 += (unsigned __int128)((__int128)e * e);
  }
  const int64_t eb = ms_err(ct[p->n] + (zero ? zero[p->n] : 0), shift);
  return ms_measure_sums(ms, s1, s2, eb);
}

int or_ms_reduce(const or_params* p, const or_ms_key* ms, uint64_t* ct) {
  if (!ms || !ms->count) return -1;
  double best = or_ms_measure(p, ms, ct, NULL);
  if (best <= ms->bound) return -1;
  int pick = -1;
  for (uint32_t z = 0; z < ms->count; z++) {
    const double m = or_ms_measure(p, ms, ct, ms->zeros + (size_t)z * (p->n + 1));
    if (m < best) {
      best = m;
      pick = (int)z;
      if (best <= ms->bound) break;
    }
  }
  if (pick >= 0) {
    const uint64_t* zr = ms->zeros + (size_t)pick * (p->n + 1);
    for (uint32_t i = 0; i <= p->n; i++) ct[i] += zr[i];
  }
  return pick;
}

void or_pbs(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* lwe_in,
            const uint64_t* lut, uint64_t* lwe_out) {
  or_pbs_ex(p, bsk_ntt, ksk, NULL, lwe_in, lut, lwe_out);
}

void or_pbs_ex(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const or_ms_key* ms,
               const uint64_t* lwe_in, const uint64_t* lut, uint64_t* lwe_out) {
  const size_t row = (size_t)(p->k + 1) * p->N;
  uint64_t* acc = (uint64_t*)malloc(row * 8);
  uint64_t* big = (uint64_t*)malloc(((size_t)p->k * p->N + 1) * 8);
  if (p->order == 0) {
    or_blind_rotate(p, bsk_ntt, 0, lwe_in, lut, acc);
    or_sample_extract(p, acc, big);
    or_keyswitch(p, ksk, big, lwe_out);
  } else {
    uint64_t* small = (uint64_t*)malloc(((size_t)p->n + 1) * 8);
    or_keyswitch(p, ksk, lwe_in, small);
    or_ms_reduce(p, ms, small);
    or_blind_rotate(p, bsk_ntt, 0, small, lut, acc);
    or_sample_extract(p, acc, lwe_out);
    free(small);
  }
  free(acc); free(big);
}

void or_pbs_batch(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* lwe_in,
                  size_t B, const uint64_t* luts, size_t n_lut, const uint32_t* lut_index, uint64_t* lwe_out,
                  int threads) {
  or_pbs_batch_ex(p, bsk_ntt, ksk, NULL, lwe_in, B, luts, n_lut, lut_index, lwe_out, threads);
}

void or_pbs_batch_ex(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const or_ms_key* ms,
                     const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                     const uint32_t* lut_index, uint64_t* lwe_out, int threads) {
  const size_t din = (p->order == 0 ? p->n : p->k * p->N) + 1;
  const size_t dout = (p->order == 0 ? p->n : p->k * p->N) + 1;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
  for (size_t q = 0; q < B; q++) {
    size_t li = lut_index ? lut_index[q] : 0;
    if (li >= n_lut) li = 0;
    or_pbs_ex(p, bsk_ntt, ksk, ms, lwe_in + q * din, luts + li * p->N, lwe_out + q * dout);
  }
  (void)threads;
}

/* ======================================================================================
 * LUTs (generate_accumulator, biometrics main.rs:65-68) and the NAND gate.
 * ==================================================================================== */
void or_lut_constant(uint32_t N, uint64_t torus_value, uint64_t* lut) {
  uint64_t v = or_tor_to_p(torus_value);
  for (uint32_t i = 0; i < N; i++) lut[i] = v;
}

void or_lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* f_table, uint64_t delta_out,
                       uint64_t* lut) {
  uint32_t box = N / msg_modulus;
  uint64_t* v = (uint64_t*)malloc((size_t)N * 8);
  for (uint32_t i = 0; i < N; i++) v[i] = or_tor_to_p(f_table[i / box] * delta_out);
  /* half-box rotation: lut = X^{-box/2} v */
  or_poly_monomial_mul(lut, v, N, 2 * N - box / 2);
  free(v);
}

void or_nand(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* c1,
             const uint64_t* c2, uint64_t* out) {
  const uint32_t n = p->n;
  uint64_t* c = (uint64_t*)malloc(((size_t)n + 1) * 8);
  uint64_t* lut = (uint64_t*)malloc((size_t)p->N * 8);
  for (uint32_t i = 0; i < n; i++) c[i] = 0 - c1[i] - c2[i];
  c[n] = (1ull << 61) - c1[n] - c2[n];
  or_lut_constant(p->N, 1ull << 61, lut);
  or_pbs(p, bsk_ntt, ksk, c, lut, out);
  free(c); free(lut);
}

/* ======================================================================================
 * Packing keyswitch + compression (header: or_pks_params).
 * ==================================================================================== */
int or_pks_params_preset(int preset, or_pks_params* o) {
  if (preset != 0) return -1;
  o->in_dim = 2048; o->out_k = 1; o->out_N = 2048; o->base_log = 14; o->level = 2;
  o->lwe_per_glwe = 2048; o->storage_log = 26; o->noise_log2 = -48;
  return 0;
}

size_t or_pksk_len(const or_pks_params* pp) {
  return (size_t)pp->in_dim * pp->level * (pp->out_k + 1) * pp->out_N;
}

/* native (2^64) GLWE encryption of the plaintext polynomial m (N values, nullable = 0) */
static void glwe_encrypt_native(uint32_t k, uint32_t N, const uint64_t* key, int32_t noise_log2, or_rng* r,
                                const uint64_t* m, uint64_t* out) {
  uint64_t* body = out + (size_t)k * N;
  for (size_t i = 0; i < (size_t)k * N; i++) out[i] = or_rng_u64(r);
  for (uint32_t i = 0; i < N; i++) body[i] = (uint64_t)or_rng_gauss(r, noise_log2) + (m ? m[i] : 0);
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = out + (size_t)c * N;
    const uint64_t* S = key + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!S[j]) continue;
      for (uint32_t i = 0; i < N; i++) {
        const uint32_t d = i + j;
        if (d < N) body[d] += A[i];
        else body[d - N] -= A[i];
      }
    }
  }
}

void or_pks_keygen(const or_pks_params* pp, uint64_t seed, const uint64_t* in_key, uint64_t* out_key,
                   uint64_t* pksk) {
  const uint32_t k = pp->out_k, N = pp->out_N;
  or_rng r;
  or_rng_init(&r, seed, 4);
  for (uint32_t i = 0; i < k * N; i++) out_key[i] = or_rng_u64(&r) & 1;
  if (!pksk) return;
  const size_t row = (size_t)(k + 1) * N;
#pragma omp parallel for schedule(dynamic, 8)
  for (uint32_t j = 0; j < pp->in_dim; j++) {
    or_rng rr;
    or_rng_init(&rr, seed, 0x300000 + j);
    uint64_t* m = (uint64_t*)calloc(N, 8);
    for (uint32_t l = 0; l < pp->level; l++) {
      m[0] = in_key[j] << (64 - pp->base_log * (l + 1));
      glwe_encrypt_native(k, N, out_key, pp->noise_log2, &rr, m, pksk + ((size_t)j * pp->level + l) * row);
    }
    free(m);
  }
}

void or_pks_pack(const or_pks_params* pp, const uint64_t* pksk, const uint64_t* lwes, uint32_t count,
                 uint64_t* glwe) {
  const uint32_t k = pp->out_k, N = pp->out_N, L = pp->level;
  const size_t row = (size_t)(k + 1) * N;
  uint64_t* buf = (uint64_t*)malloc(row * 8);
  int64_t dig[64];
  memset(glwe, 0, row * 8);
  for (uint32_t d = 0; d < count; d++) {
    const uint64_t* a = lwes + (size_t)d * (pp->in_dim + 1);
    memset(buf, 0, row * 8);
    buf[(size_t)k * N] = a[pp->in_dim];
    for (uint32_t j = 0; j < pp->in_dim; j++) {
      or_decompose(a[j], pp->base_log, L, dig);
      for (uint32_t l = 0; l < L; l++) {
        if (!dig[l]) continue;
        const uint64_t* key = pksk + ((size_t)j * L + l) * row;
        const uint64_t dv = (uint64_t)dig[l];
        for (size_t t = 0; t < row; t++) buf[t] -= dv * key[t];
      }
    }
    /* out += X^d * buf, each polynomial */
    for (uint32_t c = 0; c <= k; c++) {
      const uint64_t* src = buf + (size_t)c * N;
      uint64_t* dst = glwe + (size_t)c * N;
      for (uint32_t i = 0; i < N; i++) {
        const uint32_t t = i + d;
        if (t < N) dst[t] += src[i];
        else dst[t - N] -= src[i];
      }
    }
  }
  free(buf);
}

void or_glwe_phase_native(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out) {
  memcpy(out, glwe + (size_t)k * N, (size_t)N * 8);
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = glwe + (size_t)c * N;
    const uint64_t* S = key + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!S[j]) continue;
      for (uint32_t i = 0; i < N; i++) {
        const uint32_t d = i + j;
        if (d < N) out[d] -= A[i];
        else out[d - N] += A[i];
      }
    }
  }
}

size_t or_pks_packed_words(const or_pks_params* pp, uint32_t bodies) {
  const size_t vals = (size_t)pp->out_k * pp->out_N + bodies;
  return (vals * pp->storage_log + 63) / 64;
}

void or_pks_compress(const or_pks_params* pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed) {
  const uint32_t w = pp->storage_log;
  const size_t vals = (size_t)pp->out_k * pp->out_N + bodies;
  memset(packed, 0, or_pks_packed_words(pp, bodies) * 8);
  for (size_t v = 0; v < vals; v++) {
    const uint64_t x = glwe[v];     /* mask polys then the body, contiguous */
    const uint64_t ms = (((x >> (64 - w - 1)) + 1) >> 1) & ((1ull << w) - 1);
    const size_t bit = v * w, word = bit / 64, off = bit % 64;
    packed[word] |= ms << off;
    if (off + w > 64) packed[word + 1] |= ms >> (64 - off);
  }
}

void or_pks_extract(const or_pks_params* pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe) {
  const uint32_t w = pp->storage_log;
  const size_t vals = (size_t)pp->out_k * pp->out_N + bodies;
  memset(glwe, 0, (size_t)(pp->out_k + 1) * pp->out_N * 8);
  for (size_t v = 0; v < vals; v++) {
    const size_t bit = v * w, word = bit / 64, off = bit % 64;
    uint64_t ms = packed[word] >> off;
    if (off + w > 64) ms |= packed[word + 1] << (64 - off);
    ms &= (1ull << w) - 1;
    glwe[v] = ms << (64 - w);
  }
}
