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
 * Arithmetic (option A at 128 bits): the GLWE/BSK ring is Z_Q, Q = p1 * p2 with p1 = 2^64 - 2^32 + 1
 * and p2 = 2^64 - 2^34 + 1 (both NTT-friendly), held as residues; for the gadget decomposition a
 * coefficient is lifted to [0, Q) (CRT), mapped to the torus (below) and decomposed natively with
 * gadget round(Q / 2^(B(l+1))) (see gadget()); after sample extraction each Z_Q value is
 * mapped to Z_2^128 by y = x + floor((x * c + 2^127) / 2^128), c = floor(2^256 / Q) - 2^128 (the
 * scaling by 2^128 / Q, exact integer formula shared with the device).  Parity unpinned (no squashed
 * ciphertext in the reference); message-level checks pin decrypt(squash(ct)) == decrypt(ct).
 */
#include <stdlib.h>
#include <string.h>

#include "tfhe_oracle.h"

typedef unsigned __int128 u128;

static const uint64_t SP[2] = {0xFFFFFFFF00000001ull, 0xFFFFFFFC00000001ull};

static inline uint64_t mmul(uint64_t a, uint64_t b, uint64_t p) { return (uint64_t)(((u128)a * b) % p); }
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

/* ---- Z_Q <-> Z_2^128 -------------------------------------------------------------------- */
static u128 q_value(void) { return (u128)SP[0] * SP[1]; }
/* x mod Q from residues (Garner) */
static u128 crt(uint64_t r1, uint64_t r2) {
  static uint64_t inv = 0;
  if (!inv) inv = mpow(SP[0] % SP[1], SP[1] - 2, SP[1]);
  const uint64_t t = mmul(msub(r2, r1 % SP[1], SP[1]), inv, SP[1]);
  return (u128)r1 + (u128)SP[0] * t;
}
/* high 128 bits of x * y (128 x 128 -> 256) */
static u128 mulhi128(u128 x, u128 y) {
  const uint64_t x0 = (uint64_t)x, x1 = (uint64_t)(x >> 64), y0 = (uint64_t)y, y1 = (uint64_t)(y >> 64);
  const u128 p00 = (u128)x0 * y0, p01 = (u128)x0 * y1, p10 = (u128)x1 * y0, p11 = (u128)x1 * y1;
  const u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  return p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}
/* c = floor(2^256 / Q) - 2^128 */
static u128 conv_c(void) {
  static u128 c = 0;
  if (c) return c;
  const u128 Q = q_value(), d = (u128)0 - Q; /* 2^128 - Q */
  /* 2^256 / Q = 2^128 * (1 + d/Q) ... compute by long division: floor((2^256 - 2^128*Q) / Q) = floor(2^128*d / Q) */
  u128 rem = 0, quo = 0;
  /* dividend = d * 2^128: bits of d followed by 128 zero bits */
  for (int i = 255; i >= 0; i--) {
    const int bit = i >= 128 ? (int)((d >> (i - 128)) & 1) : 0;
    const int top = (int)(rem >> 127);
    rem = (rem << 1) | (u128)bit;
    if (top || rem >= Q) { rem -= Q; if (i < 128) quo |= (u128)1 << i; }
  }
  c = quo;
  return c;
}
/* y = x + floor((x*c + 2^127) / 2^128), x in [0, Q) */
static u128 q_to_tor(u128 x) {
  const u128 c = conv_c();
  /* (x*c + 2^127) >> 128 = mulhi(x, c) + carry of (lo(x*c) + 2^127) */
  const u128 lo = x * c;
  const u128 hi = mulhi128(x, c) + (((lo >> 127) & 1) ? 1 : 0);
  return x + hi;
}
/* torus t -> Z_Q: t - floor((t*d + 2^127) / 2^128), d = 2^128 - Q (round(t * Q / 2^128)) */
static u128 tor_to_q(u128 t) {
  const u128 d = (u128)0 - q_value();
  const u128 lo = t * d;
  const u128 hi = mulhi128(t, d) + (((lo >> 127) & 1) ? 1 : 0);
  return t - hi;
}
void or_sns_tor_to_q(const uint64_t* t /* lo, hi */, uint64_t* r /* r1, r2 */) {
  const u128 v = tor_to_q(((u128)t[1] << 64) | t[0]);
  r[0] = (uint64_t)(v % SP[0]);
  r[1] = (uint64_t)(v % SP[1]);
}
void or_sns_q_to_tor(const uint64_t* r, uint64_t* t) {
  const u128 v = q_to_tor(crt(r[0], r[1]));
  t[0] = (uint64_t)v;
  t[1] = (uint64_t)(v >> 64);
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

/* gadget of level l: round(Q / 2^(B(l+1))).  The decomposition runs on y = x * 2^128 / Q (the torus
 * image of x, where a carry out of the top digit vanishes mod 2^128), so sum_l d_l * g_l = y * Q / 2^128
 * ~ x (mod Q) up to |d| / 2 per level: the carry costs Q = 0 instead of 2^128 = 2^128 - Q (~2^97.6). */
static u128 gadget(uint32_t shift) {
  const u128 Q = q_value();
  return (Q >> shift) + ((Q >> (shift - 1)) & 1);
}

/* ---- keys ---------------------------------------------------------------------------------- */
/* GLWE key: k*N bits from ChaCha stream 5.  BSK row (i, c, l): GLWE_S(0) over Z_Q with s_i * g_l added
 * to coefficient 0 of component c, g_l = round(Q / 2^(B(l+1))); stream 0x400000 + i.  Layout
 * [i][c*L + l][j][prime][N] (standard domain residues).  Masks uniform mod each prime (= uniform mod Q),
 * noise one Gaussian integer per body coefficient (same integer in both residues). */
void or_sns_keygen(const or_sns_params* sp, uint64_t seed, const uint64_t* lwe_key, uint64_t* glwe_key,
                   uint64_t* bsk) {
  const uint32_t k = sp->k, N = sp->N, L = sp->level;
  or_rng r;
  or_rng_init(&r, seed, 5);
  for (uint32_t i = 0; i < k * N; i++) glwe_key[i] = or_rng_u64(&r) & 1;
  if (!bsk) return;
  /* NTT of the key polynomials per prime */
  uint64_t* skey = (uint64_t*)malloc((size_t)2 * k * N * 8);
  for (int q = 0; q < 2; q++)
    for (uint32_t c = 0; c < k; c++) {
      uint64_t* d = skey + ((size_t)q * k + c) * N;
      memcpy(d, glwe_key + (size_t)c * N, (size_t)N * 8);
      or_sns_ntt_fwd(q, d, N);
    }
  const size_t row = (size_t)(k + 1) * 2 * N, per_i = (size_t)(k + 1) * L * row;
#pragma omp parallel for schedule(dynamic, 1)
  for (uint32_t i = 0; i < sp->n; i++) {
    or_rng rr;
    or_rng_init(&rr, seed, 0x400000 + i);
    uint64_t* tmp = (uint64_t*)malloc((size_t)N * 8);
    uint64_t* acc = (uint64_t*)malloc((size_t)N * 8);
    int64_t* e = (int64_t*)malloc((size_t)N * 8);
    for (uint32_t c = 0; c <= k; c++)
      for (uint32_t l = 0; l < L; l++) {
        uint64_t* out = bsk + per_i * i + row * (c * L + l); /* [j][prime][N] */
        for (uint32_t j = 0; j < k; j++)
          for (int q = 0; q < 2; q++)
            for (uint32_t t = 0; t < N; t++) {
              uint64_t v;
              do v = or_rng_u64(&rr); while (v >= SP[q]);
              out[((size_t)j * 2 + q) * N + t] = v;
            }
        for (uint32_t t = 0; t < N; t++) e[t] = or_rng_gauss(&rr, sp->noise_log2);
        for (int q = 0; q < 2; q++) {
          const uint64_t p = SP[q];
          for (uint32_t t = 0; t < N; t++) acc[t] = 0;
          for (uint32_t j = 0; j < k; j++) { /* acc += NTT(mask_j) * NTT(S_j) (NTT domain) */
            memcpy(tmp, out + ((size_t)j * 2 + q) * N, (size_t)N * 8);
            or_sns_ntt_fwd(q, tmp, N);
            const uint64_t* s = skey + ((size_t)q * k + j) * N;
            for (uint32_t t = 0; t < N; t++) acc[t] = madd(acc[t], mmul(tmp[t], s[t], p), p);
          }
          or_sns_ntt_inv(q, acc, N);
          uint64_t* body = out + ((size_t)k * 2 + q) * N;
          for (uint32_t t = 0; t < N; t++) body[t] = madd(acc[t], from_i64(e[t], p), p);
          if (lwe_key[i]) {
            const u128 g = gadget(sp->base_log * (l + 1));
            uint64_t* dst = out + ((size_t)c * 2 + q) * N;
            dst[0] = madd(dst[0], (uint64_t)(g % p), p);
          }
        }
      }
    free(tmp); free(acc); free(e);
  }
  free(skey);
}

/* Load-time rounding of the squashing key (the device's precision contract, tfhe_amd/csrc/sns_fft.h):
 * every coefficient x (residues r1, r2) is centred in (-Q/2, Q/2] and rounded to the nearest multiple of
 * 2^16 (ties up).  The rounding error (< 2^15 per mask and body coefficient) adds ~2^20 of phase noise
 * to a key whose own noise is 2^30; in exchange the rounded key is 2^16 x a 112-bit integer, whose seven
 * balanced 16-bit limbs make each digit x limb convolution an exact f64 FFT product on the device.
 * Both device transforms (the f64 FFT and the NTT) apply it at load; the oracle applies it here. */
void or_sns_bsk_round(const or_sns_params* sp, const uint64_t* bsk, uint64_t* out) {
  const size_t N = sp->N, pairs = or_sns_bsk_len(sp) / (2 * N);
  const u128 Q = q_value();
#pragma omp parallel for schedule(static)
  for (size_t pp = 0; pp < pairs; pp++)
    for (size_t t = 0; t < N; t++) {
      const u128 x = crt(bsk[(2 * pp) * N + t], bsk[(2 * pp + 1) * N + t]);
      const __int128 xc = x > Q / 2 ? (__int128)(x - Q) : (__int128)x;
      const __int128 rr = (xc + ((__int128)1 << 15)) >> 16; /* floor: arithmetic shift */
      const __int128 v = rr * 65536;
      for (int q = 0; q < 2; q++) {
        const __int128 m = v % (__int128)SP[q];
        out[(2 * pp + q) * N + t] = (uint64_t)(m < 0 ? m + (__int128)SP[q] : m);
      }
    }
}

void or_sns_bsk_to_ntt(const or_sns_params* sp, const uint64_t* bsk, uint64_t* bsk_ntt) {
  const size_t polys = or_sns_bsk_len(sp) / sp->N;
#pragma omp parallel for schedule(static)
  for (size_t q = 0; q < polys; q++) {
    memcpy(bsk_ntt + q * sp->N, bsk + q * sp->N, (size_t)sp->N * 8);
    or_sns_ntt_fwd((int)(q & 1), bsk_ntt + q * sp->N, sp->N);
  }
}

/* identity LUT on msg_modulus values with one padding bit: delta = 2^127 / msg_modulus, half-box
 * rotation; residues [prime][N] */
void or_sns_lut_identity(const or_sns_params* sp, uint32_t msg_modulus, uint64_t* lut) {
  const uint32_t N = sp->N, box = N / msg_modulus;
  const u128 delta = ((u128)1 << 127) / msg_modulus;
  for (uint32_t i = 0; i < N; i++) {
    const uint32_t src = i + box / 2;
    u128 t = (u128)((src < N ? src : src - N) / box) * delta;
    u128 v = tor_to_q(t);
    for (int q = 0; q < 2; q++) {
      uint64_t r = (uint64_t)(v % SP[q]);
      lut[(size_t)q * N + i] = (src < N || r == 0) ? r : SP[q] - r;
    }
  }
}

/* one ciphertext: lwe_small (n+1, native 2^64) -> acc [(k+1)][prime][N] (standard domain) */
void or_sns_blind_rotate(const or_sns_params* sp, const uint64_t* bsk_ntt, const uint64_t* lwe, const uint64_t* lut,
                         uint64_t* acc) {
  const uint32_t k = sp->k, N = sp->N, L = sp->level, twoN = 2 * N;
  const size_t poly = (size_t)2 * N; /* both primes */
  uint64_t* rot = (uint64_t*)malloc((size_t)(k + 1) * poly * 8);
  uint64_t* dig = (uint64_t*)malloc((size_t)(k + 1) * L * poly * 8);
  uint64_t* outp = (uint64_t*)malloc((size_t)(k + 1) * poly * 8);
  int64_t d[8];
  /* acc = X^{-b~} * (0, .., 0, lut) */
  memset(acc, 0, (size_t)(k + 1) * poly * 8);
  const uint32_t bt = or_mod_switch(lwe[sp->n], twoN);
  const uint32_t sh = (twoN - bt) % twoN;
  for (int q = 0; q < 2; q++)
    for (uint32_t t = 0; t < N; t++) {
      uint32_t dst = t + sh;
      int neg = 0;
      if (dst >= twoN) dst -= twoN;
      if (dst >= N) { dst -= N; neg = 1; }
      const uint64_t v = lut[(size_t)q * N + t];
      acc[(size_t)k * poly + (size_t)q * N + dst] = neg && v ? SP[q] - v : v;
    }
  const size_t bsk_i = (size_t)(k + 1) * L * (k + 1) * poly;
  for (uint32_t i = 0; i < sp->n; i++) {
    const uint32_t ai = or_mod_switch(lwe[i], twoN);
    if (!ai) continue;
    /* rot = X^{ai} * acc - acc */
    for (uint32_t c = 0; c <= k; c++)
      for (int q = 0; q < 2; q++) {
        const uint64_t p = SP[q];
        const uint64_t* a = acc + (size_t)c * poly + (size_t)q * N;
        uint64_t* o = rot + (size_t)c * poly + (size_t)q * N;
        for (uint32_t t = 0; t < N; t++) {
          uint32_t dst = t + ai;
          int neg = 0;
          if (dst >= twoN) dst -= twoN;
          if (dst >= N) { dst -= N; neg = 1; }
          o[dst] = neg ? (a[t] ? p - a[t] : 0) : a[t];
        }
        for (uint32_t t = 0; t < N; t++) o[t] = msub(o[t], a[t], p);
      }
    /* decompose each coefficient (read in Z_Q) */
    for (uint32_t c = 0; c <= k; c++)
      for (uint32_t t = 0; t < N; t++) {
        const u128 x = crt(rot[(size_t)c * poly + t], rot[(size_t)c * poly + N + t]);
        decompose128(q_to_tor(x), sp->base_log, L, d);
        for (uint32_t l = 0; l < L; l++)
          for (int q = 0; q < 2; q++) dig[((size_t)(c * L + l)) * poly + (size_t)q * N + t] = from_i64(d[l], SP[q]);
      }
    for (uint32_t r = 0; r < (k + 1) * L; r++)
      for (int q = 0; q < 2; q++) or_sns_ntt_fwd(q, dig + (size_t)r * poly + (size_t)q * N, N);
    /* out_j = sum_r dig_r * BSK_i[r][j] */
    const uint64_t* bi = bsk_ntt + bsk_i * i;
    for (uint32_t j = 0; j <= k; j++)
      for (int q = 0; q < 2; q++) {
        const uint64_t p = SP[q];
        uint64_t* o = outp + (size_t)j * poly + (size_t)q * N;
        for (uint32_t t = 0; t < N; t++) {
          uint64_t s = 0;
          for (uint32_t r = 0; r < (k + 1) * L; r++)
            s = madd(s, mmul(dig[(size_t)r * poly + (size_t)q * N + t],
                             bi[((size_t)r * (k + 1) + j) * poly + (size_t)q * N + t], p), p);
          o[t] = s;
        }
        or_sns_ntt_inv(q, o, N);
        uint64_t* a = acc + (size_t)j * poly + (size_t)q * N;
        for (uint32_t t = 0; t < N; t++) a[t] = madd(a[t], o[t], p);
      }
  }
  free(rot); free(dig); free(outp);
}

/* acc -> LWE over Z_2^128, dim k*N (+ body): u64 pairs (lo, hi) */
void or_sns_sample_extract(const or_sns_params* sp, const uint64_t* acc, uint64_t* out) {
  const uint32_t k = sp->k, N = sp->N;
  const size_t poly = (size_t)2 * N;
  for (uint32_t c = 0; c < k; c++)
    for (uint32_t t = 0; t < N; t++) {
      uint64_t r[2];
      for (int q = 0; q < 2; q++) {
        const uint64_t v = acc[(size_t)c * poly + (size_t)q * N + (t == 0 ? 0 : N - t)];
        r[q] = (t == 0 || v == 0) ? v : SP[q] - v;
      }
      or_sns_q_to_tor(r, out + 2 * ((size_t)c * N + t));
    }
  uint64_t r[2] = {acc[(size_t)k * poly], acc[(size_t)k * poly + N]};
  or_sns_q_to_tor(r, out + 2 * ((size_t)k * N));
}

void or_sns_squash(const or_sns_params* sp, const uint64_t* bsk_ntt, const uint64_t* lwe_small, size_t B,
                   uint32_t msg_modulus, uint64_t* out, int threads) {
  const size_t acc_len = (size_t)(sp->k + 1) * 2 * sp->N, out_len = 2 * ((size_t)sp->k * sp->N + 1);
  uint64_t* lut = (uint64_t*)malloc((size_t)2 * sp->N * 8);
  or_sns_lut_identity(sp, msg_modulus, lut);
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 16)
  for (size_t q = 0; q < B; q++) {
    uint64_t* acc = (uint64_t*)malloc(acc_len * 8);
    or_sns_blind_rotate(sp, bsk_ntt, lwe_small + q * (sp->n + 1), lut, acc);
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
