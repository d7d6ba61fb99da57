/*
 * exact_oracle.c — the EXACT external product, CMUX and blind rotation over the native 2^64 torus: the
 * arbiter of the FFT64 path that shares none of its operation order.
 *
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h): used by tests/ as the checker; never linked into the product.
 *
 * Why it exists.  The FFT64 kernels (tfhe_amd/csrc/pbs_fft.hip, pbs_fft2k.hip) are bit-exact against
 * fft_oracle.c, which restates their f64 operation sequence.  That pins the device to a twin, not to the
 * mathematics.  The function both approximate is the reference's exact wrapping negacyclic product
 * (ml/extensions/rust/src/computations.rs:50-54 polynomial_wrapping_mul, :101-105 ..._add_mul_assign), applied
 * to SignedDecomposer digits (ml/extensions/rust/src/encryption.rs:152-166, 191-201) inside the CMUX of
 * keyswitch_programmable_bootstrap (ml/biometrics/notebooks/main.rs:71).  This file computes that function in
 * exact integer arithmetic, so tests can bound |FFT64 result - exact result| (tests/test_exact.py,
 * tests/test_gpu_exact.py; the bound is derived in DESIGN.md §5).
 *
 * Method.  Every BSK word w (a Z_2^64 value) is split into three balanced base-2^22 limbs,
 *     w = l0 + 2^22 l1 + 2^44 l2  (mod 2^64),   l0, l1 in [-2^21, 2^21),  l2 in [-2^19, 2^19],
 * and each digit-polynomial x limb-polynomial negacyclic product is formed EXACTLY through the Goldilocks NTT
 * (or_ntt_fwd / or_ntt_inv, checked against the O(N^2) schoolbook in tests/test_oracle.py): for one output
 * column the summed integer products obey
 *     |sum_r d_r (*) l_{r,t}| <= (k+1) L N 2^(beta-1) 2^21  <=  2 * 1 * 2048 * 2^22 * 2^21 = 2^55  (P-FHEVM)
 *                                                            6 * 1024 * 2^6 * 2^21 = 2^39.6     (P-GATE)
 * which is < p/2 (p = 2^64 - 2^32 + 1), so the centred residue IS the integer.  Recombining
 * sum_t 2^(22 t) r_t mod 2^64 gives the exact wrapping product, i.e. what computations.rs:50-54 defines.  No
 * floating point anywhere; the MAC order is irrelevant (exact).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "tfhe_oracle.h"

#define EX_LIMBS 3
#define EX_LIMB_BITS 22

struct or_exact_key {
  or_params p;
  size_t polys;    /* or_bsk_len / N */
  uint64_t* limb;  /* [poly][limb][N] NTT domain, Z_p */
  double* knorm2;  /* [poly] sum_j (double)(int64)w_j^2: the signed word's squared norm (the FFT's operand) */
};

static inline uint64_t zp_from_i64(int64_t v) { return v >= 0 ? (uint64_t)v : OR_P - (uint64_t)(-v); }
static inline int64_t zp_centred(uint64_t x) { return x > OR_P / 2 ? -(int64_t)(OR_P - x) : (int64_t)x; }

/* balanced base-2^22 limbs of w (mod 2^64) */
static void limbs3(uint64_t w, int64_t out[EX_LIMBS]) {
  uint64_t rest = w;
  for (int t = 0; t < EX_LIMBS - 1; t++) {
    int64_t l = (int64_t)(rest & ((1ull << EX_LIMB_BITS) - 1));
    if (l >= (1ll << (EX_LIMB_BITS - 1))) l -= 1ll << EX_LIMB_BITS;
    out[t] = l;
    rest = (rest - (uint64_t)l) >> EX_LIMB_BITS; /* exact: rest - l is a multiple of 2^22 (mod 2^64) */
  }
  /* top limb: the remaining 20 bits as a balanced value (bits above 64 vanish mod 2^64) */
  int64_t top = (int64_t)(rest & ((1ull << (64 - 2 * EX_LIMB_BITS)) - 1));
  if (top >= (1ll << (63 - 2 * EX_LIMB_BITS))) top -= 1ll << (64 - 2 * EX_LIMB_BITS);
  out[EX_LIMBS - 1] = top;
}

or_exact_key* or_exact_key_new(const or_params* p, const uint64_t* bsk) {
  if (p->k != 1 || p->pbs_level > 8) return NULL;
  or_exact_key* K = (or_exact_key*)calloc(1, sizeof(*K));
  K->p = *p;
  K->polys = or_bsk_len(p) / p->N;
  const uint32_t N = p->N;
  K->limb = (uint64_t*)malloc(K->polys * EX_LIMBS * N * 8);
  K->knorm2 = (double*)malloc(K->polys * sizeof(double));
#pragma omp parallel for schedule(static)
  for (size_t q = 0; q < K->polys; q++) {
    uint64_t* dst = K->limb + q * EX_LIMBS * N;
    double s = 0.0;
    for (uint32_t j = 0; j < N; j++) {
      const uint64_t w = bsk[q * N + j];
      int64_t l[EX_LIMBS];
      limbs3(w, l);
      for (int t = 0; t < EX_LIMBS; t++) dst[(size_t)t * N + j] = zp_from_i64(l[t]);
      const double v = (double)(int64_t)w;
      s += v * v;
    }
    K->knorm2[q] = s;
    for (int t = 0; t < EX_LIMBS; t++) or_ntt_fwd(dst + (size_t)t * N, N);
  }
  return K;
}

void or_exact_key_free(or_exact_key* K) {
  if (!K) return;
  free(K->limb);
  free(K->knorm2);
  free(K);
}

/* (X^t * in)[i] on native torus values, t in [0, 2N) */
static void rot_torus(uint64_t* out, const uint64_t* in, uint32_t N, uint32_t t) {
  for (uint32_t i = 0; i < N; i++) {
    int64_t d = (int64_t)i - (int64_t)t;
    int neg = 0;
    while (d < 0) { d += N; neg ^= 1; }
    out[i] = neg ? 0 - in[d] : in[d];
  }
}

/* acc_out = acc_in + ExtProd(BSK_i, X^a acc_in - acc_in), exactly.  s1[j] = sum_r ||d_r||_2 ||w_{r,j}||_2 and
 * s2[j] = sum_r ||d_r||_2^2 ||w_{r,j}||_2^2 (w as signed int64: the operand the FFT transforms) for the bound. */
static void cmux_exact_one(const or_exact_key* K, uint32_t i, uint32_t a, const uint64_t* acc_in, uint64_t* acc_out,
                           double* s1, double* s2) {
  const or_params* p = &K->p;
  const uint32_t N = p->N, k = p->k, L = p->pbs_level;
  const size_t R = (size_t)(k + 1) * L, row = (size_t)(k + 1) * N;
  uint64_t* rot = (uint64_t*)malloc((size_t)N * 8);
  uint64_t* dig = (uint64_t*)malloc(R * N * 8);          /* NTT of each digit polynomial, r = c L + l */
  uint64_t* sum = (uint64_t*)calloc((k + 1) * EX_LIMBS * (size_t)N, 8); /* [j][t][N] */
  double dn2[64];
  int64_t d[64];
  for (uint32_t c = 0; c <= k; c++) {
    const uint64_t* A = acc_in + (size_t)c * N;
    rot_torus(rot, A, N, a);
    for (uint32_t l = 0; l < L; l++) dn2[c * L + l] = 0.0;
    for (uint32_t j = 0; j < N; j++) {
      or_decompose(rot[j] - A[j], p->pbs_base_log, L, d); /* d[0] most significant (gadget 2^(64-beta)) */
      for (uint32_t l = 0; l < L; l++) {
        dig[(c * L + l) * (size_t)N + j] = zp_from_i64(d[l]);
        dn2[c * L + l] += (double)d[l] * (double)d[l];
      }
    }
  }
  for (size_t r = 0; r < R; r++) or_ntt_fwd(dig + r * N, N);
  for (uint32_t j = 0; j <= k; j++) {
    double t1 = 0.0, t2 = 0.0;
    for (size_t r = 0; r < R; r++) {
      const size_t poly = ((size_t)i * R + r) * (k + 1) + j; /* BSK layout [i][c*L+l][j][coef] */
      const uint64_t* W = K->limb + poly * EX_LIMBS * N;
      const uint64_t* D = dig + r * N;
      for (int t = 0; t < EX_LIMBS; t++) {
        uint64_t* S = sum + ((size_t)j * EX_LIMBS + t) * N;
        const uint64_t* Wt = W + (size_t)t * N;
        for (uint32_t f = 0; f < N; f++) S[f] = or_add(S[f], or_mul(D[f], Wt[f]));
      }
      t1 += sqrt(dn2[r]) * sqrt(K->knorm2[poly]);
      t2 += dn2[r] * K->knorm2[poly];
    }
    if (s1) s1[j] = t1;
    if (s2) s2[j] = t2;
  }
  for (uint32_t j = 0; j <= k; j++) {
    uint64_t out[4096];
    for (uint32_t f = 0; f < N; f++) out[f] = 0;
    for (int t = 0; t < EX_LIMBS; t++) {
      uint64_t* S = sum + ((size_t)j * EX_LIMBS + t) * N;
      or_ntt_inv(S, N);
      for (uint32_t f = 0; f < N; f++) out[f] += (uint64_t)zp_centred(S[f]) << (EX_LIMB_BITS * t);
    }
    for (uint32_t f = 0; f < N; f++) acc_out[(size_t)j * N + f] = acc_in[(size_t)j * N + f] + out[f];
  }
  (void)row;
  free(rot);
  free(dig);
  free(sum);
}

void or_cmux_exact_batch(const or_exact_key* K, size_t count, const uint32_t* key_index, const uint32_t* a_tilde,
                         const uint64_t* acc_in, uint64_t* acc_out, double* s1, double* s2, int threads) {
  const or_params* p = &K->p;
  const size_t row = (size_t)(p->k + 1) * p->N;
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
  for (size_t q = 0; q < count; q++)
    cmux_exact_one(K, key_index[q], a_tilde[q], acc_in + q * row, acc_out + q * row, s1 ? s1 + q * (p->k + 1) : NULL,
                   s2 ? s2 + q * (p->k + 1) : NULL);
  (void)threads;
}

/* exact product of one digit polynomial (|d| small) and one torus polynomial, by the same limb method: the
 * self-check of this file against or_poly_mul_torus_schoolbook */
void or_poly_mul_torus_exact(uint64_t* out, const int64_t* a, const uint64_t* b, uint32_t N) {
  uint64_t* D = (uint64_t*)malloc((size_t)N * 8);
  uint64_t* W = (uint64_t*)malloc((size_t)N * 8 * EX_LIMBS);
  for (uint32_t j = 0; j < N; j++) {
    D[j] = zp_from_i64(a[j]);
    int64_t l[EX_LIMBS];
    limbs3(b[j], l);
    for (int t = 0; t < EX_LIMBS; t++) W[(size_t)t * N + j] = zp_from_i64(l[t]);
  }
  or_ntt_fwd(D, N);
  for (uint32_t f = 0; f < N; f++) out[f] = 0;
  for (int t = 0; t < EX_LIMBS; t++) {
    uint64_t* Wt = W + (size_t)t * N;
    or_ntt_fwd(Wt, N);
    for (uint32_t f = 0; f < N; f++) Wt[f] = or_mul(Wt[f], D[f]);
    or_ntt_inv(Wt, N);
    for (uint32_t f = 0; f < N; f++) out[f] += (uint64_t)zp_centred(Wt[f]) << (EX_LIMB_BITS * t);
  }
  free(D);
  free(W);
}

/* free-running exact blind rotation (same LUT convention as or_blind_rotate_fft: lut in the Z_p encoding) */
void or_blind_rotate_exact(const or_exact_key* K, const uint64_t* lwe_in, const uint64_t* lut, uint64_t* acc) {
  const or_params* p = &K->p;
  const uint32_t N = p->N, k = p->k, n = p->n;
  const size_t row = (size_t)(k + 1) * N;
  uint64_t* lt = (uint64_t*)malloc((size_t)N * 8);
  uint64_t* tmp = (uint64_t*)malloc(row * 8);
  for (uint32_t i = 0; i < N; i++) lt[i] = or_p_to_tor(lut[i]);
  memset(acc, 0, row * 8);
  const uint32_t bt = or_mod_switch(lwe_in[n], 2 * N);
  rot_torus(acc + (size_t)k * N, lt, N, (2 * N - bt) % (2 * N));
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t a = or_mod_switch(lwe_in[i], 2 * N);
    if (a == 0) continue;
    cmux_exact_one(K, i, a, acc, tmp, NULL, NULL);
    memcpy(acc, tmp, row * 8);
  }
  free(lt);
  free(tmp);
}
