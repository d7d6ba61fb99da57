/*
 * tfhe_oracle.h — CPU restatement of the TFHE programmable bootstrap (PBS) path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libtfhe_hip.so, tfhe_amd/, js/) links,
 * imports or executes this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may call it, and only as the checker / the timed CPU baseline.
 *
 * What it restates.  The reference (luxfi/tfhe monorepo) reaches its PBS through tfhe-rs
 * (npm `tfhe`/`node-tfhe` 0.8.7, packages/pnpm-lock.yaml:1988-1995; Rust git revs in
 * ml/extensions/rust/Cargo.toml:40), which is NOT vendored under /root/reference.  This file
 * restates the published CGGI/tfhe-rs algorithm with the conventions visible in the
 * reference's own call sites:
 *   - Delta encoding with one padding bit ........ ml/extensions/rust/src/encryption.rs:5-22
 *   - SignedDecomposer / closest_representable ... ml/extensions/rust/src/encryption.rs:152-166,191-201
 *   - exact negacyclic wrapping product .......... ml/extensions/rust/src/computations.rs:50-54,101-105
 *   - sample extraction .......................... ml/extensions/rust/src/computations.rs:109-132
 *   - LUT + keyswitch_programmable_bootstrap ..... ml/biometrics/notebooks/main.rs:65-77
 *   - P-FHEVM parameters ......................... sdk/relayer/src/tfhe.ts:14-19 (decoded in SURVEY App. A)
 *
 * PARITY STATUS: "parity unpinned" at the raw-ciphertext level.  No file in the reference holds
 * raw PBS input/output vectors (e2e/test/fhe.test.ts only asserts byteLength>0), and tfhe-rs
 * itself uses an f64 FFT that is not bit-reproducible.  Parity is pinned at the MESSAGE level:
 * decrypt(PBS(f)) == f(m) for every message (biometrics main.rs:77 pattern), the NAND truth
 * table, and the fhEVM operator KATs (tests/fhevm-suite/e2e/test/fhevmOperations*.ts).
 * The GPU path must match THIS oracle bit-for-bit on identical integer inputs and keys.
 *
 * Arithmetic design (SURVEY.md §7 option A):
 *   LWE / KSK : native torus Z_{2^64}
 *   GLWE / BSK: Z_p with p = 2^64 - 2^32 + 1 (Goldilocks), NTT-friendly, exact
 *   q_p -> 2^64 after sample extraction: y = x + ((x + 2^31) >> 32)
 */
#ifndef TFHE_ORACLE_H
#define TFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_P 0xFFFFFFFF00000001ull

typedef struct or_params {
  uint32_t n, k, N;
  uint32_t pbs_base_log, pbs_level;
  uint32_t ks_base_log, ks_level;
  int32_t lwe_noise_log2;   /* stddev = 2^x of the torus */
  int32_t glwe_noise_log2;
  uint32_t order;           /* 0 = PBS then KS (small key ciphertexts), 1 = KS then PBS */
  uint32_t transform;       /* 0 = NTT over Z_p (Goldilocks); 1 = f64 FFT over the native 2^64 torus */
} or_params;

/* preset 0 = P-GATE (n=630,k=1,N=1024, 7x3, 2x8), preset 1 = P-FHEVM (918,1,2048, 23x1, 4x4),
 * preset 2 = P-GATE on the FFT64 transform (fft_oracle.c); preset 3 = P-FHEVM on the FFT64 transform. */
int or_params_preset(int preset, or_params* out);

/* ---- PRNG (ChaCha20, RFC 8439 block function) -------------------------------------- */
typedef struct or_rng { uint32_t key[8]; uint32_t ctr; uint32_t buf[16]; int pos; } or_rng;
void or_rng_init(or_rng* r, uint64_t seed, uint64_t stream);
uint64_t or_rng_u64(or_rng* r);
uint64_t or_rng_mod_p(or_rng* r);
int64_t or_rng_gauss(or_rng* r, int32_t log2_sigma); /* round(N(0,1) * 2^(64+log2_sigma)) */

/* ---- Z_p arithmetic ----------------------------------------------------------------- */
uint64_t or_add(uint64_t a, uint64_t b);
uint64_t or_sub(uint64_t a, uint64_t b);
uint64_t or_mul(uint64_t a, uint64_t b);
uint64_t or_pow(uint64_t a, uint64_t e);
uint64_t or_psi(uint32_t N);      /* canonical primitive 2N-th root: psi^(2N/64) == 8 */
uint64_t or_tor_to_p(uint64_t v); /* torus 2^64 -> Z_p embedding used for LUT values */
uint64_t or_p_to_tor(uint64_t x); /* Z_p -> torus 2^64: x + ((x + 2^31) >> 32) */

/* ---- polynomials in Z_p[X]/(X^N+1) --------------------------------------------------- */
void or_poly_mul_schoolbook(uint64_t* out, const uint64_t* a, const uint64_t* b, uint32_t N);
void or_ntt_fwd(uint64_t* a, uint32_t N); /* natural order: A[j] = a(psi^(2j+1)) */
void or_ntt_inv(uint64_t* a, uint32_t N); /* exact inverse, includes 1/N */
void or_poly_mul_ntt(uint64_t* out, const uint64_t* a, const uint64_t* b, uint32_t N);
void or_poly_monomial_mul(uint64_t* out, const uint64_t* in, uint32_t N, uint32_t t); /* X^t * in */

/* ---- decomposition -------------------------------------------------------------------- */
/* tfhe-rs SignedDecomposer: closest_representable to base_log*level bits, balanced digits.
 * digits[0] is the MOST significant level (gadget 2^(64-base_log)). */
void or_decompose(uint64_t x, uint32_t base_log, uint32_t level, int64_t* digits);
uint32_t or_mod_switch(uint64_t x, uint32_t two_n); /* round(x * 2N / 2^64) mod 2N */

/* ---- sizes -------------------------------------------------------------------------- */
size_t or_bsk_len(const or_params* p); /* n*(k+1)l*(k+1)*N u64, layout [i][c*l+lvl][j][coef] */
size_t or_ksk_len(const or_params* p); /* kN*l_ks*(n+1) u64, layout [j][r][0..n] (b last) */

/* ---- keys & encryption --------------------------------------------------------------- */
void or_keygen(const or_params* p, uint64_t seed, uint64_t* lwe_key /*n*/, uint64_t* glwe_key /*kN*/,
               uint64_t* bsk /*nullable*/, uint64_t* ksk /*nullable*/);
void or_server_keygen(const or_params* p, uint64_t seed, const uint64_t* lwe_key, const uint64_t* glwe_key,
                      uint64_t* bsk, uint64_t* ksk);
/* ct q of the batch uses ChaCha stream (stream0 + q). dim = LWE dimension of key. */
void or_lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, uint64_t seed,
                    uint64_t stream0, const uint64_t* msgs, size_t count, uint64_t* out);
void or_lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out);

/* ---- bootstrap pieces ----------------------------------------------------------------- */
/* NTT-domain copy of the BSK (natural order, pre-scaled by nothing) for the fast oracle path */
void or_bsk_to_ntt(const or_params* p, const uint64_t* bsk, uint64_t* bsk_ntt);
/* acc_out: (k+1)*N u64 in Z_p.  lwe_in: dim n+1.  lut: N values in Z_p. bsk_ntt from above.
 * use_schoolbook != 0 uses the O(N^2) product against the standard-domain bsk instead. */
void or_blind_rotate(const or_params* p, const uint64_t* bsk_any, int use_schoolbook,
                     const uint64_t* lwe_in, const uint64_t* lut, uint64_t* acc_out);
void or_sample_extract(const or_params* p, const uint64_t* acc, uint64_t* lwe_big_out /*kN+1*/);
void or_keyswitch(const or_params* p, const uint64_t* ksk, const uint64_t* lwe_big /*kN+1*/,
                  uint64_t* lwe_small_out /*n+1*/);
/* Full PBS of one ciphertext (order from params). */
void or_pbs(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* lwe_in,
            const uint64_t* lut, uint64_t* lwe_out);
/* Batch PBS over B ciphertexts with OpenMP (threads<=0: all cores). lut_index nullable. */
void or_pbs_batch(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* lwe_in,
                  size_t B, const uint64_t* luts, size_t n_lut, const uint32_t* lut_index,
                  uint64_t* lwe_out, int threads);

/* ---- modulus-switch noise reduction (P-FHEVM) ------------------------
 * The P-FHEVM server key carries `count` LWE encryptions of zero under the small key (1449 in the
 * reference's parameter block, privateKey.bin @0x5e04, with ms_bound = 2^58, ms_r_sigma_factor =
 * 13.179852282053789, ms_input_variance = 2.63039184094559e-07).  Before the
 * blind rotation (after the keyswitch) the ciphertext may get ONE of them added, chosen to shrink
 * the modulus-switch error (tfhe-rs 1.x `improve_lwe_ciphertext_modulus_switch_noise_for_binary_key`,
 * absent from /root/reference; restated from its published description, parity unpinned):
 *   err(x)   = (round(x * 2N / 2^64) * 2^64/2N) - x           (signed, |err| <= 2^(63-log2 2N))
 *   measure  = |err(b) - sum_i err(a_i) / 2| + r * sqrt(sum_i err(a_i)^2 / 4 + var * 2^128)
 *              (mean and r-sigma of the switched phase error for a uniform binary key)
 *   if measure(ct) <= bound: unchanged; else add the zero with the lowest index whose measure is
 *   <= bound, or failing that the lowest-index minimiser if it beats measure(ct).
 * Sums are exact integers (i64 / u128); the double evaluation order above is fixed so the GPU
 * kernel reproduces every comparison bit-for-bit. */
#define OR_MS_FHEVM_ZEROS 1449u
#define OR_MS_FHEVM_BOUND 0x1p58
#define OR_MS_FHEVM_R_SIGMA 13.179852282053789
#define OR_MS_FHEVM_INPUT_VARIANCE 2.63039184094559e-07

typedef struct or_ms_key {
  const uint64_t* zeros; /* count x (n+1) */
  uint32_t count;
  double bound, r_sigma, input_variance;
} or_ms_key;

/* encryptions of zero under the small key: zero z uses ChaCha stream 0x200000 + z of `seed` */
void or_ms_zeros_keygen(const or_params* p, uint64_t seed, const uint64_t* lwe_key, uint32_t count,
                        uint64_t* zeros /* count x (n+1) */);
/* measure of ct (+ zero when zero != NULL); dim = p->n */
double or_ms_measure(const or_params* p, const or_ms_key* ms, const uint64_t* ct, const uint64_t* zero);
/* returns the chosen zero index or -1 and applies it to ct in place */
int or_ms_reduce(const or_params* p, const or_ms_key* ms, uint64_t* ct /* n+1 */);
/* or_pbs / or_pbs_batch with the reduction between keyswitch and blind rotation (order 1; ms nullable) */
void or_pbs_ex(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const or_ms_key* ms,
               const uint64_t* lwe_in, const uint64_t* lut, uint64_t* lwe_out);
void or_pbs_batch_ex(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const or_ms_key* ms,
                     const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                     const uint32_t* lut_index, uint64_t* lwe_out, int threads);

/* ---- LWE -> GLWE packing keyswitch + modulus-switched compression --------------
 * Restates the reference's ciphertext compression (ml/extensions/rust/src/compression.rs:246-291,
 * cpu_compress_ciphertexts_into_list -> tfhe-rs par_keyswitch_lwe_ciphertext_list_and_pack_in_glwe_
 * ciphertext, then CompressedModulusSwitchedGlweCiphertext::compress; extract :134-156):
 *   for LWE d of a chunk of <= lwe_per_glwe:  buf = (0,..,0 | b_d at coefficient 0);
 *     for each mask element a_j, digits d_l of closest_representable(a_j) (SignedDecomposer):
 *       buf -= d_l * PKSK[j][l]      (PKSK[j][l] = GLWE_S'(s_j * 2^(64 - base_log*(l+1))), native q)
 *     out += X^d * buf               (negacyclic monomial product per polynomial)
 *   compress: every mask coefficient and the first `bodies` body coefficients switched to
 *   storage_log bits (round(x / 2^(64-w))) and bit-packed LSB-first into u64 words; extract: unpack,
 *   << (64 - w), missing body coefficients 0.
 * Parameters: the reference's own PARAMS_8B_2048_NEW (ml/extensions/rust/src/fhext_classes.rs:98-112:
 * input GLWE k=1,N=2048 read as an LWE of dim 2048, pks 2 x 2^14, output k=1,N=2048, storage 26 bits,
 * pks noise stdev 2.845e-15 ~ 2^-48, lwe_per_glwe = N (fhext_classes.rs:130)).  PKSK layout
 * [j][l][(k+1)N] u64; the output GLWE key is binary from ChaCha stream 4 of the seed, PKSK row j from
 * stream 0x300000 + j.  Parity unpinned at ciphertext level (no fixture in the reference). */
typedef struct or_pks_params {
  uint32_t in_dim, out_k, out_N, base_log, level, lwe_per_glwe, storage_log;
  int32_t noise_log2;
} or_pks_params;
int or_pks_params_preset(int preset, or_pks_params* out); /* 0 = PARAMS_8B_2048_NEW */
size_t or_pksk_len(const or_pks_params* pp);              /* in_dim * level * (k+1) * N */
void or_pks_keygen(const or_pks_params* pp, uint64_t seed, const uint64_t* in_key, uint64_t* out_key /* k*N */,
                   uint64_t* pksk);
/* count <= lwe_per_glwe LWEs (count x (in_dim+1)) -> one GLWE ((k+1) x N) */
void or_pks_pack(const or_pks_params* pp, const uint64_t* pksk, const uint64_t* lwes, uint32_t count,
                 uint64_t* glwe);
/* phase polynomial body - sum_c mask_c * S_c over Z_2^64 (N values) */
void or_glwe_phase_native(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out);
size_t or_pks_packed_words(const or_pks_params* pp, uint32_t bodies);
void or_pks_compress(const or_pks_params* pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed);
void or_pks_extract(const or_pks_params* pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe);

/* ---- switch-and-squash / noise squashing to Z_2^128 (sns_oracle.c): the native 2^128 torus --------
 * Coefficients are Z_2^128 words held as two u64 planes per polynomial, [lo][N] then [hi][N]. */
typedef struct or_sns_params {
  uint32_t n, k, N, base_log, level;
  int32_t noise_log2; /* Gaussian integer noise round(N(0,1) * 2^(64 + x)) added to 128-bit bodies */
} or_sns_params;
#define OR_SNS_LIMBS 5 /* limbs of a rounded key word (2^16 x a 112-bit integer): low 48 bits + four 16-bit */
int or_sns_params_preset(int preset, or_sns_params* out); /* 0: n=918 (P-FHEVM small key) k=2 N=2048 2^24x3 */
uint64_t or_sns_prime(int which);                        /* 0: 2^64-2^32+1 (the limb products), 1: 2^64-2^34+1 */
uint64_t or_sns_psi(int which, uint32_t N);
void or_sns_ntt_fwd(int which, uint64_t* a, uint32_t N);
void or_sns_ntt_inv(int which, uint64_t* a, uint32_t N);
size_t or_sns_bsk_len(const or_sns_params* sp);          /* n*(k+1)L*(k+1)*2*N: [i][c*L+l][j][lo, hi][N] */
void or_sns_keygen(const or_sns_params* sp, uint64_t seed, const uint64_t* lwe_key, uint64_t* glwe_key /* k*N */,
                   uint64_t* bsk /* nullable */);
/* load-time rounding of the squashing key to multiples of 2^16 (signed 128-bit words; sns_oracle.c) */
void or_sns_bsk_round(const or_sns_params* sp, const uint64_t* bsk, uint64_t* out);
/* rounded key -> limb spectra [i][r][j][limb][N]: limb 0 (low 48 bits) the f64 spectrum / M as bits, limbs 1..4 NTTs mod prime 0 */
size_t or_sns_limb_ntt_len(const or_sns_params* sp);
void or_sns_bsk_to_limb_ntt(const or_sns_params* sp, const uint64_t* rounded, uint64_t* out);
void or_sns_lut_identity(const or_sns_params* sp, uint32_t msg_modulus, uint64_t* lut /* [lo, hi][N] */);
void or_sns_blind_rotate(const or_sns_params* sp, const uint64_t* bsk_limb, const uint64_t* lwe_small,
                         const uint64_t* lut, uint64_t* acc /* [(k+1)][lo, hi][N] */);
void or_sns_sample_extract(const or_sns_params* sp, const uint64_t* acc, uint64_t* out /* (kN+1) x (lo,hi) */);
void or_sns_squash(const or_sns_params* sp, const uint64_t* bsk_limb, const uint64_t* lwe_small, size_t B,
                   uint32_t msg_modulus, uint64_t* out, int threads);
void or_sns_phase(const or_sns_params* sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count,
                  uint64_t* out);

/* ---- FFT64 transform (fft_oracle.c): tfhe-rs's own external-product arithmetic ------------------
 * tfhe-rs (absent from the mount; npm tfhe/node-tfhe 0.8.7) computes the GGSW x GLWE
 * external product with an f64 FFT over the native 2^64 torus (concrete-fft): the BSK lives in the
 * Fourier domain as N/2 complex doubles per polynomial, digit polynomials are transformed, multiplied
 * pointwise, transformed back and rounded to the torus.  Restated here with ONE fixed f64 operation
 * sequence, which the device kernels (pbs_fft.hip) reproduce bit-for-bit:
 *   fold + twist   z_j = (a_j + i a_{j+N/2}) * zeta^j, zeta = e^{i pi/N}       (j < M = N/2)
 *   DFT            Z_k = sum_j z_j e^{+2 pi i jk/M}: three radix-8 passes (M = 512 = 8 x 8 x 8),
 *                  spectra in DEVICE ORDER: slot d = L + 64 e holds k = (L>>3) + 8 (L&7) + 64 e
 *                  (layout and per-element operation order: fft_oracle.c)
 *   BSK            Fourier(BSK) = DFT(twist((double)(int64)bsk)) * 2^-9     (1/M folded in)
 *   MAC            O_j = sum_r D_r (.) BSK[r][j], r = c*l + lvl in order, 4 fma per complex term
 *   inverse        z'_j = sum_k O_k e^{-2 pi i jk/M} (same passes, conjugate twiddles), untwist by
 *                  conj(zeta^j), coefficient j = Re, j + N/2 = Im, rint (ties to even), mod 2^64
 * Twiddles cos/sin(2 pi t/M) come from fixed series in plain double arithmetic (octant-reduced), so
 * tables are bit-identical on every host.  The accumulator, LUT, BSK (standard domain) and sample
 * extraction are native torus values; the LUT is handed over in the Z_p encoding of the NTT engine
 * (tfhe_hip_lut_*) and mapped back with or_p_to_tor.  Rounding noise of the transform: < 2^-30 of the
 * torus per PBS (tests/test_fft.py measures it against the exact schoolbook product).
 * Parity: GPU == this restatement bit-for-bit; vs tfhe-rs "parity unpinned" like the NTT path. */
typedef struct or_c64 { double re, im; } or_c64;
/* cos(2 pi t / M), sin(2 pi t / M) for 0 <= t < M (M a multiple of 8), fixed-series evaluation */
void or_fft_twiddle(uint32_t t, uint32_t M, double* c, double* s);
/* forward: N real values (exact doubles) -> N/2 complex in device order (see above) */
void or_fft_fwd(const double* a, uint32_t N, or_c64* out);
/* inverse WITHOUT the 1/M factor: N/2 complex in device order -> N doubles (not rounded) */
void or_fft_inv(const or_c64* in, uint32_t N, double* out);
/* round(x) mod 2^64 (ties to even) */
uint64_t or_f64_to_torus(double x);
uint64_t or_f64_to_torus_dev(double x); /* the device's accumulator increment (round 5, see fft_oracle.c) */
/* Fourier BSK: or_bsk_len/N polynomials x N/2 complex, scaled by 2^-log2(N/2) */
void or_bsk_to_fourier(const or_params* p, const uint64_t* bsk, or_c64* bsk_f);
/* acc_out: (k+1)*N native torus values.  lut: N values in the Z_p LUT encoding. */
void or_blind_rotate_fft(const or_params* p, const or_c64* bsk_f, const uint64_t* lwe_in, const uint64_t* lut,
                         uint64_t* acc_out);
void or_sample_extract_torus(const or_params* p, const uint64_t* acc, uint64_t* lwe_big_out);
void or_pbs_batch_fft(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const uint64_t* lwe_in, size_t B,
                      const uint64_t* luts, size_t n_lut, const uint32_t* lut_index, uint64_t* lwe_out, int threads);
void or_pbs_batch_fft_ex(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const or_ms_key* ms,
                         const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                         const uint32_t* lut_index, uint64_t* lwe_out, int threads);
/* fft_batch.c: or_pbs_batch_fft(_ex) for the FFT64 presets (P-GATE, P-FHEVM) with 8 (AVX-512) or 4 (AVX2) ciphertexts per vector,
 * the same operations in the same order (bit-identical outputs); -1 for any other parameter set */
int or_pbs_batch_fft_simd(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const uint64_t* lwe_in, size_t B,
                          const uint64_t* luts, size_t n_lut, const uint32_t* lut_index, uint64_t* lwe_out, int threads);
int or_pbs_batch_fft_simd_ex(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const or_ms_key* ms,
                             const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                             const uint32_t* lut_index, uint64_t* lwe_out, int threads); /* + P-FHEVM FFT64 (order 1) */
int or_fft_batch_lanes(void); /* 8 (AVX-512F) or 4 (AVX2, or ORACLE_SIMD_LANES=4) */
/* exact negacyclic product over Z_2^64 (wrapping): the independent arbiter of the FFT's rounding */
void or_poly_mul_torus_schoolbook(uint64_t* out, const int64_t* a, const uint64_t* b, uint32_t N);
/* the FFT64 blind rotation with every intermediate accumulator: trace = (n + 1) x (k+1)N words, row 0 the initial
 * X^{-b~} LUT, row i + 1 the state after CMUX i */
void or_blind_rotate_fft_trace(const or_params* p, const or_c64* bsk_f, const uint64_t* lwe_in, const uint64_t* lut,
                               uint64_t* trace);

/* ---- exact integer arithmetic over Z_2^64 (exact_oracle.c): the arbiter of the FFT64 path -----------------
 * The external product computed with no floating point: BSK words split into three balanced base-2^22 limbs, each
 * digit x limb product exact through the Goldilocks NTT (|value| <= 2^55 < p/2), recombined mod 2^64.  Equal to the
 * reference's polynomial_wrapping_mul (ml/extensions/rust/src/computations.rs:50-54) by construction. */
typedef struct or_exact_key or_exact_key;
or_exact_key* or_exact_key_new(const or_params* p, const uint64_t* bsk /* standard-domain torus BSK */);
void or_exact_key_free(or_exact_key* K);
/* acc_out[q] = acc_in[q] + ExtProd(BSK_{key_index[q]}, X^{a_tilde[q]} acc_in[q] - acc_in[q]) for q < count.
 * s1, s2 (nullable, count x (k+1)): sum_r ||d_r|| ||w_{r,j}|| and sum_r ||d_r||^2 ||w_{r,j}||^2 (w as signed int64) */
void or_cmux_exact_batch(const or_exact_key* K, size_t count, const uint32_t* key_index, const uint32_t* a_tilde,
                         const uint64_t* acc_in, uint64_t* acc_out, double* s1, double* s2, int threads);
void or_poly_mul_torus_exact(uint64_t* out, const int64_t* a, const uint64_t* b, uint32_t N);
void or_blind_rotate_exact(const or_exact_key* K, const uint64_t* lwe_in, const uint64_t* lut, uint64_t* acc);

/* ---- LUT helpers --------------------------------------------------------------------- */
void or_lut_constant(uint32_t N, uint64_t torus_value, uint64_t* lut); /* gate LUT: every coef = v */
/* tfhe-rs generate_accumulator: box = N/msg_modulus, v[i] = f(i/box)*delta_out, half-box rotation.
 * f_table has msg_modulus entries. */
void or_lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* f_table, uint64_t delta_out,
                       uint64_t* lut);

/* ---- gate bootstrap (P-GATE) --------------------------------------------------------- */
/* NAND: c = (0, 1/8) - c1 - c2 then PBS with LUT == 1/8.  Bits are +-1/8 (true = +1/8). */
void or_nand(const or_params* p, const uint64_t* bsk_ntt, const uint64_t* ksk, const uint64_t* c1,
             const uint64_t* c2, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
