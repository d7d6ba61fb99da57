/*
 * fft_batch.c — the FFT64 P-GATE PBS of fft_oracle.c on SIMD lanes: 8 ciphertexts per AVX-512 vector where the CPU
 * has AVX-512F, else 4 per AVX2 vector (ORACLE_SIMD_LANES=4 forces the AVX2 path).
 *
 * TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h): bench.py's cpu_baseline leg times it as the CPU port of the path,
 * and tests/test_fft.py checks it against the scalar restatement; never linked into the product.
 *
 * Why it exists: the scalar restatement (fft_oracle.c) is written to be read -- one ciphertext per thread,
 * array-of-structs complex values -- while tfhe-rs's own CPU path (concrete-fft, absent from the mount) runs
 * vectorised FFTs, so the scalar figure understates a CPU.  This port keeps EVERY floating-point operation of
 * fft_oracle.c in the same order (cmul, dft8, the three passes with the merged twist, the split MAC, the device
 * form of the torus update) and changes only the data layout: lane q of each vector belongs to ciphertext q of
 * the group, every vector operation is BW copies of the scalar one, and the outputs are bit-identical to
 * or_pbs_batch_fft (tests/test_fft.py).  The BSK and twiddles are shared by the lanes (broadcast); the digits and
 * accumulators differ.  fma is the vector fma (one rounding, = C fma) and the build keeps -ffp-contract=off.
 * The keyswitch of a group reads each KSK row once for all of its ciphertexts (the scalar form streams the 41 MB
 * key per ciphertext).
 *
 * Scope: the two FFT64 presets bench.py times -- P-GATE (N = 1024, k = 1, PBS 2^7 x 3, order 0: BR -> SE -> KS; the
 * headline and C3 lines) and P-FHEVM (N = 2048, k = 1, PBS 2^23 x 1, order 1: KS -> MS noise reduction -> BR -> SE);
 * other parameter sets return -1 (the caller keeps the scalar or_pbs_batch_fft_ex).
 */
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "fft_batch_body.h"

void or_fftb_blind_rotate_w4(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe,
                             const uint64_t* const* lut, uint64_t* const* acc_out);
void or_fftb_blind_rotate_w8(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe,
                             const uint64_t* const* lut, uint64_t* const* acc_out);
void or_fftb_blind_rotate2k_w4(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe,
                               const uint64_t* const* lut, uint64_t* const* acc_out);
void or_fftb_blind_rotate2k_w8(const or_params* p, const or_c64* bsk_f, const uint64_t* const* lwe,
                               const uint64_t* const* lut, uint64_t* const* acc_out);

int or_fft_batch_lanes(void) {
  const char* e = getenv("ORACLE_SIMD_LANES");
  if (e && atoi(e) == 4) return 4;
  __builtin_cpu_init();
  return __builtin_cpu_supports("avx512f") ? 8 : 4;
}

static or_fftb_tab g_t4;
static int g_t4_ready = 0;
const or_fftb_tab* or_fftb_tables(void) {
#pragma omp critical(or_fft_or_fftb_tab)
  {
    if (!g_t4_ready) {
      for (uint32_t e = 0; e < 8; e++) or_fft_twiddle(64 * e, 2 * N4, &g_t4.tw64[e].re, &g_t4.tw64[e].im);
      for (uint32_t e = 0; e < 8; e++)
        for (uint32_t L = 0; L < 64; L++) {
          or_fft_twiddle((8 * (L & 7) * e) % M4, M4, &g_t4.twB[e][L].re, &g_t4.twB[e][L].im);
          or_fft_twiddle((L * (1 + 4 * e)) % (4 * M4), 4 * M4, &g_t4.twAm[e][L].re, &g_t4.twAm[e][L].im);
          or_fft_twiddle((((L & 7) + 8 * e) * (4 * (L >> 3) + 1)) % (4 * M4), 4 * M4, &g_t4.twIm[e][L].re,
                         &g_t4.twIm[e][L].im);
        }
      __atomic_store_n(&g_t4_ready, 1, __ATOMIC_RELEASE);
    }
  }
  return &g_t4;
}


static or_fftb_tab1k g_t1k;
static int g_t1k_ready = 0;
const or_fftb_tab1k* or_fftb_tables1k(void) {
#pragma omp critical(or_fft_tab1k_simd)
  {
    if (!g_t1k_ready) {
      for (uint32_t e = 0; e < 16; e++) or_fft_twiddle(64 * e, 4096, &g_t1k.slot[e].re, &g_t1k.slot[e].im);
      for (uint32_t k = 0; k < 16; k++)
        for (uint32_t L = 0; L < 64; L++)
          or_fft_twiddle((L * (1 + 4 * k)) % 4096, 4096, &g_t1k.ta[k][L].re, &g_t1k.ta[k][L].im);
      for (uint32_t m = 0; m < 4; m++)
        for (uint32_t l = 0; l < 16; l++)
          or_fft_twiddle((64 * l * m) % 4096, 4096, &g_t1k.tb[m][l].re, &g_t1k.tb[m][l].im);
      __atomic_store_n(&g_t1k_ready, 1, __ATOMIC_RELEASE);
    }
  }
  return &g_t1k;
}

/* or_keyswitch on the G inputs of a group at once: each KSK row is read once for the group (the scalar form streams the 41 MB
 * key per ciphertext).  Digits of base 2^2 lie in [-2, 2], so m * row is +-(row << (|m| - 1)) mod 2^64 -- the same
 * words; other digit sizes multiply. */
static void keyswitch_group(const or_params* p, const uint64_t* ksk, const uint64_t* in, size_t in_stride, int G,
                            uint64_t* out) {
  const uint32_t n = p->n, big = p->k * p->N, L = p->ks_level;
  const size_t dout = (size_t)n + 1;
  memset(out, 0, (size_t)G * dout * 8);
  for (int q = 0; q < G; q++) out[q * dout + n] = in[q * in_stride + big];
  int64_t d[8][64];
  for (uint32_t j = 0; j < big; j++) {
    for (int q = 0; q < G; q++) or_decompose(in[q * in_stride + j], p->ks_base_log, L, d[q]);
    for (uint32_t l = 0; l < L; l++) {
      const uint64_t* kr = ksk + ((size_t)j * L + l) * dout;
      for (int q = 0; q < G; q++) {
        const int64_t m = d[q][l];
        uint64_t* o = out + q * dout;
        if (m == 1) for (uint32_t c = 0; c < n; c++) o[c] -= kr[c];
        else if (m == -1) for (uint32_t c = 0; c < n; c++) o[c] += kr[c];
        else if (m == 2) for (uint32_t c = 0; c < n; c++) o[c] -= kr[c] << 1;
        else if (m == -2) for (uint32_t c = 0; c < n; c++) o[c] += kr[c] << 1;
        else if (m) for (uint32_t c = 0; c < n; c++) o[c] -= (uint64_t)m * kr[c];
        if (m) o[n] -= (uint64_t)m * kr[n];
      }
    }
  }
}

/* P-FHEVM FFT64 (order 1): per group, the keyswitch of the big inputs (each KSK row once), the modulus-switch noise
 * reduction per ciphertext (or_ms_reduce, scalar), the blind rotation on the lanes and sample extraction */
static int pbs_batch_2k(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const or_ms_key* ms,
                        const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut, const uint32_t* lut_index,
                        uint64_t* lwe_out, int threads) {
  enum { N2 = 2048 };
  const int G = or_fft_batch_lanes();
  const size_t big = (size_t)N2 + 1, small = (size_t)p->n + 1, groups = (B + G - 1) / G;
  or_fftb_tables1k();
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
  for (size_t g = 0; g < groups; g++) {
    const uint64_t* lwe[8];
    const uint64_t* lut[8];
    uint64_t* acc[8];
    uint64_t* mem = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)G * (2 * N2 + big + small));
    uint64_t* in = mem + (size_t)G * 2 * N2;
    uint64_t* sm = in + (size_t)G * big;
    for (int q = 0; q < G; q++) {
      size_t b = G * g + q;
      if (b >= B) b = B - 1; /* ragged group: the last ciphertext again, its copy not stored */
      size_t li = lut_index ? lut_index[b] : 0;
      if (li >= n_lut) li = 0;
      memcpy(in + q * big, lwe_in + b * big, big * 8);
      lwe[q] = sm + q * small;
      lut[q] = luts + li * N2;
      acc[q] = mem + (size_t)q * 2 * N2;
    }
    keyswitch_group(p, ksk, in, big, G, sm);
    if (ms)
      for (int q = 0; q < G; q++) or_ms_reduce(p, ms, sm + q * small);
    if (G == 8) or_fftb_blind_rotate2k_w8(p, bsk_f, lwe, lut, acc);
    else or_fftb_blind_rotate2k_w4(p, bsk_f, lwe, lut, acc);
    for (int q = 0; q < G && G * g + q < B; q++) or_sample_extract_torus(p, acc[q], lwe_out + (G * g + q) * big);
    free(mem);
  }
  (void)threads;
  return 0;
}

int or_pbs_batch_fft_simd(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const uint64_t* lwe_in, size_t B,
                          const uint64_t* luts, size_t n_lut, const uint32_t* lut_index, uint64_t* lwe_out, int threads) {
  return or_pbs_batch_fft_simd_ex(p, bsk_f, ksk, NULL, lwe_in, B, luts, n_lut, lut_index, lwe_out, threads);
}

int or_pbs_batch_fft_simd_ex(const or_params* p, const or_c64* bsk_f, const uint64_t* ksk, const or_ms_key* ms,
                             const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                             const uint32_t* lut_index, uint64_t* lwe_out, int threads) {
  if (p->transform == 1 && p->order == 1 && p->N == 2048 && p->k == 1 && p->pbs_base_log == 23 && p->pbs_level == 1)
    return B ? pbs_batch_2k(p, bsk_f, ksk, ms, lwe_in, B, luts, n_lut, lut_index, lwe_out, threads) : 0;
  if (p->transform != 1 || p->order != 0 || p->N != N4 || p->k != 1 || p->pbs_base_log != 7 || p->pbs_level != 3)
    return -1;
  if (B == 0) return 0;
  const int G = or_fft_batch_lanes();
  const size_t din = (size_t)p->n + 1, big = (size_t)N4 + 1, groups = (B + G - 1) / G;
  or_fftb_tables();
#ifdef _OPENMP
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
#endif
  for (size_t g = 0; g < groups; g++) {
    const uint64_t* lwe[8];
    const uint64_t* lut[8];
    uint64_t* acc[8];
    uint64_t* mem = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)G * (2 * N4 + big + din));
    for (int q = 0; q < G; q++) {
      size_t b = G * g + q;
      if (b >= B) b = B - 1; /* ragged group: the last ciphertext again, its copy not stored */
      size_t li = lut_index ? lut_index[b] : 0;
      if (li >= n_lut) li = 0;
      lwe[q] = lwe_in + b * din;
      lut[q] = luts + li * N4;
      acc[q] = mem + (size_t)q * 2 * N4;
    }
    if (G == 8) or_fftb_blind_rotate_w8(p, bsk_f, lwe, lut, acc);
    else or_fftb_blind_rotate_w4(p, bsk_f, lwe, lut, acc);
    uint64_t* ext = mem + (size_t)G * 2 * N4;
    uint64_t* ksout = ext + (size_t)G * big;
    for (int q = 0; q < G; q++) or_sample_extract_torus(p, acc[q], ext + q * big);
    keyswitch_group(p, ksk, ext, big, G, ksout);
    for (int q = 0; q < G && G * g + q < B; q++) memcpy(lwe_out + (G * g + q) * din, ksout + q * din, din * 8);
    free(mem);
  }
  (void)threads;
  return 0;
}
