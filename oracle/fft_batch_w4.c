/* fft_batch_w4.c — fft_batch_body.h at 4 lanes (AVX2 + FMA, the oracle's x86-64-v3 build).  TEST INFRASTRUCTURE
 * ONLY (see tfhe_oracle.h). */
#include <immintrin.h>
#define BW 4
#define BR_SIMD or_fftb_blind_rotate_w4
#define BR_SIMD_2K or_fftb_blind_rotate2k_w4
#define VF(a, b, c) ((VD)_mm256_fmadd_pd((__m256d)(a), (__m256d)(b), (__m256d)(c)))
#define VFLOOR(x) ((VD)_mm256_floor_pd((__m256d)(x)))
#define VRINT(x) ((VD)_mm256_round_pd((__m256d)(x), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC))
#include "fft_batch_body.h"
