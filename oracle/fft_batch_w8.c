/* fft_batch_w8.c — fft_batch_body.h at 8 lanes (AVX-512F), compiled for that target whatever the build's -march;
 * fft_batch.c calls it only when the CPU reports avx512f.  TEST INFRASTRUCTURE ONLY (see tfhe_oracle.h). */
#pragma GCC target("avx512f")
#include <immintrin.h>
#define BW 8
#define BR_SIMD or_fftb_blind_rotate_w8
#define BR_SIMD_2K or_fftb_blind_rotate2k_w8
#define VF(a, b, c) ((VD)_mm512_fmadd_pd((__m512d)(a), (__m512d)(b), (__m512d)(c)))
#define VFLOOR(x) ((VD)_mm512_roundscale_pd((__m512d)(x), _MM_FROUND_TO_NEG_INF | _MM_FROUND_NO_EXC))
#define VRINT(x) ((VD)_mm512_roundscale_pd((__m512d)(x), _MM_FROUND_TO_NEAREST_INT | _MM_FROUND_NO_EXC))
#include "fft_batch_body.h"
