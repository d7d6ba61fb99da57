// ntt32.h — 32-point transforms over Z_p whose twiddles are powers of two, split over a lane pair.
//
// The N=1024 negacyclic NTT of the blind-rotate loop is factored 32 x 32 (see ntt1024 in
// pbs_kernels.hip):
//   pass A  negacyclic 32-point NTT, rho = psi^32 = 2^3 (primitive 64th root), Kyber-style
//           Cooley-Tukey: node k multiplies by rho^brv5(k)
//   twiddle psi^(i2 * (2*j1 + 1))                  (the only general multiplies: 1,024 per poly)
//   pass B  cyclic 32-point NTT, omega = psi^64 = 2^6, Cooley-Tukey over the factor tree
//           X^(2L) - w^(2t) = (X^L - w^t)(X^L + w^t): node k multiplies by omega^(t_k / 2)
// Both passes multiply only by 2^s (gl_mul_pow2): shifts and a 96/128-bit fold.
//
// Lane layout ("R16"): a 32-point sub-transform lives on the lane pair (L, L^32); lane half s
// holds positions p = 2e + s, e < 16.  Butterfly stages with span >= 2 pair elements of the SAME
// lane and the twiddle depends only on the block (lane-uniform, compile-time); the span-1 stage
// pairs the two lanes (cross-lane, in pbs_kernels.hip).
//
// All loops are fully unrolled: every index and shift is a compile-time constant.
#pragma once
#include "gl64.h"

namespace tfhe {

__host__ __device__ constexpr int brv5(int x) {
  return ((x & 1) << 4) | ((x & 2) << 2) | (x & 4) | ((x & 8) >> 2) | ((x & 16) >> 4);
}

__host__ __device__ constexpr int brv_bits(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

enum { NEGA = 0, CYC = 1 };

// exponent s of the node-k twiddle 2^s (k = 1..31)
template <int KIND>
__host__ __device__ constexpr int zeta_exp(int k) {
  if (KIND == NEGA) return 3 * brv5(k);
  int d = 0;
  while ((2 << d) <= k) d++;  // depth: k in [2^d, 2^(d+1))
  if (d == 0) return 0;
  return 6 * ((brv_bits(k - (1 << d), d) * 16) >> d);
}

// In-lane forward stages (spans FIRST, ..., 2 of the 32-point transform) on the 16 local values.
template <int KIND, int FIRST>
__host__ __device__ __forceinline__ void fwd_inlane16_from(u64 (&x)[16]) {
#pragma unroll
  for (int ln = FIRST; ln >= 2; ln >>= 1) {
#pragma unroll
    for (int e = 0; e < 16; e++) {
      if ((e % ln) < ln / 2) {
        const int k = 16 / ln + e / ln;
        const u64 t = gl_mul_pow2(x[e + ln / 2], zeta_exp<KIND>(k));
        x[e + ln / 2] = gl_sub(x[e], t);
        x[e] = gl_add(x[e], t);
      }
    }
  }
}

template <int KIND>
__host__ __device__ __forceinline__ void fwd_inlane16(u64 (&x)[16]) {
  fwd_inlane16_from<KIND, 16>(x);
}

// In-lane inverse stages (spans 2, 4, 8, 16), Gentleman-Sande, each stage x2.
template <int KIND>
__host__ __device__ __forceinline__ void inv_inlane16(u64 (&x)[16]) {
#pragma unroll
  for (int ln = 2; ln <= 16; ln <<= 1) {
#pragma unroll
    for (int e = 0; e < 16; e++) {
      if ((e % ln) < ln / 2) {
        const int k = 16 / ln + e / ln;
        const u64 u = x[e], v = x[e + ln / 2];
        x[e] = gl_add(u, v);
        x[e + ln / 2] = gl_mul_pow2(gl_sub(u, v), 192 - zeta_exp<KIND>(k));
      }
    }
  }
}

}  // namespace tfhe
