// ntt16.h — in-lane 16- and 4-point transforms over Z_p whose twiddles are powers of two.
//
// The N=1024 negacyclic NTT of the blind-rotate loop is factored 16 x (16 x 4) so that every
// butterfly stage runs inside one lane on its 16 registers (pbs_kernels.hip, ntt1024_*):
//   pass 1   negacyclic 16-point, root psi^64 = 2^6 (primitive 32nd root), Kyber-style CT tree:
//            node k multiplies by 2^(6*brv4(k))
//   tw 1     psi^(i' (2 j1 + 1))                         (general multiply, LDS table)
//   pass 2a  cyclic 16-point, root psi^128 = 2^12, CT over X^(2L) - w^(2t) = (X^L - w^t)(X^L + w^t)
//   tw 2     2^(3 i3 j2)                                 (table; a power of two)
//   pass 2b  4 cyclic 4-point transforms, root 2^48
// Multiplying by 2^s is shifts plus one mad-based fold per 32 bits (gl_shl_mod; the sign of
// 2^96 = -1 swaps the butterfly's add and sub): no general multiply inside a pass.  All loops are
// fully unrolled: every index and shift is a compile-time constant.
#pragma once
#include "gl64.h"

namespace tfhe {

__host__ __device__ constexpr int brv_bits(int x, int bits) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}
__host__ __device__ constexpr int brv4(int x) { return brv_bits(x, 4); }
__host__ __device__ constexpr int brv2(int x) { return brv_bits(x, 2); }

// node-k twiddle exponent (2^s) of a CT-tree transform of size 2^logn
//   negacyclic, root r = 2^rexp (primitive 2n-th root):  s = rexp * brv(k)
//   cyclic,     root w = 2^wexp (primitive n-th root):   s = wexp * brv_d(k - 2^d) * (n/2) / 2^d
template <bool NEGA_, int LOGN, int REXP>
__host__ __device__ constexpr int zeta_exp(int k) {
  if (NEGA_) return REXP * brv_bits(k, LOGN);
  int d = 0;
  while ((2 << d) <= k) d++;
  if (d == 0) return 0;
  return REXP * ((brv_bits(k - (1 << d), d) * (1 << (LOGN - 1))) >> d);
}

// Forward CT stages of a 2^LOGN-point transform on x[BASE .. BASE + 2^LOGN), spans FIRST .. 1.
template <bool NEGA_, int LOGN, int REXP, int FIRST, int BASE, int NX>
__host__ __device__ __forceinline__ void ct_fwd(u64 (&x)[NX]) {
  constexpr int n = 1 << LOGN;
#pragma unroll
  for (int ln = FIRST; ln >= 1; ln >>= 1) {
#pragma unroll
    for (int j = 0; j < n; j++) {
      if ((j % (2 * ln)) < ln) {
        const int k = (n / 2) / ln + j / (2 * ln);
        bool neg;  // the sign of the power-of-two twiddle swaps the butterfly's add and sub
        const u64 t = gl_pow2_twiddle(x[BASE + j + ln], zeta_exp<NEGA_, LOGN, REXP>(k), neg);
        const u64 u = x[BASE + j];
        x[BASE + j] = neg ? gl_sub(u, t) : gl_add(u, t);
        x[BASE + j + ln] = neg ? gl_add(u, t) : gl_sub(u, t);
      }
    }
  }
}

// Inverse (Gentleman-Sande) of ct_fwd on the same block, x 2^LOGN.
template <bool NEGA_, int LOGN, int REXP, int BASE, int NX>
__host__ __device__ __forceinline__ void gs_inv(u64 (&x)[NX]) {
  constexpr int n = 1 << LOGN;
#pragma unroll
  for (int ln = 1; ln <= n / 2; ln <<= 1) {
#pragma unroll
    for (int j = 0; j < n; j++) {
      if ((j % (2 * ln)) < ln) {
        const int k = (n / 2) / ln + j / (2 * ln);
        const u64 u = x[BASE + j], v = x[BASE + j + ln];
        const int z = 192 - zeta_exp<NEGA_, LOGN, REXP>(k) % 192;
        bool neg = false;  // sign known at compile time: the subtraction is ordered to absorb it
        (void)gl_pow2_twiddle(0, z, neg);
        x[BASE + j] = gl_add(u, v);
        x[BASE + j + ln] = gl_pow2_twiddle(neg ? gl_sub(v, u) : gl_sub(u, v), z, neg);
      }
    }
  }
}

// pass 1: negacyclic 16-point, root 2^6; output slot e holds the evaluation at 2^(6 (2 brv4(e) + 1))
__host__ __device__ __forceinline__ void nega16_fwd(u64 (&x)[16]) { ct_fwd<true, 4, 6, 8, 0>(x); }
__host__ __device__ __forceinline__ void nega16_fwd_from4(u64 (&x)[16]) { ct_fwd<true, 4, 6, 4, 0>(x); }
__host__ __device__ __forceinline__ void nega16_inv(u64 (&x)[16]) { gs_inv<true, 4, 6, 0>(x); }
// pass 2a: cyclic 16-point, root 2^12; slot f holds the evaluation at 2^(12 brv4(f))
__host__ __device__ __forceinline__ void cyc16_fwd(u64 (&x)[16]) { ct_fwd<false, 4, 12, 8, 0>(x); }
__host__ __device__ __forceinline__ void cyc16_inv(u64 (&x)[16]) { gs_inv<false, 4, 12, 0>(x); }
// pass 2b: four cyclic 4-point transforms (elements 4q .. 4q+3), root 2^48
__host__ __device__ __forceinline__ void cyc4x4_fwd(u64 (&x)[16]) {
  ct_fwd<false, 2, 48, 2, 0>(x);
  ct_fwd<false, 2, 48, 2, 4>(x);
  ct_fwd<false, 2, 48, 2, 8>(x);
  ct_fwd<false, 2, 48, 2, 12>(x);
}
__host__ __device__ __forceinline__ void cyc4x4_inv(u64 (&x)[16]) {
  gs_inv<false, 2, 48, 0>(x);
  gs_inv<false, 2, 48, 4>(x);
  gs_inv<false, 2, 48, 8>(x);
  gs_inv<false, 2, 48, 12>(x);
}

// Natural NTT index (A^[j] = a(psi^(2j+1))) held at (lane, element) after ntt1024_fwd.
__host__ __device__ constexpr int ntt_natural_index(int lane, int elem) {
  return brv4(lane >> 2) + 16 * (brv4(4 * (lane & 3) + (elem >> 2)) + 16 * brv2(elem & 3));
}

}  // namespace tfhe
