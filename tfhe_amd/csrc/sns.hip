// sns.hip — switch-and-squash / noise squashing (rule: oracle/sns_oracle.c).
//
// A P-FHEVM small-key ciphertext (after keyswitch + modulus-switch noise reduction) is bootstrapped
// with a BSK under a 128-bit GLWE key (k = 2, N = 2048, 2^24 x 3) and the identity LUT; the output is
// an LWE over Z_2^128 (dim 4096) with ~2^-63 noise.  The GLWE ring is Z_Q, Q = p1 p2 (p1 = 2^64-2^32+1,
// p2 = 2^64-2^34+1), as residues; arithmetic per prime is Montgomery (R = 2^64).
//
// Work shape: the accumulator (3 polys x 2 primes x 2048 = 96 KB per ciphertext) lives in HBM; each
// CMUX is two launches over the batch:
//   sns_step1  (ciphertext, component c): X^{a_i} acc - acc, CRT lift to [0, Q), map to the torus,
//              signed 2^24 x 3 digits, forward NTT of each digit polynomial in both primes (LDS)
//   sns_step2  (ciphertext, output component j, prime): MAC of the 9 digit spectra with BSK_i
//              (NTT domain, Montgomery form), inverse NTT, acc += .
// NTTs are the negacyclic Cooley-Tukey / Gentleman-Sande pair with bit-reversed psi tables (input
// natural -> spectrum bit-reversed -> natural), 2048 points in LDS, 256 threads.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "pbs_kernels.h"
#include "sns_fft.h"

namespace tfhe {
namespace {

typedef unsigned __int128 u128;
constexpr int SN = 2048, SK = 2, SL = 3, SR = (SK + 1) * SL, ST = 256;

struct SnsConst {
  u64 p[2], pinv_neg[2], r2[2];
  u64 psi_rev[2][SN];   // psi^bitrev(i) * R mod p
  u64 ipsi_rev[2][SN];  // psi^-bitrev(i) * R mod p
  u64 ninv[2];          // N^-1 * R mod p
  u64 p1inv_m;          // p1^-1 * R mod p2
  u64 conv_lo, conv_hi;  // floor(2^256 / Q) - 2^128
};

__device__ __forceinline__ u64 mont(u64 a, u64 b, u64 p, u64 pinv) {
  const u128 t = (u128)a * b;
  const u64 m = (u64)t * pinv;
  const u128 mp = (u128)m * p;
  const u64 hi_t = (u64)(t >> 64), hi_mp = (u64)(mp >> 64);
  const u64 c = (u64)t != 0;
  u64 s = hi_t + hi_mp;
  const bool ov1 = s < hi_t;
  const u64 s2 = s + c;
  const bool ov = ov1 || s2 < s;
  return (ov || s2 >= p) ? s2 - p : s2;
}
__device__ __forceinline__ u64 addm(u64 a, u64 b, u64 p) {
  const u64 s = a + b;
  return (s < a || s >= p) ? s - p : s;
}
__device__ __forceinline__ u64 subm(u64 a, u64 b, u64 p) { return a >= b ? a - b : a + (p - b); }

// The two primes as compile-time constants (prime-specialised Montgomery: with p = 2^64 - 2^a + 1 a
// constant, the m * p product folds into shifts and adds — 21 instead of 30 VALU per product,
// measured on the ISA); P_Q / PINV_Q equal SnsConst.p / pinv_neg (make_sns_const, checked there)
template <int Q>
struct Prime;
template <>
struct Prime<0> {
  static constexpr u64 p = 0xFFFFFFFF00000001ull, pinv = 0xFFFFFFFEFFFFFFFFull;
};
template <>
struct Prime<1> {
  static constexpr u64 p = 0xFFFFFFFC00000001ull, pinv = 0xFFFFFFFBFFFFFFFFull;
};
template <int Q>
__device__ __forceinline__ u64 mont_q(u64 a, u64 b) { return mont(a, b, Prime<Q>::p, Prime<Q>::pinv); }
template <int Q>
constexpr u64 prime_r2() {  // R^2 mod p (R = 2^64 = 2^64 - p mod p)
  return (u64)(((u128)((u64)0 - Prime<Q>::p) * (u128)((u64)0 - Prime<Q>::p)) % Prime<Q>::p);
}
template <int Q>
constexpr u64 prime_pow2(int e) {  // 2^e mod p
  u64 r = 1;
  for (int i = 0; i < e; i++) r = (u64)(((u128)r * 2) % Prime<Q>::p);
  return r;
}
template <int Q>
__device__ __forceinline__ u64 addm_q(u64 a, u64 b) { return addm(a, b, Prime<Q>::p); }
template <int Q>
__device__ __forceinline__ u64 subm_q(u64 a, u64 b) { return subm(a, b, Prime<Q>::p); }

__device__ __forceinline__ u128 mulhi128(u128 x, u128 y) {
  const u64 x0 = (u64)x, x1 = (u64)(x >> 64), y0 = (u64)y, y1 = (u64)(y >> 64);
  const u128 p00 = (u128)x0 * y0, p01 = (u128)x0 * y1, p10 = (u128)x1 * y0, p11 = (u128)x1 * y1;
  const u128 mid = (p00 >> 64) + (u64)p01 + (u64)p10;
  return p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

// residues -> x in [0, Q) (Garner)
__device__ __forceinline__ u128 crt_x(u64 r1, u64 r2, const SnsConst& K) {
  constexpr u64 p1 = Prime<0>::p, p2 = Prime<1>::p;
  const u64 r1m = r1 >= p2 ? r1 - p2 : r1;
  const u64 t = mont_q<1>(subm_q<1>(r2, r1m), K.p1inv_m);
  return (u128)r1 + (u128)p1 * t;
}

// signed v, |v| < 2^127 - 2^96 -> v mod p
template <int Q>
__device__ __forceinline__ u64 reduce_s128(__int128 v) {
  constexpr u64 p = Prime<Q>::p;
  const u128 u = (u128)(v + ((__int128)p << 63));
  u64 hi = (u64)(u >> 64), lo = (u64)u;
  if (hi >= p) hi -= p;
  if (lo >= p) lo -= p;
  return addm_q<Q>(lo, mont_q<Q>(hi, prime_r2<Q>()));
}

// the load-time key rounding (oracle: or_sns_bsk_round): x centred in (-Q/2, Q/2], rounded to the
// nearest multiple of 2^SF_DROP; returns x' / 2^SF_DROP (a signed 112-bit integer)
__device__ __forceinline__ __int128 round_key(u64 r1, u64 r2, const SnsConst& K) {
  constexpr u128 Qv = (u128)Prime<0>::p * Prime<1>::p;
  const u128 x = crt_x(r1, r2, K);
  const __int128 xc = x > (Qv >> 1) ? (__int128)(x - Qv) : (__int128)x;
  return (xc + ((__int128)1 << (snsf::SF_DROP - 1))) >> snsf::SF_DROP;
}

// residues -> x in [0, Q) -> torus y = x + floor((x c + 2^127) / 2^128)
__device__ __forceinline__ u128 lift_to_torus(u64 r1, u64 r2, const SnsConst& K) {
  const u128 x = crt_x(r1, r2, K);
  const u128 c = ((u128)K.conv_hi << 64) | K.conv_lo;
  const u128 lo = x * c;
  return x + mulhi128(x, c) + (u128)((lo >> 127) & 1);
}

// Negacyclic NTTs of 2048 points in LDS by 256 threads, the radix-2 stages grouped in registers: each
// thread takes an 8-element set closed under 3 consecutive stages (7 twiddles), so a transform is 4 LDS
// passes and 4 barriers instead of 11 (the last / first pass of 2 stages takes two 4-element sets).
// Cooley-Tukey forward (psi_rev, natural -> bit-reversed) and Gentleman-Sande inverse (ipsi_rev,
// bit-reversed -> natural, N^-1 folded into the last pass); the same butterflies as the stage-by-stage
// form, so the same exact residues.
template <int Q>
__device__ __forceinline__ void ct_bfly(u64& u, u64& v, u64 S) {
  const u64 V = mont_q<Q>(v, S);
  v = subm_q<Q>(u, V);
  u = addm_q<Q>(u, V);
}
template <int Q>
__device__ __forceinline__ void gs_bfly(u64& u, u64& v, u64 S) {
  const u64 U = u, V = v;
  u = addm_q<Q>(U, V);
  v = mont_q<Q>(subm_q<Q>(U, V), S);
}

// CT stages (m, t), (2m, t/2), (4m, t/4) on the set 2 i t + j + k t/4, k < 8
template <int Q, int M, int T>
__device__ __forceinline__ void ct_pass3(u64* a, const u64* __restrict__ tw) {
  constexpr int Q4 = T / 4;
  const int th = threadIdx.x, i = th / Q4, j = th % Q4;
  u64* base = a + 2 * i * T + j;
  u64 x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = base[k * Q4];
  const u64 s1 = tw[M + i], s2a = tw[2 * M + 2 * i], s2b = tw[2 * M + 2 * i + 1];
  const u64 s3[4] = {tw[4 * M + 4 * i], tw[4 * M + 4 * i + 1], tw[4 * M + 4 * i + 2], tw[4 * M + 4 * i + 3]};
#pragma unroll
  for (int k = 0; k < 4; k++) ct_bfly<Q>(x[k], x[k + 4], s1);
  ct_bfly<Q>(x[0], x[2], s2a);
  ct_bfly<Q>(x[1], x[3], s2a);
  ct_bfly<Q>(x[4], x[6], s2b);
  ct_bfly<Q>(x[5], x[7], s2b);
#pragma unroll
  for (int s = 0; s < 4; s++) ct_bfly<Q>(x[2 * s], x[2 * s + 1], s3[s]);
#pragma unroll
  for (int k = 0; k < 8; k++) base[k * Q4] = x[k];
  __syncthreads();
}

template <int Q>
__device__ void ntt_fwd_lds(u64* a, const u64* tw) {
  static_assert(SN == 2048 && ST == 256, "pass plan");
  ct_pass3<Q, 1, 1024>(a, tw);
  ct_pass3<Q, 8, 128>(a, tw);
  ct_pass3<Q, 64, 16>(a, tw);
  // stages (512, 2), (1024, 1): sets 4 i + k, k < 4, two per thread
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int i = threadIdx.x + r * ST;
    u64* base = a + 4 * i;
    u64 x0 = base[0], x1 = base[1], x2 = base[2], x3 = base[3];
    const u64 s1 = tw[512 + i];
    ct_bfly<Q>(x0, x2, s1);
    ct_bfly<Q>(x1, x3, s1);
    ct_bfly<Q>(x0, x1, tw[1024 + 2 * i]);
    ct_bfly<Q>(x2, x3, tw[1024 + 2 * i + 1]);
    base[0] = x0;
    base[1] = x1;
    base[2] = x2;
    base[3] = x3;
  }
  __syncthreads();
}

// GS stages (t, m), (2t, m/2), (4t, m/4) on the set 8 i t + j + k t, k < 8 (i = block index at m/4)
template <int Q, int M, int T, bool NINV>
__device__ __forceinline__ void gs_pass3(u64* a, const u64* __restrict__ itw, u64 ninv) {
  const int th = threadIdx.x, i = th / T, j = th % T;
  u64* base = a + 8 * i * T + j;
  u64 x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = base[k * T];
  const u64 s1[4] = {itw[M + 4 * i], itw[M + 4 * i + 1], itw[M + 4 * i + 2], itw[M + 4 * i + 3]};
  const u64 s2a = itw[M / 2 + 2 * i], s2b = itw[M / 2 + 2 * i + 1], s3 = itw[M / 4 + i];
#pragma unroll
  for (int s = 0; s < 4; s++) gs_bfly<Q>(x[2 * s], x[2 * s + 1], s1[s]);
  gs_bfly<Q>(x[0], x[2], s2a);
  gs_bfly<Q>(x[1], x[3], s2a);
  gs_bfly<Q>(x[4], x[6], s2b);
  gs_bfly<Q>(x[5], x[7], s2b);
#pragma unroll
  for (int k = 0; k < 4; k++) gs_bfly<Q>(x[k], x[k + 4], s3);
#pragma unroll
  for (int k = 0; k < 8; k++) base[k * T] = NINV ? mont_q<Q>(x[k], ninv) : x[k];
  __syncthreads();
}

template <int Q>
__device__ void ntt_inv_lds(u64* a, const u64* itw, u64 ninv) {
  static_assert(SN == 2048 && ST == 256, "pass plan");
  // stages (t 1, m 1024), (t 2, m 512): sets 4 i + k, two per thread
#pragma unroll
  for (int r = 0; r < 2; r++) {
    const int i = threadIdx.x + r * ST;
    u64* base = a + 4 * i;
    u64 x0 = base[0], x1 = base[1], x2 = base[2], x3 = base[3];
    gs_bfly<Q>(x0, x1, itw[1024 + 2 * i]);
    gs_bfly<Q>(x2, x3, itw[1024 + 2 * i + 1]);
    const u64 s2 = itw[512 + i];
    gs_bfly<Q>(x0, x2, s2);
    gs_bfly<Q>(x1, x3, s2);
    base[0] = x0;
    base[1] = x1;
    base[2] = x2;
    base[3] = x3;
  }
  __syncthreads();
  gs_pass3<Q, 256, 4, false>(a, itw, ninv);
  gs_pass3<Q, 32, 32, false>(a, itw, ninv);
  gs_pass3<Q, 4, 256, true>(a, itw, ninv);
}

__device__ __forceinline__ u32 mod_switch_4096(u64 x) { return (u32)(((x >> 51) + 1) >> 1) & 4095u; }

// BSK standard domain -> NTT domain (bit-reversed) in Montgomery form; one polynomial per workgroup
__global__ void __launch_bounds__(ST) sns_bsk_to_ntt_kernel(const u64* __restrict__ in, u64* __restrict__ out,
                                                            const SnsConst* __restrict__ Kc) {
  __shared__ u64 a[SN];
  const size_t poly = blockIdx.x;
  const int q = (int)(poly & 1);  // [..][prime][N]
  const SnsConst& K = *Kc;
  // the load-time rounding (round_key) needs both residues of each coefficient: the pair's other poly
  const u64* pr = in + (poly & ~(size_t)1) * SN;
  for (int x = threadIdx.x; x < SN; x += ST) {
    const __int128 v = round_key(pr[x], pr[SN + x], K) * ((__int128)1 << snsf::SF_DROP);
    a[x] = q ? reduce_s128<1>(v) : reduce_s128<0>(v);
  }
  __syncthreads();
  if (q) {
    ntt_fwd_lds<1>(a, K.psi_rev[1]);
    for (int x = threadIdx.x; x < SN; x += ST) out[poly * SN + x] = mont_q<1>(a[x], K.r2[1]);
  } else {
    ntt_fwd_lds<0>(a, K.psi_rev[0]);
    for (int x = threadIdx.x; x < SN; x += ST) out[poly * SN + x] = mont_q<0>(a[x], K.r2[0]);
  }
}

// acc = X^{-b~} (0, 0, lut)
__global__ void sns_init_kernel(const u64* __restrict__ lwe, int n, const u64* __restrict__ lut, u64* __restrict__ acc,
                                const SnsConst* __restrict__ Kc) {
  const int ct = blockIdx.x;
  const SnsConst& K = *Kc;
  const u32 bt = mod_switch_4096(lwe[(size_t)ct * (n + 1) + n]);
  const u32 sh = (4096u - bt) & 4095u;
  u64* a = acc + (size_t)ct * (SK + 1) * 2 * SN;
  for (int x = threadIdx.x; x < SK * 2 * SN; x += blockDim.x) a[x] = 0;
  for (int x = threadIdx.x; x < 2 * SN; x += blockDim.x) {
    const int q = x / SN, t = x % SN;
    u32 dst = (u32)t + sh;
    bool neg = false;
    if (dst >= 4096u) dst -= 4096u;
    if (dst >= (u32)SN) {
      dst -= SN;
      neg = true;
    }
    const u64 v = lut[x];
    a[(size_t)SK * 2 * SN + (size_t)q * SN + dst] = (neg && v) ? K.p[q] - v : v;
  }
}

// one digit polynomial of step 1 in prime Q: residues, forward NTT, out
template <int Q>
__device__ __forceinline__ void step1_level(const int* dg, u64* buf, const SnsConst& K, u64* out) {
  for (int t = threadIdx.x; t < SN; t += ST) {
    const int d = dg[t];
    buf[t] = d >= 0 ? (u64)d : Prime<Q>::p - (u64)(-d);
  }
  __syncthreads();
  ntt_fwd_lds<Q>(buf, K.psi_rev[Q]);
  for (int t = threadIdx.x; t < SN; t += ST) out[t] = buf[t];
  __syncthreads();
}

// step 1 of CMUX i for (ciphertext ct, component c): X^{a_i} acc_c - acc_c, CRT lift, torus map, 3 digit
// levels, forward NTT of each in both primes -> D; shared scratch rot (2 x N u64), dig (3 x N int), buf (N u64)
__device__ void step1_digits(const u64* __restrict__ lwe, int n, int i, const u64* __restrict__ acc,
                             const SnsConst& K, int ct, int c, u64 (*rot)[SN], int (*dig)[SN]) {
  const u32 ai = mod_switch_4096(lwe[(size_t)ct * (n + 1) + i]);
  const u64* a = acc + ((size_t)ct * (SK + 1) + c) * 2 * SN;
  for (int x = threadIdx.x; x < 2 * SN; x += ST) {
    const int q = x / SN, t = x % SN;
    u32 dst = (u32)t + ai;
    bool neg = false;
    if (dst >= 4096u) dst -= 4096u;
    if (dst >= (u32)SN) {
      dst -= SN;
      neg = true;
    }
    const u64 v = a[x];
    rot[q][dst] = (neg && v) ? K.p[q] - v : v;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < SN; t += ST) {
    const u64 r1 = subm_q<0>(rot[0][t], a[t]);
    const u64 r2 = subm_q<1>(rot[1][t], a[SN + t]);
    // signed decomposition of the torus image: 72 bits, 3 digits of 24 (tfhe-rs SignedDecomposer)
    const u128 y = lift_to_torus(r1, r2, K);
    u128 state = ((y >> 55) + 1) >> 1;
    state &= ((u128)1 << 72) - 1;
    for (int l = SL - 1; l >= 0; l--) {
      const u64 res = (u64)state & 0xFFFFFFull;
      state >>= 24;
      const u64 carry = ((((res - 1) | (u64)state) & res) >> 23) & 1;
      state += carry;
      dig[l][t] = (int)((long long)res - (long long)(carry << 24));
    }
  }
  __syncthreads();
}

__device__ void step1_body(const u64* __restrict__ lwe, int n, int i, const u64* __restrict__ acc,
                           u64* __restrict__ D, const SnsConst& K, int ct, int c, u64 (*rot)[SN], int (*dig)[SN],
                           u64* buf) {
  step1_digits(lwe, n, i, acc, K, ct, c, rot, dig);
  for (int l = 0; l < SL; l++) {
    step1_level<0>(dig[l], buf, K, D + (((size_t)ct * SR + c * SL + l) * 2 + 0) * SN);
    step1_level<1>(dig[l], buf, K, D + (((size_t)ct * SR + c * SL + l) * 2 + 1) * SN);
  }
}

__global__ void __launch_bounds__(ST) sns_step1_kernel(const u64* __restrict__ lwe, int n, int i,
                                                       const u64* __restrict__ acc, u64* __restrict__ D,
                                                       const SnsConst* __restrict__ Kc) {
  __shared__ u64 rot[2][SN];
  __shared__ int dig[SL][SN];
  __shared__ u64 buf[SN];
  step1_body(lwe, n, i, acc, D, *Kc, blockIdx.x / (SK + 1), blockIdx.x % (SK + 1), rot, dig, buf);
}

// step 2 for prime Q: 9-term MAC, inverse NTT, accumulate
template <int Q>
__device__ __forceinline__ void step2_body(const u64* __restrict__ D, const u64* __restrict__ bsk_i,
                                           u64* __restrict__ acc, const SnsConst& K, u64* buf, int j, int ct) {
  const u64* d = D + (size_t)ct * SR * 2 * SN + (size_t)Q * SN;
  const u64* b = bsk_i + ((size_t)j * 2 + Q) * SN;  // [r][j][prime][N]
  for (int t = threadIdx.x; t < SN; t += ST) {
    u64 s = 0;
#pragma unroll
    for (int r = 0; r < SR; r++) s = addm_q<Q>(s, mont_q<Q>(d[(size_t)r * 2 * SN + t], b[(size_t)r * (SK + 1) * 2 * SN + t]));
    buf[t] = s;
  }
  __syncthreads();
  ntt_inv_lds<Q>(buf, K.ipsi_rev[Q], K.ninv[Q]);
  u64* a = acc + (((size_t)ct * (SK + 1) + j) * 2 + Q) * SN;
  for (int t = threadIdx.x; t < SN; t += ST) a[t] = addm_q<Q>(a[t], buf[t]);
}

__global__ void __launch_bounds__(ST) sns_step2_kernel(const u64* __restrict__ D, const u64* __restrict__ bsk_i,
                                                       u64* __restrict__ acc, const SnsConst* __restrict__ Kc) {
  __shared__ u64 buf[SN];
  const int q = blockIdx.x & 1, j = (blockIdx.x >> 1) % (SK + 1), ct = (blockIdx.x >> 1) / (SK + 1);
  if (q) step2_body<1>(D, bsk_i, acc, *Kc, buf, j, ct);
  else step2_body<0>(D, bsk_i, acc, *Kc, buf, j, ct);
}

// The whole squash blind rotation of one ciphertext in ONE launch (TFHE_HIP_SNS_FUSED=1; not the
// default — see launch_sns_blind_rotate): a workgroup per ciphertext walks the CMUX loop, step 1 for the 3 components then step 2 for the 6 (output, prime) pairs, workgroup barriers
// between; D and acc stay in global memory (per-ciphertext 288 KB + 96 KB, cache-resident), the BSK row of
// CMUX i is shared by all resident workgroups through L2.  Same arithmetic as the two-kernel loop.
__global__ void __launch_bounds__(ST) sns_fused_kernel(const u64* __restrict__ lwe, int n,
                                                       const u64* __restrict__ bsk_ntt, u64* __restrict__ acc,
                                                       u64* __restrict__ D, const SnsConst* __restrict__ Kc) {
  __shared__ u64 rot[2][SN];
  __shared__ int dig[SL][SN];
  __shared__ u64 buf[SN];
  const SnsConst& K = *Kc;
  const int ct = blockIdx.x;
  const size_t bsk_row = (size_t)SR * (SK + 1) * 2 * SN;
  for (int i = 0; i < n; i++) {
    for (int c = 0; c <= SK; c++) step1_body(lwe, n, i, acc, D, K, ct, c, rot, dig, buf);
    const u64* bsk_i = bsk_ntt + bsk_row * i;
    for (int j = 0; j <= SK; j++) {
      step2_body<0>(D, bsk_i, acc, K, buf, j, ct);
      __syncthreads();
      step2_body<1>(D, bsk_i, acc, K, buf, j, ct);
      __syncthreads();
    }
  }
}

// ---- the f64 FFT external product (default; sns_fft.h) ------------------------------------------
// Layouts: key spectra Kf[i][r][j][t][M] (r = c L + l, t = limb, scaled by 1/M), digit spectra
// Df[ct][r][M], both in the DIF's digit-reversed order; tables in SnsFftConst.
using snsf::cd;
using snsf::SF_LIMBS;
using snsf::SF_M;

struct SnsFftConst {
  cd T[SF_M];           // e^{2 pi i e / M}
  cd P[SF_M];           // psi^m = e^{i pi m / N}
  u64 W[2][SF_LIMBS];   // limb weights 2^(SF_DROP + 16 t) mod p1, p2
  u64 WM[2][SF_LIMBS];  // the same in Montgomery form (x R mod p): mont(c, WM) = c 2^(SF_DROP + 16 t) mod p
};

__device__ __forceinline__ void fft_fwd_lds(cd* buf, const cd* __restrict__ T) {
#pragma unroll
  for (int s = 0; s < 5; s++) {
    snsf::dif_stage(buf, s, threadIdx.x, T);
    __syncthreads();
  }
}
// ROLLED = false: unrolled, the twiddle loads of later stages are issued early (168 VGPRs, 3 waves per
// SIMD: 159 us per CMUX launch at B = 1024); rolled, the stage loop fits 4 waves per SIMD without spills
// but waits on every stage's twiddle loads (199 us; 5 waves spill 48 VGPRs: slower still)
template <bool ROLLED = false>
__device__ __forceinline__ void fft_inv_lds(cd* buf, const cd* __restrict__ T) {
  if (ROLLED) {
#pragma unroll 1
    for (int s = 4; s >= 0; s--) {
      snsf::dit_stage(buf, s, threadIdx.x, T);
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int s = 4; s >= 0; s--) {
      snsf::dit_stage(buf, s, threadIdx.x, T);
      __syncthreads();
    }
  }
}

// BSK standard domain (residue pairs) -> rounded key, 7 balanced 16-bit limbs, spectra / M.
// One workgroup per (i, r, j) polynomial pair.
__global__ void __launch_bounds__(ST) sns_bsk_to_fft_kernel(const u64* __restrict__ in, cd* __restrict__ out,
                                                            const SnsConst* __restrict__ Kc,
                                                            const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  const size_t pair = blockIdx.x;
  const SnsConst& K = *Kc;
  const SnsFftConst& F = *Fc;
  const u64* pr = in + pair * 2 * SN;
  __int128 rr[8];  // coefficients m = tid + 256 u (u < 4) and m + 1024
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int x = threadIdx.x + 256 * u + SF_M * h;
      rr[2 * u + h] = round_key(pr[x], pr[SN + x], K);
    }
  for (int t = 0; t < SF_LIMBS; t++) {
    double lv[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      if (t == SF_LIMBS - 1) {
        lv[e] = (double)(long long)rr[e];  // the top limb keeps the remainder (|.| <= 2^15)
      } else {
        const __int128 l = ((rr[e] + 0x8000) & 0xFFFF) - 0x8000;
        rr[e] = (rr[e] - l) >> 16;
        lv[e] = (double)(long long)l;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int m = threadIdx.x + 256 * u;
      buf[m] = snsf::cmul(cd{lv[2 * u], lv[2 * u + 1]}, F.P[m]);
    }
    __syncthreads();
    fft_fwd_lds(buf, F.T);
    cd* o = out + (pair * SF_LIMBS + t) * SF_M;
    constexpr double inv_m = 1.0 / SF_M;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int f = threadIdx.x + 256 * u;
      o[f] = cd{buf[f].x * inv_m, buf[f].y * inv_m};
    }
    __syncthreads();
  }
}

// LDS visibility of a wave's own writes to its other lanes (DS ops of a wave complete in order)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// step 1 (ciphertext, component c): rotation, CRT lift, torus map, 3 digit levels (as the NTT path),
// then the folded, twisted forward FFT of each digit polynomial -> Df; wave l transforms level l in
// registers (sns_fft.h passes), its padded exchange buffer aliasing the dead digit arrays
// The rotation is read straight from global memory (coefficient t of X^{a_i} acc is +-acc[(t - a_i) mod
// 2N]), so the LDS holds only the digits, aliased by the three exchange buffers: 52 KB, 3 workgroups
// per CU (an LDS copy of the rotated residues, 56 KB, allowed 2).
__device__ __forceinline__ void step1_digits_g(const u64* __restrict__ lwe, int n, int i, const u64* __restrict__ acc,
                                               const SnsConst& K, int ct, int c, int (*dig)[SN]) {
  const u32 ai = mod_switch_4096(lwe[(size_t)ct * (n + 1) + i]);
  const u64* a = acc + ((size_t)ct * (SK + 1) + c) * 2 * SN;
  for (int t = threadIdx.x; t < SN; t += ST) {
    const u32 t1 = ((u32)t - ai) & 4095u;
    const bool neg = t1 >= (u32)SN;
    const int src = (int)(t1 & (u32)(SN - 1));
    const u64 v0 = a[src], v1 = a[SN + src];
    const u64 x0 = (neg && v0) ? Prime<0>::p - v0 : v0, x1 = (neg && v1) ? Prime<1>::p - v1 : v1;
    const u64 r1 = subm_q<0>(x0, a[t]);
    const u64 r2 = subm_q<1>(x1, a[SN + t]);
    // signed decomposition of the torus image: 72 bits, 3 digits of 24 (tfhe-rs SignedDecomposer)
    const u128 y = lift_to_torus(r1, r2, K);
    u128 state = ((y >> 55) + 1) >> 1;
    state &= ((u128)1 << 72) - 1;
    for (int l = SL - 1; l >= 0; l--) {
      const u64 res = (u64)state & 0xFFFFFFull;
      state >>= 24;
      const u64 carry = ((((res - 1) | (u64)state) & res) >> 23) & 1;
      state += carry;
      dig[l][t] = (int)((long long)res - (long long)(carry << 24));
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(ST) sns_step1f_kernel(const u64* __restrict__ lwe, int n, int i,
                                                        const u64* __restrict__ acc, cd* __restrict__ Df,
                                                        const SnsConst* __restrict__ Kc,
                                                        const SnsFftConst* __restrict__ Fc) {
  __shared__ cd xbuf[SL * snsf::SF_PADDED];  // the digits, then the waves' exchange buffers
  int (*dig)[SN] = reinterpret_cast<int (*)[SN]>(&xbuf[0]);
  static_assert(SL * SN * sizeof(int) <= sizeof(xbuf), "digits fit the exchange buffers");
  const int ct = blockIdx.x / (SK + 1), c = blockIdx.x % (SK + 1);
  const SnsFftConst& F = *Fc;
  step1_digits_g(lwe, n, i, acc, *Kc, ct, c, dig);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  cd x[16];
  if (w < SL) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = snsf::pt01(t, r);
      x[r] = snsf::cmul(cd{(double)dig[w][m], (double)dig[w][m + SF_M]}, F.P[m]);
    }
    snsf::dif_pass01(x, t, F.T);
  }
  __syncthreads();  // every digit read is done before the exchange buffers overwrite the digits
  if (w < SL) {
    cd* buf = xbuf + w * snsf::SF_PADDED;
#pragma unroll
    for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt01(t, r))] = x[r];
    wave_sync();
#pragma unroll
    for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt23(t, r))];
    snsf::dif_pass23(x, t, F.T);
#pragma unroll
    for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt23(t, r))] = x[r];
    wave_sync();
#pragma unroll
    for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt4(t, r))];
    snsf::dif_pass4(x, F.T);
    wave_sync();  // every lane has read its pass-4 inputs before the buffer takes the outputs
#pragma unroll
    for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt4(t, r))] = x[r];
    wave_sync();
    cd* o = Df + ((size_t)ct * SR + c * SL + w) * SF_M;  // spectra in DIF position order, stored contiguously
#pragma unroll
    for (int r = 0; r < 16; r++) o[64 * r + t] = buf[snsf::pad(64 * r + t)];
  }
}

// one limb of step 2: MAC over the 9 rows, inverse FFT, untwist, rint -> exact integers, weighted
// into the per-prime int128 sums
__device__ __forceinline__ void step2f_limb(const cd* __restrict__ d, const cd* __restrict__ kf, int j, int T,
                                            cd* buf, const SnsFftConst& F, __int128 (&s0)[8], __int128 (&s1)[8]) {
#pragma unroll 1
  for (int u = 0; u < 4; u++) {
    const int f = threadIdx.x + 256 * u;
    cd o = {0.0, 0.0};
#pragma unroll
    for (int r = 0; r < SR; r++)
      o = snsf::cmac(o, d[(size_t)r * SF_M + f], kf[(((size_t)r * (SK + 1) + j) * SF_LIMBS + T) * SF_M + f]);
    buf[f] = o;
  }
  __syncthreads();
  fft_inv_lds(buf, F.T);
  const __int128 w0 = (__int128)F.W[0][T], w1 = (__int128)F.W[1][T];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int m = threadIdx.x + 256 * u;
    const cd y = snsf::cmulc(buf[m], F.P[m]);
    const long long c0 = (long long)__builtin_rint(y.x), c1 = (long long)__builtin_rint(y.y);
    s0[2 * u] += (__int128)c0 * w0;
    s1[2 * u] += (__int128)c0 * w1;
    s0[2 * u + 1] += (__int128)c1 * w0;
    s1[2 * u + 1] += (__int128)c1 * w1;
  }
  __syncthreads();
}

// step 2 (ciphertext, output component j): all limbs of the external product, acc_j += (mod p1, p2)
__global__ void __launch_bounds__(ST) sns_step2f_kernel(const cd* __restrict__ Df, const cd* __restrict__ kf_i,
                                                        u64* __restrict__ acc, const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  const int j = blockIdx.x % (SK + 1), ct = blockIdx.x / (SK + 1);
  const SnsFftConst& F = *Fc;
  const cd* d = Df + (size_t)ct * SR * SF_M;
  __int128 s0[8], s1[8];
#pragma unroll
  for (int e = 0; e < 8; e++) s0[e] = s1[e] = 0;
#pragma unroll 1
  for (int t = 0; t < SF_LIMBS; t++) step2f_limb(d, kf_i, j, t, buf, F, s0, s1);
  u64* a0 = acc + ((size_t)ct * (SK + 1) + j) * 2 * SN;
  u64* a1 = a0 + SN;
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int x = threadIdx.x + 256 * u + SF_M * h;
      a0[x] = addm_q<0>(a0[x], reduce_s128<0>(s0[2 * u + h]));
      a1[x] = addm_q<1>(a1[x], reduce_s128<1>(s1[2 * u + h]));
    }
}

// Step 2 split for key reuse across ciphertexts (default): the MAC as a frequency-tiled kernel whose
// workgroup holds the CMUX's key for 16 frequencies x all 21 (output, limb) columns in LDS (48 KB)
// and streams 32 ciphertexts' digit spectra through it (8 frequencies x 64 ciphertexts, 24 KB, 4
// workgroups per CU: 108 us instead of 96, the 128-byte runs cost more than the occupancy gains), writing the products O[ct][j*7+t][M] to
// global memory; then one workgroup per (ciphertext, output) runs the 7 inverse FFTs, rint, the limb
// weights and acc_j += (mod p1, p2).  The one-kernel form (sns_step2f_kernel, TFHE_HIP_SNS_FUSED2=1)
// re-reads the ~1 MB per-output key slice for every ciphertext.
constexpr int MAC_F = 16, MAC_CT = 32, MAC_JT = (SK + 1) * SF_LIMBS;  // 21 (output, limb) columns

// Grid: (M / 16) frequency tiles x G ciphertext-group slots; slot g walks the groups g, g + G, ...
// (G = all groups: one group per workgroup), so a slot stages its key tile once for all its groups.
// The first group's digit spectra are requested before the key tile is staged, so those loads overlap
// the LDS fill (a register prefetch of the next group as well costs 100 spilled VGPRs at 3 waves/SIMD);
// the arithmetic per output is the same in every form.
__device__ __forceinline__ void mac_load(const cd* __restrict__ Df, int c0, int B, int f0, int f, int cl,
                                         cd (&da)[SR], cd (&db)[SR]) {
  const int ca = c0 + cl, cb = c0 + cl + ST / MAC_F;
#pragma unroll
  for (int r = 0; r < SR; r++) {
    da[r] = ca < B ? Df[((size_t)ca * SR + r) * SF_M + f0 + f] : cd{0.0, 0.0};
    db[r] = cb < B ? Df[((size_t)cb * SR + r) * SF_M + f0 + f] : cd{0.0, 0.0};
  }
}

__global__ void __launch_bounds__(ST, 3) sns_mac_kernel(const cd* __restrict__ Df, const cd* __restrict__ kf_i,
                                                     cd* __restrict__ O, int B) {
  __shared__ cd kt[SR * MAC_JT][MAC_F];  // [r * 21 + jt][f]
  constexpr int FT = SF_M / MAC_F;
  const int f0 = (blockIdx.x % FT) * MAC_F;
  const int slots = gridDim.x / FT, groups = (B + MAC_CT - 1) / MAC_CT;
  const int f = threadIdx.x % MAC_F, cl = threadIdx.x / MAC_F;  // MAC_F frequencies x (256 / MAC_F) ciphertext lanes
  static_assert(MAC_CT == 2 * (ST / MAC_F), "two ciphertexts per thread");
  int g = blockIdx.x / FT;
  cd da[SR], db[SR];
  mac_load(Df, g * MAC_CT, B, f0, f, cl, da, db);
  // key tile: row (r, jt) of the CMUX's key = kf_i[(r * 21 + jt) * M + f0 .. + 16]
  for (int x = threadIdx.x; x < SR * MAC_JT * MAC_F; x += ST) {
    const int row = x / MAC_F, fx = x % MAC_F;
    kt[row][fx] = kf_i[(size_t)row * SF_M + f0 + fx];
  }
  __syncthreads();
#pragma unroll 1
  for (; g < groups; g += slots) {
    const int ca = g * MAC_CT + cl, cb = ca + ST / MAC_F;
    const bool va = ca < B, vb = cb < B;
    if (g != (int)(blockIdx.x / FT)) mac_load(Df, g * MAC_CT, B, f0, f, cl, da, db);  // later groups
#pragma unroll 1
    for (int jt = 0; jt < MAC_JT; jt++) {
      cd oa = {0.0, 0.0}, ob = {0.0, 0.0};
#pragma unroll
      for (int r = 0; r < SR; r++) {
        const cd k = kt[r * MAC_JT + jt][f];
        oa = snsf::cmac(oa, da[r], k);
        ob = snsf::cmac(ob, db[r], k);
      }
      if (va) O[((size_t)ca * MAC_JT + jt) * SF_M + f0 + f] = oa;
      if (vb) O[((size_t)cb * MAC_JT + jt) * SF_M + f0 + f] = ob;
    }
  }
}

// (TFHE_HIP_SNS_INVW=1, measured slower: 2 waves/SIMD at 256 VGPRs) the 7 inverse FFTs of (ciphertext, output j) — one per wave, two rounds (limbs 0-3, 4-6) — each
// untwisted and rounded to exact int64 coefficients in the wave's buffer; every thread then folds its 8
// coefficients' limb values into two exact int128 partial sums (A = sum_{t<4} c_t 2^16t, B = sum_{t>=4}
// c_t 2^16(t-4); |A| < 2^102, |B| < 2^86), and the product 2^16 (A + 2^64 B) reduces once per prime:
// acc_j += (mod p1, p2)
__global__ void __launch_bounds__(ST, 2) sns_inv_wave_kernel(const cd* __restrict__ O, u64* __restrict__ acc,
                                                        const SnsFftConst* __restrict__ Fc) {
  __shared__ cd bufs[4][snsf::SF_PADDED];
  const int j = blockIdx.x % (SK + 1), ct = blockIdx.x / (SK + 1);
  const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
  const SnsFftConst& F = *Fc;
  cd* buf = bufs[w];
  long long* ci = reinterpret_cast<long long*>(buf);
  __int128 ab[2][8];
#pragma unroll 1
  for (int round = 0; round < 2; round++) {
    const int lim = round * 4 + w, nw = round ? SF_LIMBS - 4 : 4;
    if (lim < SF_LIMBS) {
      const cd* o = O + ((size_t)ct * MAC_JT + j * SF_LIMBS + lim) * SF_M;
      cd x[16];
#pragma unroll
      for (int r = 0; r < 16; r++) x[r] = o[snsf::pt4(t, r)];
      snsf::dit_pass4(x, F.T);
#pragma unroll
      for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt4(t, r))] = x[r];
      wave_sync();
#pragma unroll
      for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt23(t, r))];
      snsf::dit_pass32(x, t, F.T);
#pragma unroll
      for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt23(t, r))] = x[r];
      wave_sync();
#pragma unroll
      for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt01(t, r))];
      snsf::dit_pass10(x, t, F.T);
      wave_sync();  // all lanes' reads are done before the integer coefficients overwrite the buffer
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int m = snsf::pt01(t, r);
        const cd y = snsf::cmulc(x[r], F.P[m]);
        ci[m] = (long long)__builtin_rint(y.x);
        ci[m + SF_M] = (long long)__builtin_rint(y.y);
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; u++) {
      __int128 acc128 = (__int128)reinterpret_cast<const long long*>(bufs[0])[threadIdx.x + 256 * u];
      for (int q = 1; q < nw; q++)
        acc128 += (__int128)reinterpret_cast<const long long*>(bufs[q])[threadIdx.x + 256 * u] << (16 * q);
      ab[round][u] = acc128;
    }
    __syncthreads();
  }
  u64* a0 = acc + ((size_t)ct * (SK + 1) + j) * 2 * SN;
  u64* a1 = a0 + SN;
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const int x = threadIdx.x + 256 * u;
    const __int128 A = ab[0][u] << snsf::SF_DROP, Bv = ab[1][u] << snsf::SF_DROP;  // x 2^16: < 2^118, < 2^102
    const u64 r0 = addm_q<0>(reduce_s128<0>(A), mont_q<0>(reduce_s128<0>(Bv), prime_r2<0>()));  // + 2^64 B
    const u64 r1 = addm_q<1>(reduce_s128<1>(A), mont_q<1>(reduce_s128<1>(Bv), prime_r2<1>()));
    a0[x] = addm_q<0>(a0[x], r0);
    a1[x] = addm_q<1>(a1[x], r1);
  }
}

// the 7 inverse FFTs of (ciphertext, output j), one after another by all 256 threads (stage form, 16 KB
// LDS), limbs from the top: each thread folds the rounded limb values (|c| < 2^53) of its 8 coefficients
// into exact int128 Horner sums with a constant shift, B = ((c6 2^16) + c5) 2^16 + c4 (< 2^86), then
// A = c3 2^48 + ... + c0 (< 2^102), and reduces 2^16 (A + 2^64 B) once per prime: acc_j += (mod p1,
// p2).  Measured alternatives, all slower: weighting every limb value by 2^(16+16t) mod p into int128
// sums (two 64 x 64 products per coefficient and limb: 160 us), residue sums with a Montgomery product
// per limb (206-219 us), runtime-amount int128 shifts (227 us), a per-limb switch of compile-time shifts
// (60 spills, 387 us), spectra stored in the pass-4 register order (gathered loads, 264 us).
// Inverse twiddles from LDS (TWL): a per-stage table, stage s at TL_OFF[s], rows k = 1..3 of q_s = 4^(4-s)
// entries, tl[off + (k-1) q + j] = T[k (j << 2s)] (the values the global-table form reads: same products)
constexpr int TL_LEN = 3 * (256 + 64 + 16 + 4 + 1);  // 1023
__device__ __forceinline__ int tl_off(int s) { return s == 0 ? 0 : s == 1 ? 768 : s == 2 ? 960 : s == 3 ? 1008 : 1020; }
__device__ __forceinline__ void fill_tl(cd* tl, const cd* __restrict__ T) {
  for (int x = threadIdx.x; x < TL_LEN; x += ST) {
    const int s = x < 768 ? 0 : x < 960 ? 1 : x < 1008 ? 2 : x < 1020 ? 3 : 4;
    const int q = 1 << (8 - 2 * s), r = x - tl_off(s), k = r / q + 1, jj = r % q;
    tl[x] = T[k * (jj << (2 * s))];
  }
}
__device__ __forceinline__ void fft_inv_lds_tl(cd* a, const cd* tl) {
#pragma unroll
  for (int s = 4; s >= 0; s--) {
    const int lq = 8 - 2 * s, q = 1 << lq, t = threadIdx.x;
    const int jj = t & (q - 1), base = ((t >> lq) << (lq + 2)) + jj;
    const cd* w = tl + tl_off(s) + jj;
    cd y0 = a[base], y1 = snsf::cmulc(a[base + q], w[0]), y2 = snsf::cmulc(a[base + 2 * q], w[q]),
       y3 = snsf::cmulc(a[base + 3 * q], w[2 * q]);
    snsf::r4_dit(y0, y1, y2, y3, -1, tl);
    a[base] = y0;
    a[base + q] = y1;
    a[base + 2 * q] = y2;
    a[base + 3 * q] = y3;
    __syncthreads();
  }
}

// The register-ended inverse (REG, default): stage 4's butterflies (q = 1, unit twiddles) each take 4
// consecutive points, so thread t loads points 4t..4t+3 straight from global memory and transforms them
// before the first LDS write; stage 0's butterfly of thread t yields points t + 256 k, exactly the
// coefficients the thread untwists and rounds, so they stay in registers.  Same butterflies, same
// values; two LDS passes and two barriers fewer per limb (store + 5 stages + read -> 4 stages).
__device__ __forceinline__ void fft_inv_reg(const cd* __restrict__ o, cd* buf, const cd* __restrict__ T, cd (&y)[4]) {
  const int t = threadIdx.x;
  y[0] = o[4 * t];
  y[1] = o[4 * t + 1];
  y[2] = o[4 * t + 2];
  y[3] = o[4 * t + 3];
  snsf::r4_dit(y[0], y[1], y[2], y[3], 0, T);  // dit_stage(s = 4): base 4t, e = 0
#pragma unroll
  for (int k = 0; k < 4; k++) buf[4 * t + k] = y[k];
  __syncthreads();
#pragma unroll
  for (int s = 3; s >= 1; s--) {
    snsf::dit_stage(buf, s, t, T);
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 4; k++) y[k] = buf[t + 256 * k];
  snsf::r4_dit(y[0], y[1], y[2], y[3], t, T);  // dit_stage(s = 0): base t, q 256, e = t
}

template <int OCC, bool TWL, bool REG = false>  // waves per SIMD: 3 = unrolled stages (168 VGPRs), 4 / 5 = rolled
__global__ void __launch_bounds__(ST, OCC) sns_inv_kernel(const cd* __restrict__ O, u64* __restrict__ acc,
                                                          const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  __shared__ cd tl[TWL ? TL_LEN : 1];
  const int j = blockIdx.x % (SK + 1), ct = blockIdx.x / (SK + 1);
  const SnsFftConst& F = *Fc;
  if (TWL) fill_tl(tl, F.T);  // ordered before its first use by the limb loop's first barrier
  __int128 h[8], Bv[8];
#pragma unroll
  for (int e = 0; e < 8; e++) h[e] = Bv[e] = 0;
  static_assert(SF_LIMBS == 7, "B = limbs 6..4, A = limbs 3..0");
#pragma unroll 1
  for (int t = SF_LIMBS - 1; t >= 0; t--) {
    if (t == 3) {  // uniform: B complete, start A
#pragma unroll
      for (int e = 0; e < 8; e++) {
        Bv[e] = h[e];
        h[e] = 0;
      }
    }
    const cd* o = O + ((size_t)ct * MAC_JT + j * SF_LIMBS + t) * SF_M;
    cd yr[4];
    if (REG) {
      fft_inv_reg(o, buf, F.T, yr);
    } else {
#pragma unroll
      for (int u = 0; u < 4; u++) buf[threadIdx.x + 256 * u] = o[threadIdx.x + 256 * u];
      __syncthreads();
      if (TWL)
        fft_inv_lds_tl(buf, tl);
      else
        fft_inv_lds<(OCC > 3)>(buf, F.T);
#pragma unroll
      for (int u = 0; u < 4; u++) yr[u] = buf[threadIdx.x + 256 * u];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int m = threadIdx.x + 256 * u;
      const cd y = snsf::cmulc(yr[u], F.P[m]);
      h[2 * u] = (h[2 * u] << 16) + (__int128)(long long)__builtin_rint(y.x);
      h[2 * u + 1] = (h[2 * u + 1] << 16) + (__int128)(long long)__builtin_rint(y.y);
    }
    __syncthreads();
  }
  u64* a0 = acc + ((size_t)ct * (SK + 1) + j) * 2 * SN;
  u64* a1 = a0 + SN;
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
      const int x = threadIdx.x + 256 * u + SF_M * hh;
      const __int128 a = h[2 * u + hh] << snsf::SF_DROP, b = Bv[2 * u + hh] << snsf::SF_DROP;  // < 2^118, 2^102
      const u64 r0 = addm_q<0>(reduce_s128<0>(a), mont_q<0>(reduce_s128<0>(b), prime_r2<0>()));  // + 2^64 b
      const u64 r1 = addm_q<1>(reduce_s128<1>(a), mont_q<1>(reduce_s128<1>(b), prime_r2<1>()));
      a0[x] = addm_q<0>(a0[x], r0);
      a1[x] = addm_q<1>(a1[x], r1);
    }
}

// acc -> LWE over Z_2^128 (dim k N, + body), (lo, hi) pairs
__global__ void sns_extract_kernel(const u64* __restrict__ acc, u64* __restrict__ out, const SnsConst* __restrict__ Kc) {
  const int ct = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e > SK * SN) return;
  const SnsConst& K = *Kc;
  const u64* a = acc + (size_t)ct * (SK + 1) * 2 * SN;
  u64 r[2];
  if (e == SK * SN) {
    r[0] = a[(size_t)SK * 2 * SN];
    r[1] = a[(size_t)SK * 2 * SN + SN];
  } else {
    const int c = e / SN, t = e % SN;
    for (int q = 0; q < 2; q++) {
      const u64 v = a[((size_t)c * 2 + q) * SN + (t == 0 ? 0 : SN - t)];
      r[q] = (t == 0 || v == 0) ? v : K.p[q] - v;
    }
  }
  const u128 y = lift_to_torus(r[0], r[1], K);
  u64* o = out + ((size_t)ct * (SK * SN + 1) + e) * 2;
  o[0] = (u64)y;
  o[1] = (u64)(y >> 64);
}

u128 host_mulhi128(u128 x, u128 y) {
  const u64 x0 = (u64)x, x1 = (u64)(x >> 64), y0 = (u64)y, y1 = (u64)(y >> 64);
  const u128 p00 = (u128)x0 * y0, p01 = (u128)x0 * y1, p10 = (u128)x1 * y0, p11 = (u128)x1 * y1;
  const u128 mid = (p00 >> 64) + (u64)p01 + (u64)p10;
  return p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}
u64 hmul(u64 a, u64 b, u64 p) { return (u64)(((u128)a * b) % p); }
u64 hpow(u64 a, u64 e, u64 p) {
  u64 r = 1;
  for (; e; e >>= 1, a = hmul(a, a, p))
    if (e & 1) r = hmul(r, a, p);
  return r;
}

}  // namespace

size_t sns_const_bytes() { return sizeof(SnsConst); }

void make_sns_const(void* out) {
  SnsConst& K = *(SnsConst*)out;
  const u64 P[2] = {0xFFFFFFFF00000001ull, 0xFFFFFFFC00000001ull};
  for (int q = 0; q < 2; q++) {
    const u64 p = P[q];
    K.p[q] = p;
    u64 inv = 1;  // p^-1 mod 2^64 by Newton
    for (int it = 0; it < 7; it++) inv *= 2 - p * inv;
    K.pinv_neg[q] = (u64)0 - inv;
    static_assert(Prime<0>::p == 0xFFFFFFFF00000001ull && Prime<1>::p == 0xFFFFFFFC00000001ull, "SnS primes");
    const u64 R = (u64)(((u128)1 << 64) % p);
    K.r2[q] = hmul(R, R, p);
    u64 nr = 2;
    while (hpow(nr, (p - 1) / 2, p) != p - 1) nr++;
    const u64 psi = hpow(nr, (p - 1) / (2ull * SN), p), ipsi = hpow(psi, p - 2, p);
    int lg = 0;
    while ((1 << lg) < SN) lg++;
    for (int i = 0; i < SN; i++) {
      int r = 0;
      for (int b = 0; b < lg; b++)
        if (i & (1 << b)) r |= 1 << (lg - 1 - b);
      K.psi_rev[q][i] = hmul(hpow(psi, (u64)r, p), R, p);
      K.ipsi_rev[q][i] = hmul(hpow(ipsi, (u64)r, p), R, p);
    }
    K.ninv[q] = hmul(hpow(SN, p - 2, p), R, p);
  }
  const u64 R2p = (u64)(((u128)1 << 64) % P[1]);
  K.p1inv_m = hmul(hpow(P[0] % P[1], P[1] - 2, P[1]), R2p, P[1]);
  // floor(2^256 / Q) - 2^128 = floor((2^128 - Q) * 2^128 / Q) by long division
  const u128 Q = (u128)P[0] * P[1], d = (u128)0 - Q;
  u128 rem = 0, quo = 0;
  for (int i = 255; i >= 0; i--) {
    const int bit = i >= 128 ? (int)((d >> (i - 128)) & 1) : 0;
    const int top = (int)(rem >> 127);
    rem = (rem << 1) | (u128)bit;
    if (top || rem >= Q) {
      rem -= Q;
      if (i < 128) quo |= (u128)1 << i;
    }
  }
  K.conv_lo = (u64)quo;
  K.conv_hi = (u64)(quo >> 64);
  (void)host_mulhi128;
}

hipError_t launch_sns_bsk_to_ntt(const u64* bsk_std, u64* bsk_ntt, size_t polys, const void* d_const, hipStream_t s) {
  sns_bsk_to_ntt_kernel<<<(unsigned)polys, ST, 0, s>>>(bsk_std, bsk_ntt, (const SnsConst*)d_const);
  return hipGetLastError();
}

// one squash pass over B ciphertexts: acc / D workspaces (B x 3 x 2 x N, B x 9 x 2 x N u64)
hipError_t launch_sns_blind_rotate(const u64* lwe, size_t B, int n, const u64* lut, const u64* bsk_ntt, u64* acc,
                                   u64* D, const void* d_const, hipStream_t s) {
  const SnsConst* K = (const SnsConst*)d_const;
  sns_init_kernel<<<(unsigned)B, 256, 0, s>>>(lwe, n, lut, acc, K);
  // TFHE_HIP_SNS_FUSED=1: the single-launch form (measured 2.4x slower: 1024 workgroups of 4 waves with
  // the 9 jobs of a CMUX in sequence expose far less parallelism than 3072 + 6144 workgroups per CMUX)
  static const bool fused = [] {
    const char* e = getenv("TFHE_HIP_SNS_FUSED");
    return e && e[0] == '1';
  }();
  if (fused) {
    sns_fused_kernel<<<(unsigned)B, ST, 0, s>>>(lwe, n, bsk_ntt, acc, D, K);
    return hipGetLastError();
  }
  const size_t bsk_i = (size_t)SR * (SK + 1) * 2 * SN;
  for (int i = 0; i < n; i++) {
    sns_step1_kernel<<<(unsigned)(B * (SK + 1)), ST, 0, s>>>(lwe, n, i, acc, D, K);
    sns_step2_kernel<<<(unsigned)(B * (SK + 1) * 2), ST, 0, s>>>(D, bsk_ntt + bsk_i * i, acc, K);
  }
  return hipGetLastError();
}

size_t sns_fft_const_bytes() { return sizeof(SnsFftConst); }

void make_sns_fft_const(void* out) {
  SnsFftConst& F = *(SnsFftConst*)out;
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int e = 0; e < SF_M; e++) {
    F.T[e] = cd{(double)cosl(2 * pi * e / SF_M), (double)sinl(2 * pi * e / SF_M)};
    F.P[e] = cd{(double)cosl(pi * e / SN), (double)sinl(pi * e / SN)};
  }
  for (int t = 0; t < SF_LIMBS; t++) {
    F.W[0][t] = prime_pow2<0>(snsf::SF_DROP + snsf::SF_LIMB_BITS * t);
    F.W[1][t] = prime_pow2<1>(snsf::SF_DROP + snsf::SF_LIMB_BITS * t);
    F.WM[0][t] = hmul(F.W[0][t], (u64)0 - Prime<0>::p, Prime<0>::p);  // x (2^64 mod p)
    F.WM[1][t] = hmul(F.W[1][t], (u64)0 - Prime<1>::p, Prime<1>::p);
  }
}

size_t sns_fft_key_len(size_t n) { return n * SR * (SK + 1) * SF_LIMBS * SF_M; }  // in cd (16 B)

// `pairs` (i, r, j) polynomial pairs of the standard-domain key -> spectra
hipError_t launch_sns_bsk_to_fft(const u64* bsk_std, void* bsk_fft, size_t pairs, const void* d_const,
                                 const void* d_fconst, hipStream_t s) {
  sns_bsk_to_fft_kernel<<<(unsigned)pairs, ST, 0, s>>>(bsk_std, (cd*)bsk_fft, (const SnsConst*)d_const,
                                                        (const SnsFftConst*)d_fconst);
  return hipGetLastError();
}

// one squash pass over B ciphertexts on the f64 FFT path (acc B x 3 x 2 x N u64, D B x 9 x M cd)
size_t sns_fft_prod_len(size_t B) { return B * MAC_JT * SF_M; }  // O workspace, in cd

hipError_t launch_sns_blind_rotate_fft(const u64* lwe, size_t B, int n, const u64* lut, const void* bsk_fft, u64* acc,
                                       void* D, void* Oprod, const void* d_const, const void* d_fconst,
                                       hipStream_t s) {
  const SnsConst* K = (const SnsConst*)d_const;
  const SnsFftConst* F = (const SnsFftConst*)d_fconst;
  sns_init_kernel<<<(unsigned)B, 256, 0, s>>>(lwe, n, lut, acc, K);
  const size_t per_i = (size_t)SR * (SK + 1) * SF_LIMBS * SF_M;
  // measured variants (read per call, so one process can check them all): the one-kernel step 2 and the
  // one-wave-per-limb inverse
  const char* e2 = getenv("TFHE_HIP_SNS_FUSED2");
  const char* ew = getenv("TFHE_HIP_SNS_INVW");
  const bool fused2 = e2 && e2[0] == '1', invw = ew && ew[0] == '1';
  // sns_inv_kernel form: 0 (default) register-ended stages at 3 waves/SIMD; 3 / 4 / 5: all five stages
  // through LDS at that many waves/SIMD; 13 / 14: 3 / 4 with the LDS twiddle table
  const char* eo = getenv("TFHE_HIP_SNS_INVOCC");
  const int inv_occ = eo ? atoi(eo) : 0;
  // TFHE_HIP_SNS_MACG = ciphertext-group slots of the MAC grid (default 8; 0: one group per workgroup)
  const char* eg = getenv("TFHE_HIP_SNS_MACG");
  const size_t groups = (B + MAC_CT - 1) / MAC_CT, mg = eg ? (size_t)atoi(eg) : 8;
  const unsigned mac_grid = (unsigned)((SF_M / MAC_F) * (mg > 0 && mg < groups ? mg : groups));
  for (int i = 0; i < n; i++) {
    const cd* kf_i = (const cd*)bsk_fft + per_i * i;
    sns_step1f_kernel<<<(unsigned)(B * (SK + 1)), ST, 0, s>>>(lwe, n, i, acc, (cd*)D, K, F);
    if (fused2 || !Oprod) {
      sns_step2f_kernel<<<(unsigned)(B * (SK + 1)), ST, 0, s>>>((const cd*)D, kf_i, acc, F);
    } else {
      sns_mac_kernel<<<mac_grid, ST, 0, s>>>((const cd*)D, kf_i, (cd*)Oprod, (int)B);
      const unsigned ig = (unsigned)(B * (SK + 1));
      if (invw)
        sns_inv_wave_kernel<<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else if (inv_occ == 0)
        sns_inv_kernel<3, false, true><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else if (inv_occ == 4)
        sns_inv_kernel<4, false><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else if (inv_occ == 5)
        sns_inv_kernel<5, false><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else if (inv_occ == 13)
        sns_inv_kernel<3, true><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else if (inv_occ == 14)
        sns_inv_kernel<4, true><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
      else
        sns_inv_kernel<3, false><<<ig, ST, 0, s>>>((const cd*)Oprod, acc, F);
    }
  }
  return hipGetLastError();
}

hipError_t launch_sns_extract(const u64* acc, size_t B, u64* out, const void* d_const, hipStream_t s) {
  dim3 grid((SK * SN + 1 + 255) / 256, (unsigned)B);
  sns_extract_kernel<<<grid, 256, 0, s>>>(acc, out, (const SnsConst*)d_const);
  return hipGetLastError();
}

}  // namespace tfhe
