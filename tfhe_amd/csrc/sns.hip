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

#include "pbs_kernels.h"

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

__device__ __forceinline__ u128 mulhi128(u128 x, u128 y) {
  const u64 x0 = (u64)x, x1 = (u64)(x >> 64), y0 = (u64)y, y1 = (u64)(y >> 64);
  const u128 p00 = (u128)x0 * y0, p01 = (u128)x0 * y1, p10 = (u128)x1 * y0, p11 = (u128)x1 * y1;
  const u128 mid = (p00 >> 64) + (u64)p01 + (u64)p10;
  return p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

// residues -> x in [0, Q) -> torus y = x + floor((x c + 2^127) / 2^128)
__device__ __forceinline__ u128 lift_to_torus(u64 r1, u64 r2, const SnsConst& K) {
  const u64 p1 = K.p[0], p2 = K.p[1];
  const u64 r1m = r1 >= p2 ? r1 - p2 : r1;
  const u64 t = mont(subm(r2, r1m, p2), K.p1inv_m, p2, K.pinv_neg[1]);
  const u128 x = (u128)r1 + (u128)p1 * t;
  const u128 c = ((u128)K.conv_hi << 64) | K.conv_lo;
  const u128 lo = x * c;
  return x + mulhi128(x, c) + (u128)((lo >> 127) & 1);
}

__device__ void ntt_fwd_lds(u64* a, const u64* tw, u64 p, u64 pinv) {
  for (int m = 1, t = SN / 2; m < SN; m <<= 1, t >>= 1) {
    for (int b = threadIdx.x; b < SN / 2; b += ST) {
      const int i = b / t, j = 2 * i * t + (b % t);
      const u64 S = tw[m + i];
      const u64 U = a[j], V = mont(a[j + t], S, p, pinv);
      a[j] = addm(U, V, p);
      a[j + t] = subm(U, V, p);
    }
    __syncthreads();
  }
}

__device__ void ntt_inv_lds(u64* a, const u64* itw, u64 ninv, u64 p, u64 pinv) {
  for (int m = SN / 2, t = 1; m >= 1; m >>= 1, t <<= 1) {
    for (int b = threadIdx.x; b < SN / 2; b += ST) {
      const int i = b / t, j = 2 * i * t + (b % t);
      const u64 S = itw[m + i];
      const u64 U = a[j], V = a[j + t];
      a[j] = addm(U, V, p);
      a[j + t] = mont(subm(U, V, p), S, p, pinv);
    }
    __syncthreads();
  }
  for (int x = threadIdx.x; x < SN; x += ST) a[x] = mont(a[x], ninv, p, pinv);
  __syncthreads();
}

__device__ __forceinline__ u32 mod_switch_4096(u64 x) { return (u32)(((x >> 51) + 1) >> 1) & 4095u; }

// BSK standard domain -> NTT domain (bit-reversed) in Montgomery form; one polynomial per workgroup
__global__ void __launch_bounds__(ST) sns_bsk_to_ntt_kernel(const u64* __restrict__ in, u64* __restrict__ out,
                                                            const SnsConst* __restrict__ Kc) {
  __shared__ u64 a[SN];
  const size_t poly = blockIdx.x;
  const int q = (int)(poly & 1);  // [..][prime][N]
  const SnsConst& K = *Kc;
  for (int x = threadIdx.x; x < SN; x += ST) a[x] = in[poly * SN + x];
  __syncthreads();
  ntt_fwd_lds(a, K.psi_rev[q], K.p[q], K.pinv_neg[q]);
  for (int x = threadIdx.x; x < SN; x += ST) out[poly * SN + x] = mont(a[x], K.r2[q], K.p[q], K.pinv_neg[q]);
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

__global__ void __launch_bounds__(ST) sns_step1_kernel(const u64* __restrict__ lwe, int n, int i,
                                                       const u64* __restrict__ acc, u64* __restrict__ D,
                                                       const SnsConst* __restrict__ Kc) {
  __shared__ u64 rot[2][SN];
  __shared__ int dig[SL][SN];
  __shared__ u64 buf[SN];
  const int ct = blockIdx.x / (SK + 1), c = blockIdx.x % (SK + 1);
  const SnsConst& K = *Kc;
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
    const u64 r1 = subm(rot[0][t], a[t], K.p[0]);
    const u64 r2 = subm(rot[1][t], a[SN + t], K.p[1]);
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
  for (int l = 0; l < SL; l++)
    for (int q = 0; q < 2; q++) {
      const u64 p = K.p[q];
      for (int t = threadIdx.x; t < SN; t += ST) {
        const int d = dig[l][t];
        buf[t] = d >= 0 ? (u64)d : p - (u64)(-d);
      }
      __syncthreads();
      ntt_fwd_lds(buf, K.psi_rev[q], p, K.pinv_neg[q]);
      u64* out = D + (((size_t)ct * SR + c * SL + l) * 2 + q) * SN;
      for (int t = threadIdx.x; t < SN; t += ST) out[t] = buf[t];
      __syncthreads();
    }
}

__global__ void __launch_bounds__(ST) sns_step2_kernel(const u64* __restrict__ D, const u64* __restrict__ bsk_i,
                                                       u64* __restrict__ acc, const SnsConst* __restrict__ Kc) {
  __shared__ u64 buf[SN];
  const int q = blockIdx.x & 1, j = (blockIdx.x >> 1) % (SK + 1), ct = (blockIdx.x >> 1) / (SK + 1);
  const SnsConst& K = *Kc;
  const u64 p = K.p[q], pinv = K.pinv_neg[q];
  const u64* d = D + (size_t)ct * SR * 2 * SN + (size_t)q * SN;
  const u64* b = bsk_i + ((size_t)j * 2 + q) * SN;  // [r][j][prime][N]
  for (int t = threadIdx.x; t < SN; t += ST) {
    u64 s = 0;
#pragma unroll
    for (int r = 0; r < SR; r++) s = addm(s, mont(d[(size_t)r * 2 * SN + t], b[(size_t)r * (SK + 1) * 2 * SN + t], p, pinv), p);
    buf[t] = s;
  }
  __syncthreads();
  ntt_inv_lds(buf, K.ipsi_rev[q], K.ninv[q], p, pinv);
  u64* a = acc + (((size_t)ct * (SK + 1) + j) * 2 + q) * SN;
  for (int t = threadIdx.x; t < SN; t += ST) a[t] = addm(a[t], buf[t], p);
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
  const size_t bsk_i = (size_t)SR * (SK + 1) * 2 * SN;
  for (int i = 0; i < n; i++) {
    sns_step1_kernel<<<(unsigned)(B * (SK + 1)), ST, 0, s>>>(lwe, n, i, acc, D, K);
    sns_step2_kernel<<<(unsigned)(B * (SK + 1) * 2), ST, 0, s>>>(D, bsk_ntt + bsk_i * i, acc, K);
  }
  return hipGetLastError();
}

hipError_t launch_sns_extract(const u64* acc, size_t B, u64* out, const void* d_const, hipStream_t s) {
  dim3 grid((SK * SN + 1 + 255) / 256, (unsigned)B);
  sns_extract_kernel<<<grid, 256, 0, s>>>(acc, out, (const SnsConst*)d_const);
  return hipGetLastError();
}

}  // namespace tfhe
