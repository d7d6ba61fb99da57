// sns.hip — switch-and-squash / noise squashing (rule: oracle/sns_oracle.c).
//
// A P-FHEVM small-key ciphertext (after keyswitch + modulus-switch noise reduction) is bootstrapped
// with a BSK under a 128-bit GLWE key (k = 2, N = 2048, 2^24 x 3) and the identity LUT; the output is
// an LWE over Z_2^128 (dim 4096) with ~2^-63 noise.  The GLWE ring is the native 2^128 torus, as in
// tfhe-rs: a coefficient is one u128 word stored as two u64 planes, polynomial = [lo][N], [hi][N].
//
// The external product is f64 (sns_fft.h): the key, rounded at load to multiples of 2^16, is five limbs --
// the balanced low 48 bits and four balanced 16-bit limbs.  Each 9-term digit x 16-bit-limb convolution is
// an integer below 2^52.2 that an f64 FFT product returns exactly after rint(); the low limb's products are
// rounded f64 values whose error lands at weight 2^16, far below the output noise, and whose operation
// order the oracle restates.  The limbs recombine with 128-bit wrap-around shifts.
// Work shape per CMUX (accumulator, 96 KB per ciphertext, in HBM):
//   sns_step1f (ciphertext, component c): X^{a_i} acc_c - acc_c, signed 2^24 x 3 digits, forward FFT
//              of each digit polynomial (one per wave) -> Df
//   sns_mac    key-stationary MAC: a 16-frequency tile of the CMUX's key in LDS, ciphertexts streamed
//              through it -> O[ct][output j][limb t][M]
//   sns_inv    (ciphertext, output j): 5 inverse FFTs, rint, Horner over the limbs, acc_j +=
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include "pbs_kernels.h"
#include "sns_fft.h"

namespace tfhe {
namespace {

typedef unsigned __int128 u128;
constexpr int SN = 2048, SK = 2, SL = 3, SR = (SK + 1) * SL, ST = 256;

using snsf::cd;
using snsf::SF_LIMBS;
using snsf::SF_M;

static_assert(SNS_FFT_POLY_BYTES == (size_t)SF_LIMBS * SF_M * sizeof(cd), "key polynomial stride (pbs_kernels.h)");

struct SnsFftConst {
  cd T[SF_M];  // e^{2 pi i e / M}
  cd P[SF_M];  // psi^m = e^{i pi m / N}
};

__device__ __forceinline__ u32 mod_switch_4096(u64 x) { return (u32)(((x >> 51) + 1) >> 1) & 4095u; }
__device__ __forceinline__ u128 ld128(const u64* plane_lo, int t) { return ((u128)plane_lo[SN + t] << 64) | plane_lo[t]; }
__device__ __forceinline__ void st128(u64* plane_lo, int t, u128 v) {
  plane_lo[t] = (u64)v;
  plane_lo[SN + t] = (u64)(v >> 64);
}

// acc = X^{-b~} (0, 0, lut)
__global__ void sns_init_kernel(const u64* __restrict__ lwe, int n, const u64* __restrict__ lut, u64* __restrict__ acc) {
  const int ct = blockIdx.x;
  const u32 bt = mod_switch_4096(lwe[(size_t)ct * (n + 1) + n]);
  const u32 sh = (4096u - bt) & 4095u;
  u64* a = acc + (size_t)ct * (SK + 1) * 2 * SN;
  for (int x = threadIdx.x; x < SK * 2 * SN; x += blockDim.x) a[x] = 0;
  for (int t = threadIdx.x; t < SN; t += blockDim.x) {
    u32 dst = (u32)t + sh;
    bool neg = false;
    if (dst >= 4096u) dst -= 4096u;
    if (dst >= (u32)SN) {
      dst -= SN;
      neg = true;
    }
    const u128 v = ld128(lut, t);
    st128(a + (size_t)SK * 2 * SN, (int)dst, neg ? (u128)0 - v : v);
  }
}

__device__ __forceinline__ void fft_fwd_lds(cd* buf, const cd* __restrict__ T) {
#pragma unroll
  for (int s = 0; s < 5; s++) {
    snsf::dif_stage(buf, s, threadIdx.x, T);
    __syncthreads();
  }
}

// BSK words (lo, hi planes) -> rounded key, its 5 limbs (snsf::key_limb), spectra / M (oracle:
// or_sns_bsk_round + or_sns_bsk_to_limb_ntt: the same limbs).  One workgroup per (i, r, j) polynomial.
__global__ void __launch_bounds__(ST) sns_bsk_to_fft_kernel(const u64* __restrict__ in, cd* __restrict__ out,
                                                            const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  const size_t poly = blockIdx.x;
  const SnsFftConst& F = *Fc;
  const u64* pr = in + poly * 2 * SN;
  __int128 rr[8];  // coefficients m = tid + 256 u (u < 4) and m + 1024, as x' / 2^16
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int x = threadIdx.x + 256 * u + SF_M * h;
      rr[2 * u + h] = snsf::key_round16(ld128(pr, x));
    }
  for (int t = 0; t < SF_LIMBS; t++) {
    double lv[8];
#pragma unroll
    for (int e = 0; e < 8; e++) lv[e] = (double)snsf::key_limb(rr[e], t);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int m = threadIdx.x + 256 * u;
      buf[m] = snsf::cmul(cd{lv[2 * u], lv[2 * u + 1]}, F.P[m]);
    }
    __syncthreads();
    fft_fwd_lds(buf, F.T);
    cd* o = out + (poly * SF_LIMBS + t) * SF_M;
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

// The rest of a one-wave forward transform after pass 01 (x in registers, pass-01 order): two exchanges
// through the wave's padded buffer, passes 23 and 4, then the spectrum stored contiguously in DIF position order.
__device__ __forceinline__ void wave_fwd_tail(cd (&x)[16], int t, const cd* __restrict__ T, cd* buf, cd* __restrict__ o) {
#pragma unroll
  for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt01(t, r))] = x[r];
  wave_sync();
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt23(t, r))];
  snsf::dif_pass23(x, t, T);
#pragma unroll
  for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt23(t, r))] = x[r];
  wave_sync();
#pragma unroll
  for (int r = 0; r < 16; r++) x[r] = buf[snsf::pad(snsf::pt4(t, r))];
  snsf::dif_pass4(x, T);
  wave_sync();  // every lane has read its pass-4 inputs before the buffer takes the outputs
#pragma unroll
  for (int r = 0; r < 16; r++) buf[snsf::pad(snsf::pt4(t, r))] = x[r];
  wave_sync();
#pragma unroll
  for (int r = 0; r < 16; r++) o[64 * r + t] = buf[snsf::pad(64 * r + t)];
}

// step 1 digits: coefficient t of X^{a_i} acc is +-acc[(t - a_i) mod 2N], read straight from global memory
// (a shifted contiguous window, coalesced), minus acc[t], decomposed as a 128-bit word (tfhe-rs
// SignedDecomposer: 72 bits, 3 digits of 24, gadget 2^(128 - 24 (l + 1)))
__device__ __forceinline__ void step1_digits(const u64* __restrict__ lwe, int n, int i, const u64* __restrict__ acc,
                                             int ct, int c, int (*dig)[SN]) {
  const u32 ai = mod_switch_4096(lwe[(size_t)ct * (n + 1) + i]);
  const u64* a = acc + ((size_t)ct * (SK + 1) + c) * 2 * SN;
  for (int t = threadIdx.x; t < SN; t += ST) {
    const u32 t1 = ((u32)t - ai) & 4095u;
    const int src = (int)(t1 & (u32)(SN - 1));
    const u128 v = ld128(a, src);
    int d[SL];
    snsf::digits72((t1 >= (u32)SN ? (u128)0 - v : v) - ld128(a, t), d);
#pragma unroll
    for (int l = 0; l < SL; l++) dig[l][t] = d[l];
  }
  __syncthreads();
}

// The rotation is read from global memory, so the LDS holds only the digits, aliased by the three
// waves' exchange buffers: 52 KB, 3 workgroups per CU.  Wave l transforms level l in registers
// (sns_fft.h passes).
__global__ void __launch_bounds__(ST) sns_step1f_kernel(const u64* __restrict__ lwe, int n, int i,
                                                        const u64* __restrict__ acc, cd* __restrict__ Df,
                                                        const SnsFftConst* __restrict__ Fc) {
  __shared__ cd xbuf[SL * snsf::SF_PADDED];  // the digits, then the waves' exchange buffers
  int (*dig)[SN] = reinterpret_cast<int (*)[SN]>(&xbuf[0]);
  static_assert(SL * SN * sizeof(int) <= sizeof(xbuf), "digits fit the exchange buffers");
  const int ct = blockIdx.x / (SK + 1), c = blockIdx.x % (SK + 1);
  const SnsFftConst& F = *Fc;
  step1_digits(lwe, n, i, acc, ct, c, dig);
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
  if (w < SL) wave_fwd_tail(x, t, F.T, xbuf + w * snsf::SF_PADDED, Df + ((size_t)ct * SR + c * SL + w) * SF_M);
}

// The MAC as a frequency-tiled kernel whose workgroup holds the CMUX's key for 16 frequencies x all 15
// (output, limb) columns in LDS (34.6 KB) and streams 32 ciphertexts' digit spectra through it, writing the
// products O[ct][j*5+t][M] to global memory (a one-kernel step 2 re-reads the ~1 MB per-output key slice
// for every ciphertext: 6.3 GB of L2 traffic per CMUX, measured 497 us against 86).
// Grid: (M / 16) frequency tiles x G ciphertext-group slots; slot g walks the groups g, g + G, ..., so a
// slot stages its key tile once for all its groups.  The first group's digit spectra are requested before
// the key tile is staged, so those loads overlap the LDS fill.
constexpr int MAC_F = 16, MAC_CT = 32, MAC_JT = (SK + 1) * SF_LIMBS;  // 15 (output, limb) columns
#ifndef SNS_MAC_SLOTS
#define SNS_MAC_SLOTS 8  // 16 / 32 measured slower (profiles/r04g_sns_ab.txt)
#endif
constexpr int MAC_SLOTS = SNS_MAC_SLOTS;

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
  __shared__ cd kt[SR * MAC_JT][MAC_F];  // [r * 15 + jt][f]
  constexpr int FT = SF_M / MAC_F;
  const int f0 = (blockIdx.x % FT) * MAC_F;
  const int slots = gridDim.x / FT, groups = (B + MAC_CT - 1) / MAC_CT;
  const int f = threadIdx.x % MAC_F, cl = threadIdx.x / MAC_F;  // MAC_F frequencies x (256 / MAC_F) ciphertext lanes
  static_assert(MAC_CT == 2 * (ST / MAC_F), "two ciphertexts per thread");
  int g = blockIdx.x / FT;
  cd da[SR], db[SR];
  mac_load(Df, g * MAC_CT, B, f0, f, cl, da, db);
  // key tile: row (r, jt) of the CMUX's key = kf_i[(r * 15 + jt) * M + f0 .. + 16]
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

// The register-ended inverse: stage 4's butterflies (q = 1, unit twiddles) each take 4 consecutive
// points, so thread t loads points 4t..4t+3 straight from global memory and transforms them before the
// first LDS write; stage 0's butterfly of thread t yields points t + 256 k, exactly the coefficients the
// thread untwists and rounds, so they stay in registers (store + 5 stages + read -> 4 LDS passes).
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

#ifndef SNS_INV_V2
#define SNS_INV_V2 1
#endif
#if SNS_INV_V2
// Default since round 6 (+2 %: 234.4 -> 229.8 ms per 1024 squashes on one box, 4,369 -> 4,457/s, the squash tests
// bit-exact; profiles/r06i_sns_inv2_ab.txt): the same inverse (every butterfly, twiddle and rounding identical) with
//   * the thread's 12 stage twiddles and 4 untwist factors read once per workgroup into registers (the limbs share them),
//   * LDS-only barriers (s_waitcnt lgkmcnt(0) + s_barrier: __syncthreads also drains vmcnt),
//   * the next limb's 4 points requested before this limb's stages, so their global latency overlaps them.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void r4_dit_w(cd& y0, cd& y1, cd& y2, cd& y3, cd w1, cd w2, cd w3) {
  y1 = snsf::cmulc(y1, w1);
  y2 = snsf::cmulc(y2, w2);
  y3 = snsf::cmulc(y3, w3);
  const cd b0 = snsf::cadd(y0, y2), b1 = snsf::csub(y0, y2), b2 = snsf::cadd(y1, y3), d = snsf::csub(y1, y3);
  const cd b3 = {d.y, -d.x};
  y0 = snsf::cadd(b0, b2);
  y1 = snsf::cadd(b1, b3);
  y2 = snsf::csub(b0, b2);
  y3 = snsf::csub(b1, b3);
}
#endif

// (ciphertext, output j): the 5 inverse transforms one after another by all 256 threads, top limb first;
// each thread untwists and rounds its 8 coefficients (limbs 4..1: |c| < 2^53, exact) and folds them into u128
// Horner sums h = (h << 16) + c, then h = (h << 48) + c_0 for the low limb (|c_0| < 2^85, converted from the
// double's bits); the sums wrap mod 2^128 like the torus, acc_j += h << 16.
// Measured slower (profiles/r04g_sns_ab.txt): a prefetch of the next limb's points and of the accumulator
// words (a barrier waits for every outstanding global load, so the requests only lengthened each pass), and
// the next CMUX's step 1 fused into this kernel (staged words in LDS, each transform wave decomposing its
// own 32 points: 242.4 vs 235.3 ms per 1024).
#ifndef SNS_INV_OCC
#define SNS_INV_OCC 3  // 4 spills (92 B) and runs 25 % slower
#endif
__global__ void __launch_bounds__(ST, SNS_INV_OCC) sns_inv_kernel(const cd* __restrict__ O, u64* __restrict__ acc,
                                                        const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  const int j = blockIdx.x % (SK + 1), ct = blockIdx.x / (SK + 1);
  const SnsFftConst& F = *Fc;
  u128 h[8];
#pragma unroll
  for (int e = 0; e < 8; e++) h[e] = 0;
#pragma unroll 1
  for (int t = SF_LIMBS - 1; t >= 0; t--) {
    const cd* o = O + ((size_t)ct * MAC_JT + j * SF_LIMBS + t) * SF_M;
    cd yr[4];
    fft_inv_reg(o, buf, F.T, yr);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int m = threadIdx.x + 256 * u;
      const cd y = snsf::cmulc(yr[u], F.P[m]);
      if (t > 0) {
        h[2 * u] = snsf::horner16(h[2 * u], __builtin_rint(y.x));
        h[2 * u + 1] = snsf::horner16(h[2 * u + 1], __builtin_rint(y.y));
      } else {
        h[2 * u] = snsf::horner_low(h[2 * u], __builtin_rint(y.x));
        h[2 * u + 1] = snsf::horner_low(h[2 * u + 1], __builtin_rint(y.y));
      }
    }
    __syncthreads();
  }
  u64* a = acc + ((size_t)ct * (SK + 1) + j) * 2 * SN;
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
      const int x = threadIdx.x + 256 * u + SF_M * hh;
      st128(a, x, ld128(a, x) + (h[2 * u + hh] << 16));
    }
}

#if SNS_INV_V2
__global__ void __launch_bounds__(ST, SNS_INV_OCC) sns_inv2_kernel(const cd* __restrict__ O, u64* __restrict__ acc,
                                                         const SnsFftConst* __restrict__ Fc) {
  __shared__ cd buf[SF_M];
  const int j = blockIdx.x % (SK + 1), ct = blockIdx.x / (SK + 1);
  const SnsFftConst& F = *Fc;
  const int t = threadIdx.x;
  const cd* ob = O + ((size_t)ct * MAC_JT + j * SF_LIMBS) * SF_M;
  cd nx[4];  // the next limb's points 4t .. 4t + 3
#pragma unroll
  for (int k = 0; k < 4; k++) nx[k] = ob[(size_t)(SF_LIMBS - 1) * SF_M + 4 * t + k];
  // stage twiddles (dit_stage s = 3, 2, 1: e = (t & (q - 1)) << 2s; stage 0: e = t) and the untwist factors
  cd w[4][3], pu[4];
#pragma unroll
  for (int s = 3; s >= 1; s--) {
    const int lq = 8 - 2 * s, e = (t & ((1 << lq) - 1)) << (2 * s);
    w[s][0] = F.T[e];
    w[s][1] = F.T[2 * e];
    w[s][2] = F.T[3 * e];
  }
  const cd w4 = F.T[0];
  w[0][0] = F.T[t];
  w[0][1] = F.T[2 * t];
  w[0][2] = F.T[3 * t];
#pragma unroll
  for (int u = 0; u < 4; u++) pu[u] = F.P[t + 256 * u];
  u128 h[8];
#pragma unroll
  for (int e = 0; e < 8; e++) h[e] = 0;
#pragma unroll 1
  for (int l = SF_LIMBS - 1; l >= 0; l--) {
    cd y[4] = {nx[0], nx[1], nx[2], nx[3]};
    if (l > 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) nx[k] = ob[(size_t)(l - 1) * SF_M + 4 * t + k];
    }
    r4_dit_w(y[0], y[1], y[2], y[3], w4, w4, w4);  // stage 4: e = 0, the shipped kernel's multiplies by T[0] kept
#pragma unroll
    for (int k = 0; k < 4; k++) buf[4 * t + k] = y[k];
    lds_barrier();
#pragma unroll
    for (int s = 3; s >= 1; s--) {
      const int lq = 8 - 2 * s;
      const int q = 1 << lq, jj = t & (q - 1), base = ((t >> lq) << (lq + 2)) + jj;
      cd z0 = buf[base], z1 = buf[base + q], z2 = buf[base + 2 * q], z3 = buf[base + 3 * q];
      r4_dit_w(z0, z1, z2, z3, w[s][0], w[s][1], w[s][2]);
      buf[base] = z0;
      buf[base + q] = z1;
      buf[base + 2 * q] = z2;
      buf[base + 3 * q] = z3;
      lds_barrier();
    }
#pragma unroll
    for (int k = 0; k < 4; k++) y[k] = buf[t + 256 * k];
    r4_dit_w(y[0], y[1], y[2], y[3], w[0][0], w[0][1], w[0][2]);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const cd yy = snsf::cmulc(y[u], pu[u]);
      if (l > 0) {
        h[2 * u] = snsf::horner16(h[2 * u], __builtin_rint(yy.x));
        h[2 * u + 1] = snsf::horner16(h[2 * u + 1], __builtin_rint(yy.y));
      } else {
        h[2 * u] = snsf::horner_low(h[2 * u], __builtin_rint(yy.x));
        h[2 * u + 1] = snsf::horner_low(h[2 * u + 1], __builtin_rint(yy.y));
      }
    }
    lds_barrier();
  }
  u64* a = acc + ((size_t)ct * (SK + 1) + j) * 2 * SN;
#pragma unroll
  for (int u = 0; u < 4; u++)
#pragma unroll
    for (int hh = 0; hh < 2; hh++) {
      const int x = threadIdx.x + 256 * u + SF_M * hh;
      st128(a, x, ld128(a, x) + (h[2 * u + hh] << 16));
    }
}
#endif

// acc -> LWE over Z_2^128 (dim k N, + body), (lo, hi) pairs: a'_(cN) = A_c[0], a'_(cN + t) = -A_c[N - t]
__global__ void sns_extract_kernel(const u64* __restrict__ acc, u64* __restrict__ out) {
  const int ct = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e > SK * SN) return;
  const u64* a = acc + (size_t)ct * (SK + 1) * 2 * SN;
  u128 y;
  if (e == SK * SN) {
    y = ld128(a + (size_t)SK * 2 * SN, 0);
  } else {
    const int c = e / SN, t = e % SN;
    const u128 v = ld128(a + (size_t)c * 2 * SN, t == 0 ? 0 : SN - t);
    y = t == 0 ? v : (u128)0 - v;
  }
  u64* o = out + ((size_t)ct * (SK * SN + 1) + e) * 2;
  o[0] = (u64)y;
  o[1] = (u64)(y >> 64);
}

}  // namespace

size_t sns_fft_const_bytes() { return sizeof(SnsFftConst); }

void make_sns_fft_const(void* out) {
  SnsFftConst& F = *(SnsFftConst*)out;
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int e = 0; e < SF_M; e++) {
    F.T[e] = cd{(double)cosl(2 * pi * e / SF_M), (double)sinl(2 * pi * e / SF_M)};
    F.P[e] = cd{(double)cosl(pi * e / SN), (double)sinl(pi * e / SN)};
  }
}

size_t sns_fft_key_len(size_t n) { return n * SR * (SK + 1) * SF_LIMBS * SF_M; }  // in cd (16 B)
size_t sns_digit_len(size_t B) { return B * SR * SF_M; }                          // in cd
size_t sns_fft_prod_len(size_t B) { return B * MAC_JT * SF_M; }                   // in cd

hipError_t launch_sns_bsk_to_fft(const u64* bsk_std, void* bsk_fft, size_t polys, const void* d_fconst,
                                 hipStream_t s) {
  sns_bsk_to_fft_kernel<<<(unsigned)polys, ST, 0, s>>>(bsk_std, (cd*)bsk_fft, (const SnsFftConst*)d_fconst);
  return hipGetLastError();
}

hipError_t launch_sns_blind_rotate(const u64* lwe, size_t B, int n, const u64* lut, const void* bsk_fft, u64* acc,
                                   void* D, void* Oprod, const void* d_fconst, hipStream_t s) {
  const SnsFftConst* F = (const SnsFftConst*)d_fconst;
  sns_init_kernel<<<(unsigned)B, 256, 0, s>>>(lwe, n, lut, acc);
  const size_t per_i = (size_t)SR * (SK + 1) * SF_LIMBS * SF_M;
  const size_t groups = (B + MAC_CT - 1) / MAC_CT;
  const unsigned mac_grid = (unsigned)((SF_M / MAC_F) * (MAC_SLOTS < groups ? MAC_SLOTS : groups));
  const unsigned g3 = (unsigned)(B * (SK + 1));
  for (int i = 0; i < n; i++) {
    sns_step1f_kernel<<<g3, ST, 0, s>>>(lwe, n, i, acc, (cd*)D, F);
    sns_mac_kernel<<<mac_grid, ST, 0, s>>>((const cd*)D, (const cd*)bsk_fft + per_i * i, (cd*)Oprod, (int)B);
#if SNS_INV_V2
    sns_inv2_kernel<<<g3, ST, 0, s>>>((const cd*)Oprod, acc, F);
#else
    sns_inv_kernel<<<g3, ST, 0, s>>>((const cd*)Oprod, acc, F);
#endif
  }
  return hipGetLastError();
}

hipError_t launch_sns_extract(const u64* acc, size_t B, u64* out, hipStream_t s) {
  dim3 grid((SK * SN + 1 + 255) / 256, (unsigned)B);
  sns_extract_kernel<<<grid, 256, 0, s>>>(acc, out);
  return hipGetLastError();
}

}  // namespace tfhe
