// fft1k.h — the 1024-point complex DFT of one N = 2048 polynomial in ONE wavefront (gfx950): 16 complex per lane,
// M = 1024 = 16 x 4 x 16.  One fixed f64 operation sequence, restated in oracle/fft_oracle.c (fft1k_fwd / fft1k_inv);
// contraction stays off in every file that includes this header.
//
// Natural input: slot e of lane L holds z_n, n = L + 64 e, z_n = (a_n + i a_{n + 1024}) zeta^n, zeta = e^{2 pi i / 4096}.
//   A  DFT16 over the slots (e -> k1), then x[k1] *= ta[k1][L] = zeta^{L (1 + 4 k1)} (the lane part of the twist
//      rides here; the slot part zeta^{64 e} is a compile-time constant applied before)
//   X  two register exchanges: v_permlane32_swap (slot bit 3 <-> lane bit 5), v_permlane16_swap (slot bit 2 <->
//      lane bit 4) -- 64 cross-lane moves, no LDS
//   B  radix-4 over the two slot bits that arrived (l1 -> m0), then x *= tb[m0][l0] = e^{2 pi i l0 m0 / 64}
//   T  ONE LDS transpose of lane bits 0..3 with the 4 slot bits (XOR-swizzled or padded rows: conflict-free)
//   C  DFT16 over the slots (l0 -> m1)
// Device order out: slot m1 of lane L holds Z[k], k = (L & 3) + 4 (L >> 4) + 16 ((L >> 2) & 3) + 64 m1.  The inverse
// runs the stages reversed with conjugate twiddles (no 1/M).  Against the two-wave form it replaces (two 512-point
// halves + an LDS combine exchange, fft512.h), a polynomial costs one LDS transpose instead of four plus the pair
// exchange, and no wave pairs wait for each other.
#pragma once
#pragma clang fp contract(off)
#include "fft512.h"

namespace tfhe {
namespace fft1k {
using namespace fftk;

constexpr int M1 = 1024;
constexpr double C16 = 0.92387953251128675613, S16 = 0.38268343236508977173;  // cos, sin (pi / 8)
// table (complex, global memory and LDS): ta [16][64] | tb [4][16]
constexpr int K_TA = 0, K_TB = 1024, K_C64 = 1088;
// per-wave LDS area: the transpose's element (hi, s, l0) (hi = lane >> 4, slot s, l0 = lane & 15); also the
// 2048-u64 rotation image and the spectra [slot][lane].  Row side: lane (hi, l0) touches (hi, s, l0), s = 0..15;
// column side: lane (hi, l0) touches (hi, l0, c), c = 0..15.  Layouts (all conflict-free for every 16-lane group):
// F1_SWZ = 2 (round 4 default) skewed 16 KB rows, 1 XOR-swizzled 16 KB rows, 0 rows padded to 17 complex (17 KB).
// 16 KB areas let a 2-ciphertext workgroup fit twice per CU (80 KB).
#ifndef F1_SWZ
#define F1_SWZ 2
#endif
#if F1_SWZ == 2
// skewed rows: element (hi, s, l0) at 256 hi + 16 s + ((l0 + s) & 15).  Row side (lane l0, s = 0..15) and column
// side (lane = row s, c = 0..15) are each "one of two lane bases + an immediate": the wrap picks the base.
constexpr int AREA_C64 = 1024;
struct TAddr {
  int w1, w2, r1, r2, l0;  // row side: w1 + 17 s (s < 16 - l0) or w2 + 17 s; column side: r1 + c or r2 + c
  __device__ __forceinline__ TAddr(int lane) {
    const int hi = lane >> 4;
    l0 = lane & 15;
    w1 = 256 * hi + l0;
    w2 = w1 - 16;
    r1 = 256 * hi + 17 * l0;
    r2 = r1 - 16;
  }
  __device__ __forceinline__ int row(int s) const { return (s < 16 - l0 ? w1 : w2) + 17 * s; }
  __device__ __forceinline__ int col(int c) const { return (c < 16 - l0 ? r1 : r2) + c; }
};
#elif F1_SWZ == 1
// XOR rows: element (hi, s, l0) at 256 hi + 16 s + (l0 ^ s)
constexpr int AREA_C64 = 1024;
struct TAddr {
  int hi, l0;
  __device__ __forceinline__ TAddr(int lane) : hi(lane >> 4), l0(lane & 15) {}
  __device__ __forceinline__ int row(int s) const { return 256 * hi + 16 * s + (l0 ^ s); }
  __device__ __forceinline__ int col(int c) const { return 256 * hi + 16 * l0 + (c ^ l0); }
};
#else
// padded rows of 17 complex (17 KB areas)
constexpr int AS = 17, AH = 272, AREA_C64 = 4 * AH;
struct TAddr {
  int w, r;
  __device__ __forceinline__ TAddr(int lane) : w(AH * (lane >> 4) + (lane & 15)), r(AH * (lane >> 4) + AS * (lane & 15)) {}
  __device__ __forceinline__ int row(int s) const { return w + AS * s; }
  __device__ __forceinline__ int col(int c) const { return r + c; }
};
#endif

// cos / sin (2 pi t / m) evaluated at compile time with the host table generator's series (fftk::twiddle)
namespace ctw16 {
constexpr ctw::c64 oct(unsigned t, unsigned m) {
  const double x = (double)t * (6.28318530717958647692 / (double)m);
  return ctw::c64{ctw::cos_s(x), ctw::sin_s(x)};
}
constexpr ctw::c64 quarter(unsigned t, unsigned m) {
  if (8 * t > m) {
    const ctw::c64 u = oct(m / 4 - t, m);
    return ctw::c64{u.y, u.x};
  }
  return oct(t, m);
}
constexpr ctw::c64 slot(int e) { return quarter(64u * (unsigned)e, 4096u); }  // 64 e <= 960 <= 4096 / 4
constexpr ctw::c64 SLOT[16] = {slot(0), slot(1), slot(2),  slot(3),  slot(4),  slot(5),  slot(6),  slot(7),
                               slot(8), slot(9), slot(10), slot(11), slot(12), slot(13), slot(14), slot(15)};
}  // namespace ctw16

// radix-4 DFT in place, natural order: t0 = a + c, t1 = a - c, t2 = b + d, t3 = b - d;
// (a, b, c, d) <- (t0 + t2, t1 + i t3, t0 - t2, t1 - i t3) (INV: b and d swapped)
template <bool INV>
__device__ __forceinline__ void r4(double& ar, double& ai, double& br, double& bi, double& cr, double& ci, double& dr,
                                   double& di) {
  const double t0r = ar + cr, t0i = ai + ci, t1r = ar - cr, t1i = ai - ci;
  const double t2r = br + dr, t2i = bi + di, t3r = br - dr, t3i = bi - di;
  ar = t0r + t2r;
  ai = t0i + t2i;
  cr = t0r - t2r;
  ci = t0i - t2i;
  const double pr = t1r - t3i, pi = t1i + t3r, qr = t1r + t3i, qi = t1i - t3r;
  br = INV ? qr : pr;
  bi = INV ? qi : pi;
  dr = INV ? pr : qr;
  di = INV ? pi : qi;
}

// t * W16^K (INV: conjugate), the oracle's w16
template <bool INV, int K>
__device__ __forceinline__ void w16(double& re, double& im) {
  if constexpr (K == 1) cmul<INV>(re, im, make_double2(C16, S16));
  else if constexpr (K == 3) cmul<INV>(re, im, make_double2(S16, C16));
  else if constexpr (K == 9) cmul<INV>(re, im, make_double2(-C16, -S16));
  else if constexpr (K == 2) w8<INV, 1>(re, im);
  else if constexpr (K == 6) w8<INV, 3>(re, im);
  else w8<INV, 2>(re, im);  // K == 4: i
}

// F1_DFT16_FMA 1 (default since round 5): the sqrt(1/2) of the W16^2 / W16^6 twiddles folded into the second radix-4
// pass as fmas (as fft512.h's FFT_DFT8_FMA): group k0 = 2 takes b = s u9, d = s u11 (t2, t3 scaled by s: 4 fmas per
// output pair), groups 1 and 3 take c = s u6 / s u14 (t0, t1 = a +- s u: 2 fmas each) -- 8 multiplies fewer per
// DFT16, -32 f64 per wave and CMUX.  Restated in oracle/fft_oracle.c:dft16; 0 = the round-4 form.
#ifndef F1_DFT16_FMA
#define F1_DFT16_FMA 1
#endif
// w8^J (J = 1, 3) without its sqrt(1/2) factor: the oracle's w8u
template <bool INV, int J>
__device__ __forceinline__ void w8u(double& re, double& im) {
  const double p = re, q = im;
  if (J == 1) {
    if (!INV) { re = p - q; im = p + q; }
    else { re = p + q; im = q - p; }
  } else {
    if (!INV) { re = -(p + q); im = p - q; }
    else { re = q - p; im = -(p + q); }
  }
}
// r4 with c = s cu (cu given unscaled): t0 = a + s cu, t1 = a - s cu as fmas, the rest as r4
template <bool INV>
__device__ __forceinline__ void r4_cs(double& ar, double& ai, double& br, double& bi, double& cr, double& ci, double& dr,
                                      double& di) {
  const double t0r = __builtin_fma(SQRT1_2, cr, ar), t0i = __builtin_fma(SQRT1_2, ci, ai);
  const double t1r = __builtin_fma(-SQRT1_2, cr, ar), t1i = __builtin_fma(-SQRT1_2, ci, ai);
  const double t2r = br + dr, t2i = bi + di, t3r = br - dr, t3i = bi - di;
  ar = t0r + t2r;
  ai = t0i + t2i;
  cr = t0r - t2r;
  ci = t0i - t2i;
  const double pr = t1r - t3i, pi = t1i + t3r, qr = t1r + t3i, qi = t1i - t3r;
  br = INV ? qr : pr;
  bi = INV ? qi : pi;
  dr = INV ? pr : qr;
  di = INV ? pi : qi;
}
// r4 with b = s bu, d = s du (unscaled): t2, t3 carry the factor s into the output fmas
template <bool INV>
__device__ __forceinline__ void r4_bds(double& ar, double& ai, double& br, double& bi, double& cr, double& ci, double& dr,
                                       double& di) {
  const double t0r = ar + cr, t0i = ai + ci, t1r = ar - cr, t1i = ai - ci;
  const double t2r = br + dr, t2i = bi + di, t3r = br - dr, t3i = bi - di;  // / s
  ar = __builtin_fma(SQRT1_2, t2r, t0r);
  ai = __builtin_fma(SQRT1_2, t2i, t0i);
  cr = __builtin_fma(-SQRT1_2, t2r, t0r);
  ci = __builtin_fma(-SQRT1_2, t2i, t0i);
  // p = t1 + i t3, q = t1 - i t3 with t3 = s t3'
  const double pr = __builtin_fma(-SQRT1_2, t3i, t1r), pi = __builtin_fma(SQRT1_2, t3r, t1i);
  const double qr = __builtin_fma(SQRT1_2, t3i, t1r), qi = __builtin_fma(-SQRT1_2, t3r, t1i);
  br = INV ? qr : pr;
  bi = INV ? qi : pi;
  dr = INV ? pr : qr;
  di = INV ? pi : qi;
}

// 16-point DFT in registers, natural order in and out: radix-4 over n1 (positions n0 + 4 k0), W16^{n0 k0}, radix-4
// over n0 (positions 4 k0 + k1), X[k0 + 4 k1] = position 4 k0 + k1 (a renaming)
template <bool INV>
__device__ __forceinline__ void dft16(double (&xr)[16], double (&xi)[16]) {
#pragma unroll
  for (int n0 = 0; n0 < 4; n0++)
    r4<INV>(xr[n0], xi[n0], xr[n0 + 4], xi[n0 + 4], xr[n0 + 8], xi[n0 + 8], xr[n0 + 12], xi[n0 + 12]);
#if F1_DFT16_FMA
  r4<INV>(xr[0], xi[0], xr[1], xi[1], xr[2], xi[2], xr[3], xi[3]);
  w16<INV, 1>(xr[5], xi[5]);  // group 1: W^0, W^1, s u(W^2), W^3
  w8u<INV, 1>(xr[6], xi[6]);
  w16<INV, 3>(xr[7], xi[7]);
  r4_cs<INV>(xr[4], xi[4], xr[5], xi[5], xr[6], xi[6], xr[7], xi[7]);
  w8u<INV, 1>(xr[9], xi[9]);  // group 2: W^0, s u(W^2), W^4 = i, s u(W^6)
  w16<INV, 4>(xr[10], xi[10]);
  w8u<INV, 3>(xr[11], xi[11]);
  r4_bds<INV>(xr[8], xi[8], xr[9], xi[9], xr[10], xi[10], xr[11], xi[11]);
  w16<INV, 3>(xr[13], xi[13]);  // group 3: W^0, W^3, s u(W^6), W^9
  w8u<INV, 3>(xr[14], xi[14]);
  w16<INV, 9>(xr[15], xi[15]);
  r4_cs<INV>(xr[12], xi[12], xr[13], xi[13], xr[14], xi[14], xr[15], xi[15]);
#else
  w16<INV, 1>(xr[5], xi[5]);
  w16<INV, 2>(xr[6], xi[6]);
  w16<INV, 3>(xr[7], xi[7]);
  w16<INV, 2>(xr[9], xi[9]);
  w16<INV, 4>(xr[10], xi[10]);
  w16<INV, 6>(xr[11], xi[11]);
  w16<INV, 3>(xr[13], xi[13]);
  w16<INV, 6>(xr[14], xi[14]);
  w16<INV, 9>(xr[15], xi[15]);
#pragma unroll
  for (int k0 = 0; k0 < 4; k0++)
    r4<INV>(xr[4 * k0], xi[4 * k0], xr[4 * k0 + 1], xi[4 * k0 + 1], xr[4 * k0 + 2], xi[4 * k0 + 2], xr[4 * k0 + 3],
            xi[4 * k0 + 3]);
#endif
  double yr[16], yi[16];
#pragma unroll
  for (int k0 = 0; k0 < 4; k0++)
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) {
      yr[k0 + 4 * k1] = xr[4 * k0 + k1];
      yi[k0 + 4 * k1] = xi[4 * k0 + k1];
    }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    xr[k] = yr[k];
    xi[k] = yi[k];
  }
}

// slot bit 3 <-> lane bit 5 and slot bit 2 <-> lane bit 4 (an involution)
__device__ __forceinline__ void exchange_hi(double (&xr)[16], double (&xi)[16]) {
#pragma unroll
  for (int s = 0; s < 8; s++) {
    swap32_d(xr[s], xr[s + 8]);
    swap32_d(xi[s], xi[s + 8]);
  }
#pragma unroll
  for (int s = 0; s < 16; s++)
    if ((s & 4) == 0) {
      swap16_d(xr[s], xr[s + 4]);
      swap16_d(xi[s], xi[s + 4]);
    }
}

// this lane's pass-B twiddles tb[m][lane & 15], m = 1..3
struct TwB {
  double2 w[4];
  __device__ __forceinline__ void load(const double2* tab, int lane) {
#pragma unroll
    for (int m = 1; m < 4; m++) w[m] = tab[K_TB + 16 * m + (lane & 15)];
  }
};

// forward: natural order in (slot e <-> n = L + 64 e, the twist NOT yet applied), device order out.  ta: pass A's
// table (LDS), area: this wave's LDS area (the transpose)
__device__ __forceinline__ void fft1k_fwd(double (&xr)[16], double (&xi)[16], double2* area, int lane,
                                          const double2* ta, const TwB& tb) {
#pragma unroll
  for (int e = 1; e < 16; e++) cmul<false>(xr[e], xi[e], make_double2(ctw16::SLOT[e].x, ctw16::SLOT[e].y));
  dft16<false>(xr, xi);
#pragma unroll
  for (int k = 0; k < 16; k++) cmul<false>(xr[k], xi[k], ta[64 * k + lane]);
  exchange_hi(xr, xi);
#pragma unroll
  for (int g = 0; g < 4; g++) {
    r4<false>(xr[g], xi[g], xr[g + 4], xi[g + 4], xr[g + 8], xi[g + 8], xr[g + 12], xi[g + 12]);
#pragma unroll
    for (int m = 1; m < 4; m++) cmul<false>(xr[g + 4 * m], xi[g + 4 * m], tb.w[m]);
  }
  const TAddr ad(lane);
#pragma unroll
  for (int s = 0; s < 16; s++) area[ad.row(s)] = make_double2(xr[s], xi[s]);
  lds_order();
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const double2 v = area[ad.col(r)];
    xr[r] = v.x;
    xi[r] = v.y;
  }
  lds_order();
  dft16<false>(xr, xi);
}

// inverse (no 1/M): device order in, natural order out (the untwist applied)
__device__ __forceinline__ void fft1k_inv(double (&xr)[16], double (&xi)[16], double2* area, int lane,
                                          const double2* ta, const TwB& tb) {
  dft16<true>(xr, xi);
  const TAddr ad(lane);
#pragma unroll
  for (int r = 0; r < 16; r++) area[ad.col(r)] = make_double2(xr[r], xi[r]);
  lds_order();
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const double2 v = area[ad.row(s)];
    xr[s] = v.x;
    xi[s] = v.y;
  }
  lds_order();
#pragma unroll
  for (int g = 0; g < 4; g++) {
#pragma unroll
    for (int m = 1; m < 4; m++) cmul<true>(xr[g + 4 * m], xi[g + 4 * m], tb.w[m]);
    r4<true>(xr[g], xi[g], xr[g + 4], xi[g + 4], xr[g + 8], xi[g + 8], xr[g + 12], xi[g + 12]);
  }
  exchange_hi(xr, xi);
#pragma unroll
  for (int k = 0; k < 16; k++) cmul<true>(xr[k], xi[k], ta[64 * k + lane]);
  dft16<true>(xr, xi);
#pragma unroll
  for (int e = 1; e < 16; e++) cmul<true>(xr[e], xi[e], make_double2(ctw16::SLOT[e].x, ctw16::SLOT[e].y));
}

}  // namespace fft1k
}  // namespace tfhe
