// fft512p.h — the 512-point negacyclic transform of the P-GATE FFT64 path (N = 1024) with ONE LDS transpose
// (round 4), in two shapes over the same f64 operation sequence (restated in oracle/fft_oracle.c: fft512p_fwd /
// fft512p_inv; contraction stays off in every file that includes this header):
//   pair   two polynomials in one wave (16 slots per lane: slots 8p + e hold polynomial p), the batch kernel's
//          shape: both components of a ciphertext at one decomposition level, or the two outputs of a CMUX
//   single one polynomial in one wave (8 slots per lane), for the latency kernel, the key conversion and tests;
//          after the transpose lanes 32-63 mirror lanes 0-31
// M = 512 = 8 x 4 x 16.  Natural input: slot e of lane L holds z_n, n = L + 64 e, z_n = a_n + i a_{n + 512}.
//   A  x[e] *= zeta^{64 e} (e > 0, compile-time constants), DFT8 over the slots (e -> k2), x[k2] *= ta[k2][L] =
//      zeta^{L (1 + 4 k2)}, zeta = e^{2 pi i / 2048} (twist and the first twiddle merged, fft512.h's TW_A table)
//   X  v_permlane32_swap (slot bit 2 <-> lane bit 5), v_permlane16_swap (slot bit 1 <-> lane bit 4): lane
//      L' = l0 + 16 (k2 >> 1) holds slot s' = (k2 & 1) + 2 l1  (L = l0 + 16 l1)
//   B  radix-4 over l1 (slots g + 2 l1, g = k2 & 1) -> m0, then x *= tb[m0][l0] = e^{2 pi i l0 m0 / 64}  (m0 > 0)
//   T  ONE LDS transpose: lane lam = g + 2 m0 + 8 k2b2 + 16 k2b1 + 32 p (k2 = g + 2 k2b1 + 4 k2b2) holds slot l0
//      (rows of 17 complex in blocks of 16 rows: conflict-free in both directions, DS immediate offsets only)
//   C  DFT16 over l0 -> m1 (fft1k.h's dft16)
// Device order: slot m1 of lane lam (lam < 32, polynomial p's lanes 32 p + lam) holds Z[k],
//   k = (lam & 1) + 2 ((lam >> 4) & 1) + 4 ((lam >> 3) & 1) + 8 ((lam >> 1) & 3) + 32 m1,
// stored at index d = lam + 32 m1 of the polynomial's 512 (the key's layout too).  The inverse runs the stages
// reversed with conjugate twiddles (no 1/M).  Against fft512.h's three radix-8 passes (two LDS round trips per
// polynomial) a pair costs one round trip: 16 writes + 16 reads of 1 KB instead of 32 + 32.
#pragma once
#pragma clang fp contract(off)
#include "fft1k.h"

namespace tfhe {
namespace fftp {
using namespace fftk;
using fft1k::dft16;
using fft1k::r4;

constexpr int MP = 512;
// table (complex, global): ta [8][64] | tb [4][16]
constexpr int P_TA = 0, P_TB = 512, P_C64 = 576;
// per-wave transpose area: row lam at 17 (lam & 15) + 272 (lam >> 4), 64 rows of 16 complex (pair) or 32 (single)
constexpr int PA_C64 = 1088, PS_C64 = 544;

// this lane's twiddles ta[k][lane] (8) and tb[m][lane & 15] (m = 1..3): held in registers (TwP) or read from a
// copy of the table in LDS at each use (TwL: 22 registers fewer, 11 ds_read_b128 more per transform)
struct TwP {
  double2 ra[8], rb[4];
  __device__ __forceinline__ void load(const double2* __restrict__ tab, int lane) {
#pragma unroll
    for (int k = 0; k < 8; k++) ra[k] = tab[P_TA + 64 * k + lane];
#pragma unroll
    for (int m = 1; m < 4; m++) rb[m] = tab[P_TB + 16 * m + (lane & 15)];
  }
  __device__ __forceinline__ double2 a(int k) const { return ra[k]; }
  __device__ __forceinline__ double2 b(int m) const { return rb[m]; }
};
struct TwL {
  const double2* ta;  // LDS table + lane
  const double2* tb;  // LDS table + (lane & 15)
  __device__ __forceinline__ TwL(const double2* lds_tab, int lane)
      : ta(lds_tab + P_TA + lane), tb(lds_tab + P_TB + (lane & 15)) {}
  __device__ __forceinline__ double2 a(int k) const { return ta[64 * k]; }
  __device__ __forceinline__ double2 b(int m) const { return tb[16 * m]; }
};

typedef double d8[8];
__device__ __forceinline__ d8& half(double (&x)[16], int p) { return *reinterpret_cast<d8*>(&x[8 * p]); }

// per-lane transpose bases (complex index): pre-transpose side (lane L': writes slot s at wb + off(s)) and
// post-transpose side (lane lam reads slot l0 at rb + l0)
struct TBaseP {
  int wb, rb;
  __device__ __forceinline__ explicit TBaseP(int lane, bool single)
      : wb(136 * (lane >> 5) + 272 * ((lane >> 4) & 1) + (lane & 15)),
        rb(17 * (lane & 15) + 272 * ((single ? lane & 31 : lane) >> 4)) {}
};
__host__ __device__ constexpr int woff(int s) { return 17 * (s & 7) + 544 * (s >> 3); }

// stage A on polynomial half h (forward)
template <class TW>
__device__ __forceinline__ void stage_a_fwd(d8& xr, d8& xi, const TW& w) {
  twist_slots<false>(xr, xi);
  dft8<false>(xr, xi);
#pragma unroll
  for (int k = 0; k < 8; k++) cmul<false>(xr[k], xi[k], w.a(k));
}
template <class TW>
__device__ __forceinline__ void stage_a_inv(d8& xr, d8& xi, const TW& w) {
#pragma unroll
  for (int k = 0; k < 8; k++) cmul<true>(xr[k], xi[k], w.a(k));
  dft8<true>(xr, xi);
  twist_slots<true>(xr, xi);
}
// slot bit 2 <-> lane bit 5, slot bit 1 <-> lane bit 4 within one 8-slot half (an involution)
__device__ __forceinline__ void exchange8(d8& xr, d8& xi) {
#pragma unroll
  for (int s = 0; s < 4; s++) {
    swap32_d(xr[s], xr[s + 4]);
    swap32_d(xi[s], xi[s + 4]);
  }
#pragma unroll
  for (int s = 0; s < 8; s++)
    if ((s & 2) == 0) {
      swap16_d(xr[s], xr[s + 2]);
      swap16_d(xi[s], xi[s + 2]);
    }
}
template <bool INV, class TW>
__device__ __forceinline__ void stage_b(d8& xr, d8& xi, const TW& w) {
#pragma unroll
  for (int g = 0; g < 2; g++) {
    if (INV) {
#pragma unroll
      for (int m = 1; m < 4; m++) cmul<true>(xr[g + 2 * m], xi[g + 2 * m], w.b(m));
    }
    r4<INV>(xr[g], xi[g], xr[g + 2], xi[g + 2], xr[g + 4], xi[g + 4], xr[g + 6], xi[g + 6]);
    if (!INV) {
#pragma unroll
      for (int m = 1; m < 4; m++) cmul<false>(xr[g + 2 * m], xi[g + 2 * m], w.b(m));
    }
  }
}

// pair forward: natural order in (slots 8 p + e), device order out (lane 32 p + lam, slot m1)
template <class TW>
__device__ __forceinline__ void fwd_pair(double (&xr)[16], double (&xi)[16], double2* area, TBaseP tb, const TW& w) {
#pragma unroll
  for (int p = 0; p < 2; p++) stage_a_fwd(half(xr, p), half(xi, p), w);
#pragma unroll
  for (int p = 0; p < 2; p++) exchange8(half(xr, p), half(xi, p));
#pragma unroll
  for (int p = 0; p < 2; p++) stage_b<false>(half(xr, p), half(xi, p), w);
#pragma unroll
  for (int s = 0; s < 16; s++) area[tb.wb + woff(s)] = make_double2(xr[s], xi[s]);
  lds_order();
#pragma unroll
  for (int l = 0; l < 16; l++) {
    const double2 v = area[tb.rb + l];
    xr[l] = v.x;
    xi[l] = v.y;
  }
  lds_order();
  dft16<false>(xr, xi);
}

// pair inverse (no 1/M): device order in, natural order out
template <class TW>
__device__ __forceinline__ void inv_pair(double (&xr)[16], double (&xi)[16], double2* area, TBaseP tb, const TW& w) {
  dft16<true>(xr, xi);
#pragma unroll
  for (int l = 0; l < 16; l++) area[tb.rb + l] = make_double2(xr[l], xi[l]);
  lds_order();
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const double2 v = area[tb.wb + woff(s)];
    xr[s] = v.x;
    xi[s] = v.y;
  }
  lds_order();
#pragma unroll
  for (int p = 0; p < 2; p++) stage_b<true>(half(xr, p), half(xi, p), w);
#pragma unroll
  for (int p = 0; p < 2; p++) exchange8(half(xr, p), half(xi, p));
#pragma unroll
  for (int p = 0; p < 2; p++) stage_a_inv(half(xr, p), half(xi, p), w);
}

// single forward: in = 8 slots (natural), out = 16 slots (device order, lane lam & 31); tb = TBaseP(lane, true)
template <class TW>
__device__ __forceinline__ void fwd_single(const double (&ar)[8], const double (&ai)[8], double (&xr)[16],
                                           double (&xi)[16], double2* area, TBaseP tb, const TW& w) {
  d8 yr, yi;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    yr[e] = ar[e];
    yi[e] = ai[e];
  }
  stage_a_fwd(yr, yi, w);
  exchange8(yr, yi);
  stage_b<false>(yr, yi, w);
#pragma unroll
  for (int s = 0; s < 8; s++) area[tb.wb + woff(s)] = make_double2(yr[s], yi[s]);
  lds_order();
#pragma unroll
  for (int l = 0; l < 16; l++) {
    const double2 v = area[tb.rb + l];
    xr[l] = v.x;
    xi[l] = v.y;
  }
  lds_order();
  dft16<false>(xr, xi);
}

// single inverse: in = 16 slots (device order, lanes lam and lam + 32 alike), out = 8 slots (natural)
template <class TW>
__device__ __forceinline__ void inv_single(double (&xr)[16], double (&xi)[16], double (&ar)[8], double (&ai)[8],
                                           double2* area, TBaseP tb, const TW& w) {
  dft16<true>(xr, xi);
#pragma unroll
  for (int l = 0; l < 16; l++) area[tb.rb + l] = make_double2(xr[l], xi[l]);  // lanes 32-63 rewrite the same
  lds_order();
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const double2 v = area[tb.wb + woff(s)];
    ar[s] = v.x;
    ai[s] = v.y;
  }
  lds_order();
  stage_b<true>(ar, ai, w);
  exchange8(ar, ai);
  stage_a_inv(ar, ai, w);
}

}  // namespace fftp
}  // namespace tfhe
