// sns_fft.h — the f64 negacyclic FFT of the noise-squashing external product (sns.hip),
// shared by the device kernels and the host accuracy check (tools/sns_fft_check.cpp).
//
// The squashing ring is Z_Q (Q = p1 p2 ~ 2^128, see sns.hip).  Its product digits x BSK is computed as
// EXACT integer convolutions: the BSK coefficient, centred in (-Q/2, Q/2] and rounded to a multiple of
// 2^SF_DROP (the load-time rounding; oracle: or_sns_bsk_round), is split into SF_LIMBS balanced 16-bit
// limbs, and each digit-polynomial x limb-polynomial convolution (|value| <= 9 * 2048 * 2^23 * 2^15 =
// 2^52.2) is one f64 FFT product whose rounding error stays far below 1/2 (tools/sns_fft_check.cpp
// measures it), so rint() returns the exact integer and the product mod Q is bit-identical to the
// oracle's NTT over p1, p2.  The limbs recombine with the weights 2^(SF_DROP + 16 t) mod p.
//
// Transform: N = 2048 real coefficients folded to M = 1024 complex z_m = (a_m + i a_{m+1024}) psi^m,
// psi = e^{i pi / 2048} (so the cyclic DFT of z evaluates a at the odd powers of psi), then a radix-4
// decimation-in-frequency DFT (5 stages, natural order in, base-4 digit-reversed out); the inverse is
// the mirror decimation-in-time pass with conjugate twiddles (digit-reversed in, natural out), scaled by
// M (the 1/M is folded into the key spectra).  Spectra stay in digit-reversed order: the MAC is
// pointwise, so key and digits only need the same order.
#pragma once

#if defined(__HIPCC__)
#define SF_HD __host__ __device__ __forceinline__
#else
#define SF_HD inline
#endif

namespace tfhe {
namespace snsf {

struct cd {
  double x, y;
};

constexpr int SF_N = 2048, SF_M = 1024, SF_NT = 256;  // coefficients, complex points, threads per transform
constexpr int SF_LIMBS = 7, SF_LIMB_BITS = 16, SF_DROP = 16;

SF_HD cd cadd(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
SF_HD cd csub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
SF_HD cd cmul(cd a, cd b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
SF_HD cd cmulc(cd a, cd b) { return {a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y}; }  // a * conj(b)
SF_HD cd cmac(cd acc, cd a, cd b) { return {acc.x + a.x * b.x - a.y * b.y, acc.y + a.x * b.y + a.y * b.x}; }

// One radix-4 DIF butterfly of stage s (span L = M / 4^s) for thread t < 256; T[e] = e^{2 pi i e / M}.
SF_HD void dif_stage(cd* a, int s, int t, const cd* T) {
  const int lq = 8 - 2 * s;  // log2(L / 4)
  const int q = 1 << lq, j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j;
  const cd x0 = a[base], x1 = a[base + q], x2 = a[base + 2 * q], x3 = a[base + 3 * q];
  const cd a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), d = csub(x1, x3);
  const cd a3 = {-d.y, d.x};  // i (x1 - x3)
  const int e = j << (2 * s);  // j * M / L
  a[base] = cadd(a0, a2);
  a[base + q] = cmul(cadd(a1, a3), T[e]);
  a[base + 2 * q] = cmul(csub(a0, a2), T[2 * e]);
  a[base + 3 * q] = cmul(csub(a1, a3), T[3 * e]);
}

// The inverse butterfly of stage s: conjugate twiddles first, then the radix-4 DFT with -i.
SF_HD void dit_stage(cd* a, int s, int t, const cd* T) {
  const int lq = 8 - 2 * s;
  const int q = 1 << lq, j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j;
  const int e = j << (2 * s);
  const cd y0 = a[base], y1 = cmulc(a[base + q], T[e]), y2 = cmulc(a[base + 2 * q], T[2 * e]),
           y3 = cmulc(a[base + 3 * q], T[3 * e]);
  const cd b0 = cadd(y0, y2), b1 = csub(y0, y2), b2 = cadd(y1, y3), d = csub(y1, y3);
  const cd b3 = {d.y, -d.x};  // -i (y1 - y3)
  a[base] = cadd(b0, b2);
  a[base + q] = cadd(b1, b3);
  a[base + 2 * q] = csub(b0, b2);
  a[base + 3 * q] = csub(b1, b3);
}

}  // namespace snsf
}  // namespace tfhe
