// sns_fft.h — the f64 negacyclic FFT of the noise-squashing external product (sns.hip) and the
// native 2^128 word arithmetic around it, shared by the device kernels and the host checks
// (tools/sns_fft_check.cpp: FFT accuracy; tools/sns_native_check.cpp: the whole CMUX vs the oracle).
//
// The squashing ring is the native 2^128 torus.  Every BSK word, read as a signed 128-bit integer and
// rounded to a multiple of 2^16 (the load-time rounding; oracle: or_sns_bsk_round), is 2^16 x a 112-bit
// integer, split into SF_LIMBS = 5 limbs (round 4; seven 16-bit limbs before): limb 0 is the balanced
// low 48 bits, limbs 1..4 are balanced 16-bit limbs (the top one keeps the remainder).
//  * limbs 1..4: each digit-polynomial x limb-polynomial convolution (|value| <= 9 * 2048 * 2^23 * 2^15 =
//    2^52.2) is one f64 FFT product whose rounding error stays far below 1/2 (tools/sns_fft_check.cpp
//    measures it), so rint() returns the exact integer;
//  * limb 0 (|l| <= 2^47): its products reach 2^84 and are NOT exact; their f64 rounding error (measured by
//    tools/sns_fft_check.cpp: <= 2^28 for random operands, 2^33.3 for the all-maximum worst case) lands at
//    weight 2^16 of the accumulator, <= 2^49.3 against the squashed ciphertext's ~2^64 noise.  Only the low limb can be inexact: an error in limb t > 0 is multiplied by 2^(64 + 16 (t - 1)).
//    Its value is defined by THIS file's operation order -- explicit fma in cmul / cmulc / cmac,
//    contraction off, the stage order below -- which oracle/sns_oracle.c restates word for word, so the
//    device, the host replay and the oracle agree bit for bit.
// The limbs recombine as h = ((c4 2^16 + c3) 2^16 + c2) 2^16 + c1) 2^48 + c0, acc += h << 16 mod 2^128.
//
// Transform: N = 2048 real coefficients folded to M = 1024 complex z_m = (a_m + i a_{m+1024}) psi^m,
// psi = e^{i pi / 2048} (so the cyclic DFT of z evaluates a at the odd powers of psi), then a radix-4
// decimation-in-frequency DFT (5 stages, natural order in, base-4 digit-reversed out); the inverse is
// the mirror decimation-in-time pass with conjugate twiddles (digit-reversed in, natural out), scaled by
// M (the 1/M is folded into the key spectra).  Spectra stay in digit-reversed order: the MAC is
// pointwise, so key and digits only need the same order.
#pragma once
#if defined(__clang__)
#pragma clang fp contract(off)
#endif

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
constexpr int SF_LIMBS = 5, SF_LIMB_BITS = 16, SF_LOW_BITS = 48, SF_DROP = 16;

// complex arithmetic with explicit fused multiply-adds (oracle/sns_oracle.c: sf_cmul, sf_cmulc, sf_cmac)
SF_HD cd cadd(cd a, cd b) { return {a.x + b.x, a.y + b.y}; }
SF_HD cd csub(cd a, cd b) { return {a.x - b.x, a.y - b.y}; }
SF_HD cd cmul(cd a, cd b) { return {__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x)}; }
SF_HD cd cmulc(cd a, cd b) {  // a * conj(b)
  return {__builtin_fma(a.x, b.x, a.y * b.y), __builtin_fma(a.y, b.x, -(a.x * b.y))};
}
SF_HD cd cmac(cd acc, cd a, cd b) {
  return {__builtin_fma(-a.y, b.y, __builtin_fma(a.x, b.x, acc.x)), __builtin_fma(a.y, b.x, __builtin_fma(a.x, b.y, acc.y))};
}

// Radix-4 DIF butterfly with output twiddles T[e k] (e = j * 4^s), and its DIT inverse (conjugate
// input twiddles, then the butterfly with -i): dit(dif(x)) = 4 x.
SF_HD void r4_dif(cd& x0, cd& x1, cd& x2, cd& x3, int e, const cd* T) {
  const cd a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), d = csub(x1, x3);
  const cd a3 = {-d.y, d.x};  // i (x1 - x3)
  x0 = cadd(a0, a2);
  x1 = cmul(cadd(a1, a3), T[e]);  // T[0] = 1 exactly: e = 0 needs no branch
  x2 = cmul(csub(a0, a2), T[2 * e]);
  x3 = cmul(csub(a1, a3), T[3 * e]);
}
SF_HD void r4_dif0(cd& x0, cd& x1, cd& x2, cd& x3) {  // e = 0
  const cd a0 = cadd(x0, x2), a1 = csub(x0, x2), a2 = cadd(x1, x3), d = csub(x1, x3);
  const cd a3 = {-d.y, d.x};
  x0 = cadd(a0, a2);
  x1 = cadd(a1, a3);
  x2 = csub(a0, a2);
  x3 = csub(a1, a3);
}
SF_HD void r4_dit(cd& y0, cd& y1, cd& y2, cd& y3, int e, const cd* T) {
  if (e >= 0) {  // e < 0: no twiddles (r4_dit0)
    y1 = cmulc(y1, T[e]);
    y2 = cmulc(y2, T[2 * e]);
    y3 = cmulc(y3, T[3 * e]);
  }
  const cd b0 = cadd(y0, y2), b1 = csub(y0, y2), b2 = cadd(y1, y3), d = csub(y1, y3);
  const cd b3 = {d.y, -d.x};  // -i (y1 - y3)
  y0 = cadd(b0, b2);
  y1 = cadd(b1, b3);
  y2 = csub(b0, b2);
  y3 = csub(b1, b3);
}

// One radix-4 DIF butterfly of stage s (span L = M / 4^s) for thread t < 256; T[e] = e^{2 pi i e / M}.
SF_HD void dif_stage(cd* a, int s, int t, const cd* T) {
  const int lq = 8 - 2 * s;  // log2(L / 4)
  const int q = 1 << lq, j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j;
  r4_dif(a[base], a[base + q], a[base + 2 * q], a[base + 3 * q], j << (2 * s), T);
}
// The inverse butterfly of stage s.
SF_HD void dit_stage(cd* a, int s, int t, const cd* T) {
  const int lq = 8 - 2 * s;
  const int q = 1 << lq, j = t & (q - 1), base = ((t >> lq) << (lq + 2)) + j;
  r4_dit(a[base], a[base + q], a[base + 2 * q], a[base + 3 * q], j << (2 * s), T);
}

// ---- one transform per wave (64 lanes x 16 points): the same 5 stages grouped as passes (0,1),
// (2,3), (4) in registers, two wave-private LDS exchanges.  Lane t's registers x[4 k1 + k2]:
//   pass 01: point t + 64 k2 + 256 k1   (stage 0 over k1 at j = t + 64 k2, stage 1 over k2 at j = t)
//   pass 23: point 64 b + j + 16 k1 + 4 k2, t = 4 b + j   (stage 2 over k1 at j + 4 k2, stage 3 over k2 at j)
//   pass 4 : point 4 (t + 64 k1) + k2   (stage 4 over k2, no twiddles)
// The exchange buffer is padded by one complex per 16 (pad(p) = p + p/16, 1088 entries): each of the
// three access patterns then covers 16 distinct 16-byte slots per 16 lanes (no bank conflicts).
constexpr int SF_PADDED = SF_M + SF_M / 16;
SF_HD int pad(int p) { return p + (p >> 4); }
SF_HD int pt01(int t, int r) { return t + 64 * (r & 3) + 256 * (r >> 2); }
SF_HD int pt23(int t, int r) { return 64 * (t >> 2) + (t & 3) + 16 * (r >> 2) + 4 * (r & 3); }
SF_HD int pt4(int t, int r) { return 4 * (t + 64 * (r >> 2)) + (r & 3); }
// Spectra live in global memory in DIF position order (a one-wave transform stores them through its
// exchange buffer, contiguously); storing them in the pass-4 register order instead made the 256-thread
// inverse's loads gathers (measured slower).

SF_HD void dif_pass01(cd (&x)[16], int t, const cd* T) {
  for (int k2 = 0; k2 < 4; k2++) r4_dif(x[k2], x[4 + k2], x[8 + k2], x[12 + k2], t + 64 * k2, T);
  for (int k1 = 0; k1 < 4; k1++) r4_dif(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3], 4 * t, T);
}
SF_HD void dif_pass23(cd (&x)[16], int t, const cd* T) {
  const int j = t & 3;
  for (int k2 = 0; k2 < 4; k2++) r4_dif(x[k2], x[4 + k2], x[8 + k2], x[12 + k2], 16 * (j + 4 * k2), T);
  for (int k1 = 0; k1 < 4; k1++) r4_dif(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3], 64 * j, T);
}
SF_HD void dif_pass4(cd (&x)[16], const cd* T) {
  for (int k1 = 0; k1 < 4; k1++) r4_dif0(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3]);
}
SF_HD void dit_pass4(cd (&x)[16], const cd* T) {
  for (int k1 = 0; k1 < 4; k1++) r4_dit(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3], -1, T);
}
SF_HD void dit_pass32(cd (&x)[16], int t, const cd* T) {
  const int j = t & 3;
  for (int k1 = 0; k1 < 4; k1++) r4_dit(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3], 64 * j, T);
  for (int k2 = 0; k2 < 4; k2++) r4_dit(x[k2], x[4 + k2], x[8 + k2], x[12 + k2], 16 * (j + 4 * k2), T);
}
SF_HD void dit_pass10(cd (&x)[16], int t, const cd* T) {
  for (int k1 = 0; k1 < 4; k1++) r4_dit(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3], 4 * t, T);
  for (int k2 = 0; k2 < 4; k2++) r4_dit(x[k2], x[4 + k2], x[8 + k2], x[12 + k2], t + 64 * k2, T);
}

// ---- native 2^128 words ---------------------------------------------------------------------------
typedef unsigned __int128 w128;

// load-time key rounding: the word as a signed integer, to the nearest multiple of 2^16 (ties up), / 2^16.
// The add wraps mod 2^128, so a word within 2^15 of 2^127 rounds to -2^127: the same torus point.
SF_HD __int128 key_round16(w128 w) { return (__int128)(w + ((w128)1 << 15)) >> 16; }

// limb t of a rounded key word (rr = word / 2^16), consumed from the bottom (call t = 0, 1, .., 4 in order):
// t = 0 the balanced low 48 bits (|.| <= 2^47, exact in a double), t = 1..3 balanced 16-bit limbs, t = 4 the
// remainder (|.| <= 2^15)
SF_HD long long key_limb(__int128& rr, int t) {
  if (t == SF_LIMBS - 1) return (long long)rr;
  const int bits = t == 0 ? SF_LOW_BITS : SF_LIMB_BITS;
  const __int128 half = (__int128)1 << (bits - 1), mask = ((__int128)1 << bits) - 1;
  const __int128 l = ((rr + half) & mask) - half;
  rr = (rr - l) >> bits;
  return (long long)l;
}

// tfhe-rs SignedDecomposer on a 128-bit word, 72 bits as 3 digits of 24 (gadget 2^(128 - 24 (l + 1)),
// d[0] most significant): closest representable, then balanced digits with the tie carry rule
SF_HD void digits72(w128 y, int (&d)[3]) {
  const w128 state = ((y >> 55) + 1) >> 1;
  unsigned long long lo = (unsigned long long)state, hi = (unsigned long long)(state >> 64) & 0xFFu;
  for (int l = 2; l >= 0; l--) {
    const unsigned long long res = lo & 0xFFFFFFull;
    lo = (lo >> 24) | (hi << 40);
    hi >>= 24;
    const unsigned long long carry = ((((res - 1) | lo) & res) >> 23) & 1;
    lo += carry;  // lo < 2^48 after the first shift: no carry into hi
    d[l] = (int)((long long)res - (long long)(carry << 24));
  }
}

// one Horner step over the exact limbs (top limb first): h = sum_(t >= 1) c_t 2^(16 (t - 1))
SF_HD w128 horner16(w128 h, double c_rounded) { return (h << 16) + (w128)(__int128)(long long)c_rounded; }

// an integer-valued double (|v| < 2^127) as a word mod 2^128: the low limb's products exceed 2^63
SF_HD w128 f64_int_to_w128(double v) {
  if (v < 0x1p62 && v > -0x1p62) return (w128)(__int128)(long long)v;
  const unsigned long long bits = __builtin_bit_cast(unsigned long long, v);
  const int e = (int)((bits >> 52) & 0x7FF) - 1075;  // >= 10 here
  const w128 m = (w128)((bits & 0xFFFFFFFFFFFFFull) | 0x10000000000000ull) << e;
  return (bits >> 63) ? (w128)0 - m : m;
}
// the last step: h = h 2^48 + c_0 (the low limb); acc += h << 16
SF_HD w128 horner_low(w128 h, double c_rounded) { return (h << SF_LOW_BITS) + f64_int_to_w128(c_rounded); }

}  // namespace snsf
}  // namespace tfhe
