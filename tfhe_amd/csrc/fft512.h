// fft512.h — the 512-point complex DFT building blocks of the FFT64 engine (gfx950), shared by the
// N = 1024 kernels (pbs_fft.hip: one wave per polynomial) and the N = 2048 kernels (pbs_fft2k.hip: two
// waves per polynomial, each running one 512-point half).  One fixed f64 operation sequence, restated
// in oracle/fft_oracle.c; contraction stays off in every file that includes this header.
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include "gl64.h"
#include "ntt1024.h"

namespace tfhe {
namespace fftk {

constexpr int M = 512;
constexpr int S1 = 72, S2 = 65;   // transpose row strides (complex): T1 (passes A|B), T2 (passes B|C)
constexpr int T_C64 = 576;        // per-wave transpose scratch (9,216 B; also holds 1024 u64)
constexpr int TW_TWIST = 0, TW_A = 512, TW_B = 1024, TW_I = 1536, TW_C64 = 2048;  // table offsets (complex)
constexpr double SQRT1_2 = 0.70710678118654752440;

// Order between a wave's own LDS writes and reads of its private scratch.  DS instructions of one
// wavefront execute in issue order, so a compiler-only fence would do (FFT_LDS_WAIT=0); measured on
// MI355X it is 4 % SLOWER (31.97 vs 30.71 ms per 4096-PBS blind rotation: hipcc then interleaves the
// transpose reads with the butterflies and stalls on them one by one), so the full lgkmcnt(0) drain
// stays the default.
#ifndef FFT_LDS_WAIT
#define FFT_LDS_WAIT 1
#endif
__device__ __forceinline__ void lds_order() {
#if FFT_LDS_WAIT
  wave_lds_sync();
#else
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#endif
}

// z * w (INV: z * conj(w)), the oracle's cmul(z, w.re, +-w.im)
template <bool INV>
__device__ __forceinline__ void cmul(double& re, double& im, double2 w) {
  const double p = re, q = im;
  if (!INV) {
    re = __builtin_fma(p, w.x, -(q * w.y));
    im = __builtin_fma(p, w.y, q * w.x);
  } else {
    re = __builtin_fma(p, w.x, q * w.y);
    im = __builtin_fma(p, -w.y, q * w.x);
  }
}

// t * e^{+-i pi j / 4} (oracle w8)
template <bool INV, int J>
__device__ __forceinline__ void w8(double& re, double& im) {
  const double p = re, q = im;
  if (J == 1) {
    if (!INV) { re = (p - q) * SQRT1_2; im = (p + q) * SQRT1_2; }
    else { re = (p + q) * SQRT1_2; im = (q - p) * SQRT1_2; }
  } else if (J == 2) {
    if (!INV) { re = -q; im = p; }
    else { re = q; im = -p; }
  } else {
    if (!INV) { re = -((p + q) * SQRT1_2); im = (p - q) * SQRT1_2; }
    else { re = (q - p) * SQRT1_2; im = -((p + q) * SQRT1_2); }
  }
}

// FFT_DFT8_FMA 1 (default since round 5): the odd half of the 8-point DFT with the sqrt(1/2) factor folded into the
// last stage's fmas.  With y5 = s u5, y7 = s u7 (u the unscaled w8 forms, s = sqrt(1/2)), z5 = s (u5 + u7) and
// z7 = s (u5 - u7), so x1 / x5 = z4 +- s (u5 + u7) and x3 / x7 = z6 +- (+-i) s (u5 - u7) are 8 fmas: 52 f64 instructions
// per DFT8 instead of 56 (4 multiplies fewer), -48 per wave and CMUX in the P-GATE pair kernel.  A different rounding
// sequence, restated in oracle/fft_oracle.c:dft8 (and judged by the exact arbiter); 0 = the round-1..4 form.
#ifndef FFT_DFT8_FMA
#define FFT_DFT8_FMA 1
#endif
// 8-point DFT in registers, natural order in and out (radix-2 DIF, bit-reversal by renaming)
template <bool INV>
__device__ __forceinline__ void dft8(double (&xr)[8], double (&xi)[8]) {
#if FFT_DFT8_FMA
  double yr[4], yi[4];  // stage 1, even half: y_j = x_j + x_(j+4)
#pragma unroll
  for (int j = 0; j < 4; j++) {
    yr[j] = xr[j] + xr[j + 4];
    yi[j] = xi[j] + xi[j + 4];
  }
  // odd half: t_j = x_j - x_(j+4); y4 = t0, y6 = (+-i) t2, y5 / y7 = s u5 / s u7 (u5, u7 kept unscaled)
  const double t0r = xr[0] - xr[4], t0i = xi[0] - xi[4];
  const double t1r = xr[1] - xr[5], t1i = xi[1] - xi[5];
  const double t2r = xr[2] - xr[6], t2i = xi[2] - xi[6];
  const double t3r = xr[3] - xr[7], t3i = xi[3] - xi[7];
  double ar, ai, cr, ci;  // u5 = (ar, ai), u7 = (cr, ci)
  if (!INV) {
    ar = t1r - t1i; ai = t1r + t1i;        // w8^1 / s
    cr = -(t3r + t3i); ci = t3r - t3i;     // w8^3 / s
  } else {
    ar = t1r + t1i; ai = t1i - t1r;
    cr = t3i - t3r; ci = -(t3r + t3i);
  }
  const double z5r = ar + cr, z5i = ai + ci;  // z5 / s
  const double z7r = ar - cr, z7i = ai - ci;  // z7 / s (before its rotation by +-i)
  // z4 = y4 + y6, z6 = y4 - y6 with y6 = (+-i) t2
  const double z4r = INV ? t0r + t2i : t0r - t2i, z4i = INV ? t0i - t2r : t0i + t2r;
  const double z6r = INV ? t0r - t2i : t0r + t2i, z6i = INV ? t0i + t2r : t0i - t2r;
  // even half: stages 2 and 3 as before
  const double e0r = yr[0] + yr[2], e0i = yi[0] + yi[2];
  const double e2r = yr[0] - yr[2], e2i = yi[0] - yi[2];
  const double e1r = yr[1] + yr[3], e1i = yi[1] + yi[3];
  double e3r = yr[1] - yr[3], e3i = yi[1] - yi[3];
  w8<INV, 2>(e3r, e3i);
  xr[0] = e0r + e1r; xi[0] = e0i + e1i;
  xr[4] = e0r - e1r; xi[4] = e0i - e1i;
  xr[2] = e2r + e3r; xi[2] = e2i + e3i;
  xr[6] = e2r - e3r; xi[6] = e2i - e3i;
  // odd half, stage 3 with s folded: x1 = z4 + s z5', x5 = z4 - s z5', x3 = z6 + r(s z7'), x7 = z6 - r(s z7'),
  // r = multiplication by +i (forward) / -i (inverse)
  xr[1] = __builtin_fma(SQRT1_2, z5r, z4r); xi[1] = __builtin_fma(SQRT1_2, z5i, z4i);
  xr[5] = __builtin_fma(-SQRT1_2, z5r, z4r); xi[5] = __builtin_fma(-SQRT1_2, z5i, z4i);
  if (!INV) {  // r z = (-z.im, z.re)
    xr[3] = __builtin_fma(-SQRT1_2, z7i, z6r); xi[3] = __builtin_fma(SQRT1_2, z7r, z6i);
    xr[7] = __builtin_fma(SQRT1_2, z7i, z6r); xi[7] = __builtin_fma(-SQRT1_2, z7r, z6i);
  } else {     // r z = (z.im, -z.re)
    xr[3] = __builtin_fma(SQRT1_2, z7i, z6r); xi[3] = __builtin_fma(-SQRT1_2, z7r, z6i);
    xr[7] = __builtin_fma(-SQRT1_2, z7i, z6r); xi[7] = __builtin_fma(SQRT1_2, z7r, z6i);
  }
#else
  double yr[8], yi[8];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    yr[j] = xr[j] + xr[j + 4];
    yi[j] = xi[j] + xi[j + 4];
    yr[j + 4] = xr[j] - xr[j + 4];
    yi[j + 4] = xi[j] - xi[j + 4];
  }
  w8<INV, 1>(yr[5], yi[5]);
  w8<INV, 2>(yr[6], yi[6]);
  w8<INV, 3>(yr[7], yi[7]);
  double zr[8], zi[8];
#pragma unroll
  for (int h = 0; h < 8; h += 4)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      zr[h + j] = yr[h + j] + yr[h + j + 2];
      zi[h + j] = yi[h + j] + yi[h + j + 2];
      zr[h + j + 2] = yr[h + j] - yr[h + j + 2];
      zi[h + j + 2] = yi[h + j] - yi[h + j + 2];
    }
  w8<INV, 2>(zr[3], zi[3]);
  w8<INV, 2>(zr[7], zi[7]);
  // u[g] = z[g] + z[g+1], u[g+1] = z[g] - z[g+1];  X[k] = u[brv3(k)]
  xr[0] = zr[0] + zr[1]; xi[0] = zi[0] + zi[1];
  xr[4] = zr[0] - zr[1]; xi[4] = zi[0] - zi[1];
  xr[2] = zr[2] + zr[3]; xi[2] = zi[2] + zi[3];
  xr[6] = zr[2] - zr[3]; xi[6] = zi[2] - zi[3];
  xr[1] = zr[4] + zr[5]; xi[1] = zi[4] + zi[5];
  xr[5] = zr[4] - zr[5]; xi[5] = zi[4] - zi[5];
  xr[3] = zr[6] + zr[7]; xi[3] = zi[6] + zi[7];
  xr[7] = zr[6] - zr[7]; xi[7] = zi[6] - zi[7];
#endif
}

// Transpose 1 in registers (FFT_T1_PERM=1; measured and NOT the default: the P-GATE batch kernel 27.40 ->
// 28.80 ms, the N = 2048 kernel 52.18 -> 52.00 ms — the 96 cross-lane moves and selects per transpose cost
// more VALU time than the 16 LDS operations and two waits they replace): slot bits (0, 1, 2) <-> lane bits (3, 4, 5), the
// permutation the T1 round trip through LDS performs in both directions (it is an involution).  Lane bit
// 5 <-> slot bit 2 is v_permlane32_swap, lane bit 4 <-> slot bit 1 v_permlane16_swap (gfx950: each swaps
// one operand's upper 32-lane half / odd 16-lane rows with the other's lower half / even rows, probed in
// tools/microbench/permlane_probe.hip), lane bit 3 <-> slot bit 0 a DPP row_ror:8 exchange with selects.
// Pure data movement: the transform's arithmetic and results are unchanged.
#ifndef FFT_T1_PERM
#define FFT_T1_PERM 0
#endif
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void swap32_d(double& a, double& b) {
  const u32x2v x = __builtin_bit_cast(u32x2v, a), y = __builtin_bit_cast(u32x2v, b);
  const auto lo = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
  a = __builtin_bit_cast(double, (u32x2v){lo[0], hi[0]});
  b = __builtin_bit_cast(double, (u32x2v){lo[1], hi[1]});
}
__device__ __forceinline__ void swap16_d(double& a, double& b) {
  const u32x2v x = __builtin_bit_cast(u32x2v, a), y = __builtin_bit_cast(u32x2v, b);
  const auto lo = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
  a = __builtin_bit_cast(double, (u32x2v){lo[0], hi[0]});
  b = __builtin_bit_cast(double, (u32x2v){lo[1], hi[1]});
}
// 2 x 2 transpose of (a, b) with lane bit 3: new_a[L] = b3 ? b[L ^ 8] : a[L], new_b[L] = b3 ? b[L] : a[L ^ 8]
__device__ __forceinline__ void swap8_u32(unsigned& a, unsigned& b, bool b3) {
  const unsigned t = b3 ? a : b;
  const unsigned u = (unsigned)__builtin_amdgcn_update_dpp(0, (int)t, 0x128, 0xF, 0xF, false);  // row_ror:8
  a = b3 ? u : a;
  b = b3 ? b : u;
}
__device__ __forceinline__ void swap8_d(double& a, double& b, bool b3) {
  const u32x2v x = __builtin_bit_cast(u32x2v, a), y = __builtin_bit_cast(u32x2v, b);
  unsigned xl = x.x, xh = x.y, yl = y.x, yh = y.y;
  swap8_u32(xl, yl, b3);
  swap8_u32(xh, yh, b3);
  a = __builtin_bit_cast(double, (u32x2v){xl, xh});
  b = __builtin_bit_cast(double, (u32x2v){yl, yh});
}
__device__ __forceinline__ void t1_regs(double (&xr)[8], double (&xi)[8], int lane) {
#pragma unroll
  for (int e = 0; e < 4; e++) {
    swap32_d(xr[e], xr[e + 4]);
    swap32_d(xi[e], xi[e + 4]);
  }
#pragma unroll
  for (int e = 0; e < 8; e++)
    if ((e & 2) == 0) {
      swap16_d(xr[e], xr[e + 2]);
      swap16_d(xi[e], xi[e + 2]);
    }
  const bool b3 = (lane >> 3) & 1;
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    swap8_d(xr[e], xr[e + 1], b3);
    swap8_d(xi[e], xi[e + 1], b3);
  }
}

template <bool INV>
__device__ __forceinline__ void twist_slots(double (&xr)[8], double (&xi)[8]);

// FFT_TDFT8 1 (default since round 5): the N = 1024 forward's slot twist and pass A's DFT8 as ONE twisted DFT8.
// Slot e carries zeta^(64 e) = e^(i pi e / 16) before the DFT8 over e, so pass A evaluates x(X) = sum_e x_e X^e at the
// 8 roots of X^8 = i, X_k = e^(i pi (1 + 4 k) / 16) -- a negacyclic-style split:
//   stage 1  X^8 - i = (X^4 - w)(X^4 + w), w = e^(i pi/4):       u_e = x_e + w x_(e+4),  v_e = x_e - w x_(e+4)
//   stage 2  u: (X^2 -+ e^(i pi/8)),  v: (X^2 -+ e^(i 5pi/8))    pairs (e, e + 2)
//   stage 3  roots +-e^(i pi/16), +-e^(i 9pi/16), +-e^(i 5pi/16), +-e^(i 13pi/16) -> X_0 X_4, X_2 X_6, X_1 X_5, X_3 X_7
// Each of the 12 butterflies a +- e^(i th) b takes b through a tangent (or cotangent) form, u = (b.re - t b.im,
// b.im + t b.re), and folds cos th (or sin th) into the two output fmas: 6 f64 instructions, 72 for the whole step
// against 28 (7 slot cmuls) + 52 (DFT8) = 80.  Measured SLOWER on MI355X (round 5, same box, three rounds: 24.76 vs 24.62
// ms per 4096, profiles/r05c_ab_tdft8.txt: the three dependent fma stages and 3 spilled VGPRs cost more than the 24 f64
// instructions saved), so 0 -- twist, then DFT8 -- is the default and the one oracle/fft_oracle.c restates (its tdft8_fwd
// is kept for the A/B build only).
#ifndef FFT_TDFT8
#define FFT_TDFT8 0
#endif
namespace tdft {
constexpr double T8 = 0.41421356237309504880, C8 = 0.92387953251128675613;     // tan, cos (pi / 8)
constexpr double T16 = 0.19891236737965800691, C16 = 0.98078528040323044913;   // tan, cos (pi / 16)
constexpr double T316 = 0.66817863791929891999, C316 = 0.83146961230254523708; // tan, cos (3 pi / 16)
}  // namespace tdft
// a + e^(i th) b -> a, a - e^(i th) b -> b, with e^(i th) b = sc (u), u = (b.re - t b.im, b.im + t b.re) (COT = false:
// t = tan th, sc = cos th) or u = (t b.re - b.im, b.re + t b.im) (COT: t = cot th, sc = sin th)
template <bool COT>
__device__ __forceinline__ void tbfly(double& ar, double& ai, double& br, double& bi, double t, double sc) {
  double ur, ui;
  if (!COT) {
    ur = __builtin_fma(-t, bi, br);
    ui = __builtin_fma(t, br, bi);
  } else {
    ur = __builtin_fma(t, br, -bi);
    ui = __builtin_fma(t, bi, br);
  }
  const double pr = ar, pi = ai;
  ar = __builtin_fma(sc, ur, pr);
  ai = __builtin_fma(sc, ui, pi);
  br = __builtin_fma(-sc, ur, pr);
  bi = __builtin_fma(-sc, ui, pi);
}
// the slot twist + pass A's DFT8 of the N = 1024 forward transform (natural order in and out)
__device__ __forceinline__ void twist_dft8_fwd(double (&xr)[8], double (&xi)[8]) {
#if FFT_TDFT8
  using namespace tdft;
#pragma unroll
  for (int e = 0; e < 4; e++) {  // stage 1, w = e^(i pi/4): u = (b.re - b.im, b.im + b.re), sc = sqrt(1/2)
    const double ur = xr[e + 4] - xi[e + 4], ui = xi[e + 4] + xr[e + 4];
    const double pr = xr[e], pi = xi[e];
    xr[e] = __builtin_fma(SQRT1_2, ur, pr);
    xi[e] = __builtin_fma(SQRT1_2, ui, pi);
    xr[e + 4] = __builtin_fma(-SQRT1_2, ur, pr);
    xi[e + 4] = __builtin_fma(-SQRT1_2, ui, pi);
  }
  // stage 2: u pairs at th = pi/8 (tan), v pairs at th = 5 pi/8 (cot = -tan(pi/8), sin = cos(pi/8))
  tbfly<false>(xr[0], xi[0], xr[2], xi[2], T8, C8);
  tbfly<false>(xr[1], xi[1], xr[3], xi[3], T8, C8);
  tbfly<true>(xr[4], xi[4], xr[6], xi[6], -T8, C8);
  tbfly<true>(xr[5], xi[5], xr[7], xi[7], -T8, C8);
  // stage 3: (0, 1) pi/16 -> X0, X4; (2, 3) 9 pi/16 (cot = -tan(pi/16), sin = cos(pi/16)) -> X2, X6;
  //          (4, 5) 5 pi/16 (cot = tan(3 pi/16), sin = cos(3 pi/16)) -> X1, X5; (6, 7) 13 pi/16 (tan = -tan(3 pi/16),
  //          cos = -cos(3 pi/16)) -> X3, X7
  tbfly<false>(xr[0], xi[0], xr[1], xi[1], T16, C16);
  tbfly<true>(xr[2], xi[2], xr[3], xi[3], -T16, C16);
  tbfly<true>(xr[4], xi[4], xr[5], xi[5], T316, C316);
  tbfly<false>(xr[6], xi[6], xr[7], xi[7], -T316, -C316);
  // positions 0..7 now hold X0 X4 X2 X6 X1 X5 X3 X7: rename to natural order
  const double r1 = xr[4], i1 = xi[4], r2 = xr[2], i2 = xi[2], r3 = xr[6], i3 = xi[6], r4 = xr[1], i4 = xi[1];
  const double r6 = xr[3], i6 = xi[3];
  xr[1] = r1; xi[1] = i1;
  xr[2] = r2; xi[2] = i2;
  xr[3] = r3; xi[3] = i3;
  xr[4] = r4; xi[4] = i4;
  xr[6] = r6; xi[6] = i6;
  // 5 (X5) and 7 (X7) are in place, 0 (X0) too
#else
  twist_slots<false>(xr, xi);
  dft8<false>(xr, xi);
#endif
}

// per-lane transpose bases: b1 = T1 read / inverse write, b2 = T2 read / inverse write
struct TBase {
  int b1, b2;
  __device__ __forceinline__ explicit TBase(int lane)
      : b1((lane >> 3) * S1 + (lane & 7)), b2((lane & 7) * S2 + 8 * (lane >> 3)) {}
};

// forward 512-point DFT: natural order in (lane L, slot e <-> L + 64 e), device order out.
// TW0: pass A multiplies slot 0 too (the N = 1024 tables fold the lane part of the twist into pass A)
// (twA / twB: the pass A / pass B tables, 512 complex each, [64 e + L])
// TWIN: the input is not yet twisted and pass A's DFT8 is the twisted one (twist_dft8_fwd; N = 1024 only)
template <bool TW0 = false, bool TWIN = false>
__device__ __forceinline__ void dft512_fwd_t(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const double2* twA, const double2* twB) {
  if constexpr (TWIN) twist_dft8_fwd(xr, xi);
  else dft8<false>(xr, xi);
#pragma unroll
  for (int e = TW0 ? 0 : 1; e < 8; e++) cmul<false>(xr[e], xi[e], twA[64 * e + lane]);
#if FFT_T1_PERM
  t1_regs(xr, xi, lane);
#else
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S1 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b1 + 8 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
#endif
  dft8<false>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<false>(xr[e], xi[e], twB[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S2 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b2 + e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
}

// the same with pass A's twiddles (this lane's 8, slot 0 included: the merged twist) held in registers
template <bool TWIN = false>
__device__ __forceinline__ void dft512_fwd_ra(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                              const double2 (&wa)[8], const double2* twB) {
  if constexpr (TWIN) twist_dft8_fwd(xr, xi);
  else dft8<false>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<false>(xr[e], xi[e], wa[e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S1 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b1 + 8 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<false>(xr[e], xi[e], twB[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S2 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b2 + e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
}

// pass A and pass B twiddles both in registers (wb[0] unused)
template <bool TWIN = false>
__device__ __forceinline__ void dft512_fwd_rab(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                               const double2 (&wa)[8], const double2 (&wb)[8]) {
  if constexpr (TWIN) twist_dft8_fwd(xr, xi);
  else dft8<false>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<false>(xr[e], xi[e], wa[e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S1 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b1 + 8 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<false>(xr[e], xi[e], wb[e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S2 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b2 + e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
}

// inverse with pass C''s twiddles (= pass B's table, conjugated by cmul<true>) in registers, pass B' from twI
__device__ __forceinline__ void dft512_inv_rb(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                              const double2 (&wb)[8], const double2* twI) {
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<true>(xr[e], xi[e], wb[e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b2 + e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S2 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<true>(xr[e], xi[e], twI[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b1 + 8 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S1 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
}

// Round 6 (three waves per SIMD): every twiddle read from LDS, pass B's from the COMPACT table.  TW_B[e][L] =
// w512^(8 (L & 7) e) depends on L & 7 only, so the 64 distinct values sit in 1 KB as [e][L & 7]: a lane reads
// twBc[8 e] from its base twBc + (L & 7) (8 distinct addresses per instruction, broadcast, conflict-free), the same
// bits as the 8 KB table.  twAl = TW_A + L (pass A, slot 0 included: the merged twist), twIl = TW_I + L.
template <bool TWIN = false, int BSTR = 8>
__device__ __forceinline__ void dft512_fwd_c(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const double2* twAl, const double2* twBc) {
  if constexpr (TWIN) twist_dft8_fwd(xr, xi);
  else dft8<false>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<false>(xr[e], xi[e], twAl[64 * e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S1 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b1 + 8 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<false>(xr[e], xi[e], twBc[BSTR * e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[lane + S2 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[tb.b2 + e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<false>(xr, xi);
}

// the matching inverse: pass C' conjugates the compact pass B table, pass B' reads twIl[64 e]
// (BSTR: the pass B table's slot stride, 8 for the compact table, 64 for the full one)
template <int BSTR = 8>
__device__ __forceinline__ void dft512_inv_c(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const double2* twBc, const double2* twIl) {
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<true>(xr[e], xi[e], twBc[BSTR * e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b2 + e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S2 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<true>(xr[e], xi[e], twIl[64 * e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b1 + 8 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S1 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
}

template <bool TW0 = false, bool TWIN = false>
__device__ __forceinline__ void dft512_fwd(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                           const double2* tw) {
  dft512_fwd_t<TW0, TWIN>(xr, xi, T, lane, tb, tw + TW_A, tw + TW_B);
}

// inverse (no 1/M): device order in, natural order out — the forward's passes reversed
// (twB / twI: the pass C' / pass B' tables)
__device__ __forceinline__ void dft512_inv_t(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const double2* twB, const double2* twI) {
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<true>(xr[e], xi[e], twB[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b2 + e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S2 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<true>(xr[e], xi[e], twI[64 * e + lane]);
#if FFT_T1_PERM
  t1_regs(xr, xi, lane);
#else
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b1 + 8 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S1 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
#endif
  dft8<true>(xr, xi);
}

__device__ __forceinline__ void dft512_inv(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                           const double2* tw) {
  dft512_inv_t(xr, xi, T, lane, tb, tw + TW_B, tw + TW_I);
}

// this lane's inverse twiddles (pass C' slots 1..7, pass B' slots 0..7) in registers, for back-to-back inverses
struct InvTw {
  double2 b[8], i[8];
  __device__ __forceinline__ void load(const double2* tw, int lane) {
#pragma unroll
    for (int e = 1; e < 8; e++) b[e] = tw[TW_B + 64 * e + lane];
#pragma unroll
    for (int e = 0; e < 8; e++) i[e] = tw[TW_I + 64 * e + lane];
  }
};
__device__ __forceinline__ void dft512_inv_r(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const InvTw& w) {
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 1; e < 8; e++) cmul<true>(xr[e], xi[e], w.b[e]);
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b2 + e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S2 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
  dft8<true>(xr, xi);
#pragma unroll
  for (int e = 0; e < 8; e++) cmul<true>(xr[e], xi[e], w.i[e]);
#if FFT_T1_PERM
  t1_regs(xr, xi, lane);
#else
#pragma unroll
  for (int e = 0; e < 8; e++) T[tb.b1 + 8 * e] = make_double2(xr[e], xi[e]);
  lds_order();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = T[lane + S1 * e];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  lds_order();
#endif
  dft8<true>(xr, xi);
}

// ---------------------------------------------------------------------------------------------
// N = 1024 (P-GATE) merged twist.  z_j = a_j zeta^j with j = L + 64 e splits as zeta^L * zeta^(64 e): the
// slot part c_e = zeta^(64 e) is a per-slot constant (an SGPR operand, no table read) applied before
// pass A, and the lane part zeta^L commutes with pass A's 8-point DFT over the slots, so it is folded
// into pass A's table: TW_A[e][L] = w^(L e) zeta^L = zeta^(L (1 + 4 e)).  The inverse does the mirror
// image: zeta^(n0 + 8 n1) rides in pass B''s table (TW_I[e][L] = zeta^((n0 + 8 e)(4 k0 + 1)), L = n0 + 8
// k0), conj(c_e) is applied after pass A'.  Saves 15 of the 54 LDS reads of a forward digit transform
// and 8 of an inverse (oracle/fft_oracle.c: or_fft_fwd / or_fft_inv at N = 1024 restate the order).
// N = 2048 (pbs_fft2k.hip) does the same per parity h: zeta_4096^(2 m + h) = zeta^(2 L + h) zeta^(128 e), the
// slot constants are the same values (128 e / 4096 = 64 e / 2048), the tables A'_h, I'_h per parity.
// The constants come from the table generator's own series, evaluated at compile time (IEEE double,
// no contraction in constant evaluation) so they equal the host tables bit for bit.
namespace ctw {
constexpr double sin_s(double x) {
  double x2 = x * x, term = x, sum = 0.0;
  for (int i = 1; i <= 21; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
constexpr double cos_s(double x) {
  double x2 = x * x, term = 1.0, sum = 0.0;
  for (int i = 0; i <= 20; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
struct c64 {
  double x, y;
};
// cos / sin (2 pi t / 2048) for t = 64 e, e = 0..7 (t <= 448 < M / 4: octant and quarter cases only)
constexpr c64 slot(int e) {
  const unsigned t = 64u * (unsigned)e, m = 2048u;
  if (8 * t > m) {
    const double x = (double)(m / 4 - t) * (6.28318530717958647692 / (double)m);
    return c64{sin_s(x), cos_s(x)};
  }
  const double x = (double)t * (6.28318530717958647692 / (double)m);
  return c64{cos_s(x), sin_s(x)};
}
constexpr c64 SLOT[8] = {slot(0), slot(1), slot(2), slot(3), slot(4), slot(5), slot(6), slot(7)};
}  // namespace ctw

// z * c_e (forward) / z * conj(c_e) (inverse) for slot e > 0, c_e a compile-time constant; the
// operation order of cmul
template <bool INV>
__device__ __forceinline__ void twist_slots(double (&xr)[8], double (&xi)[8]) {
#pragma unroll
  for (int e = 1; e < 8; e++) {
    const double wr = ctw::SLOT[e].x, wi = ctw::SLOT[e].y;
    const double p = xr[e], q = xi[e];
    if (!INV) {
      xr[e] = __builtin_fma(p, wr, -(q * wi));
      xi[e] = __builtin_fma(p, wi, q * wr);
    } else {
      xr[e] = __builtin_fma(p, wr, q * wi);
      xi[e] = __builtin_fma(p, -wi, q * wr);
    }
  }
}

// (double)(int64)x, correctly rounded: exact hi * 2^32 plus exact lo, one rounding
__device__ __forceinline__ double i64_to_f64(u64 x) {
  return __builtin_fma((double)(int)(x >> 32), 0x1p32, (double)(u32)x);
}

// rint(x) mod 2^64 (every step after the rint is exact)
// h = floor(t / 2^32) is an integer with |h| < 2^51, so h + 1.5 * 2^52 is exact and its low
// mantissa word is h mod 2^32
__device__ __forceinline__ u64 f64_to_torus(double x) {
  const double t = __builtin_rint(x);
  const double h = __builtin_floor(t * 0x1p-32);
  const double l = __builtin_fma(-h, 0x1p32, t);
  const u32 hm = (u32)__double_as_longlong(h + 0x1.8p52);
  return ((u64)hm << 32) | (u64)(u32)l;
}

// FFT_TORUS_NORINT 1 (default since round 5): the accumulator update without the rint and without building the u64 from
// two halves.  h = floor(x 2^-32), l = fma(-h, 2^32, x) (exact whenever |x| >= 2^32 or h = 0; for -2^32 < x < 0 it is
// x + 2^32 rounded once), and the two words come straight out of doubles' bit patterns:
//   l + 2^52                     bits = 0x43300000_00000000 + rint(l)        (rint(l) may be 2^32: the carry is kept)
//   h + (1.5 2^52 - 0x43300000)  low word = (h - 0x43300000) mod 2^32       (|h| < 2^51 - 2^32)
// acc += (hb << 32) + lb (two v_lshl_add_u64), the 0x43300000 offsets cancel mod 2^64.  The value is h 2^32 + rint(l):
// rint(x) mod 2^64 exactly, except that a tiny negative x (|x| < 2^32) rounds twice (x + 2^32, then to an integer) --
// oracle/fft_oracle.c:or_f64_to_torus_dev restates the same operations.  7 VALU per coefficient instead of 8 (P-GATE)
// and 10 instead of 12 (P-FHEVM, below).
#ifndef FFT_TORUS_NORINT
#define FFT_TORUS_NORINT 1
#endif
// acc + (low word of d's bit pattern) << 32: a 32-bit add on acc's high word (no carry can come from below; hipcc
// otherwise moves the word into the high half of a fresh pair for a 64-bit add -- v_lshl_add_u64 shifts by 0..4 only)
__device__ __forceinline__ u64 add_hi_word(u64 acc, double d) {
  const u32x2v a = __builtin_bit_cast(u32x2v, acc);
  const u32x2v w = __builtin_bit_cast(u32x2v, d);
  return __builtin_bit_cast(u64, (u32x2v){a.x, a.y + w.x});
}
// Used only by FFT_Y32 = 0 A/B builds of the N = 1024 kernels (the default FFT_Y32 = 1 updates through torus_acc_add_y
// below).  The oracle restates the rint-free update (or_f64_to_torus_dev) at both N, so this function takes the rint-free
// form too (FFT_TORUS_NORINT_1K 1, round 6): the rint form differs from it for tiny negative x and would make
// such a build fail bit-exact parity.  (Round 5 measured the two forms within 0.3 % of each other on the pair kernel,
// profiles/r05f_ab_norint.txt.)
#ifndef FFT_TORUS_NORINT_1K
#define FFT_TORUS_NORINT_1K 1
#endif
__device__ __forceinline__ u64 torus_acc_add(u64 acc, double x) {
#if FFT_TORUS_NORINT && FFT_TORUS_NORINT_1K
  const double h = __builtin_floor(x * 0x1p-32);
  const double l = __builtin_fma(-h, 0x1p32, x);
  const double lb = l + 0x1p52;
  const double hb = h + (0x1.8p52 - 1127219200.0);  // 1.5 * 2^52 - 0x43300000, an exact double
  return add_hi_word(acc, hb) + (u64)__double_as_longlong(lb);
#else
  return acc + f64_to_torus(x);
#endif
}

// the same for any |x| < 2^115 (N = 2048 with 23-bit digits reaches |x| ~ 2^91, beyond the magic-number
// step above): the high word comes off a second exact floor/fma split
__device__ __forceinline__ u64 f64_to_torus_wide(double x) {
  const double t = __builtin_rint(x);
  const double h = __builtin_floor(t * 0x1p-32);
  const double l = __builtin_fma(-h, 0x1p32, t);
  const double hh = __builtin_floor(h * 0x1p-32);
  const double hm = __builtin_fma(-hh, 0x1p32, h);
  return ((u64)(u32)hm << 32) | (u64)(u32)l;
}
// torus_acc_add of x = y * 2^32 (|x| < 2^83), given y: the N = 1024 keys' spectra carry 2^-32 (bsk_to_fourier_kernel
// scales by 2^-41, FFT_Y32) and, as for torus_acc_add_wide_y below, the MAC and the inverse transform then return
// x * 2^-32 bit for bit.  h = floor(y), (y - h) + 2^20 = 2^-32 RN(l + 2^52) (low word rint(l), high word 0x41300000),
// h + 1.5 2^52 - 0x41300000 (low word h - 0x41300000 mod 2^32): the rint-free update above, bit for bit, in four f64
// operations instead of five (the oracle's or_f64_to_torus_dev)
__device__ __forceinline__ u64 torus_acc_add_y(u64 acc, double y) {
  const double h = __builtin_floor(y);
  const double lb = (y - h) + 0x1p20;
  const double hb = h + (0x1.8p52 - 1093664768.0);  // 1.5 * 2^52 - 0x41300000
  return add_hi_word(acc, hb) + (u64)__double_as_longlong(lb);
}

// torus_acc_add for |x| < 2^115 (FFT_TORUS_NORINT): h mod 2^32 off a second exact floor/fma split, then the same two
// bit-pattern words
__device__ __forceinline__ u64 torus_acc_add_wide(u64 acc, double x) {
#if FFT_TORUS_NORINT
  const double h = __builtin_floor(x * 0x1p-32);
  const double l = __builtin_fma(-h, 0x1p32, x);
  const double lb = l + 0x1p52;
  const double hh = __builtin_floor(h * 0x1p-32);
  const double hm = __builtin_fma(-hh, 0x1p32, h);    // h mod 2^32, exact, in [0, 2^32)
  const double hb = hm + (0x1.8p52 - 1127219200.0);
  return add_hi_word(acc, hb) + (u64)__double_as_longlong(lb);
#else
  return acc + f64_to_torus_wide(x);
#endif
}

// torus_acc_add_wide of x = y * 2^32, given y: the N = 2048 keys' spectra carry the factor 2^-32 (launch_bsk_to_fourier2k
// scales by 2^-42 instead of 2^-10) and every later step -- the MAC's fmas, the inverse transform's adds, multiplies and
// fmas -- rounds a power-of-two multiple of its exact value, so y is x * 2^-32 bit for bit.  Then h = floor(y) directly,
// and y - h = 2^-32 RN(x - 2^32 h) (the same scaling argument), so (y - h) + 2^20 = 2^-32 RN(l + 2^52): the same low
// word as lb above (ulp 2^-32 at 2^20), the high word 0x41300000 instead of 0x43300000 (hb's constant compensates), one
// f64 operation (the x * 2^-32) fewer per coefficient.  The oracle keeps the x form.
// The high word: h is an integer, so fract(h 2^-32) = (h mod 2^32) 2^-32 exactly (granularity 2^-32, any sign), and
// fract + 2^20 carries h mod 2^32 in its low word; the two 0x41300000 high words cost one v_add3_u32 operand.
// Six f64 operations per coefficient against eight.
__device__ __forceinline__ u64 torus_acc_add_wide_y(u64 acc, double y) {
  const double h = __builtin_floor(y);
  const double lb = (y - h) + 0x1p20;
  const double hb = __builtin_amdgcn_fract(h * 0x1p-32) + 0x1p20;
  const u32x2v a = __builtin_bit_cast(u32x2v, acc);
  const u32x2v w = __builtin_bit_cast(u32x2v, hb);
  return __builtin_bit_cast(u64, (u32x2v){a.x, a.y + w.x - 0x41300000u}) + (u64)__double_as_longlong(lb);
}

}  // namespace fftk

// cos / sin (2 pi t / m): fixed series in plain double, octant-reduced (the oracle's or_fft_twiddle)
void fft_twiddle(uint32_t t, uint32_t m, double* c, double* s);

}  // namespace tfhe
