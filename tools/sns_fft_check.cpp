// Host accuracy check of the noise-squashing f64 FFT product (tfhe_amd/csrc/sns_fft.h): 9-term sums of
// digit (|d| <= 2^23) x limb (|l| <= 2^15) negacyclic convolutions at N = 2048 through the same stage
// functions the device runs, against the exact int128 schoolbook product.  Prints the largest distance
// of an f64 output from its exact integer: the device rounds with rint(), so it must stay below 1/2.
// With a third argument 48 the limb is the low 48-bit limb (|l| <= 2^47): products up to 2^84, inexact by
// design; the tool then reports the error (it lands at weight 2^16 of the accumulator).
//   g++ -O2 -std=c++17 -ffp-contract=off -I tfhe_amd/csrc tools/sns_fft_check.cpp -o /tmp/sns_fft_check &&
//   /tmp/sns_fft_check [trials] [s|w] [16|48]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "sns_fft.h"

using namespace tfhe::snsf;
typedef __int128 i128;

static cd T[SF_M], P[SF_M];

static void tables() {
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int e = 0; e < SF_M; e++) {
    T[e] = {(double)cosl(2 * pi * e / SF_M), (double)sinl(2 * pi * e / SF_M)};
    P[e] = {(double)cosl(pi * e / SF_N), (double)sinl(pi * e / SF_N)};
  }
}

static bool g_wave = false;  // the one-wave pass form instead of the 256-thread stages

// 64 simulated lanes: registers -> padded buffer -> registers between passes
static void wave_fwd(cd* z) {
  static cd x[64][16], buf[SF_PADDED];
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = z[pt01(t, r)];
    dif_pass01(x[t], t, T);
    for (int r = 0; r < 16; r++) buf[pad(pt01(t, r))] = x[t][r];
  }
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = buf[pad(pt23(t, r))];
    dif_pass23(x[t], t, T);
    for (int r = 0; r < 16; r++) buf[pad(pt23(t, r))] = x[t][r];
  }
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = buf[pad(pt4(t, r))];
    dif_pass4(x[t], T);
    for (int r = 0; r < 16; r++) z[pt4(t, r)] = x[t][r];
  }
}
static void wave_inv(cd* z) {
  static cd x[64][16], buf[SF_PADDED];
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = z[pt4(t, r)];
    dit_pass4(x[t], T);
    for (int r = 0; r < 16; r++) buf[pad(pt4(t, r))] = x[t][r];
  }
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = buf[pad(pt23(t, r))];
    dit_pass32(x[t], t, T);
    for (int r = 0; r < 16; r++) buf[pad(pt23(t, r))] = x[t][r];
  }
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) x[t][r] = buf[pad(pt01(t, r))];
    dit_pass10(x[t], t, T);
    for (int r = 0; r < 16; r++) z[pt01(t, r)] = x[t][r];
  }
}

static void fwd(const int64_t* a, cd* z) {
  for (int m = 0; m < SF_M; m++) z[m] = cmul(cd{(double)a[m], (double)a[m + SF_M]}, P[m]);
  if (g_wave) return wave_fwd(z);
  for (int s = 0; s < 5; s++)
    for (int t = 0; t < SF_NT; t++) dif_stage(z, s, t, T);
}

static void inv(cd* z, double* out) {
  if (g_wave)
    wave_inv(z);
  else
    for (int s = 4; s >= 0; s--)
      for (int t = 0; t < SF_NT; t++) dit_stage(z, s, t, T);
  for (int m = 0; m < SF_M; m++) {
    const cd y = cmulc(z[m], P[m]);
    out[m] = y.x;
    out[m + SF_M] = y.y;
  }
}

int main(int argc, char** argv) {
  tables();
  const int trials = argc > 1 ? atoi(argv[1]) : 6;
  g_wave = argc > 2 && argv[2][0] == 'w';
  const int lbits = argc > 3 ? atoi(argv[3]) : 16;
  const int64_t lh = (int64_t)1 << (lbits - 1);
  {  // the wave form computes the same spectrum positions as the stage form
    std::mt19937_64 g0(7);
    std::vector<int64_t> a(SF_N);
    for (auto& v : a) v = (int64_t)(g0() % (1u << 24)) - (1 << 23);
    std::vector<cd> z1(SF_M), z2(SF_M);
    const bool w = g_wave;
    g_wave = false;
    fwd(a.data(), z1.data());
    g_wave = true;
    fwd(a.data(), z2.data());
    g_wave = w;
    double d = 0;
    for (int f = 0; f < SF_M; f++) d = fmax(d, fmax(fabs(z1[f].x - z2[f].x), fabs(z1[f].y - z2[f].y)));
    printf("stage form vs wave form spectra: max |diff| = %.3e\n", d);
    if (d > 1e-3) return 1;
  }
  std::mt19937_64 g(12345);
  double worst = 0;
  for (int tr = 0; tr < trials; tr++) {
    const int mode = tr % 3;  // 0 uniform, 1 extreme magnitudes, 2 all-max (worst-case magnitude)
    std::vector<int64_t> d(9 * SF_N), l(9 * SF_N);
    for (int i = 0; i < 9 * SF_N; i++) {
      if (mode == 2) {
        d[i] = -(1 << 23);
        l[i] = -lh;
      } else if (mode == 1) {
        d[i] = (g() & 1) ? (1 << 23) - 1 : -(1 << 23);
        l[i] = (g() & 1) ? lh - 1 : -lh;
      } else {
        d[i] = (int64_t)(g() % (1u << 24)) - (1 << 23);
        l[i] = (int64_t)(g() % (2 * (uint64_t)lh)) - lh;
      }
    }
    std::vector<cd> O(SF_M, cd{0, 0}), zd(SF_M), zl(SF_M);
    for (int r = 0; r < 9; r++) {
      fwd(&d[r * SF_N], zd.data());
      fwd(&l[r * SF_N], zl.data());
      for (int f = 0; f < SF_M; f++) {
        const cd k = {zl[f].x / SF_M, zl[f].y / SF_M};
        O[f] = cmac(O[f], zd[f], k);
      }
    }
    std::vector<double> got(SF_N);
    inv(O.data(), got.data());
    double err = 0;
    i128 maxmag = 0;
    for (int n = 0; n < SF_N; n++) {
      i128 ex = 0;
      for (int r = 0; r < 9; r++)
        for (int i = 0; i < SF_N; i++) {
          const int j = n - i;
          const i128 pr = (i128)d[r * SF_N + i] * l[r * SF_N + (j >= 0 ? j : j + SF_N)];
          ex += j >= 0 ? pr : -pr;
        }
      const double e = fabs(got[n] - (double)ex);
      if (e > err) err = e;
      if ((ex < 0 ? -ex : ex) > maxmag) maxmag = ex < 0 ? -ex : ex;
    }
    printf("trial %d mode %d: max |f64 - exact| = %.3e, max |exact| = 2^%.2f\n", tr, mode, err,
           log2((double)maxmag));
    if (err > worst) worst = err;
  }
  if (lbits > 16) {  // the low limb: an error e lands as e * 2^16 in a 2^128 accumulator with ~2^64 noise
    printf("worst %.3e = 2^%.1f (%s)\n", worst, log2(worst), worst < 0x1p34 ? "OK: below 2^34" : "FAIL");
    return worst < 0x1p34 ? 0 : 1;
  }
  printf("worst %.3e (%s)\n", worst, worst < 0.25 ? "OK: rint exact" : "FAIL");
  return worst < 0.25 ? 0 : 1;
}
