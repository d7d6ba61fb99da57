// Host accuracy check of the noise-squashing f64 FFT product (tfhe_amd/csrc/sns_fft.h): 9-term sums of
// digit (|d| <= 2^23) x limb (|l| <= 2^15) negacyclic convolutions at N = 2048 through the same stage
// functions the device runs, against the exact int128 schoolbook product.  Prints the largest distance
// of an f64 output from its exact integer: the device rounds with rint(), so it must stay below 1/2.
//   g++ -O2 -std=c++17 -I tfhe_amd/csrc tools/sns_fft_check.cpp -o /tmp/sns_fft_check && /tmp/sns_fft_check
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

static void fwd(const int64_t* a, cd* z) {
  for (int m = 0; m < SF_M; m++) z[m] = cmul(cd{(double)a[m], (double)a[m + SF_M]}, P[m]);
  for (int s = 0; s < 5; s++)
    for (int t = 0; t < SF_NT; t++) dif_stage(z, s, t, T);
}

static void inv(cd* z, double* out) {
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
  std::mt19937_64 g(12345);
  double worst = 0;
  for (int tr = 0; tr < trials; tr++) {
    const int mode = tr % 3;  // 0 uniform, 1 extreme magnitudes, 2 all-max (worst-case magnitude)
    std::vector<int64_t> d(9 * SF_N), l(9 * SF_N);
    for (int i = 0; i < 9 * SF_N; i++) {
      if (mode == 2) {
        d[i] = -(1 << 23);
        l[i] = -(1 << 15);
      } else if (mode == 1) {
        d[i] = (g() & 1) ? (1 << 23) - 1 : -(1 << 23);
        l[i] = (g() & 1) ? (1 << 15) - 1 : -(1 << 15);
      } else {
        d[i] = (int64_t)(g() % (1u << 24)) - (1 << 23);
        l[i] = (int64_t)(g() % (1u << 16)) - (1 << 15);
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
  printf("worst %.3e (%s)\n", worst, worst < 0.25 ? "OK: rint exact" : "FAIL");
  return worst < 0.25 ? 0 : 1;
}
