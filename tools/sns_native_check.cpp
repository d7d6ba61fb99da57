// Host replay of the noise-squashing blind rotation exactly as the device computes it (tfhe_amd/csrc/sns.hip),
// against the oracle (oracle/sns_oracle.c, linked as liboracle.so: this is a test tool).  Shared with the
// device through sns_fft.h: the key rounding and limb split (key_round16 / key_limb), the 128-bit
// decomposition (digits72), the Horner recombination (horner16, horner_low) and the FFT passes -- the one-wave form of
// step 1 for the digit spectra, the 256-thread stage form for the key spectra and the inverse.  Run at a
// reduced input dimension with arbitrary 64-bit input words; prints the accumulator words that differ.
//   g++ -O2 -std=c++17 -ffp-contract=off -I tfhe_amd/csrc -I oracle tools/sns_native_check.cpp -L oracle -loracle \
//       -Wl,-rpath,$PWD/oracle -o /tmp/sns_native_check && /tmp/sns_native_check [n] [cts]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

extern "C" {
#include "tfhe_oracle.h"
}
#include "sns_fft.h"

using namespace tfhe::snsf;

static cd T[SF_M], P[SF_M];
static constexpr int N = SF_N, K = 2, L = 3, R = (K + 1) * L, LIMBS = SF_LIMBS;

static void tables() {  // make_sns_fft_const's tables
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int e = 0; e < SF_M; e++) {
    T[e] = {(double)cosl(2 * pi * e / SF_M), (double)sinl(2 * pi * e / SF_M)};
    P[e] = {(double)cosl(pi * e / SF_N), (double)sinl(pi * e / SF_N)};
  }
}

static w128 ld(const uint64_t* plane_lo, int t) { return ((w128)plane_lo[N + t] << 64) | plane_lo[t]; }
static void st(uint64_t* plane_lo, int t, w128 v) {
  plane_lo[t] = (uint64_t)v;
  plane_lo[N + t] = (uint64_t)(v >> 64);
}
static uint32_t ms4096(uint64_t x) { return (uint32_t)(((x >> 51) + 1) >> 1) & 4095u; }

// sns_step1f_kernel's one-wave forward transform (64 simulated lanes)
static void wave_fwd(const int* d, cd* out) {
  static cd x[64][16], buf[SF_PADDED];
  for (int t = 0; t < 64; t++) {
    for (int r = 0; r < 16; r++) {
      const int m = pt01(t, r);
      x[t][r] = cmul(cd{(double)d[m], (double)d[m + SF_M]}, P[m]);
    }
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
    for (int r = 0; r < 16; r++) buf[pad(pt4(t, r))] = x[t][r];
  }
  for (int f = 0; f < SF_M; f++) out[f] = buf[pad(f)];
}

int main(int argc, char** argv) {
  tables();
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 6;
  const int cts = argc > 2 ? atoi(argv[2]) : 3;
  or_sns_params sp;
  or_sns_params_preset(0, &sp);
  sp.n = n;
  std::mt19937_64 g(0x5A5A);
  std::vector<uint64_t> lwe_key(n), glwe_key((size_t)K * N), bsk(or_sns_bsk_len(&sp)), rounded(bsk.size());
  for (auto& b : lwe_key) b = g() & 1;
  or_sns_keygen(&sp, 0x7F4E0001ull, lwe_key.data(), glwe_key.data(), bsk.data());
  or_sns_bsk_round(&sp, bsk.data(), rounded.data());
  std::vector<uint64_t> limb(or_sns_limb_ntt_len(&sp)), lut(2 * (size_t)N);
  or_sns_bsk_to_limb_ntt(&sp, rounded.data(), limb.data());
  or_sns_lut_identity(&sp, 16, lut.data());

  // sns_bsk_to_fft_kernel: per (i, r, j) polynomial, 5 limb spectra / M (stage form)
  const size_t polys = bsk.size() / (2 * N);
  std::vector<cd> kf(polys * LIMBS * SF_M);
  std::vector<__int128> rr(N);
  std::vector<cd> z(SF_M);
  for (size_t p = 0; p < polys; p++) {
    for (int x = 0; x < N; x++) rr[x] = key_round16(ld(&bsk[p * 2 * N], x));
    for (int t = 0; t < LIMBS; t++) {
      std::vector<double> lv(N);
      for (int x = 0; x < N; x++) lv[x] = (double)key_limb(rr[x], t);
      for (int m = 0; m < SF_M; m++) z[m] = cmul(cd{lv[m], lv[m + SF_M]}, P[m]);
      for (int s = 0; s < 5; s++)
        for (int th = 0; th < SF_NT; th++) dif_stage(z.data(), s, th, T);
      for (int f = 0; f < SF_M; f++) kf[(p * LIMBS + t) * SF_M + f] = cd{z[f].x * (1.0 / SF_M), z[f].y * (1.0 / SF_M)};
    }
  }

  long bad = 0;
  for (int q = 0; q < cts; q++) {
    std::vector<uint64_t> lwe(n + 1);
    for (auto& w : lwe) w = g();
    if (q == 1)
      for (uint32_t i = 0; i < n; i++) lwe[i] = 0;  // trivial mask
    std::vector<uint64_t> ref((size_t)(K + 1) * 2 * N), acc((size_t)(K + 1) * 2 * N, 0);
    or_sns_blind_rotate(&sp, limb.data(), lwe.data(), lut.data(), ref.data());
    // sns_init_kernel
    const uint32_t sh = (4096u - ms4096(lwe[n])) & 4095u;
    for (int t = 0; t < N; t++) {
      uint32_t dst = (uint32_t)t + sh;
      bool neg = false;
      if (dst >= 4096u) dst -= 4096u;
      if (dst >= (uint32_t)N) dst -= N, neg = true;
      const w128 v = ld(lut.data(), t);
      st(&acc[(size_t)K * 2 * N], (int)dst, neg ? (w128)0 - v : v);
    }
    std::vector<cd> Df((size_t)R * SF_M);
    std::vector<int> dig((size_t)L * N);
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t ai = ms4096(lwe[i]);
      for (int c = 0; c <= K; c++) {  // sns_step1f_kernel
        const uint64_t* a = &acc[(size_t)c * 2 * N];
        for (int t = 0; t < N; t++) {
          const uint32_t t1 = ((uint32_t)t - ai) & 4095u;
          const w128 v = ld(a, (int)(t1 & (N - 1)));
          int d[3];
          digits72((t1 >= (uint32_t)N ? (w128)0 - v : v) - ld(a, t), d);
          for (int l = 0; l < L; l++) dig[(size_t)l * N + t] = d[l];
        }
        for (int l = 0; l < L; l++) wave_fwd(&dig[(size_t)l * N], &Df[(size_t)(c * L + l) * SF_M]);
      }
      const cd* kfi = &kf[(size_t)i * R * (K + 1) * LIMBS * SF_M];
      for (int j = 0; j <= K; j++) {  // sns_mac_kernel + sns_inv_kernel
        std::vector<w128> h(N, 0);
        for (int t = LIMBS - 1; t >= 0; t--) {
          for (int f = 0; f < SF_M; f++) {
            cd o = {0.0, 0.0};
            for (int r = 0; r < R; r++) o = cmac(o, Df[(size_t)r * SF_M + f], kfi[((size_t)r * (K + 1) * LIMBS + j * LIMBS + t) * SF_M + f]);
            z[f] = o;
          }
          for (int s = 4; s >= 0; s--)
            for (int th = 0; th < SF_NT; th++) dit_stage(z.data(), s, th, T);
          for (int m = 0; m < SF_M; m++) {
            const cd y = cmulc(z[m], P[m]);
            h[m] = t ? horner16(h[m], rint(y.x)) : horner_low(h[m], rint(y.x));
            h[m + SF_M] = t ? horner16(h[m + SF_M], rint(y.y)) : horner_low(h[m + SF_M], rint(y.y));
          }
        }
        uint64_t* a = &acc[(size_t)j * 2 * N];
        for (int x = 0; x < N; x++) st(a, x, ld(a, x) + (h[x] << 16));
      }
    }
    long diff = 0;
    for (size_t e = 0; e < acc.size(); e++) diff += acc[e] != ref[e];
    printf("ciphertext %d: %ld of %zu accumulator words differ from the oracle\n", q, diff, acc.size());
    bad += diff;
  }
  printf("%s\n", bad ? "FAIL" : "OK: device arithmetic == oracle");
  return bad ? 1 : 0;
}
