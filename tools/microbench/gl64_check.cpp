// Host check of the Goldilocks primitives in tfhe_amd/csrc/gl64.h against 128-bit reference
// arithmetic: random words plus the edge values around 0, p, 2^32 and 2^64 (inputs need not be
// canonical).  Build: hipcc -O2 -std=c++17 -I tfhe_amd/csrc tools/microbench/gl64_check.cpp
#include <cstdio>
#include <random>
#include <vector>
#include "gl64.h"
using namespace tfhe;
typedef unsigned __int128 u128;
static const u128 P = GL_P;
static u64 ref_mod(u128 x) { return (u64)(x % P); }
static u64 ref_pow2(int r) { u128 v = 1; for (int i = 0; i < r; i++) v = (v * 2) % P; return (u64)v; }

int main() {
  std::mt19937_64 rng(12345);
  std::vector<u64> edge = {0, 1, 2, GL_EPS - 1, GL_EPS, GL_EPS + 1, 1ull << 32, GL_P - 2, GL_P - 1, GL_P, GL_P + 1,
                           GL_P + GL_EPS - 1, ~0ull, ~0ull - 1, 1ull << 63, (1ull << 63) - 1, 0xFFFFFFFF00000000ull,
                           0x00000000FFFFFFFFull, 0x8000000080000000ull};
  long bad = 0, n = 0;
  auto val = [&](long i) -> u64 {
    if (i < (long)edge.size()) return edge[i];
    u64 r = rng();
    switch (rng() % 4) {
      case 0: return r;
      case 1: return GL_P - 1 - (r & 0xFFFF);         // near p (canonical)
      case 2: return GL_P + (r % GL_EPS);             // non-canonical
      default: return r | 0xFFFFFFFF00000000ull;      // high word all ones
    }
  };
  for (long i = 0; i < 3000000; i++) {
    const u64 a = val(i % 4000 < (long)edge.size() ? i % 4000 : 1000), b = val(i % 19), z = val((i * 7) % 23);
    const u64 aa = i < 400 ? edge[i % edge.size()] : (i & 1 ? a : rng()), bb = i < 400 ? edge[(i / edge.size()) % edge.size()] : (i & 2 ? b : rng());
    const u64 zz = i & 4 ? z : rng();
    n++;
    // gl_mul: canonical inputs -> canonical product
    const u64 ca = aa % GL_P, cb = bb % GL_P;
    u64 m = gl_mul(ca, cb);
    if (m != ref_mod((u128)ca * cb)) { if (bad++ < 5) printf("mul %lx %lx -> %lx\n", ca, cb, m); }
    // gl_mul on non-canonical inputs must still be canonical & correct
    m = gl_mul(aa, bb);
    if (m != ref_mod((u128)aa * bb)) { if (bad++ < 5) printf("mul(nc) %lx %lx -> %lx\n", aa, bb, m); }
    // mac128 exact
    u64 hi, lo;
    gl_mac128(aa, bb, zz, hi, lo);
    if ((((u128)hi << 64) | lo) != (u128)aa * bb + zz) { if (bad++ < 5) printf("mac128 %lx %lx %lx\n", aa, bb, zz); }
    // lazy mac: congruent
    const u64 l = gl_mac_lazy(zz, aa, bb);
    if (l % GL_P != ref_mod((u128)aa * bb + zz)) { if (bad++ < 5) printf("mac_lazy %lx %lx %lx -> %lx\n", zz, aa, bb, l); }
    if (gl_canon(l) != ref_mod((u128)aa * bb + zz)) { if (bad++ < 5) printf("canon\n"); }
    // reductions on arbitrary (hi, lo)
    const u64 h2 = rng() ^ (i & 8 ? ~0ull : 0), l2 = (i & 16) ? zz : rng();
    if (gl_reduce128(h2, l2) != ref_mod(((u128)h2 << 64) | l2)) { if (bad++ < 5) printf("red128 %lx %lx\n", h2, l2); }
    if (gl_reduce128_lazy(h2, l2) % GL_P != ref_mod(((u128)h2 << 64) | l2)) { if (bad++ < 5) printf("red128l\n"); }
    const u64 h3 = h2 >> 32;
    if (gl_reduce96(h3, l2) != ref_mod(((u128)h3 << 64) | l2)) { if (bad++ < 5) printf("red96 %lx %lx\n", h3, l2); }
    if (gl_reduce96_lazy(h3, l2) % GL_P != ref_mod(((u128)h3 << 64) | l2)) { if (bad++ < 5) printf("red96l\n"); }
    // add / sub on canonical inputs
    if (gl_add(ca, cb) != ref_mod((u128)ca + cb)) { if (bad++ < 5) printf("add\n"); }
    if (gl_sub(ca, cb) != ref_mod((u128)ca + P - cb)) { if (bad++ < 5) printf("sub\n"); }
  }
  // shl_mod / mul_pow2 for every exponent
  std::vector<u64> pw(192);
  for (int r = 0; r < 192; r++) pw[r] = ref_pow2(r);
  for (long i = 0; i < 200000; i++) {
    const u64 x = i < (long)edge.size() ? edge[i] : val(1000);
    const int r = (int)(i % 96);
    const u64 s = gl_shl_mod(x, r);
    const u64 want = ref_mod((u128)x * pw[r]);
    if (r > 0 ? s != want : s != x) { if (bad++ < 5) printf("shl %lx r=%d -> %lx want %lx\n", x, r, s, want); }
    if (r >= 1 && r <= 32) {  // x * 2^-r == x * 2^(192 - r)
      const u64 sr = gl_shr_mod(x, r);
      if (sr != ref_mod((u128)x * pw[192 - r])) { if (bad++ < 5) printf("shr %lx r=%d -> %lx\n", x, r, sr); }
    }
    for (int z = (int)(i % 7); z < 192; z += 7) {
      bool ng = false;
      const u64 tv = gl_pow2_twiddle(x, z, ng);
      const u64 got = ng ? (GL_P - tv % GL_P) % GL_P : tv % GL_P;
      if (got != ref_mod((u128)x * pw[z])) { if (bad++ < 5) printf("tw %lx z=%d\n", x, z); }
    }
    const u64 cx = x % GL_P;
    const int s2 = (int)(i % 192);
    if (gl_mul_pow2(cx, s2) != ref_mod((u128)cx * pw[s2])) { if (bad++ < 5) printf("pow2 %lx s=%d\n", cx, s2); }
    n++;
  }
  printf("%s: %ld cases, %ld mismatches\n", bad ? "FAIL" : "OK", n, bad);
  return bad != 0;
}
