// client.cpp — client-side key material for libtfhe_hip.so (host C++, std::thread).
//
// Replaces the key-generation / encryption role the reference delegates to tfhe-rs WASM
// (sdk/relayer/src/tfhe.ts:20-28, generateKeys.js:20-31) and the server /encrypt + /decrypt
// endpoints (packages/luxfhejs/src/index.ts:127-141, packages/hardhat-plugin/src/index.ts:71-75),
// for the deterministic seeded key sets this engine consumes.  Compiled with -ffp-contract=off:
// the Gaussian sampler uses only IEEE + - * / sqrt, so keys are bit-identical on every host.
#include <math.h>
#include <stdint.h>
#include <errno.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/tfhe_hip.h"
#include "client.h"

namespace tfhe {
namespace client {

static constexpr uint64_t P = 0xFFFFFFFF00000001ull;

// Static-partition parallel for over [0, count) on hardware threads (std::thread, no OpenMP runtime).
template <class F>
static void parallel_for(int64_t count, F&& f) {
  unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int64_t nt = std::min<int64_t>(std::min<int64_t>(hw, 32), count);
  if (nt <= 1) {
    for (int64_t i = 0; i < count; i++) f(i);
    return;
  }
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; t++)
    th.emplace_back([&, t] {
      for (int64_t i = t; i < count; i += nt) f(i);
    });
  for (auto& x : th) x.join();
}

// ---------------------------------------------------------------- ChaCha20 (RFC 8439) stream
// A 64-bit seed maps to the rng key (seed, "tfhe-amd chacha!"): the reproducible streams that tests,
// golden vectors and the oracle use.  Production keys / encryptions take 192 bits of OS entropy
// instead (rng_key_entropy), so nothing about them follows from public constants.
tfhe_rng_key rng_key_from_seed(uint64_t seed) {
  static const uint8_t tag[16] = {'t', 'f', 'h', 'e', '-', 'a', 'm', 'd', ' ', 'c', 'h', 'a', 'c', 'h', 'a', '!'};
  tfhe_rng_key k;
  k.w[0] = (uint32_t)seed;
  k.w[1] = (uint32_t)(seed >> 32);
  memcpy(&k.w[2], tag, 16);
  return k;
}

bool rng_key_entropy(tfhe_rng_key* k) {
  uint8_t* p = (uint8_t*)k->w;
  size_t got = 0;
  while (got < sizeof(k->w)) {
    const ssize_t r = getrandom(p + got, sizeof(k->w) - got, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    got += (size_t)r;
  }
  return true;
}

struct ChaCha {
  uint32_t key[8];
  uint32_t ctr = 0;
  uint32_t buf[16];
  int pos = 16;

  // key words 0, 1, 4..7 = the 192-bit rng key, words 2, 3 = the stream index
  ChaCha(const tfhe_rng_key& rk, uint64_t stream) {
    key[0] = rk.w[0];
    key[1] = rk.w[1];
    key[2] = (uint32_t)stream;
    key[3] = (uint32_t)(stream >> 32);
    for (int i = 0; i < 4; i++) key[4 + i] = rk.w[2 + i];
  }
  static inline uint32_t rl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
  void refill() {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4],      key[5],      key[6],      key[7],      ctr++,  0,      0,      0};
    uint32_t x[16];
    memcpy(x, s, sizeof(x));
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; r++) {
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; i++) buf[i] = x[i] + s[i];
    pos = 0;
  }
  uint64_t next() {
    if (pos >= 16) refill();
    uint64_t v = (uint64_t)buf[pos] | ((uint64_t)buf[pos + 1] << 32);
    pos += 2;
    return v;
  }
  uint64_t next_mod_p() {
    for (;;) {
      uint64_t v = next();
      if (v < P) return v;
    }
  }
  // Box-Muller (cosine branch) with series log / cos in plain IEEE double arithmetic.
  static double dlog(double u) {
    int ex;
    double m = frexp(u, &ex);
    if (m < 0.70710678118654752) { m *= 2.0; ex -= 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double term = s, acc = 0.0;
    for (int i = 1; i <= 23; i += 2) { acc += term / (double)i; term *= s2; }
    return (double)ex * 6.93147180369123816490e-01 + ((double)ex * 1.90821492927058770002e-10 + 2.0 * acc);
  }
  static double dsin(double x) {
    const double x2 = x * x;
    double term = x, acc = 0.0;
    for (int i = 1; i <= 21; i += 2) { acc += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
    return acc;
  }
  static double dcos(double x) {
    const double x2 = x * x;
    double term = 1.0, acc = 0.0;
    for (int i = 0; i <= 20; i += 2) { acc += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
    return acc;
  }
  static double dcos2pi(double u) {
    const double two_pi = 6.28318530717958647692;
    double v = u <= 0.5 ? u : 1.0 - u, sg = 1.0;
    if (v > 0.25) { sg = -1.0; v = 0.5 - v; }
    if (v > 0.125) return sg * dsin(two_pi * (0.25 - v));
    return sg * dcos(two_pi * v);
  }
  int64_t gauss(int32_t log2_sigma) {
    const double u1 = (double)((next() >> 11) + 1) * 0x1.0p-53;
    const double u2 = (double)(next() >> 11) * 0x1.0p-53;
    const double z = sqrt(-2.0 * dlog(u1)) * dcos2pi(u2);
    return (int64_t)llrint(ldexp(z, 64 + log2_sigma));
  }
};

// ---------------------------------------------------------------- Z_p helpers (host)
static inline uint64_t padd(uint64_t a, uint64_t b) {
  uint64_t s = a + b;
  return (s < a || s >= P) ? s + 0xFFFFFFFFull : s;
}
static inline uint64_t psub(uint64_t a, uint64_t b) { return a < b ? a - b + P : a - b; }
static inline uint64_t pfrom(int64_t v) {
  if (v >= 0) return (uint64_t)v;
  uint64_t m = (0ull - (uint64_t)v) % P;
  return m ? P - m : 0;
}

size_t bsk_len(const tfhe_params& p) { return (size_t)p.n * (p.k + 1) * p.pbs_level * (p.k + 1) * p.N; }
size_t ksk_len(const tfhe_params& p) { return (size_t)p.k * p.N * p.ks_level * (p.n + 1); }

// GLWE_S(0) over Z_p: masks uniform, body = sum_c A_c * S_c + E.  S is binary, so the product is
// a signed sum of rotated masks.
static void glwe_zero(const tfhe_params& p, const uint64_t* S, ChaCha& r, uint64_t* out) {
  const uint32_t N = p.N, k = p.k;
  for (uint32_t c = 0; c < k; c++)
    for (uint32_t i = 0; i < N; i++) out[(size_t)c * N + i] = r.next_mod_p();
  uint64_t* body = out + (size_t)k * N;
  for (uint32_t i = 0; i < N; i++) body[i] = pfrom(r.gauss(p.glwe_noise_log2));
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = out + (size_t)c * N;
    const uint64_t* Sc = S + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!Sc[j]) continue;
      // body[d] += A[d - j] for d >= j ; body[d] -= A[d - j + N] for d < j
      for (uint32_t d = 0; d < j; d++) body[d] = psub(body[d], A[d + N - j]);
      for (uint32_t d = j; d < N; d++) body[d] = padd(body[d], A[d - j]);
    }
  }
}

static void glwe_native(uint32_t k, uint32_t N, const uint64_t* key, int32_t noise_log2, ChaCha& r, const uint64_t* m,
                        uint64_t* out);

static void lwe_one(uint32_t dim, const uint64_t* key, int32_t noise_log2, ChaCha& r, uint64_t m, uint64_t* out) {
  uint64_t acc = 0;
  for (uint32_t i = 0; i < dim; i++) {
    out[i] = r.next();
    acc += out[i] * key[i];
  }
  acc += (uint64_t)r.gauss(noise_log2);
  out[dim] = acc + m;
}

void keygen(const tfhe_params& p, const tfhe_rng_key& rk, uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk,
            uint64_t* ksk) {
  {
    ChaCha r(rk, 1);
    for (uint32_t i = 0; i < p.n; i++) lwe_key[i] = r.next() & 1;
  }
  {
    ChaCha r(rk, 2);
    for (uint32_t i = 0; i < p.k * p.N; i++) glwe_key[i] = r.next() & 1;
  }
  server_keygen(p, rk, lwe_key, glwe_key, bsk, ksk);
}

void server_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t* lwe_key, const uint64_t* glwe_key,
                   uint64_t* bsk, uint64_t* ksk) {
  if (bsk) {
    const size_t row = (size_t)(p.k + 1) * p.N, per_i = (size_t)(p.k + 1) * p.pbs_level * row;
    parallel_for((int64_t)p.n, [&](int64_t i) {
      ChaCha r(rk, 0x1000 + (uint64_t)i);
      for (uint32_t c = 0; c <= p.k; c++)
        for (uint32_t l = 0; l < p.pbs_level; l++) {
          uint64_t* out = bsk + per_i * i + row * (c * p.pbs_level + l);
          const uint64_t g = 1ull << (64 - p.pbs_base_log * (l + 1));
          if (p.transform == TFHE_HIP_TRANSFORM_FFT64) {  // native-torus GGSW
            glwe_native(p.k, p.N, glwe_key, p.glwe_noise_log2, r, nullptr, out);
            if (lwe_key[i]) out[(size_t)c * p.N] += g;
          } else {
            glwe_zero(p, glwe_key, r, out);
            if (lwe_key[i]) out[(size_t)c * p.N] = padd(out[(size_t)c * p.N], g);
          }
        }
    });
  }
  if (ksk) {
    const size_t per_j = (size_t)p.ks_level * (p.n + 1);
    parallel_for((int64_t)(p.k * p.N), [&](int64_t j) {
      ChaCha r(rk, 0x100000 + (uint64_t)j);
      for (uint32_t l = 0; l < p.ks_level; l++)
        lwe_one(p.n, lwe_key, p.lwe_noise_log2, r, glwe_key[j] << (64 - p.ks_base_log * (l + 1)),
                ksk + per_j * j + (size_t)l * (p.n + 1));
    });
  }
}

// modulus-switch zeros of the P-FHEVM server key: zero z on ChaCha stream 0x200000 + z
void ms_zeros_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t* lwe_key, uint32_t count, uint64_t* zeros) {
  parallel_for((int64_t)count, [&](int64_t z) {
    ChaCha r(rk, 0x200000 + (uint64_t)z);
    lwe_one(p.n, lwe_key, p.lwe_noise_log2, r, 0, zeros + (size_t)z * (p.n + 1));
  });
}

// count Gaussian noise words of ChaCha stream `stream` (the seeded keys' noise, seeded.cpp)
void noise_words(const tfhe_rng_key& rk, uint64_t stream, int32_t log2_sigma, size_t count, int64_t* out) {
  ChaCha r(rk, stream);
  for (size_t i = 0; i < count; i++) out[i] = r.gauss(log2_sigma);
}

void lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key& rk, uint64_t stream0,
                 const uint64_t* msgs, size_t count, uint64_t* out) {
  auto one = [&](int64_t q) {
    ChaCha r(rk, stream0 + (uint64_t)q);
    lwe_one(dim, key, noise_log2, r, msgs[q], out + (size_t)q * (dim + 1));
  };
  if (count > 256) parallel_for((int64_t)count, one);
  else for (int64_t q = 0; q < (int64_t)count; q++) one(q);
}

void lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out) {
  for (size_t q = 0; q < count; q++) {
    const uint64_t* c = ct + q * (dim + 1);
    uint64_t s = 0;
    for (uint32_t i = 0; i < dim; i++) s += c[i] * key[i];
    out[q] = c[dim] - s;
  }
}

static inline uint64_t tor_to_p(uint64_t v) { return v - ((v >> 32) + ((v >> 31) & 1)); }

void lut_constant(uint32_t N, uint64_t v, uint64_t* lut) {
  const uint64_t g = tor_to_p(v);
  for (uint32_t i = 0; i < N; i++) lut[i] = g;
}

// tfhe-rs generate_accumulator layout: box = N / msg_modulus, v[i] = f(i / box) * delta,
// then X^{-box/2} (half-box negacyclic rotation) so message m lands in the middle of its box.
void lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* table, uint64_t delta, uint64_t* lut) {
  const uint32_t box = N / msg_modulus, half = box / 2;
  for (uint32_t i = 0; i < N; i++) {
    const uint32_t src = i + half;  // lut[i] = (X^{-half} v)[i] = v[i + half], negated past N
    if (src < N) lut[i] = tor_to_p(table[src / box] * delta);
    else {
      const uint64_t g = tor_to_p(table[(src - N) / box] * delta);
      lut[i] = g ? P - g : 0;
    }
  }
}

// ------------------------------------------------------------ packing keyswitch key / compression
size_t pksk_len(const tfhe_pks_params& pp) { return (size_t)pp.in_dim * pp.level * (pp.out_k + 1) * pp.out_N; }

// native (2^64) GLWE encryption of the plaintext polynomial m (binary key: rotated-copy products)
static void glwe_native(uint32_t k, uint32_t N, const uint64_t* key, int32_t noise_log2, ChaCha& r, const uint64_t* m,
                        uint64_t* out) {
  uint64_t* body = out + (size_t)k * N;
  for (size_t i = 0; i < (size_t)k * N; i++) out[i] = r.next();
  for (uint32_t i = 0; i < N; i++) body[i] = (uint64_t)r.gauss(noise_log2) + (m ? m[i] : 0);
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = out + (size_t)c * N;
    const uint64_t* S = key + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!S[j]) continue;
      for (uint32_t i = 0; i < N; i++) {
        const uint32_t d = i + j;
        if (d < N) body[d] += A[i];
        else body[d - N] -= A[i];
      }
    }
  }
}

// output GLWE key from ChaCha stream 4, PKSK row j from stream 0x300000 + j
void pks_keygen(const tfhe_pks_params& pp, const tfhe_rng_key& rk, const uint64_t* in_key, uint64_t* out_key, uint64_t* pksk) {
  const uint32_t k = pp.out_k, N = pp.out_N;
  {
    ChaCha r(rk, 4);
    for (uint32_t i = 0; i < k * N; i++) out_key[i] = r.next() & 1;
  }
  if (!pksk) return;
  const size_t row = (size_t)(k + 1) * N;
  parallel_for((int64_t)pp.in_dim, [&](int64_t j) {
    ChaCha r(rk, 0x300000 + (uint64_t)j);
    std::vector<uint64_t> m(N, 0);
    for (uint32_t l = 0; l < pp.level; l++) {
      m[0] = in_key[j] << (64 - pp.base_log * (l + 1));
      glwe_native(k, N, out_key, pp.noise_log2, r, m.data(), pksk + ((size_t)j * pp.level + l) * row);
    }
  });
}

void glwe_phase_native(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out) {
  memcpy(out, glwe + (size_t)k * N, (size_t)N * 8);
  for (uint32_t c = 0; c < k; c++) {
    const uint64_t* A = glwe + (size_t)c * N;
    const uint64_t* S = key + (size_t)c * N;
    for (uint32_t j = 0; j < N; j++) {
      if (!S[j]) continue;
      for (uint32_t i = 0; i < N; i++) {
        const uint32_t d = i + j;
        if (d < N) out[d] -= A[i];
        else out[d - N] += A[i];
      }
    }
  }
}

size_t pks_packed_words(const tfhe_pks_params& pp, uint32_t bodies) {
  return (((size_t)pp.out_k * pp.out_N + bodies) * pp.storage_log + 63) / 64;
}

// modulus switch to storage_log bits, LSB-first bit packing (mask coefficients, then `bodies` body ones)
void pks_compress(const tfhe_pks_params& pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed) {
  const uint32_t w = pp.storage_log;
  const size_t vals = (size_t)pp.out_k * pp.out_N + bodies;
  const uint64_t mask = (w == 64) ? ~0ull : ((1ull << w) - 1);
  memset(packed, 0, pks_packed_words(pp, bodies) * 8);
  for (size_t v = 0; v < vals; v++) {
    const uint64_t x = glwe[v];
    const uint64_t ms = (((x >> (64 - w - 1)) + 1) >> 1) & mask;
    const size_t bit = v * w, word = bit >> 6, off = bit & 63;
    packed[word] |= ms << off;
    if (off + w > 64) packed[word + 1] |= ms >> (64 - off);
  }
}

void pks_extract(const tfhe_pks_params& pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe) {
  const uint32_t w = pp.storage_log;
  const size_t vals = (size_t)pp.out_k * pp.out_N + bodies;
  const uint64_t mask = (w == 64) ? ~0ull : ((1ull << w) - 1);
  memset(glwe, 0, (size_t)(pp.out_k + 1) * pp.out_N * 8);
  for (size_t v = 0; v < vals; v++) {
    const size_t bit = v * w, word = bit >> 6, off = bit & 63;
    uint64_t ms = packed[word] >> off;
    if (off + w > 64) ms |= packed[word + 1] << (64 - off);
    glwe[v] = (ms & mask) << (64 - w);
  }
}

// ------------------------------------------------------------ noise squashing (128-bit GLWE, native 2^128 torus)
// Words of Z_2^128 as two u64 planes per polynomial ([lo][N] then [hi][N]); oracle/sns_oracle.c is the rule.
typedef unsigned __int128 u128;

size_t sns_bsk_len(const tfhe_sns_params& sp) {
  return (size_t)sp.n * (sp.k + 1) * sp.level * (sp.k + 1) * 2 * sp.N;
}

static inline u128 sns_ld(const uint64_t* plane, size_t N, size_t t) { return ((u128)plane[N + t] << 64) | plane[t]; }
static inline void sns_st(uint64_t* plane, size_t N, size_t t, u128 v) {
  plane[t] = (uint64_t)v;
  plane[N + t] = (uint64_t)(v >> 64);
}

// GLWE key from ChaCha stream 5; BSK row i from stream 0x400000 + i: masks uniform over Z_2^128 (lo word, then hi
// word, per coefficient), one Gaussian integer per body coefficient, body = sum_j mask_j (*) S_j + e (exact
// negacyclic products mod 2^128: the binary key's set bits add rotated masks), s_i 2^(128 - B (l + 1)) on
// coefficient 0 of component c.  Layout [i][c*L+l][j][lo, hi][N].
void sns_keygen(const tfhe_sns_params& sp, const tfhe_rng_key& rk, const uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk) {
  const uint32_t k = sp.k, N = sp.N, L = sp.level;
  {
    ChaCha r(rk, 5);
    for (uint32_t i = 0; i < k * N; i++) glwe_key[i] = r.next() & 1;
  }
  if (!bsk) return;
  // set-bit lists of the key polynomials
  std::vector<std::vector<uint32_t>> bits(k);
  for (uint32_t j = 0; j < k; j++)
    for (uint32_t u = 0; u < N; u++)
      if (glwe_key[(size_t)j * N + u]) bits[j].push_back(u);
  const size_t row = (size_t)(k + 1) * 2 * N, per_i = (size_t)(k + 1) * L * row;
  parallel_for((int64_t)sp.n, [&](int64_t i) {
    ChaCha r(rk, 0x400000 + (uint64_t)i);
    std::vector<u128> body(N), mask(N);
    for (uint32_t c = 0; c <= k; c++)
      for (uint32_t l = 0; l < L; l++) {
        uint64_t* out = bsk + per_i * i + row * (c * L + l);
        for (uint32_t j = 0; j < k; j++)
          for (uint32_t t = 0; t < N; t++) {
            const uint64_t lo = r.next(), hi = r.next();
            sns_st(out + (size_t)j * 2 * N, N, t, ((u128)hi << 64) | lo);
          }
        for (uint32_t t = 0; t < N; t++) body[t] = (u128)(__int128)r.gauss(sp.noise_log2);
        for (uint32_t j = 0; j < k; j++) {
          for (uint32_t t = 0; t < N; t++) mask[t] = sns_ld(out + (size_t)j * 2 * N, N, t);
          for (const uint32_t u : bits[j]) {
            for (uint32_t x = 0; x < u; x++) body[x] -= mask[x + N - u];
            for (uint32_t x = u; x < N; x++) body[x] += mask[x - u];
          }
        }
        for (uint32_t t = 0; t < N; t++) sns_st(out + (size_t)k * 2 * N, N, t, body[t]);
        if (lwe_key[i]) {
          uint64_t* dst = out + (size_t)c * 2 * N;
          sns_st(dst, N, 0, sns_ld(dst, N, 0) + ((u128)1 << (128 - sp.base_log * (l + 1))));
        }
      }
  });
}

// identity LUT over msg_modulus values (delta = 2^127 / msg_modulus, half-box rotation): [lo, hi][N]
void sns_lut_identity(const tfhe_sns_params& sp, uint32_t msg_modulus, uint64_t* lut) {
  const uint32_t N = sp.N, box = N / msg_modulus;
  const u128 delta = ((u128)1 << 127) / msg_modulus;
  for (uint32_t i = 0; i < N; i++) {
    const uint32_t src = i + box / 2;
    const u128 t = (u128)((src < N ? src : src - N) / box) * delta;
    sns_st(lut, N, i, src < N ? t : (u128)0 - t);
  }
}

void sns_phase(const tfhe_sns_params& sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count, uint64_t* out) {
  const size_t dim = (size_t)sp.k * sp.N;
  for (size_t q = 0; q < count; q++) {
    const uint64_t* c = cts + q * 2 * (dim + 1);
    u128 s = 0;
    for (size_t i = 0; i < dim; i++)
      if (glwe_key[i]) s += ((u128)c[2 * i + 1] << 64) | c[2 * i];
    const u128 ph = (((u128)c[2 * dim + 1] << 64) | c[2 * dim]) - s;
    out[2 * q] = (uint64_t)ph;
    out[2 * q + 1] = (uint64_t)(ph >> 64);
  }
}

}  // namespace client
}  // namespace tfhe
