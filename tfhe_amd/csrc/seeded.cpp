// seeded.cpp — compressed (seeded) server keys: the CompressedServerKey half of SURVEY §8f f3 (host C++).
//
// tfhe-rs ships evaluation keys compressed: every GLWE / LWE ciphertext of the bootstrapping key, the keyswitching
// key and the modulus-switch zeros keeps only its body, and the masks are regenerated from a 128-bit seed
// (tfhe-rs core_crypto decompress_seeded_lwe_bootstrap_key, decompress_seeded_lwe_keyswitch_key,
// decompress_seeded_lwe_ciphertext_list; the fhEVM coprocessor keeps its tenants' keys this way,
// tests/fhevm-suite/fhevm/docker-compose/coprocessor-docker-compose.yml:96).  tfhe-rs is absent from the reference
// mount, and the mount holds no server-key file, so this restates the published algorithm and is PARITY UNPINNED
// at the byte level; AES-128 itself is pinned by the FIPS-197 known answer (tests/test_seeded.py).
//
// Mask stream (tfhe-csprng AesCtrGenerator, software backend, as restated here):
//   AES-128 key = the seed's 16 bytes, little endian; block b of the stream = AES_key(b as a 128-bit little-endian
//   counter); the generator starts at table index SECOND (block 0, byte 1: the first byte is never output); a
//   native-modulus mask element is the next 8 bytes, little endian.  Forks hand out consecutive byte ranges, so
//   the masks of a whole key are one contiguous run of the stream in the order the encryption walks them:
//     bootstrapping key   GGSW i < n, level l < L (most significant first), row c <= k: k*N mask words
//     keyswitching key    input key element j < k*N, storage row s < ks_level: n mask words, where storage row s
//                         holds decomposition level ks_level - s (tfhe-rs generate_lwe_keyswitch_key walks the
//                         levels (1..=level_count).rev(), least significant first, so a block lines up with the
//                         SignedDecomposer's low-to-high digit iterator); this engine's KSK row l is level l + 1
//                         (most significant first), so storage row s <-> engine row ks_level - 1 - s
//     ciphertext list     ciphertext z: dim mask words
// A GGSW row c < k of tfhe-rs encrypts -m*g*S_c and row k encrypts m*g (g = 2^(64 - beta (l + 1))); this engine's
// keygen adds m*g to mask c of an encryption of zero instead.  Both have the same phase, which is all the external
// product uses, so an ingested row is stored as it is.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/tfhe_hip.h"
#include "client.h"

namespace tfhe {
namespace seeded {

// ------------------------------------------------------------------------------- AES-128 (FIPS-197)
namespace {
uint8_t SBOX[256];

inline uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
inline uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ ((x >> 7) * 0x1b)); }

void init_sbox() {
  // walk the multiplicative group by p *= 3, q = p^-1 (q /= 3), S(p) = affine(q)
  uint8_t p = 1, q = 1;
  do {
    p = (uint8_t)(p ^ (p << 1) ^ (p & 0x80 ? 0x1b : 0));
    q ^= (uint8_t)(q << 1);
    q ^= (uint8_t)(q << 2);
    q ^= (uint8_t)(q << 4);
    if (q & 0x80) q ^= 0x09;
    SBOX[p] = (uint8_t)(q ^ rotl8(q, 1) ^ rotl8(q, 2) ^ rotl8(q, 3) ^ rotl8(q, 4) ^ 0x63);
  } while (p != 1);
  SBOX[0] = 0x63;
}

struct Aes128 {
  uint8_t rk[176];
  explicit Aes128(const uint8_t key[16]) {
    static const uint8_t RCON[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
    memcpy(rk, key, 16);
    for (int i = 4; i < 44; i++) {
      uint8_t t[4] = {rk[4 * (i - 1)], rk[4 * (i - 1) + 1], rk[4 * (i - 1) + 2], rk[4 * (i - 1) + 3]};
      if (i % 4 == 0) {
        const uint8_t t0 = t[0];
        t[0] = (uint8_t)(SBOX[t[1]] ^ RCON[i / 4 - 1]);
        t[1] = SBOX[t[2]];
        t[2] = SBOX[t[3]];
        t[3] = SBOX[t0];
      }
      for (int b = 0; b < 4; b++) rk[4 * i + b] = (uint8_t)(rk[4 * (i - 4) + b] ^ t[b]);
    }
  }
  // state byte r + 4 c = row r, column c
  void encrypt(const uint8_t in[16], uint8_t out[16]) const {
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int round = 1; round <= 10; round++) {
      uint8_t t[16];
      for (int c = 0; c < 4; c++)  // SubBytes + ShiftRows
        for (int r = 0; r < 4; r++) t[r + 4 * c] = SBOX[s[r + 4 * ((c + r) & 3)]];
      if (round < 10)
        for (int c = 0; c < 4; c++) {  // MixColumns
          const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
          const uint8_t x = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
          t[4 * c] = (uint8_t)(a0 ^ x ^ xt((uint8_t)(a0 ^ a1)));
          t[4 * c + 1] = (uint8_t)(a1 ^ x ^ xt((uint8_t)(a1 ^ a2)));
          t[4 * c + 2] = (uint8_t)(a2 ^ x ^ xt((uint8_t)(a2 ^ a3)));
          t[4 * c + 3] = (uint8_t)(a3 ^ x ^ xt((uint8_t)(a3 ^ a0)));
        }
      for (int i = 0; i < 16; i++) s[i] = (uint8_t)(t[i] ^ rk[16 * round + i]);
    }
    memcpy(out, s, 16);
  }
};

struct SboxInit {
  SboxInit() { init_sbox(); }
};
const SboxInit sbox_init;

// stream bytes [byte0, byte0 + n) of the seed's AES-CTR stream (absolute byte index: block = index / 16)
void stream_bytes(const Aes128& aes, uint64_t byte0, size_t n, uint8_t* out) {
  uint64_t blk = byte0 / 16;
  size_t off = (size_t)(byte0 % 16), done = 0;
  while (done < n) {
    uint8_t ctr[16] = {0}, ks[16];
    for (int b = 0; b < 8; b++) ctr[b] = (uint8_t)(blk >> (8 * b));  // 128-bit little-endian counter (< 2^64 here)
    aes.encrypt(ctr, ks);
    const size_t take = std::min((size_t)16 - off, n - done);
    memcpy(out + done, ks + off, take);
    done += take;
    off = 0;
    blk++;
  }
}

template <class F>
void parallel_for(int64_t count, F&& f) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
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

void key_bytes(const uint64_t seed[2], uint8_t key[16]) {
  for (int b = 0; b < 8; b++) {
    key[b] = (uint8_t)(seed[0] >> (8 * b));
    key[8 + b] = (uint8_t)(seed[1] >> (8 * b));
  }
}

constexpr uint64_t STREAM_START = 1;  // TableIndex::SECOND

// mask words [w0, w0 + count) of the seed's stream
void mask_words(const Aes128& aes, uint64_t w0, size_t count, uint64_t* out) {
  std::vector<uint8_t> b(count * 8);
  stream_bytes(aes, STREAM_START + 8 * w0, b.size(), b.data());
  for (size_t i = 0; i < count; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)b[8 * i + k] << (8 * k);
    out[i] = v;
  }
}

// body += a (*) s (negacyclic, binary s)
void add_product(uint32_t N, const uint64_t* a, const uint64_t* s, uint64_t* body) {
  for (uint32_t j = 0; j < N; j++) {
    if (!s[j]) continue;
    for (uint32_t i = 0; i < N; i++) {
      const uint32_t d = i + j;
      if (d < N) body[d] += a[i];
      else body[d - N] -= a[i];
    }
  }
}
}  // namespace

void aes128_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) { Aes128(key).encrypt(in, out); }

void csprng_words(const uint64_t seed[2], uint64_t first, size_t count, uint64_t* out) {
  uint8_t key[16];
  key_bytes(seed, key);
  const Aes128 aes(key);
  const size_t chunk = 1 << 14;
  const int64_t nch = (int64_t)((count + chunk - 1) / chunk);
  parallel_for(nch, [&](int64_t c) {
    const size_t o = (size_t)c * chunk;
    mask_words(aes, first + o, std::min(chunk, count - o), out + o);
  });
}

// seeded BSK / KSK bodies for given binary secret keys; noise from the ChaCha streams of server_keygen
void seeded_server_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t bsk_seed[2],
                          const uint64_t ksk_seed[2], const uint64_t* lwe_key, const uint64_t* glwe_key,
                          uint64_t* bsk_bodies, uint64_t* ksk_bodies) {
  const uint32_t k = p.k, N = p.N, L = p.pbs_level, n = p.n;
  uint8_t key[16];
  if (bsk_bodies) {
    key_bytes(bsk_seed, key);
    const Aes128 aes(key);
    parallel_for((int64_t)n, [&](int64_t i) {
      std::vector<uint64_t> mask((size_t)k * N);
      std::vector<int64_t> e((size_t)L * (k + 1) * N);
      client::noise_words(rk, 0x1000 + (uint64_t)i, p.glwe_noise_log2, e.size(), e.data());
      for (uint32_t l = 0; l < L; l++) {
        const uint64_t g = 1ull << (64 - p.pbs_base_log * (l + 1));
        for (uint32_t c = 0; c <= k; c++) {
          const size_t row = ((size_t)i * L + l) * (k + 1) + c;
          mask_words(aes, row * k * N, (size_t)k * N, mask.data());
          uint64_t* body = bsk_bodies + row * N;
          for (uint32_t t = 0; t < N; t++) body[t] = (uint64_t)e[((size_t)l * (k + 1) + c) * N + t];
          for (uint32_t cc = 0; cc < k; cc++) add_product(N, mask.data() + (size_t)cc * N, glwe_key + (size_t)cc * N, body);
          if (lwe_key[i]) {  // plaintext -m g S_c (row c < k) / m g (row k)
            if (c < k)
              for (uint32_t t = 0; t < N; t++) body[t] -= g * glwe_key[(size_t)c * N + t];
            else
              body[0] += g;
          }
        }
      }
    });
  }
  if (ksk_bodies) {
    key_bytes(ksk_seed, key);
    const Aes128 aes(key);
    parallel_for((int64_t)k * N, [&](int64_t j) {
      std::vector<uint64_t> mask(n);
      std::vector<int64_t> e(p.ks_level);
      client::noise_words(rk, 0x100000 + (uint64_t)j, p.lwe_noise_log2, e.size(), e.data());
      for (uint32_t s = 0; s < p.ks_level; s++) {  // storage row s = engine level ks_level - 1 - s
        const size_t row = (size_t)j * p.ks_level + s;
        mask_words(aes, row * n, n, mask.data());
        uint64_t acc = (uint64_t)e[s] + (glwe_key[j] << (64 - p.ks_base_log * (p.ks_level - s)));
        for (uint32_t t = 0; t < n; t++) acc += mask[t] * lwe_key[t];
        ksk_bodies[row] = acc;
      }
    });
  }
}

void seeded_lwe_list(uint32_t dim, uint32_t count, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key& rk,
                     uint64_t stream0, const uint64_t seed[2], const uint64_t* msgs, uint64_t* bodies) {
  uint8_t kb[16];
  key_bytes(seed, kb);
  const Aes128 aes(kb);
  parallel_for((int64_t)count, [&](int64_t z) {
    std::vector<uint64_t> mask(dim);
    int64_t e;
    client::noise_words(rk, stream0 + (uint64_t)z, noise_log2, 1, &e);
    mask_words(aes, (uint64_t)z * dim, dim, mask.data());
    uint64_t acc = (uint64_t)e + (msgs ? msgs[z] : 0);
    for (uint32_t t = 0; t < dim; t++) acc += mask[t] * key[t];
    bodies[z] = acc;
  });
}

void decompress_bsk(const tfhe_params& p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* bsk) {
  const uint32_t k = p.k, N = p.N, L = p.pbs_level;
  const size_t row_len = (size_t)(k + 1) * N, per_i = (size_t)(k + 1) * L * row_len;
  uint8_t key[16];
  key_bytes(seed, key);
  const Aes128 aes(key);
  parallel_for((int64_t)p.n, [&](int64_t i) {
    for (uint32_t l = 0; l < L; l++)
      for (uint32_t c = 0; c <= k; c++) {
        const size_t row = ((size_t)i * L + l) * (k + 1) + c;
        uint64_t* out = bsk + per_i * i + row_len * (c * L + l);  // this engine's [i][c * L + l][j]
        mask_words(aes, row * k * N, (size_t)k * N, out);
        memcpy(out + (size_t)k * N, bodies + row * N, (size_t)N * 8);
      }
  });
}

void decompress_ksk(const tfhe_params& p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* ksk) {
  const uint32_t n = p.n;
  uint8_t key[16];
  key_bytes(seed, key);
  const Aes128 aes(key);
  parallel_for((int64_t)p.k * p.N, [&](int64_t j) {
    for (uint32_t s = 0; s < p.ks_level; s++) {  // storage row s (least significant first) -> engine row
      const size_t row = (size_t)j * p.ks_level + s;
      uint64_t* out = ksk + ((size_t)j * p.ks_level + (p.ks_level - 1 - s)) * (n + 1);
      mask_words(aes, row * n, n, out);
      out[n] = bodies[row];
    }
  });
}

void decompress_lwe_list(uint32_t dim, uint32_t count, const uint64_t seed[2], const uint64_t* bodies, uint64_t* out) {
  uint8_t key[16];
  key_bytes(seed, key);
  const Aes128 aes(key);
  parallel_for((int64_t)count, [&](int64_t z) {
    uint64_t* o = out + (size_t)z * (dim + 1);
    mask_words(aes, (uint64_t)z * dim, dim, o);
    o[dim] = bodies[z];
  });
}

}  // namespace seeded
}  // namespace tfhe
