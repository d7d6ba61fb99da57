// AddressSanitizer + UndefinedBehaviorSanitizer run of the HOST code (SURVEY §5 aux: memory checking):
// the product's client-side key material (tfhe_amd/csrc/client.cpp: ChaCha streams, keygen, server keys,
// MS zeros, encryption, phase, LUT builders, packing key, compression, squashing key) and the CPU oracle
// (oracle/*.c: keygen, NTT and FFT64 blind rotations, keyswitch, full PBS of both parameter sets, MS
// reduction, the native 2^128 squash blind rotation).
// Built by `make -C oracle san` into oracle/_san/ (test infrastructure; no GPU code: GPU sanitizers are
// unavailable on the pool).  Also cross-checks that client and oracle draw identical keys.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/tfhe_hip.h"
#include "../../oracle/tfhe_oracle.h"
#include "../../tfhe_amd/csrc/client.h"

using namespace tfhe;

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                     \
    }                                                              \
  } while (0)

static void run_preset(int preset) {
  tfhe_params p{};
  or_params q{};
  or_params_preset(preset, &q);
  static_assert(sizeof(tfhe_params) == sizeof(or_params), "params layouts");
  memcpy(&p, &q, sizeof(p));
  const uint64_t seed = 0x7F4E0001;
  const size_t bl = client::bsk_len(p), kl = client::ksk_len(p);
  CHECK(bl == or_bsk_len(&q) && kl == or_ksk_len(&q));
  std::vector<uint64_t> lwe(p.n), glwe((size_t)p.k * p.N), bsk(bl), ksk(kl);
  std::vector<uint64_t> olwe(p.n), oglwe((size_t)p.k * p.N), obsk(bl), oksk(kl);
  const tfhe_rng_key rk = client::rng_key_from_seed(seed);
  client::keygen(p, rk, lwe.data(), glwe.data(), bsk.data(), ksk.data());
  or_keygen(&q, seed, olwe.data(), oglwe.data(), obsk.data(), oksk.data());
  CHECK(lwe == olwe && glwe == oglwe && bsk == obsk && ksk == oksk);
  tfhe_rng_key ek;
  CHECK(client::rng_key_entropy(&ek));
  // encryption through the product code, PBS through the oracle, decryption through the product code
  const uint32_t dim = p.order == 0 ? p.n : p.k * p.N;
  const uint64_t* key = p.order == 0 ? lwe.data() : glwe.data();
  const int32_t noise = p.order == 0 ? p.lwe_noise_log2 : p.glwe_noise_log2;
  const int B = 3, mm = p.order == 0 ? 2 : 16;
  std::vector<uint64_t> msgs(B), cts((size_t)B * (dim + 1)), out((size_t)B * (dim + 1)), ph(B);
  const uint64_t delta = p.order == 0 ? (1ull << 61) : (1ull << 63) / 16;
  for (int i = 0; i < B; i++) msgs[i] = p.order == 0 ? ((i & 1) ? delta : 0 - delta) : (uint64_t)(3 * i + 1) * delta;
  client::lwe_encrypt(dim, key, noise, ek, 0, msgs.data(), B, cts.data());
  std::vector<uint64_t> table(mm), lut(p.N);
  for (int m = 0; m < mm; m++) table[m] = (uint64_t)m;
  if (p.order == 0) client::lut_constant(p.N, 1ull << 61, lut.data());
  else client::lut_from_table(p.N, mm, table.data(), delta, lut.data());
  std::vector<uint64_t> zeros;
  or_ms_key ms{};
  if (p.order == 1) {
    zeros.resize((size_t)TFHE_HIP_MS_FHEVM_ZEROS * (p.n + 1));
    client::ms_zeros_keygen(p, rk, lwe.data(), TFHE_HIP_MS_FHEVM_ZEROS, zeros.data());
    ms.zeros = zeros.data();
    ms.count = TFHE_HIP_MS_FHEVM_ZEROS;
    ms.bound = TFHE_HIP_MS_FHEVM_BOUND;
    ms.r_sigma = TFHE_HIP_MS_FHEVM_R_SIGMA;
    ms.input_variance = TFHE_HIP_MS_FHEVM_INPUT_VARIANCE;
  }
  if (q.transform == 1) {
    std::vector<or_c64> bf(bl / 2);
    or_bsk_to_fourier(&q, bsk.data(), bf.data());
    or_pbs_batch_fft_ex(&q, bf.data(), ksk.data(), p.order == 1 ? &ms : nullptr, cts.data(), B, lut.data(), 1,
                        nullptr, out.data(), 1);
    // the SIMD port (fft_batch.c) on the same inputs at both widths: bit-identical outputs
    for (const char* lanes : {"4", "8"}) {
      setenv("ORACLE_SIMD_LANES", lanes, 1);
      if (lanes[0] == '8' && or_fft_batch_lanes() != 8) continue;
      std::vector<uint64_t> out2(out.size());
      CHECK(or_pbs_batch_fft_simd_ex(&q, bf.data(), ksk.data(), p.order == 1 ? &ms : nullptr, cts.data(), B,
                                     lut.data(), 1, nullptr, out2.data(), 2) == 0);
      CHECK(out2 == out);
    }
    unsetenv("ORACLE_SIMD_LANES");
  } else {
    std::vector<uint64_t> bn(bl);
    or_bsk_to_ntt(&q, bsk.data(), bn.data());
    or_pbs_batch_ex(&q, bn.data(), ksk.data(), p.order == 1 ? &ms : nullptr, cts.data(), B, lut.data(), 1, nullptr,
                    out.data(), 1);
  }
  client::lwe_phase(dim, key, out.data(), B, ph.data());
  for (int i = 0; i < B; i++) {
    const uint64_t want = msgs[i];  // gate LUT == 1/8: sign(phase) * 1/8; P-FHEVM: the identity table
    const int64_t err = (int64_t)(ph[i] - want);
    CHECK(err < (int64_t)(delta / 2) && err > -(int64_t)(delta / 2));
  }
  printf("preset %d: keys == oracle, %d PBS decrypt\n", preset, B);
}

int main() {
  for (int preset : {0, 2, 3}) run_preset(preset);
  // packing key + compression round trip on the client side
  tfhe_pks_params pp{2048, 1, 2048, 14, 2, 2048, 26, -48};
  std::vector<uint64_t> in_key(pp.in_dim), out_key((size_t)pp.out_k * pp.out_N);
  for (uint32_t i = 0; i < pp.in_dim; i++) in_key[i] = (i * 7) & 1;
  client::pks_keygen(pp, client::rng_key_from_seed(5), in_key.data(), out_key.data(), nullptr);
  std::vector<uint64_t> glwe((size_t)(pp.out_k + 1) * pp.out_N), back(glwe.size());
  for (size_t i = 0; i < glwe.size(); i++) glwe[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
  std::vector<uint64_t> packed(client::pks_packed_words(pp, 7));
  client::pks_compress(pp, glwe.data(), 7, packed.data());
  client::pks_extract(pp, packed.data(), 7, back.data());
  // noise squashing at a reduced input dimension: client key words == oracle key words, the identity LUT,
  // the oracle's native 2^128 blind rotation (key rounding, limb NTTs, 128-bit decomposition) and phase
  {
    or_sns_params osp{};
    or_sns_params_preset(0, &osp);
    osp.n = 3;
    tfhe_sns_params sp{osp.n, osp.k, osp.N, osp.base_log, osp.level, osp.noise_log2};
    std::vector<uint64_t> lk = {1, 0, 1}, g1((size_t)sp.k * sp.N), g2(g1.size());
    std::vector<uint64_t> b1(client::sns_bsk_len(sp)), b2(or_sns_bsk_len(&osp));
    CHECK(b1.size() == b2.size());
    client::sns_keygen(sp, client::rng_key_from_seed(0x5A5), lk.data(), g1.data(), b1.data());
    or_sns_keygen(&osp, 0x5A5, lk.data(), g2.data(), b2.data());
    CHECK(g1 == g2 && b1 == b2);
    std::vector<uint64_t> l1(2 * (size_t)sp.N), l2(l1.size());
    client::sns_lut_identity(sp, 16, l1.data());
    or_sns_lut_identity(&osp, 16, l2.data());
    CHECK(l1 == l2);
    std::vector<uint64_t> rounded(b2.size()), limb(or_sns_limb_ntt_len(&osp));
    or_sns_bsk_round(&osp, b2.data(), rounded.data());
    or_sns_bsk_to_limb_ntt(&osp, rounded.data(), limb.data());
    std::vector<uint64_t> small(osp.n + 1), acc((size_t)(osp.k + 1) * 2 * osp.N), out(2 * ((size_t)osp.k * osp.N + 1));
    for (size_t i = 0; i < small.size(); i++) small[i] = 0x9E3779B97F4A7C15ull * (i + 1);
    or_sns_blind_rotate(&osp, limb.data(), small.data(), l2.data(), acc.data());
    or_sns_sample_extract(&osp, acc.data(), out.data());
    uint64_t p1[2], p2[2];
    client::sns_phase(sp, g1.data(), out.data(), 1, p1);
    or_sns_phase(&osp, g2.data(), out.data(), 1, p2);
    CHECK(p1[0] == p2[0] && p1[1] == p2[1]);
    printf("squash keys == oracle, native blind rotation clean\n");
  }
  printf(fails ? "SANITIZE FAIL %d\n" : "SANITIZE OK\n", fails);
  return fails ? 1 : 0;
}
