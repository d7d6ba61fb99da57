// client.h — host-side key material (see client.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/tfhe_hip.h"

namespace tfhe {
namespace client {
tfhe_rng_key rng_key_from_seed(uint64_t seed);
bool rng_key_entropy(tfhe_rng_key* k);  // getrandom(2), 192 bits
size_t bsk_len(const tfhe_params& p);
size_t ksk_len(const tfhe_params& p);
void keygen(const tfhe_params& p, const tfhe_rng_key& rk, uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk, uint64_t* ksk);
// BSK / KSK for given binary secret keys (e.g. an ingested tfhe-rs ClientKey); same streams as keygen
void server_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t* lwe_key, const uint64_t* glwe_key,
                   uint64_t* bsk, uint64_t* ksk);
// P-FHEVM modulus-switch zeros: count LWE encryptions of 0 under the small key, count x (n+1)
void ms_zeros_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t* lwe_key, uint32_t count, uint64_t* zeros);
void lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key& rk, uint64_t stream0,
                 const uint64_t* msgs, size_t count, uint64_t* out);
void lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out);
void noise_words(const tfhe_rng_key& rk, uint64_t stream, int32_t log2_sigma, size_t count, int64_t* out);
void lut_constant(uint32_t N, uint64_t torus_value, uint64_t* lut);
void lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* table, uint64_t delta, uint64_t* lut);
// packing keyswitch (LWE list -> GLWE) key and ciphertext compression
size_t pksk_len(const tfhe_pks_params& pp);
void pks_keygen(const tfhe_pks_params& pp, const tfhe_rng_key& rk, const uint64_t* in_key, uint64_t* out_key, uint64_t* pksk);
void glwe_phase_native(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out);
size_t pks_packed_words(const tfhe_pks_params& pp, uint32_t bodies);
void pks_compress(const tfhe_pks_params& pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed);
void pks_extract(const tfhe_pks_params& pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe);
// noise squashing (128-bit GLWE over the native 2^128 torus, words as (lo, hi) planes)
size_t sns_bsk_len(const tfhe_sns_params& sp);
void sns_keygen(const tfhe_sns_params& sp, const tfhe_rng_key& rk, const uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk);
void sns_lut_identity(const tfhe_sns_params& sp, uint32_t msg_modulus, uint64_t* lut);
void sns_phase(const tfhe_sns_params& sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count, uint64_t* out);
}  // namespace client

// compressed (seeded) server keys (seeded.cpp)
namespace seeded {
void aes128_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]);
void csprng_words(const uint64_t seed[2], uint64_t first, size_t count, uint64_t* out);
void seeded_server_keygen(const tfhe_params& p, const tfhe_rng_key& rk, const uint64_t bsk_seed[2],
                          const uint64_t ksk_seed[2], const uint64_t* lwe_key, const uint64_t* glwe_key,
                          uint64_t* bsk_bodies, uint64_t* ksk_bodies);
void seeded_lwe_list(uint32_t dim, uint32_t count, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key& rk,
                     uint64_t stream0, const uint64_t seed[2], const uint64_t* msgs, uint64_t* bodies);
void decompress_bsk(const tfhe_params& p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* bsk);
void decompress_ksk(const tfhe_params& p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* ksk);
void decompress_lwe_list(uint32_t dim, uint32_t count, const uint64_t seed[2], const uint64_t* bodies, uint64_t* out);
}  // namespace seeded
}  // namespace tfhe
