/*
 * tfhe_hip.h — C ABI of libtfhe_hip.so, the MI355X-native TFHE programmable-bootstrap engine.
 *
 * This is the drop-in boundary for the reference's PBS path.  In the reference, JS callers reach
 * the TFHE core through packages/wasm (tfhe-rs 0.8.7 compiled to WASM/N-API, an empty submodule
 * here: .gitmodules:4, packages/pnpm-lock.yaml:1988-1995) and through the FHE server's
 * /evaluate endpoint (e2e/test/fhe.test.ts:105-175).  Each entry point below names the reference
 * interface it replaces.  Plain C: pointers + sizes, no torch / HIP types in signatures
 * (streams are passed as void*).
 *
 * Conventions
 *   - LWE ciphertexts: u64[dim + 1] = (a_0 .. a_{dim-1}, b), native torus Z_{2^64}.
 *   - GLWE / BSK values: Z_p, p = 2^64 - 2^32 + 1, canonical in [0, p) (transform 0, the NTT engine);
 *     native torus Z_{2^64} (transform 1, the FFT64 engine: tfhe-rs's own f64-FFT arithmetic).
 *   - BSK (standard domain): u64[n][(k+1)*l][k+1][N]; row index = c*l + lvl (c = component that
 *     carries s_i * 2^(64 - base_log*(lvl+1))), column = GLWE component (0..k-1 mask, k body).
 *   - KSK: u64[k*N][ks_level][n + 1], KSK[j][r] = LWE_s(s'_j * 2^(64 - ks_base_log*(r+1))).
 *   - LUT ("accumulator"): u64[N] in Z_p (see tfhe_hip_lut_*) for both transforms; the FFT64 engine
 *     maps each value back to the torus (x + round(x / 2^32), exact for Delta * m, Delta >= 2^32).
 *   - Every function returns 0 on success or a negative TFHE_HIP_E* code; it never aborts.
 *     tfhe_hip_last_error() returns the message of the last failure on the calling thread.
 *   - Ownership: the caller owns every host buffer; calls read/write them synchronously (the
 *     *_async variants take DEVICE pointers and enqueue on the given HIP stream).  The library
 *     owns device keys and workspaces (freed by tfhe_hip_destroy).
 *   - Threading: a ctx is not re-entrant; calls on one ctx are serialized by an internal mutex.
 */
#ifndef TFHE_HIP_H
#define TFHE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFHE_HIP_OK 0
#define TFHE_HIP_EINVAL (-1)      /* bad argument / size mismatch */
#define TFHE_HIP_ENOMEM (-2)      /* host or device allocation failed */
#define TFHE_HIP_EDEVICE (-3)     /* HIP runtime error */
#define TFHE_HIP_ENOKEYS (-4)     /* keys not loaded */
#define TFHE_HIP_EUNSUPPORTED (-5) /* parameter set not supported by the device kernels */

#define TFHE_HIP_PRESET_GATE 0   /* n=630 k=1 N=1024, PBS 7x3, KS 2x8 (TFHE 128-bit default) */
#define TFHE_HIP_PRESET_FHEVM 1  /* n=918 k=1 N=2048, PBS 23x1, KS 4x4 (PARAM_MESSAGE_2_CARRY_2_KS_PBS) */
#define TFHE_HIP_PRESET_GATE_FFT 2 /* P-GATE on the FFT64 transform (native-torus BSK, f64 FFT) */
#define TFHE_HIP_PRESET_FHEVM_FFT 3 /* P-FHEVM on the FFT64 transform (N = 2048 as two 512-point halves) */

#define TFHE_HIP_TRANSFORM_NTT 0   /* GLWE/BSK over Z_p, Goldilocks NTT (exact integer arithmetic) */
#define TFHE_HIP_TRANSFORM_FFT64 1 /* GLWE/BSK over Z_2^64, f64 FFT (tfhe-rs FFT64; oracle/fft_oracle.c) */

typedef struct tfhe_params {
  uint32_t n, k, N;
  uint32_t pbs_base_log, pbs_level;
  uint32_t ks_base_log, ks_level;
  int32_t lwe_noise_log2;  /* stddev as log2 of a torus fraction */
  int32_t glwe_noise_log2;
  uint32_t order;          /* 0 = PBS then KS (ciphertexts under the small key), 1 = KS then PBS */
  uint32_t transform;      /* TFHE_HIP_TRANSFORM_*: external-product arithmetic (and BSK domain) */
} tfhe_params;

typedef struct tfhe_ctx tfhe_ctx;

/* ---- parameters & sizes ------------------------------------------------------------------
 * Replaces the tfhe-rs parameter constants selected by name in sdk/relayer/src/tfhe.ts:14-19. */
int tfhe_hip_params_preset(int preset, tfhe_params* out);
size_t tfhe_hip_bsk_len(const tfhe_params* p);
size_t tfhe_hip_ksk_len(const tfhe_params* p);
/* LWE dimension of PBS inputs/outputs (n for order 0, k*N for order 1). */
uint32_t tfhe_hip_io_dim(const tfhe_params* p);

/* ---- client-side key material (host) ------------------------------------------------------
 * Replaces TfheClientKey.generate / ServerKey generation (sdk/relayer/src/tfhe.ts:20-28,
 * generateKeys.js:20-31).  All randomness is ChaCha20 keyed by a 192-bit rng key plus a stream index
 * (LWE key 1, GLWE key 2, BSK_i 0x1000+i, KSK_j 0x100000+j, MS zero z 0x200000+z, ciphertext q stream0+q).
 *   - tfhe_hip_rng_key_entropy: 192 bits from the OS (getrandom) -- production keys and encryptions;
 *   - tfhe_hip_rng_key_from_seed: (seed, a public tag) -- REPRODUCIBLE streams for tests, golden vectors
 *     and the oracle.  A seeded key set is public knowledge: never use one for real data.
 * The uint64_t-seed entry points below are the seeded (test) forms of the *_k functions. */
typedef struct tfhe_rng_key {
  uint32_t w[6];
} tfhe_rng_key;
int tfhe_hip_rng_key_entropy(tfhe_rng_key* out);
int tfhe_hip_rng_key_from_seed(uint64_t seed, tfhe_rng_key* out);
int tfhe_hip_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, uint64_t* lwe_key, uint64_t* glwe_key,
                      uint64_t* bsk /* nullable */, uint64_t* ksk /* nullable */);
int tfhe_hip_keygen(const tfhe_params* p, uint64_t seed, uint64_t* lwe_key, uint64_t* glwe_key,
                    uint64_t* bsk /* nullable */, uint64_t* ksk /* nullable */);
/* BSK / KSK (standard domain) for GIVEN binary secret keys — the server-key half of keygen, for key
 * material ingested from tfhe-rs (the packages/kms loader role, SURVEY §8f f3: the ClientKey of
 * sdk/relayer/src/test/keys/privateKey.bin; tfhe_amd/keyio.py parses it).  EINVAL if a key word is not 0/1. */
int tfhe_hip_server_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t* lwe_key,
                             const uint64_t* glwe_key, uint64_t* bsk /* nullable */, uint64_t* ksk /* nullable */);
int tfhe_hip_server_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, const uint64_t* glwe_key,
                           uint64_t* bsk /* nullable */, uint64_t* ksk /* nullable */);
/* Modulus-switch noise reduction key of the P-FHEVM server key (the
 * reference's parameter block carries modulus_switch_zeros_count 1449, ms_bound 2^58,
 * ms_r_sigma_factor 13.179852282053789, ms_input_variance 2.63039184094559e-07 —
 * sdk/relayer/src/test/keys/privateKey.bin @0x5e04..0x5e30).  count LWE encryptions of 0 under
 * the small key, count x (n+1) u64. */
#define TFHE_HIP_MS_FHEVM_ZEROS 1449u
#define TFHE_HIP_MS_FHEVM_BOUND 0x1p58
#define TFHE_HIP_MS_FHEVM_R_SIGMA 13.179852282053789
#define TFHE_HIP_MS_FHEVM_INPUT_VARIANCE 2.63039184094559e-07
int tfhe_hip_ms_zeros_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t* lwe_key, uint32_t count,
                               uint64_t* zeros);
int tfhe_hip_ms_zeros_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, uint32_t count,
                             uint64_t* zeros);
/* ---- compressed (seeded) server keys, SURVEY §8f f3 ---------------------------------------------
 * Replaces tfhe-rs core_crypto decompress_seeded_lwe_bootstrap_key / decompress_seeded_lwe_keyswitch_key /
 * decompress_seeded_lwe_ciphertext_list behind CompressedServerKey::decompress, the step by which the fhEVM
 * coprocessor turns a tenant's stored key into evaluation keys (tests/fhevm-suite/fhevm/docker-compose/
 * coprocessor-docker-compose.yml:96, --tenant-key-cache-size).  Masks come from the AES-128-CTR stream of a
 * 128-bit seed (seed[0] = low 64 bits) restated from tfhe-csprng (tfhe_amd/csrc/seeded.cpp has the byte order);
 * bodies are in tfhe-rs order:
 *   BSK bodies [i < n][l < L][c <= k][N]   (GGSW i, decomposition level l most significant first, GLWE row c)
 *   KSK bodies [j < k N][s < ks_level]     (input key element j, storage row s = decomposition level ks_level - s:
 *                                           least significant first, as tfhe-rs's keygen walks (1..=levels).rev();
 *                                           engine KSK row ks_level - 1 - s; P-FHEVM: big key -> small key)
 *   list bodies [z < count]                (e.g. the modulus-switch zeros)
 * Decompressed keys land in this engine's standard layouts (tfhe_hip_load_keys, tfhe_hip_load_ms_key).  FFT64
 * presets only (native 2^64 torus).  PARITY UNPINNED at the byte level: the reference holds no server-key file. */
int tfhe_hip_aes128_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]); /* FIPS-197 check */
int tfhe_hip_csprng_words(const uint64_t seed[2], uint64_t first_word, size_t count, uint64_t* out);
int tfhe_hip_seeded_server_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t bsk_seed[2],
                                    const uint64_t ksk_seed[2], const uint64_t* lwe_key, const uint64_t* glwe_key,
                                    uint64_t* bsk_bodies /* nullable */, uint64_t* ksk_bodies /* nullable */);
int tfhe_hip_seeded_lwe_list_k(uint32_t dim, uint32_t count, const uint64_t* key, int32_t noise_log2,
                               const tfhe_rng_key* rk, uint64_t stream0, const uint64_t seed[2],
                               const uint64_t* msgs /* nullable: encryptions of zero */, uint64_t* bodies);
int tfhe_hip_decompress_bsk(const tfhe_params* p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* bsk);
int tfhe_hip_decompress_ksk(const tfhe_params* p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* ksk);
int tfhe_hip_decompress_lwe_list(uint32_t dim, uint32_t count, const uint64_t seed[2], const uint64_t* bodies,
                                 uint64_t* out /* count x (dim + 1) */);
/* Encrypt count torus messages; ciphertext q uses ChaCha stream (stream0 + q) of the rng key (a fresh
 * entropy key per call, or one key with non-overlapping stream ranges).
 * Replaces the encrypt path of packages/luxfhejs/src/index.ts:127-141 (server-side /encrypt). */
int tfhe_hip_lwe_encrypt_k(uint32_t dim, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key* rk,
                           uint64_t stream0, const uint64_t* msgs, size_t count, uint64_t* out);
int tfhe_hip_lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, uint64_t seed,
                         uint64_t stream0, const uint64_t* msgs, size_t count, uint64_t* out);
/* phase = b - <a, s> (decryption before decoding); replaces /decrypt
 * (packages/hardhat-plugin/src/index.ts:71-75). */
int tfhe_hip_lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out);
/* LUT builders.  Replaces ServerKey::generate_accumulator (ml/biometrics/notebooks/main.rs:65-68). */
int tfhe_hip_lut_constant(uint32_t N, uint64_t torus_value, uint64_t* lut);
int tfhe_hip_lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* table, uint64_t delta_out,
                            uint64_t* lut);

/* ---- device engine ------------------------------------------------------------------------
 * One engine spans ndev device "shards" (SURVEY §8b/§8e).  Each shard owns a HIP stream, a copy of the
 * keys and its workspaces.  Host-buffer calls (tfhe_hip_pbs, tfhe_hip_nand) split a batch into
 * contiguous slices, one per shard, run concurrently (one host thread per shard) and return when all
 * are done; the outputs are in input order.  Keys are uploaded once to shard 0 (pinned staging) and
 * broadcast to the others: RCCL (ncclCommInitAll + ncclBroadcast over xGMI, librccl loaded on first use)
 * when the ordinals are distinct, device copies when an ordinal repeats (a one-GPU box can run
 * devices = {0, 0} to exercise the split).  TFHE_HIP_BCAST=rccl|copy overrides the choice.
 * Stage-level entry points (blind_rotate, sample_extract, keyswitch, ms_reduce, ntt_*, fft_*) run on
 * shard 0.  Replaces the CPU worker pool of the reference's FHE service
 * (coprocessor-docker-compose.yml:97 --coprocessor-fhe-threads=8). */
int tfhe_hip_create(const tfhe_params* p, const int* devices, int ndev, tfhe_ctx** out);
void tfhe_hip_destroy(tfhe_ctx* ctx);
const char* tfhe_hip_last_error(void);
int tfhe_hip_device(const tfhe_ctx* ctx);          /* device of shard 0 */
int tfhe_hip_ndev(const tfhe_ctx* ctx);            /* number of shards */
int tfhe_hip_device_at(const tfhe_ctx* ctx, int i); /* device of shard i, -1 if out of range */
/* How the last key load reached shards 1..ndev-1: 0 = single shard, 1 = device copies, 2 = RCCL. */
int tfhe_hip_key_bcast_mode(const tfhe_ctx* ctx);
/* The key-load broadcast planner behind tfhe_hip_load_keys (host logic only, no device is touched), so the
 * N-rank call structure is testable without N GPUs.  policy: "rccl", "copy" or NULL / "" = auto (RCCL when
 * the ordinals are distinct and librccl is available, device / peer copies otherwise).  *mode as
 * tfhe_hip_key_bcast_mode.  mode 2: calls[i] = the rank issuing the i-th ncclBroadcast inside one
 * ncclGroupStart / ncclGroupEnd (root 0 first); mode 1: calls[i] = destination shard of the i-th copy from
 * shard 0.  Returns the number of calls (<= max_calls) or a negative error code. */
int tfhe_hip_bcast_plan(const int* devices, int ndev, const char* policy, int rccl_available, int* mode, int* calls,
                        int max_calls);

/* Upload standard-domain BSK and KSK from host memory through a pinned staging ring to shard 0,
 * broadcast them to every other shard, and convert them on each device (BSK to the transform domain,
 * KSK to the matrix-core byte planes).  Replaces the packages/kms key-loader role (pinned-HBM key
 * residency). */
int tfhe_hip_load_keys(tfhe_ctx* ctx, const uint64_t* bsk, size_t bsk_len, const uint64_t* ksk, size_t ksk_len);
/* Same, from DEVICE buffers on shard 0's device (e.g. after a torch.distributed broadcast of the keys). */
int tfhe_hip_load_keys_device(tfhe_ctx* ctx, const uint64_t* d_bsk, size_t bsk_len, const uint64_t* d_ksk,
                              size_t ksk_len);

/* Enable the modulus-switch noise reduction between keyswitch and blind rotation (order 1 only;
 * count = 0 disables).  Before each blind rotation the ciphertext gets the one zero whose
 * measure |E[err]| + r_sigma * sd(err) of the switch to 2N is best (tfhe-rs 1.x
 * improve_lwe_ciphertext_modulus_switch_noise_for_binary_key; exact rule in oracle/tfhe_oracle.h).
 * EUNSUPPORTED for order 0 parameter sets. */
int tfhe_hip_load_ms_key(tfhe_ctx* ctx, const uint64_t* zeros, uint32_t count, double bound, double r_sigma,
                         double input_variance);
/* Stage-level: the reduction alone on B small-key ciphertexts (B x (n+1)); picks (nullable, B
 * entries) receives the chosen zero index or -1. */
int tfhe_hip_ms_reduce(tfhe_ctx* ctx, const uint64_t* lwe_small, size_t B, uint64_t* out, int32_t* picks);

/* Full PBS of B ciphertexts: order 0 = blind-rotate -> sample-extract -> keyswitch.
 * luts: n_lut LUTs of N values; lut_index (nullable, B entries) picks the LUT per ciphertext.
 * Replaces ServerKey::keyswitch_programmable_bootstrap (ml/biometrics/notebooks/main.rs:71) and
 * the compute behind POST /evaluate (e2e/test/fhe.test.ts:141-157).  Host buffers, synchronous. */
int tfhe_hip_pbs(tfhe_ctx* ctx, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                 const uint32_t* lut_index, uint64_t* lwe_out);
/* Device buffers, enqueued on `stream` (hipStream_t; NULL = the shard's stream, TFHE_HIP_NULL_STREAM = the
 * device's legacy null stream, e.g. torch's default stream).  Inputs resident in HBM, on the device of the
 * shard that runs the batch: the first shard whose device holds d_lwe_in.  Calls on different streams
 * are ordered on the shard's workspaces by an event (a later call waits for the previous one's kernels). */
#define TFHE_HIP_NULL_STREAM ((void*)(intptr_t)-1)
int tfhe_hip_pbs_async(tfhe_ctx* ctx, const uint64_t* d_lwe_in, size_t B, const uint64_t* d_luts, size_t n_lut,
                       const uint32_t* d_lut_index, uint64_t* d_lwe_out, void* stream);

/* Stage-level entry points (host buffers) used by the parity tests. */
/* acc_out: B x (k+1) x N values in the GLWE ring (Z_p for NTT, torus for FFT64) after the CMUX loop. */
int tfhe_hip_blind_rotate(tfhe_ctx* ctx, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                          const uint32_t* lut_index, uint64_t* acc_out);
/* acc (Z_p, B x (k+1)N) -> LWE under the GLWE key, converted to 2^64: B x (kN + 1). */
int tfhe_hip_sample_extract(tfhe_ctx* ctx, const uint64_t* acc, size_t B, uint64_t* lwe_big_out);
/* B x (kN+1) -> B x (n+1). */
int tfhe_hip_keyswitch(tfhe_ctx* ctx, const uint64_t* lwe_big, size_t B, uint64_t* lwe_small_out);
/* Negacyclic NTT over Z_p of count polynomials of size N, in place, natural order:
 * A[j] = a(psi^(2j+1)), psi the primitive 2N-th root with psi^(2N/64) = 8.  ntt_inv includes 1/N. */
int tfhe_hip_ntt_fwd(tfhe_ctx* ctx, uint64_t* polys, size_t count);
int tfhe_hip_ntt_inv(tfhe_ctx* ctx, uint64_t* polys, size_t count);

/* FFT64 transform (N = 1024), natural order, for parity tests of the device FFT against
 * oracle/fft_oracle.c: fwd reads count x N torus values as int64, writes count x N/2 complex (re, im
 * doubles); inv reads count x N/2 complex and writes count x N doubles (no 1/M, no rounding).
 * EUNSUPPORTED unless the ctx was created with transform = TFHE_HIP_TRANSFORM_FFT64. */
int tfhe_hip_fft_fwd(tfhe_ctx* ctx, const uint64_t* polys, size_t count, double* out);
int tfhe_hip_fft_inv(tfhe_ctx* ctx, const double* in, size_t count, double* out);

/* Gate bootstrapping (FheBool NAND): out = PBS((0, 1/8) - c1 - c2, LUT == 1/8), B gates. */
int tfhe_hip_nand(tfhe_ctx* ctx, const uint64_t* c1, const uint64_t* c2, size_t B, uint64_t* out);

/* Batches of at most max_batch ciphertexts run the latency blind-rotate kernel (one ciphertext per
 * workgroup: 4.5x (N=1024) / 2.5x (N=2048) lower PBS latency — the lockstep levels of integer
 * circuits, single /evaluate requests, packages/luxfhejs/src/index.ts:56-141 call patterns); larger
 * batches the throughput kernel.  Defaults = the measured crossovers on MI355X (tools/latency_sweep.py,
 * tools/latency_sweep_fft.sh): NTT engine 1024 for N=1024 (55 vs 61 ms at B=1024, 69 vs 62 at 1280),
 * 512 for N=2048 (42 vs 53 ms at 512, 63 vs 53 at 768); FFT64 engine 512 for both N (PBS with the
 * latency kernel: 3.9 / 7.9 ms at N=1024 for up to 256 / 512 ciphertexts, 5.7 / 11.3 ms at N=2048;
 * batch kernel 14.5-15.5 ms up to 2048 ciphertexts at N=1024, 15.3-16.0 ms up to 1024 at N=2048);
 * 0 disables the latency kernel. */
int tfhe_hip_set_latency_batch(tfhe_ctx* ctx, size_t max_batch);
/* Name of the blind-rotate kernel the dispatch launches for a per-shard batch of `batch` ciphertexts under
 * the current latency threshold (e.g. "blind_rotate_fft_pair_kernel"), or NULL for a null ctx.  No reference
 * counterpart: a measurement aid, so a profile is matched to the kernel that actually ran (bench.py). */
const char* tfhe_hip_br_kernel(const tfhe_ctx* ctx, size_t batch);
/* Wait for all work on the ctx stream. */
int tfhe_hip_sync(tfhe_ctx* ctx);
/* Per-kernel device timing (HIP events recorded on the launch stream around every blind-rotate /
 * keyswitch launch).  reset clears the record; stats waits for the recorded events and returns the
 * summed milliseconds and the launch count.  which: 0 = blind rotate (+sample extract), 1 = keyswitch,
 * 2 = modulus-switch noise reduction.
 * Used by bench.py for the roofline figure. */
int tfhe_hip_timing_enable(tfhe_ctx* ctx, int enable);
int tfhe_hip_timing_reset(tfhe_ctx* ctx);
int tfhe_hip_timing_stats(tfhe_ctx* ctx, int which, double* total_ms, int* launches);

/* ---- LWE -> GLWE packing keyswitch and ciphertext compression ---------------
 * Replaces the reference's compression of result ciphertexts (ml/extensions/rust/src/compression.rs:
 * cpu_compress_ciphertexts_into_list :246-291 / cuda_compress_ciphertexts_into_single_glwe :190-240 ->
 * tfhe-rs par_keyswitch_lwe_ciphertext_list_and_pack_in_glwe_ciphertext, then
 * CompressedModulusSwitchedGlweCiphertext::compress; extract :134-156).  Up to lwe_per_glwe LWEs
 * (dimension in_dim, native 2^64) are keyswitched into the coefficients 0, 1, ... of one GLWE
 * (k = out_k, N = out_N) under a fresh binary GLWE key; compression switches every stored coefficient
 * to storage_log bits and bit-packs them.  Exact rule: oracle/tfhe_oracle.h (or_pks_params). */
typedef struct tfhe_pks_params {
  uint32_t in_dim, out_k, out_N, base_log, level, lwe_per_glwe, storage_log;
  int32_t noise_log2;
} tfhe_pks_params;
/* PARAMS_8B_2048_NEW (ml/extensions/rust/src/fhext_classes.rs:98-112): in 2048, pks 2 x 2^14,
 * out k=1 N=2048, lwe_per_glwe 2048, storage 26 bits, noise 2^-48 */
#define TFHE_HIP_PKS_PRESET_ML2048 0
int tfhe_hip_pks_params_preset(int preset, tfhe_pks_params* out);
size_t tfhe_hip_pksk_len(const tfhe_pks_params* pp); /* in_dim * level * (out_k+1) * out_N u64 */
/* output GLWE key (out_k*out_N bits, ChaCha stream 4) and PKSK [j][l][(k+1)N] (stream 0x300000+j) */
int tfhe_hip_pks_keygen(const tfhe_pks_params* pp, uint64_t seed, const uint64_t* in_key, uint64_t* out_key,
                        uint64_t* pksk /* nullable */);
/* the same from a 192-bit rng key (tfhe_hip_rng_key_entropy for production keys; the seeded form above
 * is tfhe_hip_rng_key_from_seed(seed) and exists for reproducible tests) */
int tfhe_hip_pks_keygen_k(const tfhe_pks_params* pp, const tfhe_rng_key* rk, const uint64_t* in_key,
                          uint64_t* out_key, uint64_t* pksk /* nullable */);
typedef struct tfhe_pks_ctx tfhe_pks_ctx;
int tfhe_hip_pks_create(const tfhe_pks_params* pp, int device, tfhe_pks_ctx** out);
void tfhe_hip_pks_destroy(tfhe_pks_ctx* ctx);
int tfhe_hip_pks_load_key(tfhe_pks_ctx* ctx, const uint64_t* pksk, size_t len);
/* count LWEs (count x (in_dim+1)) -> ceil(count / lwe_per_glwe) GLWEs ((k+1) x N each); GLWE g holds
 * LWEs g*lwe_per_glwe ... in coefficients 0, 1, ...  Host buffers, synchronous. */
int tfhe_hip_pks_pack(tfhe_pks_ctx* ctx, const uint64_t* lwes, size_t count, uint64_t* glwes);
/* Device buffers, enqueued on `stream` (NULL = the ctx stream, TFHE_HIP_NULL_STREAM = the null stream). */
int tfhe_hip_pks_pack_async(tfhe_pks_ctx* ctx, const uint64_t* d_lwes, size_t count, uint64_t* d_glwes, void* stream);
size_t tfhe_hip_pks_packed_words(const tfhe_pks_params* pp, uint32_t bodies);
int tfhe_hip_pks_compress(const tfhe_pks_params* pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed);
int tfhe_hip_pks_extract(const tfhe_pks_params* pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe);
/* client-side decryption of a native GLWE: body - sum_c mask_c * S_c (N values) */
int tfhe_hip_glwe_phase(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out);

/* ---- switch-and-squash: noise squashing to a 128-bit LWE ----------------------
 * fhEVM's sns-worker (coprocessor-docker-compose.yml:124-140) turns each 64-bit P-FHEVM ciphertext into
 * a Z_2^128 LWE with tiny noise for threshold decryption: keyswitch to the small key, modulus-switch
 * noise reduction (tfhe_hip_ms_reduce), then a PBS with a BSK under a 128-bit GLWE key (k=2, N=2048,
 * 2^24 x 3) and the identity LUT.  The GLWE ring is the native 2^128 torus (as tfhe-rs): a coefficient
 * is one u128 word, a polynomial two u64 planes [lo][N], [hi][N]; rule: oracle/sns_oracle.c.
 * Output: (k*N + 1) x (lo, hi) u64 per ciphertext. */
typedef struct tfhe_sns_params {
  uint32_t n, k, N, base_log, level;
  int32_t noise_log2; /* Gaussian noise round(N(0,1) * 2^(64 + x)) on the 128-bit bodies */
} tfhe_sns_params;
#define TFHE_HIP_SNS_PRESET_FHEVM 0 /* n = 918 (P-FHEVM small key), k = 2, N = 2048, 2^24 x 3, noise 2^30 */
int tfhe_hip_sns_params_preset(int preset, tfhe_sns_params* out);
size_t tfhe_hip_sns_bsk_len(const tfhe_sns_params* sp); /* n*(k+1)L*(k+1)*2*N: [i][c*L+l][j][lo, hi][N] */
/* 128-bit GLWE key (k*N bits, ChaCha stream 5) and BSK (stream 0x400000 + i) for the small LWE key */
int tfhe_hip_sns_keygen(const tfhe_sns_params* sp, uint64_t seed, const uint64_t* lwe_key, uint64_t* glwe_key,
                        uint64_t* bsk /* nullable */);
/* the same from a 192-bit rng key (OS entropy for production keys) */
int tfhe_hip_sns_keygen_k(const tfhe_sns_params* sp, const tfhe_rng_key* rk, const uint64_t* lwe_key,
                          uint64_t* glwe_key, uint64_t* bsk /* nullable */);
typedef struct tfhe_sns_ctx tfhe_sns_ctx;
int tfhe_hip_sns_create(const tfhe_sns_params* sp, int device, tfhe_sns_ctx** out);
void tfhe_hip_sns_destroy(tfhe_sns_ctx* ctx);
/* Loading rounds every key word (read as a signed 128-bit integer) to the nearest multiple of 2^16
 * (oracle: or_sns_bsk_round; ~2^20 of extra phase noise beside the key's 2^30).  The external product
 * splits the rounded key into seven 16-bit limbs and computes each digit x limb convolution as an
 * exact f64 FFT product (n x 9 x 3 x 7 x 1024 complex of key spectra: 2.8 GB at n = 918). */
int tfhe_hip_sns_load_key(tfhe_sns_ctx* ctx, const uint64_t* bsk, size_t len);
/* B small-key ciphertexts (B x (n+1)) -> B x (k*N+1) x 2 u64; identity LUT over msg_modulus values */
int tfhe_hip_sns_squash(tfhe_sns_ctx* ctx, const uint64_t* lwe_small, size_t B, uint32_t msg_modulus, uint64_t* out);
int tfhe_hip_sns_squash_async(tfhe_sns_ctx* ctx, const uint64_t* d_lwe_small, size_t B, uint32_t msg_modulus,
                              uint64_t* d_out, void* stream);
/* stage-level (parity tests): accumulator after the CMUX loop, B x (k+1) x (lo, hi) x N words */
int tfhe_hip_sns_blind_rotate(tfhe_sns_ctx* ctx, const uint64_t* lwe_small, size_t B, uint32_t msg_modulus,
                              uint64_t* acc_out);
/* client: phase b - <a, s> mod 2^128 of count squashed ciphertexts -> (lo, hi) pairs */
int tfhe_hip_sns_phase(const tfhe_sns_params* sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count,
                       uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
