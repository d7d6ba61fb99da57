// pbs_kernels.h — launchers of the gfx950 PBS kernels (pbs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "gl64.h"

namespace tfhe {
// 4 x 1024 twiddle tables of the device NTT layout, for the canonical psi (psi^32 = 8).
void make_ntt_tables(u64 psi, u64* tw);
hipError_t launch_bsk_to_ntt(const u64* bsk_std, u64* bsk_ntt, int n, const u64* tw, u64 ninv, hipStream_t s);
// batches of at most latency_max_batch ciphertexts use the latency kernel (one ciphertext per
// workgroup); larger ones the batch kernel (8 ciphertexts per workgroup)
hipError_t launch_blind_rotate(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index, int n_lut,
                               const u64* bsk, const u64* tw, u64* out_big, u64* out_acc, hipStream_t s,
                               size_t latency_max_batch = 0);
hipError_t launch_sample_extract(const u64* acc, size_t B, u64* out, hipStream_t s);
hipError_t launch_keyswitch(const u64* in_big, size_t B, int big_dim, const u64* ksk, int n, int base_log, int levels,
                           u64* out, hipStream_t s);
hipError_t launch_ntt_fwd(u64* polys, size_t count, const u64* tw, hipStream_t s);
hipError_t launch_ntt_inv(u64* polys, size_t count, const u64* tw, u64 ninv, hipStream_t s);
// keyswitch as eight int8 GEMMs on the matrix cores (ks_mfma.hip): KSK byte planes built once per key
// load, digits staged in a workspace of ks_digits_bytes(B, ...) bytes
size_t ks_planes_bytes(int big_dim, int levels, int n);
size_t ks_digits_bytes(size_t B, int big_dim, int levels);
hipError_t launch_ksk_planes(const u64* ksk, int big_dim, int levels, int n, void* planes, hipStream_t s);
hipError_t launch_keyswitch_mfma(const u64* in_big, size_t B, int big_dim, const void* planes, int n, int base_log,
                                 int levels, void* digits, u64* out, hipStream_t s);

// FFT64 transform (pbs_fft.hip), N = 1024: tables = 1536 complex (twist | pass A | pass B);
// Fourier BSK = polys x 512 complex
size_t fft_tables_len();  // doubles
void make_fft_tables(double* tw);
bool fft_slot_constants_ok();  // the N = 1024 kernels' compile-time twist constants == the host tables
hipError_t launch_bsk_to_fourier(const u64* bsk_std, double* bsk_f, size_t polys, const double* tw, hipStream_t s);
// batches of at most latency_max_batch ciphertexts use the latency kernel (one ciphertext per workgroup)
hipError_t launch_blind_rotate_fft(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                   int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                   hipStream_t s, size_t latency_max_batch = 0);
hipError_t launch_sample_extract_torus(const u64* acc, size_t B, u64* out, hipStream_t s);
hipError_t launch_fft_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s);
hipError_t launch_fft_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s);
// FFT64 transform, N = 2048, one wave per polynomial (pbs_fft2k.hip, fft1k.h): table = pass A [16][64] |
// pass B [4][16] (complex)
size_t fft2k_tables_len();  // doubles
void make_fft2k_tables(double* tw);
bool fft2k_slot_constants_ok();
hipError_t launch_bsk_to_fourier2k(const u64* bsk_std, double* bsk_f, size_t polys, const double* tw, hipStream_t s);
hipError_t launch_blind_rotate_fft2k(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                     int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                     hipStream_t s, size_t latency_max_batch);
hipError_t launch_sample_extract_torus2k(const u64* acc, size_t B, u64* out, hipStream_t s);
hipError_t launch_fft2k_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s);
hipError_t launch_fft2k_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s);

// N = 2048 (P-FHEVM, pbs_n2048.hip): tables = [1024-point tables of psi^2 (4096) | combine
// twiddles psi^(2j+1) (2048) | inverses (2048)]
void make_ntt2048_tables(u64 psi, u64* tw);
size_t ntt2048_tables_len();
hipError_t launch_bsk_to_ntt_2048(const u64* bsk_std, u64* bsk_ntt, size_t polys, const u64* tw, u64 ninv,
                                  hipStream_t s);
hipError_t launch_blind_rotate_2048(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                   int n_lut, const u64* bsk, const u64* tw, u64* out_big, u64* out_acc,
                                   hipStream_t s, size_t latency_max_batch = 0);
hipError_t launch_sample_extract_2048(const u64* acc, size_t B, u64* out, hipStream_t s);
hipError_t launch_ntt2048_fwd(u64* polys, size_t count, const u64* tw, hipStream_t s);
// noise squashing on the native 2^128 torus (sns.hip; sns_fft.h): d_fconst = device copy of
// make_sns_fft_const(); words as (lo, hi) planes per polynomial
size_t sns_fft_const_bytes();
void make_sns_fft_const(void* out);
size_t sns_fft_key_len(size_t n);  // key limb spectra, in 16-byte complex
size_t sns_digit_len(size_t B);    // digit spectra workspace, in 16-byte complex
size_t sns_fft_prod_len(size_t B);  // MAC product workspace, in 16-byte complex
constexpr size_t SNS_FFT_POLY_BYTES = 5 * 1024 * 16;  // limb spectra of one (i, r, j) key polynomial (sns_fft.h SF_LIMBS)
hipError_t launch_sns_bsk_to_fft(const u64* bsk_std, void* bsk_fft, size_t polys, const void* d_fconst,
                                 hipStream_t s);
hipError_t launch_sns_blind_rotate(const u64* lwe, size_t B, int n, const u64* lut, const void* bsk_fft, u64* acc,
                                   void* D, void* Oprod, const void* d_fconst, hipStream_t s);
hipError_t launch_sns_extract(const u64* acc, size_t B, u64* out, hipStream_t s);
// packing keyswitch (pks.hip)
hipError_t launch_pks_corr(const u64* pksk, int K, int Nc, int base_log, u64* corr, hipStream_t s);
hipError_t launch_pks_pack(const u64* lwes, size_t count, int in_dim, int base_log, int L, int k, int N, int lpg,
                           const u64* pksk, const u64* corr, u32* A, u64* T, u64* out, hipStream_t s);
// the same on the matrix cores (ks_mfma.hip): the GEMM, then pks.hip's shift-and-sum
size_t pks_mfma_rows(size_t count);
hipError_t launch_pks_gemm_mfma(const u64* lwes, size_t count, int in_dim, int base_log, int LV, int Nc,
                                const void* planes, void* A0, void* A1, u64* T, hipStream_t s);
hipError_t launch_pks_pack_mfma(const u64* lwes, size_t count, int in_dim, int base_log, int L, int k, int N, int lpg,
                                const void* planes, void* A0, void* A1, u64* T, u64* out, hipStream_t s);
// modulus-switch noise reduction (ms_reduce.hip), in place on B x (n+1); picks (device, nullable).
// `zeros` holds the rows [count][n+1] followed by their element-major transpose [n+1][ms_zeros_pitch(count)]
// (padding columns zero).
inline size_t ms_zeros_pitch(size_t count) { return (count + 63) / 64 * 64; }
hipError_t launch_ms_reduce(u64* lwe, size_t B, int n, const u64* zeros, int count, int log2_2N, double bound,
                            double r_sigma, double var128, int* picks, hipStream_t s);
hipError_t launch_ntt2048_inv(u64* polys, size_t count, const u64* tw, u64 ninv, hipStream_t s);
}  // namespace tfhe
