// ks_mfma.hip — LWE keyswitch big -> n as an exact integer GEMM on the gfx950 matrix cores.
//
// The keyswitch of a batch is one matrix product modulo 2^64 (tfhe-rs
// keyswitch_lwe_ciphertext, restated in oracle/tfhe_oracle.c or_keyswitch):
//   out[b][col] = [col == n] * body_b  -  sum_k  D[b][k] * KSK[k][col]          (mod 2^64)
// with k = j * LV + r (input coefficient j, level r, r = 0 the most significant) and D the tfhe-rs
// SignedDecomposer digits (|D| <= 2^(base_log-1): 2 at P-GATE, 8 at P-FHEVM).
//
// Exactness without 64-bit multiplies: every KSK word is recoded once, at key load, into eight
// signed bytes s_t in [-128, 127] with KSK = sum_t s_t 2^(8t) (mod 2^64) (balanced recoding, the
// carry out of the top byte is a multiple of 2^64).  Then
//   sum_k D[b][k] KSK[k][col] = sum_t 2^(8t) * C_t[b][col],   C_t = D x S_t   (exact in int32:
//   |C_t| <= K * 8 * 128 = 2^23 at K = 8192)
// so the keyswitch is eight int8 GEMMs (v_mfma_i32_16x16x64_i8) sharing the digit operand, combined
// in registers: the eight plane accumulators of one (b, col) sit in the same lane and register slot.
//
// Layouts (fragment-major, so every operand load is one coalesced 16-byte-per-lane read):
//   digits  A[mt][ks][lane][16]      b = 16 mt + (lane & 15),  k = 64 ks + 16 (lane >> 4) + q
//   planes  P[nt][ks][t][lane][16]   col = 16 nt + (lane & 15), same k;  byte t of the recoded KSK
// The A and B fragments of v_mfma_i32_16x16x64_i8 use one lane -> k map for both operands, so
// storing k = 16 (lane >> 4) + q in both pairs every digit with its key byte whatever the hardware's
// internal k order is; rows / columns follow lane & 15, and C/D is col = lane & 15,
// row = 4 (lane >> 4) + reg (cdna_hip_programming.md §3), checked bit-exact against the oracle.
//
// Kernels:
//   ksk_planes_kernel  (key load)  one thread per (k, col): recode + scatter 8 bytes
//   ks_digits_kernel               one thread per (b, j): LV digits -> LV bytes of A (zero rows pad
//                                  the batch to the workgroup tile)
//   ks_gemm_kernel                 workgroup = 4 waves = 256 ciphertexts x 16 columns x 8 planes;
//                                  wave = 4 M-tiles x 8 planes = 32 accumulators (128 VGPRs), per
//                                  64-deep k step 4 digit + 8 plane fragments, 32 MFMAs
#include <hip/hip_runtime.h>

#include "pbs_kernels.h"

namespace tfhe {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int KM_WAVES = 4;                         // waves per workgroup, stacked along the batch
constexpr int KM_MT = 4;                            // 16-row M-tiles per wave
constexpr int KM_ROWS = 16 * KM_MT * KM_WAVES;      // ciphertexts per workgroup (256)
constexpr int KM_PLANES = 8;

// tfhe-rs SignedDecomposer at base 2^BL x LV (closest representable at BL*LV bits, balanced digits,
// tie carry rule): byte r of the result = level r (0 = most significant), as a signed byte
__device__ __forceinline__ unsigned long long ks_digits_packed(u64 x, int BL, int LV) {
  const int P = BL * LV;
  u32 state = (u32)(((x >> (63 - P)) + 1) >> 1) & (u32)((1ull << P) - 1);
  unsigned long long packed = 0;
  for (int l = LV - 1; l >= 0; l--) {
    const u32 res = state & ((1u << BL) - 1);
    state >>= BL;
    const u32 carry = ((((res - 1u) | state) & res) >> (BL - 1)) & 1u;
    state += carry;
    const int d = (int)res - (int)(carry << BL);
    packed |= (unsigned long long)(unsigned char)(signed char)d << (8 * l);
  }
  return packed;
}

// byte offset of element (row-or-col index within its 16-tile = i16, k) inside the fragment block of a
// k step: lane = 16 * ((k >> 4) & 3) + i16, byte q = k & 15
__device__ __forceinline__ size_t frag_off(int i16, int k) { return (size_t)(16 * ((k >> 4) & 3) + i16) * 16 + (k & 15); }

__global__ void ksk_planes_kernel(const u64* __restrict__ ksk, int K, int n, int NT, signed char* __restrict__ P) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int cols = NT * 16;
  if (idx >= (size_t)K * cols) return;
  const int k = (int)(idx / cols), col = (int)(idx % cols);
  u64 v = col <= n ? ksk[(size_t)k * (n + 1) + col] : 0ull;
  const int KS = K / 64, nt = col >> 4, ks = k >> 6;
  signed char* base = P + ((size_t)nt * KS + ks) * KM_PLANES * 1024 + frag_off(col & 15, k);
  u32 carry = 0;
#pragma unroll
  for (int t = 0; t < KM_PLANES; t++) {
    const u32 byte = (u32)(v & 0xFF) + carry;  // 0 .. 256
    v >>= 8;
    carry = byte >= 128u;
    base[(size_t)t * 1024] = (signed char)(int)(carry ? (int)byte - 256 : (int)byte);
  }
}

__global__ void ks_digits_kernel(const u64* __restrict__ in_big, int big_dim, size_t B, size_t rows, int BL, int LV,
                                 unsigned char* __restrict__ A) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * (size_t)big_dim) return;
  const size_t b = idx / big_dim;
  const int j = (int)(idx % big_dim);
  const u64 x = b < B ? in_big[b * (size_t)(big_dim + 1) + j] : 0ull;
  const unsigned long long d = b < B ? ks_digits_packed(x, BL, LV) : 0ull;
  const int K = big_dim * LV, KS = K / 64, k0 = j * LV;
  unsigned char* dst = A + ((b >> 4) * KS + (k0 >> 6)) * 1024 + frag_off((int)(b & 15), k0);
  if (LV == 8) *(unsigned long long*)dst = d;
  else if (LV == 4) *(u32*)dst = (u32)d;
  else
    for (int r = 0; r < LV; r++) dst[r] = (unsigned char)(d >> (8 * r));
}

__global__ __launch_bounds__(64 * KM_WAVES) void ks_gemm_kernel(const v4i* __restrict__ A, const v4i* __restrict__ P,
                                                                 int KS, const u64* __restrict__ in_big, int big_dim,
                                                                 size_t B, int n, u64* __restrict__ out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt = blockIdx.x;
  const size_t mt0 = ((size_t)blockIdx.y * KM_WAVES + wave) * KM_MT;
  const v4i* a = A + mt0 * KS * 64 + lane;
  const v4i* p = P + (size_t)nt * KS * KM_PLANES * 64 + lane;
  v4i acc[KM_MT][KM_PLANES];
#pragma unroll
  for (int m = 0; m < KM_MT; m++)
#pragma unroll
    for (int t = 0; t < KM_PLANES; t++) acc[m][t] = (v4i){0, 0, 0, 0};
  for (int ks = 0; ks < KS; ks++) {
    v4i af[KM_MT], bf[KM_PLANES];
#pragma unroll
    for (int m = 0; m < KM_MT; m++) af[m] = a[((size_t)m * KS + ks) * 64];
#pragma unroll
    for (int t = 0; t < KM_PLANES; t++) bf[t] = p[((size_t)ks * KM_PLANES + t) * 64];
#pragma unroll
    for (int m = 0; m < KM_MT; m++)
#pragma unroll
      for (int t = 0; t < KM_PLANES; t++) acc[m][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[m], bf[t], acc[m][t], 0, 0, 0);
  }
  const int col = nt * 16 + (lane & 15);
  if (col > n) return;
#pragma unroll
  for (int m = 0; m < KM_MT; m++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const size_t b = (mt0 + m) * 16 + 4 * (lane >> 4) + r;
      if (b >= B) continue;
      u64 v = 0;
#pragma unroll
      for (int t = 0; t < KM_PLANES; t++) v += (u64)(long long)acc[m][t][r] << (8 * t);
      const u64 body = col == n ? in_big[b * (size_t)(big_dim + 1) + big_dim] : 0ull;
      out[b * (size_t)(n + 1) + col] = body - v;
    }
}

// ---------------------------------------------------------------------------------------------
// Packing keyswitch GEMM on the matrix cores (pks.hip's T = D x PKSK mod 2^64).
// The digits are tfhe-rs SignedDecomposer digits at base 2^B (B <= 16): two signed bytes each,
// d = d0 + 2^8 d1 (d0 in [-128, 127], |d1| <= 2^(B-9)), so
//   sum_k d[k] PKSK[k][n] = sum_t 2^(8t) (D0 x S_t + D1 x S_(t-1))[n]      (mod 2^64, S_-1 = 0)
// with S_t the key's balanced byte planes (ksk_planes_kernel, the same recoding as the keyswitch).
// Fifteen int8 GEMMs per (row, column) tile, all exact in int32: |acc| <= K * 2 * 128 * 128 = 2^27 at
// K = 4096.  Layouts as above: digit bytes A0 / A1[mt][ks][lane][16], planes P[nt][ks][t][lane][16].
__global__ void pks_digits_mfma_kernel(const u64* __restrict__ lwes, size_t count, size_t rows, int in_dim, int BL,
                                       int LV, unsigned char* __restrict__ A0, unsigned char* __restrict__ A1) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * (size_t)in_dim) return;
  const size_t m = idx / in_dim;
  const int j = (int)(idx % in_dim);
  const int K = in_dim * LV, KS = K / 64;
  const u64 x = m < count ? lwes[m * (size_t)(in_dim + 1) + j] : 0ull;
  const int prec = BL * LV, nonrep = 64 - prec;
  u64 state = m < count ? (((x >> (nonrep - 1)) + 1) >> 1) & ((1ull << prec) - 1) : 0ull;
  const u64 mask = (1ull << BL) - 1;
  for (int l = LV - 1; l >= 0; l--) {  // k = j * LV + l (level l = 0 the most significant)
    const u64 res = state & mask;
    state >>= BL;
    const u64 carry = ((((res - 1) | state) & res) >> (BL - 1)) & 1;
    state += carry;
    const int d = (int)((long long)res - (long long)(carry << BL));
    const int d0 = ((d + 128) & 255) - 128, d1 = (d - d0) >> 8;
    const int k = j * LV + l;
    const size_t off = ((m >> 4) * KS + (k >> 6)) * 1024 + frag_off((int)(m & 15), k);
    A0[off] = (unsigned char)(signed char)d0;
    A1[off] = (unsigned char)(signed char)d1;
  }
}

// workgroup = 4 waves stacked along the rows; wave = PM_MT row tiles x PM_NT column tiles x 8 planes
#ifndef PM_NT
#define PM_NT 2
#endif
constexpr int PM_WAVES = 4, PM_MT = 4, PM_ROWS = 16 * PM_MT * PM_WAVES;  // 256 rows x 16 PM_NT columns

__global__ __launch_bounds__(64 * PM_WAVES, 1) void pks_gemm_mfma_kernel(const v4i* __restrict__ A0,
                                                                      const v4i* __restrict__ A1,
                                                                      const v4i* __restrict__ P, int KS, size_t M,
                                                                      int Nc, u64* __restrict__ T) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nt0 = blockIdx.x * PM_NT;
  const size_t mt0 = ((size_t)blockIdx.y * PM_WAVES + wave) * PM_MT;
  const v4i* a0 = A0 + mt0 * KS * 64 + lane;
  const v4i* a1 = A1 + mt0 * KS * 64 + lane;
  const v4i* p = P + (size_t)nt0 * KS * KM_PLANES * 64 + lane;
  v4i acc[PM_MT][PM_NT][KM_PLANES];
#pragma unroll
  for (int m = 0; m < PM_MT; m++)
#pragma unroll
    for (int c = 0; c < PM_NT; c++)
#pragma unroll
      for (int t = 0; t < KM_PLANES; t++) acc[m][c][t] = (v4i){0, 0, 0, 0};
  for (int ks = 0; ks < KS; ks++) {
    v4i f0[PM_MT], f1[PM_MT];
#pragma unroll
    for (int m = 0; m < PM_MT; m++) {
      f0[m] = a0[((size_t)m * KS + ks) * 64];
      f1[m] = a1[((size_t)m * KS + ks) * 64];
    }
#pragma unroll
    for (int c = 0; c < PM_NT; c++) {
      v4i bf[KM_PLANES];
#pragma unroll
      for (int t = 0; t < KM_PLANES; t++) bf[t] = p[(((size_t)c * KS + ks) * KM_PLANES + t) * 64];
#pragma unroll
      for (int m = 0; m < PM_MT; m++)
#pragma unroll
        for (int t = 0; t < KM_PLANES; t++) {
          acc[m][c][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f0[m], bf[t], acc[m][c][t], 0, 0, 0);
          if (t > 0) acc[m][c][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(f1[m], bf[t - 1], acc[m][c][t], 0, 0, 0);
        }
    }
  }
#pragma unroll
  for (int c = 0; c < PM_NT; c++) {
    const int col = (nt0 + c) * 16 + (lane & 15);
#pragma unroll
    for (int m = 0; m < PM_MT; m++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const size_t row = (mt0 + m) * 16 + 4 * (lane >> 4) + r;
        if (row >= M) continue;
        u64 v = 0;
#pragma unroll
        for (int t = 0; t < KM_PLANES; t++) v += (u64)(long long)acc[m][c][t][r] << (8 * t);
        T[row * (size_t)Nc + col] = v;
      }
  }
}

int ks_k(int big_dim, int levels) { return big_dim * levels; }
int ks_nt(int n) { return (n + 1 + 15) / 16; }
size_t ks_rows(size_t B) { return (B + KM_ROWS - 1) / KM_ROWS * KM_ROWS; }

}  // namespace

size_t ks_planes_bytes(int big_dim, int levels, int n) {
  return (size_t)ks_nt(n) * ks_k(big_dim, levels) * KM_PLANES * 16;
}

size_t ks_digits_bytes(size_t B, int big_dim, int levels) { return ks_rows(B) * (size_t)ks_k(big_dim, levels); }

hipError_t launch_ksk_planes(const u64* ksk, int big_dim, int levels, int n, void* planes, hipStream_t s) {
  const int K = ks_k(big_dim, levels);
  if (K % 64 || levels > 8) return hipErrorInvalidValue;
  const size_t total = (size_t)K * ks_nt(n) * 16;
  hipLaunchKernelGGL(ksk_planes_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, ksk, K, n, ks_nt(n),
                     (signed char*)planes);
  return hipGetLastError();
}

size_t pks_mfma_rows(size_t count) { return (count + PM_ROWS - 1) / PM_ROWS * PM_ROWS; }

// T[count][Nc] = D x PKSK (mod 2^64) on the matrix cores; A0 / A1: pks_mfma_rows(count) * in_dim * LV bytes each;
// planes from launch_ksk_planes(pksk, in_dim, LV, Nc - 1, ...)
hipError_t launch_pks_gemm_mfma(const u64* lwes, size_t count, int in_dim, int base_log, int LV, int Nc,
                                const void* planes, void* A0, void* A1, u64* T, hipStream_t s) {
  if (count == 0) return hipSuccess;
  const int K = in_dim * LV;
  if (K % 64 || Nc % (16 * PM_NT) || base_log < 2 || base_log > 16 || base_log * LV >= 64 ||
      (long long)K * 2 * 128 * 128 >= (1ll << 31))
    return hipErrorInvalidValue;
  const size_t rows = pks_mfma_rows(count), el = rows * (size_t)in_dim;
  hipLaunchKernelGGL(pks_digits_mfma_kernel, dim3((unsigned)((el + 255) / 256)), dim3(256), 0, s, lwes, count, rows,
                     in_dim, base_log, LV, (unsigned char*)A0, (unsigned char*)A1);
  dim3 grid((unsigned)(Nc / (16 * PM_NT)), (unsigned)(rows / PM_ROWS));
  hipLaunchKernelGGL(pks_gemm_mfma_kernel, grid, dim3(64 * PM_WAVES), 0, s, (const v4i*)A0, (const v4i*)A1,
                     (const v4i*)planes, K / 64, count, Nc, T);
  return hipGetLastError();
}

hipError_t launch_keyswitch_mfma(const u64* in_big, size_t B, int big_dim, const void* planes, int n, int base_log,
                                 int levels, void* digits, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const int K = ks_k(big_dim, levels);
  // the digit bytes must be int8 (|d| <= 2^(base_log-1) <= 64) and the int32 plane sums exact
  if (K % 64 || levels > 8 || base_log < 1 || base_log > 7 || (long long)K * 128 * (1 << (base_log - 1)) >= (1ll << 31))
    return hipErrorInvalidValue;
  const size_t rows = ks_rows(B);
  const size_t el = rows * (size_t)big_dim;
  hipLaunchKernelGGL(ks_digits_kernel, dim3((unsigned)((el + 255) / 256)), dim3(256), 0, s, in_big, big_dim, B, rows,
                     base_log, levels, (unsigned char*)digits);
  dim3 grid((unsigned)ks_nt(n), (unsigned)(rows / KM_ROWS));
  hipLaunchKernelGGL(ks_gemm_kernel, grid, dim3(64 * KM_WAVES), 0, s, (const v4i*)digits, (const v4i*)planes, K / 64,
                     in_big, big_dim, B, n, out);
  return hipGetLastError();
}

}  // namespace tfhe
