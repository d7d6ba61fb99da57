// pks.hip — LWE -> GLWE packing keyswitch (rule: oracle/tfhe_oracle.h or_pks_params).
//
// For a group of up to lwe_per_glwe LWEs packed into one GLWE:
//   out = sum_d X^d * ((0 | b_d) - T_d),   T_d = sum_{j,l} digit_{d,j,l} * PKSK[j][l]   (mod 2^64)
// The T_d of all LWEs form one integer GEMM  T[M][(k+1)N] = D[M][in_dim*L] x PKSK[in_dim*L][(k+1)N]
// (the shape that dominates: 2048 x 4096 x 4096 per GLWE at the ML preset), followed by a
// negacyclic shift-and-sum that reads each T element exactly once.  Digits are stored offset to
// [0, 2^base_log) so the GEMM multiplies u32 x u64; the offset's contribution, (B/2) * column sum of
// the key, is subtracted in the GEMM epilogue (precomputed once per key).
//
// Kernels:
//   pks_digits_kernel   one thread per mask element: SignedDecomposer digits (closest_representable)
//   pks_gemm_kernel     64 x 64 output tile per 256-thread workgroup, 4 x 4 per thread, K staged
//                       through LDS in steps of 16; u64 wrapping MAC on VALU (3 instructions)
//   pks_shift_sum_kernel one thread per output coefficient: sum_d +-T_d[(t - d) mod N] + bodies
#include <hip/hip_runtime.h>

#include "pbs_kernels.h"

namespace tfhe {
namespace {

constexpr int PG_BM = 64, PG_BN = 64, PG_BK = 16, PG_THREADS = 256;

__global__ void pks_digits_kernel(const u64* __restrict__ lwes, size_t count, int in_dim, int base_log, int L,
                                  u32* __restrict__ A) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= count * (size_t)in_dim) return;
  const size_t m = idx / in_dim, j = idx % in_dim;
  const u64 x = lwes[m * (in_dim + 1) + j];
  const int prec = base_log * L, nonrep = 64 - prec;
  u64 state = ((x >> (nonrep - 1)) + 1) >> 1;
  state &= (1ull << prec) - 1;
  const u64 B = 1ull << base_log, mask = B - 1, half = B >> 1;
  u32* out = A + m * (size_t)in_dim * L + j * (size_t)L;
  for (int l = L - 1; l >= 0; l--) {
    const u64 res = state & mask;
    state >>= base_log;
    const u64 carry = ((((res - 1) | state) & res) >> (base_log - 1)) & 1;
    state += carry;
    const long long d = (long long)res - (long long)(carry << base_log);
    out[l] = (u32)(d + (long long)half);
  }
}

__global__ void __launch_bounds__(PG_THREADS) pks_gemm_kernel(const u32* __restrict__ A, const u64* __restrict__ P,
                                                              const u64* __restrict__ corr, u64* __restrict__ T,
                                                              int M, int K, int Nc) {
  __shared__ u32 As[PG_BK][PG_BM];
  __shared__ u64 Bs[PG_BK][PG_BN];
  const int tid = threadIdx.x, tx = tid % 16, ty = tid / 16;
  const int n0 = blockIdx.x * PG_BN, m0 = blockIdx.y * PG_BM;
  u64 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = 0;
  for (int k0 = 0; k0 < K; k0 += PG_BK) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int e = tid + r * PG_THREADS;  // 1024 elements of each tile
      const int am = e / PG_BK, ak = e % PG_BK;
      As[ak][am] = (m0 + am < M) ? A[(size_t)(m0 + am) * K + k0 + ak] : 0u;
      const int bk = e / PG_BN, bn = e % PG_BN;
      Bs[bk][bn] = P[(size_t)(k0 + bk) * Nc + n0 + bn];
    }
    __syncthreads();
#pragma unroll 4
    for (int kk = 0; kk < PG_BK; kk++) {
      u32 a[4];
      u64 b[4];
#pragma unroll
      for (int i = 0; i < 4; i++) a[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; j++) b[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] += (u64)a[i] * b[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int n = n0 + tx * 4 + j;
      T[(size_t)m * Nc + n] = acc[i][j] - corr[n];
    }
  }
}

__global__ void pks_shift_sum_kernel(const u64* __restrict__ T, const u64* __restrict__ lwes, size_t count, int in_dim,
                                     int k, int N, int lpg, size_t groups, u64* __restrict__ out) {
  const int Nc = (k + 1) * N;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= groups * (size_t)Nc) return;
  const size_t g = idx / Nc;
  const int ct = (int)(idx % Nc), c = ct / N, t = ct % N;
  const size_t first = g * (size_t)lpg;
  const int cnt = (int)min((size_t)lpg, count - first);
  const u64* Tg = T + first * (size_t)Nc + (size_t)c * N;
  u64 acc = 0;
  for (int d = 0; d <= t && d < cnt; d++) acc -= Tg[(size_t)d * Nc + (t - d)];
  for (int d = t + 1; d < cnt; d++) acc += Tg[(size_t)d * Nc + (t - d + N)];
  if (c == k && t < cnt) acc += lwes[(first + t) * (in_dim + 1) + in_dim];
  out[g * (size_t)Nc + ct] = acc;
}

// column sums of the key times B/2 (the digit offset's contribution)
__global__ void pks_corr_kernel(const u64* __restrict__ P, int K, int Nc, u64 half, u64* __restrict__ corr) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= Nc) return;
  u64 s = 0;
  for (int r = 0; r < K; r++) s += P[(size_t)r * Nc + n];
  corr[n] = s * half;
}

}  // namespace

hipError_t launch_pks_corr(const u64* pksk, int K, int Nc, int base_log, u64* corr, hipStream_t s) {
  pks_corr_kernel<<<(Nc + 255) / 256, 256, 0, s>>>(pksk, K, Nc, 1ull << (base_log - 1), corr);
  return hipGetLastError();
}

// T workspace: count x Nc u64; A workspace: count x in_dim*L u32
hipError_t launch_pks_pack(const u64* lwes, size_t count, int in_dim, int base_log, int L, int k, int N, int lpg,
                           const u64* pksk, const u64* corr, u32* A, u64* T, u64* out, hipStream_t s) {
  if (count == 0) return hipSuccess;
  const int K = in_dim * L, Nc = (k + 1) * N;
  const size_t el = count * (size_t)in_dim;
  pks_digits_kernel<<<(unsigned)((el + 255) / 256), 256, 0, s>>>(lwes, count, in_dim, base_log, L, A);
  dim3 grid(Nc / PG_BN, (unsigned)((count + PG_BM - 1) / PG_BM));
  pks_gemm_kernel<<<grid, PG_THREADS, 0, s>>>(A, pksk, corr, T, (int)count, K, Nc);
  const size_t groups = (count + lpg - 1) / lpg, outs = groups * (size_t)Nc;
  pks_shift_sum_kernel<<<(unsigned)((outs + 255) / 256), 256, 0, s>>>(T, lwes, count, in_dim, k, N, lpg, groups, out);
  return hipGetLastError();
}

hipError_t launch_pks_pack_mfma(const u64* lwes, size_t count, int in_dim, int base_log, int L, int k, int N, int lpg,
                                const void* planes, void* A0, void* A1, u64* T, u64* out, hipStream_t s) {
  if (count == 0) return hipSuccess;
  const int Nc = (k + 1) * N;
  hipError_t e = launch_pks_gemm_mfma(lwes, count, in_dim, base_log, L, Nc, planes, A0, A1, T, s);
  if (e != hipSuccess) return e;
  const size_t groups = (count + lpg - 1) / lpg, outs = groups * (size_t)Nc;
  pks_shift_sum_kernel<<<(unsigned)((outs + 255) / 256), 256, 0, s>>>(T, lwes, count, in_dim, k, N, lpg, groups, out);
  return hipGetLastError();
}

}  // namespace tfhe
