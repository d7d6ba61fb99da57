// ms_reduce.hip — modulus-switch noise reduction of the P-FHEVM (KS -> PBS) path (SURVEY §8a a3,
// §8f f4): between the keyswitch and the blind rotation, add to each small-key ciphertext the one
// encryption of zero (of the server key's `count`, 1449 in the reference's parameter block) that
// shrinks the error of the switch to 2N.  Algorithm and the exact evaluation order of the measure:
// oracle/tfhe_oracle.h (or_ms_key); this kernel reproduces every comparison bit-for-bit.
//
// Work shape: one workgroup per tile of MS_CT ciphertexts; it scans the zeros in index order, MS_ZT
// at a time (one (ciphertext, zero) pair per thread, both operand tiles staged through LDS in
// element chunks), and stops as soon as every ciphertext of the tile has found a zero whose measure
// is within the bound (the sequential early exit of the algorithm, so typically 1-2 tiles of zeros
// are read).  Integer sums are exact (i64 / u128); the measure is then one fixed sequence of IEEE
// double operations with contraction off, identical to the oracle's.  Cost: ~0.1 ms per 4096
// ciphertexts against ~0.2 s of blind rotation.
#include <hip/hip_runtime.h>

#include "pbs_kernels.h"

namespace tfhe {
namespace {

#ifndef MS_CT_N
#define MS_CT_N 8
#endif
#ifndef MS_ZT_N
#define MS_ZT_N 32
#endif
constexpr int MS_CT = MS_CT_N;  // ciphertexts per workgroup
constexpr int MS_ZT = MS_ZT_N;  // zeros per scan step
constexpr int MS_IC = 128;   // elements per LDS chunk
constexpr int MS_THREADS = MS_CT * MS_ZT;
// the per-ciphertext loop steps by MS_THREADS / 64 waves: a workgroup below one wave would never advance
static_assert(MS_THREADS % 64 == 0 && MS_THREADS >= 64, "MS_CT_N * MS_ZT_N must be a positive multiple of 64");

typedef long long i64;
typedef unsigned __int128 u128;

__device__ __forceinline__ i64 ms_err(u64 x, int shift) {
  const u64 r = ((x >> (shift - 1)) + 1) >> 1;
  return (i64)((r << shift) - x);
}

__device__ __forceinline__ double ms_measure(i64 s1, u128 s2, i64 eb, double r_sigma, double var128) {
#pragma clang fp contract(off)
  const double mean = (double)(2 * eb - s1) * 0.5;
  const double sq = (double)(u64)(s2 >> 64) * 0x1p64 + (double)(u64)s2;
  const double var = sq * 0.25 + var128;
  const double sd = sqrt(var);
  const double dev = r_sigma * sd;
  return fabs(mean) + dev;
}

struct MsShared {
  u64 a[MS_CT][MS_IC + 1];
  u64 z[MS_ZT][MS_IC + 1];  // +1: the 32 rows a half-wave reads hit distinct bank pairs
  double m[MS_CT][MS_ZT];
  double best[MS_CT];
  int pick[MS_CT];
  int done[MS_CT];
  int all_done;
};

__global__ void __launch_bounds__(MS_THREADS) ms_reduce_kernel(u64* __restrict__ lwe, int B, int n,
                                                               const u64* __restrict__ zeros, int count, int shift,
                                                               double bound, double r_sigma, double var128,
                                                               int* __restrict__ picks) {
  __shared__ MsShared S;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = blockIdx.x * MS_CT;
  const size_t dim = (size_t)n + 1;

  // measure of each ciphertext alone: wave w takes ciphertexts w, w + (waves), ...
  for (int c = wave; c < MS_CT; c += MS_THREADS / 64) {
    const int b = b0 + c;
    i64 s1 = 0;
    u128 s2 = 0;
    if (b < B) {
      const u64* ct = lwe + (size_t)b * dim;
      for (int i = lane; i < n; i += 64) {
        const i64 e = ms_err(ct[i], shift);
        const u64 u = (u64)(e < 0 ? -e : e);
        s1 += e;
        s2 += (u128)u * u;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      s1 += __shfl_xor(s1, off);
      const u64 lo = (u64)s2, hi = (u64)(s2 >> 64);
      const u64 olo = __shfl_xor(lo, off), ohi = __shfl_xor(hi, off);
      s2 = (((u128)hi << 64) | lo) + (((u128)ohi << 64) | olo);
    }
    if (lane == 0) {
      if (b < B) {
        const double m0 = ms_measure(s1, s2, ms_err(lwe[(size_t)b * dim + n], shift), r_sigma, var128);
        S.best[c] = m0;
        S.done[c] = m0 <= bound || count == 0;
      } else {
        S.best[c] = 0;
        S.done[c] = 1;
      }
      S.pick[c] = -1;
    }
  }
  __syncthreads();
  if (tid == 0) {
    int all = 1;
    for (int c = 0; c < MS_CT; c++) all &= S.done[c];
    S.all_done = all;
  }
  __syncthreads();

  const int tc = tid / MS_ZT, tz = tid % MS_ZT;
  for (int z0 = 0; z0 < count && !S.all_done; z0 += MS_ZT) {
    i64 s1 = 0;
    u128 s2 = 0;
    for (int c0 = 0; c0 < n; c0 += MS_IC) {
      const int len = min(MS_IC, n - c0);
      for (int idx = tid; idx < MS_CT * MS_IC; idx += MS_THREADS) {
        const int r = idx / MS_IC, col = idx % MS_IC, b = b0 + r;
        S.a[r][col] = (b < B && col < len) ? lwe[(size_t)b * dim + c0 + col] : 0;
      }
      for (int idx = tid; idx < MS_ZT * MS_IC; idx += MS_THREADS) {
        const int r = idx / MS_IC, col = idx % MS_IC, zi = z0 + r;
        S.z[r][col] = (zi < count && col < len) ? zeros[(size_t)zi * dim + c0 + col] : 0;
      }
      __syncthreads();
      for (int i = 0; i < len; i++) {
        const i64 e = ms_err(S.a[tc][i] + S.z[tz][i], shift);
        const u64 u = (u64)(e < 0 ? -e : e);
        s1 += e;
        s2 += (u128)u * u;
      }
      __syncthreads();
    }
    const int b = b0 + tc, zi = z0 + tz;
    double m = __builtin_inf();
    if (b < B && zi < count)
      m = ms_measure(s1, s2, ms_err(lwe[(size_t)b * dim + n] + zeros[(size_t)zi * dim + n], shift), r_sigma, var128);
    S.m[tc][tz] = m;
    __syncthreads();
    if (tid < MS_CT && !S.done[tid]) {
      // the sequential rule, in index order: take strict improvements, stop once within the bound
      double best = S.best[tid];
      int pick = S.pick[tid], done = 0;
      for (int j = 0; j < MS_ZT && z0 + j < count; j++) {
        const double mj = S.m[tid][j];
        if (mj < best) {
          best = mj;
          pick = z0 + j;
          if (best <= bound) {
            done = 1;
            break;
          }
        }
      }
      S.best[tid] = best;
      S.pick[tid] = pick;
      S.done[tid] = done;
    }
    __syncthreads();
    if (tid == 0) {
      int all = 1;
      for (int c = 0; c < MS_CT; c++) all &= S.done[c];
      S.all_done = all;
    }
    __syncthreads();
  }

  // apply the chosen zeros
  for (int idx = tid; idx < MS_CT * (int)dim; idx += MS_THREADS) {
    const int c = idx / (int)dim, i = idx % (int)dim, b = b0 + c;
    const int pk = S.pick[c];
    if (b < B && pk >= 0) lwe[(size_t)b * dim + i] += zeros[(size_t)pk * dim + i];
  }
  if (picks && tid < MS_CT && b0 + tid < B) picks[b0 + tid] = S.pick[tid];
}

}  // namespace

hipError_t launch_ms_reduce(u64* lwe, size_t B, int n, const u64* zeros, int count, int log2_2N, double bound,
                            double r_sigma, double var128, int* picks, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const unsigned grid = (unsigned)((B + MS_CT - 1) / MS_CT);
  ms_reduce_kernel<<<grid, MS_THREADS, 0, s>>>(lwe, (int)B, n, zeros, count, 64 - log2_2N, bound, r_sigma, var128,
                                               picks);
  return hipGetLastError();
}

}  // namespace tfhe
