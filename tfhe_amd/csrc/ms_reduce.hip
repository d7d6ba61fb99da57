// ms_reduce.hip — modulus-switch noise reduction of the P-FHEVM (KS -> PBS) path (SURVEY §8a a3,
// §8f f4): between the keyswitch and the blind rotation, add to each small-key ciphertext the one
// encryption of zero (of the server key's `count`, 1449 in the reference's parameter block) that
// shrinks the error of the switch to 2N.  Algorithm and the exact evaluation order of the measure:
// oracle/tfhe_oracle.h (or_ms_key); this kernel reproduces every comparison bit-for-bit.
//
// Work shape: one wave per ciphertext, no barriers, so every wave stops as soon as its own
// ciphertext is resolved (a real keyswitch output needs zero index < 64 for ~97 % of ciphertexts:
// one tile).  First the measure of the ciphertext alone (lanes over elements, exact shuffle sums);
// then the zeros in index order, 64 at a time, one zero per lane: the ciphertext's elements are
// wave-uniform (scalar loads), the zeros' elements come 64 per coalesced load from the element-major
// transpose of the key (pbs_kernels.h: ms_zeros_pitch).  Per element the switch error needs only the
// low `shift` bits of x = a + z:  e = 2^(s-1) - y  with  y = (x + 2^(s-1)) mod 2^s, so the exact sums
// are  Σe = n 2^(s-1) - Σy  and  Σe² = n 2^(2s-2) - 2^s Σy + Σy², with y = yh 2^26 + yl and Σy² from
// three u64 sums of 32x32 products (Σyh², Σyh·yl, Σyl²) — ten VALU operations per element.  The
// measure is then the oracle's fixed sequence of IEEE double operations with contraction off.
#include <hip/hip_runtime.h>

#include "pbs_kernels.h"

namespace tfhe {
namespace {

constexpr int MS_WAVES = 4;   // ciphertexts (one wave each) per workgroup
constexpr int MS_BATCH = 16;  // zero-tile loads in flight per wave

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

struct YSums {
  u64 y = 0, hh = 0, hl = 0, ll = 0;
  __device__ __forceinline__ void add(u64 a_half, u64 z, u64 ymask) {
    const u64 x = (a_half + z) & ymask;
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    y += x;
    const u32 yh = __builtin_amdgcn_alignbit(hi, lo, 26), yl = lo & 0x3FFFFFFu;
    hh += (u64)yh * yh;
    hl += (u64)yh * yl;
    ll += (u64)yl * yl;
  }
};

__device__ __forceinline__ u64 zload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(u64, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

__device__ __forceinline__ double wave_min(double v) {
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off));
  return v;
}

__global__ void __launch_bounds__(64 * MS_WAVES) ms_reduce_kernel(u64* __restrict__ lwe, int B, int n,
                                                                  const u64* __restrict__ zeros,
                                                                  const u64* __restrict__ zt, int zp, int count,
                                                                  int shift, double bound, double r_sigma,
                                                                  double var128, int* __restrict__ picks) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * MS_WAVES + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (b >= B) return;
  const size_t dim = (size_t)n + 1;
  u64* ct = lwe + (size_t)b * dim;

  // measure of the ciphertext alone (lanes over elements; the xor reductions leave the sums in every lane)
  double best;
  {
    i64 s1 = 0;
    u128 s2 = 0;
    for (int i = lane; i < n; i += 64) {
      const i64 e = ms_err(ct[i], shift);
      const u64 u = (u64)(e < 0 ? -e : e);
      s1 += e;
      s2 += (u128)u * u;
    }
    for (int off = 32; off > 0; off >>= 1) {
      s1 += __shfl_xor(s1, off);
      const u64 lo = (u64)s2, hi = (u64)(s2 >> 64);
      const u64 olo = __shfl_xor(lo, off), ohi = __shfl_xor(hi, off);
      s2 = (((u128)hi << 64) | lo) + (((u128)ohi << 64) | olo);
    }
    best = ms_measure(s1, s2, ms_err(ct[n], shift), r_sigma, var128);
  }
  int pick = -1;
  bool done = best <= bound || count == 0;

  const u64 half = 1ull << (shift - 1);
  const u64 ymask = ((u64)((1u << (shift - 32)) - 1) << 32) | 0xFFFFFFFFull;  // 2^shift - 1, shift > 32
  const int nb = n / MS_BATCH * MS_BATCH;
  // the transpose through a buffer resource: lane offset in the VGPR, the element row in the SGPR offset
  const __amdgpu_buffer_rsrc_t zr =
      __builtin_amdgcn_make_buffer_rsrc((void*)zt, (short)0, (int)((size_t)(n + 1) * zp * 8), 0x00020000);
  const int rowb = zp * 8;
  for (int z0 = 0; z0 < count && !done; z0 += 64) {
    const int vo = (z0 + lane) * 8;
    YSums s;
    for (int i0 = 0; i0 < nb; i0 += MS_BATCH) {
      u64 zv[MS_BATCH];
#pragma unroll
      for (int j = 0; j < MS_BATCH; j++) zv[j] = zload(zr, vo, (i0 + j) * rowb);
#pragma unroll
      for (int j = 0; j < MS_BATCH; j++) s.add(ct[i0 + j] + half, zv[j], ymask);
    }
    for (int i = nb; i < n; i++) s.add(ct[i] + half, zload(zr, vo, i * rowb), ymask);
    // Σe, Σe² exactly (u128 wraps cancel: the true Σe² is non-negative and < 2^128)
    const u128 y2 = ((u128)s.hh << 52) + ((u128)s.hl << 27) + s.ll;
    const i64 s1 = (i64)(((u64)n << (shift - 1)) - s.y);
    const u128 s2 = ((u128)(u64)n << (2 * shift - 2)) - ((u128)s.y << shift) + y2;
    const int zi = z0 + lane;
    double m = __builtin_inf();
    if (zi < count) m = ms_measure(s1, s2, ms_err(ct[n] + zload(zr, vo, n * rowb), shift), r_sigma, var128);
    // the sequential rule over this tile, in index order (best > bound here): the first zero within the
    // bound wins; else the first minimiser, if it is a strict improvement
    const unsigned long long hit = __ballot(m <= bound);
    if (hit) {
      const int l = __ffsll(hit) - 1;
      best = __shfl(m, l);
      pick = z0 + l;
      done = true;
    } else {
      const double mn = wave_min(m);
      if (mn < best) {
        best = mn;
        pick = z0 + __ffsll(__ballot(m == mn)) - 1;
      }
    }
  }

  if (pick >= 0) {
    const u64* zr = zeros + (size_t)pick * dim;
    for (int i = lane; i < (int)dim; i += 64) ct[i] += zr[i];
  }
  if (picks && lane == 0) picks[b] = pick;
}

}  // namespace

hipError_t launch_ms_reduce(u64* lwe, size_t B, int n, const u64* zeros, int count, int log2_2N, double bound,
                            double r_sigma, double var128, int* picks, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const int shift = 64 - log2_2N;
  // exactness of the u64 partial sums: y < 2^shift split at bit 26, each of n (+1) terms < 2^(2 (shift - 26))
  if (shift < 33 || shift > 58 || n < 1 || (double)(n + 1) * std::ldexp(1.0, 2 * (shift - 26)) >= 0x1p64 ||
      (double)(n + 1) * std::ldexp(1.0, shift) >= 0x1p64)
    return hipErrorInvalidValue;
  // the kernel's buffer-resource offsets are 32-bit (tfhe_hip_load_ms_key refuses larger keys first)
  if (count < 0 || (double)(n + 1) * (double)ms_zeros_pitch((size_t)count) * 8.0 >= 0x1p31) return hipErrorInvalidValue;
  const int zp = (int)ms_zeros_pitch((size_t)count);
  const u64* zt = zeros + (size_t)count * (n + 1);
  const unsigned grid = (unsigned)((B + MS_WAVES - 1) / MS_WAVES);
  ms_reduce_kernel<<<grid, 64 * MS_WAVES, 0, s>>>(lwe, (int)B, n, zeros, zt, zp, count, shift, bound, r_sigma,
                                                  var128, picks);
  return hipGetLastError();
}

}  // namespace tfhe
