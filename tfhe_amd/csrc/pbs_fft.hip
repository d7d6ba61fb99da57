// pbs_fft.hip — the FFT64 transform of the PBS hot path for gfx950 (P-GATE shape: N = 1024, k = 1,
// PBS 2^7 x 3): the external product computed the way tfhe-rs computes it, with an f64 negacyclic
// FFT over the native 2^64 torus, instead of the Goldilocks NTT of pbs_kernels.hip.
//
// Why: MI355X runs f64 add / mul / fma at the full VALU rate (4-5 cycles per wave-instruction, the same
// as a 32-bit integer op), and a complex radix-2 butterfly is ~8 such instructions where a Goldilocks
// butterfly is ~30 integer ones.  Same BSK bytes (N/2 complex doubles = N u64 per polynomial).
//
// Arithmetic (one fixed f64 operation sequence, restated in oracle/fft_oracle.c, which this file
// reproduces bit-for-bit — every product is written as an explicit fma or a lone multiply, and
// contraction is off for the whole file):
//   fold + twist  z_j = (a_j + i a_{j+512}) * zeta^j,   zeta = e^{i pi / 1024}
//   DFT           Z_k = sum_j z_j e^{+2 pi i jk / 512}: fft512p.h (DFT8 over the slots, a register exchange,
//                 radix-4, ONE LDS transpose, DFT16), natural order in, DEVICE ORDER out (fft512p.h); the
//                 inverse runs the stages reversed, device order in, natural order out
//   MAC           O_j = one fma chain per frequency over the levels least significant first and, within a level,
//                 c = 0, 1 (each level's digits come off a running carry state, so the device BSK stores the
//                 level rows least significant first: [i][q][c][j], q = 2 - l); the first term a multiply
//   inverse       conjugate stages, untwist by conj(zeta^j), rint, mod 2^64, add to the accumulator
// Coefficient 64 e + L of a u64 register polynomial (slot e of lane L, e < 16) meets coefficient
// 64 (e + 8) + L in the same lane, so folding and unfolding move no data.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fft512p.h"
#include "gl64.h"
#include "ntt1024.h"
#include "pbs_kernels.h"

namespace tfhe {
namespace fftk {

__device__ __forceinline__ int ms2048(u64 x) { return (int)((((x >> 52) + 1) >> 1) & 2047u); }

// tfhe-rs SignedDecomposer 2^7 x 3 (closest_representable at 21 bits, balanced digits, carry
// rule carry = (((res - 1) | state) & res) >> 6), restated as one step per level, least significant
// first, on the running state st (21 bits to start; == or_decompose for every state, tests/test_fft.py):
//   b = bit 13 of st (level 2 and 1; 0 for the top level), W = st + 63 + b,
//   digit = (W & 127) - 63 - b, st' = W >> 7
__device__ __forceinline__ u32 decomp_state(u64 x) { return ((u32)(x >> 32) + 1024u) >> 11; }
// bmask = 1 below the top level, 0 at the top level
// (W & 127) - 63 - b = st - (W & ~127): the digit is the old state minus the new one shifted back
__device__ __forceinline__ int decomp_step(u32& st, u32 bmask) {
  const u32 b = __builtin_amdgcn_ubfe(st, 13, bmask);
  const u32 W = st + 63u + b;
  const int d = (int)(st - (W & ~127u));  // 5 VALU per digit with the bfe, add3 and shift
  st = W >> 7;
  return d;
}
// the top level (b = 0, no next state): 3 VALU per digit
__device__ __forceinline__ int decomp_top(u32 st) { return (int)(st - ((st + 63u) & ~127u)); }

// o = D (.) K as the first term of the fma chain: a multiply where the chain would add to +0 (the oracle's
// first term; the two differ only in the sign of an exact zero, which no later step can turn into a non-zero)
__device__ __forceinline__ void mac_first(double& re, double& im, double dr, double di, double2 k) {
  re = dr * k.x;
  re = __builtin_fma(-di, k.y, re);
  im = dr * k.y;
  im = __builtin_fma(di, k.x, im);
}
__device__ __forceinline__ void mac_next(double& re, double& im, double dr, double di, double2 k) {
  re = __builtin_fma(dr, k.x, re);
  re = __builtin_fma(-di, k.y, re);
  im = __builtin_fma(dr, k.y, im);
  im = __builtin_fma(di, k.x, im);
}

}  // namespace fftk

namespace fftp {
using fftk::decomp_state;
using fftk::decomp_step;
using fftk::decomp_top;
using fftk::mac_first;
using fftk::mac_next;
using fftk::ms2048;

// ---------------------------------------------------------------------------------------------
// BSK conversion: one wavefront per standard-layout polynomial [i][c * 3 + l][j] (l = 0 most significant) ->
// device layout [i][q = 2 - l][c][j], 512 complex in device order, x 2^-9
__global__ __launch_bounds__(64) void bsk_to_fourier_kernel(const u64* __restrict__ bsk_std,
                                                            double2* __restrict__ bsk_f,
                                                            const double2* __restrict__ tab) {
  __shared__ __attribute__((aligned(16))) double2 area[PS_C64];
  const int lane = threadIdx.x;
  TwP w;
  w.load(tab, lane);
  const size_t qs = blockIdx.x;
  const u64* src = bsk_std + qs * N1K;
  double ar[8], ai[8], xr[16], xi[16];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    ar[e] = i64_to_f64(src[64 * e + lane]);
    ai[e] = i64_to_f64(src[64 * e + 512 + lane]);
  }
  fwd_single(ar, ai, xr, xi, area, TBaseP(lane, true), w);
  const size_t j = qs % 2, r = (qs / 2) % 6, i = qs / 12, c = r / 3, q = 2 - r % 3;
  double2* dst = bsk_f + ((i * 6 + 2 * q + c) * 2 + j) * MP;
  if (lane < 32) {
#pragma unroll
    for (int m = 0; m < 16; m++) dst[lane + 32 * m] = make_double2(xr[m] * 0x1p-9, xi[m] * 0x1p-9);
  }
}

// natural-order transforms for the parity tests (one wavefront per polynomial; spectra in device order)
__global__ __launch_bounds__(64) void fft_fwd_kernel(const u64* __restrict__ in, double2* __restrict__ out,
                                                     const double2* __restrict__ tab) {
  __shared__ __attribute__((aligned(16))) double2 area[PS_C64];
  const int lane = threadIdx.x;
  TwP w;
  w.load(tab, lane);
  const u64* src = in + (size_t)blockIdx.x * N1K;
  double ar[8], ai[8], xr[16], xi[16];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    ar[e] = i64_to_f64(src[64 * e + lane]);
    ai[e] = i64_to_f64(src[64 * e + 512 + lane]);
  }
  fwd_single(ar, ai, xr, xi, area, TBaseP(lane, true), w);
  double2* dst = out + (size_t)blockIdx.x * MP;
  if (lane < 32) {
#pragma unroll
    for (int m = 0; m < 16; m++) dst[lane + 32 * m] = make_double2(xr[m], xi[m]);
  }
}

__global__ __launch_bounds__(64) void fft_inv_kernel(const double2* __restrict__ in, double* __restrict__ out,
                                                     const double2* __restrict__ tab) {
  __shared__ __attribute__((aligned(16))) double2 area[PS_C64];
  const int lane = threadIdx.x;
  TwP w;
  w.load(tab, lane);
  const double2* src = in + (size_t)blockIdx.x * MP;
  double xr[16], xi[16], ar[8], ai[8];
#pragma unroll
  for (int m = 0; m < 16; m++) {
    const double2 v = src[(lane & 31) + 32 * m];
    xr[m] = v.x;
    xi[m] = v.y;
  }
  inv_single(xr, xi, ar, ai, area, TBaseP(lane, true), w);
  double* dst = out + (size_t)blockIdx.x * N1K;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    dst[64 * e + lane] = ar[e];
    dst[64 * e + 512 + lane] = ai[e];
  }
}

// ---------------------------------------------------------------------------------------------
// One-wave-per-ciphertext batch kernel (round 4, the default above the latency range).  A workgroup is CTS
// ciphertexts, one wave each; the wave holds both accumulator polynomials (32 u64 per lane).  Per CMUX i:
//   rotate + decompose both components through the wave's LDS area (rotation by DS offsets)
//   level steps q = 0, 1, 2 (least significant first): digits of BOTH components -> ONE pair transform
//     (fft512p.h: one LDS round trip for two polynomials) -> lane 32 p + lam holds D_p at slots m1; one
//     v_permlane32_swap per value then gives every lane D_0 and D_1 at the same 8 frequencies
//     (m1 = i + 8 (lane >> 5), i = slot) -> MAC into O_0, O_1 (the oracle's chain: (q, c = 0), (q, c = 1), ...)
//     against the level step's chunk (rows (c, j) of level q of BSK_i, 32 KB) streamed once per workgroup
//     into LDS by global_load_lds
//   a second permlane32 swap returns O_0 to lanes 0-31 and O_1 to lanes 32-63 (all 16 slots), ONE pair
//   inverse transform, acc += rint mod 2^64
// Against round 3's component-pair kernel (a wave per component, two 512-point transforms of two LDS round trips
// each per level, a partial-sum exchange through LDS and two barriers): per ciphertext and CMUX 5 LDS round trips
// instead of 20, 80 KB of LDS stores instead of 160 KB, no exchange.  Registers: accumulators 64, partial sums 64,
// the pair in flight 64, digit states 32 — one wave per SIMD (512 registers), so CTS = 4 per CU.
// LDS: CTS = 4: two 32 KB level-step buffers + the 9 KB twiddle table + 4 x 17 KB areas = 141 KB (one workgroup per
//      CU); CTS = 2: one buffer + table + 2 areas = 75 KB (two workgroups per CU, FFT_CT_CTS=2 for A/B).
#ifndef FFT_CT_CTS
#define FFT_CT_CTS 4
#endif
// FFT_PRIO: s_setprio 1 for the upper half of the waves (round 1: the second-dispatched wave of a SIMD pair
// otherwise loses VALU arbitration after every barrier); kept switchable for the one-wave-per-SIMD layout
#ifndef FFT_PRIO
#define FFT_PRIO 0
#endif
constexpr int STEP_C64 = 4 * MP;  // rows (c, j) of one level, [c][j][512]

template <int CTS, int NBUF>
struct CtShared {
  double2 K[NBUF][STEP_C64];  // first: an area's base minus 8 KB (the rotation's wrapped reads) stays in the block
  double2 tab[P_C64];         // ta | tb (TwL reads them at each use)
  double2 T[CTS][PA_C64];
};

typedef __attribute__((address_space(3))) u64 lds_u64;

// level step g = 3 i + q: 32 KB in 1 KB blocks; wave w of CTS loads blocks (32 / CTS) w ..
template <int CTS>
__device__ __forceinline__ void load_step(const double2* __restrict__ bsk, int g, double2* dst, int wave_s, int lane) {
  const char* src = (const char*)(bsk + (size_t)g * STEP_C64);
#pragma unroll
  for (int u = 0; u < 32 / CTS; u++) {
    const int blk = wave_s * (32 / CTS) + u;
    __builtin_amdgcn_global_load_lds((const void*)(src + blk * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)((char*)dst + blk * 1024), 16, 0, 0);
  }
}

// (X^a v_c - v_c) for both components c (v[16 c + e] <-> coefficient 64 e + L of component c), to decomposition
// states.  The rotation image is the wave's area (component c at u64 offset 1024 c).  Coefficient 64 e + L reads
// image entry (u + 64 e) mod 1024 with u = (L - a) mod 1024, negated iff the negacyclic source index
// (L - a + 64 e) mod 2048 lies in [1024, 2048): reads before the per-lane wrap use base u and DS offset 512 e,
// wrapped reads the base 8 KB lower.
__device__ __forceinline__ void rotate_states2(const u64 (&v)[32], int a, int lane, double2* T, u32 (&st)[32]) {
  u64* Tu = (u64*)T;
#pragma unroll
  for (int e = 0; e < 32; e++) Tu[64 * e + lane] = v[e];
  lds_order();
  const int t0 = (lane - a) & 2047;  // a < 2048
  const int u = t0 & 1023;
  const bool neg0 = t0 >= 1024;
  const u32 a0 = (u32)(uintptr_t)(lds_u64*)&Tu[u];
#pragma unroll
  for (int c = 0; c < 2; c++)
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const bool wrap = u >= 1024 - 64 * e;
      const u32 base = (wrap ? a0 - 8192u : a0) + 8192u * c;
      const u64 x = ((const lds_u64*)(uintptr_t)base)[64 * e];
      const bool neg = neg0 != wrap;
      const u64 r = neg ? 0 - x : x;
      st[16 * c + e] = decomp_state(r - v[16 * c + e]);
    }
  lds_order();
}

template <int CTS, bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(64 * CTS, 1) void blind_rotate_fft_ct_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tab, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  constexpr int NBUF = CTS >= 4 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) CtShared<CTS, NBUF> sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const size_t b_raw = (size_t)blockIdx.x * CTS + wave;
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding waves run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  double2* T = sh.T[wave_s];
  const int n_steps = 3 * n;
  if constexpr (NBUF == 2) load_step<CTS>(bsk, 0, sh.K[0], wave_s, lane);
  for (int q = threadIdx.x; q < P_C64; q += 64 * CTS) sh.tab[q] = tab[q];

  // acc: A = 0, B = X^{-b~} * lut (LUT values in the Z_p encoding, mapped to the torus first)
  u64 acc[32];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N1K;
    const int s = (2048 - ms2048(ct[n])) & 2047;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      int d = 64 * e + lane - s;
      bool neg = false;
      if (d < 0) { d += N1K; neg = !neg; }
      if (d < 0) { d += N1K; neg = !neg; }
      const u64 v = gl_to_torus(lut[d]);
      acc[e] = 0;
      acc[16 + e] = neg ? 0 - v : v;
    }
  }
  __syncthreads();  // the twiddle table is in LDS
  const TwL w(sh.tab, lane);
  const TBaseP tb(lane, false);
  const int kb = (lane & 31) + 256 * (lane >> 5);  // this lane's 8 frequencies after the MAC swap: d = kb + 32 i
#if FFT_PRIO
  if (wave_s >= CTS / 2) __builtin_amdgcn_s_setprio(1);
#endif

  for (int i = 0; i < n; i++) {
    u32 st[32];
    rotate_states2(acc, ms2048(ct[i]), lane, T, st);
    double o0r[8], o0i[8], o1r[8], o1i[8];
    auto level = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int g = 3 * i + q;
      if constexpr (NBUF == 2) {
        glds_barrier();  // step g's chunk is in K[g & 1]; every wave is done with K[(g + 1) & 1]
        if (g + 1 < n_steps) load_step<CTS>(bsk, g + 1, sh.K[(g + 1) & 1], wave_s, lane);
      } else {
        if (g > 0) __syncthreads();  // every wave is done with step g - 1's chunk
        load_step<CTS>(bsk, g, sh.K[0], wave_s, lane);
      }
      double xr[16], xi[16];
#pragma unroll
      for (int c = 0; c < 2; c++)
#pragma unroll
        for (int e = 0; e < 8; e++) {
          if constexpr (q == 2) {
            xr[8 * c + e] = (double)decomp_top(st[16 * c + e]);
            xi[8 * c + e] = (double)decomp_top(st[16 * c + 8 + e]);
          } else {
            xr[8 * c + e] = (double)decomp_step(st[16 * c + e], 1u);
            xi[8 * c + e] = (double)decomp_step(st[16 * c + 8 + e], 1u);
          }
        }
      fwd_pair(xr, xi, T, tb, w);
      // D_0 to slots 0-7, D_1 to slots 8-15, both at frequencies m1 = i + 8 (lane >> 5)
#pragma unroll
      for (int s = 0; s < 8; s++) {
        swap32_d(xr[s], xr[s + 8]);
        swap32_d(xi[s], xi[s + 8]);
      }
      if constexpr (NBUF == 1) glds_barrier();  // step g's chunk has landed (every wave's share)
      const double2* K = sh.K[NBUF == 2 ? (g & 1) : 0] + kb;
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const double2 k00 = K[32 * s], k01 = K[MP + 32 * s], k10 = K[2 * MP + 32 * s], k11 = K[3 * MP + 32 * s];
        if constexpr (q == 0) {
          mac_first(o0r[s], o0i[s], xr[s], xi[s], k00);
          mac_first(o1r[s], o1i[s], xr[s], xi[s], k01);
        } else {
          mac_next(o0r[s], o0i[s], xr[s], xi[s], k00);
          mac_next(o1r[s], o1i[s], xr[s], xi[s], k01);
        }
        mac_next(o0r[s], o0i[s], xr[s + 8], xi[s + 8], k10);
        mac_next(o1r[s], o1i[s], xr[s + 8], xi[s + 8], k11);
      }
    };
    level(std::integral_constant<int, 0>{});
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    // O_0 to lanes 0-31, O_1 to lanes 32-63, all 16 slots
    double yr[16], yi[16];
#pragma unroll
    for (int s = 0; s < 8; s++) {
      swap32_d(o0r[s], o1r[s]);
      swap32_d(o0i[s], o1i[s]);
      yr[s] = o0r[s];
      yi[s] = o0i[s];
      yr[s + 8] = o1r[s];
      yi[s + 8] = o1i[s];
    }
    inv_pair(yr, yi, T, tb, w);
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
      for (int e = 0; e < 8; e++) {
        acc[16 * c + e] += f64_to_torus(yr[8 * c + e]);
        acc[16 * c + 8 + e] += f64_to_torus(yi[8 * c + e]);
      }
  }

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048;
#pragma unroll
    for (int e = 0; e < 32; e++) oa[64 * e + lane] = acc[e];
  }
  if (WRITE_BIG) {
    // sample extraction at degree 0 (computations.rs:109-132): a'_0 = A[0], a'_j = -A[N-j], b' = B[0]
    u64* ob = out_big + b * (size_t)(N1K + 1);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int idx = 64 * e + lane;
      if (idx == 0) ob[0] = acc[e];
      else ob[N1K - idx] = 0 - acc[e];
    }
    if (lane == 0) ob[N1K] = acc[16];
  }
}

// ---------------------------------------------------------------------------------------------
// Latency-mode blind rotation (small batches): ONE ciphertext per workgroup of 8 waves.  Per CMUX:
//   A  waves 0..5: wave r = 2 q + c (level q least significant first, component c) rotates + decomposes
//      accumulator polynomial c, keeps level q's digits and runs the single-polynomial transform -> F[r]
//   B  all 8 waves: O_j = the oracle's chain over r = 0..5 of F[r] (.) BSK_i[q][c][j] on 128 of the 512
//      frequencies each (j = wave >> 2); the key words come straight from L2 into registers, requested one CMUX
//      ahead
//   C  waves 0, 1: single inverse transform of O_j, acc_j += rint mod 2^64
// Three barriers per CMUX.  LDS: acc 16 KB | F 48 KB | 6 transpose areas 51 KB (O_0, O_1 alias areas 2, 3, dead
// after phase A) | rotation amounts 2 KB | twiddle table 9 KB = 126 KB.
constexpr int FL_THREADS = 512;
constexpr int FL_MAXN = 1024;  // rotation amounts staged in LDS up to this LWE dimension (global reads above)
struct FftLatShared {
  double2 tab[P_C64];
  u64 A[2][N1K];
  double2 F[6][MP];
  double2 T[6][PS_C64];
  unsigned short ab[FL_MAXN];  // ms2048(ct[i]) for every CMUX
};

#ifndef FFT_LAT_PREFETCH
#define FFT_LAT_PREFETCH 1
#endif
__device__ __forceinline__ void lat_load_key(const double2* __restrict__ bsk, int i, int j, int s0, int lane,
                                             double2 (&kv)[6][2]) {
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int t = 0; t < 2; t++) kv[r][t] = bsk[((size_t)(i * 6 + r) * 2 + j) * MP + 64 * (s0 + t) + lane];
}

// one CMUX of the latency kernel (phases A, B, C and their three barriers)
__device__ __forceinline__ void lat_cmux(FftLatShared& sh, const u64* __restrict__ ct, int i, int wave, int lane,
                                         const TwL& w, int j, int s0, const double2 (&kv)[6][2]) {
  const int a = i < FL_MAXN ? (int)sh.ab[i] : ms2048(ct[i]);
  if (wave < 6) {  // phase A
    const int q = wave >> 1, c = wave & 1;
    const u64* acc = sh.A[c];
    u32 st[16];
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int t = 64 * e + lane - a + 2 * N1K;
      const u64 x = acc[t & (N1K - 1)];
      const u64 r = (t & N1K) ? 0 - x : x;
      st[e] = decomp_state(r - acc[64 * e + lane]);
    }
    int dg[16];
    for (int qq = 0; qq <= q; qq++) {
      const u32 bmask = qq < 2 ? 1u : 0u;
#pragma unroll
      for (int e = 0; e < 16; e++) dg[e] = decomp_step(st[e], bmask);
    }
    double ar[8], ai[8], xr[16], xi[16];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      ar[e] = (double)dg[e];
      ai[e] = (double)dg[e + 8];
    }
    fwd_single(ar, ai, xr, xi, sh.T[wave], TBaseP(lane, true), w);
    if (lane < 32) {
#pragma unroll
      for (int m = 0; m < 16; m++) sh.F[wave][lane + 32 * m] = make_double2(xr[m], xi[m]);
    }
  }
  __syncthreads();
  {  // phase B
    double2* O = sh.T[2 + j];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int d = 64 * (s0 + t) + lane;
      double re, im;
#pragma unroll
      for (int r = 0; r < 6; r++) {
        const double2 D = sh.F[r][d], K = kv[r][t];
        if (r == 0) mac_first(re, im, D.x, D.y, K);
        else mac_next(re, im, D.x, D.y, K);
      }
      O[d] = make_double2(re, im);
    }
  }
  __syncthreads();
  if (wave < 2) {  // phase C
    const double2* O = sh.T[2 + wave];
    double xr[16], xi[16], ar[8], ai[8];
#pragma unroll
    for (int m = 0; m < 16; m++) {
      const double2 v = O[(lane & 31) + 32 * m];
      xr[m] = v.x;
      xi[m] = v.y;
    }
    inv_single(xr, xi, ar, ai, sh.T[wave], TBaseP(lane, true), w);
    u64* acc = sh.A[wave];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      acc[64 * e + lane] += f64_to_torus(ar[e]);
      acc[64 * (e + 8) + lane] += f64_to_torus(ai[e]);
    }
  }
  __syncthreads();
}

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(FL_THREADS, 1) void blind_rotate_fft_lat_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tab, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) FftLatShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = blockIdx.x;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  const TwL w(sh.tab, lane);

  for (int q = threadIdx.x; q < P_C64; q += FL_THREADS) sh.tab[q] = tab[q];
  for (int q = threadIdx.x; q < n && q < FL_MAXN; q += FL_THREADS) sh.ab[q] = (unsigned short)ms2048(ct[q]);
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N1K;
    const int s = (2048 - ms2048(ct[n])) & 2047;
    for (int q = threadIdx.x; q < N1K; q += FL_THREADS) {
      int d = q - s;
      bool neg = false;
      if (d < 0) { d += N1K; neg = !neg; }
      if (d < 0) { d += N1K; neg = !neg; }
      const u64 v = gl_to_torus(lut[d]);
      sh.A[0][q] = 0;
      sh.A[1][q] = neg ? 0 - v : v;
    }
  }
  __syncthreads();

  const int j = wave >> 2, s0 = (wave & 3) * 2;  // phase B: output j, frequencies 64 (s0 + t) + lane
#if FFT_LAT_PREFETCH
  // key words one CMUX ahead (two register sets, the loop unrolled by two): a CMUX's row arrives while the
  // previous CMUX runs instead of behind this CMUX's phase A
  double2 kva[6][2], kvb[6][2];
  lat_load_key(bsk, 0, j, s0, lane, kva);
  for (int i = 0; i < n; i += 2) {
    if (i + 1 < n) lat_load_key(bsk, i + 1, j, s0, lane, kvb);
    lat_cmux(sh, ct, i, wave, lane, w, j, s0, kva);
    if (i + 1 >= n) break;
    if (i + 2 < n) lat_load_key(bsk, i + 2, j, s0, lane, kva);
    lat_cmux(sh, ct, i + 1, wave, lane, w, j, s0, kvb);
  }
#else
  for (int i = 0; i < n; i++) {
    double2 kv[6][2];  // phase-B key words of this CMUX, requested now, consumed after phase A
    lat_load_key(bsk, i, j, s0, lane, kv);
    lat_cmux(sh, ct, i, wave, lane, w, j, s0, kv);
  }
#endif

  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048;
    for (int q = threadIdx.x; q < 2 * N1K; q += FL_THREADS) oa[q] = sh.A[q >> 10][q & (N1K - 1)];
  }
  if (WRITE_BIG) {  // sample extraction at degree 0
    u64* ob = out_big + b * (size_t)(N1K + 1);
    for (int q = threadIdx.x; q <= N1K; q += FL_THREADS)
      ob[q] = q == N1K ? sh.A[1][0] : q == 0 ? sh.A[0][0] : 0 - sh.A[0][N1K - q];
  }
}

__global__ void sample_extract_torus_kernel(const u64* __restrict__ acc, size_t B, u64* __restrict__ out) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * (N1K + 1)) return;
  const size_t b = gid / (N1K + 1);
  const int j = (int)(gid % (N1K + 1));
  const u64* A = acc + b * 2048;
  out[gid] = j == N1K ? A[N1K] : j == 0 ? A[0] : 0 - A[N1K - j];
}

}  // namespace fftp

namespace fftk {
// ---------------------------------------------------------------------------------------------
// host: tables (fixed series in plain double, octant-reduced — the oracle's or_fft_twiddle)
static double fs_sin(double x) {
  double x2 = x * x, term = x, sum = 0.0;
  for (int i = 1; i <= 21; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static double fs_cos(double x) {
  double x2 = x * x, term = 1.0, sum = 0.0;
  for (int i = 0; i <= 20; i += 2) { sum += term; term = -term * x2 / (double)((i + 1) * (i + 2)); }
  return sum;
}
static void tw_octant(uint32_t t, uint32_t m, double* c, double* s) {
  const double x = (double)t * (6.28318530717958647692 / (double)m);
  *c = fs_cos(x);
  *s = fs_sin(x);
}
static void tw_quarter(uint32_t t, uint32_t m, double* c, double* s) {
  if (8 * t > m) {
    double cu, su;
    tw_octant(m / 4 - t, m, &cu, &su);
    *c = su;
    *s = cu;
  } else {
    tw_octant(t, m, c, s);
  }
}
static void twiddle(uint32_t t, uint32_t m, double* c, double* s) {
  t %= m;
  bool neg = false;
  if (2 * t > m) { t = m - t; neg = true; }
  double cc, ss;
  if (4 * t > m) {
    double cu, su;
    tw_quarter(t - m / 4, m, &cu, &su);
    cc = -su;
    ss = cu;
  } else {
    tw_quarter(t, m, &cc, &ss);
  }
  *c = cc;
  *s = neg ? -ss : ss;
}

}  // namespace fftk

void fft_twiddle(uint32_t t, uint32_t m, double* c, double* s) { fftk::twiddle(t, m, c, s); }

size_t fft_tables_len() { return 2 * fftp::P_C64; }

// N = 1024 tables (fft512p.h): ta[k][L] = zeta^(L (1 + 4 k)), zeta = e^(2 pi i / 2048) (the twist's lane part merged
// into stage A), tb[m][l] = e^(2 pi i l m / 64) (the oracle's twAm and tb)
void make_fft_tables(double* t) {
  using namespace fftp;
  for (uint32_t k = 0; k < 8; k++)
    for (uint32_t L = 0; L < 64; L++) {
      const int o = P_TA + 64 * k + L;
      fftk::twiddle((L * (1 + 4 * k)) % 2048, 2048, &t[2 * o], &t[2 * o + 1]);
    }
  for (uint32_t m = 0; m < 4; m++)
    for (uint32_t l = 0; l < 16; l++) {
      const int o = P_TB + 16 * m + l;
      fftk::twiddle((64 * l * m) % 4096, 4096, &t[2 * o], &t[2 * o + 1]);
    }
}

// the compile-time slot constants equal the table generator's zeta^(64 e) bit for bit
bool fft_slot_constants_ok() {
  for (int e = 0; e < 8; e++) {
    double c, s, c2, s2;
    fftk::twiddle(64u * e, 2048u, &c, &s);      // N = 1024
    fftk::twiddle(128u * e, 4096u, &c2, &s2);   // N = 2048
    if (c != fftk::ctw::SLOT[e].x || s != fftk::ctw::SLOT[e].y || c2 != c || s2 != s) return false;
  }
  return true;
}

hipError_t launch_bsk_to_fourier(const u64* bsk_std, double* bsk_f, size_t polys, const double* tw, hipStream_t s) {
  hipLaunchKernelGGL(fftp::bsk_to_fourier_kernel, dim3((unsigned)polys), dim3(64), 0, s, bsk_std, (double2*)bsk_f,
                     (const double2*)tw);
  return hipGetLastError();
}

hipError_t launch_blind_rotate_fft(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                   int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                   hipStream_t s, size_t latency_max_batch) {
  using namespace fftp;
  if (B == 0) return hipSuccess;
  const double2 *bk = (const double2*)bsk_f, *t = (const double2*)tw;
  if (B <= latency_max_batch) {
    dim3 grid((unsigned)B), block(FL_THREADS);
    if (out_acc && out_big)
      hipLaunchKernelGGL((blind_rotate_fft_lat_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    else if (out_acc)
      hipLaunchKernelGGL((blind_rotate_fft_lat_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    else
      hipLaunchKernelGGL((blind_rotate_fft_lat_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    return hipGetLastError();
  }
  constexpr int CTS = FFT_CT_CTS;
  dim3 grid((unsigned)((B + CTS - 1) / CTS)), block(64 * CTS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_fft_ct_kernel<CTS, true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bk, t, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_fft_ct_kernel<CTS, true, false>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_fft_ct_kernel<CTS, false, true>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  return hipGetLastError();
}

hipError_t launch_sample_extract_torus(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (N1K + 1);
  hipLaunchKernelGGL(fftp::sample_extract_torus_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc, B,
                     out);
  return hipGetLastError();
}

hipError_t launch_fft_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fftp::fft_fwd_kernel, dim3((unsigned)count), dim3(64), 0, s, in, (double2*)out,
                     (const double2*)tw);
  return hipGetLastError();
}

hipError_t launch_fft_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fftp::fft_inv_kernel, dim3((unsigned)count), dim3(64), 0, s, (const double2*)in, out,
                     (const double2*)tw);
  return hipGetLastError();
}

}  // namespace tfhe
