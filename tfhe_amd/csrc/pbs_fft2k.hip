// pbs_fft2k.hip — the FFT64 engine for N = 2048 (P-FHEVM: n = 918, k = 1, PBS 2^23 x 1, KS 2^4 x 4,
// KS -> PBS; sdk/relayer/src/tfhe.ts:14-19): tfhe-rs's f64 negacyclic FFT external product over the
// native 2^64 torus, restated bit-for-bit in oracle/fft_oracle.c (fft2k_fwd / fft2k_inv).
//
// A polynomial is held by TWO waves: wave h owns the coefficients of parity h,
//   slot e < 8: coefficient 2 (L + 64 e) + h,   slot e >= 8: the same + 1024,
// so its folded half z_{2m+h} = (a_{2m+h} + i a_{2m+h+1024}) zeta^{2m+h} (m = L + 64 e) is exactly the
// natural-order input of the 512-point DFT of fft512.h.  The two half spectra E_0, E_1 meet in one
// radix-2 combine, Z[k'] = E_0 + w^k' E_1, Z[k' + 512] = E_0 - w^k' E_1, after an LDS exchange of the
// pair (both waves write their 8 slots, each reads E_0 and E_1 at its 4 slots 4h + q); wave h then
// holds frequencies k'(L, 4h + (s & 3)) + 512 (s >> 2) in slot s — the device order of the BSK.
//
// Blind rotation: workgroup = 4 ciphertexts x 2 waves.  LDS (152 KB of a gfx950 CU's 160):
//   T   8 x 9,216 B   per-wave transpose scratch; a pair's two regions also hold the 2048-u64
//                     rotation image and the combine / uncombine exchanges
//   tw  48 KB         all tables: pass A'/B' per parity (twist merged in), pass B, combine
//   K   2 x 16 KB     one output column of BSK_i (K_{0,j}, K_{1,j}), loaded by global_load_lds one
//                     phase ahead (column 1 under the first inverse, the next CMUX's column 0 under
//                     the second inverse, rotation and forward transforms)
// Per CMUX: rotate + decompose both components (23 x 1 digits, no exchange of digits needed: each
// wave decomposes its own coefficients), two forward transforms, then per output column j the MAC
//   O_j = fma chain over c = 0, 1 of D_c (.) BSK_i[c][j]   (the oracle's order, from (0, 0))
// and the inverse transform back to this wave's coefficients of acc_j (F2_MACORDER 2).
#include "fft512.h"
#include "pbs_kernels.h"

namespace tfhe {
namespace fft2k {
using namespace fftk;

constexpr int N2 = 2048, M2 = 1024;
// table (complex, the same layout in global memory and in LDS), the twist merged into the passes per
// parity h (fft512.h, "merged twist"): pass A'_0 | A'_1 | B | pass B' I'_0 | I'_1 | combine [h][q][L]
//   A'_h[e][L] = zeta^(L (8 e + 2) + h),  I'_h[e][L] = zeta^((n0 + 8 e)(8 k0 + 2) + h) (L = n0 + 8 k0),
//   zeta = e^(2 pi i / 4096); B as the 512-point tables of fft512.h
constexpr int G_A0 = 0, G_A1 = 512, G_B = 1024, G_I0 = 1536, G_I1 = 2048, G_WC = 2560, G_C64 = 3072;
constexpr int F2_PAIRS = 4, F2_WAVES = 8, F2_THREADS = 64 * F2_WAVES;
constexpr int CHUNK_GLDS = M2 * 16 / 1024;  // 1 KB wave-instructions per BSK polynomial (16)

__device__ __forceinline__ int ms4096(u64 x) { return (int)((((x >> 51) + 1) >> 1) & 4095u); }
__device__ __forceinline__ int kdev(int L, int e) { return (L >> 3) + 8 * (L & 7) + 64 * e; }
// coefficient held by wave h, lane L, slot e
__device__ __forceinline__ int coef(int h, int L, int e) { return 2 * (L + 64 * (e & 7)) + h + 1024 * (e >> 3); }

// tfhe-rs SignedDecomposer 2^23 x 1: closest representable at 23 bits, state st = round(x / 2^41) mod
// 2^23, digit = st - 2^23 if st > 2^22 else st (carry rule ((st - 1) & st) >> 22; the tie 2^22 stays
// positive).  Restated on the high word alone: st = (hi + 2^8) >> 9 (a wrap of hi + 2^8 past 2^32 only
// happens when st = 2^23, i.e. 0 mod 2^23), digit = ((st + 2^22 - 1) mod 2^23) - (2^22 - 1).
__device__ __forceinline__ int decomp_23x1_hi(u32 hi) {
  const u32 st = (hi + 256u) >> 9;
  return (int)((st + 0x3FFFFFu) & 0x7FFFFFu) - 0x3FFFFF;
}

// The pair exchanges' barriers (workgroup-wide s_barrier; the two waves of a pair need each other's
// LDS writes).  Diagnostic builds (-DF2_STAMPS=1) also sum the cycles waves spend in them.
#ifndef F2_STAMPS
#define F2_STAMPS 0
#endif
#if F2_STAMPS
__device__ unsigned long long f2_pair_wait[16][8];
#endif
__device__ __forceinline__ void pair_sync() {
#if F2_STAMPS
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if ((threadIdx.x & 63) == 0 && (blockIdx.x & 63) == 0 && (blockIdx.x >> 6) < 16)
    f2_pair_wait[blockIdx.x >> 6][threadIdx.x >> 6] += t1 - t0;
#else
  __syncthreads();
#endif
}

// forward: 16 reals per lane (slot e < 8 real part, e + 8 imaginary part) -> half spectrum in xr/xi
// (slot s: frequency k'(L, 4h + (s & 3)) + 512 (s >> 2)).  Contains two pair barriers: every wave of
// the workgroup calls it in lockstep.  T0 / T1: the pair's regions (wave 0 / wave 1).
// The exchange moves only what the partner needs: wave h combines at slots 4h + q, so wave 0 sends E_0 at
// slots 4..7 and wave 1 sends E_1 at slots 0..3 (4 writes and 4 reads per wave; its own 4 stay in registers).
template <int H, bool TRAIL>
__device__ __forceinline__ void combine_fwd(double (&xr)[8], double (&xi)[8], int lane, double2* Tm,
                                            const double2* Tp, const double2* tg) {
#pragma unroll
  for (int q = 0; q < 4; q++) Tm[64 * (4 * (1 - H) + q) + lane] = make_double2(xr[4 * (1 - H) + q], xi[4 * (1 - H) + q]);
  pair_sync();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int e = 4 * H + q;
    const double2 p = Tp[64 * e + lane];
    const double e0r = H ? p.x : xr[e], e0i = H ? p.y : xi[e];
    double tr = H ? xr[e] : p.x, ti = H ? xi[e] : p.y;
    cmul<false>(tr, ti, tg[G_WC + 256 * H + 64 * q + lane]);
    xr[q] = e0r + tr;
    xi[q] = e0i + ti;
    xr[q + 4] = e0r - tr;
    xi[q + 4] = e0i - ti;
  }
  if (TRAIL) pair_sync();
}
// TRAIL = false: the caller's next barrier comes before either wave of the pair writes the region the
// other one read (the partner's reads were at slots 4 (1 - h) + q of this wave's region)
template <bool TRAIL = true>
__device__ __forceinline__ void fwd_half(double (&xr)[8], double (&xi)[8], int h, int lane, TBase tb,
                                         double2* T0, double2* T1, const double2* tg) {
  double2* Tm = h ? T1 : T0;
  twist_slots<false>(xr, xi);
  dft512_fwd_t<true>(xr, xi, Tm, lane, tb, tg + (h ? G_A1 : G_A0), tg + G_B);
  if (__builtin_amdgcn_readfirstlane(h)) combine_fwd<1, TRAIL>(xr, xi, lane, T1, T0, tg);
  else combine_fwd<0, TRAIL>(xr, xi, lane, T0, T1, tg);
}

// inverse, first half: uncombine this wave's 4 slot pairs (slot 4h + q) into E_0 and E_1; keep E_h, send
// E_(1-h) to the partner through this wave's region, take the partner's E_h at slots 4(1-h) + q.  Two
// pair barriers.
template <int H, typename Mid>
__device__ __forceinline__ void uncombine_inv(double (&xr)[8], double (&xi)[8], int lane, double2* Tm,
                                              const double2* Tp, const double2* tg, Mid&& mid) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int e = 4 * H + q;
    const double lr = xr[q], li = xi[q], hr = xr[q + 4], hi = xi[q + 4];
    double dr = lr - hr, di = li - hi;
    cmul<true>(dr, di, tg[G_WC + 256 * H + 64 * q + lane]);
    const double sr = lr + hr, si = li + hi;  // E_0 at slot e; (dr, di) = E_1 at slot e
    Tm[64 * e + lane] = H ? make_double2(sr, si) : make_double2(dr, di);
    xr[e] = H ? dr : sr;
    xi[e] = H ? di : si;
  }
  pair_sync();
  mid();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int e = 4 * (1 - H) + q;
    const double2 v = Tp[64 * e + lane];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  pair_sync();
}
// mid(): run by every wave right after the exchange's first (workgroup-wide) barrier
template <typename Mid>
__device__ __forceinline__ void inv_exchange(double (&xr)[8], double (&xi)[8], int h, int lane, double2* T0,
                                             double2* T1, const double2* tg, Mid&& mid) {
  if (__builtin_amdgcn_readfirstlane(h)) uncombine_inv<1>(xr, xi, lane, T1, T0, tg, mid);
  else uncombine_inv<0>(xr, xi, lane, T0, T1, tg, mid);
}
__device__ __forceinline__ void inv_exchange(double (&xr)[8], double (&xi)[8], int h, int lane, double2* T0,
                                             double2* T1, const double2* tg) {
  inv_exchange(xr, xi, h, lane, T0, T1, tg, [] {});
}

// inverse, second half (wave-private): 512-point inverse + untwist -> reals (slot e < 8: re, e + 8: im)
__device__ __forceinline__ void inv_half(double (&xr)[8], double (&xi)[8], int h, int lane, TBase tb, double2* Tm,
                                         const double2* tg) {
  dft512_inv_t(xr, xi, Tm, lane, tb, tg + G_B, tg + (h ? G_I1 : G_I0));
  twist_slots<true>(xr, xi);
}

// ---------------------------------------------------------------------------------------------
// transform kernels (one polynomial per 2-wave workgroup): BSK conversion and the parity tests
__global__ __launch_bounds__(128) void fwd2k_kernel(const u64* __restrict__ in, double2* __restrict__ out,
                                                    const double2* __restrict__ tg, double scale) {
  __shared__ __attribute__((aligned(16))) double2 T[2][T_C64];
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64* src = in + (size_t)blockIdx.x * N2;
  double xr[8], xi[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    xr[e] = i64_to_f64(src[coef(h, lane, e)]);
    xi[e] = i64_to_f64(src[coef(h, lane, e + 8)]);
  }
  fwd_half(xr, xi, h, lane, TBase(lane), T[0], T[1], tg);
  double2* dst = out + (size_t)blockIdx.x * M2 + h * 512;
#pragma unroll
  for (int s = 0; s < 8; s++) dst[64 * s + lane] = make_double2(xr[s] * scale, xi[s] * scale);
}

__global__ __launch_bounds__(128) void inv2k_kernel(const double2* __restrict__ in, double* __restrict__ out,
                                                    const double2* __restrict__ tg) {
  __shared__ __attribute__((aligned(16))) double2 T[2][T_C64];
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const double2* src = in + (size_t)blockIdx.x * M2 + h * 512;
  double xr[8], xi[8];
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const double2 v = src[64 * s + lane];
    xr[s] = v.x;
    xi[s] = v.y;
  }
  inv_exchange(xr, xi, h, lane, T[0], T[1], tg);
  inv_half(xr, xi, h, lane, TBase(lane), T[h], tg);
  double* dst = out + (size_t)blockIdx.x * N2;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    dst[coef(h, lane, e)] = xr[e];
    dst[coef(h, lane, e + 8)] = xi[e];
  }
}

// ---------------------------------------------------------------------------------------------
// F2_PRIO: s_setprio 1 for waves 4-7 over the CMUX loop (56.6 -> 56.1 ms per 4096, same-box A/B)
#ifndef F2_PRIO
#define F2_PRIO 1
#endif
// F2_MACORDER = 1: transform both components, then one MAC per output column, both MACs before the
// inverses (35 spilled VGPRs: O_0, O_1, D_0, D_1 and the accumulators live together); 2 (default): the
// first inverse between the two MACs, no spills (round 2: 52.1 -> 51.2 ms per 4096, same-box A/B)
#ifndef F2_MACORDER
#define F2_MACORDER 2
#endif
// barrier trims of the order-2 loop: A (default) the second forward transform's trailing pair barrier
// (51.13 -> 51.02 ms); B the barrier before the next CMUX's column-0 load, C the one before the column-1
// load, the loads then issued inside the next exchange after its first barrier (B: +-0, C: +0.2 %, all
// three together 51.3 -> 51.8 ms; kept as switches)
#ifndef F2_TRIM_A
#define F2_TRIM_A 1
#endif
#ifndef F2_TRIM_B
#define F2_TRIM_B 0
#endif
#ifndef F2_TRIM_C
#define F2_TRIM_C 0
#endif

// the whole table first (every twiddle read: a per-lane base plus a 16-bit DS immediate offset), then
// the transpose scratch, then two BSK polynomials (K_{c,0}, K_{c,1} of the component in flight)
struct F2Shared {
  double2 tw[G_C64];           // 49,152 B (G_* layout)
  double2 T[F2_WAVES][T_C64];  // 73,728 B
  double2 K[2][M2];            // 32,768 B
};
typedef __attribute__((address_space(3))) const double lds_f64;
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const f64x2 lds_c64;  // one complex: a single ds_read_b128

// F2_ACC_AGPR: the two accumulator polynomials live in AGPRs between their uses (rotation and the
// accumulate after each inverse), moved by v_accvgpr_read / write, to take the 33 spilled VGPRs off
// scratch.  Rejected: with any AGPR in use at 2 waves / SIMD the allocator splits the unified 256 registers
// 128 / 128 and spills 58-72 VGPRs instead (hipcc ROCm 7.2; no source-level knob for the split)
#ifndef F2_ACC_AGPR
#define F2_ACC_AGPR 0
#endif
struct AccRegs {
  u32 lo[16], hi[16];
};
__device__ __forceinline__ void acc_put(AccRegs& s, const u64 (&v)[16]) {
#pragma unroll
  for (int e = 0; e < 16; e++) {
    asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(s.lo[e]) : "v"((u32)v[e]));
    asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(s.hi[e]) : "v"((u32)(v[e] >> 32)));
  }
}
__device__ __forceinline__ void acc_get(u64 (&v)[16], const AccRegs& s) {
#pragma unroll
  for (int e = 0; e < 16; e++) {
    u32 lo, hi;
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(lo) : "a"(s.lo[e]));
    asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(hi) : "a"(s.hi[e]));
    v[e] = ((u64)hi << 32) | lo;
  }
}

// BSK_i[c][0..1] (32 KB) into K: wave w loads the 1 KB blocks 4w .. 4w + 3 (wave-uniform scalar bases)
__device__ __forceinline__ void load_pair(const double2* __restrict__ bsk, int i, int c, F2Shared& sh, int wave_s,
                                          int lane) {
  constexpr int PER_WAVE = 2 * CHUNK_GLDS / F2_WAVES;
  const char* src = (const char*)(bsk + ((size_t)i * 4 + 2 * c) * M2) + wave_s * (PER_WAVE * 1024);
  char* dst = (char*)sh.K + wave_s * (PER_WAVE * 1024);
#pragma unroll
  for (int q = 0; q < PER_WAVE; q++)
    __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, 0, 0);
}

// (X^a acc - acc) of this wave's coefficients, decomposed: the pair's 2048-u64 image in LDS, written by
// both waves, read rotated.  Split layout (coefficient c at R[(c & 1) * 1024 + (c >> 1)]): every write
// and every rotated read is 64 consecutive u64, free of bank conflicts (the natural layout's stride-2
// accesses conflicted 4-way).  Two barriers.
__device__ __forceinline__ int rsplit(int c) { return ((c & 1) << 10) | ((c >> 1) & 1023); }
__device__ __forceinline__ void rotate_decompose(const u64 (&acc)[16], int a, int h, int lane, u64* R, int (&dig)[16]) {
#pragma unroll
  for (int e = 0; e < 16; e++) R[rsplit(coef(h, lane, e))] = acc[e];
  pair_sync();
  // (X^a v)[c] = (-1)^bit11(t) v[t mod 2048], t = c - a + 4096 (a < 4096)
  const int t0 = coef(h, lane, 0) + 2 * N2 - a;
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const int t = t0 + (coef(h, 0, e) - h);
    const u64 x = R[rsplit(t)];
    const u64 m = 0ull - (u64)((t >> 11) & 1);  // all ones iff negated
    const u64 y = ((x ^ m) - m) - acc[e];
    dig[e] = decomp_23x1_hi((u32)(y >> 32));
  }
  pair_sync();
}

// F2_ROT_OWN (default): the rotation image in split halves, half p (the parity-p coefficients) in the transpose area
// of the pair's wave p, so each wave writes only its own area: the barrier that guarded the partner's previous
// inverse transposes goes, and the rotated reads take the P-GATE form.  For this wave's coefficient c = 2 m + h
// (m = L + 64 e) the source c - a has the uniform parity p = (h - a) mod 2 and position (t >> 1) mod 1024 in half p,
// t >> 1 = L + K + 64 e with K = (h - a + 4096) >> 1; negated iff bit 10 of t >> 1 is set.  So: base u = (L + K) mod
// 1024, DS offset 512 e, the base 8 KB lower after the per-lane wrap, sign = bit 10 of (L + K) xor wrap.
#ifndef F2_ROT_OWN
#define F2_ROT_OWN 1
#endif
typedef __attribute__((address_space(3))) u64 lds_u64;
__device__ __forceinline__ void rotate_decompose_own(const u64 (&acc)[16], int a, int h, int lane, double2* Tm,
                                                     const double2* T0, const double2* T1, int (&dig)[16]) {
  u64* Tu = (u64*)Tm;
#pragma unroll
  for (int e = 0; e < 16; e++) Tu[64 * e + lane] = acc[e];
  pair_sync();
  const int p = (h - a) & 1;  // wave-uniform
  const int u0 = (lane + ((h - a + 4096) >> 1)) & 2047;
  const int u = u0 & 1023;
  const bool neg0 = u0 >= 1024;
  const u64* src = (const u64*)(p ? T1 : T0);
  const u32 a0 = (u32)(uintptr_t)(const lds_u64*)&src[u];
  const u32 a1 = a0 - 8192u;
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const bool wrap = u >= 1024 - 64 * e;
    const u64 x = ((const lds_u64*)(uintptr_t)(wrap ? a1 : a0))[64 * e];
    const u64 m = 0ull - (u64)(neg0 != wrap);  // all ones iff negated
    const u64 y = ((x ^ m) - m) - acc[e];
    dig[e] = decomp_23x1_hi((u32)(y >> 32));
  }
  pair_sync();
}

// LDS address of this wave's slot 0 in K, laundered: with K's absolute offset folded in, the MAC's
// reads would exceed the 16-bit DS immediate and each take a VGPR of its own
__device__ __forceinline__ lds_c64* kbase(const double2* kbuf, int h, int lane) {
  u32 a = (u32)(uintptr_t)(lds_f64*)&kbuf[h * 512 + lane];
  asm volatile("" : "+v"(a));
  return (lds_c64*)(uintptr_t)a;
}

// output column j of BSK_i (K_{0,j}, K_{1,j}: two 16 KB polynomials) into K[0], K[1]: waves 0-3 load the
// first, waves 4-7 the second, 4 x 1 KB each
// (dst: the key buffer K, or for column 1 the transpose area, free between the forward transforms'
// last exchange and the inverse transforms' first)
__device__ __forceinline__ void load_column(const double2* __restrict__ bsk, int i, int j, double2* kbuf,
                                            int wave_s, int lane) {
  constexpr int PER_WAVE = 2 * CHUNK_GLDS / F2_WAVES;
  const int c = wave_s >> 2, part = wave_s & 3;
  const char* src = (const char*)(bsk + ((size_t)i * 4 + 2 * c + j) * M2) + part * (PER_WAVE * 1024);
  char* dst = (char*)(kbuf + c * M2) + part * (PER_WAVE * 1024);
#pragma unroll
  for (int q = 0; q < PER_WAVE; q++)
    __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)(dst + q * 1024), 16, 0, 0);
}

// O = D_0 (.) K[0] + D_1 (.) K[1], the oracle's fma chain from (0, 0) (c = 0 first)
__device__ __forceinline__ void mac_column(lds_c64* kp, const double (&ar)[8], const double (&ai)[8],
                                           const double (&br)[8], const double (&bi)[8], double (&or_)[8],
                                           double (&oi)[8]) {
#pragma unroll
  for (int s = 0; s < 8; s++) {
    const f64x2 u = kp[64 * s], v = kp[M2 + 64 * s];
    or_[s] = __builtin_fma(ar[s], u.x, 0.0);
    or_[s] = __builtin_fma(-ai[s], u.y, or_[s]);
    oi[s] = __builtin_fma(ar[s], u.y, 0.0);
    oi[s] = __builtin_fma(ai[s], u.x, oi[s]);
    or_[s] = __builtin_fma(br[s], v.x, or_[s]);
    or_[s] = __builtin_fma(-bi[s], v.y, or_[s]);
    oi[s] = __builtin_fma(br[s], v.y, oi[s]);
    oi[s] = __builtin_fma(bi[s], v.x, oi[s]);
  }
}

// F2_STAMPS (diagnostic builds only, never the shipped library): s_memtime stamps at the phase
// boundaries of the CMUX loop, summed per wave of every 64th workgroup into f2_stamps[slot][wave][phase]
// (cdna_hip_programming.md, "In-kernel stamps"); read with tfhe_hip_debug_stamps.  Read the SHARES.
[[maybe_unused]] constexpr int F2_NPH = 12;
#if F2_STAMPS
__device__ unsigned long long f2_stamps[16][F2_WAVES][F2_NPH];
#define F2_STAMP(k)                                                                              \
  do {                                                                                           \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    unsigned long long _t;                                                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                     \
    __builtin_amdgcn_sched_barrier(0);                                                           \
    st_acc[k] += _t - st_prev;                                                                   \
    st_prev = _t;                                                                                \
  } while (0)
#else
#define F2_STAMP(k) \
  do {              \
  } while (0)
#endif

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(F2_THREADS, 1) void blind_rotate_fft2k_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tg, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) F2Shared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = wave & 1, pr = wave >> 1;
  const size_t b_raw = (size_t)blockIdx.x * F2_PAIRS + pr;
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding pairs run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  double2* T0 = sh.T[2 * pr];
  double2* T1 = sh.T[2 * pr + 1];
  double2* Tm = sh.T[wave];
  [[maybe_unused]] u64* R = (u64*)T0;  // 16 KB across the pair's two regions (F2_ROT_OWN = 0)
  const double2* tt = sh.tw;
  const TBase tb(lane);

  for (int q = threadIdx.x; q < G_C64; q += F2_THREADS) sh.tw[q] = tg[q];
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
#if F2_MACORDER
  load_column(bsk, 0, 0, &sh.K[0][0], wave_s, lane);
#else
  load_pair(bsk, 0, 0, sh, wave_s, lane);
#endif

  u64 accA[16], accB[16];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N2;
    const int s = (4096 - ms4096(ct[n])) & 4095;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      int d = coef(h, lane, e) - s;
      bool neg = false;
      if (d < 0) { d += N2; neg = !neg; }
      if (d < 0) { d += N2; neg = !neg; }
      const u64 v = gl_to_torus(lut[d]);
      accA[e] = 0;
      accB[e] = neg ? 0 - v : v;
    }
  }

#if F2_PRIO
  if (wave_s >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#if F2_MACORDER == 2
  // column order with the first inverse between the two MACs: O_0 = D_0 K_{0,0} + D_1 K_{1,0}, then
  // acc_0 += iFFT(O_0) while column 1 streams into the key buffer, then O_1 and its inverse.  At no point
  // are O_0 and O_1 live together (the column-1 MAC of order 1 held both beside D_0, D_1 and the
  // accumulators: 33 spilled VGPRs)
  for (int i = 0; i < n; i++) {
    const int a = ms4096(ct[i]);
    int dg[16];
    double d0r[8], d0i[8], xr[8], xi[8], o0r[8], o0i[8];
#if F2_ROT_OWN
    rotate_decompose_own(accA, a, h, lane, Tm, T0, T1, dg);
#else
    __syncthreads();  // the previous CMUX's inverse transforms are done with T
    rotate_decompose(accA, a, h, lane, R, dg);
#endif
#pragma unroll
    for (int e = 0; e < 8; e++) {
      d0r[e] = (double)dg[e];
      d0i[e] = (double)dg[e + 8];
    }
    fwd_half(d0r, d0i, h, lane, tb, T0, T1, tt);
#if F2_ROT_OWN
    rotate_decompose_own(accB, a, h, lane, Tm, T0, T1, dg);
#else
    rotate_decompose(accB, a, h, lane, R, dg);
#endif
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xr[e] = (double)dg[e];
      xi[e] = (double)dg[e + 8];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's share of column 0; fwd_half's barrier publishes it
    fwd_half<!F2_TRIM_A>(xr, xi, h, lane, tb, T0, T1, tt);  // the exchange below is the next barrier
    mac_column(kbase(&sh.K[0][0], h, lane), d0r, d0i, xr, xi, o0r, o0i);
#if F2_TRIM_C
    // column 1 into the key buffer under the first inverse, issued once every wave is past MAC 0 (the
    // exchange's first barrier)
    inv_exchange(o0r, o0i, h, lane, T0, T1, tt, [&] { load_column(bsk, i, 1, &sh.K[0][0], wave_s, lane); });
#else
    __syncthreads();  // every wave is done with column 0
    load_column(bsk, i, 1, &sh.K[0][0], wave_s, lane);  // column 1, under the first inverse
    inv_exchange(o0r, o0i, h, lane, T0, T1, tt);
#endif
    inv_half(o0r, o0i, h, lane, tb, Tm, tt);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      accA[e] += f64_to_torus_wide(o0r[e]);
      accA[e + 8] += f64_to_torus_wide(o0i[e]);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();  // column 1 visible
    {
      double o1r[8], o1i[8];
      mac_column(kbase(&sh.K[0][0], h, lane), d0r, d0i, xr, xi, o1r, o1i);
#if F2_TRIM_B
      // the next CMUX's column 0, once every wave is past MAC 1
      inv_exchange(o1r, o1i, h, lane, T0, T1, tt, [&] {
        if (i + 1 < n) load_column(bsk, i + 1, 0, &sh.K[0][0], wave_s, lane);
      });
#else
      __syncthreads();  // every wave is done with column 1
      if (i + 1 < n) load_column(bsk, i + 1, 0, &sh.K[0][0], wave_s, lane);
      inv_exchange(o1r, o1i, h, lane, T0, T1, tt);
#endif
      inv_half(o1r, o1i, h, lane, tb, Tm, tt);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        accB[e] += f64_to_torus_wide(o1r[e]);
        accB[e + 8] += f64_to_torus_wide(o1i[e]);
      }
    }
  }
#elif F2_MACORDER
  // both components are transformed first (D_0 held in registers, not the 64 registers of O), then
  // O_0 = D_0 K_{0,0} + D_1 K_{1,0} and O_1 = D_0 K_{0,1} + D_1 K_{1,1}: the key buffer holds output
  // column 0 (K_{0,0}, K_{1,0}); column 1 streams into the transpose area while MAC 0 runs
#if F2_STAMPS
  unsigned long long st_acc[F2_NPH] = {0}, st_prev;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
#endif
#if F2_ACC_AGPR
  AccRegs sA, sB;
  acc_put(sA, accA);
  acc_put(sB, accB);
#endif
  for (int i = 0; i < n; i++) {
    const int a = ms4096(ct[i]);
    int dg[16];
    double d0r[8], d0i[8], xr[8], xi[8], o0r[8], o0i[8], o1r[8], o1i[8];
    F2_STAMP(11);
    __syncthreads();  // the previous CMUX's inverse transforms are done with T
    F2_STAMP(0);
#if F2_ACC_AGPR
    acc_get(accA, sA);
#endif
    rotate_decompose(accA, a, h, lane, R, dg);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      d0r[e] = (double)dg[e];
      d0i[e] = (double)dg[e + 8];
    }
    F2_STAMP(1);
    fwd_half(d0r, d0i, h, lane, tb, T0, T1, tt);
    F2_STAMP(2);
#if F2_ACC_AGPR
    acc_get(accB, sB);
#endif
    rotate_decompose(accB, a, h, lane, R, dg);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xr[e] = (double)dg[e];
      xi[e] = (double)dg[e + 8];
    }
    F2_STAMP(3);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's share of column 0; fwd_half's barriers publish it
    F2_STAMP(4);
    fwd_half(xr, xi, h, lane, tb, T0, T1, tt);
    F2_STAMP(5);
    double2* const kt = &sh.T[0][0];
    load_column(bsk, i, 1, kt, wave_s, lane);  // column 1 into the (now idle) transpose area, under MAC 0
    mac_column(kbase(&sh.K[0][0], h, lane), d0r, d0i, xr, xi, o0r, o0i);
    F2_STAMP(6);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();  // column 1 visible; every wave is done with column 0
    F2_STAMP(7);
    if (i + 1 < n) load_column(bsk, i + 1, 0, &sh.K[0][0], wave_s, lane);
    mac_column(kbase(kt, h, lane), d0r, d0i, xr, xi, o1r, o1i);
    __syncthreads();  // every wave is done with column 1: the transpose area is free again
    F2_STAMP(8);
    inv_exchange(o0r, o0i, h, lane, T0, T1, tt);
    inv_half(o0r, o0i, h, lane, tb, Tm, tt);
#if F2_ACC_AGPR
    acc_get(accA, sA);
#endif
#pragma unroll
    for (int e = 0; e < 8; e++) {
      accA[e] += f64_to_torus_wide(o0r[e]);
      accA[e + 8] += f64_to_torus_wide(o0i[e]);
    }
#if F2_ACC_AGPR
    acc_put(sA, accA);
#endif
    F2_STAMP(9);
    __syncthreads();  // the partner's inverse transposes are done with its region
    F2_STAMP(10);
    inv_exchange(o1r, o1i, h, lane, T0, T1, tt);
    inv_half(o1r, o1i, h, lane, tb, Tm, tt);
#if F2_ACC_AGPR
    acc_get(accB, sB);
#endif
#pragma unroll
    for (int e = 0; e < 8; e++) {
      accB[e] += f64_to_torus_wide(o1r[e]);
      accB[e + 8] += f64_to_torus_wide(o1i[e]);
    }
#if F2_ACC_AGPR
    acc_put(sB, accB);
#endif
  }
#if F2_ACC_AGPR
  acc_get(accA, sA);
  acc_get(accB, sB);
#endif
#if F2_STAMPS
  F2_STAMP(11);
  if ((blockIdx.x & 63) == 0 && lane == 0 && (blockIdx.x >> 6) < 16)
    for (int k = 0; k < F2_NPH; k++) f2_stamps[blockIdx.x >> 6][wave][k] = st_acc[k];
#endif
#else
  for (int i = 0; i < n; i++) {
    const int a = ms4096(ct[i]);
    int dg[16];
    double xr[8], xi[8], o0r[8], o0i[8], o1r[8], o1i[8];
    __syncthreads();  // the previous CMUX's inverse transforms are done with T
    rotate_decompose(accA, a, h, lane, R, dg);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xr[e] = (double)dg[e];
      xi[e] = (double)dg[e + 8];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's share of K_{0,*}; fwd_half's barriers publish it
    fwd_half(xr, xi, h, lane, tb, T0, T1, tt);
    {  // MAC, c = 0 (oracle order: from (0, 0)); slot s of this wave = BSK index h * 512 + 64 s + L
      lds_c64* kp = kbase(&sh.K[0][0], h, lane);
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const f64x2 k0 = kp[64 * s], k1 = kp[M2 + 64 * s];  // whole complexes: two separate b64 reads 16 B apart conflict 2-way
        const double k0r = k0.x, k0i = k0.y, k1r = k1.x, k1i = k1.y;
        o0r[s] = __builtin_fma(xr[s], k0r, 0.0);
        o0r[s] = __builtin_fma(-xi[s], k0i, o0r[s]);
        o0i[s] = __builtin_fma(xr[s], k0i, 0.0);
        o0i[s] = __builtin_fma(xi[s], k0r, o0i[s]);
        o1r[s] = __builtin_fma(xr[s], k1r, 0.0);
        o1r[s] = __builtin_fma(-xi[s], k1i, o1r[s]);
        o1i[s] = __builtin_fma(xr[s], k1i, 0.0);
        o1i[s] = __builtin_fma(xi[s], k1r, o1i[s]);
      }
    }
    __syncthreads();  // every wave is done with K_{0,*}
    load_pair(bsk, i, 1, sh, wave_s, lane);
    rotate_decompose(accB, a, h, lane, R, dg);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xr[e] = (double)dg[e];
      xi[e] = (double)dg[e + 8];
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): K_{1,*}
    fwd_half(xr, xi, h, lane, tb, T0, T1, tt);

    {  // MAC, c = 1
      lds_c64* kp = kbase(&sh.K[0][0], h, lane);
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const f64x2 k0 = kp[64 * s], k1 = kp[M2 + 64 * s];  // whole complexes: two separate b64 reads 16 B apart conflict 2-way
        const double k0r = k0.x, k0i = k0.y, k1r = k1.x, k1i = k1.y;
        o0r[s] = __builtin_fma(xr[s], k0r, o0r[s]);
        o0r[s] = __builtin_fma(-xi[s], k0i, o0r[s]);
        o0i[s] = __builtin_fma(xr[s], k0i, o0i[s]);
        o0i[s] = __builtin_fma(xi[s], k0r, o0i[s]);
        o1r[s] = __builtin_fma(xr[s], k1r, o1r[s]);
        o1r[s] = __builtin_fma(-xi[s], k1i, o1r[s]);
        o1i[s] = __builtin_fma(xr[s], k1i, o1i[s]);
        o1i[s] = __builtin_fma(xi[s], k1r, o1i[s]);
      }
    }
    __syncthreads();  // every wave is done with K_{1,*} and with the pair exchanges
    if (i + 1 < n) load_pair(bsk, i + 1, 0, sh, wave_s, lane);
    inv_exchange(o0r, o0i, h, lane, T0, T1, tt);
    inv_half(o0r, o0i, h, lane, tb, Tm, tt);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      accA[e] += f64_to_torus_wide(o0r[e]);
      accA[e + 8] += f64_to_torus_wide(o0i[e]);
    }
    __syncthreads();  // the partner's inverse transposes are done with its region
    inv_exchange(o1r, o1i, h, lane, T0, T1, tt);
    inv_half(o1r, o1i, h, lane, tb, Tm, tt);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      accB[e] += f64_to_torus_wide(o1r[e]);
      accB[e + 8] += f64_to_torus_wide(o1i[e]);
    }
  }

#endif

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * (2 * N2);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      oa[coef(h, lane, e)] = accA[e];
      oa[N2 + coef(h, lane, e)] = accB[e];
    }
  }
  if (WRITE_BIG) {
    // sample extraction at degree 0: a'_0 = A[0], a'_j = -A[N-j], b' = B[0]
    u64* ob = out_big + b * (size_t)(N2 + 1);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int c = coef(h, lane, e);
      if (c == 0) ob[0] = accA[e];
      else ob[N2 - c] = 0 - accA[e];
    }
    if (h == 0 && lane == 0) ob[N2] = accB[0];
  }
}

// ---------------------------------------------------------------------------------------------
// Latency-mode blind rotation at N = 2048 (small batches: the radix layer's lockstep levels): ONE
// ciphertext per workgroup of 8 waves; the accumulator lives in LDS (split by parity), so no wave
// pair exchanges the rotation.  Per CMUX:
//   A  waves 0..3: wave (c, h) rotates + decomposes the parity-h coefficients of component c,
//      transforms its 512-point half and, after one pair exchange, writes its half of the combined
//      spectrum D_c to F[c]                                           (2 transforms in parallel)
//   B  all 8 waves: O_j = D_0 (.) BSK_i[0][j] then + D_1 (.) BSK_i[1][j] (the oracle's fma chain) on
//      4 of the 16 slots each (j = wave >> 2); key words prefetched into registers before phase A
//   C  waves 0..3: wave (j, h) uncombines O_j straight from LDS into E_h, runs the 512-point inverse
//      and adds the parity-h coefficients to acc_j                      (2 inverses in parallel)
// Five barriers per CMUX.  LDS: table 48 KB | acc 32 KB | F 32 KB | 4 transpose areas 36 KB (O
// aliases them between phase B and the uncombine) = 148 KB.
constexpr int F2L_THREADS = 512;
constexpr int F2L_MAXN = 1024;  // rotation amounts staged in LDS up to this LWE dimension (global reads above)
// F2L_PREFETCH: the key words of CMUX i + 1 requested while CMUX i runs (two register sets, loop unrolled by 2)
#ifndef F2L_PREFETCH
#define F2L_PREFETCH 1
#endif
struct F2LatShared {
  double2 tw[G_C64];
  u64 A[2][N2];        // split layout: coefficient c at (c & 1) * 1024 + (c >> 1)
  double2 F[2][M2];    // spectra, device order (index h * 512 + 64 s + L)
  double2 T[4][T_C64];  // transposes; O_0, O_1 (2 x 1024 complex) alias T[0..3] after phase A
  unsigned short ab[F2L_MAXN];  // ms4096(ct[i]) for every CMUX
};

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(F2L_THREADS, 1) void blind_rotate_fft2k_lat_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tg, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) F2LatShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = blockIdx.x;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  const TBase tb(lane);
  const double2* tt = sh.tw;
  double2* O = sh.T[0];  // 2 x 1024 complex across the four transpose areas

  for (int q = threadIdx.x; q < G_C64; q += F2L_THREADS) sh.tw[q] = tg[q];
  for (int q = threadIdx.x; q < n && q < F2L_MAXN; q += F2L_THREADS) sh.ab[q] = (unsigned short)ms4096(ct[q]);
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N2;
    const int s = (4096 - ms4096(ct[n])) & 4095;
    for (int q = threadIdx.x; q < N2; q += F2L_THREADS) {
      int d = q - s;
      bool neg = false;
      if (d < 0) { d += N2; neg = !neg; }
      if (d < 0) { d += N2; neg = !neg; }
      const u64 v = gl_to_torus(lut[d]);
      sh.A[0][rsplit(q)] = 0;
      sh.A[1][rsplit(q)] = neg ? 0 - v : v;
    }
  }
  __syncthreads();

  const int j = wave >> 2, sb = (wave & 3) * 4;  // phase B: output j, slots sb .. sb + 3 of 16
  const int c = (wave >> 1) & 1, h = wave & 1;   // phases A / C (waves 0..3): component or output, parity
  auto load_key = [&](int i, double2 (&kv)[2][4]) {
#pragma unroll
    for (int cc = 0; cc < 2; cc++)
#pragma unroll
      for (int t = 0; t < 4; t++) kv[cc][t] = bsk[((size_t)(i * 2 + cc) * 2 + j) * M2 + 64 * (sb + t) + lane];
  };
  auto cmux = [&](int i, const double2 (&kv)[2][4]) {
    const int a = i < F2L_MAXN ? (int)sh.ab[i] : ms4096(ct[i]);
    // ---- phase A
    double xr[8], xi[8];
    if (wave < 4) {
      const u64* acc = sh.A[c];
      const int t0 = coef(h, lane, 0) + 2 * N2 - a;
#pragma unroll
      for (int e = 0; e < 8; e++) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
          const int ee = e + 8 * u;
          const int t = t0 + (coef(h, 0, ee) - h);
          const u64 x = acc[rsplit(t)];
          const u64 m = 0ull - (u64)((t >> 11) & 1);
          const u64 y = ((x ^ m) - m) - acc[rsplit(coef(h, lane, ee))];
          const double dv = (double)decomp_23x1_hi((u32)(y >> 32));
          if (u == 0) xr[e] = dv;
          else xi[e] = dv;
        }
      }
      twist_slots<false>(xr, xi);
      dft512_fwd_t<true>(xr, xi, sh.T[wave], lane, tb, tt + (h ? G_A1 : G_A0), tt + G_B);
#pragma unroll
      for (int e = 0; e < 8; e++) sh.T[wave][64 * e + lane] = make_double2(xr[e], xi[e]);
    }
    __syncthreads();
    if (wave < 4) {
      const double2* T0 = sh.T[2 * c];
      const double2* T1 = sh.T[2 * c + 1];
      double2* F = sh.F[c] + h * 512;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int e = 4 * h + q;
        const double2 e0 = T0[64 * e + lane], e1 = T1[64 * e + lane];
        double tr = e1.x, ti = e1.y;
        cmul<false>(tr, ti, tt[G_WC + 256 * h + 64 * q + lane]);
        F[64 * q + lane] = make_double2(e0.x + tr, e0.y + ti);
        F[64 * (q + 4) + lane] = make_double2(e0.x - tr, e0.y - ti);
      }
    }
    __syncthreads();
    // ---- phase B (O overwrites the transpose areas: every exchange read is done)
#pragma unroll
    for (int t = 0; t < 4; t++) {
      const int q = 64 * (sb + t) + lane;
      const double2 d0 = sh.F[0][q], d1 = sh.F[1][q], k0 = kv[0][t], k1 = kv[1][t];
      double re = __builtin_fma(d0.x, k0.x, 0.0);
      re = __builtin_fma(-d0.y, k0.y, re);
      double im = __builtin_fma(d0.x, k0.y, 0.0);
      im = __builtin_fma(d0.y, k0.x, im);
      re = __builtin_fma(d1.x, k1.x, re);
      re = __builtin_fma(-d1.y, k1.y, re);
      im = __builtin_fma(d1.x, k1.y, im);
      im = __builtin_fma(d1.y, k1.x, im);
      O[j * M2 + q] = make_double2(re, im);
    }
    __syncthreads();
    // ---- phase C: uncombine O_j into E_h (all 8 slots of the 512-point half), then the inverse
    if (wave < 4) {
      const double2* Oj = O + c * M2;  // here c = output j
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const int hh = e >> 2, q = e & 3;
        const double2 lo = Oj[hh * 512 + 64 * q + lane], hi = Oj[hh * 512 + 64 * (q + 4) + lane];
        if (h == 0) {
          xr[e] = lo.x + hi.x;
          xi[e] = lo.y + hi.y;
        } else {
          double dr = lo.x - hi.x, di = lo.y - hi.y;
          cmul<true>(dr, di, tt[G_WC + 256 * hh + 64 * q + lane]);
          xr[e] = dr;
          xi[e] = di;
        }
      }
    }
    __syncthreads();  // O is read before the inverse transposes overwrite the areas
    if (wave < 4) {
      inv_half(xr, xi, h, lane, tb, sh.T[wave], tt);
      u64* acc = sh.A[c];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        acc[rsplit(coef(h, lane, e))] += f64_to_torus_wide(xr[e]);
        acc[rsplit(coef(h, lane, e + 8))] += f64_to_torus_wide(xi[e]);
      }
    }
    __syncthreads();
  };
#if F2L_PREFETCH
  double2 kva[2][4], kvb[2][4];
  load_key(0, kva);
  for (int i = 0; i < n; i += 2) {
    if (i + 1 < n) load_key(i + 1, kvb);
    cmux(i, kva);
    if (i + 1 >= n) break;
    if (i + 2 < n) load_key(i + 2, kva);
    cmux(i + 1, kvb);
  }
#else
  for (int i = 0; i < n; i++) {
    double2 kv[2][4];
    load_key(i, kv);
    cmux(i, kv);
  }
#endif

  if (WRITE_ACC) {
    u64* oa = out_acc + b * (2 * N2);
    for (int q = threadIdx.x; q < 2 * N2; q += F2L_THREADS) oa[q] = sh.A[q >> 11][rsplit(q & (N2 - 1))];
  }
  if (WRITE_BIG) {  // sample extraction at degree 0
    u64* ob = out_big + b * (size_t)(N2 + 1);
    for (int q = threadIdx.x; q <= N2; q += F2L_THREADS)
      ob[q] = q == N2 ? sh.A[1][0] : q == 0 ? sh.A[0][0] : 0 - sh.A[0][rsplit(N2 - q)];
  }
}

__global__ void sample_extract_torus2k_kernel(const u64* __restrict__ acc, size_t B, u64* __restrict__ out) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * (N2 + 1)) return;
  const size_t b = gid / (N2 + 1);
  const int j = (int)(gid % (N2 + 1));
  const u64* A = acc + b * (2 * N2);
  out[gid] = j == N2 ? A[N2] : j == 0 ? A[0] : 0 - A[N2 - j];
}

}  // namespace fft2k

hipError_t launch_sample_extract_torus2k(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (fft2k::N2 + 1);
  hipLaunchKernelGGL(fft2k::sample_extract_torus2k_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc,
                     B, out);
  return hipGetLastError();
}

size_t fft2k_tables_len() { return 2 * fft2k::G_C64; }

void make_fft2k_tables(double* t) {
  using namespace fft2k;
  constexpr int Mh = 512;
  for (uint32_t e = 0; e < 8; e++)
    for (uint32_t L = 0; L < 64; L++) {
      const int q = 64 * e + L;
      fft_twiddle((8 * (L & 7) * e) % Mh, Mh, &t[2 * (G_B + q)], &t[2 * (G_B + q) + 1]);
      for (uint32_t h = 0; h < 2; h++) {
        const int a = (h ? G_A1 : G_A0) + q, i = (h ? G_I1 : G_I0) + q;
        fft_twiddle((L * (8 * e + 2) + h) % 4096, 4096, &t[2 * a], &t[2 * a + 1]);
        fft_twiddle((((L & 7) + 8 * e) * (8 * (L >> 3) + 2) + h) % 4096, 4096, &t[2 * i], &t[2 * i + 1]);
      }
    }
  for (int h = 0; h < 2; h++)
    for (int q = 0; q < 4; q++)
      for (int L = 0; L < 64; L++) {
        const int k = (L >> 3) + 8 * (L & 7) + 64 * (4 * h + q);
        const int o = G_WC + 256 * h + 64 * q + L;
        fft_twiddle((uint32_t)k, 1024, &t[2 * o], &t[2 * o + 1]);
      }
}

hipError_t launch_bsk_to_fourier2k(const u64* bsk_std, double* bsk_f, size_t polys, const double* tw, hipStream_t s) {
  if (polys == 0) return hipSuccess;
  hipLaunchKernelGGL(fft2k::fwd2k_kernel, dim3((unsigned)polys), dim3(128), 0, s, bsk_std, (double2*)bsk_f,
                     (const double2*)tw, 0x1p-10);
  return hipGetLastError();
}

hipError_t launch_fft2k_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fft2k::fwd2k_kernel, dim3((unsigned)count), dim3(128), 0, s, in, (double2*)out,
                     (const double2*)tw, 1.0);
  return hipGetLastError();
}

hipError_t launch_fft2k_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fft2k::inv2k_kernel, dim3((unsigned)count), dim3(128), 0, s, (const double2*)in, out,
                     (const double2*)tw);
  return hipGetLastError();
}

#if F2_STAMPS
hipError_t read_fft2k_stamps(unsigned long long* out) {  // 16 x 8 x F2_NPH, then 16 x 8 pair-barrier waits
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(fft2k::f2_stamps), sizeof(fft2k::f2_stamps), 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(out + 16 * 8 * fft2k::F2_NPH, HIP_SYMBOL(fft2k::f2_pair_wait), sizeof(fft2k::f2_pair_wait), 0,
                             hipMemcpyDeviceToHost);
}
#endif

hipError_t launch_blind_rotate_fft2k(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                     int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                     hipStream_t s, size_t latency_max_batch) {
  using namespace fft2k;
  if (B == 0) return hipSuccess;
  const double2 *bk = (const double2*)bsk_f, *t = (const double2*)tw;
  if (B <= latency_max_batch) {
    dim3 grid((unsigned)B), block(F2L_THREADS);
    if (out_acc && out_big)
      hipLaunchKernelGGL((blind_rotate_fft2k_lat_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    else if (out_acc)
      hipLaunchKernelGGL((blind_rotate_fft2k_lat_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts,
                         lut_index, n_lut, bk, t, out_big, out_acc);
    else
      hipLaunchKernelGGL((blind_rotate_fft2k_lat_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts,
                         lut_index, n_lut, bk, t, out_big, out_acc);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((B + F2_PAIRS - 1) / F2_PAIRS)), block(F2_THREADS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bk, t, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bk, t, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bk, t, out_big, out_acc);
  return hipGetLastError();
}

}  // namespace tfhe
