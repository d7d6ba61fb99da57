// pbs_fft2k.hip — P-FHEVM (N = 2048, k = 1, PBS 2^23 x 1) blind rotation with ONE wave per polynomial component
// (round 4): the 1024-point transform of fft1k.h, restated in oracle/fft_oracle.c (fft1k_fwd / fft1k_inv).
//
// Batch mode (round 4): workgroup = 4 waves = 2 ciphertexts x 2 components, TWO workgroups per CU (80 KB of LDS
// each: the 16 KB pass-A table + 4 skewed 16 KB areas, fft1k.h), so the barriers of one workgroup overlap the other's
// work; latency mode: 8 waves, CTS = 2 (below).  Waves w < 2 CTS are the transform waves (p, c) = (w >> 1, w & 1),
// each holding component c of ciphertext p (2048 u64 = 32 per lane, registers).
// Per CMUX i:
//   transform waves: (X^a acc_c - acc_c) through the wave's LDS area (rotation by DS offsets), 23-bit digits, the
//     forward transform (one LDS transpose), the spectrum D_c stored to the area [slot][lane]
//   barrier
//   MAC, all waves: wave w owns 16 / NW slots of every ciphertext of the workgroup,
//     O_j = D_0 (.) K_{0,j} + D_1 (.) K_{1,j}  (the oracle's fma chain from (0, 0), c = 0 first)
//     with the key words of those slots in registers (two slots requested at the CMUX start, the others when the
//     MAC starts; shared by the CTS ciphertexts), O_j written over D_j in the areas
//   barrier
//   transform waves: O_c from the own area, the inverse transform, acc_c += rint mod 2^64 (two-split form: the
//     23-bit digits give |x| up to 2^106)
// Two barriers per CMUX (the round-1..3 two-wave kernel had five to six: 512-point halves + a combine exchange per
// transform) and no wave waits for a partner mid-transform.  In latency mode (CTS = 2: four transform waves, one per
// SIMD, and four MAC-only waves) a workgroup takes two ciphertexts at the per-CMUX latency of one.  LDS: pass A table
// 16 KB (first, so an area's base minus 16 KB stays inside the block for the rotation's wrapped reads) | 2 CTS areas
// x 16 KB.  (Rounds 1-3 / early round 4: 4 ciphertexts x 8 waves, 8 padded 17 KB areas = 152 KB, one workgroup per CU:
// 45.8 ms per 4096; two workgroups per CU 44.4 ms, with the priority scheme below 42.8 ms,
// profiles/r04i_fhevm_2wg_ab.txt.)
#include "fft1k.h"
#include "pbs_kernels.h"

namespace tfhe {
namespace fft1k {

constexpr int N2 = 2048;

__device__ __forceinline__ int ms4096(u64 x) { return (int)((((x >> 51) + 1) >> 1) & 4095u); }
// tfhe-rs SignedDecomposer 2^23 x 1 on the high word (pbs_fft2k.hip: decomp_23x1_hi; tests/test_fft.py)
__device__ __forceinline__ int dig23(u32 hi) {
  // ((((hi + 2^8) >> 9) + 2^22 - 1) mod 2^23) - (2^22 - 1): the offset folded in before the shift (a multiple of 2^9
  // there), the mod 2^23 is the u32 wrap after >> 9 -- 3 VALU instead of 5, the same value
  return (int)((hi + (256u + (0x3FFFFFu << 9))) >> 9) - 0x3FFFFF;
}
// -dig23(hi) in 2 VALU: dig23(h) = ceil((h - 255) / 512) in the signed reading of h with the digit range
// (-2^22, 2^22], so -dig23(h) = floor((255 - h) / 512) = (int)(255 - h) >> 9 (the i32 wrap of 255 - h lands exactly
// the tie h in [2^31 - 256, 2^31 + 256) on -2^22); checked for all 2^32 words.  With F1_NEGDIG the transforms run on
// the negated digits against negated key spectra (launch_bsk_to_fourier2k), and every product of the MAC -- digit
// term times key term -- is the same double, so the accumulators do not change by a bit.
__device__ __forceinline__ int dig23_neg(u32 hi) { return (int)(255u - hi) >> 9; }
#ifndef F1_NEGDIG
#define F1_NEGDIG 1
#endif
typedef __attribute__((address_space(3))) u64 lds_u64;
#ifndef F1_KPF
#define F1_KPF 0
#endif
// F1_PRIO 3 (default since late round 4): in the two-workgroup batch kernel the workgroups of the second dispatch
// half (blockIdx bit 8: with 256 CUs, the second workgroup each CU receives first) run at the higher wave
// priority, so the two workgroups of a CU drift apart instead of reaching their barriers together:
// 44.24 -> 43.35 ms per 4096 on the same box (profiles/r04i_fhevm_2wg_ab.txt).  1: the MAC-only waves of the
// 8-wave form; 0: none.
#ifndef F1_PRIO
#define F1_PRIO 3
#endif
// F1_MACPRIO 1 (default): every wave runs the short MAC phase at the top priority and then returns to its
// workgroup's F1_PRIO level, so a CU's MAC phases are not stalled behind the other workgroup's transforms:
// 43.43 -> 42.77 ms per 4096 on the same box (profiles/r04i_fhevm_2wg_ab.txt)
#ifndef F1_MACPRIO
#define F1_MACPRIO 1
#endif
#ifndef F1_PRIO_ASM
#define F1_PRIO_ASM 0
#endif
#ifndef F1_STAGGER
#define F1_STAGGER 0
#endif
#ifndef F1_PRIO_SH
#define F1_PRIO_SH 0
#endif
#ifndef F1_TAILWG
#define F1_TAILWG 512
#endif
#ifndef F1_PAIRMAC
#define F1_PAIRMAC 0
#endif
#ifndef F1_PAIRMAC_KG
#define F1_PAIRMAC_KG 2
#endif

// F1_LDSBAR (A/B, round 6): the CMUX's two barriers wait for LDS only (s_waitcnt lgkmcnt(0) + s_barrier) instead of
// __syncthreads' vmcnt(0) as well, so key words requested ahead (F1_KPF) stay in flight across them
#ifndef F1_LDSBAR
#define F1_LDSBAR 0
#endif
__device__ __forceinline__ void f1_barrier() {
#if F1_LDSBAR
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
}

template <int CTS>
struct F1Shared {
  double2 ta[M1];                 // pass A table (K_TA)
  double2 area[2 * CTS][AREA_C64];
};

__device__ __forceinline__ void load_ta(double2* ta, const double2* __restrict__ tg) {
  for (int q = threadIdx.x; q < M1; q += blockDim.x) ta[q] = tg[K_TA + q];
}

// (X^a v - v) through the area, then 23-bit digits as doubles: xr[e] <- coefficient L + 64 e, xi[e] <- + 1024
// F1_ROT_UNIFORM 1 (default since round 5): every per-slot decision wave-uniform, as pbs_fft.hip's FFT_ROT_UNIFORM
// (a = 2048 s + 64 A + r; the image is W = X^r v, only slot 31 of the lanes L + r >= 64 wraps on the write; slot e
// reads W[L + 64 (e - A)] for e >= A, -W[L + 64 (e - A + 32)] for e < A, sign xor s): 10 VALU per coefficient with
// dig23 instead of 14, the same values
#ifndef F1_ROT_UNIFORM
#define F1_ROT_UNIFORM 1
#endif
#ifndef F1_ROT_FOLD
#define F1_ROT_FOLD 1
#endif
// F1_Y32 1 (round 5): the keys' spectra carry 2^-32 (scale 2^-42 at conversion), so the inverse transform returns
// y = x * 2^-32 bit for bit and the accumulator update starts at floor(y) (fft512.h: torus_acc_add_wide_y)
#ifndef F1_Y32
#define F1_Y32 1
#endif
__device__ __forceinline__ void rotate_digits(const u64 (&v)[32], int a, int lane, double2* area, double (&xr)[16],
                                              double (&xi)[16]) {
  u64* Tu = (u64*)area;
#if F1_ROT_UNIFORM
  a = __builtin_amdgcn_readfirstlane(a);  // ms4096(ct[i]): the same for every lane
  const int A = (a >> 6) & 31, r = a & 63;
  const bool sgn = a >= 2048;
  {
    const u32 wb = (u32)(uintptr_t)(lds_u64*)&Tu[lane + r];
#pragma unroll
    for (int e = 0; e < 31; e++) ((lds_u64*)(uintptr_t)wb)[64 * e] = v[e];
    const bool w31 = lane + r >= 64;  // coefficient 1984 + L + r >= 2048: to L + r - 64, negated
    const u32 a31 = w31 ? wb + 1984u * 8u - 16384u : wb + 1984u * 8u;
    *(lds_u64*)(uintptr_t)a31 = w31 ? 0 - v[31] : v[31];
  }
  lds_order();
  const u32 rb = (u32)(uintptr_t)(lds_u64*)&Tu[lane] - 512u * (u32)A;  // >= area - 15.5 KB: the table lies below
  // bit e of wmask: slot e reads the wrapped part (e < A); bit e of mbits: slot e negated.  Bit-field extracts of
  // these SGPR words keep every per-slot decision scalar (a compare would be rebuilt as a per-lane select)
  const u32 wmask = (1u << A) - 1u;
  const u32 mbits = __builtin_amdgcn_readfirstlane(wmask ^ (sgn ? ~0u : 0u));
#pragma unroll
  for (int e = 0; e < 32; e++) {
    // s_bfe_i32 (0 or -1) in inline asm: hipcc's known-bits treat the width-1 sbfe builtin as non-negative and drop
    // the sign extension (a probe kernel stores hi = 0 for it)
    int m32;
    asm("s_bfe_i32 %0, %1, %2" : "=s"(m32) : "s"(mbits), "i"(e | (1 << 16)));
    const u64 M = (u64)(long long)m32;
    const u64 x = ((const lds_u64*)(uintptr_t)(rb + (__builtin_amdgcn_ubfe(wmask, e, 1) << 14)))[64 * e];
#if F1_NEGDIG && F1_ROT_FOLD
    // 255 - hi(y) = hi(~y) + 256 = hi((v + M + 2^40 - 1) - (x ^ M)): the offset rides in the scalar M, so the negated
    // digit is one arithmetic shift of the high word (one VALU fewer per coefficient, the same value)
    const u64 Mz = M + ((1ull << 40) - 1);
    const double d = (double)((int)(u32)(((v[e] + Mz) - (x ^ M)) >> 32) >> 9);
#elif F1_NEGDIG
    const u64 y = (x ^ M) - (v[e] + M);
    const double d = (double)dig23_neg((u32)(y >> 32));
#else
    const u64 y = (x ^ M) - (v[e] + M);
    const double d = (double)dig23((u32)(y >> 32));
#endif
    if (e < 16) xr[e] = d;
    else xi[e - 16] = d;
  }
  lds_order();
#else
#pragma unroll
  for (int e = 0; e < 32; e++) Tu[64 * e + lane] = v[e];
  lds_order();
  const int t0 = (lane - a) & 4095;  // a < 4096
  const int u = t0 & 2047;
  const bool neg0 = t0 >= 2048;
  const u32 a0 = (u32)(uintptr_t)(lds_u64*)&Tu[u];
  const u32 a1 = a0 - 16384u;        // wrapped reads: the image 16 KB lower
#pragma unroll
  for (int e = 0; e < 32; e++) {
    const bool wrap = u >= 2048 - 64 * e;
    const u64 x = ((const lds_u64*)(uintptr_t)(wrap ? a1 : a0))[64 * e];
    const u64 m = 0ull - (u64)(neg0 != wrap);  // all ones iff negated
    const u64 y = ((x ^ m) - m) - v[e];
    const double d = (double)(F1_NEGDIG ? dig23_neg((u32)(y >> 32)) : dig23((u32)(y >> 32)));
    if (e < 16) xr[e] = d;
    else xi[e - 16] = d;
  }
  lds_order();
#endif
}

// NW waves per workgroup: 8 (the MAC spread over 8 waves, 2 slots each) or 2 CTS (every wave a transform wave,
// 16 / NW slots each; with CTS = 2 and 16 KB areas two workgroups share a CU)
#ifndef FFT_WGTIME
#define FFT_WGTIME 0
#endif
#if FFT_WGTIME
// diagnostic build only (as pbs_fft.hip): per-workgroup start / end, HW_ID, XCC_ID of the last launch
__device__ unsigned long long g_wgt2k[4 * 16384];
#endif
template <int CTS, int NW, bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(64 * NW, 8 / NW) void blind_rotate_fft2k_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tg, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) F1Shared<CTS> sh;
#if FFT_WGTIME
  const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const bool tw_wave = wave_s < 2 * CTS;
  const int c = wave & 1, p = tw_wave ? wave >> 1 : 0;
  [[maybe_unused]] const int c_u = wave_s & 1;  // wave-uniform c (scalar branches)
  const size_t b_raw = (size_t)blockIdx.x * CTS + p;
  const bool live = tw_wave && b_raw < B;
  const size_t b = b_raw < B ? b_raw : B - 1;  // padding waves run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  double2* area = sh.area[tw_wave ? wave : 0];

  load_ta(sh.ta, tg);
  TwB tb;
  tb.load(tg, lane);
  u64 acc[32];
  if (tw_wave) {  // acc_c: A = 0, B = X^{-b~} * lut (LUT values in the Z_p encoding, mapped to the torus)
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N2;
    const int s = (4096 - ms4096(ct[n])) & 4095;
#pragma unroll
    for (int e = 0; e < 32; e++) {
      int d = 64 * e + lane - s;
      bool neg = false;
      if (d < 0) { d += N2; neg = !neg; }
      if (d < 0) { d += N2; neg = !neg; }
      const u64 v = gl_to_torus(lut[d]);
      acc[e] = c ? (neg ? 0 - v : v) : 0;
    }
  }
  __syncthreads();

  int a_next = tw_wave ? ms4096(ct[0]) : 0;
  constexpr int SPW = 16 / NW;  // MAC slots per wave
  static_assert(NW == 8 || NW == 2 * CTS, "waves: 8, or one per polynomial");
  const int s0 = SPW * wave_s;  // MAC slots s0 .. s0 + SPW - 1
#if F1_PRIO_ASM
#if F1_PRIO == 6
  // A/B (round 6, as pbs_fft.hip FFT_PRIO 6): the base priority alternates every 2^F1_PRIO_SH CMUXes, in opposite
  // phase for the two dispatch halves
  const unsigned prio_ph = __builtin_amdgcn_readfirstlane((blockIdx.x >> 8) & 1);
  unsigned prio_flag = prio_ph;
#elif F1_PRIO == 7
  // A/B (round 6): F1_PRIO 3's dispatch-half alternation, except the last F1_TAILWG workgroups of the grid run at
  // the base level, so the two final workgroups of a CU fall back to oldest-first arbitration (the one that started
  // earlier finishes first) instead of the alternation's fast / slow pair (profiles/r06g_wgt_f2k_4096.json: the two
  // slots of a CU end 1.9 ms apart)
  const unsigned prio_flag = __builtin_amdgcn_readfirstlane(
      (((blockIdx.x >> 8) & 1) && blockIdx.x + F1_TAILWG < gridDim.x) ? 1u : 0u);
#elif F1_PRIO == 8
  // A/B: the dispatch-half alternation inverted for the last F1_TAILWG workgroups
  const unsigned prio_flag = __builtin_amdgcn_readfirstlane(
      ((((blockIdx.x >> 8) & 1) != 0) != (blockIdx.x + F1_TAILWG >= gridDim.x)) ? 1u : 0u);
#else
  const unsigned prio_flag = __builtin_amdgcn_readfirstlane(
      (F1_PRIO == 3 && NW == 2 * CTS && ((blockIdx.x >> 8) & 1)) || (F1_PRIO == 1 && wave_s >= 4) ? 1u : 0u);
#endif
#endif
#if F1_STAGGER
  // A/B (round 6, as pbs_fft.hip FFT_STAGGER): the second workgroup of each CU in the first dispatch round starts late
  if (blockIdx.x < 512 && ((blockIdx.x >> 8) & 1))
    for (int k = 0; k < F1_STAGGER; k++) __builtin_amdgcn_s_sleep(127);
#endif
#if F1_PRIO == 1
  if (wave_s >= 4) __builtin_amdgcn_s_setprio(1);
#elif F1_PRIO == 3
  // bit 8 of the workgroup index = the second dispatch half on a 256-CU part (MI355X only; on other CU counts
  // the two workgroups of a CU just get an arbitrary split)
  if constexpr (NW == 2 * CTS)
    if ((blockIdx.x >> 8) & 1) __builtin_amdgcn_s_setprio(1);
#elif (F1_PRIO == 7 || F1_PRIO == 8) && F1_PRIO_ASM
  asm volatile(
      "s_cmp_lg_u32 %0, 0\n\ts_cbranch_scc0 .Lfi0_%=\n\ts_setprio 1\n\ts_branch .Lfi1_%=\n"
      ".Lfi0_%=:\n\ts_setprio 0\n.Lfi1_%=:" ::"s"(prio_flag) : "scc");
#endif
  // key words of CMUX i for the MAC phase: kv[t][cc][j] = K_{cc,j}[slot s0 + t][lane].  The first KPRE slots are
  // requested at the CMUX start (their latency hides behind the forward transform); with 4 slots per wave the
  // other two are requested after the forward transform (holding all four across the transform spills).
  constexpr int KPRE = SPW < 2 ? SPW : 2;
  auto load_key = [&](int i, double2 (&kv)[SPW][2][2], bool late) {
#pragma unroll
    for (int t = 0; t < SPW; t++)
      if ((t >= KPRE) == late)
#pragma unroll
        for (int cc = 0; cc < 2; cc++)
#pragma unroll
          for (int j = 0; j < 2; j++) kv[t][cc][j] = bsk[((size_t)(i * 2 + cc) * 2 + j) * M1 + 64 * (s0 + t) + lane];
  };
  auto cmux = [&](int i, double2 (&kv)[SPW][2][2]) {
#if F1_PRIO_ASM && F1_PRIO == 6
    prio_flag = ((unsigned)i >> F1_PRIO_SH ^ prio_ph) & 1u;
    asm volatile(
        "s_cmp_lg_u32 %0, 0\n\ts_cbranch_scc0 .Lfq0_%=\n\ts_setprio 1\n\ts_branch .Lfq1_%=\n"
        ".Lfq0_%=:\n\ts_setprio 0\n.Lfq1_%=:" ::"s"(prio_flag) : "scc");
#endif
    const int a = a_next;
    if (tw_wave && i + 1 < n) a_next = ms4096(ct[i + 1]);
    if (tw_wave) {
      double xr[16], xi[16];
      rotate_digits(acc, a, lane, area, xr, xi);
      fft1k_fwd(xr, xi, area, lane, sh.ta, tb);
#pragma unroll
      for (int s = 0; s < 16; s++) area[64 * s + lane] = make_double2(xr[s], xi[s]);
    }
    // the other key slots: requested before the barrier (the transform's registers are free by now), so their
    // latency overlaps the wait (+0.3-0.5 %, profiles/r04i_fhevm_2wg_ab.txt)
    if constexpr (SPW > KPRE) load_key(i, kv, true);
    f1_barrier();
#if F1_MACPRIO
    __builtin_amdgcn_s_setprio(3);  // the short MAC phase ahead of the other workgroup's transforms
#endif
#pragma unroll
    for (int q = 0; q < CTS; q++) {
#pragma unroll
      for (int t = 0; t < SPW; t++) {
        const int idx = 64 * (s0 + t) + lane;
        const double2 d0 = sh.area[2 * q][idx], d1 = sh.area[2 * q + 1][idx];
        double2 o[2];
#pragma unroll
        for (int j = 0; j < 2; j++) {
          const double2 k0 = kv[t][0][j], k1 = kv[t][1][j];
#if F1_PAIRMAC
          // the split order (oracle: per-component products, then one add -- as the P-GATE kernels)
          double r0 = d0.x * k0.x;
          r0 = __builtin_fma(-d0.y, k0.y, r0);
          double i0 = d0.x * k0.y;
          i0 = __builtin_fma(d0.y, k0.x, i0);
          double r1 = d1.x * k1.x;
          r1 = __builtin_fma(-d1.y, k1.y, r1);
          double i1 = d1.x * k1.y;
          i1 = __builtin_fma(d1.y, k1.x, i1);
          o[j] = make_double2(r0 + r1, i0 + i1);
#else
          double re = __builtin_fma(d0.x, k0.x, 0.0);
          re = __builtin_fma(-d0.y, k0.y, re);
          double im = __builtin_fma(d0.x, k0.y, 0.0);
          im = __builtin_fma(d0.y, k0.x, im);
          re = __builtin_fma(d1.x, k1.x, re);
          re = __builtin_fma(-d1.y, k1.y, re);
          im = __builtin_fma(d1.x, k1.y, im);
          im = __builtin_fma(d1.y, k1.x, im);
          o[j] = make_double2(re, im);
#endif
        }
        sh.area[2 * q][idx] = o[0];
        sh.area[2 * q + 1][idx] = o[1];
      }
    }
    f1_barrier();
#if F1_MACPRIO  // back to the workgroup's level (F1_PRIO)
#if F1_PRIO_ASM
    // one asm block with its own scalar branch (as pbs_fft.hip's base_prio): no C-level branch in the CMUX loop
    asm volatile(
        "s_cmp_lg_u32 %0, 0\n\ts_cbranch_scc0 .Lfp0_%=\n\ts_setprio 1\n\ts_branch .Lfp1_%=\n"
        ".Lfp0_%=:\n\ts_setprio 0\n.Lfp1_%=:" ::"s"(prio_flag) : "scc");
#else
    if (F1_PRIO == 3 && NW == 2 * CTS && ((blockIdx.x >> 8) & 1)) __builtin_amdgcn_s_setprio(1);
    else if (F1_PRIO == 1 && wave_s >= 4) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#endif
#endif
    if (tw_wave) {
      double xr[16], xi[16];
#pragma unroll
      for (int s = 0; s < 16; s++) {
        const double2 v = area[64 * s + lane];
        xr[s] = v.x;
        xi[s] = v.y;
      }
      fft1k_inv(xr, xi, area, lane, sh.ta, tb);
#pragma unroll
      for (int e = 0; e < 16; e++) {
#if F1_Y32
        acc[e] = torus_acc_add_wide_y(acc[e], xr[e]);
        acc[e + 16] = torus_acc_add_wide_y(acc[e + 16], xi[e]);
#else
        acc[e] = torus_acc_add_wide(acc[e], xr[e]);
        acc[e + 16] = torus_acc_add_wide(acc[e + 16], xi[e]);
#endif
      }
    }
  };
#if F1_PAIRMAC
  // A/B (round 6): the batch form with the P-GATE kernel's MAC.  Wave (p, c) multiplies its own spectrum D_c by both
  // key polynomials of component c (read from L2, four slots ahead), publishes the product for the other output
  // (D_c (.) K_(c, 1-c)) in its area and keeps D_c (.) K_(c, c) in registers; after one barrier it adds the partner's
  // D_(1-c) (.) K_(1-c, c): O_c = O_c^0 + O_c^1, the oracle's split order.  Against the slot-owned MAC: no spectrum
  // store, no MAC-phase reads / writes of both spectra (16 b128 LDS writes and 16 reads fewer per wave and CMUX), twice
  // the key words per wave from L2 (32 instead of 16 b128 loads), one barrier pair as before.
  if constexpr (NW == 2 * CTS) {
    const double2* Tp = sh.area[wave ^ 1];
    for (int i = 0; i < n; i++) {
      const int a = a_next;
      if (i + 1 < n) a_next = ms4096(ct[i + 1]);
      const double2* kc = bsk + (size_t)(i * 2 + c) * 2 * M1 + lane;  // K_(c, j)[s] = kc[j M1 + 64 s]
      constexpr int KG = F1_PAIRMAC_KG;  // key slots per prefetch group
      double2 kv[KG][2];
#pragma unroll
      for (int t = 0; t < KG; t++) {
        kv[t][0] = kc[64 * t];
        kv[t][1] = kc[M1 + 64 * t];
      }
      double xr[16], xi[16];
      rotate_digits(acc, a, lane, area, xr, xi);
      fft1k_fwd(xr, xi, area, lane, sh.ta, tb);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 16 / KG; g++) {
        __builtin_amdgcn_sched_barrier(0);  // keep each group's key loads in their group (no hoisting of all 32)
        double2 kn[KG][2];
        if (g + 1 < 16 / KG) {
#pragma unroll
          for (int t = 0; t < KG; t++) {
            kn[t][0] = kc[64 * (KG * (g + 1) + t)];
            kn[t][1] = kc[M1 + 64 * (KG * (g + 1) + t)];
          }
        }
#pragma unroll
        for (int t = 0; t < KG; t++) {
          const int sl = KG * g + t;
          const double dr = xr[sl], di = xi[sl];
          double pr[2], pi[2];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const double2 k = kv[t][j];
            pr[j] = dr * k.x;
            pr[j] = __builtin_fma(-di, k.y, pr[j]);
            pi[j] = dr * k.y;
            pi[j] = __builtin_fma(di, k.x, pi[j]);
          }
          // c wave-uniform: the own output c stays, output 1 - c goes to the area
          if (c_u) {
            area[64 * sl + lane] = make_double2(pr[0], pi[0]);
            xr[sl] = pr[1];
            xi[sl] = pi[1];
          } else {
            area[64 * sl + lane] = make_double2(pr[1], pi[1]);
            xr[sl] = pr[0];
            xi[sl] = pi[0];
          }
        }
        if (g + 1 < 16 / KG) {
#pragma unroll
          for (int t = 0; t < KG; t++) {
            kv[t][0] = kn[t][0];
            kv[t][1] = kn[t][1];
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int sl = 0; sl < 16; sl++) {
        const double2 v = Tp[64 * sl + lane];
        xr[sl] = xr[sl] + v.x;
        xi[sl] = xi[sl] + v.y;
      }
      __syncthreads();  // the partner has read this wave's area before the inverse overwrites it
      fft1k_inv(xr, xi, area, lane, sh.ta, tb);
#pragma unroll
      for (int e = 0; e < 16; e++) {
        acc[e] = torus_acc_add_wide_y(acc[e], xr[e]);
        acc[e + 16] = torus_acc_add_wide_y(acc[e + 16], xi[e]);
      }
    }
  } else
#endif
#if F1_KPF
  double2 kva[SPW][2][2], kvb[SPW][2][2];  // one CMUX ahead
  load_key(0, kva, false);
  for (int i = 0; i < n; i += 2) {
    if (i + 1 < n) load_key(i + 1, kvb, false);
    cmux(i, kva);
    if (i + 1 >= n) break;
    if (i + 2 < n) load_key(i + 2, kva, false);
    cmux(i + 1, kvb);
  }
#else
  for (int i = 0; i < n; i++) {
    double2 kv[SPW][2][2];  // requested at the CMUX start, consumed after the rotation and forward transform
    load_key(i, kv, false);
    cmux(i, kv);
  }
#endif
#if FFT_WGTIME
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    g_wgt2k[4 * blockIdx.x] = wg_t0;
    g_wgt2k[4 * blockIdx.x + 1] = t1;
    g_wgt2k[4 * blockIdx.x + 2] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));
    g_wgt2k[4 * blockIdx.x + 3] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
#endif

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * (2 * N2) + c * N2;
#pragma unroll
    for (int e = 0; e < 32; e++) oa[64 * e + lane] = acc[e];
  }
  if (WRITE_BIG) {  // sample extraction at degree 0: a'_0 = A[0], a'_j = -A[N-j], b' = B[0]
    u64* ob = out_big + b * (size_t)(N2 + 1);
    if (c == 0) {
#pragma unroll
      for (int e = 0; e < 32; e++) {
        const int t = 64 * e + lane;
        if (t == 0) ob[0] = acc[e];
        else ob[N2 - t] = 0 - acc[e];
      }
    } else if (lane == 0) {
      ob[N2] = acc[0];
    }
  }
}

// one wave per polynomial: natural coefficients (int64 torus words) -> spectrum [slot][lane] x scale
__global__ __launch_bounds__(64) void fwd2k_kernel(const u64* __restrict__ in, double2* __restrict__ out,
                                                   const double2* __restrict__ tg, double scale) {
  __shared__ __attribute__((aligned(16))) double2 ta[M1];
  __shared__ __attribute__((aligned(16))) double2 area[AREA_C64];
  const int lane = threadIdx.x;
  load_ta(ta, tg);
  TwB tb;
  tb.load(tg, lane);
  const u64* src = in + (size_t)blockIdx.x * N2;
  double xr[16], xi[16];
#pragma unroll
  for (int e = 0; e < 16; e++) {
    xr[e] = i64_to_f64(src[64 * e + lane]);
    xi[e] = i64_to_f64(src[64 * e + lane + M1]);
  }
  __syncthreads();
  fft1k_fwd(xr, xi, area, lane, ta, tb);
  double2* dst = out + (size_t)blockIdx.x * M1;
#pragma unroll
  for (int s = 0; s < 16; s++) dst[64 * s + lane] = make_double2(xr[s] * scale, xi[s] * scale);
}

// inverse for the parity tests: spectrum [slot][lane] -> 2048 doubles (no 1/M, no rounding)
__global__ __launch_bounds__(64) void inv2k_kernel(const double2* __restrict__ in, double* __restrict__ out,
                                                   const double2* __restrict__ tg) {
  __shared__ __attribute__((aligned(16))) double2 ta[M1];
  __shared__ __attribute__((aligned(16))) double2 area[AREA_C64];
  const int lane = threadIdx.x;
  load_ta(ta, tg);
  TwB tb;
  tb.load(tg, lane);
  const double2* src = in + (size_t)blockIdx.x * M1;
  double xr[16], xi[16];
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const double2 v = src[64 * s + lane];
    xr[s] = v.x;
    xi[s] = v.y;
  }
  __syncthreads();
  fft1k_inv(xr, xi, area, lane, ta, tb);
  double* dst = out + (size_t)blockIdx.x * N2;
#pragma unroll
  for (int e = 0; e < 16; e++) {
    dst[64 * e + lane] = xr[e];
    dst[64 * e + lane + M1] = xi[e];
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

}  // namespace fft1k

#if FFT_WGTIME
extern "C" int tfhe_hip_debug_wgtimes2k(unsigned long long* out, size_t n) {
  if (n > 4 * 16384) n = 4 * 16384;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fft1k::g_wgt2k), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_sample_extract_torus2k(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (fft1k::N2 + 1);
  hipLaunchKernelGGL(fft1k::sample_extract_torus2k_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc,
                     B, out);
  return hipGetLastError();
}

size_t fft2k_tables_len() { return 2 * fft1k::K_C64; }

// ta[k][L] = zeta^{L (1 + 4 k)}, tb[m][l0] = zeta^{64 l0 m}, zeta = e^{2 pi i / 4096} (the oracle's tab1k)
void make_fft2k_tables(double* t) {
  using namespace fft1k;
  for (uint32_t k = 0; k < 16; k++)
    for (uint32_t L = 0; L < 64; L++) {
      const int o = K_TA + 64 * k + L;
      fft_twiddle((L * (1 + 4 * k)) % 4096, 4096, &t[2 * o], &t[2 * o + 1]);
    }
  for (uint32_t m = 0; m < 4; m++)
    for (uint32_t l = 0; l < 16; l++) {
      const int o = K_TB + 16 * m + l;
      fft_twiddle((64 * l * m) % 4096, 4096, &t[2 * o], &t[2 * o + 1]);
    }
}

// the compile-time slot constants equal the table generator's zeta^{64 e} bit for bit
bool fft2k_slot_constants_ok() {
  for (int e = 0; e < 16; e++) {
    double c, s;
    fft_twiddle(64u * e, 4096u, &c, &s);
    if (c != fft1k::ctw16::SLOT[e].x || s != fft1k::ctw16::SLOT[e].y) return false;
  }
  return true;
}

hipError_t launch_bsk_to_fourier2k(const u64* bsk_std, double* bsk_f, size_t polys, const double* tw, hipStream_t s) {
  if (polys == 0) return hipSuccess;
  hipLaunchKernelGGL(fft1k::fwd2k_kernel, dim3((unsigned)polys), dim3(64), 0, s, bsk_std, (double2*)bsk_f,
                     (const double2*)tw, (F1_NEGDIG ? -1.0 : 1.0) * (F1_Y32 ? 0x1p-42 : 0x1p-10));
  return hipGetLastError();
}

hipError_t launch_fft2k_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fft1k::fwd2k_kernel, dim3((unsigned)count), dim3(64), 0, s, in, (double2*)out,
                     (const double2*)tw, 1.0);
  return hipGetLastError();
}

hipError_t launch_fft2k_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fft1k::inv2k_kernel, dim3((unsigned)count), dim3(64), 0, s, (const double2*)in, out,
                     (const double2*)tw);
  return hipGetLastError();
}

template <int CTS, int NW>
static hipError_t launch_br2k(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index, int n_lut,
                              const double2* bk, const double2* t, u64* out_big, u64* out_acc, hipStream_t s) {
  using namespace fft1k;
  dim3 grid((unsigned)((B + CTS - 1) / CTS)), block(64 * NW);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<CTS, NW, true, true>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<CTS, NW, true, false>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_fft2k_kernel<CTS, NW, false, true>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  return hipGetLastError();
}

// batches up to latency_max_batch: two ciphertexts per workgroup (four transform waves on four SIMDs, eight MAC
// waves); larger batches: F1_BATCH2 = 1 two per workgroup of four waves, two workgroups per CU (16 KB areas);
// 0: four per workgroup of eight waves (two transform waves per SIMD)
#ifndef F1_BATCH2
#define F1_BATCH2 1
#endif
hipError_t launch_blind_rotate_fft2k(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                     int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                     hipStream_t s, size_t latency_max_batch) {
  if (B == 0) return hipSuccess;
  const double2 *bk = (const double2*)bsk_f, *t = (const double2*)tw;
  if (B <= latency_max_batch) return launch_br2k<2, 8>(lwe_in, B, n, luts, lut_index, n_lut, bk, t, out_big, out_acc, s);
#if F1_BATCH2 && F1_SWZ != 0
  return launch_br2k<2, 4>(lwe_in, B, n, luts, lut_index, n_lut, bk, t, out_big, out_acc, s);
#else
  return launch_br2k<4, 8>(lwe_in, B, n, luts, lut_index, n_lut, bk, t, out_big, out_acc, s);
#endif
}

}  // namespace tfhe
