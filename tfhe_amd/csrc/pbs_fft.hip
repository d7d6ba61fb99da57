// pbs_fft.hip — the FFT64 transform of the PBS hot path for gfx950 (P-GATE shape: N = 1024, k = 1,
// PBS 2^7 x 3): the external product computed the way tfhe-rs computes it, with an f64 negacyclic
// FFT over the native 2^64 torus, instead of the Goldilocks NTT of pbs_kernels.hip.
//
// Why: MI355X runs f64 add / mul / fma at the full VALU rate (~6 cycles per wave-instruction, the
// same as a 32-bit integer op, tools/microbench/f64_rates.hip), and a complex radix-2 butterfly is ~8
// such instructions where a Goldilocks butterfly is ~30 integer ones.  Same BSK bytes (N/2 complex
// doubles = N u64 per polynomial); the batch kernel walks the CMUX loop with 4 ciphertexts x 2 component
// waves per workgroup in lockstep, the BSK level steps streamed once per workgroup into LDS by
// global_load_lds, double-buffered.
//
// Arithmetic (one fixed f64 operation sequence, restated in oracle/fft_oracle.c, which this file
// reproduces bit-for-bit — every product is written as an explicit fma or a lone multiply, and
// contraction is off for the whole file):
//   fold + twist  z_j = (a_j + i a_{j+512}) * zeta^j,   zeta = e^{i pi / 1024}
//   DFT           Z_k = sum_j z_j e^{+2 pi i jk / 512}: 3 radix-8 passes over the wave's 64 lanes
//                 x 8 registers, natural order in, DEVICE ORDER out (slot e of lane L holds
//                 k = (L >> 3) + 8 (L & 7) + 64 e); the inverse runs the passes reversed (DIT), device
//                 order in, natural order out.  Two LDS transposes each way with plain padded rows
//                 (strides 72 and 65 complex): every ds_write_b128 / ds_read_b128 is conflict-free and
//                 every address is a per-lane base plus an immediate offset
//   MAC           O_j += D_(c,l) (.) BSK_i[(c,l)][j], 4 fma per complex; c ascending, levels least
//                 significant first (each level's digits come off a running carry state, so the device
//                 BSK stores the level rows of each component reversed)
//   inverse       conjugate passes, untwist by conj(zeta^j), rint, mod 2^64, add to the accumulator
// Coefficient 64 e + L of a u64 register polynomial (slot e of lane L, e < 16) meets coefficient
// 64 (e + 8) + L in the same lane, so folding and unfolding move no data.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <type_traits>

#include "fft512.h"
#include "gl64.h"
#include "ntt1024.h"
#include "pbs_kernels.h"

namespace tfhe {
namespace fftk {

// forward transform of a real polynomial held as 16 doubles per lane (slot e <-> coefficient 64 e + L)
// (twist: slot constants here, the lane part inside pass A — fft512.h, "N = 1024 merged twist")
__device__ __forceinline__ void fft_fwd_real(const double (&a)[16], double (&xr)[8], double (&xi)[8], double2* T,
                                             int lane, const double2* tw) {
#pragma unroll
  for (int e = 0; e < 8; e++) {
    xr[e] = a[e];
    xi[e] = a[e + 8];
  }
  dft512_fwd<true, true>(xr, xi, T, lane, TBase(lane), tw);  // the slot twist inside pass A (twist_dft8_fwd)
}

// inverse transform (no 1/M) + untwist: slot e -> coefficient 64 e + L (re), 64 (e + 8) + L (im)
__device__ __forceinline__ void fft_inv_real(double (&xr)[8], double (&xi)[8], double2* T, int lane, TBase tb,
                                             const double2* tw) {
  dft512_inv(xr, xi, T, lane, tb, tw);
  twist_slots<true>(xr, xi);  // the lane part of the untwist rode in pass B''s table
}

__device__ __forceinline__ int ms2048(u64 x) { return (int)((((x >> 52) + 1) >> 1) & 2047u); }

// tfhe-rs SignedDecomposer 2^7 x 3 (closest_representable at 21 bits, balanced digits, carry
// rule carry = (((res - 1) | state) & res) >> 6), restated as one step per level, least significant
// first, on the running state st (21 bits to start; == or_decompose for every state, tests/test_fft.py):
//   b = bit 13 of st (level 2 and 1; 0 for the top level), W = st + 63 + b,
//   digit = (W & 127) - 63 - b, st' = W >> 7
__device__ __forceinline__ u32 decomp_state(u64 x) { return ((u32)(x >> 32) + 1024u) >> 11; }
// bmask = 1 below the top level, 0 at the top level
// (W & 127) - 63 - b = st - (W & ~127): the digit is the old state minus the new one shifted back
// FFT_DIG_MAD 1 (default since round 5): the digit as st - 128 st' in one v_mad_i32_i24 (st < 2^22, st' < 2^15 fit the
// 24-bit operands): 4 VALU per digit instead of 5 (hipcc turns the multiply into a shift + subtract, hence the asm;
// -128 is not a VOP3 inline constant on gfx9, so it rides in an SGPR)
#ifndef FFT_DIG_MAD
#define FFT_DIG_MAD 1
#endif
__device__ __forceinline__ int decomp_step(u32& st, u32 bmask) {
  const u32 b = __builtin_amdgcn_ubfe(st, 13, bmask);
  const u32 W = st + 63u + b;
#if FFT_DIG_MAD
  const u32 stn = W >> 7;
  int d;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(stn), "s"(-128), "v"(st));
  st = stn;
#else
  const int d = (int)(st - (W & ~127u));  // 5 VALU per digit with the bfe, add3 and shift
  st = W >> 7;
#endif
  return d;
}
// the top level (b = 0, no next state): 3 VALU per digit
__device__ __forceinline__ int decomp_top(u32 st) { return (int)(st - ((st + 63u) & ~127u)); }

// o = D (.) K as the first term of an fma chain: a multiply where the chain would add to +0 (the oracle's
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

// ---------------------------------------------------------------------------------------------
// BSK conversion: one wavefront per polynomial; [i][r][j] order kept, 512 complex natural, x 2^-9 (x 2^-41 with
// FFT_Y32: the blind rotations then update their accumulators from y = x 2^-32, fft512.h torus_acc_add_y)
#ifndef FFT_Y32
#define FFT_Y32 1
#endif
constexpr double BSK_SCALE = FFT_Y32 ? 0x1p-41 : 0x1p-9;
#if FFT_Y32
#define ACC_ADD torus_acc_add_y
#else
#define ACC_ADD torus_acc_add
#endif
__global__ __launch_bounds__(64) void bsk_to_fourier_kernel(const u64* __restrict__ bsk_std,
                                                            double2* __restrict__ bsk_f,
                                                            const double2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) double2 T[T_C64];
  const int lane = threadIdx.x;
  const size_t q = blockIdx.x;  // standard layout [i][c*3 + l][j]
  const u64* src = bsk_std + q * N1K;
  double a[16], xr[8], xi[8];
#pragma unroll
  for (int e = 0; e < 16; e++) a[e] = i64_to_f64(src[64 * e + lane]);
  fft_fwd_real(a, xr, xi, T, lane, tw);
  const size_t j = q % 2, r = (q / 2) % 6, i = q / 12;  // device layout [i][c*3 + (2 - l)][j]
  double2* dst = bsk_f + ((i * 6 + (r / 3) * 3 + (2 - r % 3)) * 2 + j) * M;
#pragma unroll
  for (int e = 0; e < 8; e++) dst[64 * e + lane] = make_double2(xr[e] * BSK_SCALE, xi[e] * BSK_SCALE);
}

// natural-order transforms for the parity tests (one wavefront per polynomial)
__global__ __launch_bounds__(64) void fft_fwd_kernel(const u64* __restrict__ in, double2* __restrict__ out,
                                                     const double2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) double2 T[T_C64];
  const int lane = threadIdx.x;
  const u64* src = in + (size_t)blockIdx.x * N1K;
  double a[16], xr[8], xi[8];
#pragma unroll
  for (int e = 0; e < 16; e++) a[e] = i64_to_f64(src[64 * e + lane]);
  fft_fwd_real(a, xr, xi, T, lane, tw);
  double2* dst = out + (size_t)blockIdx.x * M;
#pragma unroll
  for (int e = 0; e < 8; e++) dst[64 * e + lane] = make_double2(xr[e], xi[e]);
}

__global__ __launch_bounds__(64) void fft_inv_kernel(const double2* __restrict__ in, double* __restrict__ out,
                                                     const double2* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) double2 T[T_C64];
  const int lane = threadIdx.x;
  const double2* src = in + (size_t)blockIdx.x * M;
  double xr[8], xi[8];
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 v = src[64 * e + lane];
    xr[e] = v.x;
    xi[e] = v.y;
  }
  fft_inv_real(xr, xi, T, lane, TBase(lane), tw);
  double* dst = out + (size_t)blockIdx.x * N1K;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    dst[64 * e + lane] = xr[e];
    dst[64 * (e + 8) + lane] = xi[e];
  }
}

// ---------------------------------------------------------------------------------------------
// FFT_PRIO: the waves' base priority (what FFT_MACPRIO drops back to after each MAC phase).
//   3 (default since round 6): the workgroups with bit 8 of blockIdx set -- on 256 CUs the second workgroup each CU
//     receives, then every other dispatch half-round -- at base priority 1.  The hardware arbitrates oldest-first, so
//     of the two workgroups that share a CU the older always ran ahead: in a 4096 launch one slot of every CU
//     finished its four workgroups 2.4 ms before the other and idled (profiles/r06d_wgt_4096.json, per-workgroup
//     s_memrealtime stamps, tools/wg_timeline.py).  With the alternation the two slots end 0.33 ms apart and the
//     CU-slot busy fraction rises 0.945 -> 0.980: 24.04 -> 23.04 ms per 4096, C2 6.45 -> 6.24 ms (same box, three
//     boxes; profiles/r06e_ab_prio.txt).  Round 4 had measured this scheme "neutral" -- with a C-level branch around
//     s_setprio that made hipcc spill (below).
//   1: s_setprio 1 for waves 4-7 of an 8-wave workgroup (round 1; no effect on the 4-wave CTS = 2 workgroup)
//   4 / 5: A/B forms (the last FFT_TAILWG workgroups high; bit 8 xor bit 9)
#ifndef FFT_PRIO
#define FFT_PRIO 3
#endif

// Component-pair batch kernel (round 3, the default above the latency range): workgroup = CTS ciphertexts x 2
// waves (CTS = 2 by default, 4 in round 3), wave (p, c) owns COMPONENT c of ciphertext p.  Per CMUX i:
//   rotate + decompose acc_c (wave-local: the wave's own transpose area holds the rotation image)
//   level steps q = 0, 1, 2 (least significant first): digits -> twist -> DFT -> MAC into BOTH outputs'
//     partial sums  O_j^c = fma chain over q of D_(c,q) (.) BSK_i[(c, q)][j]      (j = 0, 1)
//     one step's chunk = rows (0, q) and (1, q) of BSK_i (32 KB), streamed once per workgroup by
//     global_load_lds (CTS = 4: double-buffered; CTS = 2: one buffer, loaded at the step's start)
//   exchange: wave c publishes O_(1-c)^c in its transpose area and takes O_c^(1-c) from its partner's:
//     O_c = O_c^c + O_c^(1-c)  (= O_c^0 + O_c^1: f64 addition commutes, the oracle's split order)
//   ONE inverse transform: acc_c += rint(iFFT(O_c)) mod 2^64
// Against round 2's 8-ciphertext kernel (one wave per ciphertext, retired in round 4): the same transforms per
// ciphertext, half of them per wave, 1/2 the accumulator / partial-sum registers per wave, and twice the waves
// per ciphertext -- a batch of 1024 fills all 256 CUs at 2 waves / SIMD.
// The MAC order (per-component chains, then one add) is restated in oracle/fft_oracle.c.
// LDS at CTS = 4: 8 x 9 KB transpose areas | 2 x 32 KB level steps | pass A, B, B' tables (24 KB) = 160 KB;
// at CTS = 2: B' table (8 KB) | one 32 KB level step | 4 x 9 KB transpose areas = 76 KB, two workgroups per CU.
// FFT_ROT_BATCH: the rotation's 16 image reads issued together before their first use (measured with the
// first level peeled: 27.04 -> 27.55 ms per 4096, slower; kept for A/B runs)
#ifndef FFT_ROT_BATCH
#define FFT_ROT_BATCH 0
#endif
// FFT_PAIR_TWREG: pass A's twiddles held in registers across the CMUX loop (the round-2 ablation: -4 %)
#ifndef FFT_PAIR_TWREG
#define FFT_PAIR_TWREG 2
#endif
constexpr int STEP_C64 = 4 * M;                    // rows (0, q), (1, q), j = 0, 1
// CTS = ciphertexts per workgroup.  2 (default since round 4): 4 waves, TWO independent workgroups per CU (76 KB
// each: only the inverse's TW_I table in LDS, passes A / B from registers, one level-step buffer), so the two
// workgroups drift apart and one's LDS phases overlap the other's VALU phases on every SIMD: 27.01 -> 26.63 ms per
// 4096 on the same box (profiles/r04a_cts_ab.txt, two rounds).  4 (FFT_PAIR_CTS=4): 8 waves, one workgroup per CU,
// all tables in LDS, level steps double-buffered (the round-3 kernel).
// FFT_PAIR_LDSTW: the round-3 layout (all tables in LDS, level steps double-buffered) for CTS = 4; 0 (round 6 A/B):
// CTS = 4 with the CTS = 2 program (passes A / B in registers, one level-step buffer): 8 waves, one workgroup per CU
#ifndef FFT_PAIR_LDSTW
#define FFT_PAIR_LDSTW 1
#endif
template <int CTS, bool LDS_TW = (CTS == 4 && FFT_PAIR_LDSTW)>
struct FpShared {
  double2 tw[3 * M];                               // TW_A | TW_B | TW_I of the global table (no twist table)
  double2 T[2 * CTS][T_C64];                       // after the tables: T - 8 KB is still inside the block
  double2 K[2][STEP_C64];
};
template <int CTS>
struct FpShared<CTS, false> {
  double2 twI[M];                                  // TW_I only (passes A, B: registers, loaded from global)
  double2 K[1][STEP_C64];
  double2 T[2 * CTS][T_C64];
};
#ifndef FFT_PAIR_CTS
#define FFT_PAIR_CTS 2
#endif
// FFT_MACPRIO 1 (default since late round 4): each level step's MAC runs at the top wave priority (back to 0
// when the next step starts and after the last), so the short MAC phase of one workgroup is not stalled behind
// the other workgroup's transforms on the same SIMD: 26.62 -> 25.26 ms per 4096 on the same box, 152.2k ->
// 160.4k PBS/s (profiles/r04k_pgate_macprio_ab.txt)
#ifndef FFT_MACPRIO
#define FFT_MACPRIO 1
#endif
#ifndef FFT_STAGGER
#define FFT_STAGGER 1
#endif
#ifndef FFT_TAILWG
#define FFT_TAILWG 256
#endif
#ifndef FFT_PRIO_SH
#define FFT_PRIO_SH 0
#endif
#ifndef FFT_ROTPRIO
#define FFT_ROTPRIO 0
#endif
#ifndef FFT_XCHPRIO
#define FFT_XCHPRIO 0
#endif
typedef __attribute__((address_space(3))) u64 lds_u64;

// FFT_ROT_UNIFORM 1 (default since round 5): the rotation split so that every per-slot decision is wave-uniform.
// a (uniform) = 1024 s + 64 A + r.  The image written is W = X^r v (lane part: each lane writes at +r, only slot 15
// of the lanes L + r >= 64 wraps, negated, to the image start); the reads take (X^(64 A) W)[L + 64 e] = W[L + 64 (e -
// A)] for e >= A and -W[L + 64 (e - A + 16)] for e < A, so slot e's base (two per-lane bases 8 KB apart) and sign
// (xor s) depend only on the SGPR comparison e < A.  Per slot 8 VALU instead of 10 (no compare, no negate-and-select:
// y = (x ^ M) - (v + M), M = 0 or all ones); the values are the same, so no operation order changes.
#ifndef FFT_ROT_UNIFORM
#define FFT_ROT_UNIFORM 1
#endif
// (X^a v - v), v = this wave's polynomial (slot e <-> coefficient 64 e + L), to decomposition states.  The
// rotation image is the wave's transpose area.  Coefficient 64 e + L reads image entry (u + 64 e) mod 1024 with
// u = (L - a) mod 1024, negated iff the negacyclic source index (L - a + 64 e) mod 2048 lies in [1024, 2048):
// reads before the per-lane wrap use base u and DS offset 512 e, wrapped reads the base 8 KB lower (one compare
// and one select per slot instead of the index arithmetic; the sign mask is an SGPR xor).
__device__ __forceinline__ void rotate_states(const u64 (&v)[16], int a, int lane, double2* T, u32 (&st)[16]) {
  u64* Tu = (u64*)T;
#if FFT_ROT_UNIFORM
  a = __builtin_amdgcn_readfirstlane(a);  // ms2048(ct[i]): the same for every lane
  const int A = (a >> 6) & 15, r = a & 63;
  const bool sgn = a >= 1024;
  {
    const u32 wb = (u32)(uintptr_t)(lds_u64*)&Tu[lane + r];
#pragma unroll
    for (int e = 0; e < 15; e++) ((lds_u64*)(uintptr_t)wb)[64 * e] = v[e];
    const bool w15 = lane + r >= 64;  // coefficient 960 + L + r >= 1024: to L + r - 64, negated
    const u32 a15 = w15 ? wb + 960u * 8u - 8192u : wb + 960u * 8u;
    *(lds_u64*)(uintptr_t)a15 = w15 ? 0 - v[15] : v[15];
  }
  lds_order();
  const u32 rb = (u32)(uintptr_t)(lds_u64*)&Tu[lane] - 512u * (u32)A;  // >= T - 7.5 KB: inside the block
  // bit e of wmask: slot e reads the wrapped part (e < A); bit e of mbits: slot e negated.  Bit-field extracts of
  // these SGPR words keep every per-slot decision scalar (a compare would be rebuilt as a per-lane select)
  const u32 wmask = (1u << A) - 1u;
  const u32 mbits = __builtin_amdgcn_readfirstlane(wmask ^ (sgn ? ~0u : 0u));
#pragma unroll
  for (int e = 0; e < 16; e++) {
    // s_bfe_i32 (0 or -1) in inline asm: hipcc's known-bits treat the width-1 sbfe builtin as non-negative and drop
    // the sign extension (a probe kernel stores hi = 0 for it)
    int m32;
    asm("s_bfe_i32 %0, %1, %2" : "=s"(m32) : "s"(mbits), "i"(e | (1 << 16)));
    const u64 M = (u64)(long long)m32;
    const u64 x = ((const lds_u64*)(uintptr_t)(rb + (__builtin_amdgcn_ubfe(wmask, e, 1) << 13)))[64 * e];
    st[e] = decomp_state((x ^ M) - (v[e] + M));
  }
  lds_order();
#else
#pragma unroll
  for (int e = 0; e < 16; e++) Tu[64 * e + lane] = v[e];
  lds_order();
  const int t0 = (lane - a) & 2047;        // a < 2048
  const int u = t0 & 1023;
  const bool neg0 = t0 >= 1024;
  const u32 a0 = (u32)(uintptr_t)(lds_u64*)&Tu[u];
  const u32 a1 = a0 - 8192u;
#if FFT_ROT_BATCH
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const bool wrap = u >= 1024 - 64 * e;
    x[e] = ((const lds_u64*)(uintptr_t)(wrap ? a1 : a0))[64 * e];
  }
  __builtin_amdgcn_sched_barrier(0);  // all 16 reads in flight before the first use
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const bool neg = neg0 != (u >= 1024 - 64 * e);
    const u64 r = neg ? 0 - x[e] : x[e];
    st[e] = decomp_state(r - v[e]);
  }
#else
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const bool wrap = u >= 1024 - 64 * e;
    const u32 base = wrap ? a1 : a0;
    const u64 x = ((const lds_u64*)(uintptr_t)base)[64 * e];
    const bool neg = neg0 != wrap;
    const u64 r = neg ? 0 - x : x;
    st[e] = decomp_state(r - v[e]);
  }
#endif
  lds_order();
#endif
}

// the partial-sum exchange of wave c (compile-time): publish O_(1-c)^c in this wave's area, add O_c^(1-c) from
// the partner's (two workgroup barriers)
template <int C>
__device__ __forceinline__ void exchange_partials(const double (&o0r)[8], const double (&o0i)[8], const double (&o1r)[8],
                                                  const double (&o1i)[8], double (&xr)[8], double (&xi)[8], double2* T,
                                                  const double2* Tp, int lane) {
#pragma unroll
  for (int e = 0; e < 8; e++) {
    T[64 * e + lane] = C ? make_double2(o0r[e], o0i[e]) : make_double2(o1r[e], o1i[e]);
    xr[e] = C ? o1r[e] : o0r[e];
    xi[e] = C ? o1i[e] : o0i[e];
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const double2 w = Tp[64 * e + lane];
    xr[e] = xr[e] + w.x;
    xi[e] = xi[e] + w.y;
  }
  __syncthreads();  // the partner has read this wave's area before the inverse overwrites it
}

// level step g = 3 i + q: 32 KB in 1 KB blocks; wave w of NW loads blocks (32 / NW) w .. (16 per component row)
template <int NW>
__device__ __forceinline__ void load_step(const double2* __restrict__ bsk, int g, double2* dst, int wave_s, int lane) {
  const int i = g / 3, q = g - 3 * (g / 3);
#pragma unroll
  for (int u = 0; u < 32 / NW; u++) {
    const int blk = wave_s * (32 / NW) + u;
    const int c = blk >> 4;
    const char* src = (const char*)(bsk + ((size_t)i * 6 + c * 3 + q) * (2 * M)) + (blk & 15) * 1024;
    __builtin_amdgcn_global_load_lds((const void*)(src + lane * 16),
                                     (__attribute__((address_space(3))) void*)((char*)dst + blk * 1024), 16, 0, 0);
  }
}
// FFT_BUF_LDS 1 (default since round 5): the same level-step chunk through buffer_load_dwordx4 ... lds with the BSK as a
// buffer resource: the per-load byte offset is an SGPR (soffset) and the lane offset one loop-invariant VGPR, so the
// 24 loads of a CMUX cost no VALU (the global_load_lds form needs a 64-bit VALU address add per load)
#ifndef FFT_BUF_LDS
#define FFT_BUF_LDS 1
#endif
template <int NW>
__device__ __forceinline__ void load_step_buf(__amdgpu_buffer_rsrc_t bsr, int g, double2* dst, int wave_s, int voff) {
  const int i = g / 3, q = g - 3 * (g / 3);
#pragma unroll
  for (int u = 0; u < 32 / NW; u++) {
    const int blk = wave_s * (32 / NW) + u;
    const int c = blk >> 4;
    const int soff = ((i * 6 + c * 3 + q) * (2 * M)) * (int)sizeof(double2) + (blk & 15) * 1024;  // < 2^31: BSK < 2 GB
    __builtin_amdgcn_raw_ptr_buffer_load_lds(bsr, (__attribute__((address_space(3))) void*)((char*)dst + blk * 1024),
                                             16, voff, soff, 0, 0);
  }
}

#ifndef FFT_WGTIME
#define FFT_WGTIME 0
#endif
#if FFT_WGTIME
// diagnostic build only: per-workgroup start / end (s_memrealtime, 100 MHz), HW_ID and XCC_ID of the last launch
__device__ unsigned long long g_wgt[4 * 16384];
#endif
template <int CTS, bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(128 * CTS, 4 / CTS) void blind_rotate_fft_pair_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  constexpr int NW = 2 * CTS;
  constexpr bool LDS_TW = CTS == 4 && FFT_PAIR_LDSTW;
  __shared__ __attribute__((aligned(16))) FpShared<CTS> sh;
#if FFT_WGTIME
  const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = wave & 1;
  const size_t b_raw = (size_t)blockIdx.x * CTS + (wave >> 1);
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding pairs run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  double2* T = sh.T[wave];
  const double2* Tp = sh.T[wave ^ 1];
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int c_s = wave_s & 1;
  const int n_steps = 3 * n;

#if FFT_BUF_LDS
  // the BSK as a raw buffer (num_records = its byte size; gfx9 dword 3 = 0x00020000, as composable_kernel uses on gfx9)
  const __amdgpu_buffer_rsrc_t bsr =
      __builtin_amdgcn_make_buffer_rsrc((void*)bsk, (short)0, n * 6 * 2 * M * (int)sizeof(double2), 0x00020000);
  const int voff = lane * 16;
#endif
  if constexpr (LDS_TW) {
    for (int q = threadIdx.x; q < 3 * M; q += 64 * NW) sh.tw[q] = tw_g[TW_A + q];
    load_step<NW>(bsk, 0, sh.K[0], wave_s, lane);
  } else {
    for (int q = threadIdx.x; q < M; q += 64 * NW) sh.twI[q] = tw_g[TW_I + q];
  }

  // acc_c: A = 0, B = X^{-b~} * lut (LUT values in the Z_p encoding, mapped to the torus first)
  u64 acc[16];
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
      acc[e] = c ? (neg ? 0 - v : v) : 0;
    }
  }

  const TBase tb(lane);
  const double2* twA = tw_g + TW_A;
  const double2* twI;
  if constexpr (LDS_TW) {
    twA = sh.tw;
    twI = sh.tw + 2 * M;
  } else {
    twI = sh.twI;
  }
  const double2* twB = twA + M;
#if FFT_PAIR_TWREG
  double2 wa[8];  // pass A's twiddles (twist merged) for the whole CMUX loop: 8 LDS reads fewer per transform
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 8; e++) wa[e] = twA[64 * e + lane];
#endif
#if FFT_PAIR_TWREG >= 2
  double2 wb[8];  // and pass B's (the inverse's pass C' conjugates the same table): 7 more per forward, 7 per inverse
#pragma unroll
  for (int e = 1; e < 8; e++) wb[e] = twB[64 * e + lane];
  wb[0] = make_double2(1.0, 0.0);
#endif
  // the wave's base priority (FFT_PRIO), also what FFT_MACPRIO drops back to after each MAC phase
#if FFT_PRIO == 1
  const bool prio_hi = NW > 4 && wave_s >= 4;  // the 4-wave CTS = 2 workgroup has no second wave per SIMD
#elif FFT_PRIO == 3
  // with two workgroups per CU, one of them (by dispatch half-round) at the higher priority.  Bit 8 of the
  // workgroup index is the second dispatch half on a 256-CU part (MI355X only; other CU counts just alternate)
  const bool prio_hi = (blockIdx.x >> 8) & 1;
#elif FFT_PRIO == 6
  [[maybe_unused]] constexpr bool prio_hi = false;  // the per-CMUX alternation below
#elif FFT_PRIO == 5
  // A/B: bit 8 xor bit 9 of the workgroup index (the alternation flips every other dispatch round)
  const bool prio_hi = ((blockIdx.x >> 8) ^ (blockIdx.x >> 9)) & 1;
#elif FFT_PRIO == 4
  // A/B (round 6): the workgroups of the final dispatch half-round (the last FFT_TAILWG of the grid; on 256 CUs these
  // take the slot of each CU that frees last) at the higher base priority, against the hardware's oldest-first
  // arbitration, so the two final workgroups of a CU end closer together (profiles/r06d_wgt_*: without it one slot
  // of every CU idles ~2.4 ms at the end of a 4096 launch)
  const bool prio_hi = blockIdx.x + FFT_TAILWG >= gridDim.x;
#else
  constexpr bool prio_hi = false;
#endif
#if FFT_PRIO == 1 || FFT_PRIO == 0
  auto base_prio = [&]() {
    if (prio_hi) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  };
#else
  // a runtime (wave-uniform) priority as ONE asm block with its own scalar branch: a C-level branch around the two
  // s_setprio forms splits every level step into basic blocks and hipcc then spills ~195 VGPRs (measured 71 ms)
#if FFT_PRIO == 6
  // A/B (round 6): the base priority alternates every 2^FFT_PRIO_SH CMUXes, in opposite phase for the two dispatch
  // halves (blockIdx bit 8), so the two workgroups of a CU take turns instead of the older one always winning
  const unsigned prio_ph = __builtin_amdgcn_readfirstlane((blockIdx.x >> 8) & 1);
  unsigned prio_flag = prio_ph;
#else
  const unsigned prio_flag = __builtin_amdgcn_readfirstlane(prio_hi ? 1u : 0u);
#endif
  auto base_prio = [&]() {
    asm volatile(
        "s_cmp_lg_u32 %0, 0\n\ts_cbranch_scc0 .Lbp0_%=\n\ts_setprio 1\n\ts_branch .Lbp1_%=\n"
        ".Lbp0_%=:\n\ts_setprio 0\n.Lbp1_%=:" ::"s"(prio_flag) : "scc");
  };
#endif
  base_prio();
#if FFT_STAGGER
  // round 6 (default 1): the second workgroup of each CU in the first dispatch round (blockIdx bit 8 on 256 CUs) starts
  // FFT_STAGGER x ~3.4 us late, so the two workgroups of a CU do not run their phases in lockstep from the start
  // (with FFT_PRIO 3: 23.04 -> 22.97 ms per 4096, C2 6.24 -> 6.19 ms; alone 24.04 -> 23.87 ms; 2 and 4 x 3.4 us: neutral)
  if (blockIdx.x < 512 && ((blockIdx.x >> 8) & 1))
    for (int k = 0; k < FFT_STAGGER; k++) __builtin_amdgcn_s_sleep(127);
#endif
  for (int i = 0; i < n; i++) {
#if FFT_PRIO == 6
    prio_flag = ((unsigned)i >> FFT_PRIO_SH ^ prio_ph) & 1u;
    base_prio();
#endif
    // (X^a acc_c - acc_c), decomposed: the rotation image in this wave's own transpose area (its previous
    // user, the last inverse, is this wave: DS operations of a wave run in order)
    u32 st[16];
#if FFT_ROTPRIO
    __builtin_amdgcn_s_setprio(FFT_ROTPRIO);  // A/B: the rotation phase at a raised priority
#endif
    rotate_states(acc, ms2048(ct[i]), lane, T, st);
    double o0r[8], o0i[8], o1r[8], o1i[8];
    // level steps q = 0, 1, 2 (least significant first), each specialised at compile time: q = 0 starts the two
    // fma chains with a multiply (no zeroed partial sums), q = 2 takes the top digit (no carry bit, no next state)
    auto level = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int g = 3 * i + q;
#if FFT_MACPRIO
      if (q > 0 || FFT_ROTPRIO) base_prio();
#endif
      if constexpr (LDS_TW) {
        glds_barrier();  // step g's chunk is in K[g & 1]; every wave is done with K[(g + 1) & 1]
        if (g + 1 < n_steps) load_step<NW>(bsk, g + 1, sh.K[(g + 1) & 1], wave_s, lane);
      } else {
        // one buffer: every wave is done with step g - 1's chunk (the exchange's barriers order q = 0)
        if (q > 0) __syncthreads();
#if FFT_BUF_LDS
        load_step_buf<NW>(bsr, g, sh.K[0], wave_s, voff);
#else
        load_step<NW>(bsk, g, sh.K[0], wave_s, lane);
#endif
      }
      double xr[8], xi[8];
#pragma unroll
      for (int e = 0; e < 8; e++) {
        if constexpr (q == 2) {
          xr[e] = (double)decomp_top(st[e]);
          xi[e] = (double)decomp_top(st[e + 8]);
        } else {
          xr[e] = (double)decomp_step(st[e], 1u);
          xi[e] = (double)decomp_step(st[e + 8], 1u);
        }
      }
      // the slot twist rides in pass A's twisted DFT8 (twist_dft8_fwd)
#if FFT_PAIR_TWREG >= 2
      dft512_fwd_rab<true>(xr, xi, T, lane, tb, wa, wb);
#elif FFT_PAIR_TWREG
      dft512_fwd_ra<true>(xr, xi, T, lane, tb, wa, twB);
#else
      dft512_fwd_t<true, true>(xr, xi, T, lane, tb, twA, twB);
#endif
      if constexpr (!LDS_TW) glds_barrier();  // step g's chunk has landed
#if FFT_MACPRIO
      __builtin_amdgcn_s_setprio(3);  // the short MAC ahead of the other workgroup's transforms
#endif
      const double2* k0 = sh.K[LDS_TW ? (g & 1) : 0] + c * (2 * M) + lane;
      const double2* k1 = k0 + M;
#pragma unroll
      for (int e = 0; e < 8; e++) {
        const double2 u = k0[64 * e], v = k1[64 * e];
        if constexpr (q == 0) {
          mac_first(o0r[e], o0i[e], xr[e], xi[e], u);
          mac_first(o1r[e], o1i[e], xr[e], xi[e], v);
        } else {
          mac_next(o0r[e], o0i[e], xr[e], xi[e], u);
          mac_next(o1r[e], o1i[e], xr[e], xi[e], v);
        }
      }
    };
    level(std::integral_constant<int, 0>{});
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
#if FFT_MACPRIO && !FFT_XCHPRIO
    base_prio();
#endif
    // exchange the partial sums: publish O_(1-c)^c, take O_c^(1-c) (c wave-uniform: a scalar branch, no selects)
    double xr[8], xi[8];
    if (c_s) exchange_partials<1>(o0r, o0i, o1r, o1i, xr, xi, T, Tp, lane);
    else exchange_partials<0>(o0r, o0i, o1r, o1i, xr, xi, T, Tp, lane);
#if FFT_MACPRIO && FFT_XCHPRIO
    base_prio();  // A/B: the partial-sum exchange still at the MAC's priority
#endif
#if FFT_PAIR_TWREG >= 2
    dft512_inv_rb(xr, xi, T, lane, tb, wb, twI);
#else
    dft512_inv_t(xr, xi, T, lane, tb, twB, twI);
#endif
    twist_slots<true>(xr, xi);
#pragma unroll
    for (int e = 0; e < 8; e++) {
      acc[e] = ACC_ADD(acc[e], xr[e]);
      acc[e + 8] = ACC_ADD(acc[e + 8], xi[e]);
    }
  }
#if FFT_WGTIME
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    g_wgt[4 * blockIdx.x] = wg_t0;
    g_wgt[4 * blockIdx.x + 1] = t1;
    g_wgt[4 * blockIdx.x + 2] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID
    g_wgt[4 * blockIdx.x + 3] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC_ID
  }
#endif

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048 + c * N1K;
#pragma unroll
    for (int e = 0; e < 16; e++) oa[64 * e + lane] = acc[e];
  }
  if (WRITE_BIG) {
    // sample extraction at degree 0 (computations.rs:109-132): a'_0 = A[0], a'_j = -A[N-j], b' = B[0]
    u64* ob = out_big + b * (size_t)(N1K + 1);
    if (c == 0) {
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int idx = 64 * e + lane;
        if (idx == 0) ob[0] = acc[e];
        else ob[N1K - idx] = 0 - acc[e];
      }
    } else if (lane == 0) {
      ob[N1K] = acc[0];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Three waves per SIMD (round 6, FFT_G3): ONE workgroup per CU of G3_CTS = 6 ciphertexts x 2 component waves (768
// threads, <= 168 VGPRs).  The per-wave program is the pair kernel's -- rotate + decompose acc_c, three level steps
// (digits, DFT, MAC into both outputs' partial sums), the partial-sum exchange, one inverse -- with the same
// operation order (the oracle is unchanged), but
//   * every twiddle comes from LDS (pass A and the inverse's pass B' from their 8 KB tables, pass B / C' from the
//     1 KB compact table, fft512.h dft512_fwd_c), which frees the 60 registers the pair kernel keeps them in;
//   * one 32 KB level-step chunk serves 6 ciphertexts instead of 2: a third of the LDS-DMA bytes and of the BSK
//     stream per ciphertext;
//   * the batch is spread over rounds of one workgroup per CU with the ciphertext counts balanced (4096 on 256 CUs:
//     3 rounds, 16 ciphertexts per CU as 6 + 5 + 5) instead of a fixed 6 per workgroup (2.67 rounds).  Pairs beyond a
//     workgroup's count skip all compute but keep the barrier sequence.
// LDS: TW_A 8 KB | TW_I 8 KB | TW_B compact 1 KB | one 32 KB level step | 12 x 9 KB transpose areas = 160,768 B.
#ifndef FFT_G3
#define FFT_G3 0
#endif
#ifndef G3_TW_GLOBAL
#define G3_TW_GLOBAL 0
#endif
constexpr int G3_CTS = 6;
constexpr int G3_NW = 2 * G3_CTS;
struct G3Shared {
  double2 twA[M];
  double2 twI[M];
  double2 twB[64];                                 // [e][L & 7]
  double2 K[STEP_C64];
  double2 T[G3_NW][T_C64];
};
static_assert(sizeof(G3Shared) <= 163840, "G3 LDS");

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(64 * G3_NW, 1) void blind_rotate_fft_g3_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) G3Shared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = wave & 1;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  const int c_s = wave_s & 1;
  // balanced split: workgroup w takes B / G or B / G + 1 ciphertexts (G = gridDim.x)
  const size_t G = gridDim.x, w = blockIdx.x;
  const size_t per = B / G, extra = B % G;
  const size_t cnt = per + (w < extra ? 1 : 0);
  const size_t b0 = w * per + (w < extra ? w : extra);
  const int p = wave_s >> 1;
  const bool live = (size_t)p < cnt;
  const size_t b = live ? b0 + p : b0;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  double2* T = sh.T[wave];
  const double2* Tp = sh.T[wave ^ 1];
  const int n_steps = 3 * n;
  (void)n_steps;

  const __amdgpu_buffer_rsrc_t bsr =
      __builtin_amdgcn_make_buffer_rsrc((void*)bsk, (short)0, n * 6 * 2 * M * (int)sizeof(double2), 0x00020000);
  const int voff = lane * 16;
  for (int q = threadIdx.x; q < M; q += 64 * G3_NW) {
    sh.twA[q] = tw_g[TW_A + q];
    sh.twI[q] = tw_g[TW_I + q];
  }
  if (threadIdx.x < 64) sh.twB[threadIdx.x] = tw_g[TW_B + 64 * (threadIdx.x >> 3) + (threadIdx.x & 7)];

  u64 acc[16];
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
      acc[e] = c ? (neg ? 0 - v : v) : 0;
    }
  }
  __syncthreads();
  const TBase tb(lane);
#if G3_TW_GLOBAL
  // A/B: the twiddles straight from the global tables (L1 / L2 hits) instead of LDS
  const double2* twAl = tw_g + TW_A + lane;
  const double2* twIl = tw_g + TW_I + lane;
  const double2* twBc = tw_g + TW_B + (lane & 7);  // the full table at stride 64
  constexpr int BSTR = 64;
#else
  const double2* twAl = sh.twA + lane;
  const double2* twIl = sh.twI + lane;
  const double2* twBc = sh.twB + (lane & 7);
  constexpr int BSTR = 8;
#endif

  for (int i = 0; i < n; i++) {
    u32 st[16];
    if (live) rotate_states(acc, ms2048(ct[i]), lane, T, st);
    double o0r[8], o0i[8], o1r[8], o1i[8];
    auto level = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
      const int g = 3 * i + q;
#if FFT_MACPRIO
      if (q > 0) __builtin_amdgcn_s_setprio(0);
#endif
      if (q > 0) __syncthreads();  // every wave is done with step g - 1's chunk (the exchange's barriers order q = 0)
      {
        const int ii = g / 3;
        for (int blk = wave_s; blk < 32; blk += G3_NW) {
          const int cc = blk >> 4;
          const int soff = ((ii * 6 + cc * 3 + q) * (2 * M)) * (int)sizeof(double2) + (blk & 15) * 1024;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              bsr, (__attribute__((address_space(3))) void*)((char*)sh.K + blk * 1024), 16, voff, soff, 0, 0);
        }
      }
      double xr[8], xi[8];
      if (live) {
#pragma unroll
        for (int e = 0; e < 8; e++) {
          if constexpr (q == 2) {
            xr[e] = (double)decomp_top(st[e]);
            xi[e] = (double)decomp_top(st[e + 8]);
          } else {
            xr[e] = (double)decomp_step(st[e], 1u);
            xi[e] = (double)decomp_step(st[e + 8], 1u);
          }
        }
        dft512_fwd_c<true, BSTR>(xr, xi, T, lane, tb, twAl, twBc);
      }
      glds_barrier();  // step g's chunk has landed
      if (live) {
#if FFT_MACPRIO
        __builtin_amdgcn_s_setprio(3);
#endif
        const double2* k0 = sh.K + c * (2 * M) + lane;
        const double2* k1 = k0 + M;
#pragma unroll
        for (int e = 0; e < 8; e++) {
          const double2 u = k0[64 * e], v = k1[64 * e];
          if constexpr (q == 0) {
            mac_first(o0r[e], o0i[e], xr[e], xi[e], u);
            mac_first(o1r[e], o1i[e], xr[e], xi[e], v);
          } else {
            mac_next(o0r[e], o0i[e], xr[e], xi[e], u);
            mac_next(o1r[e], o1i[e], xr[e], xi[e], v);
          }
        }
      }
    };
    level(std::integral_constant<int, 0>{});
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
#if FFT_MACPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    double xr[8], xi[8];
    if (live) {
      if (c_s) exchange_partials<1>(o0r, o0i, o1r, o1i, xr, xi, T, Tp, lane);
      else exchange_partials<0>(o0r, o0i, o1r, o1i, xr, xi, T, Tp, lane);
      dft512_inv_c<BSTR>(xr, xi, T, lane, tb, twBc, twIl);
      twist_slots<true>(xr, xi);
#pragma unroll
      for (int e = 0; e < 8; e++) {
        acc[e] = ACC_ADD(acc[e], xr[e]);
        acc[e + 8] = ACC_ADD(acc[e + 8], xi[e]);
      }
    } else {
      __syncthreads();  // the exchange's two barriers
      __syncthreads();
    }
  }

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048 + c * N1K;
#pragma unroll
    for (int e = 0; e < 16; e++) oa[64 * e + lane] = acc[e];
  }
  if (WRITE_BIG) {
    u64* ob = out_big + b * (size_t)(N1K + 1);
    if (c == 0) {
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int idx = 64 * e + lane;
        if (idx == 0) ob[0] = acc[e];
        else ob[N1K - idx] = 0 - acc[e];
      }
    } else if (lane == 0) {
      ob[N1K] = acc[0];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Latency-mode blind rotation (small batches): ONE ciphertext per workgroup of 8 waves.  Per CMUX:
//   A  waves 0..5: wave r = chain position (c, q) (c = r / 3; q = 0, 1, 2: levels least significant
//      first) rotates + decomposes accumulator polynomial c, keeps step q's digits and transforms
//      them -> F[r]                                                     (6 transforms in parallel)
//   B  all 8 waves: O_j = O_j^0 + O_j^1, O_j^c = fma chain over r = 3c .. 3c + 2 of F[r] (.) BSK_i[r][j]
//      (the oracle's split order) on 2 of the 8 slots each (j = wave >> 2); the BSK words come straight from L2, loaded into
//      registers before phase A so their latency hides behind the transforms
//   C  waves 0, 1: inverse transform of O_j, acc_j += rint mod 2^64      (2 transforms in parallel)
// Three barriers per CMUX; the critical path is 1 forward + 1 inverse transform + 1/4 of the MAC
// instead of 6 + 2 + all of it.  LDS (tables first: small DS immediates): tw 32 KB | acc 16 KB |
// F 48 KB | 6 transpose areas 54 KB (O_0, O_1 alias areas 2, 3, dead after phase A) = 150 KB.
constexpr int FL_THREADS = 512;
constexpr int FL_MAXN = 1024;  // rotation amounts staged in LDS up to this LWE dimension (global reads above)
struct FftLatShared {
  double2 tw[TW_C64];
  u64 A[2][N1K];
  double2 F[6][M];
  double2 T[6][T_C64];
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
    for (int t = 0; t < 2; t++) kv[r][t] = bsk[((size_t)(i * 6 + r) * 2 + j) * M + 64 * (s0 + t) + lane];
}

// FFT_LAT_LDSBAR 1 (round 6): the latency kernel's three barriers per CMUX wait for LDS only (s_waitcnt lgkmcnt(0) +
// s_barrier).  Every cross-wave exchange of the kernel goes through LDS; __syncthreads also drains vmcnt, which made
// the first barrier of CMUX i wait for the key words of CMUX i + 1 that FFT_LAT_PREFETCH had just requested (an L2 /
// HBM round trip on the critical path of every CMUX) -- with LDS-only barriers they stay in flight for a whole CMUX.
#ifndef FFT_LAT_LDSBAR
#define FFT_LAT_LDSBAR 1
#endif
__device__ __forceinline__ void lat_barrier() {
#if FFT_LAT_LDSBAR
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  __syncthreads();
#endif
}

// one CMUX of the latency kernel (phases A, B, C and their three barriers)
#ifndef FFT_LATSTAMP
#define FFT_LATSTAMP 0
#endif
#if FFT_LATSTAMP
// diagnostic build only: per-CMUX phase times of the latency kernel (s_memrealtime, 100 MHz), summed per wave:
// [0] CMUX start -> this wave done with phase A (before barrier 1), [1] -> past barrier 1, [2] -> done with phase B,
// [3] -> past barrier 2, [4] -> done with phase C, [5] -> past barrier 3
struct LatStamp {
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0}, t0 = 0;
  __device__ __forceinline__ void start() { t0 = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void mark(int k) { acc[k] += __builtin_amdgcn_s_memrealtime() - t0; }
};
__device__ unsigned long long g_latst[8 * 8 * 6];  // workgroup 0..7 x wave x phase mark
#define LS_START(st) st.start()
#define LS_MARK(st, k) st.mark(k)
#else
struct LatStamp {};
#define LS_START(st)
#define LS_MARK(st, k)
#endif
__device__ __forceinline__ void lat_cmux(FftLatShared& sh, const u64* __restrict__ ct, int i, int wave, int lane,
                                         TBase tb, int j, int s0, const double2 (&kv)[6][2], LatStamp& ls) {
  LS_START(ls);
  const int a = i < FL_MAXN ? (int)sh.ab[i] : ms2048(ct[i]);
  if (wave < 6) {  // phase A
    const int c = wave / 3, q = wave % 3;
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
    double xr[8], xi[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      xr[e] = (double)dg[e];
      xi[e] = (double)dg[e + 8];
    }
    dft512_fwd<true, true>(xr, xi, sh.T[wave], lane, tb, sh.tw);
#pragma unroll
    for (int e = 0; e < 8; e++) sh.F[wave][64 * e + lane] = make_double2(xr[e], xi[e]);
  }
  LS_MARK(ls, 0);
  lat_barrier();
  LS_MARK(ls, 1);
  {  // phase B
    double2* O = sh.T[2 + j];
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const int e = s0 + t;
      double re[2], im[2];  // per-component chains (the first term a multiply), then one add (oracle order)
#pragma unroll
      for (int r = 0; r < 6; r++) {
        const double2 D = sh.F[r][64 * e + lane], K = kv[r][t];
        const int cc = r / 3;
        if (r % 3 == 0) mac_first(re[cc], im[cc], D.x, D.y, K);
        else mac_next(re[cc], im[cc], D.x, D.y, K);
      }
      O[64 * e + lane] = make_double2(re[0] + re[1], im[0] + im[1]);
    }
  }
  LS_MARK(ls, 2);
  lat_barrier();
  LS_MARK(ls, 3);
  if (wave < 2) {  // phase C
    const double2* O = sh.T[2 + wave];
    double xr[8], xi[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const double2 v = O[64 * e + lane];
      xr[e] = v.x;
      xi[e] = v.y;
    }
    fft_inv_real(xr, xi, sh.T[wave], lane, tb, sh.tw);
    u64* acc = sh.A[wave];
#pragma unroll
    for (int e = 0; e < 8; e++) {
      acc[64 * e + lane] = ACC_ADD(acc[64 * e + lane], xr[e]);
      acc[64 * (e + 8) + lane] = ACC_ADD(acc[64 * (e + 8) + lane], xi[e]);
    }
  }
  LS_MARK(ls, 4);
  lat_barrier();
  LS_MARK(ls, 5);
}

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(FL_THREADS, 1) void blind_rotate_fft_lat_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const double2* __restrict__ bsk, const double2* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) FftLatShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = blockIdx.x;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  const TBase tb(lane);

  for (int q = threadIdx.x; q < TW_C64; q += FL_THREADS) sh.tw[q] = tw_g[q];
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

  const int j = wave >> 2, s0 = (wave & 3) * 2;  // phase B: output j, slots s0, s0 + 1
  LatStamp ls;
#if FFT_LAT_PREFETCH
  // key words one CMUX ahead (two register sets, the loop unrolled by two): a CMUX's row arrives while the
  // previous CMUX runs instead of behind this CMUX's phase A
  double2 kva[6][2], kvb[6][2];
  lat_load_key(bsk, 0, j, s0, lane, kva);
  for (int i = 0; i < n; i += 2) {
    if (i + 1 < n) lat_load_key(bsk, i + 1, j, s0, lane, kvb);
    lat_cmux(sh, ct, i, wave, lane, tb, j, s0, kva, ls);
    if (i + 1 >= n) break;
    if (i + 2 < n) lat_load_key(bsk, i + 2, j, s0, lane, kva);
    lat_cmux(sh, ct, i + 1, wave, lane, tb, j, s0, kvb, ls);
  }
#else
  for (int i = 0; i < n; i++) {
    double2 kv[6][2];  // phase-B key words of this CMUX, requested now, consumed after phase A
    lat_load_key(bsk, i, j, s0, lane, kv);
    lat_cmux(sh, ct, i, wave, lane, tb, j, s0, kv, ls);
  }
#endif

#if FFT_LATSTAMP
  if (lane == 0 && b < 8)
    for (int k = 0; k < 6; k++) g_latst[(b * 8 + wave) * 6 + k] = ls.acc[k];
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

size_t fft_tables_len() { return 2 * fftk::TW_C64; }

// N = 1024 tables with the twist merged into the passes (fft512.h, "N = 1024 merged twist"):
//   TW_A[e][L] = zeta^(L (1 + 4 e)),  TW_B as before,  TW_I[e][L] = zeta^((n0 + 8 e)(4 k0 + 1)) (L = n0 + 8 k0),
// zeta = e^(2 pi i / 2048); TW_TWIST keeps zeta^j (the slot constants are its entries j = 64 e)
void make_fft_tables(double* t) {
  using namespace fftk;
  for (uint32_t j = 0; j < (uint32_t)M; j++) twiddle(j, 4 * M, &t[2 * (TW_TWIST + j)], &t[2 * (TW_TWIST + j) + 1]);
  for (uint32_t e = 0; e < 8; e++)
    for (uint32_t L = 0; L < 64; L++) {
      twiddle((L * (1 + 4 * e)) % (4 * M), 4 * M, &t[2 * (TW_A + 64 * e + L)], &t[2 * (TW_A + 64 * e + L) + 1]);
      twiddle((8 * (L & 7) * e) % M, M, &t[2 * (TW_B + 64 * e + L)], &t[2 * (TW_B + 64 * e + L) + 1]);
      twiddle((((L & 7) + 8 * e) * (4 * (L >> 3) + 1)) % (4 * M), 4 * M, &t[2 * (TW_I + 64 * e + L)],
              &t[2 * (TW_I + 64 * e + L) + 1]);
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
  hipLaunchKernelGGL(fftk::bsk_to_fourier_kernel, dim3((unsigned)polys), dim3(64), 0, s, bsk_std, (double2*)bsk_f,
                     (const double2*)tw);
  return hipGetLastError();
}

hipError_t launch_blind_rotate_fft(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                   int n_lut, const double* bsk_f, const double* tw, u64* out_big, u64* out_acc,
                                   hipStream_t s, size_t latency_max_batch) {
  using namespace fftk;
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
#if FFT_G3
  {
    // rounds of one workgroup per CU, at most G3_CTS ciphertexts each, counts balanced over the whole grid
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    const size_t rounds = (B + (size_t)G3_CTS * cus - 1) / ((size_t)G3_CTS * cus);
    size_t nwg = rounds * (size_t)cus;
    if (nwg > B) nwg = B;
    dim3 grid((unsigned)nwg), block(64 * G3_NW);
    if (out_acc && out_big)
      hipLaunchKernelGGL((blind_rotate_fft_g3_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    else if (out_acc)
      hipLaunchKernelGGL((blind_rotate_fft_g3_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    else
      hipLaunchKernelGGL((blind_rotate_fft_g3_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bk, t, out_big, out_acc);
    return hipGetLastError();
  }
#endif
  constexpr int CTS = FFT_PAIR_CTS;
  dim3 grid((unsigned)((B + CTS - 1) / CTS)), block(128 * CTS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_fft_pair_kernel<CTS, true, true>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_fft_pair_kernel<CTS, true, false>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_fft_pair_kernel<CTS, false, true>), grid, block, 0, s, lwe_in, n, B, luts,
                       lut_index, n_lut, bk, t, out_big, out_acc);
  return hipGetLastError();
}

#if FFT_LATSTAMP
extern "C" int tfhe_hip_debug_latstamps(unsigned long long* out, size_t n) {
  if (n > 8 * 8 * 6) n = 8 * 8 * 6;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fftk::g_latst), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
#if FFT_WGTIME
extern "C" int tfhe_hip_debug_wgtimes(unsigned long long* out, size_t n) {
  if (n > 4 * 16384) n = 4 * 16384;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fftk::g_wgt), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_sample_extract_torus(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (N1K + 1);
  hipLaunchKernelGGL(fftk::sample_extract_torus_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc, B,
                     out);
  return hipGetLastError();
}

hipError_t launch_fft_fwd(const u64* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fftk::fft_fwd_kernel, dim3((unsigned)count), dim3(64), 0, s, in, (double2*)out,
                     (const double2*)tw);
  return hipGetLastError();
}

hipError_t launch_fft_inv(const double* in, size_t count, double* out, const double* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(fftk::fft_inv_kernel, dim3((unsigned)count), dim3(64), 0, s, (const double2*)in, out,
                     (const double2*)tw);
  return hipGetLastError();
}

}  // namespace tfhe
