// pbs_n2048.hip — gfx950 PBS kernels for N = 2048 (P-FHEVM: n = 918, k = 1, PBS 2^23 x 1,
// KS 2^4 x 4, KS -> PBS order; SURVEY §8f f4, parameters from sdk/relayer/src/tfhe.ts:14-19).
//
// A 2048-coefficient polynomial is held by TWO wavefronts: wave h owns coefficients 2m + h
// (m = 64 e + L, the natural layout of a 1024-point half).  The negacyclic NTT is decimation in
// time:  a(x) = a_e(x^2) + x a_o(x^2), so at x = psi^(2j+1) (psi: primitive 4096-th root)
//   A[j] = E[j] + psi^(2j+1) O[j],   A[j + 1024] = E[j] - psi^(2j+1) O[j],
// where E / O are the 1024-point negacyclic NTTs of the halves with root psi^2 — each wave runs the
// unchanged ntt1024_fwd (ntt1024.h) on its half.  Slot (L, e) holds the same j in both waves, so
// the combine needs 8 values per lane from the partner wave (one LDS exchange): wave h keeps the
// slots e in [8h, 8h + 8) and produces, in register slot s (p = s & 7, upper = s >> 3),
//   A[ntt_natural_index(L, 8h + p) + 1024 upper].
// The inverse mirrors it (GS combine, exchange back, ntt1024_inv): x 1024 x 2 = x N, folded into the
// BSK together with the forward scaling.
#include <hip/hip_runtime.h>

#include "gl64.h"
#include "ntt1024.h"
#include "ntt16.h"
#include "pbs_kernels.h"

namespace tfhe {

constexpr int N2K = 2048;
constexpr int TWC_FWD = TW_U64;           // combine twiddles psi^(2j+1), [h][p][L] (1024 per h)
constexpr int TWC_INV = TW_U64 + N2K;     // and their inverses
constexpr int TW2K_U64 = TW_U64 + 2 * N2K;

// round(x * 4096 / 2^64) mod 4096
__device__ __forceinline__ int ms4096(u64 x) { return (int)((((x >> 51) + 1) >> 1) & 4095u); }

// (X^t v)[i] for a negacyclic length-2048 polynomial v held in LDS in split layout
// (coefficient c at R[(c & 1) * 1024 + (c >> 1)]), t in [0, 4096).
__device__ __forceinline__ u64 rot_read_split(const u64* R, int i, int t) {
  int d = i - t;
  bool neg = false;
  if (d < 0) { d += N2K; neg = !neg; }
  if (d < 0) { d += N2K; neg = !neg; }
  const u64 x = R[(d & 1) * N1K + (d >> 1)];
  return neg ? gl_neg(x) : x;
}

// same, natural layout in global memory (the LUT)
__device__ __forceinline__ u64 rot_read_2048(const u64* v, int i, int t) {
  int d = i - t;
  bool neg = false;
  if (d < 0) { d += N2K; neg = !neg; }
  if (d < 0) { d += N2K; neg = !neg; }
  const u64 x = v[d];
  return neg ? gl_neg(x) : x;
}

// tfhe-rs SignedDecomposer, base 2^23 x 1 level: closest representable at 23 bits, digit in
// [-2^22, 2^22] (the tie 2^22 stays positive: the next state is 0, so no carry).
__device__ __forceinline__ int decomp_23x1(u64 x) {
  const u32 state = (u32)(((x >> 40) + 1) >> 1) & 0x7FFFFFu;
  const u32 carry = (((state - 1u) & state) >> 22) & 1u;
  return (int)state - (int)(carry << 23);
}

// Forward combine (after each wave's ntt1024_fwd of its half).  S = this wave's LDS exchange
// area, P = the partner's.  Contains one __syncthreads: all waves of the block must call it.
template <int h>
__device__ __forceinline__ void combine_fwd(u64 (&x)[16], u64* S, const u64* P, int lane, const u64* twc) {
#pragma unroll
  for (int p = 0; p < 8; p++) S[64 * p + lane] = x[8 * (1 - h) + p];  // the slots the partner keeps
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 8; p++) {
    const u64 r = P[64 * p + lane];
    const u64 E = h ? r : x[p];
    const u64 O = h ? x[8 + p] : r;
    const u64 t = gl_mul(O, twc[(8 * h + p) * 64 + lane]);
    x[p] = gl_add(E, t);
    x[8 + p] = gl_sub(E, t);
  }
}

// Inverse combine: slots (A[j], A[j + 1024]) -> wave 0 gets 2E (all 16 slots), wave 1 gets 2O.
// Two __syncthreads (the exchange area is the caller's NTT scratch, reused right after).
template <int h>
__device__ __forceinline__ void combine_inv(u64 (&x)[16], u64* S, const u64* P, int lane, const u64* twci) {
  u64 keep[8];
#pragma unroll
  for (int p = 0; p < 8; p++) {
    const u64 a = x[p], b = x[8 + p];
    const u64 Ep = gl_add(a, b);
    const u64 Op = gl_mul(gl_sub(a, b), twci[(8 * h + p) * 64 + lane]);
    S[64 * p + lane] = h ? Ep : Op;  // wave 0 sends O', wave 1 sends E'
    keep[p] = h ? Op : Ep;
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 8; p++) {
    const u64 r = P[64 * p + lane];
    x[h ? p : 8 + p] = r;            // partner's slots
    x[h ? 8 + p : p] = keep[p];      // own slots
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// BSK conversion and natural-order NTTs: one block = 2 wavefronts = one polynomial.
__global__ __launch_bounds__(128) void bsk_to_ntt2048_kernel(const u64* __restrict__ bsk_std, u64* __restrict__ bsk_ntt,
                                                             const u64* __restrict__ tw, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[2][T_LDS];
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t q = blockIdx.x;
  const u64* src = bsk_std + q * N2K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = src[2 * (64 * e + lane) + h];
  ntt1024_fwd(x, T[h], lane, tw);
  if (h) combine_fwd<1>(x, T[1], T[0], lane, tw + TWC_FWD);
  else combine_fwd<0>(x, T[0], T[1], lane, tw + TWC_FWD);
  u64* dst = bsk_ntt + q * N2K + h * N1K;
#pragma unroll
  for (int s = 0; s < 16; s++) dst[64 * s + lane] = gl_mul(x[s], ninv);
}

__global__ __launch_bounds__(128) void ntt2048_fwd_kernel(u64* __restrict__ polys, const u64* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) u64 T[2][T_LDS];
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u64* p = polys + (size_t)blockIdx.x * N2K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = p[2 * (64 * e + lane) + h];
  __syncthreads();  // both halves read before anything is written back
  ntt1024_fwd(x, T[h], lane, tw);
  if (h) combine_fwd<1>(x, T[1], T[0], lane, tw + TWC_FWD);
  else combine_fwd<0>(x, T[0], T[1], lane, tw + TWC_FWD);
#pragma unroll
  for (int s = 0; s < 16; s++) p[ntt_natural_index(lane, 8 * h + (s & 7)) + N1K * (s >> 3)] = x[s];
}

__global__ __launch_bounds__(128) void ntt2048_inv_kernel(u64* __restrict__ polys, const u64* __restrict__ tw, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[2][T_LDS];
  const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u64* p = polys + (size_t)blockIdx.x * N2K;
  u64 x[16];
#pragma unroll
  for (int s = 0; s < 16; s++) x[s] = p[ntt_natural_index(lane, 8 * h + (s & 7)) + N1K * (s >> 3)];
  __syncthreads();
  if (h) combine_inv<1>(x, T[1], T[0], lane, tw + TWC_INV);
  else combine_inv<0>(x, T[0], T[1], lane, tw + TWC_INV);
  ntt1024_inv(x, T[h], lane, tw);
#pragma unroll
  for (int e = 0; e < 16; e++) p[2 * (64 * e + lane) + h] = gl_mul(x[e], ninv);
}

// ---------------------------------------------------------------------------------------------
// Blind rotation, N = 2048: a workgroup = 8 wavefronts = 4 ciphertexts x 2 halves, walking the CMUX
// loop in lockstep.  Per CMUX and component c (accumulator polynomial): both halves are written to
// the ciphertext's LDS area in split layout, rotated + decomposed (1 level), forward-transformed
// (ntt1024 + combine), then MAC'd against BSK_i[c][j] for j = 0, 1.  The BSK is consumed in 4 steps
// of one 16 KB polynomial (device layout [i][c][j][h][s][L]) streamed once per workgroup into LDS
// (global_load_lds, double-buffered).  LDS: 4 x 17 KB (rotation buffer aliased with the two waves'
// NTT scratch / exchange areas) + 32 KB BSK + 32 KB twiddles = 134 KB; the combine twiddles are read
// from global memory (L1/L2 resident).
constexpr int B2_CTS = 4;
constexpr int B2_THREADS = 128 * B2_CTS;
constexpr int B2_CHUNK = N2K;                       // one BSK polynomial: 16 KB
constexpr int B2_CHUNK_GLDS = B2_CHUNK * 8 / 1024;  // 16 x 1 KB wave-instructions

struct Br2Shared {
  u64 T[B2_CTS][2 * T_LDS];
  u64 K[2][B2_CHUNK];
  u64 tw[TW_U64];
};

__device__ __forceinline__ void load_chunk2(const u64* __restrict__ bsk, int g, u64* dst, int wave, int lane) {
  const char* src = (const char*)(bsk + (size_t)g * B2_CHUNK);
#pragma unroll
  for (int q = 0; q < B2_CHUNK_GLDS / 8; q++) {
    const int blk = wave * (B2_CHUNK_GLDS / 8) + q;
    __builtin_amdgcn_global_load_lds((const void*)(src + blk * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)((char*)dst + blk * 1024), 16, 0, 0);
  }
}

// component c of CMUX i: rotate/decompose acc_c, transform, accumulate into out0 / out1
template <int h>
__device__ __forceinline__ void ext_prod_2048(const u64 (&acc)[16], int a, int c, int i, int n_steps, Br2Shared& sh,
                                              u64* R, u64* S, const u64* P, int wave, int lane,
                                              const u64* __restrict__ bsk, const u64* __restrict__ twc,
                                              u64 (&out0)[16], u64 (&out1)[16]) {
#pragma unroll
  for (int e = 0; e < 16; e++) R[h * N1K + 64 * e + lane] = acc[e];
  __syncthreads();
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) {
    const int d = decomp_23x1(gl_sub(rot_read_split(R, 2 * (64 * e + lane) + h, a), acc[e]));
    x[e] = gl_from_i32(d);
  }
  __syncthreads();  // rotation reads done before the NTT scratch (aliased) is written
  ntt1024_fwd(x, S, lane, sh.tw);
  combine_fwd<h>(x, S, P, lane, twc);
#pragma unroll 1
  for (int j = 0; j < 2; j++) {
    const int g = i * 4 + c * 2 + j;
    glds_barrier();  // chunk g landed everywhere; buffer (g+1)&1 free; exchange reads done
    if (g + 1 < n_steps) load_chunk2(bsk, g + 1, sh.K[(g + 1) & 1], wave, lane);
    const u64* k = sh.K[g & 1] + h * N1K + lane;
    if (j == 0) {
#pragma unroll
      for (int s = 0; s < 16; s++) out0[s] = gl_mac_lazy(out0[s], x[s], k[64 * s]);
    } else {
#pragma unroll
      for (int s = 0; s < 16; s++) out1[s] = gl_mac_lazy(out1[s], x[s], k[64 * s]);
    }
  }
}

// the body for half h (compile-time: no wave-uniform selects); both halves run the same barriers
template <int h, bool WRITE_ACC, bool WRITE_BIG>
__device__ __forceinline__ void br2048_body(Br2Shared& sh, const u64* __restrict__ lwe_in, int n, size_t B,
                                            const u64* __restrict__ luts, const u32* __restrict__ lut_index, int n_lut,
                                            const u64* __restrict__ bsk, const u64* __restrict__ tw_g,
                                            u64* __restrict__ out_big, u64* __restrict__ out_acc) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = wave >> 1;
  const size_t b_raw = (size_t)blockIdx.x * B2_CTS + q;
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding ciphertexts run a copy of the last one, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  u64* R = sh.T[q];
  u64* S = sh.T[q] + h * T_LDS;
  const u64* P = sh.T[q] + (1 - h) * T_LDS;
  const int n_steps = n * 4;
  const u64* twc = tw_g + TWC_FWD;
  const u64* twci = tw_g + TWC_INV;

  for (int t = threadIdx.x; t < TW_U64; t += B2_THREADS) sh.tw[t] = tw_g[t];
  load_chunk2(bsk, 0, sh.K[0], wave, lane);

  u64 accA[16], accB[16];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N2K;
    const int s0 = (4096 - ms4096(ct[n])) & 4095;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      accA[e] = 0;
      accB[e] = rot_read_2048(lut, 2 * (64 * e + lane) + h, s0);
    }
  }

  for (int i = 0; i < n; i++) {
    const int a = ms4096(ct[i]);
    // opaque per-iteration copies: keeps the compiler from hoisting the 32 loop-invariant combine
    // twiddle loads out of the CMUX loop (that would pin 64 VGPRs and spill)
    const u64* twc_i = twc;
    const u64* twci_i = twci;
    asm volatile("" : "+s"(twc_i), "+s"(twci_i));
    u64 out0[16], out1[16];
#pragma unroll
    for (int s = 0; s < 16; s++) { out0[s] = 0; out1[s] = 0; }
    __syncthreads();  // the previous CMUX's inverse transforms are done with the LDS area
    ext_prod_2048<h>(accA, a, 0, i, n_steps, sh, R, S, P, wave, lane, bsk, twc_i, out0, out1);
    ext_prod_2048<h>(accB, a, 1, i, n_steps, sh, R, S, P, wave, lane, bsk, twc_i, out0, out1);
#pragma unroll
    for (int s = 0; s < 16; s++) { out0[s] = gl_canon(out0[s]); out1[s] = gl_canon(out1[s]); }
    combine_inv<h>(out0, S, P, lane, twci_i);
    ntt1024_inv(out0, S, lane, sh.tw);
#pragma unroll
    for (int e = 0; e < 16; e++) accA[e] = gl_add(accA[e], out0[e]);
    combine_inv<h>(out1, S, P, lane, twci_i);
    ntt1024_inv(out1, S, lane, sh.tw);
#pragma unroll
    for (int e = 0; e < 16; e++) accB[e] = gl_add(accB[e], out1[e]);
  }

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * (2 * N2K);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int idx = 2 * (64 * e + lane) + h;
      oa[idx] = accA[e];
      oa[N2K + idx] = accB[e];
    }
  }
  if (WRITE_BIG) {
    // sample extraction at degree 0 (computations.rs:109-132 semantics), Z_p -> 2^64
    u64* ob = out_big + b * (size_t)(N2K + 1);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int idx = 2 * (64 * e + lane) + h;
      if (idx == 0) ob[0] = gl_to_torus(accA[e]);
      else ob[N2K - idx] = gl_to_torus(gl_neg(accA[e]));
    }
    if (h == 0 && lane == 0) ob[N2K] = gl_to_torus(accB[0]);
  }
}

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(B2_THREADS, 1) void blind_rotate2048_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const u64* __restrict__ bsk, const u64* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) Br2Shared sh;
  if ((threadIdx.x >> 6) & 1)
    br2048_body<1, WRITE_ACC, WRITE_BIG>(sh, lwe_in, n, B, luts, lut_index, n_lut, bsk, tw_g, out_big, out_acc);
  else
    br2048_body<0, WRITE_ACC, WRITE_BIG>(sh, lwe_in, n, B, luts, lut_index, n_lut, bsk, tw_g, out_big, out_acc);
}

// ---------------------------------------------------------------------------------------------
// Latency-mode blind rotation, N = 2048: ONE ciphertext per workgroup of 8 waves (radix circuits'
// lockstep levels).  Per CMUX:
//   A   waves 0..3 = (c, h): rotate/decompose half h of accumulator polynomial c, ntt1024_fwd,
//       send the partner's combine slots through LDS;   A2: combine -> F[c] (device layout)
//   B   all 8 waves: pointwise MAC over 256 positions each, both outputs j, in place in F
//   C   waves 0..3 = (j, h): inverse combine (exchange), ntt1024_inv, acc_j half += ...
// Five barriers per CMUX, executed by all waves.  LDS: accumulator 32 KB (split layout), F 32 KB,
// 4 NTT scratch areas 35 KB, 4 exchange areas 16 KB, twiddles 32 KB = 147 KB.
struct Lat2Shared {
  u64 A[2][N2K];          // accumulator polynomials, split layout [h][m]
  u64 F[2][N2K];          // NTT(digits_c), then MAC outputs out_j, device layout [h][s][L]
  u64 T[4][T_LDS];        // NTT scratch of waves 0..3
  u64 X[4][8 * 64];       // combine exchange areas
  u64 tw[TW_U64];
};

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(512, 1) void blind_rotate2048_lat_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const u64* __restrict__ bsk, const u64* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) Lat2Shared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = blockIdx.x;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  const bool act = wave < 4;
  const int hi = wave >> 1, h = wave & 1;  // (c or j, half) of the active waves
  const u64* twc = tw_g + TWC_FWD;
  const u64* twci = tw_g + TWC_INV;

  for (int q = threadIdx.x; q < TW_U64; q += 512) sh.tw[q] = tw_g[q];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N2K;
    const int s0 = (4096 - ms4096(ct[n])) & 4095;
    for (int i = threadIdx.x; i < N2K; i += 512) {
      sh.A[0][(i & 1) * N1K + (i >> 1)] = 0;
      sh.A[1][(i & 1) * N1K + (i >> 1)] = rot_read_2048(lut, i, s0);
    }
  }

  for (int i = 0; i < n; i++) {
    const int a = ms4096(ct[i]);
    __syncthreads();  // B0: accumulator (and twiddles, first time) visible
    u64 x[16];
    if (act) {  // A: digits of half h of polynomial c = hi, forward transform
      const u64* acc = sh.A[hi];
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int m = 64 * e + lane;
        x[e] = gl_from_i32(decomp_23x1(gl_sub(rot_read_split(acc, 2 * m + h, a), acc[h * N1K + m])));
      }
      ntt1024_fwd(x, sh.T[wave], lane, sh.tw);
#pragma unroll
      for (int p = 0; p < 8; p++) sh.X[wave][64 * p + lane] = x[8 * (1 - h) + p];
    }
    __syncthreads();  // B1
    if (act) {  // A2: combine with the partner's slots
      const u64* P = sh.X[wave ^ 1];
#pragma unroll
      for (int p = 0; p < 8; p++) {
        const u64 r = P[64 * p + lane];
        const u64 E = h ? r : x[p];
        const u64 O = h ? x[8 + p] : r;
        const u64 t = gl_mul(O, twc[(8 * h + p) * 64 + lane]);
        sh.F[hi][h * N1K + 64 * p + lane] = gl_add(E, t);
        sh.F[hi][h * N1K + 64 * (8 + p) + lane] = gl_sub(E, t);
      }
    }
    __syncthreads();  // B2
    {  // B: out_j[pos] = F0[pos] BSK[i][0][j][pos] + F1[pos] BSK[i][1][j][pos], in place
      const u64* k = bsk + (size_t)i * 4 * N2K;
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int pos = wave * 256 + 64 * t + lane;
        const u64 f0 = sh.F[0][pos], f1 = sh.F[1][pos];
        u64 o0 = gl_mac_lazy(0, f0, k[pos]);
        o0 = gl_mac_lazy(o0, f1, k[2 * N2K + pos]);
        u64 o1 = gl_mac_lazy(0, f0, k[N2K + pos]);
        o1 = gl_mac_lazy(o1, f1, k[3 * N2K + pos]);
        sh.F[0][pos] = gl_canon(o0);
        sh.F[1][pos] = gl_canon(o1);
      }
    }
    __syncthreads();  // B3
    u64 keep[8];
    if (act) {  // C: inverse combine of out_j (j = hi), own slots p, send the partner's
#pragma unroll
      for (int p = 0; p < 8; p++) {
        const u64 y0 = sh.F[hi][h * N1K + 64 * p + lane], y1 = sh.F[hi][h * N1K + 64 * (8 + p) + lane];
        const u64 Ep = gl_add(y0, y1);
        const u64 Op = gl_mul(gl_sub(y0, y1), twci[(8 * h + p) * 64 + lane]);
        sh.X[wave][64 * p + lane] = h ? Ep : Op;
        keep[p] = h ? Op : Ep;
      }
    }
    __syncthreads();  // B4
    if (act) {  // C2: assemble the half, inverse transform, accumulate
      const u64* P = sh.X[wave ^ 1];
#pragma unroll
      for (int p = 0; p < 8; p++) {
        x[h ? p : 8 + p] = P[64 * p + lane];
        x[h ? 8 + p : p] = keep[p];
      }
      ntt1024_inv(x, sh.T[wave], lane, sh.tw);
      u64* acc = sh.A[hi] + h * N1K;
#pragma unroll
      for (int e = 0; e < 16; e++) acc[64 * e + lane] = gl_add(acc[64 * e + lane], x[e]);
    }
  }
  __syncthreads();

  if (WRITE_ACC) {
    u64* oa = out_acc + b * (2 * N2K);
    for (int i = threadIdx.x; i < N2K; i += 512) {
      oa[i] = sh.A[0][(i & 1) * N1K + (i >> 1)];
      oa[N2K + i] = sh.A[1][(i & 1) * N1K + (i >> 1)];
    }
  }
  if (WRITE_BIG) {
    u64* ob = out_big + b * (size_t)(N2K + 1);
    for (int q = threadIdx.x; q <= N2K; q += 512) {
      u64 v;
      if (q == N2K) v = sh.A[1][0];
      else if (q == 0) v = sh.A[0][0];
      else v = gl_neg(sh.A[0][((N2K - q) & 1) * N1K + ((N2K - q) >> 1)]);
      ob[q] = gl_to_torus(v);
    }
  }
}

__global__ void sample_extract2048_kernel(const u64* __restrict__ acc, size_t B, u64* __restrict__ out) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * (N2K + 1)) return;
  const size_t b = gid / (N2K + 1);
  const int j = (int)(gid % (N2K + 1));
  const u64* A = acc + b * (2 * N2K);
  u64 v;
  if (j == N2K) v = A[N2K];
  else if (j == 0) v = A[0];
  else v = gl_neg(A[N2K - j]);
  out[gid] = gl_to_torus(v);
}

// ---------------------------------------------------------------------------------------------
void make_ntt2048_tables(u64 psi, u64* tw) {
  make_ntt_tables(gl_mul(psi, psi), tw);  // the halves' 1024-point transforms use psi^2
  for (int h = 0; h < 2; h++)
    for (int p = 0; p < 8; p++)
      for (int L = 0; L < 64; L++) {
        const int j = ntt_natural_index(L, 8 * h + p);
        const u64 w = gl_pow(psi, (u64)(2 * j + 1));
        tw[TWC_FWD + (8 * h + p) * 64 + L] = w;
        tw[TWC_INV + (8 * h + p) * 64 + L] = gl_pow(w, GL_P - 2);
      }
}

size_t ntt2048_tables_len() { return TW2K_U64; }

hipError_t launch_bsk_to_ntt_2048(const u64* bsk_std, u64* bsk_ntt, size_t polys, const u64* tw, u64 ninv,
                                  hipStream_t s) {
  if (polys == 0) return hipSuccess;
  hipLaunchKernelGGL(bsk_to_ntt2048_kernel, dim3((unsigned)polys), dim3(128), 0, s, bsk_std, bsk_ntt, tw, ninv);
  return hipGetLastError();
}

hipError_t launch_blind_rotate_2048(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index,
                                   int n_lut, const u64* bsk, const u64* tw, u64* out_big, u64* out_acc,
                                   hipStream_t s, size_t latency_max_batch) {
  if (B == 0) return hipSuccess;
  if (B <= latency_max_batch) {
    dim3 grid((unsigned)B), block(512);
    if (out_acc && out_big)
      hipLaunchKernelGGL((blind_rotate2048_lat_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bsk, tw, out_big, out_acc);
    else if (out_acc)
      hipLaunchKernelGGL((blind_rotate2048_lat_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts,
                         lut_index, n_lut, bsk, tw, out_big, out_acc);
    else
      hipLaunchKernelGGL((blind_rotate2048_lat_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts,
                         lut_index, n_lut, bsk, tw, out_big, out_acc);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((B + B2_CTS - 1) / B2_CTS)), block(B2_THREADS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate2048_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                       bsk, tw, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate2048_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bsk, tw, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate2048_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                       n_lut, bsk, tw, out_big, out_acc);
  return hipGetLastError();
}

hipError_t launch_sample_extract_2048(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (N2K + 1);
  hipLaunchKernelGGL(sample_extract2048_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc, B, out);
  return hipGetLastError();
}

hipError_t launch_ntt2048_fwd(u64* polys, size_t count, const u64* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt2048_fwd_kernel, dim3((unsigned)count), dim3(128), 0, s, polys, tw);
  return hipGetLastError();
}

hipError_t launch_ntt2048_inv(u64* polys, size_t count, const u64* tw, u64 ninv, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt2048_inv_kernel, dim3((unsigned)count), dim3(128), 0, s, polys, tw, ninv);
  return hipGetLastError();
}

}  // namespace tfhe
