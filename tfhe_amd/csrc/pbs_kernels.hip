// pbs_kernels.hip — gfx950 kernels of the PBS hot path (P-GATE: n=630, k=1, N=1024, 7x3, KS 2x8).
//
//   bsk_to_ntt      standard-domain BSK -> device NTT layout (x N^-1), once per key load
//   blind_rotate    the CMUX loop: 8 wavefronts (8 ciphertexts) per workgroup walk the loop in
//                   lockstep; per CMUX: decompose -> NTT (in registers, 2 LDS transposes) ->
//                   GGSW MAC with the BSK chunk streamed once per workgroup into LDS -> inverse
//                   NTT -> accumulate; sample extract + Z_p -> 2^64 fused in the epilogue
//   keyswitch       batched LWE keyswitch kN -> n (64 ciphertexts x 64 columns per workgroup)
//   ntt_fwd/inv     natural-order NTT over the same device routines (parity tests of the NTT)
//   sample_extract  stage-level entry point (the fused epilogue's twin)
//
// Register layout: one wavefront processes one polynomial at a time, 16 u64 per lane.
//   natural (coefficient) layout: lane L, element e  <->  coefficient 64 e + L
//   NTT layout (after ntt1024_fwd): lane L, element e <-> A^[ntt_natural_index(L, e)]
// A ciphertext's accumulator (2 polys), the two external-product outputs (2 polys), one working
// polynomial and its packed digits stay in VGPRs (256/lane, 2 waves per SIMD).
#include <hip/hip_runtime.h>

#include "gl64.h"
#include "ntt1024.h"
#include "ntt16.h"
#include "pbs_kernels.h"

namespace tfhe {

// round(x * 2048 / 2^64) mod 2048  (modulus switch)
__device__ __forceinline__ int ms2048(u64 x) { return (int)((((x >> 52) + 1) >> 1) & 2047u); }

// (X^s * v)[idx] for a negacyclic length-1024 polynomial v, s in [0, 2048).
__device__ __forceinline__ u64 rot_read(const u64* v, int idx, int s) {
  int d = idx - s;
  bool neg = false;
  if (d < 0) { d += N1K; neg = !neg; }
  if (d < 0) { d += N1K; neg = !neg; }
  const u64 x = v[d];
  return neg ? gl_neg(x) : x;
}

// tfhe-rs SignedDecomposer, base 2^7 x 3 levels, on the Z_p residue read as a 64-bit word.
// Returns the 3 digits packed as bytes (d + 64), byte l = level l (0 = most significant).
__device__ __forceinline__ u32 decomp_7x3(u64 x) {
  u32 state = (u32)(((x >> 42) + 1) >> 1) & 0x1FFFFFu;
  u32 packed = 0;
#pragma unroll
  for (int l = 2; l >= 0; l--) {
    const u32 res = state & 127u;
    state >>= 7;
    const u32 carry = ((((res - 1u) | state) & res) >> 6) & 1u;
    state += carry;
    const int d = (int)res - (int)(carry << 7);
    packed |= (u32)(d + 64) << (8 * l);
  }
  return packed;
}

// Forward NTT of a digit polynomial (|d| <= 64, byte l of dig[e] holds d + 64): the first
// pass-1 stage (span 8, twiddle 2^48) is exact in int64 (|d + 2^48 d'| < 2^55): no reduction.
__device__ __forceinline__ void ntt1024_fwd_digits(const u32 (&dig)[16], int l, u64 (&x)[16], u64* T, int lane,
                                                   const u64* tw) {
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const long long u = (long long)((dig[e] >> (8 * l)) & 0xFFu) - 64;
    const long long w = ((long long)((dig[e + 8] >> (8 * l)) & 0xFFu) - 64) * (1ll << 48);
    const long long a = u + w, b = u - w;
    x[e] = (u64)a + (a < 0 ? GL_P : 0ull);
    x[e + 8] = (u64)b + (b < 0 ? GL_P : 0ull);
  }
  nega16_fwd_from4(x);
  ntt1024_fwd_tail(x, T, lane, tw);
}

// ---------------------------------------------------------------------------------------------
// BSK conversion: one wavefront per polynomial (i, r, j); device layout [i][r][j][e][L] — the
// standard layout's polynomial order, each polynomial in NTT layout, scaled by N^-1.
__global__ __launch_bounds__(64) void bsk_to_ntt_kernel(const u64* __restrict__ bsk_std, u64* __restrict__ bsk_ntt,
                                                        const u64* __restrict__ tw, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  const size_t q = blockIdx.x;
  const u64* src = bsk_std + q * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = src[64 * e + lane];
  ntt1024_fwd(x, T, lane, tw);
  u64* dst = bsk_ntt + q * N1K;
#pragma unroll
  for (int e = 0; e < 16; e++) dst[64 * e + lane] = gl_mul(x[e], ninv);
}

// ---------------------------------------------------------------------------------------------
// Blind rotation + sample extraction.
//
// A workgroup = BR_WAVES wavefronts = BR_WAVES ciphertexts that walk the CMUX loop in lockstep.
// The external product consumes the BSK in 6 "level steps" per CMUX (row r = c*3 + l, both
// columns j: 16 KB contiguous in the device layout).  Each step's chunk is streamed ONCE per
// workgroup into LDS with global_load_lds (16 B/lane, lane-linear image), double-buffered: chunk
// g+1 is in flight while step g computes, so the MAC reads BSK from LDS instead of waiting on L2 /
// MALL latency with only 2 waves per SIMD.  Twiddles are LDS-resident.  Per wavefront LDS: the
// 8.7 KB transpose/rotation scratch.  Total 134 KB -> one workgroup (8 waves, 2/SIMD) per CU.
constexpr int BR_WAVES = 8;
constexpr int BR_THREADS = 64 * BR_WAVES;
constexpr int CHUNK_U64 = 2 * N1K;                // one level step: rows (c,l), j = 0,1
constexpr int CHUNK_GLDS = CHUNK_U64 * 8 / 1024;  // 1 KB wave-instructions per chunk (16)

struct BrShared {
  u64 T[BR_WAVES][T_LDS];  // per-wave transpose / rotation scratch
  u64 K[2][CHUNK_U64];     // double-buffered BSK chunk
  u64 tw[TW_U64];          // twiddle tables
};

// issue this wave's share of chunk g (2 x 1 KB) into buffer dst
__device__ __forceinline__ void load_chunk(const u64* __restrict__ bsk, int g, u64* dst, int wave, int lane) {
  const char* src = (const char*)(bsk + (size_t)g * CHUNK_U64);
#pragma unroll
  for (int q = 0; q < CHUNK_GLDS / BR_WAVES; q++) {
    const int blk = wave * (CHUNK_GLDS / BR_WAVES) + q;  // which 1 KB piece
    __builtin_amdgcn_global_load_lds((const void*)(src + blk * 1024 + lane * 16),
                                     (__attribute__((address_space(3))) void*)((char*)dst + blk * 1024), 16, 0, 0);
  }
}

// One component c of the external product for CMUX i: decompose (X^a - 1) * acc_c, then for each
// level l (global step g = 6i + 3c + l) accumulate NTT(digits) (.) BSK_i[(c, l)][j] into out_j.
__device__ __forceinline__ void ext_prod_component(const u64 (&acc)[16], int a, int c, int i, int n_steps,
                                                   BrShared& sh, u64* T, int wave, int lane,
                                                   const u64* __restrict__ bsk, u64 (&out0)[16], u64 (&out1)[16]) {
#pragma unroll
  for (int e = 0; e < 16; e++) T[64 * e + lane] = acc[e];
  wave_lds_sync();
  u32 dig[16];
#pragma unroll
  for (int e = 0; e < 16; e++) dig[e] = decomp_7x3(gl_sub(rot_read(T, 64 * e + lane, a), acc[e]));
  wave_lds_sync();
#pragma unroll 1
  for (int l = 0; l < 3; l++) {
    const int g = i * 6 + c * 3 + l;
    // chunk g has landed (every wave drains its own LDS DMA, then the barrier) and every wave is
    // done reading buffer (g+1)&1 (step g-1): refill it with chunk g+1
    glds_barrier();
    if (g + 1 < n_steps) load_chunk(bsk, g + 1, sh.K[(g + 1) & 1], wave, lane);
    u64 x[16];
    ntt1024_fwd_digits(dig, l, x, T, lane, sh.tw);
    const u64* k0 = sh.K[g & 1] + lane;
    const u64* k1 = sh.K[g & 1] + N1K + lane;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      out0[e] = gl_mac_lazy(out0[e], x[e], k0[64 * e]);  // lazily reduced: canonicalized before the
      out1[e] = gl_mac_lazy(out1[e], x[e], k1[64 * e]);  // inverse NTT
    }
  }
}

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(BR_THREADS, 1) void blind_rotate_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const u64* __restrict__ bsk, const u64* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) BrShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b_raw = (size_t)blockIdx.x * BR_WAVES + wave;
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding waves run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  u64* T = sh.T[wave];
  const int n_steps = n * 6;

  for (int q = threadIdx.x; q < TW_U64; q += BR_THREADS) sh.tw[q] = tw_g[q];
  load_chunk(bsk, 0, sh.K[0], wave, lane);

  // acc = (0, X^{-b~} * lut)
  u64 accA[16], accB[16];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N1K;
    const int s = (2048 - ms2048(ct[n])) & 2047;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      accA[e] = 0;
      accB[e] = rot_read(lut, 64 * e + lane, s);
    }
  }

  // No per-ciphertext skip of a~_i == 0 steps: the workgroup walks the loop in lockstep; such a
  // step decomposes 0 and adds exactly 0, so the result is bit-identical.
  for (int i = 0; i < n; i++) {
    const int a = ms2048(ct[i]);
    u64 out0[16], out1[16];
#pragma unroll
    for (int e = 0; e < 16; e++) { out0[e] = 0; out1[e] = 0; }
    ext_prod_component(accA, a, 0, i, n_steps, sh, T, wave, lane, bsk, out0, out1);
    ext_prod_component(accB, a, 1, i, n_steps, sh, T, wave, lane, bsk, out0, out1);
#pragma unroll
    for (int e = 0; e < 16; e++) { out0[e] = gl_canon(out0[e]); out1[e] = gl_canon(out1[e]); }
    ntt1024_inv(out0, T, lane, sh.tw);
#pragma unroll
    for (int e = 0; e < 16; e++) accA[e] = gl_add(accA[e], out0[e]);
    ntt1024_inv(out1, T, lane, sh.tw);
#pragma unroll
    for (int e = 0; e < 16; e++) accB[e] = gl_add(accB[e], out1[e]);
  }

  if (!live) return;
  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      oa[64 * e + lane] = accA[e];
      oa[N1K + 64 * e + lane] = accB[e];
    }
  }
  if (WRITE_BIG) {
    // sample extraction at degree 0 (computations.rs:109-132 semantics): a'_0 = A[0],
    // a'_j = -A[N-j], b' = B[0]; each converted Z_p -> 2^64.
    u64* ob = out_big + b * (size_t)(N1K + 1);
#pragma unroll
    for (int e = 0; e < 16; e++) {
      const int idx = 64 * e + lane;
      if (idx == 0) ob[0] = gl_to_torus(accA[e]);
      else ob[N1K - idx] = gl_to_torus(gl_neg(accA[e]));
    }
    if (lane == 0) ob[N1K] = gl_to_torus(accB[0]);
  }
}

// ---------------------------------------------------------------------------------------------
// Latency-mode blind rotation: ONE ciphertext per workgroup of 8 wavefronts (small batches: the
// integer circuits' lockstep levels, single /evaluate requests).  Per CMUX:
//   A  waves 0..5: wave w = (c, l) rotates + decomposes accumulator polynomial c (LDS), takes
//      digit level l and runs its forward NTT -> F[w]                       (6 NTTs in parallel)
//   B  all 8 waves: pointwise MAC out_j = sum_w F[w] (.) BSK_i[w][j] over a quarter of the slots
//      each (j = wave >> 2), BSK read straight from L2 (each word once per workgroup) -> O[j]
//   C  waves 0, 1: inverse NTT of O[j], acc_j += ..., written back to A[j]   (2 NTTs in parallel)
// Three barriers per CMUX; the critical path is ~2 forward + 1 inverse NTT instead of 6 + 2, so a
// PBS completes ~5x sooner than in the batch kernel (which is faster per PBS once >~1.3k
// ciphertexts fill the GPU: the host picks the kernel by batch size).  LDS: A 16 KB, F 48 KB,
// 6 NTT scratch areas 52 KB (O aliases scratch 2..3, dead after phase A), twiddles 32 KB = 148 KB.
constexpr int LAT_THREADS = 512;

struct LatShared {
  u64 A[2][N1K];
  u64 F[6][N1K];
  u64 T[6][T_LDS];
  u64 tw[TW_U64];
};

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(LAT_THREADS, 1) void blind_rotate_lat_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const u64* __restrict__ bsk, const u64* __restrict__ tw_g, u64* __restrict__ out_big,
    u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) LatShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b = blockIdx.x;
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  u64* O = sh.T[2];  // 2 x 1024 u64 alias of scratch areas 2 and 3

  for (int q = threadIdx.x; q < TW_U64; q += LAT_THREADS) sh.tw[q] = tw_g[q];
  {
    int li = lut_index ? (int)lut_index[b] : 0;
    li = (li < 0 || li >= n_lut) ? 0 : li;
    const u64* lut = luts + (size_t)li * N1K;
    const int s = (2048 - ms2048(ct[n])) & 2047;
    for (int q = threadIdx.x; q < N1K; q += LAT_THREADS) {
      sh.A[0][q] = 0;
      sh.A[1][q] = rot_read(lut, q, s);
    }
  }
  __syncthreads();

  const int j = wave >> 2, e0 = (wave & 3) * 4;  // phase B: output j, slots e0 .. e0 + 3
  for (int i = 0; i < n; i++) {
    const int a = ms2048(ct[i]);
    if (wave < 6) {  // phase A
      const int c = wave / 3, l = wave % 3;
      const u64* acc = sh.A[c];
      u32 dig[16];
#pragma unroll
      for (int e = 0; e < 16; e++) {
        const int idx = 64 * e + lane;
        dig[e] = decomp_7x3(gl_sub(rot_read(acc, idx, a), acc[idx]));
      }
      u64 x[16];
      ntt1024_fwd_digits(dig, l, x, sh.T[wave], lane, sh.tw);
#pragma unroll
      for (int e = 0; e < 16; e++) sh.F[wave][64 * e + lane] = x[e];
    }
    __syncthreads();
    {  // phase B
      const u64* k = bsk + (size_t)i * 12 * N1K + (size_t)j * N1K + lane;
      u64 o[4] = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < 6; r++)
#pragma unroll
        for (int t = 0; t < 4; t++)
          o[t] = gl_mac_lazy(o[t], sh.F[r][64 * (e0 + t) + lane], k[(size_t)r * 2 * N1K + 64 * (e0 + t)]);
#pragma unroll
      for (int t = 0; t < 4; t++) O[j * N1K + 64 * (e0 + t) + lane] = gl_canon(o[t]);
    }
    __syncthreads();
    if (wave < 2) {  // phase C
      u64 x[16];
#pragma unroll
      for (int e = 0; e < 16; e++) x[e] = O[wave * N1K + 64 * e + lane];
      ntt1024_inv(x, sh.T[wave], lane, sh.tw);
#pragma unroll
      for (int e = 0; e < 16; e++) sh.A[wave][64 * e + lane] = gl_add(sh.A[wave][64 * e + lane], x[e]);
    }
    __syncthreads();
  }

  if (WRITE_ACC) {
    u64* oa = out_acc + b * 2048;
    for (int q = threadIdx.x; q < 2 * N1K; q += LAT_THREADS) oa[q] = sh.A[q >> 10][q & (N1K - 1)];
  }
  if (WRITE_BIG) {
    u64* ob = out_big + b * (size_t)(N1K + 1);
    for (int q = threadIdx.x; q <= N1K; q += LAT_THREADS) {
      u64 v;
      if (q == N1K) v = sh.A[1][0];
      else if (q == 0) v = sh.A[0][0];
      else v = gl_neg(sh.A[0][N1K - q]);
      ob[q] = gl_to_torus(v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
__global__ void sample_extract_kernel(const u64* __restrict__ acc, size_t B, u64* __restrict__ out) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= B * (N1K + 1)) return;
  const size_t b = gid / (N1K + 1);
  const int j = (int)(gid % (N1K + 1));
  const u64* A = acc + b * 2048;
  u64 v;
  if (j == N1K) v = A[N1K];
  else if (j == 0) v = A[0];
  else v = gl_neg(A[N1K - j]);
  out[gid] = gl_to_torus(v);
}

// ---------------------------------------------------------------------------------------------
// Keyswitch big -> n (tfhe-rs SignedDecomposer digits): P-GATE base 2^2 x 8 levels (digits in
// {-2..2}), P-FHEVM base 2^4 x 4 (digits in [-8, 8]).  Workgroup = 64 output columns x 64
// ciphertexts; wave w owns ciphertexts 16w..16w+15 of the tile; digits staged in LDS as bytes.
constexpr int KS_TILE_CT = 64;
constexpr int KS_JCHUNK = 32;

// closest representable at BL*LV bits, then balanced base-2^BL digits; byte r = level r (0 = MSB)
template <int BL, int LV>
__device__ __forceinline__ unsigned long long ks_digits(u64 x) {
  constexpr int P = BL * LV;
  u32 state = (u32)(((x >> (63 - P)) + 1) >> 1) & (u32)((1ull << P) - 1);
  unsigned long long packed = 0;
#pragma unroll
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

template <int BL, int LV>
__global__ __launch_bounds__(256) void keyswitch_kernel(const u64* __restrict__ in_big, int big_dim, int B,
                                                        const u64* __restrict__ ksk, int n, u64* __restrict__ out) {
  __shared__ unsigned long long dig[KS_TILE_CT][KS_JCHUNK];  // 16 KB: LV signed byte digits per (ct, j)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int col = blockIdx.x * 64 + lane;
  const int ct0 = blockIdx.y * KS_TILE_CT;
  u64 acc[16];
#pragma unroll
  for (int q = 0; q < 16; q++) acc[q] = 0;
  for (int j0 = 0; j0 < big_dim; j0 += KS_JCHUNK) {
    for (int q = tid; q < KS_TILE_CT * KS_JCHUNK; q += 256) {
      const int c = q / KS_JCHUNK, jj = q % KS_JCHUNK, b = ct0 + c;
      const u64 v = (b < B) ? in_big[(size_t)b * (big_dim + 1) + j0 + jj] : 0ull;
      dig[c][jj] = ks_digits<BL, LV>(v);
    }
    __syncthreads();
    if (col <= n) {
      for (int jj = 0; jj < KS_JCHUNK; jj++) {
        u64 kv[LV];
#pragma unroll
        for (int r = 0; r < LV; r++) kv[r] = ksk[((size_t)(j0 + jj) * LV + r) * (n + 1) + col];
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const unsigned long long dd = dig[w * 16 + q][jj];
#pragma unroll
          for (int r = 0; r < LV; r++) {
            const long long d = (long long)(signed char)(dd >> (8 * r));
            acc[q] -= (u64)d * kv[r];
          }
        }
      }
    }
    __syncthreads();
  }
  if (col <= n) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int b = ct0 + w * 16 + q;
      if (b < B) out[(size_t)b * (n + 1) + col] = acc[q] + (col == n ? in_big[(size_t)b * (big_dim + 1) + big_dim] : 0ull);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Natural-order NTT over the device routines (one block = one polynomial).
__global__ __launch_bounds__(64) void ntt_fwd_kernel(u64* __restrict__ polys, const u64* __restrict__ tw) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  u64* p = polys + (size_t)blockIdx.x * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = p[64 * e + lane];
  ntt1024_fwd(x, T, lane, tw);
#pragma unroll
  for (int e = 0; e < 16; e++) p[ntt_natural_index(lane, e)] = x[e];
}

__global__ __launch_bounds__(64) void ntt_inv_kernel(u64* __restrict__ polys, const u64* __restrict__ tw, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  u64* p = polys + (size_t)blockIdx.x * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = p[ntt_natural_index(lane, e)];
  __syncthreads();
  ntt1024_inv(x, T, lane, tw);
#pragma unroll
  for (int e = 0; e < 16; e++) p[64 * e + lane] = gl_mul(x[e], ninv);
}

// ---------------------------------------------------------------------------------------------
// host-side twiddle tables for the device NTT layout (4 x 1024 u64: tw1 fwd, tw2 fwd, tw1 inv, tw2 inv)
void make_ntt_tables(u64 psi, u64* tw) {
  const u64 psi_inv = gl_pow(psi, GL_P - 2), two_inv = gl_pow(2, GL_P - 2);
  for (int e = 0; e < 16; e++)
    for (int L = 0; L < 64; L++) {
      const u64 e1x = (u64)L * (2 * brv4(e) + 1);  // tw1: psi^(i' (2 j1 + 1)), i' = L, j1 = brv4(e)
      const u64 e2x = (u64)3 * (L & 3) * brv4(e);   // tw2: 2^(3 i3 j2), i3 = L & 3, j2 = brv4(f = e)
      tw[64 * e + L] = gl_pow(psi, e1x);
      tw[N1K + 64 * e + L] = gl_pow(2, e2x);
      tw[2 * N1K + 64 * e + L] = gl_pow(psi_inv, e1x);
      tw[3 * N1K + 64 * e + L] = gl_pow(two_inv, e2x);
    }
}

// launchers
hipError_t launch_bsk_to_ntt(const u64* bsk_std, u64* bsk_ntt, int n, const u64* tw, u64 ninv, hipStream_t s) {
  hipLaunchKernelGGL(bsk_to_ntt_kernel, dim3((unsigned)n * 12), dim3(64), 0, s, bsk_std, bsk_ntt, tw, ninv);
  return hipGetLastError();
}

hipError_t launch_blind_rotate(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index, int n_lut,
                               const u64* bsk, const u64* tw, u64* out_big, u64* out_acc, hipStream_t s,
                               size_t latency_max_batch) {
  if (B == 0) return hipSuccess;
  if (B <= latency_max_batch) {
    dim3 grid((unsigned)B), block(LAT_THREADS);
    if (out_acc && out_big)
      hipLaunchKernelGGL((blind_rotate_lat_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                         bsk, tw, out_big, out_acc);
    else if (out_acc)
      hipLaunchKernelGGL((blind_rotate_lat_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bsk, tw, out_big, out_acc);
    else
      hipLaunchKernelGGL((blind_rotate_lat_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index,
                         n_lut, bsk, tw, out_big, out_acc);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(BR_THREADS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut, bsk,
                       tw, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                       bsk, tw, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                       bsk, tw, out_big, out_acc);
  return hipGetLastError();
}

hipError_t launch_sample_extract(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (N1K + 1);
  hipLaunchKernelGGL(sample_extract_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc, B, out);
  return hipGetLastError();
}

hipError_t launch_keyswitch(const u64* in_big, size_t B, int big_dim, const u64* ksk, int n, int base_log, int levels,
                           u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (big_dim % KS_JCHUNK) return hipErrorInvalidValue;
  dim3 grid((unsigned)((n + 1 + 63) / 64), (unsigned)((B + KS_TILE_CT - 1) / KS_TILE_CT));
  if (base_log == 2 && levels == 8)
    hipLaunchKernelGGL((keyswitch_kernel<2, 8>), grid, dim3(256), 0, s, in_big, big_dim, (int)B, ksk, n, out);
  else if (base_log == 4 && levels == 4)
    hipLaunchKernelGGL((keyswitch_kernel<4, 4>), grid, dim3(256), 0, s, in_big, big_dim, (int)B, ksk, n, out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_ntt_fwd(u64* polys, size_t count, const u64* tw, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt_fwd_kernel, dim3((unsigned)count), dim3(64), 0, s, polys, tw);
  return hipGetLastError();
}

hipError_t launch_ntt_inv(u64* polys, size_t count, const u64* tw, u64 ninv, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt_inv_kernel, dim3((unsigned)count), dim3(64), 0, s, polys, tw, ninv);
  return hipGetLastError();
}

}  // namespace tfhe
