// pbs_kernels.hip — gfx950 kernels of the PBS hot path (P-GATE: n=630, k=1, N=1024, 7x3, KS 2x8).
//
//   bsk_to_ntt      standard-domain BSK -> device NTT layout (x N^-1), once per key load
//   blind_rotate    the CMUX loop: one wavefront owns one ciphertext for all n iterations;
//                   decompose -> 32x32 NTT (in registers + one LDS transpose) -> GGSW MAC with the
//                   BSK row streamed from L2/HBM -> inverse NTT -> accumulate; sample extract and the
//                   Z_p -> 2^64 switch are fused into the epilogue
//   keyswitch       batched LWE keyswitch kN -> n (64 ciphertexts x 64 columns per workgroup)
//   ntt_fwd/inv     natural-order NTT over the same device routines (parity tests of the NTT)
//   sample_extract  stage-level entry point (the fused epilogue's twin)
//
// Register layout ("R16"): one wavefront processes one polynomial at a time; lane L holds the 16
// coefficients {64*e + L : e < 16}.  In the NTT domain lane L = 32*s + m, element e holds
// A^[brv5(m) + 32*brv5(2e + s)].  A ciphertext's accumulator (2 polys), the two external-product
// outputs (2 polys), one working polynomial and its packed digits all stay in VGPRs (~210/lane,
// 2 waves per SIMD); LDS holds only the 8.4 KB transpose / rotation scratch of each wavefront.
#include <hip/hip_runtime.h>

#include "gl64.h"
#include "ntt32.h"
#include "pbs_kernels.h"

namespace tfhe {

constexpr int N1K = 1024;
constexpr int TSTRIDE = 33;            // LDS row stride (u64) of the 32x32 transpose: conflict-free
constexpr int T_LDS = 32 * TSTRIDE;    // u64 of LDS scratch per wavefront (>= 1024 natural layout)

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

// Cross-lane pair exchange with v_permlane32_swap: with both operands = v, every lane receives
// (u, w) = (value of lane L & 31, value of lane (L & 31) + 32) — the two inputs of the pair's
// butterfly — with no selects and no LDS round trip (ds_bpermute).
__device__ __forceinline__ void pair_values(u64 v, u64& lo, u64& hi) {
  const u32 v0 = (u32)v, v1 = (u32)(v >> 32);
  const auto r0 = __builtin_amdgcn_permlane32_swap(v0, v0, false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(v1, v1, false, false);
  lo = (u64)r0[0] | ((u64)r1[0] << 32);
  hi = (u64)r0[1] | ((u64)r1[1] << 32);
}

// span-1 stage of the 32-point transform: positions (2e, 2e+1) live on lanes (L, L^32).
// Lane half 0 keeps u + t, half 1 keeps u - t, t = zeta * v: computed as u + (+-t).
template <int KIND>
__device__ __forceinline__ void fwd_cross(u64 (&x)[16], bool hi) {
#pragma unroll
  for (int e = 0; e < 16; e++) {
    u64 u, v;
    pair_values(x[e], u, v);
    const u64 t = gl_mul_pow2(v, zeta_exp<KIND>(16 + e));
    x[e] = gl_add(u, hi ? gl_neg(t) : t);
  }
}

template <int KIND>
__device__ __forceinline__ void inv_cross(u64 (&x)[16], bool hi) {
#pragma unroll
  for (int e = 0; e < 16; e++) {
    u64 U, V;
    pair_values(x[e], U, V);
    x[e] = hi ? gl_mul_pow2(gl_sub(U, V), 192 - zeta_exp<KIND>(16 + e)) : gl_add(U, V);
  }
}

// Forward negacyclic NTT of the wavefront's polynomial: natural layout in, NTT layout out.
__device__ __forceinline__ void ntt1024_fwd(u64 (&x)[16], u64* T, int lane, const u64* twf) {
  asm volatile("" : "+s"(twf));  // keep the twiddle loads inside the CMUX loop (no LICM: saves 32 VGPRs)
  const bool hi = lane >= 32;
  const int c = lane & 31, s = lane >> 5;
  fwd_inlane16<NEGA>(x);
  fwd_cross<NEGA>(x, hi);
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], twf[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 16; e++) T[(2 * e + s) * TSTRIDE + c] = x[e];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[c * TSTRIDE + 2 * e + s];
  __syncthreads();
  fwd_inlane16<CYC>(x);
  fwd_cross<CYC>(x, hi);
}

// Inverse (x 1024; the 1/N is folded into the BSK): NTT layout in, natural layout out.
__device__ __forceinline__ void ntt1024_inv(u64 (&x)[16], u64* T, int lane, const u64* twi) {
  asm volatile("" : "+s"(twi));  // keep the twiddle loads inside the CMUX loop (no LICM: saves 32 VGPRs)
  const bool hi = lane >= 32;
  const int c = lane & 31, s = lane >> 5;
  inv_cross<CYC>(x, hi);
  inv_inlane16<CYC>(x);
#pragma unroll
  for (int e = 0; e < 16; e++) T[c * TSTRIDE + 2 * e + s] = x[e];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[(2 * e + s) * TSTRIDE + c];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], twi[64 * e + lane]);
  inv_cross<NEGA>(x, hi);
  inv_inlane16<NEGA>(x);
}

// ------------------------------------------------------------------------------------------
// BSK conversion: one wavefront per polynomial (i, r, j); device layout [i][r][j][e][L] — the same
// polynomial order as the standard layout, each polynomial in NTT layout, scaled by N^-1.
__global__ __launch_bounds__(64) void bsk_to_ntt_kernel(const u64* __restrict__ bsk_std, u64* __restrict__ bsk_ntt,
                                                        const u64* __restrict__ twf, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  const size_t q = blockIdx.x;
  const u64* src = bsk_std + q * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = src[64 * e + lane];
  ntt1024_fwd(x, T, lane, twf);
  u64* dst = bsk_ntt + q * N1K;
#pragma unroll
  for (int e = 0; e < 16; e++) dst[64 * e + lane] = gl_mul(x[e], ninv);
}

// ------------------------------------------------------------------------------------------
// Blind rotation + sample extraction.
//
// A workgroup = BR_WAVES wavefronts = BR_WAVES ciphertexts that walk the CMUX loop in lockstep.
// The external product consumes the BSK in 6 "level steps" per CMUX (row r = c*3 + l, both
// columns j: 16 KB contiguous in the device layout).  Each step's chunk is streamed ONCE per
// workgroup into LDS with global_load_lds (16 B/lane, lane-linear image), double-buffered: chunk
// g+1 is in flight while step g computes, so the MAC reads BSK from LDS instead of waiting on L2 /
// MALL latency with only 2 waves per SIMD (ablation: the register-streamed MAC took 1/3 of the
// kernel).  Twiddles are LDS-resident too.  Per wavefront LDS: the 8.4 KB transpose/rotation
// scratch.  Total 114 KB -> one workgroup (8 waves, 2 per SIMD) per CU.
constexpr int BR_WAVES = 8;
constexpr int BR_THREADS = 64 * BR_WAVES;
constexpr int CHUNK_U64 = 2 * N1K;                 // one level step: rows (c,l), j = 0,1
constexpr int CHUNK_GLDS = CHUNK_U64 * 8 / 1024;   // 1 KB wave-instructions per chunk (16)

struct BrShared {
  u64 T[BR_WAVES][T_LDS];        // per-wave transpose / rotation scratch
  u64 K[2][CHUNK_U64];           // double-buffered BSK chunk
  u64 tw[2][N1K];                // forward / inverse twiddles
};

// ordering of one wavefront's own LDS writes before its reads (LDS executes a wave's ops in order;
// this only stops the compiler from moving them and waits for the writes to retire)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

__device__ __forceinline__ void ntt1024_fwd_digits_lds(const u32 (&dig)[16], int l, u64 (&x)[16], u64* T, int lane,
                                                       const u64* tw) {
  const bool hi = lane >= 32;
  const int c = lane & 31, s = lane >> 5;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const long long u = (long long)((dig[e] >> (8 * l)) & 0xFFu) - 64;
    const long long w = ((long long)((dig[e + 8] >> (8 * l)) & 0xFFu) - 64) * (1ll << 48);
    const long long a = u + w, b = u - w;
    x[e] = (u64)a + (a < 0 ? GL_P : 0ull);
    x[e + 8] = (u64)b + (b < 0 ? GL_P : 0ull);
  }
  fwd_inlane16_from<NEGA, 8>(x);
  fwd_cross<NEGA>(x, hi);
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], tw[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 16; e++) T[(2 * e + s) * TSTRIDE + c] = x[e];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[c * TSTRIDE + 2 * e + s];
  wave_lds_sync();
  fwd_inlane16<CYC>(x);
  fwd_cross<CYC>(x, hi);
}

__device__ __forceinline__ void ntt1024_inv_lds(u64 (&x)[16], u64* T, int lane, const u64* tw) {
  const bool hi = lane >= 32;
  const int c = lane & 31, s = lane >> 5;
  inv_cross<CYC>(x, hi);
  inv_inlane16<CYC>(x);
#pragma unroll
  for (int e = 0; e < 16; e++) T[c * TSTRIDE + 2 * e + s] = x[e];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[(2 * e + s) * TSTRIDE + c];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], tw[64 * e + lane]);
  inv_cross<NEGA>(x, hi);
  inv_inlane16<NEGA>(x);
}

// One component c of the external product for CMUX i: decompose (X^a - 1) * acc_c, then for each
// level l (global step g = 6i + 3c + l) accumulate NTT(digits) (.) BSK_i[(c, l)][j] into out_j.
__device__ __forceinline__ void ext_prod_component_wg(const u64 (&acc)[16], int a, int c, int i, int n_steps,
                                                      BrShared& sh, u64* T, int wave, int lane,
                                                      const u64* __restrict__ bsk, u64 (&out0)[16],
                                                      u64 (&out1)[16]) {
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
    // chunk g has landed (every wave drained its glds: __syncthreads waits vmcnt(0)) and every wave
    // is done reading buffer (g+1)&1 (step g-1): refill it with chunk g+1
    __syncthreads();
    if (g + 1 < n_steps) load_chunk(bsk, g + 1, sh.K[(g + 1) & 1], wave, lane);
    u64 x[16];
    ntt1024_fwd_digits_lds(dig, l, x, T, lane, sh.tw[0]);
    const u64* k0 = sh.K[g & 1] + lane;
    const u64* k1 = sh.K[g & 1] + N1K + lane;
#pragma unroll
    for (int e = 0; e < 16; e++) {
      out0[e] = gl_add(out0[e], gl_mul(x[e], k0[64 * e]));
      out1[e] = gl_add(out1[e], gl_mul(x[e], k1[64 * e]));
    }
  }
}

template <bool WRITE_ACC, bool WRITE_BIG>
__global__ __launch_bounds__(BR_THREADS, 1) void blind_rotate_kernel(
    const u64* __restrict__ lwe_in, int n, size_t B, const u64* __restrict__ luts, const u32* __restrict__ lut_index,
    int n_lut, const u64* __restrict__ bsk, const u64* __restrict__ twf, const u64* __restrict__ twi,
    u64* __restrict__ out_big, u64* __restrict__ out_acc) {
  __shared__ __attribute__((aligned(16))) BrShared sh;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t b_raw = (size_t)blockIdx.x * BR_WAVES + wave;
  const bool live = b_raw < B;
  const size_t b = live ? b_raw : B - 1;  // padding waves run a copy of the last ciphertext, store nothing
  const u64* ct = lwe_in + b * (size_t)(n + 1);
  u64* T = sh.T[wave];
  const int n_steps = n * 6;

  for (int q = threadIdx.x; q < N1K; q += BR_THREADS) {
    sh.tw[0][q] = twf[q];
    sh.tw[1][q] = twi[q];
  }
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
    ext_prod_component_wg(accA, a, 0, i, n_steps, sh, T, wave, lane, bsk, out0, out1);
    ext_prod_component_wg(accB, a, 1, i, n_steps, sh, T, wave, lane, bsk, out0, out1);
    ntt1024_inv_lds(out0, T, lane, sh.tw[1]);
#pragma unroll
    for (int e = 0; e < 16; e++) accA[e] = gl_add(accA[e], out0[e]);
    ntt1024_inv_lds(out1, T, lane, sh.tw[1]);
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

// ------------------------------------------------------------------------------------------
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

// ------------------------------------------------------------------------------------------
// Keyswitch kN -> n, base 2^2 x 8 levels (tfhe-rs SignedDecomposer digits in {-2..2}).
// Workgroup = 64 output columns x 64 ciphertexts; wave w owns ciphertexts 16w..16w+15 of the tile.
constexpr int KS_LEVELS = 8;
constexpr int KS_TILE_CT = 64;
constexpr int KS_JCHUNK = 32;

__device__ __forceinline__ unsigned long long ks_digits_2x8(u64 x) {
  // closest representable at 16 bits, then balanced base-4 digits; byte r = level r (0 = MSB)
  u32 state = (u32)(((x >> 47) + 1) >> 1) & 0xFFFFu;
  unsigned long long packed = 0;
#pragma unroll
  for (int l = KS_LEVELS - 1; l >= 0; l--) {
    const u32 res = state & 3u;
    state >>= 2;
    const u32 carry = ((((res - 1u) | state) & res) >> 1) & 1u;
    state += carry;
    const int d = (int)res - (int)(carry << 2);
    packed |= (unsigned long long)(unsigned char)(signed char)d << (8 * l);
  }
  return packed;
}

__global__ __launch_bounds__(256) void keyswitch_kernel(const u64* __restrict__ in_big, int big_dim, int B,
                                                        const u64* __restrict__ ksk, int n, u64* __restrict__ out) {
  __shared__ unsigned long long dig[KS_TILE_CT][KS_JCHUNK];  // 16 KB: 8 signed byte digits per (ct, j)
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
      dig[c][jj] = ks_digits_2x8(v);
    }
    __syncthreads();
    if (col <= n) {
      for (int jj = 0; jj < KS_JCHUNK; jj++) {
        u64 kv[KS_LEVELS];
#pragma unroll
        for (int r = 0; r < KS_LEVELS; r++) kv[r] = ksk[((size_t)(j0 + jj) * KS_LEVELS + r) * (n + 1) + col];
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const unsigned long long dd = dig[w * 16 + q][jj];
#pragma unroll
          for (int r = 0; r < KS_LEVELS; r++) {
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

// ------------------------------------------------------------------------------------------
// Natural-order NTT over the device routines (one block = one polynomial).
__global__ __launch_bounds__(64) void ntt_fwd_kernel(u64* __restrict__ polys, const u64* __restrict__ twf) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  u64* p = polys + (size_t)blockIdx.x * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = p[64 * e + lane];
  ntt1024_fwd(x, T, lane, twf);
#pragma unroll
  for (int e = 0; e < 16; e++) p[brv5(lane & 31) + 32 * brv5(2 * e + (lane >> 5))] = x[e];
}

__global__ __launch_bounds__(64) void ntt_inv_kernel(u64* __restrict__ polys, const u64* __restrict__ twi, u64 ninv) {
  __shared__ __attribute__((aligned(16))) u64 T[T_LDS];
  const int lane = threadIdx.x;
  u64* p = polys + (size_t)blockIdx.x * N1K;
  u64 x[16];
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = p[brv5(lane & 31) + 32 * brv5(2 * e + (lane >> 5))];
  __syncthreads();
  ntt1024_inv(x, T, lane, twi);
#pragma unroll
  for (int e = 0; e < 16; e++) p[64 * e + lane] = gl_mul(x[e], ninv);
}

// ------------------------------------------------------------------------------------------
// launchers
hipError_t launch_bsk_to_ntt(const u64* bsk_std, u64* bsk_ntt, int n, const u64* twf, u64 ninv, hipStream_t s) {
  hipLaunchKernelGGL(bsk_to_ntt_kernel, dim3((unsigned)n * 12), dim3(64), 0, s, bsk_std, bsk_ntt, twf, ninv);
  return hipGetLastError();
}

hipError_t launch_blind_rotate(const u64* lwe_in, size_t B, int n, const u64* luts, const u32* lut_index, int n_lut,
                               const u64* bsk, const u64* twf, const u64* twi, u64* out_big, u64* out_acc,
                               hipStream_t s) {
  if (B == 0) return hipSuccess;
  dim3 grid((unsigned)((B + BR_WAVES - 1) / BR_WAVES)), block(BR_THREADS);
  if (out_acc && out_big)
    hipLaunchKernelGGL((blind_rotate_kernel<true, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut, bsk,
                       twf, twi, out_big, out_acc);
  else if (out_acc)
    hipLaunchKernelGGL((blind_rotate_kernel<true, false>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                       bsk, twf, twi, out_big, out_acc);
  else
    hipLaunchKernelGGL((blind_rotate_kernel<false, true>), grid, block, 0, s, lwe_in, n, B, luts, lut_index, n_lut,
                       bsk, twf, twi, out_big, out_acc);
  return hipGetLastError();
}

hipError_t launch_sample_extract(const u64* acc, size_t B, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const size_t total = B * (N1K + 1);
  hipLaunchKernelGGL(sample_extract_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, acc, B, out);
  return hipGetLastError();
}

hipError_t launch_keyswitch(const u64* in_big, size_t B, int big_dim, const u64* ksk, int n, u64* out, hipStream_t s) {
  if (B == 0) return hipSuccess;
  dim3 grid((unsigned)((n + 1 + 63) / 64), (unsigned)((B + KS_TILE_CT - 1) / KS_TILE_CT));
  hipLaunchKernelGGL(keyswitch_kernel, grid, dim3(256), 0, s, in_big, big_dim, (int)B, ksk, n, out);
  return hipGetLastError();
}

hipError_t launch_ntt_fwd(u64* polys, size_t count, const u64* twf, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt_fwd_kernel, dim3((unsigned)count), dim3(64), 0, s, polys, twf);
  return hipGetLastError();
}

hipError_t launch_ntt_inv(u64* polys, size_t count, const u64* twi, u64 ninv, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(ntt_inv_kernel, dim3((unsigned)count), dim3(64), 0, s, polys, twi, ninv);
  return hipGetLastError();
}

}  // namespace tfhe
