// ntt1024.h — the wavefront-level 1024-point negacyclic NTT shared by the N = 1024 (P-GATE) and
// N = 2048 (P-FHEVM, two 1024-point halves per polynomial) kernels.  Factorization and layout:
// ntt16.h and DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>

#include "gl64.h"
#include "ntt16.h"

namespace tfhe {

constexpr int N1K = 1024;
constexpr int T1_STRIDE = 68;              // transpose-1 row stride (u64): conflict-free reads/writes
constexpr int T_LDS = 16 * T1_STRIDE;      // u64 of LDS scratch per wavefront (>= 1024)
constexpr int TW_U64 = 4 * N1K;            // twiddle tables: tw1 fwd, tw2 fwd, tw1 inv, tw2 inv

// Ordering of one wavefront's own LDS writes before its reads of another lane's data (LDS runs a
// wave's operations in order; this stops the compiler moving them and retires the writes).
// Barrier that also publishes LDS written by global_load_lds (LDS DMA): the DMA completes on the
// VECTOR memory counter, which the compiler does not wait for before s_barrier on its own (it
// does not model the LDS write), so every wave drains vmcnt(0) first — otherwise a wave can read a
// BSK chunk slice another wave's DMA has not finished writing.
__device__ __forceinline__ void glds_barrier() {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------------
// 1024-point negacyclic NTT of the wavefront's polynomial (ntt16.h for the factorization).
// tw points at the 4 tables [tw1 fwd | tw2 fwd | tw1 inv | tw2 inv] (LDS or global).
// Transpose 1: lane L, slot e -> T[e][L] (stride 68) -> lane (e1 = L >> 2, i3 = L & 3) reads
//              T[e1][4 e2 + i3].  Transpose 2: lane L2, slot f -> T[f][L2 ^ (f >> 2 & 3)]
//              (XOR swizzle) -> lane (e1, fhi = L & 3) reads element 4 flo + i3 from
//              T[4 fhi + flo][(4 e1 + i3) ^ fhi].  Both are bank-conflict free.
__device__ __forceinline__ void ntt1024_fwd_tail(u64 (&x)[16], u64* T, int lane, const u64* tw) {
  const int e1 = lane >> 2, q = lane & 3;
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], tw[64 * e + lane]);
#pragma unroll
  for (int e = 0; e < 16; e++) T[e * T1_STRIDE + lane] = x[e];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[e1 * T1_STRIDE + 4 * e + q];
  wave_lds_sync();
  cyc16_fwd(x);
#pragma unroll
  for (int f = 1; f < 16; f++) x[f] = gl_mul(x[f], tw[N1K + 64 * f + lane]);  // tw2 column f = 0 is 1
#pragma unroll
  for (int f = 0; f < 16; f++) T[f * 64 + (lane ^ ((f >> 2) & 3))] = x[f];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[(4 * q + (e >> 2)) * 64 + ((4 * e1 + (e & 3)) ^ q)];
  wave_lds_sync();
  cyc4x4_fwd(x);
}

__device__ __forceinline__ void ntt1024_fwd(u64 (&x)[16], u64* T, int lane, const u64* tw) {
  nega16_fwd(x);
  ntt1024_fwd_tail(x, T, lane, tw);
}

// Inverse, x 1024 (the 1/N is folded into the BSK): NTT layout in, natural layout out.
__device__ __forceinline__ void ntt1024_inv(u64 (&x)[16], u64* T, int lane, const u64* tw) {
  const int e1 = lane >> 2, q = lane & 3;
  cyc4x4_inv(x);
#pragma unroll
  for (int e = 0; e < 16; e++) T[(4 * q + (e >> 2)) * 64 + ((4 * e1 + (e & 3)) ^ q)] = x[e];
  wave_lds_sync();
#pragma unroll
  for (int f = 0; f < 16; f++) x[f] = T[f * 64 + (lane ^ ((f >> 2) & 3))];
  wave_lds_sync();
#pragma unroll
  for (int f = 1; f < 16; f++) x[f] = gl_mul(x[f], tw[3 * N1K + 64 * f + lane]);  // f = 0 is 1
  cyc16_inv(x);
#pragma unroll
  for (int e = 0; e < 16; e++) T[e1 * T1_STRIDE + 4 * e + q] = x[e];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = T[e * T1_STRIDE + lane];
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < 16; e++) x[e] = gl_mul(x[e], tw[2 * N1K + 64 * e + lane]);
  nega16_inv(x);
}

}  // namespace tfhe
