// Microbenchmark: Goldilocks (2^64-2^32+1) mulmod throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned long long u64;
#define P 0xFFFFFFFF00000001ull

__device__ __forceinline__ u64 reduce128(u64 hi, u64 lo) {
  u64 hh = hi >> 32, hl = hi & 0xFFFFFFFFull;
  u64 t0 = lo - hh; if (lo < hh) t0 -= 0xFFFFFFFFull;
  u64 t1 = (hl << 32) - hl;
  u64 t2 = t0 + t1; if (t2 < t1) t2 += 0xFFFFFFFFull;
  return t2;
}
__device__ __forceinline__ u64 mulmod(u64 a, u64 b) {
  return reduce128(__umul64hi(a, b), a * b);
}
// 32x32->64 via mad_u64_u32 style
__device__ __forceinline__ u64 mul32(unsigned a, unsigned b) { return (u64)a * (u64)b; }
__device__ __forceinline__ u64 mulmod_split(u64 a, u64 b) {
  unsigned a0 = (unsigned)a, a1 = a >> 32, b0 = (unsigned)b, b1 = b >> 32;
  u64 ll = mul32(a0, b0), lh = mul32(a0, b1), hl = mul32(a1, b0), hh = mul32(a1, b1);
  u64 mid = lh + hl; u64 midc = (mid < lh) ? (1ull << 32) : 0;
  u64 lo = ll + (mid << 32); u64 c = lo < ll;
  u64 hi = hh + (mid >> 32) + midc + c;
  return reduce128(hi, lo);
}
__device__ __forceinline__ u64 shiftmul(u64 a, int s) { // s in [1,63]
  return reduce128(a >> (64 - s), a << s);
}

template <int MODE>
__global__ void k(u64* out, u64 seed, int iters) {
  u64 x[8];
  for (int i = 0; i < 8; i++) x[i] = seed * (threadIdx.x + 1 + i * 977) + blockIdx.x;
  u64 w = seed | 12345;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (MODE == 0) x[i] = mulmod(x[i], w);
      else if (MODE == 1) x[i] = mulmod_split(x[i], w);
      else if (MODE == 2) x[i] = shiftmul(x[i], 3 + i * 5);
      else if (MODE == 3) { unsigned lo = (unsigned)x[i], hi = x[i] >> 32; lo = lo * (unsigned)w; hi = hi * (unsigned)w + 7; x[i] = ((u64)hi << 32) | lo; }
      else if (MODE == 4) { unsigned lo = (unsigned)x[i], hi = x[i] >> 32; lo = __umulhi(lo, (unsigned)w); hi = __umulhi(hi, (unsigned)w) + 7; x[i] = ((u64)hi << 32) | lo; }
      else if (MODE == 5) { unsigned lo = (unsigned)x[i], hi = x[i] >> 32; lo = lo + (unsigned)w; hi = hi ^ lo; x[i] = ((u64)hi << 32) | lo; }
    }
  }
  u64 s = 0;
  for (int i = 0; i < 8; i++) s ^= x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(const char* name, double ops_per_inner) {
  int blocks = 256 * 8, threads = 256, iters = 4096;
  u64* d; hipMalloc(&d, (size_t)blocks * threads * 8);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 3ull, 16);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 3ull, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double n = (double)blocks * threads * iters * 8;
  printf("%-14s %8.3f ms  %8.2f G op/s  (%.2f G lane-instr/s at %.0f instr/op)\n", name, ms, n / ms / 1e6,
         n * ops_per_inner / ms / 1e6, ops_per_inner);
  hipFree(d);
}

int main() {
  run<0>("mulmod_u64", 1);
  run<1>("mulmod_split", 1);
  run<2>("shiftmul", 1);
  run<3>("mul_lo_u32x2", 2);
  run<4>("mul_hi_u32x2", 2);
  run<5>("add_xor", 2);
  return 0;
}
