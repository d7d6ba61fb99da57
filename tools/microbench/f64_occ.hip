// f64 VALU throughput on gfx950 as a function of waves per SIMD and independent chains per wave:
// is ~6 cycles per wave64 v_fma_f64 (f64_rates.hip, 2 waves / SIMD) an issue limit or a latency limit?
// Every lane runs C independent fma chains (no instruction reads a result of the previous C - 1);
// v_add_u32 and v_pk_fma_f32 at the same shape calibrate the clock.  s_memtime brackets each wave's
// loop too (cycles of the 100 MHz-invariant counter are not used: the figure is wall time at 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void k_fma(double* out, int iters) {
  double a[C];
#pragma unroll
  for (int c = 0; c < C; c++) a[c] = threadIdx.x * (1.0 + c);
  const double m = 1.0000001, s = 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 32 / C; r++)
#pragma unroll
      for (int c = 0; c < C; c++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(m), "v"(s));
  }
  double t = 0;
#pragma unroll
  for (int c = 0; c < C; c++) t += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int C>
__global__ void k_add_u32(double* out, int iters) {
  unsigned a[C];
#pragma unroll
  for (int c = 0; c < C; c++) a[c] = threadIdx.x * (1 + c);
  const unsigned m = 12345;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 32 / C; r++)
#pragma unroll
      for (int c = 0; c < C; c++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(m));
  }
  unsigned t = 0;
#pragma unroll
  for (int c = 0; c < C; c++) t += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int C>
__global__ void k_add_f64(double* out, int iters) {
  double a[C];
#pragma unroll
  for (int c = 0; c < C; c++) a[c] = threadIdx.x * (1.0 + c);
  const double m = 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 32 / C; r++)
#pragma unroll
      for (int c = 0; c < C; c++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[c]) : "v"(m));
  }
  double t = 0;
#pragma unroll
  for (int c = 0; c < C; c++) t += a[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

typedef void (*kfn)(double*, int);
static void run(const char* name, int chains, kfn k, int waves_per_simd) {
  const int threads = 256;  // 4 waves per workgroup = 1 per SIMD
  const int blocks = 256 * waves_per_simd, iters = 20000;
  double* d;
  hipMalloc(&d, (size_t)blocks * threads * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 10);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double waves = blocks * threads / 64.0, instr = waves * iters * 32.0;
  const double cyc = (ms * 1e-3 * 2.4e9) / (instr / 1024.0);
  printf("%-10s chains %2d  waves/SIMD %d  %8.3f ms  %.2f cycles / wave-instr / SIMD (2.4 GHz)\n", name, chains,
         waves_per_simd, ms, cyc);
  hipFree(d);
}

#define RUNALL(NAME, K)                                    \
  for (int w : {1, 2, 4, 8}) {                             \
    run(NAME, 1, K<1>, w);                                 \
    run(NAME, 2, K<2>, w);                                 \
    run(NAME, 4, K<4>, w);                                 \
    run(NAME, 8, K<8>, w);                                 \
    run(NAME, 16, K<16>, w);                               \
  }

int main() {
  RUNALL("add_u32", k_add_u32)
  RUNALL("fma_f64", k_fma)
  RUNALL("add_f64", k_add_f64)
  return 0;
}
