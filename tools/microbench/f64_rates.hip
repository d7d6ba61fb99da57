// Per-instruction f64 VALU throughput on gfx950 (inline asm, 8 independent chains per lane,
// 2 waves/SIMD): the instructions an f64 FFT external product is made of.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define X8(s) s s s s s s s s
#define KERNELF(NAME, ASM)                                                          \
  __global__ void NAME(double* out, int iters) {                                    \
    double a0 = threadIdx.x * 1.5, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19; \
    for (int it = 0; it < iters; it++) { ASM }                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7; \
  }
KERNELF(k_fma_f64, asm volatile(X8("v_fma_f64 %0, %0, %1, %2\n v_fma_f64 %3, %3, %4, %5\n v_fma_f64 %6, %6, %7, %1\n v_fma_f64 %2, %2, %3, %4\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_add_f64, asm volatile(X8("v_add_f64 %0, %0, %1\n v_add_f64 %2, %2, %3\n v_add_f64 %4, %4, %5\n v_add_f64 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_mul_f64, asm volatile(X8("v_mul_f64 %0, %0, %1\n v_mul_f64 %2, %2, %3\n v_mul_f64 %4, %4, %5\n v_mul_f64 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_pk_add_f32_as_f64, asm volatile(X8("v_pk_add_f32 %0, %0, %1\n v_pk_add_f32 %2, %2, %3\n v_pk_add_f32 %4, %4, %5\n v_pk_add_f32 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_rndne_f64, asm volatile(X8("v_rndne_f64 %0, %1\n v_rndne_f64 %2, %3\n v_rndne_f64 %4, %5\n v_rndne_f64 %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_floor_f64, asm volatile(X8("v_floor_f64 %0, %1\n v_floor_f64 %2, %3\n v_floor_f64 %4, %5\n v_floor_f64 %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNELF(k_ldexp_f64, asm volatile(X8("v_ldexp_f64 %0, %1, 3\n v_ldexp_f64 %2, %3, 5\n v_ldexp_f64 %4, %5, 7\n v_ldexp_f64 %6, %7, 9\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)

__global__ void k_cvt_f64_i32(double* out, int iters) {
  double a0 = 0, a2 = 0, a4 = 0, a6 = 0;
  int b1 = threadIdx.x, b3 = threadIdx.x * 3, b5 = threadIdx.x * 5, b7 = threadIdx.x * 7;
  for (int it = 0; it < iters; it++) {
    asm volatile(X8("v_cvt_f64_i32 %0, %1\n v_cvt_f64_i32 %2, %3\n v_cvt_f64_i32 %4, %5\n v_cvt_f64_i32 %6, %7\n")
                 : "+v"(a0), "+v"(b1), "+v"(a2), "+v"(b3), "+v"(a4), "+v"(b5), "+v"(a6), "+v"(b7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a2 + a4 + a6 + b1 + b3 + b5 + b7;
}
__global__ void k_cvt_u32_f64(double* out, int iters) {
  double a0 = threadIdx.x, a2 = a0 * 3, a4 = a0 * 5, a6 = a0 * 7;
  unsigned b1 = 0, b3 = 0, b5 = 0, b7 = 0;
  for (int it = 0; it < iters; it++) {
    asm volatile(X8("v_cvt_u32_f64 %1, %0\n v_cvt_u32_f64 %3, %2\n v_cvt_u32_f64 %5, %4\n v_cvt_u32_f64 %7, %6\n")
                 : "+v"(a0), "+v"(b1), "+v"(a2), "+v"(b3), "+v"(a4), "+v"(b5), "+v"(a6), "+v"(b7));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a2 + a4 + a6 + b1 + b3 + b5 + b7;
}

typedef void (*kfn)(double*, int);
static void run(const char* name, kfn k, int instr_per_iter) {
  int blocks = 256 * 2, threads = 256, iters = 40000;  // 2 waves / SIMD
  double* d; hipMalloc(&d, (size_t)blocks * threads * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 10); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double waves = blocks * threads / 64.0, instr = waves * iters * instr_per_iter;
  double cyc = (ms * 1e-3 * 2.4e9) / (instr / 1024.0);
  printf("%-20s %8.3f ms  %.2f cycles / wave-instr / SIMD (2.4 GHz nominal)\n", name, ms, cyc);
  hipFree(d);
}

int main() {
  run("v_fma_f64", k_fma_f64, 32);
  run("v_add_f64", k_add_f64, 32);
  run("v_mul_f64", k_mul_f64, 32);
  run("v_pk_add_f32", k_pk_add_f32_as_f64, 32);
  run("v_rndne_f64", k_rndne_f64, 32);
  run("v_floor_f64", k_floor_f64, 32);
  run("v_ldexp_f64", k_ldexp_f64, 32);
  run("v_cvt_f64_i32", k_cvt_f64_i32, 32);
  run("v_cvt_u32_f64", k_cvt_u32_f64, 32);
  return 0;
}
