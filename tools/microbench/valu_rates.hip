// Per-instruction VALU throughput on gfx950 (inline asm, 8 independent chains per lane, 2 waves/SIMD).
// Also checks v_permlane32_swap semantics.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define BODY(INSTR)                                                                   \
  for (int it = 0; it < iters; it++) {                                                \
    asm volatile(REP8(INSTR " %0, %1\n" INSTR " %2, %3\n" INSTR " %4, %5\n" INSTR " %6, %7\n") \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)); \
  }

// templates for different operand shapes
#define KERNEL(NAME, ASM)                                                           \
  __global__ void NAME(uint64_t* out, int iters) {                                  \
    uint64_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19; \
    for (int it = 0; it < iters; it++) { ASM }                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
  }

#define X8(s) s s s s s s s s
#define KERNEL32(NAME, ASM)                                                         \
  __global__ void NAME(uint64_t* out, int iters) {                                  \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19; \
    for (int it = 0; it < iters; it++) { ASM }                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
  }
// 64-bit add: v_lshl_add_u64 d, a, 0, b
KERNEL(k_lshl_add_u64, asm volatile(X8("v_lshl_add_u64 %0, %0, 0, %1\n v_lshl_add_u64 %2, %2, 0, %3\n v_lshl_add_u64 %4, %4, 0, %5\n v_lshl_add_u64 %6, %6, 0, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL(k_lshlrev_b64, asm volatile(X8("v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 5, %1\n v_lshlrev_b64 %2, 7, %2\n v_lshlrev_b64 %3, 9, %3\n v_lshlrev_b64 %4, 3, %4\n v_lshlrev_b64 %5, 5, %5\n v_lshlrev_b64 %6, 7, %6\n v_lshlrev_b64 %7, 9, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
__global__ void k_mad_u64_u32(uint64_t* out, int iters) {
  uint64_t a0 = threadIdx.x, a2 = a0 * 5, a4 = a0 * 11, a6 = a0 * 17;
  uint32_t b1 = threadIdx.x * 3, b3 = threadIdx.x * 7, b5 = threadIdx.x * 13, b7 = threadIdx.x * 19;
  for (int it = 0; it < iters; it++) {
    asm volatile(X8("v_mad_u64_u32 %0, s[0:1], %1, %1, %0\n v_mad_u64_u32 %2, s[0:1], %3, %3, %2\n v_mad_u64_u32 %4, s[0:1], %5, %5, %4\n v_mad_u64_u32 %6, s[0:1], %7, %7, %6\n")
                 : "+v"(a0), "+v"(b1), "+v"(a2), "+v"(b3), "+v"(a4), "+v"(b5), "+v"(a6), "+v"(b7) :: "s0", "s1");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ b1 ^ a2 ^ b3 ^ a4 ^ b5 ^ a6 ^ b7;
}
KERNEL32(k_mul_lo_u32, asm volatile(X8("v_mul_lo_u32 %0, %0, %1\n v_mul_lo_u32 %2, %2, %3\n v_mul_lo_u32 %4, %4, %5\n v_mul_lo_u32 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL32(k_mul_hi_u32, asm volatile(X8("v_mul_hi_u32 %0, %0, %1\n v_mul_hi_u32 %2, %2, %3\n v_mul_hi_u32 %4, %4, %5\n v_mul_hi_u32 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL32(k_add_u32, asm volatile(X8("v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n v_add_u32 %4, %4, %5\n v_add_u32 %6, %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL(k_cmp_u64, asm volatile(X8("v_cmp_lt_u64 s[0:1], %0, %1\n v_cmp_lt_u64 s[2:3], %2, %3\n v_cmp_lt_u64 s[4:5], %4, %5\n v_cmp_lt_u64 s[6:7], %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "s0","s1","s2","s3","s4","s5","s6","s7");)
KERNEL32(k_cndmask, asm volatile("s_mov_b64 s[0:1], -1\n" X8("v_cndmask_b32 %0, %0, %1, s[0:1]\n v_cndmask_b32 %2, %2, %3, s[0:1]\n v_cndmask_b32 %4, %4, %5, s[0:1]\n v_cndmask_b32 %6, %6, %7, s[0:1]\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "s0","s1");)
KERNEL32(k_add_co, asm volatile(X8("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %2, vcc, %2, %3, vcc\n v_add_co_u32 %4, vcc, %4, %5\n v_addc_co_u32 %6, vcc, %6, %7, vcc\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");)
KERNEL32(k_permlane32, asm volatile(X8("v_permlane32_swap_b32 %0, %1\n v_permlane32_swap_b32 %2, %3\n v_permlane32_swap_b32 %4, %5\n v_permlane32_swap_b32 %6, %7\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL32(k_bitop3, asm volatile(X8("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n v_bitop3_b32 %3, %3, %4, %5 bitop3:0x96\n v_bitop3_b32 %6, %6, %7, %1 bitop3:0x96\n v_bitop3_b32 %2, %2, %3, %4 bitop3:0x96\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
KERNEL32(k_alignbit, asm volatile(X8("v_alignbit_b32 %0, %0, %1, 7\n v_alignbit_b32 %2, %2, %3, 9\n v_alignbit_b32 %4, %4, %5, 11\n v_alignbit_b32 %6, %6, %7, 13\n") : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)

__global__ void perm_check(unsigned* out) {
  unsigned x = threadIdx.x * 100u, y = threadIdx.x * 100u + 1u;
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[threadIdx.x * 2] = r[0];
  out[threadIdx.x * 2 + 1] = r[1];
}

typedef void (*kfn)(uint64_t*, int);
static void run(const char* name, kfn k, int instr_per_iter, bool b64 = false) {
  int blocks = 256 * 2, threads = 256, iters = 40000;  // 2 waves / SIMD
  uint64_t* d; hipMalloc(&d, (size_t)blocks * threads * 8);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, 10); hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d, iters);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double waves = blocks * threads / 64.0, instr = waves * iters * instr_per_iter;
  // cycles per wave-instruction per SIMD at 2.4 GHz: (ms*1e-3*2.4e9) / (instr / (256*4))
  double cyc = (ms * 1e-3 * 2.4e9) / (instr / 1024.0);
  printf("%-16s %8.3f ms  %.2f cycles / wave-instr / SIMD (2.4 GHz nominal)\n", name, ms, cyc);
  hipFree(d);
}

int main() {
  run("v_add_u32", k_add_u32, 32);
  run("v_lshl_add_u64", k_lshl_add_u64, 32);
  run("v_lshlrev_b64", k_lshlrev_b64, 64);
  run("v_alignbit_b32", k_alignbit, 32);
  run("v_bitop3_b32", k_bitop3, 32);
  run("v_mul_lo_u32", k_mul_lo_u32, 32);
  run("v_mul_hi_u32", k_mul_hi_u32, 32);
  run("v_mad_u64_u32", k_mad_u64_u32, 32);
  run("v_cmp_lt_u64", k_cmp_u64, 32);
  run("v_cndmask_b32", k_cndmask, 32);
  run("v_add_co/addc", k_add_co, 32);
  run("v_permlane32_swap", k_permlane32, 32);
  unsigned* d; hipMalloc(&d, 64 * 2 * 4);
  hipLaunchKernelGGL(perm_check, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("permlane32_swap(x=100*l, y=100*l+1): lane0 -> {%u,%u} lane1 -> {%u,%u} lane32 -> {%u,%u} lane33 -> {%u,%u}\n",
         h[0], h[1], h[2], h[3], h[64], h[65], h[66], h[67]);
  return 0;
}
