// LDS instruction throughput on gfx950 for the FFT64 transposes' access shapes: cycles per wave
// instruction per CU with 8 waves per CU (2 per SIMD, the blind-rotation kernels' occupancy), every wave
// streaming DS instructions on its own 9 KB region, lgkmcnt drained once per 16 instructions.
//   w128   ds_write_b128 at lane * 16 (+ 1 KB per instruction): the transposes' contiguous writes
//   w64    ds_write_b64 at lane * 8 (+ 512 B): split re / im planes, two per complex slot
//   w2_64  ds_write2_b64 of two 8-byte values 512 B apart (one instruction per complex slot, planes)
//   r128   ds_read_b128 contiguous
//   r128g1 ds_read_b128 at the T1 gather (lane >> 3) * 72 + (lane & 7) (complex units)
//   r128g2 ds_read_b128 at the T2 gather (lane & 7) * 65 + 8 (lane >> 3)
//   r64    ds_read_b64 contiguous; r2_64 ds_read2_b64 512 B apart
//   r64g2  ds_read_b64 at the T2 gather in 8-byte units (plane layout, stride 65)
#include <hip/hip_runtime.h>
#include <cstdio>

enum Op { W128, W64, W2_64, R128, R128G1, R128G2, R64, R2_64, R64G2 };

template <Op OP>
__global__ __launch_bounds__(512, 1) void k_lds(double* out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[8 * 9216];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  char* base = lds + wave * 9216;
  unsigned addr;
  switch (OP) {
    case W128: case R128: addr = lane * 16; break;
    case R128G1: addr = ((lane >> 3) * 72 + (lane & 7)) * 16; break;
    case R128G2: addr = ((lane & 7) * 65 + 8 * (lane >> 3)) * 16; break;
    case R64G2: addr = ((lane & 7) * 65 + 8 * (lane >> 3)) * 8; break;
    default: addr = lane * 8; break;
  }
  addr += (unsigned)(size_t)(__attribute__((address_space(3))) char*)base;
  typedef double v2d __attribute__((ext_vector_type(2)));
  v2d v = {1.0 * threadIdx.x, 2.0};
  double s = 3.0;
  v2d acc = {0, 0};
  double acs = 0;
  for (int it = 0; it < iters; it++) {
#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
    if (OP == W128) {
#define W(i) asm volatile("ds_write_b128 %0, %1 offset:" #i "*512" ::"v"(addr), "v"(v) : "memory");
      // offsets: i * 512 within 9 KB (16 x 512 = 8 KB)
      REP16(W)
#undef W
    } else if (OP == W64) {
#define W(i) asm volatile("ds_write_b64 %0, %1 offset:" #i "*512" ::"v"(addr), "v"(s) : "memory");
      REP16(W)
#undef W
    } else if (OP == W2_64) {
#define W(i) asm volatile("ds_write2_b64 %0, %1, %2 offset0:" #i "*4 offset1:" #i "*4+64" ::"v"(addr), "v"(s), "v"(s) : "memory");
      REP16(W)
#undef W
    } else if (OP == R128 || OP == R128G1 || OP == R128G2) {
#define R(i)                                                                              \
  {                                                                                       \
    v2d t;                                                                                \
    asm volatile("ds_read_b128 %0, %1 offset:" #i "*64" : "=v"(t) : "v"(addr) : "memory"); \
    acc += t;                                                                             \
  }
      REP16(R)
#undef R
    } else if (OP == R64 || OP == R64G2) {
#define R(i)                                                                              \
  {                                                                                       \
    double t;                                                                             \
    asm volatile("ds_read_b64 %0, %1 offset:" #i "*64" : "=v"(t) : "v"(addr) : "memory"); \
    acs += t;                                                                             \
  }
      REP16(R)
#undef R
    } else if (OP == R2_64) {
#define R(i)                                                                                                   \
  {                                                                                                            \
    v2d t;                                                                                                     \
    asm volatile("ds_read2_b64 %0, %1 offset0:" #i "*4 offset1:" #i "*4+64" : "=v"(t) : "v"(addr) : "memory"); \
    acc += t;                                                                                                  \
  }
      REP16(R)
#undef R
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc.x + acc.y + acs;
}

typedef void (*kfn)(double*, int);
static void run(const char* name, kfn k, int bytes_per_lane) {
  const int blocks = 256, threads = 512, iters = 20000;
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
  const double instr_per_cu = 8.0 * iters * 16, cyc = ms * 1e-3 * 2.4e9 / instr_per_cu;
  printf("%-8s %7.3f ms  %6.2f cycles / wave-instr / CU  %6.1f B/clk/CU\n", name, ms, cyc, 64.0 * bytes_per_lane / cyc);
  hipFree(d);
}

int main() {
  run("w128", k_lds<W128>, 16);
  run("w64", k_lds<W64>, 8);
  run("w2_64", k_lds<W2_64>, 16);
  run("r128", k_lds<R128>, 16);
  run("r128g1", k_lds<R128G1>, 16);
  run("r128g2", k_lds<R128G2>, 16);
  run("r64", k_lds<R64>, 8);
  run("r2_64", k_lds<R2_64>, 16);
  run("r64g2", k_lds<R64G2>, 8);
  return 0;
}
