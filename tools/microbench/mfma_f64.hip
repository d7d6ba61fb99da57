// v_mfma_f64_16x16x4_f64 on gfx950: throughput, overlap with VALU f64 and rounding semantics
// ("trial v_mfma_f64_16x16x4_f64 for the radix-8 passes").
//  1. rate: C independent 16x16 accumulators per wave, 1 / 2 waves per SIMD -> cycles per MFMA per SIMD
//  2. overlap: the same MFMA stream plus an independent v_fma_f64 stream in the same wave, against each
//     alone (does the matrix pipe run beside the VALU?)
//  3. semantics: one wave, random operands with mixed exponents; A, B, C, D dumped raw to
//     gpurun_out/mfma_f64_probe.bin for tools/microbench/mfma_f64_check.py (exact rational analysis)
// Layout (cdna_hip_programming.md §3): A lane l = A[l & 15][l >> 4], B lane l = B[l >> 4][l & 15],
// C/D reg r of lane l = D[(l >> 4) + 4 r][l & 15].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

typedef double v4d __attribute__((ext_vector_type(4)));

template <int C, int V>
__global__ void k_mix(double* out, int iters) {
  v4d acc[C > 0 ? C : 1];
  double f[V > 0 ? V : 1];
  const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
#pragma unroll
  for (int c = 0; c < (C > 0 ? C : 1); c++) acc[c] = (v4d){c * 1.0, 0.5, 0.25, 0.125};
#pragma unroll
  for (int v = 0; v < (V > 0 ? V : 1); v++) f[v] = threadIdx.x * (1.0 + v);
  const double m = 1.0000001, s = 1e-9;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 4; r++) {
#pragma unroll
      for (int c = 0; c < C; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < V; v++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f[v]) : "v"(m), "v"(s));
    }
  }
  double t = 0;
#pragma unroll
  for (int c = 0; c < C; c++) t += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
#pragma unroll
  for (int v = 0; v < V; v++) t += f[v];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void k_probe(const double* A, const double* B, const double* Cin, double* D, int reps) {
  const int l = threadIdx.x;
  for (int t = 0; t < reps; t++) {
    const v4d c = {Cin[(t * 64 + l) * 4 + 0], Cin[(t * 64 + l) * 4 + 1], Cin[(t * 64 + l) * 4 + 2],
                   Cin[(t * 64 + l) * 4 + 3]};
    const v4d d = __builtin_amdgcn_mfma_f64_16x16x4f64(A[t * 64 + l], B[t * 64 + l], c, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) D[(t * 64 + l) * 4 + r] = d[r];
  }
}

typedef void (*kfn)(double*, int);
static double run(const char* name, kfn k, int mfma_per_iter, int fma_per_iter, int waves_per_simd) {
  const int threads = 256, blocks = 256 * waves_per_simd, iters = 4000;
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
  const double wps = waves_per_simd, cyc = ms * 1e-3 * 2.4e9 / (iters * 4.0 * wps);  // SIMD cycles per wave-iteration-quarter
  printf("%-24s waves/SIMD %d  %8.3f ms  %7.2f cycles per (%d MFMA + %d FMA) group per wave", name, waves_per_simd, ms,
         cyc, mfma_per_iter, fma_per_iter);
  if (mfma_per_iter) printf("  = %.2f cycles/MFMA (%.1f f64 FMA/clk/SIMD)", cyc / mfma_per_iter, 1024.0 * mfma_per_iter / cyc);
  printf("\n");
  hipFree(d);
  return cyc;
}

int main(int argc, char** argv) {
  const char* dump = argc > 1 ? argv[1] : "gpurun_out/mfma_f64_probe.bin";
  for (int w : {1, 2}) {
    run("mfma C=1", k_mix<1, 0>, 1, 0, w);
    run("mfma C=2", k_mix<2, 0>, 2, 0, w);
    run("mfma C=4", k_mix<4, 0>, 4, 0, w);
    run("mfma C=8", k_mix<8, 0>, 8, 0, w);
    run("fma V=16", k_mix<0, 16>, 0, 16, w);
    run("mfma C=4 + fma V=16", k_mix<4, 16>, 4, 16, w);
    run("fma V=32", k_mix<0, 32>, 0, 32, w);
    run("mfma C=4 + fma V=32", k_mix<4, 32>, 4, 32, w);
  }
  // semantics probe
  const int reps = 256, n = reps * 64;
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::uniform_int_distribution<int> ex(-40, 40);
  double *hA = (double*)malloc(n * 8), *hB = (double*)malloc(n * 8), *hC = (double*)malloc(n * 32),
         *hD = (double*)malloc(n * 32);
  for (int i = 0; i < n; i++) {
    hA[i] = ldexp(u(g), ex(g) / 4);
    hB[i] = ldexp(u(g), ex(g) / 4);
  }
  for (int i = 0; i < 4 * n; i++) hC[i] = (i % 3 == 0) ? 0.0 : ldexp(u(g), ex(g) / 4);
  double *dA, *dB, *dC, *dD;
  hipMalloc(&dA, n * 8);
  hipMalloc(&dB, n * 8);
  hipMalloc(&dC, n * 32);
  hipMalloc(&dD, n * 32);
  hipMemcpy(dA, hA, n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, n * 8, hipMemcpyHostToDevice);
  hipMemcpy(dC, hC, n * 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD, reps);
  hipMemcpy(hD, dD, n * 32, hipMemcpyDeviceToHost);
  FILE* fp = fopen(dump, "wb");
  if (!fp) { printf("cannot write %s\n", dump); return 1; }
  const int hdr[2] = {reps, 64};
  fwrite(hdr, 4, 2, fp);
  fwrite(hA, 8, n, fp);
  fwrite(hB, 8, n, fp);
  fwrite(hC, 8, 4 * n, fp);
  fwrite(hD, 8, 4 * n, fp);
  fclose(fp);
  printf("probe: %d MFMAs dumped to %s\n", reps, dump);
  return 0;
}
