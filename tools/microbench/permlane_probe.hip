#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int L = threadIdx.x;
  unsigned a = L, b = 100 + L;
  auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  out[L] = r16[0]; out[64 + L] = r16[1]; out[128 + L] = r32[0]; out[192 + L] = r32[1];
  // DPP row_ror:8 on a
  out[256 + L] = __builtin_amdgcn_update_dpp(0, (int)a, 0x128, 0xF, 0xF, false);  // row_ror:8
  out[320 + L] = __builtin_amdgcn_update_dpp(0, (int)a, 0x141, 0xF, 0xF, false);  // row_half_mirror
}
int main() {
  int* d; hipMalloc(&d, 384 * 4); hipLaunchKernelGGL(k, 1, 64, 0, 0, d); int h[384]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[6] = {"p16[0]", "p16[1]", "p32[0]", "p32[1]", "ror8", "hmirror"};
  for (int r = 0; r < 6; r++) { printf("%-8s", nm[r]); for (int L = 0; L < 64; L++) printf(" %d", h[r * 64 + L]); printf("\n"); }
  return 0;
}
