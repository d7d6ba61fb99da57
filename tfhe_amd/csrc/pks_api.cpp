// pks_api.cpp — C ABI of the packing keyswitch / compression (include/tfhe_hip.h, tfhe_hip_pks_*):
// key residency, workspace, chunked launches.  Kernels: pks.hip; host key material: client.cpp.
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "../../include/tfhe_hip.h"
#include "client.h"
#include "pbs_kernels.h"

using tfhe::u32;
using tfhe::u64;

// shared error slot of the library (api.cpp)
int tfhe_hip_set_error(int code, const char* msg);

namespace {

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return tfhe_hip_set_error(code, buf);
}

#define PKS_TRY(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess)                                                                                \
      return fail(_e == hipErrorOutOfMemory ? TFHE_HIP_ENOMEM : TFHE_HIP_EDEVICE, "%s: %s (%s:%d)", #expr, \
                  hipGetErrorString(_e), __FILE__, __LINE__);                                            \
  } while (0)

bool pks_valid(const tfhe_pks_params* pp) {
  return pp && pp->in_dim > 0 && pp->in_dim % 16 == 0 && pp->out_k > 0 && pp->out_N >= 32 &&
         (pp->out_N & (pp->out_N - 1)) == 0 && ((pp->out_k + 1) * pp->out_N) % 64 == 0 && pp->base_log >= 2 &&
         pp->level > 0 && pp->base_log * pp->level < 64 && pp->base_log <= 31 && pp->lwe_per_glwe > 0 &&
         pp->lwe_per_glwe <= pp->out_N && pp->storage_log > 0 && pp->storage_log < 64 && pp->noise_log2 < 0 &&
         pp->noise_log2 > -64;
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != d) (void)hipSetDevice(d);
  }
  ~DevGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

constexpr size_t PKS_T_BUDGET = 512ull << 20;  // T workspace per chunk of groups

}  // namespace

struct tfhe_pks_ctx {
  tfhe_pks_params pp{};
  int device = 0;
  hipStream_t stream = nullptr;
  u64* d_pksk = nullptr;
  u64* d_corr = nullptr;
  bool key = false;
  u32* d_A = nullptr;
  u64* d_T = nullptr;
  size_t rows_cap = 0;  // LWEs the A / T workspaces hold
  // matrix-core path (default; TFHE_HIP_PKS_VALU=1 keeps the VALU GEMM): the key's byte planes and the
  // two digit-byte operands
  bool valu = false;
  void* d_planes = nullptr;
  void* d_A0 = nullptr;
  void* d_A1 = nullptr;
  u64* d_io = nullptr;
  size_t io_cap = 0;  // bytes
  std::mutex mu;
};

namespace {

int ensure_rows(tfhe_pks_ctx* c, size_t rows) {
  if (c->rows_cap >= rows) return 0;
  for (void* p : {(void*)c->d_A, (void*)c->d_T, c->d_A0, c->d_A1}) (void)hipFree(p);
  c->d_A = nullptr;
  c->d_T = nullptr;
  c->d_A0 = c->d_A1 = nullptr;
  c->rows_cap = 0;
  const size_t K = (size_t)c->pp.in_dim * c->pp.level, Nc = (size_t)(c->pp.out_k + 1) * c->pp.out_N;
  if (c->valu) {
    PKS_TRY(hipMalloc(&c->d_A, rows * K * sizeof(u32)));
  } else {
    const size_t r = tfhe::pks_mfma_rows(rows);
    PKS_TRY(hipMalloc(&c->d_A0, r * K));
    PKS_TRY(hipMalloc(&c->d_A1, r * K));
  }
  PKS_TRY(hipMalloc(&c->d_T, rows * Nc * sizeof(u64)));
  c->rows_cap = rows;
  return 0;
}

int pack_device(tfhe_pks_ctx* c, const u64* d_lwes, size_t count, u64* d_out, hipStream_t s) {
  const tfhe_pks_params& p = c->pp;
  const size_t Nc = (size_t)(p.out_k + 1) * p.out_N, lpg = p.lwe_per_glwe;
  const size_t groups_per_chunk = std::max<size_t>(1, PKS_T_BUDGET / (lpg * Nc * 8));
  const size_t rows = std::min(count, groups_per_chunk * lpg);
  int rc = ensure_rows(c, rows);
  if (rc) return rc;
  for (size_t first = 0; first < count; first += rows) {
    const size_t n = std::min(rows, count - first);
    if (c->valu)
      PKS_TRY(tfhe::launch_pks_pack(d_lwes + first * (p.in_dim + 1), n, (int)p.in_dim, (int)p.base_log, (int)p.level,
                                    (int)p.out_k, (int)p.out_N, (int)lpg, c->d_pksk, c->d_corr, c->d_A, c->d_T,
                                    d_out + (first / lpg) * Nc, s));
    else
      PKS_TRY(tfhe::launch_pks_pack_mfma(d_lwes + first * (p.in_dim + 1), n, (int)p.in_dim, (int)p.base_log,
                                         (int)p.level, (int)p.out_k, (int)p.out_N, (int)lpg, c->d_planes, c->d_A0,
                                         c->d_A1, c->d_T, d_out + (first / lpg) * Nc, s));
  }
  return 0;
}

}  // namespace

extern "C" {

int tfhe_hip_pks_params_preset(int preset, tfhe_pks_params* o) {
  if (!o) return fail(TFHE_HIP_EINVAL, "pks_params_preset: null out");
  if (preset != TFHE_HIP_PKS_PRESET_ML2048) return fail(TFHE_HIP_EINVAL, "unknown packing preset %d", preset);
  *o = tfhe_pks_params{2048, 1, 2048, 14, 2, 2048, 26, -48};
  return 0;
}

size_t tfhe_hip_pksk_len(const tfhe_pks_params* pp) { return pp ? tfhe::client::pksk_len(*pp) : 0; }

int tfhe_hip_pks_keygen_k(const tfhe_pks_params* pp, const tfhe_rng_key* rk, const uint64_t* in_key,
                          uint64_t* out_key, uint64_t* pksk) {
  if (!pks_valid(pp) || !rk || !in_key || !out_key) return fail(TFHE_HIP_EINVAL, "pks_keygen: bad arguments");
  for (uint32_t j = 0; j < pp->in_dim; j++)
    if (in_key[j] > 1) return fail(TFHE_HIP_EINVAL, "pks_keygen: in_key[%u] is not binary", j);
  tfhe::client::pks_keygen(*pp, *rk, in_key, out_key, pksk);
  return 0;
}

int tfhe_hip_pks_keygen(const tfhe_pks_params* pp, uint64_t seed, const uint64_t* in_key, uint64_t* out_key,
                        uint64_t* pksk) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_pks_keygen_k(pp, &rk, in_key, out_key, pksk);
}

int tfhe_hip_pks_create(const tfhe_pks_params* pp, int device, tfhe_pks_ctx** out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "pks_create: null out");
  *out = nullptr;
  if (!pks_valid(pp)) return fail(TFHE_HIP_EINVAL, "pks_create: invalid parameters");
  int ndev = 0;
  PKS_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TFHE_HIP_EINVAL, "pks_create: device %d of %d", device, ndev);
  DevGuard g(device);
  tfhe_pks_ctx* c = new tfhe_pks_ctx();
  c->pp = *pp;
  c->device = device;
  {
    const char* e = getenv("TFHE_HIP_PKS_VALU");
    // the matrix-core GEMM needs int8 digit bytes (base <= 16) and 64-deep k steps
    c->valu = (e && e[0] == '1') || pp->base_log > 16 || (pp->in_dim * pp->level) % 64 != 0;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(TFHE_HIP_EDEVICE, "pks_create: hipStreamCreate failed");
  }
  *out = c;
  return 0;
}

void tfhe_hip_pks_destroy(tfhe_pks_ctx* c) {
  if (!c) return;
  {
    DevGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_pksk);
    (void)hipFree(c->d_corr);
    (void)hipFree(c->d_A);
    (void)hipFree(c->d_T);
    (void)hipFree(c->d_io);
    (void)hipFree(c->d_planes);
    (void)hipFree(c->d_A0);
    (void)hipFree(c->d_A1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

int tfhe_hip_pks_load_key(tfhe_pks_ctx* c, const uint64_t* pksk, size_t len) {
  if (!c || !pksk) return fail(TFHE_HIP_EINVAL, "pks_load_key: null argument");
  if (len != tfhe::client::pksk_len(c->pp))
    return fail(TFHE_HIP_EINVAL, "pks_load_key: length %zu, expected %zu", len, tfhe::client::pksk_len(c->pp));
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  c->key = false;
  const size_t Nc = (size_t)(c->pp.out_k + 1) * c->pp.out_N;
  if (!c->d_pksk) PKS_TRY(hipMalloc(&c->d_pksk, len * 8));
  if (!c->d_corr) PKS_TRY(hipMalloc(&c->d_corr, Nc * 8));
  PKS_TRY(hipMemcpyAsync(c->d_pksk, pksk, len * 8, hipMemcpyHostToDevice, c->stream));
  PKS_TRY(tfhe::launch_pks_corr(c->d_pksk, (int)(c->pp.in_dim * c->pp.level), (int)Nc, (int)c->pp.base_log, c->d_corr,
                                c->stream));
  if (!c->valu) {  // balanced byte planes of the key (ks_mfma.hip's recoding, Nc columns)
    if (!c->d_planes)
      PKS_TRY(hipMalloc(&c->d_planes, tfhe::ks_planes_bytes((int)c->pp.in_dim, (int)c->pp.level, (int)Nc - 1)));
    PKS_TRY(tfhe::launch_ksk_planes(c->d_pksk, (int)c->pp.in_dim, (int)c->pp.level, (int)Nc - 1, c->d_planes, c->stream));
  }
  PKS_TRY(hipStreamSynchronize(c->stream));
  c->key = true;
  return 0;
}

int tfhe_hip_pks_pack_async(tfhe_pks_ctx* c, const uint64_t* d_lwes, size_t count, uint64_t* d_glwes, void* stream) {
  if (!c) return fail(TFHE_HIP_EINVAL, "pks_pack: null ctx");
  if (!c->key) return fail(TFHE_HIP_ENOKEYS, "pks_pack: key not loaded");
  if (count == 0) return 0;
  if (!d_lwes || !d_glwes) return fail(TFHE_HIP_EINVAL, "pks_pack: null buffer");
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  return pack_device(c, d_lwes, count, d_glwes, stream == TFHE_HIP_NULL_STREAM ? (hipStream_t)0 : stream ? (hipStream_t)stream : c->stream);
}

int tfhe_hip_pks_pack(tfhe_pks_ctx* c, const uint64_t* lwes, size_t count, uint64_t* glwes) {
  if (!c) return fail(TFHE_HIP_EINVAL, "pks_pack: null ctx");
  if (!c->key) return fail(TFHE_HIP_ENOKEYS, "pks_pack: key not loaded");
  if (count == 0) return 0;
  if (!lwes || !glwes) return fail(TFHE_HIP_EINVAL, "pks_pack: null buffer");
  if (count > 0x7FFFFFFF) return fail(TFHE_HIP_EINVAL, "pks_pack: too many ciphertexts");
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  const tfhe_pks_params& p = c->pp;
  const size_t in_bytes = count * (p.in_dim + 1) * 8, groups = (count + p.lwe_per_glwe - 1) / p.lwe_per_glwe;
  const size_t out_bytes = groups * (p.out_k + 1) * p.out_N * 8, in_off = (out_bytes + 255) & ~(size_t)255;
  if (c->io_cap < in_off + in_bytes) {
    (void)hipFree(c->d_io);
    c->d_io = nullptr;
    c->io_cap = 0;
    PKS_TRY(hipMalloc(&c->d_io, in_off + in_bytes));
    c->io_cap = in_off + in_bytes;
  }
  u64* d_out = c->d_io;
  u64* d_in = (u64*)((char*)c->d_io + in_off);
  PKS_TRY(hipMemcpyAsync(d_in, lwes, in_bytes, hipMemcpyHostToDevice, c->stream));
  int rc = pack_device(c, d_in, count, d_out, c->stream);
  if (rc) return rc;
  PKS_TRY(hipMemcpyAsync(glwes, d_out, out_bytes, hipMemcpyDeviceToHost, c->stream));
  PKS_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

size_t tfhe_hip_pks_packed_words(const tfhe_pks_params* pp, uint32_t bodies) {
  return pp ? tfhe::client::pks_packed_words(*pp, bodies) : 0;
}

int tfhe_hip_pks_compress(const tfhe_pks_params* pp, const uint64_t* glwe, uint32_t bodies, uint64_t* packed) {
  if (!pks_valid(pp) || !glwe || !packed || bodies > pp->out_N) return fail(TFHE_HIP_EINVAL, "pks_compress: bad arguments");
  tfhe::client::pks_compress(*pp, glwe, bodies, packed);
  return 0;
}

int tfhe_hip_pks_extract(const tfhe_pks_params* pp, const uint64_t* packed, uint32_t bodies, uint64_t* glwe) {
  if (!pks_valid(pp) || !glwe || !packed || bodies > pp->out_N) return fail(TFHE_HIP_EINVAL, "pks_extract: bad arguments");
  tfhe::client::pks_extract(*pp, packed, bodies, glwe);
  return 0;
}

int tfhe_hip_glwe_phase(uint32_t k, uint32_t N, const uint64_t* key, const uint64_t* glwe, uint64_t* out) {
  if (!k || !N || !key || !glwe || !out) return fail(TFHE_HIP_EINVAL, "glwe_phase: bad arguments");
  tfhe::client::glwe_phase_native(k, N, key, glwe, out);
  return 0;
}

}  // extern "C"
