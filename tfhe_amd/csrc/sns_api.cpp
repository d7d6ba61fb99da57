// sns_api.cpp — C ABI of noise squashing (include/tfhe_hip.h, tfhe_hip_sns_*): key residency,
// workspaces, chunked launches.  Kernels: sns.hip; host key material: client.cpp.
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/tfhe_hip.h"
#include "client.h"
#include "pbs_kernels.h"

using tfhe::u64;

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

#define SNS_TRY(expr)                                                                                    \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess)                                                                                \
      return fail(_e == hipErrorOutOfMemory ? TFHE_HIP_ENOMEM : TFHE_HIP_EDEVICE, "%s: %s (%s:%d)", #expr, \
                  hipGetErrorString(_e), __FILE__, __LINE__);                                            \
  } while (0)

// the device kernels of this build: k = 2, N = 2048, 2^24 x 3 (any n), words over Z_2^128
bool sns_valid(const tfhe_sns_params* sp) {
  return sp && sp->n > 0 && sp->k == 2 && sp->N == 2048 && sp->base_log == 24 && sp->level == 3 &&
         sp->noise_log2 < 0 && sp->noise_log2 > -64;
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

// ciphertexts per pass (acc 96 KB + digit spectra 147 KB + MAC products 246 KB each); TFHE_HIP_SNS_CHUNK overrides.
// 512 since round 6: a 1024 batch as two 512 chunks measured 4,819 vs 4,556 squashes/s (256: 4,455) on one box
// (profiles/r06c_sns_chunk.txt; round 5: 4,687 vs 4,568): the inverse gains more from the smaller per-CMUX working set
// than the MAC and step 1 lose to the half-size grids
size_t sns_chunk() {
  static const size_t v = [] {
    const char* e = getenv("TFHE_HIP_SNS_CHUNK");
    const long x = e ? atol(e) : 0;
    return x > 0 ? (size_t)x : (size_t)512;
  }();
  return v;
}

}  // namespace

struct tfhe_sns_ctx {
  tfhe_sns_params sp{};
  int device = 0;
  hipStream_t stream = nullptr;
  void* d_fconst = nullptr;
  void* d_bskf = nullptr;  // key limb spectra (n x 9 x 3 x 5 x 1024 complex f64)
  bool key = false;
  u64* d_acc = nullptr;    // chunk x 3 x (lo, hi) x N
  void* d_D = nullptr;     // digit spectra (chunk x 9 x 1024 complex)
  void* d_O = nullptr;     // MAC products (chunk x 15 x 1024 complex)
  u64* d_lut = nullptr;
  uint32_t lut_mm = 0;
  size_t ws_cap = 0;
  u64* d_io = nullptr;
  size_t io_cap = 0;
  std::mutex mu;
};

namespace {

int ensure_ws(tfhe_sns_ctx* c, size_t B) {
  if (c->ws_cap >= B) return 0;
  (void)hipFree(c->d_acc);
  (void)hipFree(c->d_D);
  (void)hipFree(c->d_O);
  c->d_acc = nullptr;
  c->d_D = c->d_O = nullptr;
  c->ws_cap = 0;
  const size_t poly = 2 * (size_t)c->sp.N;
  SNS_TRY(hipMalloc(&c->d_acc, B * (c->sp.k + 1) * poly * 8));
  SNS_TRY(hipMalloc(&c->d_D, tfhe::sns_digit_len(B) * 16));
  SNS_TRY(hipMalloc(&c->d_O, tfhe::sns_fft_prod_len(B) * 16));
  c->ws_cap = B;
  return 0;
}

int ensure_lut(tfhe_sns_ctx* c, uint32_t mm) {
  if (c->d_lut && c->lut_mm == mm) return 0;
  std::vector<u64> lut(2 * (size_t)c->sp.N);
  tfhe::client::sns_lut_identity(c->sp, mm, lut.data());
  if (!c->d_lut) SNS_TRY(hipMalloc(&c->d_lut, lut.size() * 8));
  SNS_TRY(hipMemcpy(c->d_lut, lut.data(), lut.size() * 8, hipMemcpyHostToDevice));
  c->lut_mm = mm;
  return 0;
}

// squash (out != null) or blind rotate only (acc_out != null) of B device ciphertexts
int run_device(tfhe_sns_ctx* c, const u64* d_in, size_t B, u64* d_out, u64* d_acc_out, hipStream_t s) {
  const size_t chunk = std::min(B, sns_chunk());
  int rc = ensure_ws(c, chunk);
  if (rc) return rc;
  const size_t in_dim = c->sp.n + 1, out_dim = 2 * ((size_t)c->sp.k * c->sp.N + 1);
  const size_t acc_len = (size_t)(c->sp.k + 1) * 2 * c->sp.N;
  for (size_t f = 0; f < B; f += chunk) {
    const size_t nb = std::min(chunk, B - f);
    SNS_TRY(tfhe::launch_sns_blind_rotate(d_in + f * in_dim, nb, (int)c->sp.n, c->d_lut, c->d_bskf, c->d_acc, c->d_D,
                                          c->d_O, c->d_fconst, s));
    if (d_out) SNS_TRY(tfhe::launch_sns_extract(c->d_acc, nb, d_out + f * out_dim, s));
    if (d_acc_out)
      SNS_TRY(hipMemcpyAsync(d_acc_out + f * acc_len, c->d_acc, nb * acc_len * 8, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

int host_call(tfhe_sns_ctx* c, const u64* in, size_t B, uint32_t mm, u64* out, bool acc_only) {
  if (!c) return fail(TFHE_HIP_EINVAL, "sns: null ctx");
  if (!c->key) return fail(TFHE_HIP_ENOKEYS, "sns: key not loaded");
  if (B == 0) return 0;
  if (!in || !out || !mm || mm > c->sp.N || (c->sp.N % mm)) return fail(TFHE_HIP_EINVAL, "sns: bad arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  int rc = ensure_lut(c, mm);
  if (rc) return rc;
  const size_t in_bytes = B * (c->sp.n + 1) * 8;
  const size_t out_bytes = acc_only ? B * (c->sp.k + 1) * 2 * c->sp.N * 8 : B * 2 * ((size_t)c->sp.k * c->sp.N + 1) * 8;
  const size_t off = (out_bytes + 255) & ~(size_t)255;
  if (c->io_cap < off + in_bytes) {
    (void)hipFree(c->d_io);
    c->d_io = nullptr;
    c->io_cap = 0;
    SNS_TRY(hipMalloc(&c->d_io, off + in_bytes));
    c->io_cap = off + in_bytes;
  }
  u64* d_out = c->d_io;
  u64* d_in = (u64*)((char*)c->d_io + off);
  SNS_TRY(hipMemcpyAsync(d_in, in, in_bytes, hipMemcpyHostToDevice, c->stream));
  rc = run_device(c, d_in, B, acc_only ? nullptr : d_out, acc_only ? d_out : nullptr, c->stream);
  if (rc) return rc;
  SNS_TRY(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, c->stream));
  SNS_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

}  // namespace

extern "C" {

int tfhe_hip_sns_params_preset(int preset, tfhe_sns_params* o) {
  if (!o) return fail(TFHE_HIP_EINVAL, "sns_params_preset: null out");
  if (preset != TFHE_HIP_SNS_PRESET_FHEVM) return fail(TFHE_HIP_EINVAL, "unknown squashing preset %d", preset);
  *o = tfhe_sns_params{918, 2, 2048, 24, 3, -34};
  return 0;
}

size_t tfhe_hip_sns_bsk_len(const tfhe_sns_params* sp) { return sp ? tfhe::client::sns_bsk_len(*sp) : 0; }

int tfhe_hip_sns_keygen_k(const tfhe_sns_params* sp, const tfhe_rng_key* rk, const uint64_t* lwe_key,
                          uint64_t* glwe_key, uint64_t* bsk) {
  if (!sns_valid(sp) || !rk || !lwe_key || !glwe_key) return fail(TFHE_HIP_EINVAL, "sns_keygen: bad arguments");
  for (uint32_t i = 0; i < sp->n; i++)
    if (lwe_key[i] > 1) return fail(TFHE_HIP_EINVAL, "sns_keygen: lwe_key[%u] is not binary", i);
  tfhe::client::sns_keygen(*sp, *rk, lwe_key, glwe_key, bsk);
  return 0;
}

int tfhe_hip_sns_keygen(const tfhe_sns_params* sp, uint64_t seed, const uint64_t* lwe_key, uint64_t* glwe_key,
                        uint64_t* bsk) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_sns_keygen_k(sp, &rk, lwe_key, glwe_key, bsk);
}

int tfhe_hip_sns_create(const tfhe_sns_params* sp, int device, tfhe_sns_ctx** out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "sns_create: null out");
  *out = nullptr;
  if (!sns_valid(sp))
    return fail(TFHE_HIP_EUNSUPPORTED, "sns_create: the device kernels cover k = 2, N = 2048, 2^24 x 3");
  int ndev = 0;
  SNS_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TFHE_HIP_EINVAL, "sns_create: device %d of %d", device, ndev);
  DevGuard g(device);
  tfhe_sns_ctx* c = new tfhe_sns_ctx();
  c->sp = *sp;
  c->device = device;
  std::vector<unsigned char> F(tfhe::sns_fft_const_bytes());
  tfhe::make_sns_fft_const(F.data());
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_fconst, F.size()) != hipSuccess ||
      hipMemcpy(c->d_fconst, F.data(), F.size(), hipMemcpyHostToDevice) != hipSuccess) {
    tfhe_hip_sns_destroy(c);
    return fail(TFHE_HIP_EDEVICE, "sns_create: device setup failed");
  }
  *out = c;
  return 0;
}

void tfhe_hip_sns_destroy(tfhe_sns_ctx* c) {
  if (!c) return;
  {
    DevGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : {c->d_fconst, c->d_bskf, (void*)c->d_acc, c->d_D, c->d_O, (void*)c->d_lut, (void*)c->d_io})
      (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

int tfhe_hip_sns_load_key(tfhe_sns_ctx* c, const uint64_t* bsk, size_t len) {
  if (!c || !bsk) return fail(TFHE_HIP_EINVAL, "sns_load_key: null argument");
  if (len != tfhe::client::sns_bsk_len(c->sp))
    return fail(TFHE_HIP_EINVAL, "sns_load_key: length %zu, expected %zu", len, tfhe::client::sns_bsk_len(c->sp));
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  c->key = false;
  if (!c->d_bskf) SNS_TRY(hipMalloc(&c->d_bskf, tfhe::sns_fft_key_len(c->sp.n) * 16));
  // stage the key words in chunks of polynomials (lo, hi planes) through the io buffer, convert to limb spectra
  const size_t poly_words = 2 * (size_t)c->sp.N, polys = len / poly_words, per = 2048;
  const size_t bytes = per * poly_words * 8;
  if (c->io_cap < bytes) {
    (void)hipFree(c->d_io);
    c->d_io = nullptr;
    c->io_cap = 0;
    SNS_TRY(hipMalloc(&c->d_io, bytes));
    c->io_cap = bytes;
  }
  for (size_t f = 0; f < polys; f += per) {
    const size_t np = std::min(per, polys - f);
    SNS_TRY(hipMemcpyAsync(c->d_io, bsk + f * poly_words, np * poly_words * 8, hipMemcpyHostToDevice, c->stream));
    SNS_TRY(tfhe::launch_sns_bsk_to_fft(c->d_io, (char*)c->d_bskf + f * tfhe::SNS_FFT_POLY_BYTES, np, c->d_fconst,
                                        c->stream));
    // the io buffer is reused by the next chunk's copy: same stream, ordered
  }
  SNS_TRY(hipStreamSynchronize(c->stream));
  c->key = true;
  return 0;
}

int tfhe_hip_sns_squash(tfhe_sns_ctx* c, const uint64_t* in, size_t B, uint32_t mm, uint64_t* out) {
  return host_call(c, in, B, mm, out, false);
}

int tfhe_hip_sns_blind_rotate(tfhe_sns_ctx* c, const uint64_t* in, size_t B, uint32_t mm, uint64_t* acc_out) {
  return host_call(c, in, B, mm, acc_out, true);
}

int tfhe_hip_sns_squash_async(tfhe_sns_ctx* c, const uint64_t* d_in, size_t B, uint32_t mm, uint64_t* d_out,
                              void* stream) {
  if (!c) return fail(TFHE_HIP_EINVAL, "sns: null ctx");
  if (!c->key) return fail(TFHE_HIP_ENOKEYS, "sns: key not loaded");
  if (B == 0) return 0;
  if (!d_in || !d_out || !mm || mm > c->sp.N || (c->sp.N % mm)) return fail(TFHE_HIP_EINVAL, "sns: bad arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  int rc = ensure_lut(c, mm);
  if (rc) return rc;
  hipStream_t s = stream == TFHE_HIP_NULL_STREAM ? (hipStream_t)0 : stream ? (hipStream_t)stream : c->stream;
  return run_device(c, d_in, B, d_out, nullptr, s);
}

int tfhe_hip_sns_phase(const tfhe_sns_params* sp, const uint64_t* glwe_key, const uint64_t* cts, size_t count,
                       uint64_t* out) {
  if (!sp || !glwe_key || (count && (!cts || !out))) return fail(TFHE_HIP_EINVAL, "sns_phase: bad arguments");
  tfhe::client::sns_phase(*sp, glwe_key, cts, count, out);
  return 0;
}

}  // extern "C"
