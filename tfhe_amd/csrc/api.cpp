// api.cpp — the C ABI of libtfhe_hip.so (include/tfhe_hip.h): device context, key residency,
// launch sequencing, error reporting.  Host code; kernels live in pbs_kernels.hip.
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/tfhe_hip.h"
#include "client.h"
#include "gl64.h"
#include "pbs_kernels.h"

using tfhe::u64;
using tfhe::u32;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return fail(_e == hipErrorOutOfMemory ? TFHE_HIP_ENOMEM : TFHE_HIP_EDEVICE, "%s: %s (%s:%d)", #expr, \
                  hipGetErrorString(_e), __FILE__, __LINE__);                                  \
  } while (0)

bool params_valid(const tfhe_params* p) {
  return p && p->n > 0 && p->k > 0 && p->N >= 32 && (p->N & (p->N - 1)) == 0 && p->pbs_level > 0 &&
         p->pbs_base_log > 0 && p->pbs_base_log * p->pbs_level < 64 && p->ks_level > 0 && p->ks_base_log > 0 &&
         p->ks_base_log * p->ks_level < 64 && p->transform <= TFHE_HIP_TRANSFORM_FFT64;
}

// the device kernels of this build: P-GATE (N = 1024, PBS -> KS) and P-FHEVM (N = 2048, KS -> PBS)
bool params_on_device(const tfhe_params* p) {
  const bool gate = p->k == 1 && p->N == 1024 && p->pbs_base_log == 7 && p->pbs_level == 3 && p->ks_base_log == 2 &&
                    p->ks_level == 8 && p->order == 0;
  const bool fhevm = p->k == 1 && p->N == 2048 && p->pbs_base_log == 23 && p->pbs_level == 1 &&
                     p->ks_base_log == 4 && p->ks_level == 4 && p->order == 1;
  return gate || fhevm;
}

bool is_fft(const tfhe_params& p) { return p.transform == TFHE_HIP_TRANSFORM_FFT64; }

// canonical psi: primitive 2N-th root of unity with psi^(2N/64) = 8 (generator 7)
u64 canonical_psi(uint32_t N) {
  using namespace tfhe;
  const u64 w = gl_pow(7, (GL_P - 1) / (2ull * N));
  const u64 r = gl_pow(w, 2ull * N / 64);
  u64 k = 0, t = 1;
  for (k = 0; k < 64; k++) {
    if (t == r) break;
    t = gl_mul(t, 8);
  }
  u64 m = 1;
  while ((k * m) % 64 != 1) m += 2;
  return gl_pow(w, m);
}

}  // namespace

struct tfhe_ctx {
  tfhe_params p{};
  int device = 0;
  hipStream_t stream = nullptr;
  u64* d_bsk = nullptr;  // NTT layout, x N^-1
  u64* d_ksk = nullptr;
  void* d_ks_planes = nullptr;  // KSK recoded into 8 signed byte planes (ks_mfma.hip)
  bool ks_valu = false;         // TFHE_HIP_KS_VALU=1: the VALU keyswitch kernel instead (A/B runs)
  u64* d_tw = nullptr;  // 4 x 1024 twiddle tables of the device NTT layout
  u64 ninv = 0;
  bool keys = false;
  size_t lat_max = 1024;  // batches up to this size use the latency blind-rotate kernel
  // modulus-switch noise reduction (order 1): zeros resident in HBM
  u64* d_ms_zeros = nullptr;
  uint32_t ms_count = 0;
  double ms_bound = 0, ms_r_sigma = 0, ms_var128 = 0;
  // workspaces
  u64* d_big = nullptr;
  size_t big_cap = 0;  // u64 elements
  void* d_stage = nullptr;
  size_t stage_cap = 0;  // bytes
  void* d_ks_dig = nullptr;
  size_t ks_dig_cap = 0;  // bytes
  std::mutex mu;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev[3];  // start/stop pairs, flattened
  std::vector<hipEvent_t> ev_pool;
};

namespace {

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int grow(void** ptr, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return 0;
  if (*ptr) (void)hipFree(*ptr);
  *ptr = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(ptr, bytes));
  *cap = bytes;
  return 0;
}

hipEvent_t take_event(tfhe_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void timed_begin(tfhe_ctx* c, int which, hipStream_t s) {
  if (!c->timing) return;
  hipEvent_t e = take_event(c);
  if (e) {
    (void)hipEventRecord(e, s);
    c->ev[which].push_back(e);
  }
}
void timed_end(tfhe_ctx* c, int which, hipStream_t s) {
  if (!c->timing) return;
  if (c->ev[which].size() % 2 == 0) return;  // begin failed
  hipEvent_t e = take_event(c);
  if (e) {
    (void)hipEventRecord(e, s);
    c->ev[which].push_back(e);
  } else {
    c->ev_pool.push_back(c->ev[which].back());
    c->ev[which].pop_back();
  }
}

uint32_t io_dim(const tfhe_params& p) { return p.order == 0 ? p.n : p.k * p.N; }

hipError_t launch_br(tfhe_ctx* c, const u64* in, size_t B, const u64* luts, const u32* idx, size_t n_lut, u64* out_big,
                     u64* out_acc, hipStream_t s) {
  if (is_fft(c->p) && c->p.N == 2048)
    return tfhe::launch_blind_rotate_fft2k(in, B, (int)c->p.n, luts, idx, (int)n_lut, (const double*)c->d_bsk,
                                           (const double*)c->d_tw, out_big, out_acc, s, c->lat_max);
  if (is_fft(c->p))
    return tfhe::launch_blind_rotate_fft(in, B, (int)c->p.n, luts, idx, (int)n_lut, (const double*)c->d_bsk,
                                         (const double*)c->d_tw, out_big, out_acc, s, c->lat_max);
  if (c->p.N == 2048)
    return tfhe::launch_blind_rotate_2048(in, B, (int)c->p.n, luts, idx, (int)n_lut, c->d_bsk, c->d_tw, out_big, out_acc,
                                          s, c->lat_max);
  return tfhe::launch_blind_rotate(in, B, (int)c->p.n, luts, idx, (int)n_lut, c->d_bsk, c->d_tw, out_big, out_acc, s,
                                   c->lat_max);
}

uint32_t log2u(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) l++;
  return l;
}

hipError_t launch_ms(tfhe_ctx* c, u64* small, size_t B, int* picks, hipStream_t s) {
  return tfhe::launch_ms_reduce(small, B, (int)c->p.n, c->d_ms_zeros, (int)c->ms_count, (int)log2u(2 * c->p.N),
                                c->ms_bound, c->ms_r_sigma, c->ms_var128, picks, s);
}

hipError_t launch_ks(tfhe_ctx* c, const u64* in_big, size_t B, u64* out, hipStream_t s) {
  const int big_dim = (int)(c->p.k * c->p.N);
  if (c->ks_valu || !c->d_ks_planes)
    return tfhe::launch_keyswitch(in_big, B, big_dim, c->d_ksk, (int)c->p.n, (int)c->p.ks_base_log,
                                  (int)c->p.ks_level, out, s);
  if (grow(&c->d_ks_dig, &c->ks_dig_cap, tfhe::ks_digits_bytes(B, big_dim, (int)c->p.ks_level)))
    return hipErrorOutOfMemory;
  return tfhe::launch_keyswitch_mfma(in_big, B, big_dim, c->d_ks_planes, (int)c->p.n, (int)c->p.ks_base_log,
                                     (int)c->p.ks_level, c->d_ks_dig, out, s);
}

// PBS on device buffers (caller holds c->mu, device set).  Order 0 (P-GATE): BR + SE -> KS;
// order 1 (P-FHEVM): KS -> [MS noise reduction] -> BR + SE.  Timing slots 0 = blind rotate,
// 1 = keyswitch, 2 = modulus-switch noise reduction.
int pbs_device(tfhe_ctx* c, const u64* d_in, size_t B, const u64* d_luts, size_t n_lut, const u32* d_idx, u64* d_out,
               hipStream_t s) {
  const size_t big = (size_t)c->p.k * c->p.N + 1, small = (size_t)c->p.n + 1;
  int rc = grow((void**)&c->d_big, &c->big_cap, B * (c->p.order == 0 ? big : small) * sizeof(u64));
  if (rc) return rc;
  if (c->p.order == 0) {
    timed_begin(c, 0, s);
    HIP_TRY(launch_br(c, d_in, B, d_luts, d_idx, n_lut, c->d_big, nullptr, s));
    timed_end(c, 0, s);
    timed_begin(c, 1, s);
    HIP_TRY(launch_ks(c, c->d_big, B, d_out, s));
    timed_end(c, 1, s);
  } else {
    timed_begin(c, 1, s);
    HIP_TRY(launch_ks(c, d_in, B, c->d_big, s));
    timed_end(c, 1, s);
    if (c->ms_count) {
      timed_begin(c, 2, s);
      HIP_TRY(launch_ms(c, c->d_big, B, nullptr, s));
      timed_end(c, 2, s);
    }
    timed_begin(c, 0, s);
    HIP_TRY(launch_br(c, c->d_big, B, d_luts, d_idx, n_lut, d_out, nullptr, s));
    timed_end(c, 0, s);
  }
  return 0;
}

// Stage host buffers into one device allocation. Returns device pointers in order.
int stage(tfhe_ctx* c, std::initializer_list<std::pair<const void*, size_t>> in, std::vector<void*>& dptr,
          size_t extra_out_bytes) {
  size_t total = 0;
  std::vector<size_t> off;
  for (auto& x : in) {
    off.push_back(total);
    total += (x.second + 255) & ~(size_t)255;
  }
  const size_t out_off = total;
  total += (extra_out_bytes + 255) & ~(size_t)255;
  int rc = grow(&c->d_stage, &c->stage_cap, total ? total : 256);
  if (rc) return rc;
  size_t i = 0;
  dptr.clear();
  for (auto& x : in) {
    void* d = (char*)c->d_stage + off[i++];
    if (x.first && x.second) HIP_TRY(hipMemcpyAsync(d, x.first, x.second, hipMemcpyHostToDevice, c->stream));
    dptr.push_back(x.first ? d : nullptr);
  }
  dptr.push_back((char*)c->d_stage + out_off);
  return 0;
}

}  // namespace

// error slot shared with pks_api.cpp
int tfhe_hip_set_error(int code, const char* msg) {
  g_err = msg;
  return code;
}

extern "C" {

const char* tfhe_hip_last_error(void) { return g_err.c_str(); }

int tfhe_hip_params_preset(int preset, tfhe_params* o) {
  if (!o) return fail(TFHE_HIP_EINVAL, "null params");
  memset(o, 0, sizeof(*o));
  if (preset == TFHE_HIP_PRESET_GATE) {
    *o = tfhe_params{630, 1, 1024, 7, 3, 2, 8, -15, -25, 0, TFHE_HIP_TRANSFORM_NTT};
    return 0;
  }
  if (preset == TFHE_HIP_PRESET_FHEVM) {
    *o = tfhe_params{918, 1, 2048, 23, 1, 4, 4, -19, -47, 1, TFHE_HIP_TRANSFORM_NTT};
    return 0;
  }
  if (preset == TFHE_HIP_PRESET_GATE_FFT) {
    *o = tfhe_params{630, 1, 1024, 7, 3, 2, 8, -15, -25, 0, TFHE_HIP_TRANSFORM_FFT64};
    return 0;
  }
  if (preset == TFHE_HIP_PRESET_FHEVM_FFT) {
    *o = tfhe_params{918, 1, 2048, 23, 1, 4, 4, -19, -47, 1, TFHE_HIP_TRANSFORM_FFT64};
    return 0;
  }
  return fail(TFHE_HIP_EINVAL, "unknown preset %d", preset);
}

size_t tfhe_hip_bsk_len(const tfhe_params* p) { return p ? tfhe::client::bsk_len(*p) : 0; }
size_t tfhe_hip_ksk_len(const tfhe_params* p) { return p ? tfhe::client::ksk_len(*p) : 0; }
uint32_t tfhe_hip_io_dim(const tfhe_params* p) { return p ? io_dim(*p) : 0; }

int tfhe_hip_keygen(const tfhe_params* p, uint64_t seed, uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk,
                    uint64_t* ksk) {
  if (!params_valid(p) || !lwe_key || !glwe_key) return fail(TFHE_HIP_EINVAL, "keygen: bad arguments");
  tfhe::client::keygen(*p, seed, lwe_key, glwe_key, bsk, ksk);
  return 0;
}

int tfhe_hip_server_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, const uint64_t* glwe_key,
                           uint64_t* bsk, uint64_t* ksk) {
  if (!params_valid(p) || !lwe_key || !glwe_key) return fail(TFHE_HIP_EINVAL, "server_keygen: bad arguments");
  for (uint32_t i = 0; i < p->n; i++)
    if (lwe_key[i] > 1) return fail(TFHE_HIP_EINVAL, "server_keygen: lwe_key[%u] is not binary", i);
  for (uint32_t i = 0; i < p->k * p->N; i++)
    if (glwe_key[i] > 1) return fail(TFHE_HIP_EINVAL, "server_keygen: glwe_key[%u] is not binary", i);
  tfhe::client::server_keygen(*p, seed, lwe_key, glwe_key, bsk, ksk);
  return 0;
}

int tfhe_hip_ms_zeros_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, uint32_t count,
                             uint64_t* zeros) {
  if (!params_valid(p) || !lwe_key || (count && !zeros)) return fail(TFHE_HIP_EINVAL, "ms_zeros_keygen: bad arguments");
  tfhe::client::ms_zeros_keygen(*p, seed, lwe_key, count, zeros);
  return 0;
}

int tfhe_hip_lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, uint64_t seed, uint64_t stream0,
                         const uint64_t* msgs, size_t count, uint64_t* out) {
  if (!dim || !key || (count && (!msgs || !out))) return fail(TFHE_HIP_EINVAL, "lwe_encrypt: bad arguments");
  if (noise_log2 >= 0 || noise_log2 < -63) return fail(TFHE_HIP_EINVAL, "lwe_encrypt: noise_log2 out of range");
  tfhe::client::lwe_encrypt(dim, key, noise_log2, seed, stream0, msgs, count, out);
  return 0;
}

int tfhe_hip_lwe_phase(uint32_t dim, const uint64_t* key, const uint64_t* ct, size_t count, uint64_t* out) {
  if (!dim || !key || (count && (!ct || !out))) return fail(TFHE_HIP_EINVAL, "lwe_phase: bad arguments");
  tfhe::client::lwe_phase(dim, key, ct, count, out);
  return 0;
}

int tfhe_hip_lut_constant(uint32_t N, uint64_t v, uint64_t* lut) {
  if (!N || !lut) return fail(TFHE_HIP_EINVAL, "lut_constant: bad arguments");
  tfhe::client::lut_constant(N, v, lut);
  return 0;
}

int tfhe_hip_lut_from_table(uint32_t N, uint32_t msg_modulus, const uint64_t* table, uint64_t delta_out,
                            uint64_t* lut) {
  if (!N || !msg_modulus || msg_modulus > N || (N % msg_modulus) || !table || !lut)
    return fail(TFHE_HIP_EINVAL, "lut_from_table: bad arguments (N=%u, msg_modulus=%u)", N, msg_modulus);
  tfhe::client::lut_from_table(N, msg_modulus, table, delta_out, lut);
  return 0;
}

int tfhe_hip_create(const tfhe_params* p, int device, tfhe_ctx** out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "create: null out");
  *out = nullptr;
  if (!params_valid(p)) return fail(TFHE_HIP_EINVAL, "create: invalid parameters");
  if (!params_on_device(p))
    return fail(TFHE_HIP_EUNSUPPORTED,
                "create: device kernels of this build cover P-GATE (k=1, N=1024, PBS 7x3, KS 2x8, PBS->KS; NTT or "
                "FFT64) and P-FHEVM (k=1, N=2048, PBS 23x1, KS 4x4, KS->PBS; NTT or FFT64); got "
                "k=%u N=%u pbs %ux%u ks %ux%u order %u transform %u",
                p->k, p->N, p->pbs_base_log, p->pbs_level, p->ks_base_log, p->ks_level, p->order, p->transform);
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(TFHE_HIP_EINVAL, "create: device %d of %d", device, ndev);
  DeviceGuard g(device);
  tfhe_ctx* c = new tfhe_ctx();
  c->p = *p;
  c->device = device;
  c->lat_max = p->N == 2048 ? 512 : 1024;  // measured crossovers (tools/latency_sweep.py)
  {
    const char* e = getenv("TFHE_HIP_KS_VALU");
    c->ks_valu = e && e[0] == '1';
  }
  auto cleanup = [&](int rc) {
    tfhe_hip_destroy(c);
    return rc;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return cleanup(fail(TFHE_HIP_EDEVICE, "create: hipStreamCreate failed"));
  using namespace tfhe;
  if (is_fft(*p)) {  // FFT64: twist / pass tables (pbs_fft.hip: make_fft_tables); latency kernel at N = 1024
    // measured crossovers (tools/latency_sweep_fft.sh), 512 for both N: N = 1024 7.9 ms (latency, two
    // rounds) vs 14.8 (batch) at B = 512, 20.9 vs 14.9 at 768 (from the third round on, workgroups that
    // start staggered stream the BSK from L2 at different CMUX indices and fall out of L2); N = 2048
    // 11.3 vs 15.3 ms at 512, 18.0 vs 17.5 at 640
    c->lat_max = 512;
    std::vector<double> tw(p->N == 2048 ? fft2k_tables_len() : fft_tables_len());
    if (p->N == 2048) make_fft2k_tables(tw.data());
    else make_fft_tables(tw.data());
    if (hipMalloc(&c->d_tw, tw.size() * 8) != hipSuccess)
      return cleanup(fail(TFHE_HIP_ENOMEM, "create: twiddle allocation failed"));
    if (hipMemcpy(c->d_tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail(TFHE_HIP_EDEVICE, "create: twiddle upload failed"));
    *out = c;
    return 0;
  }
  // twiddle tables of the device NTT layout (pbs_kernels.hip: make_ntt_tables)
  const uint32_t N = p->N;
  std::vector<u64> tw(N == 2048 ? ntt2048_tables_len() : 4 * N);
  if (N == 2048) make_ntt2048_tables(canonical_psi(N), tw.data());
  else make_ntt_tables(canonical_psi(N), tw.data());
  c->ninv = gl_pow(N, GL_P - 2);
  if (hipMalloc(&c->d_tw, tw.size() * 8) != hipSuccess)
    return cleanup(fail(TFHE_HIP_ENOMEM, "create: twiddle allocation failed"));
  if (hipMemcpy(c->d_tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(TFHE_HIP_EDEVICE, "create: twiddle upload failed"));
  *out = c;
  return 0;
}

void tfhe_hip_destroy(tfhe_ctx* c) {
  if (!c) return;
  {
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int w = 0; w < 3; w++)
      for (auto e : c->ev[w]) (void)hipEventDestroy(e);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    (void)hipFree(c->d_bsk);
    (void)hipFree(c->d_ksk);
    (void)hipFree(c->d_ks_planes);
    (void)hipFree(c->d_ks_dig);
    (void)hipFree(c->d_tw);
    (void)hipFree(c->d_ms_zeros);
    (void)hipFree(c->d_big);
    (void)hipFree(c->d_stage);
    if (c->stream) (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

int tfhe_hip_device(const tfhe_ctx* c) { return c ? c->device : -1; }

static int load_keys_impl(tfhe_ctx* c, const uint64_t* bsk, size_t bsk_len, const uint64_t* ksk, size_t ksk_len,
                          hipMemcpyKind kind) {
  if (!c || !bsk || !ksk) return fail(TFHE_HIP_EINVAL, "load_keys: null argument");
  if (bsk_len != tfhe::client::bsk_len(c->p) || ksk_len != tfhe::client::ksk_len(c->p))
    return fail(TFHE_HIP_EINVAL, "load_keys: sizes %zu/%zu, expected %zu/%zu", bsk_len, ksk_len,
                tfhe::client::bsk_len(c->p), tfhe::client::ksk_len(c->p));
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  c->keys = false;
  if (!c->d_bsk) HIP_TRY(hipMalloc(&c->d_bsk, bsk_len * 8));
  if (!c->d_ksk) HIP_TRY(hipMalloc(&c->d_ksk, ksk_len * 8));
  HIP_TRY(hipMemcpyAsync(c->d_ksk, ksk, ksk_len * 8, kind, c->stream));
  if (!c->ks_valu) {  // byte planes of the KSK for the matrix-core keyswitch
    const int big_dim = (int)(c->p.k * c->p.N);
    if (!c->d_ks_planes)
      HIP_TRY(hipMalloc(&c->d_ks_planes, tfhe::ks_planes_bytes(big_dim, (int)c->p.ks_level, (int)c->p.n)));
    HIP_TRY(tfhe::launch_ksk_planes(c->d_ksk, big_dim, (int)c->p.ks_level, (int)c->p.n, c->d_ks_planes, c->stream));
  }
  // standard-domain BSK staged in the workspace, converted in one launch
  void* tmp = nullptr;
  if (kind == hipMemcpyHostToDevice) {
    int rc = grow(&c->d_stage, &c->stage_cap, bsk_len * 8);
    if (rc) return rc;
    tmp = c->d_stage;
    HIP_TRY(hipMemcpyAsync(tmp, bsk, bsk_len * 8, kind, c->stream));
  } else {
    tmp = (void*)bsk;
  }
  const size_t polys = bsk_len / c->p.N;
  if (is_fft(c->p) && c->p.N == 2048)
    HIP_TRY(tfhe::launch_bsk_to_fourier2k((const u64*)tmp, (double*)c->d_bsk, polys, (const double*)c->d_tw, c->stream));
  else if (is_fft(c->p))
    HIP_TRY(tfhe::launch_bsk_to_fourier((const u64*)tmp, (double*)c->d_bsk, polys, (const double*)c->d_tw, c->stream));
  else if (c->p.N == 2048)
    HIP_TRY(tfhe::launch_bsk_to_ntt_2048((const u64*)tmp, c->d_bsk, polys, c->d_tw, c->ninv, c->stream));
  else
    HIP_TRY(tfhe::launch_bsk_to_ntt((const u64*)tmp, c->d_bsk, (int)(polys / 12), c->d_tw, c->ninv, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->keys = true;
  return 0;
}

int tfhe_hip_load_keys(tfhe_ctx* c, const uint64_t* bsk, size_t bsk_len, const uint64_t* ksk, size_t ksk_len) {
  return load_keys_impl(c, bsk, bsk_len, ksk, ksk_len, hipMemcpyHostToDevice);
}

int tfhe_hip_load_keys_device(tfhe_ctx* c, const uint64_t* d_bsk, size_t bsk_len, const uint64_t* d_ksk,
                              size_t ksk_len) {
  return load_keys_impl(c, d_bsk, bsk_len, d_ksk, ksk_len, hipMemcpyDeviceToDevice);
}

int tfhe_hip_load_ms_key(tfhe_ctx* c, const uint64_t* zeros, uint32_t count, double bound, double r_sigma,
                         double input_variance) {
  if (!c || (count && !zeros)) return fail(TFHE_HIP_EINVAL, "load_ms_key: bad arguments");
  if (c->p.order != 1 && count)
    return fail(TFHE_HIP_EUNSUPPORTED, "load_ms_key: the noise reduction runs between keyswitch and blind rotation "
                                       "(KS -> PBS parameter sets only)");
  if (count > 0x7FFFFFFF || !(bound >= 0) || !(r_sigma >= 0) || !(input_variance >= 0))
    return fail(TFHE_HIP_EINVAL, "load_ms_key: count %u / bound / r_sigma / variance out of range", count);
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  HIP_TRY(hipStreamSynchronize(c->stream));
  (void)hipFree(c->d_ms_zeros);
  c->d_ms_zeros = nullptr;
  c->ms_count = 0;
  if (!count) return 0;
  const size_t bytes = (size_t)count * (c->p.n + 1) * 8;
  HIP_TRY(hipMalloc(&c->d_ms_zeros, bytes));
  HIP_TRY(hipMemcpy(c->d_ms_zeros, zeros, bytes, hipMemcpyHostToDevice));
  c->ms_count = count;
  c->ms_bound = bound;
  c->ms_r_sigma = r_sigma;
  c->ms_var128 = input_variance * 0x1p128;
  return 0;
}

int tfhe_hip_ms_reduce(tfhe_ctx* c, const uint64_t* in, size_t B, uint64_t* out, int32_t* picks) {
  if (!c || (B && (!in || !out))) return fail(TFHE_HIP_EINVAL, "ms_reduce: bad arguments");
  if (c->p.order != 1) return fail(TFHE_HIP_EUNSUPPORTED, "ms_reduce: KS -> PBS parameter sets only");
  if (B == 0) return 0;
  if (B > 0x7FFFFFFF) return fail(TFHE_HIP_EINVAL, "ms_reduce: batch too large");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t small = (size_t)c->p.n + 1;
  std::vector<void*> d;
  int rc = stage(c, {{in, B * small * 8}}, d, B * 4);
  if (rc) return rc;
  HIP_TRY(launch_ms(c, (u64*)d[0], B, (int*)d[1], c->stream));
  HIP_TRY(hipMemcpyAsync(out, d[0], B * small * 8, hipMemcpyDeviceToHost, c->stream));
  if (picks) HIP_TRY(hipMemcpyAsync(picks, d[1], B * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_pbs_async(tfhe_ctx* c, const uint64_t* d_in, size_t B, const uint64_t* d_luts, size_t n_lut,
                       const uint32_t* d_idx, uint64_t* d_out, void* stream) {
  if (!c) return fail(TFHE_HIP_EINVAL, "pbs: null ctx");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "pbs: keys not loaded");
  if (B == 0) return 0;
  if (!d_in || !d_luts || !n_lut || !d_out) return fail(TFHE_HIP_EINVAL, "pbs: null buffer or n_lut == 0");
  if (B > 0x7FFFFFFF) return fail(TFHE_HIP_EINVAL, "pbs: batch too large");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return pbs_device(c, d_in, B, d_luts, n_lut, d_idx, d_out, stream == TFHE_HIP_NULL_STREAM ? (hipStream_t)0 : stream ? (hipStream_t)stream : c->stream);
}

int tfhe_hip_pbs(tfhe_ctx* c, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                 const uint32_t* lut_index, uint64_t* lwe_out) {
  if (!c) return fail(TFHE_HIP_EINVAL, "pbs: null ctx");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "pbs: keys not loaded");
  if (B == 0) return 0;
  if (!lwe_in || !luts || !n_lut || !lwe_out) return fail(TFHE_HIP_EINVAL, "pbs: null buffer or n_lut == 0");
  if (lut_index)
    for (size_t q = 0; q < B; q++)
      if (lut_index[q] >= n_lut) return fail(TFHE_HIP_EINVAL, "pbs: lut_index[%zu] = %u >= n_lut %zu", q, lut_index[q], n_lut);
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t dim = io_dim(c->p) + 1;
  std::vector<void*> d;
  int rc = stage(c, {{lwe_in, B * dim * 8}, {luts, n_lut * c->p.N * 8}, {lut_index, lut_index ? B * 4 : 0}}, d,
                 B * dim * 8);
  if (rc) return rc;
  rc = pbs_device(c, (const u64*)d[0], B, (const u64*)d[1], n_lut, (const u32*)d[2], (u64*)d[3], c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(lwe_out, d[3], B * dim * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_blind_rotate(tfhe_ctx* c, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                          const uint32_t* lut_index, uint64_t* acc_out) {
  if (!c) return fail(TFHE_HIP_EINVAL, "blind_rotate: null ctx");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "blind_rotate: keys not loaded");
  if (B == 0) return 0;
  if (!lwe_in || !luts || !n_lut || !acc_out) return fail(TFHE_HIP_EINVAL, "blind_rotate: null buffer");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t din = (size_t)c->p.n + 1, acc_len = (size_t)(c->p.k + 1) * c->p.N;
  std::vector<void*> d;
  int rc = stage(c, {{lwe_in, B * din * 8}, {luts, n_lut * c->p.N * 8}, {lut_index, lut_index ? B * 4 : 0}}, d,
                 B * acc_len * 8);
  if (rc) return rc;
  HIP_TRY(launch_br(c, (const u64*)d[0], B, (const u64*)d[1], (const u32*)d[2], n_lut, nullptr, (u64*)d[3], c->stream));
  HIP_TRY(hipMemcpyAsync(acc_out, d[3], B * acc_len * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_sample_extract(tfhe_ctx* c, const uint64_t* acc, size_t B, uint64_t* out) {
  if (!c || (B && (!acc || !out))) return fail(TFHE_HIP_EINVAL, "sample_extract: bad arguments");
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t acc_len = (size_t)(c->p.k + 1) * c->p.N, big = (size_t)c->p.k * c->p.N + 1;
  std::vector<void*> d;
  int rc = stage(c, {{acc, B * acc_len * 8}}, d, B * big * 8);
  if (rc) return rc;
  if (is_fft(c->p) && c->p.N == 2048)
    HIP_TRY(tfhe::launch_sample_extract_torus2k((const u64*)d[0], B, (u64*)d[1], c->stream));
  else if (is_fft(c->p)) HIP_TRY(tfhe::launch_sample_extract_torus((const u64*)d[0], B, (u64*)d[1], c->stream));
  else if (c->p.N == 2048) HIP_TRY(tfhe::launch_sample_extract_2048((const u64*)d[0], B, (u64*)d[1], c->stream));
  else HIP_TRY(tfhe::launch_sample_extract((const u64*)d[0], B, (u64*)d[1], c->stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], B * big * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_keyswitch(tfhe_ctx* c, const uint64_t* in, size_t B, uint64_t* out) {
  if (!c || (B && (!in || !out))) return fail(TFHE_HIP_EINVAL, "keyswitch: bad arguments");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "keyswitch: keys not loaded");
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t big = (size_t)c->p.k * c->p.N + 1, small = (size_t)c->p.n + 1;
  std::vector<void*> d;
  int rc = stage(c, {{in, B * big * 8}}, d, B * small * 8);
  if (rc) return rc;
  HIP_TRY(launch_ks(c, (const u64*)d[0], B, (u64*)d[1], c->stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], B * small * 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

static int ntt_impl(tfhe_ctx* c, uint64_t* polys, size_t count, bool inverse) {
  if (!c || (count && !polys)) return fail(TFHE_HIP_EINVAL, "ntt: bad arguments");
  if (is_fft(c->p)) return fail(TFHE_HIP_EUNSUPPORTED, "ntt: this ctx runs the FFT64 transform (tfhe_hip_fft_*)");
  if (count == 0) return 0;
  for (size_t i = 0; i < count * c->p.N; i++)
    if (polys[i] >= tfhe::GL_P) return fail(TFHE_HIP_EINVAL, "ntt: value at %zu not reduced mod p", i);
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t bytes = count * c->p.N * 8;
  std::vector<void*> d;
  int rc = stage(c, {{polys, bytes}}, d, 0);
  if (rc) return rc;
  if (c->p.N == 2048) {
    if (inverse) HIP_TRY(tfhe::launch_ntt2048_inv((u64*)d[0], count, c->d_tw, c->ninv, c->stream));
    else HIP_TRY(tfhe::launch_ntt2048_fwd((u64*)d[0], count, c->d_tw, c->stream));
  } else {
    if (inverse) HIP_TRY(tfhe::launch_ntt_inv((u64*)d[0], count, c->d_tw, c->ninv, c->stream));
    else HIP_TRY(tfhe::launch_ntt_fwd((u64*)d[0], count, c->d_tw, c->stream));
  }
  HIP_TRY(hipMemcpyAsync(polys, d[0], bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_ntt_fwd(tfhe_ctx* c, uint64_t* polys, size_t count) { return ntt_impl(c, polys, count, false); }

int tfhe_hip_fft_fwd(tfhe_ctx* c, const uint64_t* polys, size_t count, double* out) {
  if (!c || (count && (!polys || !out))) return fail(TFHE_HIP_EINVAL, "fft_fwd: bad arguments");
  if (!is_fft(c->p)) return fail(TFHE_HIP_EUNSUPPORTED, "fft_fwd: ctx transform is not FFT64");
  if (count == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t bytes = count * c->p.N * 8;
  std::vector<void*> d;
  int rc = stage(c, {{polys, bytes}}, d, bytes);
  if (rc) return rc;
  if (c->p.N == 2048)
    HIP_TRY(tfhe::launch_fft2k_fwd((const u64*)d[0], count, (double*)d[1], (const double*)c->d_tw, c->stream));
  else HIP_TRY(tfhe::launch_fft_fwd((const u64*)d[0], count, (double*)d[1], (const double*)c->d_tw, c->stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_fft_inv(tfhe_ctx* c, const double* in, size_t count, double* out) {
  if (!c || (count && (!in || !out))) return fail(TFHE_HIP_EINVAL, "fft_inv: bad arguments");
  if (!is_fft(c->p)) return fail(TFHE_HIP_EUNSUPPORTED, "fft_inv: ctx transform is not FFT64");
  if (count == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  const size_t bytes = count * c->p.N * 8;
  std::vector<void*> d;
  int rc = stage(c, {{in, bytes}}, d, bytes);
  if (rc) return rc;
  if (c->p.N == 2048)
    HIP_TRY(tfhe::launch_fft2k_inv((const double*)d[0], count, (double*)d[1], (const double*)c->d_tw, c->stream));
  else HIP_TRY(tfhe::launch_fft_inv((const double*)d[0], count, (double*)d[1], (const double*)c->d_tw, c->stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], bytes, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}
int tfhe_hip_ntt_inv(tfhe_ctx* c, uint64_t* polys, size_t count) { return ntt_impl(c, polys, count, true); }

int tfhe_hip_nand(tfhe_ctx* c, const uint64_t* c1, const uint64_t* c2, size_t B, uint64_t* out) {
  if (!c || (B && (!c1 || !c2 || !out))) return fail(TFHE_HIP_EINVAL, "nand: bad arguments");
  if (c->p.order != 0) return fail(TFHE_HIP_EUNSUPPORTED, "nand: gate bootstrapping needs a PBS->KS (small-key) parameter set");
  if (B == 0) return 0;
  const size_t dim = (size_t)c->p.n + 1;
  std::vector<u64> in(B * dim), lut(c->p.N);
  const u64 mu = 1ull << 61;  // 1/8
  for (size_t q = 0; q < B; q++) {
    for (size_t i = 0; i + 1 < dim; i++) in[q * dim + i] = 0 - c1[q * dim + i] - c2[q * dim + i];
    in[q * dim + dim - 1] = mu - c1[q * dim + dim - 1] - c2[q * dim + dim - 1];
  }
  tfhe::client::lut_constant(c->p.N, mu, lut.data());
  return tfhe_hip_pbs(c, in.data(), B, lut.data(), 1, nullptr, out);
}

int tfhe_hip_set_latency_batch(tfhe_ctx* c, size_t max_batch) {
  if (!c) return fail(TFHE_HIP_EINVAL, "set_latency_batch: null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->lat_max = max_batch;
  return 0;
}

int tfhe_hip_sync(tfhe_ctx* c) {
  if (!c) return fail(TFHE_HIP_EINVAL, "sync: null ctx");
  DeviceGuard g(c->device);
  HIP_TRY(hipStreamSynchronize(c->stream));
  return 0;
}

int tfhe_hip_timing_enable(tfhe_ctx* c, int enable) {
  if (!c) return fail(TFHE_HIP_EINVAL, "timing: null ctx");
  c->timing = enable != 0;
  return 0;
}

int tfhe_hip_timing_reset(tfhe_ctx* c) {
  if (!c) return fail(TFHE_HIP_EINVAL, "timing: null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  for (int w = 0; w < 3; w++) {
    for (auto e : c->ev[w]) c->ev_pool.push_back(e);
    c->ev[w].clear();
  }
  return 0;
}

int tfhe_hip_timing_stats(tfhe_ctx* c, int which, double* total_ms, int* launches) {
  if (!c || which < 0 || which > 2 || !total_ms || !launches) return fail(TFHE_HIP_EINVAL, "timing: bad arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  double tot = 0;
  int cnt = 0;
  auto& v = c->ev[which];
  for (size_t i = 0; i + 1 < v.size(); i += 2) {
    HIP_TRY(hipEventSynchronize(v[i + 1]));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, v[i], v[i + 1]));
    tot += ms;
    cnt++;
  }
  *total_ms = tot;
  *launches = cnt;
  return 0;
}

}  // extern "C"
