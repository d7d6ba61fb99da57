// api.cpp — the C ABI of libtfhe_hip.so (include/tfhe_hip.h): device shards, key residency and
// broadcast, launch sequencing, error reporting.  Host code; kernels live in the .hip files.
//
// An engine (tfhe_ctx) spans ndev device shards.  A shard = one device ordinal + its own stream,
// key copy, twiddle tables and workspaces.  Keys reach shard 0 through a pinned staging ring and the
// other shards by RCCL broadcast (distinct ordinals) or device copies (a repeated ordinal); host-buffer
// PBS batches split into contiguous slices that the shards run concurrently.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tfhe_hip.h"
#include "client.h"
#include "gl64.h"
#include "pbs_kernels.h"

using tfhe::u32;
using tfhe::u64;

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

#define RC_TRY(expr)      \
  do {                    \
    int _rc = (expr);     \
    if (_rc) return _rc;  \
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

// ---- RCCL, loaded on first use (a process that already holds torch's librccl reuses that copy) -----------
struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*bcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*err)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  static std::mutex m;
  std::lock_guard<std::mutex> lk(m);
  if (r.tried) return r;
  r.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    r.why = std::string("dlopen librccl.so.1: ") + dlerror();
    return r;
  }
  r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
  r.bcast = (decltype(r.bcast))dlsym(h, "ncclBroadcast");
  r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
  r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
  r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
  r.err = (decltype(r.err))dlsym(h, "ncclGetErrorString");
  r.ok = r.comm_init_all && r.bcast && r.group_start && r.group_end && r.comm_destroy && r.err;
  if (!r.ok) r.why = "librccl.so.1 lacks ncclCommInitAll / ncclBroadcast / ncclGroupStart / ncclGroupEnd";
  return r;
}

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

}  // namespace

// One device's slice of an engine.
struct tfhe_shard {
  int device = 0;
  hipStream_t stream = nullptr;
  u64* d_bsk = nullptr;         // transform domain (NTT layout x N^-1, or Fourier)
  u64* d_ksk = nullptr;         // standard KSK (VALU keyswitch; RCCL broadcast source / target)
  void* d_ks_planes = nullptr;  // KSK recoded into 8 signed byte planes (ks_mfma.hip)
  u64* d_tw = nullptr;          // twiddle tables of the device transform
  u64* d_ms_zeros = nullptr;    // modulus-switch noise reduction zeros (order 1)
  // workspaces: every user waits for `ws_free` (the previous user's completion) on its own stream
  u64* d_big = nullptr;
  size_t big_cap = 0;  // bytes
  void* d_stage = nullptr;
  size_t stage_cap = 0;  // bytes
  void* d_ks_dig = nullptr;
  size_t ks_dig_cap = 0;  // bytes
  hipEvent_t ws_free = nullptr;
  hipStream_t ws_last = nullptr;
  bool ws_used = false;
  // timing: start/stop event pairs per slot (0 = blind rotate, 1 = keyswitch, 2 = MS noise reduction)
  std::vector<hipEvent_t> ev[3];
  std::vector<hipEvent_t> ev_pool;
};

struct tfhe_ctx {
  tfhe_params p{};
  std::vector<tfhe_shard> sh;
  bool keys = false;
  bool ks_valu = false;  // TFHE_HIP_KS_VALU=1: the VALU keyswitch kernel instead (A/B runs)
  size_t lat_max = 1024; // batches up to this size (per shard) use the latency blind-rotate kernel
  u64 ninv = 0;
  uint32_t ms_count = 0;
  double ms_bound = 0, ms_r_sigma = 0, ms_var128 = 0;
  int bcast_mode = 0;  // tfhe_hip_key_bcast_mode
  std::vector<ncclComm_t> comms;
  std::mutex mu;
  bool timing = false;
};

namespace {

using shard = tfhe_shard;

int grow(shard& s, void** ptr, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return 0;
  if (s.ws_used) HIP_TRY(hipEventSynchronize(s.ws_free));  // no launch may still read the old buffer
  if (*ptr) (void)hipFree(*ptr);
  *ptr = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(ptr, bytes));
  *cap = bytes;
  return 0;
}

// Workspace ordering across streams (tfhe_hip_pbs_async may be called on any stream): the stream that
// uses the shard's workspaces next waits for the event recorded after the previous use.
int ws_begin(shard& s, hipStream_t st) {
  if (s.ws_used && s.ws_last != st) HIP_TRY(hipStreamWaitEvent(st, s.ws_free, 0));
  return 0;
}
int ws_end(shard& s, hipStream_t st) {
  HIP_TRY(hipEventRecord(s.ws_free, st));
  s.ws_last = st;
  s.ws_used = true;
  return 0;
}

hipEvent_t take_event(shard& s) {
  if (!s.ev_pool.empty()) {
    hipEvent_t e = s.ev_pool.back();
    s.ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void timed_begin(tfhe_ctx* c, shard& s, int which, hipStream_t st) {
  if (!c->timing) return;
  hipEvent_t e = take_event(s);
  if (e) {
    (void)hipEventRecord(e, st);
    s.ev[which].push_back(e);
  }
}
void timed_end(tfhe_ctx* c, shard& s, int which, hipStream_t st) {
  if (!c->timing) return;
  if (s.ev[which].size() % 2 == 0) return;  // begin failed
  hipEvent_t e = take_event(s);
  if (e) {
    (void)hipEventRecord(e, st);
    s.ev[which].push_back(e);
  } else {
    s.ev_pool.push_back(s.ev[which].back());
    s.ev[which].pop_back();
  }
}

uint32_t io_dim(const tfhe_params& p) { return p.order == 0 ? p.n : p.k * p.N; }

hipError_t launch_br(tfhe_ctx* c, shard& s, const u64* in, size_t B, const u64* luts, const u32* idx, size_t n_lut,
                     u64* out_big, u64* out_acc, hipStream_t st) {
  if (is_fft(c->p) && c->p.N == 2048)
    return tfhe::launch_blind_rotate_fft2k(in, B, (int)c->p.n, luts, idx, (int)n_lut, (const double*)s.d_bsk,
                                           (const double*)s.d_tw, out_big, out_acc, st, c->lat_max);
  if (is_fft(c->p))
    return tfhe::launch_blind_rotate_fft(in, B, (int)c->p.n, luts, idx, (int)n_lut, (const double*)s.d_bsk,
                                         (const double*)s.d_tw, out_big, out_acc, st, c->lat_max);
  if (c->p.N == 2048)
    return tfhe::launch_blind_rotate_2048(in, B, (int)c->p.n, luts, idx, (int)n_lut, s.d_bsk, s.d_tw, out_big, out_acc,
                                          st, c->lat_max);
  return tfhe::launch_blind_rotate(in, B, (int)c->p.n, luts, idx, (int)n_lut, s.d_bsk, s.d_tw, out_big, out_acc, st,
                                   c->lat_max);
}

uint32_t log2u(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) l++;
  return l;
}

hipError_t launch_ms(tfhe_ctx* c, shard& s, u64* small, size_t B, int* picks, hipStream_t st) {
  return tfhe::launch_ms_reduce(small, B, (int)c->p.n, s.d_ms_zeros, (int)c->ms_count, (int)log2u(2 * c->p.N),
                                c->ms_bound, c->ms_r_sigma, c->ms_var128, picks, st);
}

int launch_ks(tfhe_ctx* c, shard& s, const u64* in_big, size_t B, u64* out, hipStream_t st) {
  const int big_dim = (int)(c->p.k * c->p.N);
  if (c->ks_valu || !s.d_ks_planes) {
    HIP_TRY(tfhe::launch_keyswitch(in_big, B, big_dim, s.d_ksk, (int)c->p.n, (int)c->p.ks_base_log,
                                   (int)c->p.ks_level, out, st));
    return 0;
  }
  RC_TRY(grow(s, &s.d_ks_dig, &s.ks_dig_cap, tfhe::ks_digits_bytes(B, big_dim, (int)c->p.ks_level)));
  HIP_TRY(tfhe::launch_keyswitch_mfma(in_big, B, big_dim, s.d_ks_planes, (int)c->p.n, (int)c->p.ks_base_log,
                                      (int)c->p.ks_level, s.d_ks_dig, out, st));
  return 0;
}

// PBS on device buffers (caller holds c->mu and has set the shard's device; workspaces ordered by the
// caller's ws_begin / ws_end).  Order 0 (P-GATE): BR + SE -> KS; order 1 (P-FHEVM): KS -> [MS noise
// reduction] -> BR + SE.
int pbs_device(tfhe_ctx* c, shard& s, const u64* d_in, size_t B, const u64* d_luts, size_t n_lut, const u32* d_idx,
               u64* d_out, hipStream_t st) {
  const size_t big = (size_t)c->p.k * c->p.N + 1, small = (size_t)c->p.n + 1;
  RC_TRY(grow(s, (void**)&s.d_big, &s.big_cap, B * (c->p.order == 0 ? big : small) * sizeof(u64)));
  if (c->p.order == 0) {
    timed_begin(c, s, 0, st);
    HIP_TRY(launch_br(c, s, d_in, B, d_luts, d_idx, n_lut, s.d_big, nullptr, st));
    timed_end(c, s, 0, st);
    timed_begin(c, s, 1, st);
    RC_TRY(launch_ks(c, s, s.d_big, B, d_out, st));
    timed_end(c, s, 1, st);
  } else {
    timed_begin(c, s, 1, st);
    RC_TRY(launch_ks(c, s, d_in, B, s.d_big, st));
    timed_end(c, s, 1, st);
    if (c->ms_count) {
      timed_begin(c, s, 2, st);
      HIP_TRY(launch_ms(c, s, s.d_big, B, nullptr, st));
      timed_end(c, s, 2, st);
    }
    timed_begin(c, s, 0, st);
    HIP_TRY(launch_br(c, s, s.d_big, B, d_luts, d_idx, n_lut, d_out, nullptr, st));
    timed_end(c, s, 0, st);
  }
  return 0;
}

// Stage host buffers into the shard's staging allocation (on the shard stream).  Returns device pointers
// in order, plus one for `extra_out_bytes` of output.
int stage(shard& s, std::initializer_list<std::pair<const void*, size_t>> in, std::vector<void*>& dptr,
          size_t extra_out_bytes) {
  size_t total = 0;
  std::vector<size_t> off;
  for (auto& x : in) {
    off.push_back(total);
    total += (x.second + 255) & ~(size_t)255;
  }
  const size_t out_off = total;
  total += (extra_out_bytes + 255) & ~(size_t)255;
  RC_TRY(grow(s, &s.d_stage, &s.stage_cap, total ? total : 256));
  size_t i = 0;
  dptr.clear();
  for (auto& x : in) {
    void* d = (char*)s.d_stage + off[i++];
    if (x.first && x.second) HIP_TRY(hipMemcpyAsync(d, x.first, x.second, hipMemcpyHostToDevice, s.stream));
    dptr.push_back(x.first ? d : nullptr);
  }
  dptr.push_back((char*)s.d_stage + out_off);
  return 0;
}

// Host -> device copy through a pinned staging ring (2 x 16 MB): the CPU fills one slot while the DMA
// engine drains the other.  Pageable sources would otherwise go through the runtime's own bounce buffer
// one synchronous piece at a time.
int upload_pinned(shard& s, void* dst, const void* src, size_t bytes) {
  const size_t slot = 16u << 20;
  void* ring[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  int rc = 0;
  auto cleanup = [&]() {
    for (int i = 0; i < 2; i++) {
      if (done[i]) (void)hipEventDestroy(done[i]);
      if (ring[i]) (void)hipHostFree(ring[i]);
    }
  };
  for (int i = 0; i < 2 && !rc; i++) {
    if (hipHostMalloc(&ring[i], slot, hipHostMallocDefault) != hipSuccess) rc = fail(TFHE_HIP_ENOMEM, "pinned staging alloc");
    else if (hipEventCreateWithFlags(&done[i], hipEventDisableTiming) != hipSuccess) rc = fail(TFHE_HIP_EDEVICE, "event");
  }
  bool used[2] = {false, false};
  for (size_t off = 0, k = 0; off < bytes && !rc; off += slot, k ^= 1) {
    const size_t n = std::min(slot, bytes - off);
    if (used[k] && hipEventSynchronize(done[k]) != hipSuccess) rc = fail(TFHE_HIP_EDEVICE, "staging sync");
    if (rc) break;
    memcpy(ring[k], (const char*)src + off, n);
    if (hipMemcpyAsync((char*)dst + off, ring[k], n, hipMemcpyHostToDevice, s.stream) != hipSuccess ||
        hipEventRecord(done[k], s.stream) != hipSuccess)
      rc = fail(TFHE_HIP_EDEVICE, "staged upload failed");
    used[k] = true;
  }
  if (hipStreamSynchronize(s.stream) != hipSuccess && !rc) rc = fail(TFHE_HIP_EDEVICE, "staged upload sync");
  cleanup();
  return rc;
}

bool devices_distinct(const tfhe_ctx* c) {
  for (size_t i = 0; i < c->sh.size(); i++)
    for (size_t j = i + 1; j < c->sh.size(); j++)
      if (c->sh[i].device == c->sh[j].device) return false;
  return true;
}

// Broadcast planner (tfhe_hip_bcast_plan): which replication the key load takes and the per-rank call list.
//   policy "rccl": RCCL even for one device (the plumbing test); "copy": device / peer copies; NULL or "" = auto:
//   RCCL when the ordinals are distinct and librccl loads, device / peer copies otherwise (a repeated ordinal, or
//   no RCCL: hipMemcpyPeerAsync reaches every xGMI peer without it).
//   mode 2: calls[i] = rank i's ncclBroadcast inside ONE ncclGroupStart / ncclGroupEnd, root 0 (sends in place)
//   first, every rank on its own communicator member and stream; mode 1: calls[i - 1] = destination shard i of
//   copy i from shard 0; mode 0: nothing to do.  Returns the call count or a negative error.
int bcast_plan(const int* devices, int ndev, const char* policy, bool rccl_ok, int* mode, int* calls, int max_calls,
               std::string* why) {
  const bool forced = policy && strcmp(policy, "rccl") == 0;
  const bool copy = policy && strcmp(policy, "copy") == 0;
  if (policy && *policy && !forced && !copy) {
    if (why) *why = std::string("unknown broadcast policy '") + policy + "' (rccl | copy)";
    return TFHE_HIP_EINVAL;
  }
  bool distinct = true;
  for (int i = 0; i < ndev; i++)
    for (int j = i + 1; j < ndev; j++)
      if (devices[i] == devices[j]) distinct = false;
  *mode = 0;
  if (ndev < 2 && !forced) return 0;
  if (forced) {
    if (!distinct) {
      if (why) *why = "RCCL broadcast needs distinct device ordinals";
      return TFHE_HIP_EINVAL;
    }
    if (!rccl_ok) {
      if (why) *why = "RCCL forced but unavailable";
      return TFHE_HIP_EDEVICE;
    }
  }
  const bool use_rccl = forced || (!copy && distinct && rccl_ok);
  const int n = use_rccl ? ndev : ndev - 1;
  if (calls && n > max_calls) {
    if (why) *why = "call list too small";
    return TFHE_HIP_EINVAL;
  }
  for (int i = 0; calls && i < n; i++) calls[i] = use_rccl ? i : i + 1;
  *mode = use_rccl ? 2 : 1;
  return n;
}

// Broadcast `count` u64 from src (on shard 0's device) into dst[i] of every shard i >= 1, as planned above.
int broadcast(tfhe_ctx* c, const u64* src, const std::vector<u64*>& dst, size_t count) {
  const int nd = (int)c->sh.size();
  const char* env = getenv("TFHE_HIP_BCAST");
  std::vector<int> devs(nd), calls(nd);
  for (int i = 0; i < nd; i++) devs[i] = c->sh[i].device;
  bool distinct = true;
  for (int i = 0; i < nd; i++)
    for (int j = i + 1; j < nd; j++) distinct = distinct && devs[i] != devs[j];
  // librccl is only probed when the plan could use it
  const bool want = (env && strcmp(env, "rccl") == 0) || (nd > 1 && distinct && !(env && strcmp(env, "copy") == 0));
  Rccl* R = want ? &rccl() : nullptr;
  int mode = 0;
  std::string why;
  const int ncalls = bcast_plan(devs.data(), nd, env, R && R->ok, &mode, calls.data(), nd, &why);
  if (ncalls < 0)
    return fail(ncalls, "key broadcast: %s%s%s", why.c_str(), R && !R->ok ? ": " : "", R && !R->ok ? R->why.c_str() : "");
  if (mode == 2) {
    if (c->comms.empty()) {
      c->comms.assign(nd, nullptr);
      const ncclResult_t r = R->comm_init_all(c->comms.data(), nd, devs.data());
      if (r != ncclSuccess) {
        c->comms.clear();
        return fail(TFHE_HIP_EDEVICE, "ncclCommInitAll: %s", R->err(r));
      }
    }
    R->group_start();
    ncclResult_t r = ncclSuccess;
    for (int k = 0; k < ncalls && r == ncclSuccess; k++) {
      const int i = calls[k];
      DeviceGuard g(c->sh[i].device);
      r = R->bcast(i == 0 ? (const void*)src : (const void*)dst[i], i == 0 ? (void*)src : (void*)dst[i], count,
                   ncclUint64, 0, c->comms[i], c->sh[i].stream);
    }
    const ncclResult_t r2 = R->group_end();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(TFHE_HIP_EDEVICE, "ncclBroadcast: %s", R->err(r != ncclSuccess ? r : r2));
    for (int i = 0; i < nd; i++) {
      DeviceGuard g(c->sh[i].device);
      HIP_TRY(hipStreamSynchronize(c->sh[i].stream));
    }
    c->bcast_mode = 2;
    return 0;
  }
  if (mode == 0) return 0;
  for (int k = 0; k < ncalls; k++) {
    shard& s = c->sh[calls[k]];
    DeviceGuard g(s.device);
    if (s.device == c->sh[0].device)
      HIP_TRY(hipMemcpyAsync(dst[calls[k]], src, count * 8, hipMemcpyDeviceToDevice, s.stream));
    else
      HIP_TRY(hipMemcpyPeerAsync(dst[calls[k]], s.device, src, c->sh[0].device, count * 8, s.stream));
    HIP_TRY(hipStreamSynchronize(s.stream));
  }
  c->bcast_mode = 1;
  return 0;
}

// Convert a standard-domain BSK at `std_bsk` (on the shard's device) to the transform domain and the KSK
// at s.d_ksk to byte planes.
int convert_keys(tfhe_ctx* c, shard& s, const u64* std_bsk, size_t bsk_len) {
  const size_t polys = bsk_len / c->p.N;
  DeviceGuard g(s.device);
  if (!c->ks_valu) {
    const int big_dim = (int)(c->p.k * c->p.N);
    if (!s.d_ks_planes)
      HIP_TRY(hipMalloc(&s.d_ks_planes, tfhe::ks_planes_bytes(big_dim, (int)c->p.ks_level, (int)c->p.n)));
    HIP_TRY(tfhe::launch_ksk_planes(s.d_ksk, big_dim, (int)c->p.ks_level, (int)c->p.n, s.d_ks_planes, s.stream));
  }
  if (is_fft(c->p) && c->p.N == 2048)
    HIP_TRY(tfhe::launch_bsk_to_fourier2k(std_bsk, (double*)s.d_bsk, polys, (const double*)s.d_tw, s.stream));
  else if (is_fft(c->p))
    HIP_TRY(tfhe::launch_bsk_to_fourier(std_bsk, (double*)s.d_bsk, polys, (const double*)s.d_tw, s.stream));
  else if (c->p.N == 2048)
    HIP_TRY(tfhe::launch_bsk_to_ntt_2048(std_bsk, s.d_bsk, polys, s.d_tw, c->ninv, s.stream));
  else
    HIP_TRY(tfhe::launch_bsk_to_ntt(std_bsk, s.d_bsk, (int)(polys / 12), s.d_tw, c->ninv, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

int shard_init(tfhe_ctx* c, shard& s) {
  DeviceGuard g(s.device);
  HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&s.ws_free, hipEventDisableTiming));
  const tfhe_params& p = c->p;
  using namespace tfhe;
  if (is_fft(p)) {  // FFT64: twist / pass tables (pbs_fft.hip: make_fft_tables)
    std::vector<double> tw(p.N == 2048 ? fft2k_tables_len() : fft_tables_len());
    if (p.N == 2048) make_fft2k_tables(tw.data());
    else make_fft_tables(tw.data());
    if (!fft_slot_constants_ok() || !fft2k_slot_constants_ok())
      return fail(TFHE_HIP_EUNSUPPORTED, "FFT64: compile-time twist constants differ from the host tables");
    HIP_TRY(hipMalloc(&s.d_tw, tw.size() * 8));
    HIP_TRY(hipMemcpy(s.d_tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
    return 0;
  }
  // twiddle tables of the device NTT layout (pbs_kernels.hip: make_ntt_tables)
  std::vector<u64> tw(p.N == 2048 ? ntt2048_tables_len() : 4 * p.N);
  if (p.N == 2048) make_ntt2048_tables(canonical_psi(p.N), tw.data());
  else make_ntt_tables(canonical_psi(p.N), tw.data());
  HIP_TRY(hipMalloc(&s.d_tw, tw.size() * 8));
  HIP_TRY(hipMemcpy(s.d_tw, tw.data(), tw.size() * 8, hipMemcpyHostToDevice));
  return 0;
}

void shard_free(shard& s) {
  DeviceGuard g(s.device);
  if (s.stream) (void)hipStreamSynchronize(s.stream);
  for (int w = 0; w < 3; w++)
    for (auto e : s.ev[w]) (void)hipEventDestroy(e);
  for (auto e : s.ev_pool) (void)hipEventDestroy(e);
  (void)hipFree(s.d_bsk);
  (void)hipFree(s.d_ksk);
  (void)hipFree(s.d_ks_planes);
  (void)hipFree(s.d_ks_dig);
  (void)hipFree(s.d_tw);
  (void)hipFree(s.d_ms_zeros);
  (void)hipFree(s.d_big);
  (void)hipFree(s.d_stage);
  if (s.ws_free) (void)hipEventDestroy(s.ws_free);
  if (s.stream) (void)hipStreamDestroy(s.stream);
}

// Run fn(shard index, lo, hi) for contiguous slices of [0, B) on every shard concurrently (one host
// thread per shard beyond the first); the first error (with its message) is returned on this thread.
template <class F>
int for_each_slice(tfhe_ctx* c, size_t B, F&& fn) {
  const size_t nd = c->sh.size();
  std::vector<int> rc(nd, 0);
  std::vector<std::string> msg(nd);
  auto run = [&](size_t i) {
    const size_t lo = B * i / nd, hi = B * (i + 1) / nd;
    if (lo == hi) return;
    DeviceGuard g(c->sh[i].device);
    rc[i] = fn(i, lo, hi);
    if (rc[i]) msg[i] = g_err;
  };
  if (nd == 1) {
    run(0);
    return rc[0];
  }
  std::vector<std::thread> th;
  for (size_t i = 1; i < nd; i++) th.emplace_back(run, i);
  run(0);
  for (auto& t : th) t.join();
  for (size_t i = 0; i < nd; i++)
    if (rc[i]) {
      g_err = "shard " + std::to_string(i) + " (device " + std::to_string(c->sh[i].device) + "): " + msg[i];
      return rc[i];
    }
  return 0;
}

}  // namespace


// error slot shared with pks_api.cpp / sns_api.cpp
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

int tfhe_hip_rng_key_entropy(tfhe_rng_key* out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "rng_key_entropy: null out");
  if (!tfhe::client::rng_key_entropy(out)) return fail(TFHE_HIP_EDEVICE, "rng_key_entropy: getrandom failed");
  return 0;
}

int tfhe_hip_rng_key_from_seed(uint64_t seed, tfhe_rng_key* out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "rng_key_from_seed: null out");
  *out = tfhe::client::rng_key_from_seed(seed);
  return 0;
}

static int check_binary(const uint64_t* key, size_t len, const char* what) {
  for (size_t i = 0; i < len; i++)
    if (key[i] > 1) return fail(TFHE_HIP_EINVAL, "%s[%zu] is not binary", what, i);
  return 0;
}

int tfhe_hip_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, uint64_t* lwe_key, uint64_t* glwe_key,
                      uint64_t* bsk, uint64_t* ksk) {
  if (!params_valid(p) || !rk || !lwe_key || !glwe_key) return fail(TFHE_HIP_EINVAL, "keygen: bad arguments");
  tfhe::client::keygen(*p, *rk, lwe_key, glwe_key, bsk, ksk);
  return 0;
}

int tfhe_hip_keygen(const tfhe_params* p, uint64_t seed, uint64_t* lwe_key, uint64_t* glwe_key, uint64_t* bsk,
                    uint64_t* ksk) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_keygen_k(p, &rk, lwe_key, glwe_key, bsk, ksk);
}

int tfhe_hip_server_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t* lwe_key,
                             const uint64_t* glwe_key, uint64_t* bsk, uint64_t* ksk) {
  if (!params_valid(p) || !rk || !lwe_key || !glwe_key) return fail(TFHE_HIP_EINVAL, "server_keygen: bad arguments");
  RC_TRY(check_binary(lwe_key, p->n, "server_keygen: lwe_key"));
  RC_TRY(check_binary(glwe_key, (size_t)p->k * p->N, "server_keygen: glwe_key"));
  tfhe::client::server_keygen(*p, *rk, lwe_key, glwe_key, bsk, ksk);
  return 0;
}

int tfhe_hip_server_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, const uint64_t* glwe_key,
                           uint64_t* bsk, uint64_t* ksk) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_server_keygen_k(p, &rk, lwe_key, glwe_key, bsk, ksk);
}

int tfhe_hip_ms_zeros_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t* lwe_key, uint32_t count,
                               uint64_t* zeros) {
  if (!params_valid(p) || !rk || !lwe_key || (count && !zeros))
    return fail(TFHE_HIP_EINVAL, "ms_zeros_keygen: bad arguments");
  tfhe::client::ms_zeros_keygen(*p, *rk, lwe_key, count, zeros);
  return 0;
}

// ---- compressed (seeded) server keys (seeded.cpp)
static bool native_torus(const tfhe_params* p) { return params_valid(p) && p->transform == TFHE_HIP_TRANSFORM_FFT64; }

int tfhe_hip_aes128_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
  if (!key || !in || !out) return fail(TFHE_HIP_EINVAL, "aes128_block: null argument");
  tfhe::seeded::aes128_block(key, in, out);
  return 0;
}

int tfhe_hip_csprng_words(const uint64_t seed[2], uint64_t first_word, size_t count, uint64_t* out) {
  if (!seed || (count && !out)) return fail(TFHE_HIP_EINVAL, "csprng_words: null argument");
  tfhe::seeded::csprng_words(seed, first_word, count, out);
  return 0;
}

int tfhe_hip_seeded_server_keygen_k(const tfhe_params* p, const tfhe_rng_key* rk, const uint64_t bsk_seed[2],
                                    const uint64_t ksk_seed[2], const uint64_t* lwe_key, const uint64_t* glwe_key,
                                    uint64_t* bsk_bodies, uint64_t* ksk_bodies) {
  if (!native_torus(p) || !rk || !lwe_key || !glwe_key || (bsk_bodies && !bsk_seed) || (ksk_bodies && !ksk_seed))
    return fail(TFHE_HIP_EINVAL, "seeded_server_keygen: bad arguments (FFT64 presets only)");
  RC_TRY(check_binary(lwe_key, p->n, "seeded_server_keygen: lwe_key"));
  RC_TRY(check_binary(glwe_key, (size_t)p->k * p->N, "seeded_server_keygen: glwe_key"));
  tfhe::seeded::seeded_server_keygen(*p, *rk, bsk_seed, ksk_seed, lwe_key, glwe_key, bsk_bodies, ksk_bodies);
  return 0;
}

int tfhe_hip_seeded_lwe_list_k(uint32_t dim, uint32_t count, const uint64_t* key, int32_t noise_log2,
                               const tfhe_rng_key* rk, uint64_t stream0, const uint64_t seed[2], const uint64_t* msgs,
                               uint64_t* bodies) {
  if (!dim || !key || !rk || !seed || (count && !bodies)) return fail(TFHE_HIP_EINVAL, "seeded_lwe_list: bad arguments");
  RC_TRY(check_binary(key, dim, "seeded_lwe_list: key"));
  tfhe::seeded::seeded_lwe_list(dim, count, key, noise_log2, *rk, stream0, seed, msgs, bodies);
  return 0;
}

int tfhe_hip_decompress_bsk(const tfhe_params* p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* bsk) {
  if (!native_torus(p) || !seed || !bodies || !bsk)
    return fail(TFHE_HIP_EINVAL, "decompress_bsk: bad arguments (FFT64 presets only)");
  tfhe::seeded::decompress_bsk(*p, seed, bodies, bsk);
  return 0;
}

int tfhe_hip_decompress_ksk(const tfhe_params* p, const uint64_t seed[2], const uint64_t* bodies, uint64_t* ksk) {
  if (!native_torus(p) || !seed || !bodies || !ksk)
    return fail(TFHE_HIP_EINVAL, "decompress_ksk: bad arguments (FFT64 presets only)");
  tfhe::seeded::decompress_ksk(*p, seed, bodies, ksk);
  return 0;
}

int tfhe_hip_decompress_lwe_list(uint32_t dim, uint32_t count, const uint64_t seed[2], const uint64_t* bodies,
                                 uint64_t* out) {
  if (!dim || !seed || (count && (!bodies || !out))) return fail(TFHE_HIP_EINVAL, "decompress_lwe_list: bad arguments");
  tfhe::seeded::decompress_lwe_list(dim, count, seed, bodies, out);
  return 0;
}

int tfhe_hip_ms_zeros_keygen(const tfhe_params* p, uint64_t seed, const uint64_t* lwe_key, uint32_t count,
                             uint64_t* zeros) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_ms_zeros_keygen_k(p, &rk, lwe_key, count, zeros);
}

int tfhe_hip_lwe_encrypt_k(uint32_t dim, const uint64_t* key, int32_t noise_log2, const tfhe_rng_key* rk,
                           uint64_t stream0, const uint64_t* msgs, size_t count, uint64_t* out) {
  if (!dim || !key || !rk || (count && (!msgs || !out))) return fail(TFHE_HIP_EINVAL, "lwe_encrypt: bad arguments");
  if (noise_log2 >= 0 || noise_log2 < -63) return fail(TFHE_HIP_EINVAL, "lwe_encrypt: noise_log2 out of range");
  tfhe::client::lwe_encrypt(dim, key, noise_log2, *rk, stream0, msgs, count, out);
  return 0;
}

int tfhe_hip_lwe_encrypt(uint32_t dim, const uint64_t* key, int32_t noise_log2, uint64_t seed, uint64_t stream0,
                         const uint64_t* msgs, size_t count, uint64_t* out) {
  const tfhe_rng_key rk = tfhe::client::rng_key_from_seed(seed);
  return tfhe_hip_lwe_encrypt_k(dim, key, noise_log2, &rk, stream0, msgs, count, out);
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

int tfhe_hip_create(const tfhe_params* p, const int* devices, int ndev, tfhe_ctx** out) {
  if (!out) return fail(TFHE_HIP_EINVAL, "create: null out");
  *out = nullptr;
  if (!params_valid(p)) return fail(TFHE_HIP_EINVAL, "create: invalid parameters");
  if (!params_on_device(p))
    return fail(TFHE_HIP_EUNSUPPORTED,
                "create: device kernels of this build cover P-GATE (k=1, N=1024, PBS 7x3, KS 2x8, PBS->KS; NTT or "
                "FFT64) and P-FHEVM (k=1, N=2048, PBS 23x1, KS 4x4, KS->PBS; NTT or FFT64); got "
                "k=%u N=%u pbs %ux%u ks %ux%u order %u transform %u",
                p->k, p->N, p->pbs_base_log, p->pbs_level, p->ks_base_log, p->ks_level, p->order, p->transform);
  if (!devices || ndev < 1 || ndev > 64) return fail(TFHE_HIP_EINVAL, "create: need 1..64 device ordinals, got %d", ndev);
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  for (int i = 0; i < ndev; i++)
    if (devices[i] < 0 || devices[i] >= count)
      return fail(TFHE_HIP_EINVAL, "create: device %d of %d (devices[%d])", devices[i], count, i);
  std::unique_ptr<tfhe_ctx> c(new tfhe_ctx());
  c->p = *p;
  // measured latency-kernel crossovers (tools/latency_sweep.py, tools/latency_sweep_fft.sh): NTT engine
  // 1024 (N = 1024) / 512 (N = 2048); FFT64 512 for both N (from the third round of latency workgroups
  // on, workgroups that start staggered stream the BSK from L2 at different CMUX indices)
  // round 3: the P-GATE FFT64 component-pair batch kernel runs any batch up to 1024 in one 6.7 ms round, the
  // latency kernel 3.5-3.7 ms up to 256 and 7.1 ms from 257 (profiles/r03_latsweep.json): crossover 256
  // round 4: P-FHEVM FFT64 runs its one-wave kernel in latency mode (two ciphertexts per workgroup, one transform
  // wave per SIMD) up to 512 ciphertexts (one round over 256 CUs), four per workgroup above
  c->lat_max = is_fft(*p) ? (p->N == 1024 ? 256 : 512) : p->N == 2048 ? 512 : 1024;
  {
    const char* e = getenv("TFHE_HIP_KS_VALU");
    c->ks_valu = e && e[0] == '1';
  }
  if (!is_fft(*p)) c->ninv = tfhe::gl_pow(p->N, tfhe::GL_P - 2);
  c->sh.resize(ndev);
  for (int i = 0; i < ndev; i++) c->sh[i].device = devices[i];
  for (int i = 0; i < ndev; i++) {
    const int rc = shard_init(c.get(), c->sh[i]);
    if (rc) {
      std::string m = g_err;
      tfhe_hip_destroy(c.release());
      return fail(rc, "create: shard %d (device %d): %s", i, devices[i], m.c_str());
    }
  }
  *out = c.release();
  return 0;
}

void tfhe_hip_destroy(tfhe_ctx* c) {
  if (!c) return;
  for (auto& s : c->sh) shard_free(s);
  if (!c->comms.empty() && rccl().ok)
    for (auto cm : c->comms)
      if (cm) rccl().comm_destroy(cm);
  delete c;
}

int tfhe_hip_device(const tfhe_ctx* c) { return c && !c->sh.empty() ? c->sh[0].device : -1; }
int tfhe_hip_ndev(const tfhe_ctx* c) { return c ? (int)c->sh.size() : 0; }
int tfhe_hip_device_at(const tfhe_ctx* c, int i) {
  return c && i >= 0 && i < (int)c->sh.size() ? c->sh[(size_t)i].device : -1;
}
int tfhe_hip_key_bcast_mode(const tfhe_ctx* c) { return c ? c->bcast_mode : -1; }

int tfhe_hip_bcast_plan(const int* devices, int ndev, const char* policy, int rccl_available, int* mode, int* calls,
                        int max_calls) {
  if (!devices || ndev < 1 || !mode || (max_calls > 0 && !calls)) return fail(TFHE_HIP_EINVAL, "bcast_plan: bad arguments");
  std::string why;
  const int n = bcast_plan(devices, ndev, policy, rccl_available != 0, mode, max_calls > 0 ? calls : nullptr, max_calls,
                           &why);
  return n < 0 ? fail(n, "bcast_plan: %s", why.c_str()) : n;
}

static int load_keys_impl(tfhe_ctx* c, const uint64_t* bsk, size_t bsk_len, const uint64_t* ksk, size_t ksk_len,
                          bool from_host) {
  if (!c || !bsk || !ksk) return fail(TFHE_HIP_EINVAL, "load_keys: null argument");
  if (bsk_len != tfhe::client::bsk_len(c->p) || ksk_len != tfhe::client::ksk_len(c->p))
    return fail(TFHE_HIP_EINVAL, "load_keys: sizes %zu/%zu, expected %zu/%zu", bsk_len, ksk_len,
                tfhe::client::bsk_len(c->p), tfhe::client::ksk_len(c->p));
  std::lock_guard<std::mutex> lk(c->mu);
  c->keys = false;
  c->bcast_mode = 0;
  const size_t nd = c->sh.size();
  // every shard: key buffers + a standard-domain BSK staging area (its d_stage)
  for (auto& s : c->sh) {
    DeviceGuard g(s.device);
    if (s.ws_used) HIP_TRY(hipEventSynchronize(s.ws_free));
    if (!s.d_bsk) HIP_TRY(hipMalloc(&s.d_bsk, bsk_len * 8));
    if (!s.d_ksk) HIP_TRY(hipMalloc(&s.d_ksk, ksk_len * 8));
    RC_TRY(grow(s, &s.d_stage, &s.stage_cap, bsk_len * 8));
  }
  shard& s0 = c->sh[0];
  const u64* bsk0 = (const u64*)bsk;  // standard BSK on shard 0's device
  {
    DeviceGuard g(s0.device);
    if (from_host) {
      RC_TRY(upload_pinned(s0, s0.d_stage, bsk, bsk_len * 8));
      RC_TRY(upload_pinned(s0, s0.d_ksk, ksk, ksk_len * 8));
      bsk0 = (const u64*)s0.d_stage;
    } else {
      HIP_TRY(hipMemcpyAsync(s0.d_ksk, ksk, ksk_len * 8, hipMemcpyDeviceToDevice, s0.stream));
      HIP_TRY(hipStreamSynchronize(s0.stream));
    }
  }
  if (nd > 1 || getenv("TFHE_HIP_BCAST")) {  // standard keys from shard 0 to every other shard, once
    std::vector<u64*> dst_b(nd), dst_k(nd);
    for (size_t i = 0; i < nd; i++) {
      dst_b[i] = (u64*)c->sh[i].d_stage;
      dst_k[i] = c->sh[i].d_ksk;
    }
    RC_TRY(broadcast(c, bsk0, dst_b, bsk_len));
    RC_TRY(broadcast(c, s0.d_ksk, dst_k, ksk_len));
  }
  for (size_t i = 0; i < nd; i++)
    RC_TRY(convert_keys(c, c->sh[i], i == 0 ? bsk0 : (const u64*)c->sh[i].d_stage, bsk_len));
  c->keys = true;
  return 0;
}

int tfhe_hip_load_keys(tfhe_ctx* c, const uint64_t* bsk, size_t bsk_len, const uint64_t* ksk, size_t ksk_len) {
  return load_keys_impl(c, bsk, bsk_len, ksk, ksk_len, true);
}

int tfhe_hip_load_keys_device(tfhe_ctx* c, const uint64_t* d_bsk, size_t bsk_len, const uint64_t* d_ksk,
                              size_t ksk_len) {
  return load_keys_impl(c, d_bsk, bsk_len, d_ksk, ksk_len, false);
}

int tfhe_hip_load_ms_key(tfhe_ctx* c, const uint64_t* zeros, uint32_t count, double bound, double r_sigma,
                         double input_variance) {
  if (!c || (count && !zeros)) return fail(TFHE_HIP_EINVAL, "load_ms_key: bad arguments");
  if (c->p.order != 1 && count)
    return fail(TFHE_HIP_EUNSUPPORTED, "load_ms_key: the noise reduction runs between keyswitch and blind rotation "
                                       "(KS -> PBS parameter sets only)");
  if (count > 0x7FFFFFFF || !(bound >= 0) || !(r_sigma >= 0) || !(input_variance >= 0))
    return fail(TFHE_HIP_EINVAL, "load_ms_key: count %u / bound / r_sigma / variance out of range", count);
  // the scan addresses the element-major transpose through a buffer resource with 32-bit byte offsets
  // (ms_reduce.hip): (n + 1) x pitch x 8 must stay below 2^31, or raw loads past num_records would read zeros
  // silently.  n = 918 allows ~292 k zeros; the reference's key carries 1449.
  if ((double)(c->p.n + 1) * (double)tfhe::ms_zeros_pitch(count) * 8.0 >= 0x1p31)
    return fail(TFHE_HIP_EINVAL, "load_ms_key: %u zeros x %u elements exceed the 2 GiB scan window", count,
                (unsigned)(c->p.n + 1));
  std::lock_guard<std::mutex> lk(c->mu);
  c->ms_count = 0;
  // two layouts in one allocation: rows [count][n+1] (the add of the chosen zero) then the element-major
  // transpose [n+1][zp] the scan reads 64 zeros per load from (pbs_kernels.h: ms_zeros_pitch)
  const size_t dim = c->p.n + 1, zp = tfhe::ms_zeros_pitch(count);
  const size_t bytes = (count * dim + dim * zp) * 8;
  std::vector<uint64_t> tr;
  if (count) {
    tr.assign(dim * zp, 0);
    for (size_t z = 0; z < count; z++)
      for (size_t i = 0; i < dim; i++) tr[i * zp + z] = zeros[z * dim + i];
  }
  for (auto& s : c->sh) {
    DeviceGuard g(s.device);
    HIP_TRY(hipStreamSynchronize(s.stream));
    if (s.ws_used) HIP_TRY(hipEventSynchronize(s.ws_free));
    (void)hipFree(s.d_ms_zeros);
    s.d_ms_zeros = nullptr;
    if (!count) continue;
    HIP_TRY(hipMalloc(&s.d_ms_zeros, bytes));
    HIP_TRY(hipMemcpy(s.d_ms_zeros, zeros, count * dim * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(s.d_ms_zeros + count * dim, tr.data(), tr.size() * 8, hipMemcpyHostToDevice));
  }
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
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t small = (size_t)c->p.n + 1;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{in, B * small * 8}}, d, B * 4));
  HIP_TRY(launch_ms(c, s, (u64*)d[0], B, (int*)d[1], s.stream));
  HIP_TRY(hipMemcpyAsync(out, d[0], B * small * 8, hipMemcpyDeviceToHost, s.stream));
  if (picks) HIP_TRY(hipMemcpyAsync(picks, d[1], B * 4, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
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
  size_t si = 0;
  if (c->sh.size() > 1) {  // the shard whose device holds the input
    hipPointerAttribute_t a;
    HIP_TRY(hipPointerGetAttributes(&a, d_in));
    si = c->sh.size();
    for (size_t i = 0; i < c->sh.size() && si == c->sh.size(); i++)
      if (c->sh[i].device == a.device) si = i;
    if (si == c->sh.size()) return fail(TFHE_HIP_EINVAL, "pbs_async: input on device %d, no shard there", a.device);
  }
  shard& s = c->sh[si];
  DeviceGuard g(s.device);
  hipStream_t st = stream == TFHE_HIP_NULL_STREAM ? (hipStream_t)0 : stream ? (hipStream_t)stream : s.stream;
  RC_TRY(ws_begin(s, st));
  RC_TRY(pbs_device(c, s, d_in, B, d_luts, n_lut, d_idx, d_out, st));
  return ws_end(s, st);
}

int tfhe_hip_pbs(tfhe_ctx* c, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                 const uint32_t* lut_index, uint64_t* lwe_out) {
  if (!c) return fail(TFHE_HIP_EINVAL, "pbs: null ctx");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "pbs: keys not loaded");
  if (B == 0) return 0;
  if (!lwe_in || !luts || !n_lut || !lwe_out) return fail(TFHE_HIP_EINVAL, "pbs: null buffer or n_lut == 0");
  if (B > 0x7FFFFFFF) return fail(TFHE_HIP_EINVAL, "pbs: batch too large");
  if (lut_index)
    for (size_t q = 0; q < B; q++)
      if (lut_index[q] >= n_lut) return fail(TFHE_HIP_EINVAL, "pbs: lut_index[%zu] = %u >= n_lut %zu", q, lut_index[q], n_lut);
  std::lock_guard<std::mutex> lk(c->mu);
  const size_t dim = io_dim(c->p) + 1;
  return for_each_slice(c, B, [&](size_t i, size_t lo, size_t hi) -> int {
    shard& s = c->sh[i];
    const size_t b = hi - lo;
    RC_TRY(ws_begin(s, s.stream));
    std::vector<void*> d;
    RC_TRY(stage(s, {{lwe_in + lo * dim, b * dim * 8}, {luts, n_lut * c->p.N * 8},
                     {lut_index ? lut_index + lo : nullptr, lut_index ? b * 4 : 0}},
                 d, b * dim * 8));
    RC_TRY(pbs_device(c, s, (const u64*)d[0], b, (const u64*)d[1], n_lut, (const u32*)d[2], (u64*)d[3], s.stream));
    HIP_TRY(hipMemcpyAsync(lwe_out + lo * dim, d[3], b * dim * 8, hipMemcpyDeviceToHost, s.stream));
    RC_TRY(ws_end(s, s.stream));
    HIP_TRY(hipStreamSynchronize(s.stream));
    return 0;
  });
}

int tfhe_hip_blind_rotate(tfhe_ctx* c, const uint64_t* lwe_in, size_t B, const uint64_t* luts, size_t n_lut,
                          const uint32_t* lut_index, uint64_t* acc_out) {
  if (!c) return fail(TFHE_HIP_EINVAL, "blind_rotate: null ctx");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "blind_rotate: keys not loaded");
  if (B == 0) return 0;
  if (!lwe_in || !luts || !n_lut || !acc_out) return fail(TFHE_HIP_EINVAL, "blind_rotate: null buffer");
  if (lut_index)
    for (size_t q = 0; q < B; q++)
      if (lut_index[q] >= n_lut) return fail(TFHE_HIP_EINVAL, "blind_rotate: lut_index[%zu] >= n_lut", q);
  std::lock_guard<std::mutex> lk(c->mu);
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t din = (size_t)c->p.n + 1, acc_len = (size_t)(c->p.k + 1) * c->p.N;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{lwe_in, B * din * 8}, {luts, n_lut * c->p.N * 8}, {lut_index, lut_index ? B * 4 : 0}}, d,
               B * acc_len * 8));
  HIP_TRY(launch_br(c, s, (const u64*)d[0], B, (const u64*)d[1], (const u32*)d[2], n_lut, nullptr, (u64*)d[3], s.stream));
  HIP_TRY(hipMemcpyAsync(acc_out, d[3], B * acc_len * 8, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

int tfhe_hip_sample_extract(tfhe_ctx* c, const uint64_t* acc, size_t B, uint64_t* out) {
  if (!c || (B && (!acc || !out))) return fail(TFHE_HIP_EINVAL, "sample_extract: bad arguments");
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t acc_len = (size_t)(c->p.k + 1) * c->p.N, big = (size_t)c->p.k * c->p.N + 1;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{acc, B * acc_len * 8}}, d, B * big * 8));
  if (is_fft(c->p) && c->p.N == 2048)
    HIP_TRY(tfhe::launch_sample_extract_torus2k((const u64*)d[0], B, (u64*)d[1], s.stream));
  else if (is_fft(c->p)) HIP_TRY(tfhe::launch_sample_extract_torus((const u64*)d[0], B, (u64*)d[1], s.stream));
  else if (c->p.N == 2048) HIP_TRY(tfhe::launch_sample_extract_2048((const u64*)d[0], B, (u64*)d[1], s.stream));
  else HIP_TRY(tfhe::launch_sample_extract((const u64*)d[0], B, (u64*)d[1], s.stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], B * big * 8, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

int tfhe_hip_keyswitch(tfhe_ctx* c, const uint64_t* in, size_t B, uint64_t* out) {
  if (!c || (B && (!in || !out))) return fail(TFHE_HIP_EINVAL, "keyswitch: bad arguments");
  if (!c->keys) return fail(TFHE_HIP_ENOKEYS, "keyswitch: keys not loaded");
  if (B == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t big = (size_t)c->p.k * c->p.N + 1, small = (size_t)c->p.n + 1;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{in, B * big * 8}}, d, B * small * 8));
  RC_TRY(launch_ks(c, s, (const u64*)d[0], B, (u64*)d[1], s.stream));
  HIP_TRY(hipMemcpyAsync(out, d[1], B * small * 8, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

static int ntt_impl(tfhe_ctx* c, uint64_t* polys, size_t count, bool inverse) {
  if (!c || (count && !polys)) return fail(TFHE_HIP_EINVAL, "ntt: bad arguments");
  if (is_fft(c->p)) return fail(TFHE_HIP_EUNSUPPORTED, "ntt: this ctx runs the FFT64 transform (tfhe_hip_fft_*)");
  if (count == 0) return 0;
  for (size_t i = 0; i < count * c->p.N; i++)
    if (polys[i] >= tfhe::GL_P) return fail(TFHE_HIP_EINVAL, "ntt: value at %zu not reduced mod p", i);
  std::lock_guard<std::mutex> lk(c->mu);
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t bytes = count * c->p.N * 8;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{polys, bytes}}, d, 0));
  if (c->p.N == 2048) {
    if (inverse) HIP_TRY(tfhe::launch_ntt2048_inv((u64*)d[0], count, s.d_tw, c->ninv, s.stream));
    else HIP_TRY(tfhe::launch_ntt2048_fwd((u64*)d[0], count, s.d_tw, s.stream));
  } else {
    if (inverse) HIP_TRY(tfhe::launch_ntt_inv((u64*)d[0], count, s.d_tw, c->ninv, s.stream));
    else HIP_TRY(tfhe::launch_ntt_fwd((u64*)d[0], count, s.d_tw, s.stream));
  }
  HIP_TRY(hipMemcpyAsync(polys, d[0], bytes, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

int tfhe_hip_ntt_fwd(tfhe_ctx* c, uint64_t* polys, size_t count) { return ntt_impl(c, polys, count, false); }
int tfhe_hip_ntt_inv(tfhe_ctx* c, uint64_t* polys, size_t count) { return ntt_impl(c, polys, count, true); }

static int fft_impl(tfhe_ctx* c, const void* in, size_t count, double* out, bool inverse) {
  if (!c || (count && (!in || !out))) return fail(TFHE_HIP_EINVAL, "fft: bad arguments");
  if (!is_fft(c->p)) return fail(TFHE_HIP_EUNSUPPORTED, "fft: ctx transform is not FFT64");
  if (count == 0) return 0;
  std::lock_guard<std::mutex> lk(c->mu);
  shard& s = c->sh[0];
  DeviceGuard g(s.device);
  const size_t bytes = count * c->p.N * 8;
  RC_TRY(ws_begin(s, s.stream));
  std::vector<void*> d;
  RC_TRY(stage(s, {{in, bytes}}, d, bytes));
  const double* tw = (const double*)s.d_tw;
  if (!inverse) {
    if (c->p.N == 2048) HIP_TRY(tfhe::launch_fft2k_fwd((const u64*)d[0], count, (double*)d[1], tw, s.stream));
    else HIP_TRY(tfhe::launch_fft_fwd((const u64*)d[0], count, (double*)d[1], tw, s.stream));
  } else {
    if (c->p.N == 2048) HIP_TRY(tfhe::launch_fft2k_inv((const double*)d[0], count, (double*)d[1], tw, s.stream));
    else HIP_TRY(tfhe::launch_fft_inv((const double*)d[0], count, (double*)d[1], tw, s.stream));
  }
  HIP_TRY(hipMemcpyAsync(out, d[1], bytes, hipMemcpyDeviceToHost, s.stream));
  RC_TRY(ws_end(s, s.stream));
  HIP_TRY(hipStreamSynchronize(s.stream));
  return 0;
}

int tfhe_hip_fft_fwd(tfhe_ctx* c, const uint64_t* polys, size_t count, double* out) {
  return fft_impl(c, polys, count, out, false);
}
int tfhe_hip_fft_inv(tfhe_ctx* c, const double* in, size_t count, double* out) {
  return fft_impl(c, in, count, out, true);
}

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

// mirrors launch_br / the launchers' B <= latency_max_batch switch
const char* tfhe_hip_br_kernel(const tfhe_ctx* c, size_t B) {
  if (!c) return nullptr;
  const bool lat = B <= c->lat_max;
  if (is_fft(c->p) && c->p.N == 2048) return "blind_rotate_fft2k_kernel";  // <2, ...> latency, <4, ...> batch
  if (is_fft(c->p)) return lat ? "blind_rotate_fft_lat_kernel" : "blind_rotate_fft_pair_kernel";
  if (c->p.N == 2048) return lat ? "blind_rotate2048_lat_kernel" : "blind_rotate2048_kernel";
  return lat ? "blind_rotate_lat_kernel" : "blind_rotate_kernel";
}

int tfhe_hip_sync(tfhe_ctx* c) {
  if (!c) return fail(TFHE_HIP_EINVAL, "sync: null ctx");
  for (auto& s : c->sh) {
    DeviceGuard g(s.device);
    HIP_TRY(hipStreamSynchronize(s.stream));
    if (s.ws_used) HIP_TRY(hipEventSynchronize(s.ws_free));
  }
  return 0;
}

int tfhe_hip_timing_enable(tfhe_ctx* c, int enable) {
  if (!c) return fail(TFHE_HIP_EINVAL, "timing: null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->timing = enable != 0;
  return 0;
}

int tfhe_hip_timing_reset(tfhe_ctx* c) {
  if (!c) return fail(TFHE_HIP_EINVAL, "timing: null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  for (auto& s : c->sh)
    for (int w = 0; w < 3; w++) {
      for (auto e : s.ev[w]) s.ev_pool.push_back(e);
      s.ev[w].clear();
    }
  return 0;
}

int tfhe_hip_timing_stats(tfhe_ctx* c, int which, double* total_ms, int* launches) {
  if (!c || which < 0 || which > 2 || !total_ms || !launches) return fail(TFHE_HIP_EINVAL, "timing: bad arguments");
  std::lock_guard<std::mutex> lk(c->mu);
  double tot = 0;
  int cnt = 0;
  for (auto& s : c->sh) {
    DeviceGuard g(s.device);
    auto& v = s.ev[which];
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
      HIP_TRY(hipEventSynchronize(v[i + 1]));
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, v[i], v[i + 1]));
      tot += ms;
      cnt++;
    }
  }
  *total_ms = tot;
  *launches = cnt;
  return 0;
}

}  // extern "C"
