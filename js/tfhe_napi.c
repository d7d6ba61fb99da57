/*
 * tfhe_napi.c — N-API binding of libtfhe_hip.so (include/tfhe_hip.h) for Node.
 *
 * Replaces the packages/wasm TFHE core that the JS SDKs reach (tfhe-rs WASM/N-API:
 * packages/pnpm-lock.yaml:1988-1995; used through global.TFHE, sdk/relayer/src/node.ts:1-4) and the
 * compute behind packages/luxfhejs' server calls (packages/luxfhejs/src/index.ts:127-141).
 *
 * Buffers cross as BigUint64Array / Uint32Array (zero-copy views of their backing stores).
 * Device work (pbs, nand, keyswitch, blindRotate) runs in napi_create_async_work and resolves a
 * Promise, so the event loop never blocks; argument buffers and the engine handle are referenced until
 * the work completes (destroyEngine during a job defers the ctx teardown to the last completion).  A failing
 * C-ABI call becomes a JS Error whose `code` is the TFHE_HIP_E* status.
 */
#include <node_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/tfhe_hip.h"

#define NAPI_CALL(env, call)                                              \
  do {                                                                    \
    if ((call) != napi_ok) {                                              \
      napi_throw_error((env), "EINTERNAL", "N-API call failed: " #call); \
      return NULL;                                                        \
    }                                                                     \
  } while (0)

static napi_value throw_tfhe(napi_env env, int rc) {
  napi_value err, msg, code;
  char cbuf[16];
  const char* m = tfhe_hip_last_error();
  napi_create_string_utf8(env, m && *m ? m : "tfhe_hip error", NAPI_AUTO_LENGTH, &msg);
  snprintf(cbuf, sizeof(cbuf), "%d", rc);
  napi_create_string_utf8(env, cbuf, NAPI_AUTO_LENGTH, &code);
  napi_create_error(env, code, msg, &err);
  napi_value num;
  napi_create_int32(env, rc, &num);
  napi_set_named_property(env, err, "status", num);
  napi_throw(env, err);
  return NULL;
}

/* typed-array argument -> data pointer + element count, checking the element type */
static int get_typed(napi_env env, napi_value v, napi_typedarray_type want, void** data, size_t* len) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return 0;
  napi_typedarray_type t;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok) return 0;
  return t == want;
}

static napi_value new_u64_array(napi_env env, size_t count, uint64_t** data) {
  napi_value ab, ta;
  void* p = NULL;
  if (napi_create_arraybuffer(env, count * 8, &p, &ab) != napi_ok) return NULL;
  memset(p, 0, count * 8);
  if (napi_create_typedarray(env, napi_biguint64_array, count, ab, 0, &ta) != napi_ok) return NULL;
  *data = (uint64_t*)p;
  return ta;
}

static int get_u64(napi_env env, napi_value v, uint64_t* out) {
  bool lossless;
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_bigint) return napi_get_value_bigint_uint64(env, v, out, &lossless) == napi_ok;
  if (t == napi_number) {
    double d;
    napi_get_value_double(env, v, &d);
    if (d < 0) return 0;
    *out = (uint64_t)d;
    return 1;
  }
  return 0;
}

/* rng argument: undefined / null -> 192 bits of OS entropy (production); BigInt / number -> the seeded
 * REPRODUCIBLE stream (tests, golden vectors; public knowledge); Uint8Array of 24 bytes -> raw key. */
static int get_rng(napi_env env, napi_value v, tfhe_rng_key* rk) {
  napi_valuetype t = napi_undefined;
  if (v && napi_typeof(env, v, &t) != napi_ok) return 0;
  if (t == napi_undefined || t == napi_null) return tfhe_hip_rng_key_entropy(rk) == 0;
  if (t == napi_bigint || t == napi_number) {
    uint64_t seed;
    return get_u64(env, v, &seed) && tfhe_hip_rng_key_from_seed(seed, rk) == 0;
  }
  uint8_t* d;
  size_t n;
  if (get_typed(env, v, napi_uint8_array, (void**)&d, &n) && n == sizeof(rk->w)) {
    memcpy(rk->w, d, sizeof(rk->w));
    return 1;
  }
  return 0;
}

static int get_params(napi_env env, napi_value v, tfhe_params* p) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  if (t == napi_number) {
    int32_t preset;
    napi_get_value_int32(env, v, &preset);
    return tfhe_hip_params_preset(preset, p) == 0;
  }
  if (t != napi_object) return 0;
  const char* names[] = {"n", "k", "N", "pbs_base_log", "pbs_level", "ks_base_log", "ks_level",
                         "lwe_noise_log2", "glwe_noise_log2", "order"};
  int32_t vals[10];
  for (int i = 0; i < 10; i++) {
    napi_value f;
    if (napi_get_named_property(env, v, names[i], &f) != napi_ok) return 0;
    if (napi_get_value_int32(env, f, &vals[i]) != napi_ok) return 0;
  }
  p->n = vals[0]; p->k = vals[1]; p->N = vals[2]; p->pbs_base_log = vals[3]; p->pbs_level = vals[4];
  p->ks_base_log = vals[5]; p->ks_level = vals[6]; p->lwe_noise_log2 = vals[7]; p->glwe_noise_log2 = vals[8];
  p->order = vals[9];
  p->transform = 0; /* optional: TFHE_HIP_TRANSFORM_* (absent = NTT) */
  {
    napi_value f;
    bool has = false;
    if (napi_has_named_property(env, v, "transform", &has) == napi_ok && has &&
        napi_get_named_property(env, v, "transform", &f) == napi_ok) {
      int32_t tr = 0;
      if (napi_get_value_int32(env, f, &tr) != napi_ok) return 0;
      p->transform = (uint32_t)tr;
    }
  }
  return 1;
}

static napi_value params_to_js(napi_env env, const tfhe_params* p) {
  napi_value o, x;
  napi_create_object(env, &o);
#define SETF(name, val) napi_create_int32(env, (int32_t)(val), &x); napi_set_named_property(env, o, name, x);
  SETF("n", p->n) SETF("k", p->k) SETF("N", p->N) SETF("pbs_base_log", p->pbs_base_log)
  SETF("pbs_level", p->pbs_level) SETF("ks_base_log", p->ks_base_log) SETF("ks_level", p->ks_level)
  SETF("lwe_noise_log2", p->lwe_noise_log2) SETF("glwe_noise_log2", p->glwe_noise_log2) SETF("order", p->order)
  SETF("transform", p->transform)
#undef SETF
  return o;
}

/* paramsPreset(preset) -> {n, k, N, ...} */
static napi_value js_params_preset(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_params p = {0};
  int32_t preset = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &preset);
  int rc = tfhe_hip_params_preset(preset, &p);
  if (rc) return throw_tfhe(env, rc);
  return params_to_js(env, &p);
}

/* keygen(params, rng[, withServerKey=true]) -> {lweKey, glweKey, bsk, ksk[, msZeros]}; rng as get_rng */
static napi_value js_keygen(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_params p = {0};
  tfhe_rng_key rk;
  if (argc < 1 || !get_params(env, argv[0], &p) || !get_rng(env, argc > 1 ? argv[1] : NULL, &rk)) {
    napi_throw_type_error(env, "EINVAL", "keygen(params[, seed | 24-byte key | undefined = OS entropy[, withServerKey]])");
    return NULL;
  }
  bool with_sk = true;
  if (argc > 2) napi_get_value_bool(env, argv[2], &with_sk);
  uint64_t *lwe, *glwe, *bsk = NULL, *ksk = NULL, *zeros = NULL;
  napi_value o, a_lwe, a_glwe, a_bsk = NULL, a_ksk = NULL, a_zeros = NULL;
  a_lwe = new_u64_array(env, p.n, &lwe);
  a_glwe = new_u64_array(env, (size_t)p.k * p.N, &glwe);
  if (!a_lwe || !a_glwe) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  if (with_sk) {
    a_bsk = new_u64_array(env, tfhe_hip_bsk_len(&p), &bsk);
    a_ksk = new_u64_array(env, tfhe_hip_ksk_len(&p), &ksk);
    if (!a_bsk || !a_ksk) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  }
  int rc = tfhe_hip_keygen_k(&p, &rk, lwe, glwe, bsk, ksk);
  if (rc) return throw_tfhe(env, rc);
  if (with_sk && p.order == 1) { /* KS -> PBS server keys carry the modulus-switch zeros */
    a_zeros = new_u64_array(env, (size_t)TFHE_HIP_MS_FHEVM_ZEROS * (p.n + 1), &zeros);
    if (!a_zeros) return throw_tfhe(env, TFHE_HIP_ENOMEM);
    rc = tfhe_hip_ms_zeros_keygen_k(&p, &rk, lwe, TFHE_HIP_MS_FHEVM_ZEROS, zeros);
    if (rc) return throw_tfhe(env, rc);
  }
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "lweKey", a_lwe);
  napi_set_named_property(env, o, "glweKey", a_glwe);
  if (with_sk) {
    napi_set_named_property(env, o, "bsk", a_bsk);
    napi_set_named_property(env, o, "ksk", a_ksk);
    if (a_zeros) napi_set_named_property(env, o, "msZeros", a_zeros);
  }
  napi_set_named_property(env, o, "params", params_to_js(env, &p));
  return o;
}

/* encrypt(key: BigUint64Array, noiseLog2, rng, stream0, msgs: BigUint64Array) -> BigUint64Array;
 * rng as get_rng (undefined = fresh OS entropy for this call) */
static napi_value js_encrypt(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint64_t *key, *msgs, stream0, *out;
  tfhe_rng_key rk;
  size_t dim, count;
  int32_t noise;
  if (argc < 5 || !get_typed(env, argv[0], napi_biguint64_array, (void**)&key, &dim) ||
      napi_get_value_int32(env, argv[1], &noise) != napi_ok || !get_rng(env, argv[2], &rk) ||
      !get_u64(env, argv[3], &stream0) || !get_typed(env, argv[4], napi_biguint64_array, (void**)&msgs, &count)) {
    napi_throw_type_error(env, "EINVAL", "encrypt(key, noiseLog2, rng, stream0, msgs)");
    return NULL;
  }
  napi_value res = new_u64_array(env, count * (dim + 1), &out);
  if (!res) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_lwe_encrypt_k((uint32_t)dim, key, noise, &rk, stream0, msgs, count, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

/* phase(key, cts) -> BigUint64Array of b - <a, s> */
static napi_value js_phase(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint64_t *key, *ct, *out;
  size_t dim, n;
  if (argc < 2 || !get_typed(env, argv[0], napi_biguint64_array, (void**)&key, &dim) ||
      !get_typed(env, argv[1], napi_biguint64_array, (void**)&ct, &n) || n % (dim + 1)) {
    napi_throw_type_error(env, "EINVAL", "phase(key, cts)");
    return NULL;
  }
  napi_value res = new_u64_array(env, n / (dim + 1), &out);
  int rc = tfhe_hip_lwe_phase((uint32_t)dim, key, ct, n / (dim + 1), out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

/* lutConstant(N, value) / lutFromTable(N, msgModulus, table: BigUint64Array, deltaOut) */
static napi_value js_lut_constant(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t N;
  uint64_t v, *out;
  if (argc < 2 || napi_get_value_uint32(env, argv[0], &N) != napi_ok || !get_u64(env, argv[1], &v)) {
    napi_throw_type_error(env, "EINVAL", "lutConstant(N, value)");
    return NULL;
  }
  napi_value res = new_u64_array(env, N, &out);
  int rc = tfhe_hip_lut_constant(N, v, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

static napi_value js_lut_from_table(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t N, mm;
  uint64_t *table, delta, *out;
  size_t tl;
  if (argc < 4 || napi_get_value_uint32(env, argv[0], &N) != napi_ok ||
      napi_get_value_uint32(env, argv[1], &mm) != napi_ok ||
      !get_typed(env, argv[2], napi_biguint64_array, (void**)&table, &tl) || tl < mm || !get_u64(env, argv[3], &delta)) {
    napi_throw_type_error(env, "EINVAL", "lutFromTable(N, msgModulus, table, deltaOut)");
    return NULL;
  }
  napi_value res = new_u64_array(env, N, &out);
  int rc = tfhe_hip_lut_from_table(N, mm, table, delta, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

/* ------------------------------------------------------------------------------ engine */
static void finalize_ctx(napi_env env, void* data, void* hint) {
  (void)env; (void)hint;
  if (data) tfhe_hip_destroy((tfhe_ctx*)data);
}

/* An engine handle.  Every queued job holds a reference to the handle's JS external (so GC cannot
 * finalize it while the job runs) and counts in `pending`; destroyEngine with jobs in flight only marks
 * the box, and the last job's completion (main thread, like destroyEngine) destroys the ctx. */
#define BOX_ENGINE 0x454E4731u /* first word of every external's payload: which handle it is */
#define BOX_AUX 0x41555831u
typedef struct {
  uint32_t magic; /* BOX_ENGINE */
  tfhe_ctx* ctx;
  tfhe_params p;
  int pending;
  int destroy_requested;
} ctx_box;

static void finalize_box(napi_env env, void* data, void* hint) {
  ctx_box* b = (ctx_box*)data;
  if (b) {
    finalize_ctx(env, b->ctx, hint);  /* unreachable with jobs pending: they reference the external */
    free(b);
  }
}

static ctx_box* get_box(napi_env env, napi_value v) {
  void* d = NULL;
  if (napi_get_value_external(env, v, &d) != napi_ok || !d || *(uint32_t*)d != BOX_ENGINE) return NULL;
  return (ctx_box*)d;
}

/* createEngine(params[, devices = 0]) -> external handle (destroyed by GC or destroyEngine).
 * devices: one ordinal or an array of ordinals (one shard each: include/tfhe_hip.h). */
static napi_value js_create(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_params p = {0};
  int devs[64] = {0};
  int ndev = 1;
  if (argc < 1 || !get_params(env, argv[0], &p)) {
    napi_throw_type_error(env, "EINVAL", "createEngine(params[, devices])");
    return NULL;
  }
  if (argc > 1) {
    bool is_arr = false;
    napi_is_array(env, argv[1], &is_arr);
    if (is_arr) {
      uint32_t len = 0;
      napi_get_array_length(env, argv[1], &len);
      if (len < 1 || len > 64) {
        napi_throw_range_error(env, "EINVAL", "createEngine: 1..64 devices");
        return NULL;
      }
      for (uint32_t i = 0; i < len; i++) {
        napi_value e;
        napi_get_element(env, argv[1], i, &e);
        if (napi_get_value_int32(env, e, &devs[i]) != napi_ok) {
          napi_throw_type_error(env, "EINVAL", "createEngine: device ordinals must be numbers");
          return NULL;
        }
      }
      ndev = (int)len;
    } else {
      napi_valuetype t;
      napi_typeof(env, argv[1], &t);
      if (t == napi_number) napi_get_value_int32(env, argv[1], &devs[0]);
      else if (t != napi_undefined && t != napi_null) {
        napi_throw_type_error(env, "EINVAL", "createEngine: devices must be a number or an array of numbers");
        return NULL;
      }
    }
  }
  tfhe_ctx* c = NULL;
  int rc = tfhe_hip_create(&p, devs, ndev, &c);
  if (rc) return throw_tfhe(env, rc);
  ctx_box* b = (ctx_box*)calloc(1, sizeof(ctx_box));
  if (!b) {
    tfhe_hip_destroy(c);
    return throw_tfhe(env, TFHE_HIP_ENOMEM);
  }
  b->magic = BOX_ENGINE;
  b->ctx = c;
  b->p = p;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, b, finalize_box, NULL, &ext));
  return ext;
}

static napi_value js_destroy(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = argc ? get_box(env, argv[0]) : NULL;
  if (b && b->ctx) {
    if (b->pending) {
      b->destroy_requested = 1;  /* the last pending job's completion destroys the ctx */
    } else {
      tfhe_hip_destroy(b->ctx);
      b->ctx = NULL;
    }
  }
  return NULL;
}

/* engineInfo(engine) -> {devices: [..], keyBroadcast: 'single' | 'copy' | 'rccl', pending} */
static napi_value js_engine_info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = argc ? get_box(env, argv[0]) : NULL;
  if (!b || !b->ctx || b->destroy_requested) {
    napi_throw_type_error(env, "EINVAL", "engineInfo(engine): engine destroyed");
    return NULL;
  }
  napi_value o, arr, x;
  napi_create_object(env, &o);
  const int nd = tfhe_hip_ndev(b->ctx);
  napi_create_array_with_length(env, (size_t)nd, &arr);
  for (int i = 0; i < nd; i++) {
    napi_create_int32(env, tfhe_hip_device_at(b->ctx, i), &x);
    napi_set_element(env, arr, (uint32_t)i, x);
  }
  napi_set_named_property(env, o, "devices", arr);
  const int m = tfhe_hip_key_bcast_mode(b->ctx);
  napi_create_string_utf8(env, m == 2 ? "rccl" : m == 1 ? "copy" : "single", NAPI_AUTO_LENGTH, &x);
  napi_set_named_property(env, o, "keyBroadcast", x);
  napi_create_int32(env, b->pending, &x);
  napi_set_named_property(env, o, "pending", x);
  return o;
}

/* loadKeys(handle, bsk, ksk) */
/* loadKeys(engine, bsk, ksk[, msZeros]) — msZeros enables the P-FHEVM modulus-switch noise reduction */
static napi_value js_load_keys(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = argc ? get_box(env, argv[0]) : NULL;
  uint64_t *bsk, *ksk;
  size_t bl, kl;
  if (!b || !b->ctx || b->destroy_requested || b->pending || argc < 3 ||
      !get_typed(env, argv[1], napi_biguint64_array, (void**)&bsk, &bl) ||
      !get_typed(env, argv[2], napi_biguint64_array, (void**)&ksk, &kl)) {
    napi_throw_type_error(env, "EINVAL", "loadKeys(engine, bsk, ksk[, msZeros]) on an idle live engine");
    return NULL;
  }
  uint64_t* zeros = NULL;
  size_t zl = 0;
  if (argc > 3) {
    napi_valuetype t;
    napi_typeof(env, argv[3], &t);
    if (t != napi_undefined && t != napi_null && !get_typed(env, argv[3], napi_biguint64_array, (void**)&zeros, &zl)) {
      napi_throw_type_error(env, "EINVAL", "loadKeys: msZeros must be a BigUint64Array");
      return NULL;
    }
  }
  int rc = tfhe_hip_load_keys(b->ctx, bsk, bl, ksk, kl);
  if (rc) return throw_tfhe(env, rc);
  if (zeros) {
    rc = tfhe_hip_load_ms_key(b->ctx, zeros, (uint32_t)(zl / (b->p.n + 1)), TFHE_HIP_MS_FHEVM_BOUND,
                              TFHE_HIP_MS_FHEVM_R_SIGMA, TFHE_HIP_MS_FHEVM_INPUT_VARIANCE);
    if (rc) return throw_tfhe(env, rc);
  }
  return NULL;
}

/* ---- async work: pbs / nand / keyswitch / blindRotate ------------------------------------ */
enum { JOB_PBS = 0, JOB_NAND = 1, JOB_KEYSWITCH = 2, JOB_BLIND_ROTATE = 3, JOB_PACK = 4, JOB_SQUASH = 5 };

/* A packing-keyswitch (tfhe_pks_ctx) or noise-squashing (tfhe_sns_ctx) context: the adjacent kernels of the
 * fhEVM coprocessor.  Same lifetime rules as an engine (pending jobs defer the teardown). */
enum { AUX_PKS = 1, AUX_SNS = 2 };
typedef struct {
  uint32_t magic; /* BOX_AUX */
  int kind;
  void* ctx;
  tfhe_pks_params pp;
  tfhe_sns_params sp;
  int pending;
  int destroy_requested;
} aux_box;

static void aux_destroy(aux_box* a) {
  if (!a->ctx) return;
  if (a->kind == AUX_PKS) tfhe_hip_pks_destroy((tfhe_pks_ctx*)a->ctx);
  else tfhe_hip_sns_destroy((tfhe_sns_ctx*)a->ctx);
  a->ctx = NULL;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref refs[5];
  int nrefs;
  ctx_box* box;  /* NULL for packing jobs */
  tfhe_ctx* ctx;
  aux_box* abox; /* packing / squashing jobs */
  int kind;
  const uint64_t *in, *in2, *luts;
  const uint32_t* lut_index;
  size_t B, n_lut;
  uint32_t msg_modulus;
  uint64_t* out;
  napi_ref out_ref;
  uint64_t* out2; /* JOB_PACK: the compressed words of every GLWE, concatenated */
  napi_ref out2_ref;
  int rc;
  char err[256];
} job_t;

/* JOB_PACK: pack on the device, then modulus-switch + bit-pack every GLWE on the host (compression.rs:246-291) */
static int run_pack(job_t* j) {
  const tfhe_pks_params* pp = &j->abox->pp;
  const size_t glwe_len = (size_t)(pp->out_k + 1) * pp->out_N;
  int rc = tfhe_hip_pks_pack((tfhe_pks_ctx*)j->abox->ctx, j->in, j->B, j->out);
  uint64_t* dst = j->out2;
  for (size_t g = 0; !rc && g * pp->lwe_per_glwe < j->B; g++) {
    const size_t left = j->B - g * pp->lwe_per_glwe;
    const uint32_t bodies = (uint32_t)(left < pp->lwe_per_glwe ? left : pp->lwe_per_glwe);
    rc = tfhe_hip_pks_compress(pp, j->out + g * glwe_len, bodies, dst);
    dst += tfhe_hip_pks_packed_words(pp, bodies);
  }
  return rc;
}

/* JOB_SQUASH: the sns-worker path of one batch of P-FHEVM big-key ciphertexts: keyswitch + modulus-switch noise
 * reduction on the engine, then the 128-bit bootstrap on the squasher */
static int run_squash(job_t* j) {
  const size_t small = (size_t)j->box->p.n + 1;
  uint64_t* ks = (uint64_t*)malloc(j->B * small * 8);
  uint64_t* ms = (uint64_t*)malloc(j->B * small * 8);
  int32_t* picks = (int32_t*)malloc(j->B * sizeof(int32_t) + 1);
  int rc = ks && ms && picks ? 0 : TFHE_HIP_ENOMEM;
  if (!rc) rc = tfhe_hip_keyswitch(j->ctx, j->in, j->B, ks);
  if (!rc) rc = tfhe_hip_ms_reduce(j->ctx, ks, j->B, ms, picks);
  if (!rc) rc = tfhe_hip_sns_squash((tfhe_sns_ctx*)j->abox->ctx, ms, j->B, j->msg_modulus, j->out);
  free(ks);
  free(ms);
  free(picks);
  return rc;
}

static void job_execute(napi_env env, void* data) {
  (void)env;
  job_t* j = (job_t*)data;
  if (j->kind == JOB_PBS) j->rc = tfhe_hip_pbs(j->ctx, j->in, j->B, j->luts, j->n_lut, j->lut_index, j->out);
  else if (j->kind == JOB_NAND) j->rc = tfhe_hip_nand(j->ctx, j->in, j->in2, j->B, j->out);
  else if (j->kind == JOB_KEYSWITCH) j->rc = tfhe_hip_keyswitch(j->ctx, j->in, j->B, j->out);
  else if (j->kind == JOB_BLIND_ROTATE)
    j->rc = tfhe_hip_blind_rotate(j->ctx, j->in, j->B, j->luts, j->n_lut, j->lut_index, j->out);
  else if (j->kind == JOB_PACK) j->rc = run_pack(j);
  else j->rc = run_squash(j);
  if (j->rc) snprintf(j->err, sizeof(j->err), "%s", tfhe_hip_last_error());
}

static void job_complete(napi_env env, napi_status status, void* data) {
  job_t* j = (job_t*)data;
  napi_value out;
  napi_get_reference_value(env, j->out_ref, &out);
  if (status == napi_ok && j->rc == 0) {
    if (j->kind == JOB_PACK) { /* {glwes, packed} */
      napi_value o, packed;
      napi_get_reference_value(env, j->out2_ref, &packed);
      napi_create_object(env, &o);
      napi_set_named_property(env, o, "glwes", out);
      napi_set_named_property(env, o, "packed", packed);
      out = o;
    }
    napi_resolve_deferred(env, j->deferred, out);
  } else {
    napi_value err, msg, code, num;
    char cbuf[16];
    snprintf(cbuf, sizeof(cbuf), "%d", j->rc);
    napi_create_string_utf8(env, j->rc ? j->err : "async work cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_string_utf8(env, cbuf, NAPI_AUTO_LENGTH, &code);
    napi_create_error(env, code, msg, &err);
    napi_create_int32(env, j->rc, &num);
    napi_set_named_property(env, err, "status", num);
    napi_reject_deferred(env, j->deferred, err);
  }
  for (int i = 0; i < j->nrefs; i++) napi_delete_reference(env, j->refs[i]);
  napi_delete_reference(env, j->out_ref);
  if (j->out2_ref) napi_delete_reference(env, j->out2_ref);
  napi_delete_async_work(env, j->work);
  ctx_box* b = j->box;
  if (b && --b->pending == 0 && b->destroy_requested && b->ctx) {
    tfhe_hip_destroy(b->ctx);
    b->ctx = NULL;
  }
  aux_box* a = j->abox;
  if (a && --a->pending == 0 && a->destroy_requested) aux_destroy(a);
  free(j);
}

/* engine: the handle (argv[0]) -- referenced by the job, so the box outlives it */
static napi_value queue_job(napi_env env, ctx_box* b, napi_value engine, job_t* j, napi_value* keep, int nkeep,
                            size_t out_len) {
  napi_value promise, out, name;
  uint64_t* outp;
  out = new_u64_array(env, out_len, &outp);
  if (!out) {
    free(j);
    return throw_tfhe(env, TFHE_HIP_ENOMEM);
  }
  j->box = b;
  j->ctx = b ? b->ctx : NULL;
  j->out = outp;
  j->work = NULL;
  napi_create_reference(env, out, 1, &j->out_ref);
  napi_create_reference(env, engine, 1, &j->refs[j->nrefs++]);
  for (int i = 0; i < nkeep; i++) napi_create_reference(env, keep[i], 1, &j->refs[j->nrefs++]);
  /* b->pending counts only jobs that were queued: on any failure below the references and the job are
   * released here and the engine stays destroyable / reloadable */
  napi_status st = napi_create_promise(env, &j->deferred, &promise);
  const int have_promise = st == napi_ok;
  if (st == napi_ok) {
    napi_create_string_utf8(env, "tfhe_hip", NAPI_AUTO_LENGTH, &name);
    st = napi_create_async_work(env, NULL, name, job_execute, job_complete, j, &j->work);
  }
  if (st == napi_ok) st = napi_queue_async_work(env, j->work);
  if (st != napi_ok) {
    if (j->work) napi_delete_async_work(env, j->work);
    for (int i = 0; i < j->nrefs; i++) napi_delete_reference(env, j->refs[i]);
    napi_delete_reference(env, j->out_ref);
    if (j->out2_ref) napi_delete_reference(env, j->out2_ref);
    if (have_promise) { /* settle the promise rather than leak its deferred */
      napi_value err, code, msg;
      napi_create_string_utf8(env, "EDEVICE", NAPI_AUTO_LENGTH, &code);
      napi_create_string_utf8(env, "could not queue the async work", NAPI_AUTO_LENGTH, &msg);
      napi_create_error(env, code, msg, &err);
      napi_reject_deferred(env, j->deferred, err);
      free(j);
      return promise;
    }
    free(j);
    napi_throw_error(env, "EDEVICE", "could not queue the async work");
    return NULL;
  }
  if (b) b->pending++;
  if (j->abox) j->abox->pending++;
  return promise;
}

static ctx_box* live_box(napi_env env, size_t argc, napi_value* argv) {
  ctx_box* b = argc ? get_box(env, argv[0]) : NULL;
  return b && b->ctx && !b->destroy_requested ? b : NULL;
}

/* optional Uint32Array lutIndex at argv[i]: 1 = ok (idx may stay NULL), 0 = wrong type */
static int get_lut_index(napi_env env, size_t argc, napi_value* argv, size_t i, uint32_t** idx, size_t* n) {
  napi_valuetype t = napi_undefined;
  if (argc > i) napi_typeof(env, argv[i], &t);
  if (t == napi_undefined || t == napi_null) return 1;
  return get_typed(env, argv[i], napi_uint32_array, (void**)idx, n);
}

/* pbs(engine, cts, luts[, lutIndex]) -> Promise<BigUint64Array>: full PBS (both orders incl. keyswitch) */
/* blindRotate(engine, cts, luts[, lutIndex]) -> Promise<BigUint64Array> of B x (k+1) x N accumulators */
static napi_value pbs_like(napi_env env, napi_callback_info info, int kind) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = live_box(env, argc, argv);
  uint64_t *in, *luts;
  uint32_t* idx = NULL;
  size_t n_in, n_l, n_idx = 0;
  const char* usage = kind == JOB_PBS ? "pbs(engine, cts, luts[, lutIndex])" : "blindRotate(engine, cts, luts[, lutIndex])";
  if (!b || argc < 3 || !get_typed(env, argv[1], napi_biguint64_array, (void**)&in, &n_in) ||
      !get_typed(env, argv[2], napi_biguint64_array, (void**)&luts, &n_l)) {
    napi_throw_type_error(env, "EINVAL", usage);
    return NULL;
  }
  if (!get_lut_index(env, argc, argv, 3, &idx, &n_idx)) {
    napi_throw_type_error(env, "EINVAL", "lutIndex must be a Uint32Array");
    return NULL;
  }
  const tfhe_params p = b->p;
  /* blind rotation inputs are small-key LWEs (n + 1), PBS inputs are io_dim + 1 */
  const size_t dim = kind == JOB_PBS ? (size_t)tfhe_hip_io_dim(&p) + 1 : (size_t)p.n + 1;
  if (n_in % dim || n_l % p.N || !n_l || (idx && n_idx != n_in / dim)) {
    napi_throw_range_error(env, "EINVAL", "buffer sizes do not match the parameter set");
    return NULL;
  }
  job_t* j = (job_t*)calloc(1, sizeof(job_t));
  if (!j) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  j->kind = kind;
  j->in = in;
  j->luts = luts;
  j->lut_index = idx;
  j->B = n_in / dim;
  j->n_lut = n_l / p.N;
  napi_value keep[3] = {argv[1], argv[2], idx ? argv[3] : argv[1]};
  const size_t out_len = kind == JOB_PBS ? n_in : j->B * (size_t)(p.k + 1) * p.N;
  return queue_job(env, b, argv[0], j, keep, 3, out_len);
}

static napi_value js_pbs(napi_env env, napi_callback_info info) { return pbs_like(env, info, JOB_PBS); }
static napi_value js_blind_rotate(napi_env env, napi_callback_info info) {
  return pbs_like(env, info, JOB_BLIND_ROTATE);
}

/* keyswitch(engine, bigLwes: B x (kN+1)) -> Promise<BigUint64Array> of B x (n+1) (LWE keyswitch, the KS half
 * of ServerKey::keyswitch_programmable_bootstrap, ml/biometrics/notebooks/main.rs:71) */
static napi_value js_keyswitch(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = live_box(env, argc, argv);
  uint64_t* in;
  size_t n_in;
  if (!b || argc < 2 || !get_typed(env, argv[1], napi_biguint64_array, (void**)&in, &n_in)) {
    napi_throw_type_error(env, "EINVAL", "keyswitch(engine, bigLwes)");
    return NULL;
  }
  const size_t big = (size_t)b->p.k * b->p.N + 1, small = (size_t)b->p.n + 1;
  if (n_in % big) {
    napi_throw_range_error(env, "EINVAL", "keyswitch: length is not a multiple of k*N + 1");
    return NULL;
  }
  job_t* j = (job_t*)calloc(1, sizeof(job_t));
  if (!j) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  j->kind = JOB_KEYSWITCH;
  j->in = in;
  j->B = n_in / big;
  napi_value keep[1] = {argv[1]};
  return queue_job(env, b, argv[0], j, keep, 1, j->B * small);
}

/* nand(engine, c1, c2) -> Promise<BigUint64Array> */
static napi_value js_nand(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ctx_box* b = live_box(env, argc, argv);
  uint64_t *c1, *c2;
  size_t n1, n2;
  if (!b || argc < 3 || !get_typed(env, argv[1], napi_biguint64_array, (void**)&c1, &n1) ||
      !get_typed(env, argv[2], napi_biguint64_array, (void**)&c2, &n2) || n1 != n2) {
    napi_throw_type_error(env, "EINVAL", "nand(engine, c1, c2) with equal-length BigUint64Arrays");
    return NULL;
  }
  const size_t dim = (size_t)b->p.n + 1;
  if (n1 % dim) {
    napi_throw_range_error(env, "EINVAL", "nand: length is not a multiple of n + 1");
    return NULL;
  }
  job_t* j = (job_t*)calloc(1, sizeof(job_t));
  if (!j) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  j->kind = JOB_NAND;
  j->in = c1;
  j->in2 = c2;
  j->B = n1 / dim;
  napi_value keep[2] = {argv[1], argv[2]};
  return queue_job(env, b, argv[0], j, keep, 2, n1);
}

/* ---- adjacent kernels: packing keyswitch + compression, noise squashing ------------------
 * The reference's consumers: ciphertext compression (ml/extensions/rust/src/compression.rs:222,276) and the
 * fhEVM sns-worker (tests/fhevm-suite/fhevm/docker-compose/coprocessor-docker-compose.yml:124-140). */
static void finalize_aux(napi_env env, void* data, void* hint) {
  (void)env; (void)hint;
  aux_box* a = (aux_box*)data;
  if (a) {
    aux_destroy(a); /* unreachable with jobs pending: they reference the external */
    free(a);
  }
}

static aux_box* get_aux(napi_env env, napi_value v, int kind) {
  void* d = NULL;
  if (napi_get_value_external(env, v, &d) != napi_ok || !d || *(uint32_t*)d != BOX_AUX) return NULL;
  aux_box* a = (aux_box*)d;
  return a->kind == kind && a->ctx && !a->destroy_requested ? a : NULL;
}

static int opt_device(napi_env env, size_t argc, napi_value* argv, size_t i, int* dev) {
  *dev = 0;
  if (argc <= i) return 1;
  napi_valuetype t;
  napi_typeof(env, argv[i], &t);
  if (t == napi_undefined || t == napi_null) return 1;
  return t == napi_number && napi_get_value_int32(env, argv[i], dev) == napi_ok;
}

/* createPacker([device = 0]) -> external (PARAMS_8B_2048_NEW packing keyswitch, the only preset) */
static napi_value js_create_packer(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int dev;
  if (!opt_device(env, argc, argv, 0, &dev)) {
    napi_throw_type_error(env, "EINVAL", "createPacker([device])");
    return NULL;
  }
  aux_box* a = (aux_box*)calloc(1, sizeof(aux_box));
  if (!a) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  a->magic = BOX_AUX;
  a->kind = AUX_PKS;
  int rc = tfhe_hip_pks_params_preset(TFHE_HIP_PKS_PRESET_ML2048, &a->pp);
  tfhe_pks_ctx* c = NULL;
  if (!rc) rc = tfhe_hip_pks_create(&a->pp, dev, &c);
  if (rc) {
    free(a);
    return throw_tfhe(env, rc);
  }
  a->ctx = c;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, a, finalize_aux, NULL, &ext));
  return ext;
}

/* createSquasher([device = 0]) -> external (k = 2, N = 2048, 2^24 x 3 squashing PBS, TFHE_HIP_SNS_PRESET_FHEVM) */
static napi_value js_create_squasher(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int dev;
  if (!opt_device(env, argc, argv, 0, &dev)) {
    napi_throw_type_error(env, "EINVAL", "createSquasher([device])");
    return NULL;
  }
  aux_box* a = (aux_box*)calloc(1, sizeof(aux_box));
  if (!a) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  a->magic = BOX_AUX;
  a->kind = AUX_SNS;
  int rc = tfhe_hip_sns_params_preset(TFHE_HIP_SNS_PRESET_FHEVM, &a->sp);
  tfhe_sns_ctx* c = NULL;
  if (!rc) rc = tfhe_hip_sns_create(&a->sp, dev, &c);
  if (rc) {
    free(a);
    return throw_tfhe(env, rc);
  }
  a->ctx = c;
  napi_value ext;
  NAPI_CALL(env, napi_create_external(env, a, finalize_aux, NULL, &ext));
  return ext;
}

/* destroyAux(handle): deferred to the last pending job like destroyEngine */
static napi_value js_destroy_aux(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void* d = NULL;
  if (argc && napi_get_value_external(env, argv[0], &d) == napi_ok && d && *(uint32_t*)d == BOX_AUX) {
    aux_box* a = (aux_box*)d;
    if (a->pending) a->destroy_requested = 1;
    else aux_destroy(a);
  }
  return NULL;
}

/* pksKeygen(inKey[, rng]) -> {outKey, pksk}: the post-packing GLWE key (client) and the packing KSK (server) */
static napi_value js_pks_keygen(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_pks_params pp;
  tfhe_rng_key rk;
  uint64_t *in_key, *ok, *pk;
  size_t n;
  if (tfhe_hip_pks_params_preset(TFHE_HIP_PKS_PRESET_ML2048, &pp) || argc < 1 ||
      !get_typed(env, argv[0], napi_biguint64_array, (void**)&in_key, &n) || n != pp.in_dim ||
      !get_rng(env, argc > 1 ? argv[1] : NULL, &rk)) {
    napi_throw_type_error(env, "EINVAL", "pksKeygen(inKey: BigUint64Array(2048)[, rng])");
    return NULL;
  }
  napi_value o, a, b;
  a = new_u64_array(env, (size_t)pp.out_k * pp.out_N, &ok);
  b = new_u64_array(env, tfhe_hip_pksk_len(&pp), &pk);
  if (!a || !b) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_pks_keygen_k(&pp, &rk, in_key, ok, pk);
  if (rc) return throw_tfhe(env, rc);
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "outKey", a);
  napi_set_named_property(env, o, "pksk", b);
  return o;
}

/* snsKeygen(lweKey[, rng]) -> {glweKey, bsk}: the 128-bit GLWE key (client) and the squashing BSK (server) */
static napi_value js_sns_keygen(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_sns_params sp;
  tfhe_rng_key rk;
  uint64_t *lwe_key, *gk, *bk;
  size_t n;
  if (tfhe_hip_sns_params_preset(TFHE_HIP_SNS_PRESET_FHEVM, &sp) || argc < 1 ||
      !get_typed(env, argv[0], napi_biguint64_array, (void**)&lwe_key, &n) || n != sp.n ||
      !get_rng(env, argc > 1 ? argv[1] : NULL, &rk)) {
    napi_throw_type_error(env, "EINVAL", "snsKeygen(lweKey: BigUint64Array(918)[, rng])");
    return NULL;
  }
  napi_value o, a, b;
  a = new_u64_array(env, (size_t)sp.k * sp.N, &gk);
  b = new_u64_array(env, tfhe_hip_sns_bsk_len(&sp), &bk);
  if (!a || !b) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_sns_keygen_k(&sp, &rk, lwe_key, gk, bk);
  if (rc) return throw_tfhe(env, rc);
  napi_create_object(env, &o);
  napi_set_named_property(env, o, "glweKey", a);
  napi_set_named_property(env, o, "bsk", b);
  return o;
}

/* loadAuxKey(handle, key): the packing KSK of a packer or the squashing BSK of a squasher */
static napi_value js_load_aux_key(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  void* d = NULL;
  uint64_t* key;
  size_t n;
  if (argc < 2 || napi_get_value_external(env, argv[0], &d) != napi_ok || !d || *(uint32_t*)d != BOX_AUX ||
      !get_typed(env, argv[1], napi_biguint64_array, (void**)&key, &n)) {
    napi_throw_type_error(env, "EINVAL", "loadAuxKey(packer | squasher, key)");
    return NULL;
  }
  aux_box* a = (aux_box*)d;
  if (!a->ctx || a->destroy_requested || a->pending) {
    napi_throw_type_error(env, "EINVAL", "loadAuxKey: destroyed or busy handle");
    return NULL;
  }
  const int rc = a->kind == AUX_PKS ? tfhe_hip_pks_load_key((tfhe_pks_ctx*)a->ctx, key, n)
                                    : tfhe_hip_sns_load_key((tfhe_sns_ctx*)a->ctx, key, n);
  if (rc) return throw_tfhe(env, rc);
  return NULL;
}

/* packCompress(packer, lwes: count x 2049) -> Promise<{glwes, packed}>: LWE -> GLWE packing keyswitch on the
 * device (chunks of 2048 LWEs per GLWE), then each GLWE modulus-switched and bit-packed (26 bits per word);
 * `packed` concatenates the GLWEs' words (tfhe_hip_pks_packed_words(bodies) each, last one ragged) */
static napi_value js_pack_compress(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  aux_box* a = argc ? get_aux(env, argv[0], AUX_PKS) : NULL;
  uint64_t* in;
  size_t n_in;
  if (!a || argc < 2 || !get_typed(env, argv[1], napi_biguint64_array, (void**)&in, &n_in)) {
    napi_throw_type_error(env, "EINVAL", "packCompress(packer, lwes)");
    return NULL;
  }
  const tfhe_pks_params* pp = &a->pp;
  const size_t dim = (size_t)pp->in_dim + 1;
  if (!n_in || n_in % dim) {
    napi_throw_range_error(env, "EINVAL", "packCompress: length is not a positive multiple of in_dim + 1");
    return NULL;
  }
  const size_t count = n_in / dim, groups = (count + pp->lwe_per_glwe - 1) / pp->lwe_per_glwe;
  size_t words = 0;
  for (size_t g = 0; g < groups; g++) {
    const size_t left = count - g * pp->lwe_per_glwe;
    words += tfhe_hip_pks_packed_words(pp, (uint32_t)(left < pp->lwe_per_glwe ? left : pp->lwe_per_glwe));
  }
  job_t* j = (job_t*)calloc(1, sizeof(job_t));
  if (!j) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  napi_value packed = new_u64_array(env, words, &j->out2);
  if (!packed) {
    free(j);
    return throw_tfhe(env, TFHE_HIP_ENOMEM);
  }
  napi_create_reference(env, packed, 1, &j->out2_ref);
  j->kind = JOB_PACK;
  j->abox = a;
  j->in = in;
  j->B = count;
  napi_value keep[1] = {argv[1]};
  return queue_job(env, NULL, argv[0], j, keep, 1, groups * (size_t)(pp->out_k + 1) * pp->out_N);
}

/* squash(squasher, engine, cts: B x 2049[, msgModulus = 16]) -> Promise<BigUint64Array> of B x (k N + 1) x 2
 * ((lo, hi) u64 per 128-bit word): keyswitch + modulus-switch noise reduction on the P-FHEVM engine, then the
 * squashing bootstrap */
static napi_value js_squash(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  aux_box* a = argc ? get_aux(env, argv[0], AUX_SNS) : NULL;
  ctx_box* b = argc > 1 ? get_box(env, argv[1]) : NULL;
  uint64_t* in;
  size_t n_in;
  uint32_t mm = 16;
  if (!a || !b || !b->ctx || b->destroy_requested || argc < 3 ||
      !get_typed(env, argv[2], napi_biguint64_array, (void**)&in, &n_in) ||
      (argc > 3 && napi_get_value_uint32(env, argv[3], &mm) != napi_ok)) {
    napi_throw_type_error(env, "EINVAL", "squash(squasher, engine, cts[, msgModulus])");
    return NULL;
  }
  if (b->p.order != 1 || b->p.n != a->sp.n) {
    napi_throw_type_error(env, "EINVAL", "squash: the engine must run the P-FHEVM (KS -> PBS) parameter set");
    return NULL;
  }
  const size_t big = (size_t)b->p.k * b->p.N + 1;
  if (!n_in || n_in % big) {
    napi_throw_range_error(env, "EINVAL", "squash: length is not a positive multiple of k*N + 1");
    return NULL;
  }
  /* the squashing LUT's own rule (tfhe_hip_sns_squash): checked here so a bad modulus throws before the
   * keyswitch and noise reduction are queued on the GPU */
  if (!mm || mm > a->sp.N || a->sp.N % mm) {
    napi_throw_range_error(env, "EINVAL", "squash: msgModulus must divide the squashing polynomial size N");
    return NULL;
  }
  job_t* j = (job_t*)calloc(1, sizeof(job_t));
  if (!j) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  j->kind = JOB_SQUASH;
  j->abox = a;
  j->in = in;
  j->B = n_in / big;
  j->msg_modulus = mm;
  napi_value keep[2] = {argv[0], argv[2]};  /* the squasher handle too: the engine is argv[1] */
  return queue_job(env, b, argv[1], j, keep, 2, j->B * ((size_t)a->sp.k * a->sp.N + 1) * 2);
}

/* extractGlwe(packed, bodies) -> BigUint64Array((k+1) N): the decompression of one compressed GLWE (host) */
static napi_value js_extract_glwe(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_pks_params pp;
  uint64_t *packed, *out;
  size_t n;
  uint32_t bodies;
  if (tfhe_hip_pks_params_preset(TFHE_HIP_PKS_PRESET_ML2048, &pp) || argc < 2 ||
      !get_typed(env, argv[0], napi_biguint64_array, (void**)&packed, &n) ||
      napi_get_value_uint32(env, argv[1], &bodies) != napi_ok || !bodies || bodies > pp.lwe_per_glwe ||
      n != tfhe_hip_pks_packed_words(&pp, bodies)) {
    napi_throw_type_error(env, "EINVAL", "extractGlwe(packed, bodies)");
    return NULL;
  }
  napi_value res = new_u64_array(env, (size_t)(pp.out_k + 1) * pp.out_N, &out);
  if (!res) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_pks_extract(&pp, packed, bodies, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

/* glwePhase(key, glwe) -> BigUint64Array(N): client-side phase of a native GLWE (k = key.length / N) */
static napi_value js_glwe_phase(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint64_t *key, *g, *out;
  size_t nk, ng;
  if (argc < 2 || !get_typed(env, argv[0], napi_biguint64_array, (void**)&key, &nk) ||
      !get_typed(env, argv[1], napi_biguint64_array, (void**)&g, &ng) || ng <= nk || ng % (ng - nk)) {
    napi_throw_type_error(env, "EINVAL", "glwePhase(key, glwe)");
    return NULL;
  }
  const size_t N = ng - nk, k = nk / N;
  napi_value res = new_u64_array(env, N, &out);
  if (!res) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_glwe_phase((uint32_t)k, (uint32_t)N, key, g, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

/* snsPhase(glweKey, cts) -> BigUint64Array of (lo, hi) phase pairs of squashed ciphertexts (client side) */
static napi_value js_sns_phase(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tfhe_sns_params sp;
  uint64_t *key, *c, *out;
  size_t nk, nc;
  if (tfhe_hip_sns_params_preset(TFHE_HIP_SNS_PRESET_FHEVM, &sp) || argc < 2 ||
      !get_typed(env, argv[0], napi_biguint64_array, (void**)&key, &nk) || nk != (size_t)sp.k * sp.N ||
      !get_typed(env, argv[1], napi_biguint64_array, (void**)&c, &nc) || nc % (2 * (nk + 1))) {
    napi_throw_type_error(env, "EINVAL", "snsPhase(glweKey, cts)");
    return NULL;
  }
  const size_t count = nc / (2 * (nk + 1));
  napi_value res = new_u64_array(env, 2 * count, &out);
  if (!res) return throw_tfhe(env, TFHE_HIP_ENOMEM);
  int rc = tfhe_hip_sns_phase(&sp, key, c, count, out);
  if (rc) return throw_tfhe(env, rc);
  return res;
}

static napi_value js_last_error(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value s;
  napi_create_string_utf8(env, tfhe_hip_last_error(), NAPI_AUTO_LENGTH, &s);
  return s;
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor d[] = {
      {"paramsPreset", 0, js_params_preset, 0, 0, 0, napi_enumerable, 0},
      {"keygen", 0, js_keygen, 0, 0, 0, napi_enumerable, 0},
      {"encrypt", 0, js_encrypt, 0, 0, 0, napi_enumerable, 0},
      {"phase", 0, js_phase, 0, 0, 0, napi_enumerable, 0},
      {"lutConstant", 0, js_lut_constant, 0, 0, 0, napi_enumerable, 0},
      {"lutFromTable", 0, js_lut_from_table, 0, 0, 0, napi_enumerable, 0},
      {"createEngine", 0, js_create, 0, 0, 0, napi_enumerable, 0},
      {"destroyEngine", 0, js_destroy, 0, 0, 0, napi_enumerable, 0},
      {"loadKeys", 0, js_load_keys, 0, 0, 0, napi_enumerable, 0},
      {"pbs", 0, js_pbs, 0, 0, 0, napi_enumerable, 0},
      {"nand", 0, js_nand, 0, 0, 0, napi_enumerable, 0},
      {"keyswitch", 0, js_keyswitch, 0, 0, 0, napi_enumerable, 0},
      {"blindRotate", 0, js_blind_rotate, 0, 0, 0, napi_enumerable, 0},
      {"engineInfo", 0, js_engine_info, 0, 0, 0, napi_enumerable, 0},
      {"lastError", 0, js_last_error, 0, 0, 0, napi_enumerable, 0},
      {"createPacker", 0, js_create_packer, 0, 0, 0, napi_enumerable, 0},
      {"createSquasher", 0, js_create_squasher, 0, 0, 0, napi_enumerable, 0},
      {"destroyAux", 0, js_destroy_aux, 0, 0, 0, napi_enumerable, 0},
      {"pksKeygen", 0, js_pks_keygen, 0, 0, 0, napi_enumerable, 0},
      {"snsKeygen", 0, js_sns_keygen, 0, 0, 0, napi_enumerable, 0},
      {"loadAuxKey", 0, js_load_aux_key, 0, 0, 0, napi_enumerable, 0},
      {"packCompress", 0, js_pack_compress, 0, 0, 0, napi_enumerable, 0},
      {"squash", 0, js_squash, 0, 0, 0, napi_enumerable, 0},
      {"extractGlwe", 0, js_extract_glwe, 0, 0, 0, napi_enumerable, 0},
      {"glwePhase", 0, js_glwe_phase, 0, 0, 0, napi_enumerable, 0},
      {"snsPhase", 0, js_sns_phase, 0, 0, 0, napi_enumerable, 0},
  };
  napi_define_properties(env, exports, sizeof(d) / sizeof(d[0]), d);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
