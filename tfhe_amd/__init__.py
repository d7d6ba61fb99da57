"""tfhe_amd — MI355X-native TFHE programmable bootstrapping, Python host side.

A thin ctypes layer over ``libtfhe_hip.so`` (C ABI: ``include/tfhe_hip.h``) plus a host-side
mirror of the reference's operator surface for this path:

* ``ClientKey`` / ``ServerKey`` / ``gen_keys`` — tfhe-rs ``gen_keys(PARAMS)`` as used by
  ``ml/biometrics/notebooks/main.rs:48`` and ``TfheClientKey.generate`` (sdk/relayer/src/tfhe.ts:20-28).
* ``Engine.generate_accumulator(f)`` + ``Engine.keyswitch_programmable_bootstrap(ct, acc)`` —
  ``ServerKey::generate_accumulator`` / ``keyswitch_programmable_bootstrap``
  (ml/biometrics/notebooks/main.rs:65-71), batched.
* ``FheBool`` gate bootstrapping (nand/and/or/xor/not) — the ``FheBool`` operator surface of
  packages/wasm (tfhe-rs high-level API) used by the Solidity ``fheBitAnd`` etc.
* ``FheUint8`` — 8 boolean ciphertexts; ``map_bits`` evaluates one LUT per bit (8 PBS / value).

Every compute call goes to the HIP library; there is no CPU fallback.  If the library is
missing the import of the engine raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, Optional, Sequence

import numpy as np

__all__ = [
    "Params", "TfheError", "lib", "ClientKey", "ServerKey", "gen_keys", "Engine", "FheBool", "FheUint8",
    "PRESET_GATE", "PRESET_FHEVM", "PRESET_GATE_FFT", "PRESET_FHEVM_FFT", "TRANSFORM_NTT", "TRANSFORM_FFT64", "MU", "encode_bool",
    "decode_bool",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# TFHE_HIP_LIB overrides the in-tree library (A/B builds of kernel variants in tools/ab.sh).
LIB_PATH = os.environ.get("TFHE_HIP_LIB") or os.path.join(_HERE, "libtfhe_hip.so")
PRESET_GATE = 0
PRESET_FHEVM = 1
PRESET_GATE_FFT = 2  # P-GATE on the FFT64 transform (tfhe-rs's f64-FFT external product)
PRESET_FHEVM_FFT = 3  # P-FHEVM on the FFT64 transform (N = 2048 as two 512-point halves)
TRANSFORM_NTT = 0
TRANSFORM_FFT64 = 1
MU = 1 << 61  # gate encoding: true = +1/8, false = -1/8 of the 2^64 torus
_U64P = ctypes.POINTER(ctypes.c_uint64)
_U32P = ctypes.POINTER(ctypes.c_uint32)

_ERRORS = {-1: "EINVAL", -2: "ENOMEM", -3: "EDEVICE", -4: "ENOKEYS", -5: "EUNSUPPORTED"}


class TfheError(RuntimeError):
    """Raised for a negative status from the C ABI (``code`` holds the TFHE_HIP_E* value)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{_ERRORS.get(code, code)}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32), ("k", ctypes.c_uint32), ("N", ctypes.c_uint32),
        ("pbs_base_log", ctypes.c_uint32), ("pbs_level", ctypes.c_uint32),
        ("ks_base_log", ctypes.c_uint32), ("ks_level", ctypes.c_uint32),
        ("lwe_noise_log2", ctypes.c_int32), ("glwe_noise_log2", ctypes.c_int32),
        ("order", ctypes.c_uint32), ("transform", ctypes.c_uint32),
    ]

    @classmethod
    def preset(cls, which: int = PRESET_GATE) -> "Params":
        p = cls()
        _check(lib().tfhe_hip_params_preset(which, ctypes.byref(p)))
        return p

    @property
    def io_dim(self) -> int:
        return self.n if self.order == 0 else self.k * self.N

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class RngKey(ctypes.Structure):
    """192-bit ChaCha20 key material (tfhe_rng_key)."""
    _fields_ = [("w", ctypes.c_uint32 * 6)]


def rng_key(seed: Optional[int] = None) -> RngKey:
    """seed None: 192 bits of OS entropy (production keys and encryptions); an int: the REPRODUCIBLE
    seeded stream that tests, golden vectors and the oracle use (public knowledge -- test data only)."""
    k = RngKey()
    if seed is None:
        _check(lib().tfhe_hip_rng_key_entropy(ctypes.byref(k)))
    else:
        _check(lib().tfhe_hip_rng_key_from_seed(ctypes.c_uint64(seed), ctypes.byref(k)))
    return k


_LIB = None

# Every symbol declared in include/tfhe_hip.h (tests check the .so exports all of them).
ABI_SYMBOLS = (
    "tfhe_hip_params_preset", "tfhe_hip_bsk_len", "tfhe_hip_ksk_len", "tfhe_hip_io_dim", "tfhe_hip_keygen",
    "tfhe_hip_lwe_encrypt", "tfhe_hip_lwe_phase", "tfhe_hip_lut_constant", "tfhe_hip_lut_from_table",
    "tfhe_hip_create", "tfhe_hip_destroy", "tfhe_hip_last_error", "tfhe_hip_device", "tfhe_hip_load_keys",
    "tfhe_hip_load_keys_device", "tfhe_hip_pbs", "tfhe_hip_pbs_async", "tfhe_hip_blind_rotate",
    "tfhe_hip_sample_extract", "tfhe_hip_keyswitch", "tfhe_hip_ntt_fwd", "tfhe_hip_ntt_inv", "tfhe_hip_nand",
    "tfhe_hip_sync", "tfhe_hip_timing_enable", "tfhe_hip_timing_reset", "tfhe_hip_timing_stats",
    "tfhe_hip_server_keygen", "tfhe_hip_set_latency_batch", "tfhe_hip_ms_zeros_keygen", "tfhe_hip_load_ms_key",
    "tfhe_hip_ms_reduce", "tfhe_hip_pks_params_preset", "tfhe_hip_pksk_len", "tfhe_hip_pks_keygen", "tfhe_hip_pks_keygen_k", "tfhe_hip_bcast_plan",
    "tfhe_hip_pks_create", "tfhe_hip_pks_destroy", "tfhe_hip_pks_load_key", "tfhe_hip_pks_pack",
    "tfhe_hip_pks_pack_async", "tfhe_hip_pks_packed_words", "tfhe_hip_pks_compress", "tfhe_hip_pks_extract",
    "tfhe_hip_glwe_phase", "tfhe_hip_sns_params_preset", "tfhe_hip_sns_bsk_len", "tfhe_hip_sns_keygen", "tfhe_hip_sns_keygen_k",
    "tfhe_hip_sns_create", "tfhe_hip_sns_destroy", "tfhe_hip_sns_load_key", "tfhe_hip_sns_squash",
    "tfhe_hip_sns_squash_async", "tfhe_hip_sns_blind_rotate", "tfhe_hip_sns_phase", "tfhe_hip_fft_fwd",
    "tfhe_hip_fft_inv", "tfhe_hip_rng_key_entropy", "tfhe_hip_rng_key_from_seed", "tfhe_hip_keygen_k",
    "tfhe_hip_server_keygen_k", "tfhe_hip_ms_zeros_keygen_k", "tfhe_hip_lwe_encrypt_k", "tfhe_hip_ndev",
    "tfhe_hip_device_at", "tfhe_hip_key_bcast_mode", "tfhe_hip_br_kernel", "tfhe_hip_aes128_block",
    "tfhe_hip_csprng_words", "tfhe_hip_seeded_server_keygen_k", "tfhe_hip_seeded_lwe_list_k", "tfhe_hip_decompress_bsk",
    "tfhe_hip_decompress_ksk", "tfhe_hip_decompress_lwe_list",
)

# P-FHEVM modulus-switch noise reduction key (include/tfhe_hip.h TFHE_HIP_MS_FHEVM_*)
MS_FHEVM = dict(count=1449, bound=2.0 ** 58, r_sigma=13.179852282053789, input_variance=2.63039184094559e-07)


def _share_hip_runtime_with_torch() -> None:
    """torch (ROCm wheel) bundles its own libamdhip64 (SONAME libamdhip64.so.7) and loads it by the
    unversioned file name.  If libtfhe_hip.so were loaded first, /opt/rocm's copy would come in under
    the same SONAME and torch would then load a SECOND HIP runtime into the process (torch.cuda then
    reports "No HIP GPUs are available").  Importing torch first makes our NEEDED libamdhip64.so.7
    resolve to the copy torch already loaded: one HIP runtime per process.  Without torch the
    library uses /opt/rocm's runtime (RUNPATH)."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libtfhe_hip.so (built in-tree by ``make -C tfhe_amd``).  Raises if it is missing."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `make -C tfhe_amd` (or __graft_entry__.build())")
        _share_hip_runtime_with_torch()
        L = ctypes.CDLL(LIB_PATH)
        L.tfhe_hip_last_error.restype = ctypes.c_char_p
        L.tfhe_hip_bsk_len.restype = ctypes.c_size_t
        L.tfhe_hip_ksk_len.restype = ctypes.c_size_t
        L.tfhe_hip_io_dim.restype = ctypes.c_uint32
        L.tfhe_hip_destroy.restype = None
        L.tfhe_hip_keygen.argtypes = [ctypes.c_void_p, ctypes.c_uint64, _U64P, _U64P, _U64P, _U64P]
        L.tfhe_hip_server_keygen.argtypes = [ctypes.c_void_p, ctypes.c_uint64, _U64P, _U64P, _U64P, _U64P]
        L.tfhe_hip_ms_zeros_keygen.argtypes = [ctypes.c_void_p, ctypes.c_uint64, _U64P, ctypes.c_uint32, _U64P]
        L.tfhe_hip_load_ms_key.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_uint32, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double]
        L.tfhe_hip_ms_reduce.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P,
                                         ctypes.POINTER(ctypes.c_int32)]
        L.tfhe_hip_lwe_encrypt.argtypes = [ctypes.c_uint32, _U64P, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint64,
                                           _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_lwe_phase.argtypes = [ctypes.c_uint32, _U64P, _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_lut_constant.argtypes = [ctypes.c_uint32, ctypes.c_uint64, _U64P]
        L.tfhe_hip_lut_from_table.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _U64P, ctypes.c_uint64, _U64P]
        L.tfhe_hip_create.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_void_p)]
        L.tfhe_hip_ndev.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_device_at.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.tfhe_hip_key_bcast_mode.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_br_kernel.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.tfhe_hip_br_kernel.restype = ctypes.c_char_p
        _RKP = ctypes.POINTER(RngKey)
        L.tfhe_hip_rng_key_entropy.argtypes = [_RKP]
        L.tfhe_hip_rng_key_from_seed.argtypes = [ctypes.c_uint64, _RKP]
        L.tfhe_hip_keygen_k.argtypes = [ctypes.c_void_p, _RKP, _U64P, _U64P, _U64P, _U64P]
        L.tfhe_hip_server_keygen_k.argtypes = [ctypes.c_void_p, _RKP, _U64P, _U64P, _U64P, _U64P]
        L.tfhe_hip_ms_zeros_keygen_k.argtypes = [ctypes.c_void_p, _RKP, _U64P, ctypes.c_uint32, _U64P]
        L.tfhe_hip_aes128_block.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p]
        L.tfhe_hip_csprng_words.argtypes = [_U64P, ctypes.c_uint64, ctypes.c_size_t, _U64P]
        L.tfhe_hip_seeded_server_keygen_k.argtypes = [ctypes.c_void_p, _RKP, _U64P, _U64P, _U64P, _U64P, _U64P, _U64P]
        L.tfhe_hip_seeded_lwe_list_k.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _U64P, ctypes.c_int32, _RKP,
                                                 ctypes.c_uint64, _U64P, _U64P, _U64P]
        L.tfhe_hip_decompress_bsk.argtypes = [ctypes.c_void_p, _U64P, _U64P, _U64P]
        L.tfhe_hip_decompress_ksk.argtypes = [ctypes.c_void_p, _U64P, _U64P, _U64P]
        L.tfhe_hip_decompress_lwe_list.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _U64P, _U64P, _U64P]
        L.tfhe_hip_lwe_encrypt_k.argtypes = [ctypes.c_uint32, _U64P, ctypes.c_int32, _RKP, ctypes.c_uint64, _U64P,
                                             ctypes.c_size_t, _U64P]
        L.tfhe_hip_destroy.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_load_keys.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P, ctypes.c_size_t]
        L.tfhe_hip_load_keys_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                ctypes.c_size_t]
        L.tfhe_hip_pbs.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P, ctypes.c_size_t, _U32P, _U64P]
        L.tfhe_hip_fft_fwd.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, ctypes.c_void_p]
        L.tfhe_hip_fft_inv.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.tfhe_hip_pbs_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.tfhe_hip_blind_rotate.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P, ctypes.c_size_t, _U32P,
                                            _U64P]
        L.tfhe_hip_sample_extract.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_keyswitch.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_ntt_fwd.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t]
        L.tfhe_hip_ntt_inv.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t]
        L.tfhe_hip_nand.argtypes = [ctypes.c_void_p, _U64P, _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_sync.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_timing_enable.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.tfhe_hip_timing_reset.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_timing_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_int)]
        L.tfhe_hip_device.argtypes = [ctypes.c_void_p]
        _LIB = L
    return _LIB


def source_id() -> str:
    """Content hash of everything that goes into libtfhe_hip.so (kernel + host sources, build flags,
    the ABI header).  Profiles under profiles/ carry the source_id of the tree they were measured on;
    bench.py only uses counter figures whose source_id equals the running tree's (a stale profile of
    another build is never reported as this build's)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(_HERE, "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc))
    files += [os.path.join(_HERE, "Makefile"), os.path.join(os.path.dirname(_HERE), "include", "tfhe_hip.h")]
    for f in files:
        h.update(os.path.relpath(f, os.path.dirname(_HERE)).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


NULL_STREAM = ctypes.c_void_p(-1).value  # TFHE_HIP_NULL_STREAM: the device's legacy null stream


def _stream_handle(stream, device: int) -> int:
    """torch.cuda.Stream / raw handle / None (torch's current stream) -> the C-ABI stream argument.
    torch's default stream has handle 0, which the C ABI reads as "ctx stream": map it to
    TFHE_HIP_NULL_STREAM so the work really is ordered with torch's default stream."""
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(device)
    h = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream or 0)
    return h if h else NULL_STREAM


def _check(rc: int) -> None:
    if rc != 0:
        raise TfheError(rc, lib().tfhe_hip_last_error().decode(errors="replace"))


def _u64(a: np.ndarray):
    return a.ctypes.data_as(_U64P)


def _c_u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


def encode_bool(b) -> np.ndarray:
    b = np.asarray(b, dtype=bool)
    return np.where(b, np.uint64(MU), np.uint64((1 << 64) - MU)).astype(np.uint64)


def decode_bool(phase) -> np.ndarray:
    return np.asarray(phase, dtype=np.uint64) < np.uint64(1 << 63)


# --------------------------------------------------------------------------------------- keys
class ClientKey:
    """Secret key material: LWE key s (dim n) and GLWE key S (k*N).  ``seed`` is the test seed the keys
    were derived from, or None for keys drawn from OS entropy."""

    def __init__(self, params: Params, seed: Optional[int], lwe_key: np.ndarray, glwe_key: np.ndarray):
        self.params, self.seed, self.lwe_key, self.glwe_key = params, seed, lwe_key, glwe_key

    # keys of the PBS input/output ciphertexts
    @property
    def io_key(self) -> np.ndarray:
        return self.lwe_key if self.params.order == 0 else self.glwe_key

    @property
    def io_noise_log2(self) -> int:
        return self.params.lwe_noise_log2 if self.params.order == 0 else self.params.glwe_noise_log2

    def encrypt_torus(self, msgs, seed: Optional[int] = None, stream0: int = 0) -> np.ndarray:
        """seed None (default): masks and noise from a fresh 192-bit OS-entropy ChaCha key per call;
        an int seed: the reproducible test stream (ciphertext q on stream stream0 + q)."""
        m = _c_u64(msgs).reshape(-1)
        dim = self.params.io_dim
        out = np.zeros((m.shape[0], dim + 1), dtype=np.uint64)
        key = _c_u64(self.io_key)
        rk = rng_key(seed)
        _check(lib().tfhe_hip_lwe_encrypt_k(dim, _u64(key), self.io_noise_log2, ctypes.byref(rk), stream0, _u64(m),
                                            m.shape[0], _u64(out)))
        return out

    def phase(self, cts: np.ndarray, key: Optional[np.ndarray] = None) -> np.ndarray:
        key = _c_u64(self.io_key if key is None else key)
        dim = key.shape[0]
        cts = _c_u64(cts).reshape(-1, dim + 1)
        out = np.zeros(cts.shape[0], dtype=np.uint64)
        _check(lib().tfhe_hip_lwe_phase(dim, _u64(key), _u64(cts), cts.shape[0], _u64(out)))
        return out

    def encrypt_bool(self, bits, seed: Optional[int] = None, stream0: int = 0) -> np.ndarray:
        return self.encrypt_torus(encode_bool(bits), seed, stream0)

    def decrypt_bool(self, cts) -> np.ndarray:
        return decode_bool(self.phase(cts))

    def encrypt(self, msgs, msg_modulus: int, seed: Optional[int] = None, stream0: int = 0) -> np.ndarray:
        """Shortint-style encoding with one padding bit: m * 2^63 / msg_modulus (encryption.rs:5-22)."""
        delta = (1 << 63) // msg_modulus
        m = (np.asarray(msgs, dtype=np.uint64) % np.uint64(msg_modulus)) * np.uint64(delta)
        return self.encrypt_torus(m, seed, stream0)

    def decrypt(self, cts, msg_modulus: int) -> np.ndarray:
        """closest_representable(phase) / delta mod msg_modulus (encryption.rs:176-203)."""
        delta = (1 << 63) // msg_modulus
        ph = self.phase(cts).astype(object)
        return np.array([((int(v) + delta // 2) // delta) % msg_modulus for v in ph], dtype=np.uint64)


class ServerKey:
    """Public evaluation keys in the standard domain: BSK over Z_p and KSK over Z_2^64; for KS -> PBS
    parameter sets (P-FHEVM) also the modulus-switch noise-reduction zeros (count x (n+1))."""

    def __init__(self, params: Params, bsk: np.ndarray, ksk: np.ndarray, ms_zeros: Optional[np.ndarray] = None):
        self.params, self.bsk, self.ksk, self.ms_zeros = params, bsk, ksk, ms_zeros


def ms_zeros_keygen(params: Params, seed: Optional[int], lwe_key: np.ndarray,
                    count: int = MS_FHEVM["count"]) -> np.ndarray:
    """Encryptions of zero under the small key for the modulus-switch noise reduction (seed None:
    OS entropy)."""
    z = np.zeros((count, params.n + 1), dtype=np.uint64)
    lwe = _c_u64(lwe_key)
    rk = rng_key(seed)
    _check(lib().tfhe_hip_ms_zeros_keygen_k(ctypes.byref(params), ctypes.byref(rk), _u64(lwe), count, _u64(z)))
    return z


def gen_keys(params: Optional[Params] = None, seed: Optional[int] = None, with_server_key: bool = True):
    """Key generation (tfhe-rs ``gen_keys`` analogue).  Returns (ClientKey, ServerKey).

    seed None (default): every key and the server-key randomness come from a fresh 192-bit OS-entropy
    ChaCha20 key.  An int seed gives the REPRODUCIBLE test key set (same streams as the oracle) --
    anyone who knows the seed knows the secret key, so seeded keys are for tests and benchmarks only."""
    params = params or Params.preset(PRESET_GATE)
    L = lib()
    lwe = np.zeros(params.n, dtype=np.uint64)
    glwe = np.zeros(params.k * params.N, dtype=np.uint64)
    bsk = ksk = None
    if with_server_key:
        bsk = np.zeros(L.tfhe_hip_bsk_len(ctypes.byref(params)), dtype=np.uint64)
        ksk = np.zeros(L.tfhe_hip_ksk_len(ctypes.byref(params)), dtype=np.uint64)
    rk = rng_key(seed)
    _check(L.tfhe_hip_keygen_k(ctypes.byref(params), ctypes.byref(rk), _u64(lwe), _u64(glwe),
                               _u64(bsk) if bsk is not None else None, _u64(ksk) if ksk is not None else None))
    ck = ClientKey(params, seed, lwe, glwe)
    if not with_server_key:
        return ck, None
    zeros = None
    if params.order == 1:
        zeros = np.zeros((MS_FHEVM["count"], params.n + 1), dtype=np.uint64)
        _check(L.tfhe_hip_ms_zeros_keygen_k(ctypes.byref(params), ctypes.byref(rk), _u64(lwe), zeros.shape[0],
                                            _u64(zeros)))
    return ck, ServerKey(params, bsk, ksk, zeros)


def server_keygen(ck: "ClientKey", seed: Optional[int] = None) -> ServerKey:
    """BSK / KSK (+ MS zeros) for the secret keys of ``ck`` (e.g. a tfhe-rs ClientKey ingested by
    tfhe_amd.keyio).  seed None (default): fresh 192-bit OS entropy, so the published evaluation keys
    reveal nothing reproducible; an int seed only for tests."""
    p = ck.params
    L = lib()
    bsk = np.zeros(L.tfhe_hip_bsk_len(ctypes.byref(p)), dtype=np.uint64)
    ksk = np.zeros(L.tfhe_hip_ksk_len(ctypes.byref(p)), dtype=np.uint64)
    lwe, glwe = _c_u64(ck.lwe_key), _c_u64(ck.glwe_key)
    rk = rng_key(seed)
    _check(L.tfhe_hip_server_keygen_k(ctypes.byref(p), ctypes.byref(rk), _u64(lwe), _u64(glwe), _u64(bsk), _u64(ksk)))
    zeros = None
    if p.order == 1:
        zeros = np.zeros((MS_FHEVM["count"], p.n + 1), dtype=np.uint64)
        _check(L.tfhe_hip_ms_zeros_keygen_k(ctypes.byref(p), ctypes.byref(rk), _u64(lwe), zeros.shape[0], _u64(zeros)))
    return ServerKey(p, bsk, ksk, zeros)


def lut_constant(N: int, torus_value: int) -> np.ndarray:
    out = np.zeros(N, dtype=np.uint64)
    _check(lib().tfhe_hip_lut_constant(N, torus_value, _u64(out)))
    return out


def lut_from_table(N: int, msg_modulus: int, table: Sequence[int], delta_out: int) -> np.ndarray:
    t = _c_u64([int(v) % (1 << 64) for v in table])
    out = np.zeros(N, dtype=np.uint64)
    _check(lib().tfhe_hip_lut_from_table(N, msg_modulus, _u64(t), delta_out, _u64(out)))
    return out


# ------------------------------------------------------------------------------------- engine
class Engine:
    """A device engine over one or more GPUs (``device``: an ordinal or a sequence of ordinals, one
    shard each; include/tfhe_hip.h).  Host-array batches split into per-device slices that run
    concurrently; keys are uploaded once and broadcast to every shard (RCCL for distinct ordinals).
    Mirrors the server-side operator surface of the path."""

    def __init__(self, params: Optional[Params] = None, device=0):
        self.params = params or Params.preset(PRESET_GATE)
        devs = [int(device)] if isinstance(device, (int, np.integer)) else [int(d) for d in device]
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_void_p()
        _check(lib().tfhe_hip_create(ctypes.byref(self.params), arr, len(devs), ctypes.byref(h)))
        self._h = h
        self.devices = devs
        self.device = devs[0]

    CUS_PER_DEVICE = 256  # MI355X; the fallback when the device cannot be queried

    @property
    def cus_per_device(self) -> int:
        """Compute units of the engine's first device (hipDeviceProp_t::multiProcessorCount, 256 on MI355X)."""
        if getattr(self, "_cus", None) is None:
            try:
                import torch
                self._cus = int(torch.cuda.get_device_properties(self.device).multi_processor_count)
            except Exception:  # noqa: BLE001 - no torch device view: the MI355X figure
                self._cus = self.CUS_PER_DEVICE
        return self._cus

    @property
    def round_size(self) -> int:
        """PBS one round of this engine's batch kernel holds across its shards (one workgroup per CU): 4
        ciphertexts per workgroup on the FFT64 kernels (N = 1024 component pairs, N = 2048 parity pairs) and on
        the N = 2048 NTT kernel, 8 on the N = 1024 NTT kernel.  The carry-out circuit's launch-round cost model
        (integer.Circuit) reads it."""
        per_wg = 8 if (self.params.transform == 0 and self.params.N == 1024) else 4
        return per_wg * self.cus_per_device * len(self.devices)

    @property
    def key_bcast_mode(self) -> str:
        return {0: "single", 1: "copy", 2: "rccl"}.get(lib().tfhe_hip_key_bcast_mode(self._h), "?")

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().tfhe_hip_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- keys -------------------------------------------------------------------------------
    def load_keys(self, sk: ServerKey) -> "Engine":
        bsk, ksk = _c_u64(sk.bsk), _c_u64(sk.ksk)
        _check(lib().tfhe_hip_load_keys(self._h, _u64(bsk), bsk.size, _u64(ksk), ksk.size))
        if getattr(sk, "ms_zeros", None) is not None:
            self.load_ms_key(sk.ms_zeros)
        return self

    def load_ms_key(self, zeros: Optional[np.ndarray], bound: float = MS_FHEVM["bound"],
                    r_sigma: float = MS_FHEVM["r_sigma"], input_variance: float = MS_FHEVM["input_variance"]):
        """Modulus-switch noise reduction between keyswitch and blind rotation (None: disable)."""
        if zeros is None:
            _check(lib().tfhe_hip_load_ms_key(self._h, None, 0, 0.0, 0.0, 0.0))
            return self
        z = _c_u64(zeros).reshape(-1, self.params.n + 1)
        _check(lib().tfhe_hip_load_ms_key(self._h, _u64(z), z.shape[0], bound, r_sigma, input_variance))
        return self

    def ms_reduce(self, small: np.ndarray):
        """Stage-level noise reduction on small-key ciphertexts -> (ciphertexts, chosen zero index or -1)."""
        x = _c_u64(small).reshape(-1, self.params.n + 1)
        out = np.zeros_like(x)
        picks = np.zeros(x.shape[0], dtype=np.int32)
        _check(lib().tfhe_hip_ms_reduce(self._h, _u64(x), x.shape[0], _u64(out),
                                        picks.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return out, picks

    def load_keys_device(self, d_bsk, d_ksk) -> "Engine":
        """Keys already in HBM on this device (torch tensors of dtype int64/uint64, e.g. after an
        RCCL broadcast)."""
        _check(lib().tfhe_hip_load_keys_device(self._h, ctypes.c_void_p(d_bsk.data_ptr()), d_bsk.numel(),
                                               ctypes.c_void_p(d_ksk.data_ptr()), d_ksk.numel()))
        return self

    # -- LUTs -------------------------------------------------------------------------------
    def generate_accumulator(self, f: Callable[[int], int], msg_modulus: int = 4,
                             delta_out: Optional[int] = None) -> np.ndarray:
        """tfhe-rs ServerKey::generate_accumulator (main.rs:65-68): LUT for m -> f(m)."""
        delta_out = delta_out if delta_out is not None else (1 << 63) // msg_modulus
        table = [f(m) % msg_modulus for m in range(msg_modulus)]
        return lut_from_table(self.params.N, msg_modulus, table, delta_out)

    def gate_lut(self) -> np.ndarray:
        return lut_constant(self.params.N, MU)

    # -- hot path ---------------------------------------------------------------------------
    def pbs(self, cts: np.ndarray, luts: np.ndarray, lut_index=None) -> np.ndarray:
        """Batched keyswitch_programmable_bootstrap over host arrays: (B, dim+1) -> (B, dim+1)."""
        dim = self.params.io_dim
        cts = _c_u64(cts).reshape(-1, dim + 1)
        luts = _c_u64(luts).reshape(-1, self.params.N)
        out = np.zeros_like(cts)
        li = None
        if lut_index is not None:
            li = np.ascontiguousarray(np.asarray(lut_index, dtype=np.uint32))
            if li.shape[0] != cts.shape[0]:
                raise ValueError("lut_index must have one entry per ciphertext")
        _check(lib().tfhe_hip_pbs(self._h, _u64(cts), cts.shape[0], _u64(luts), luts.shape[0],
                                  li.ctypes.data_as(_U32P) if li is not None else None, _u64(out)))
        return out

    def keyswitch_programmable_bootstrap(self, ct: np.ndarray, acc: np.ndarray) -> np.ndarray:
        return self.pbs(ct, acc)

    def pbs_async(self, d_in, d_luts, d_out, d_lut_index=None, stream=None) -> None:
        """Device-resident batch (torch tensors on this device), enqueued on ``stream``
        (a torch.cuda.Stream or raw handle; default torch's current stream if torch is loaded)."""
        B = d_in.shape[0]
        stream = _stream_handle(stream, self.device)
        n_lut = d_luts.numel() // self.params.N
        _check(lib().tfhe_hip_pbs_async(self._h, ctypes.c_void_p(d_in.data_ptr()), B,
                                        ctypes.c_void_p(d_luts.data_ptr()), n_lut,
                                        ctypes.c_void_p(d_lut_index.data_ptr()) if d_lut_index is not None else None,
                                        ctypes.c_void_p(d_out.data_ptr()), ctypes.c_void_p(stream)))

    def pbs_device(self, d_in, d_luts, d_lut_index=None):
        """pbs_async into a fresh tensor: (B, dim+1) int64 on this device -> the same shape, queued on torch's
        current stream (no host synchronisation)."""
        d_out = d_in.new_empty(d_in.shape)
        if d_in.shape[0]:
            self.pbs_async(d_in.contiguous(), d_luts, d_out, d_lut_index)
        return d_out

    def blind_rotate(self, cts: np.ndarray, luts: np.ndarray, lut_index=None) -> np.ndarray:
        p = self.params
        cts = _c_u64(cts).reshape(-1, p.n + 1)
        luts = _c_u64(luts).reshape(-1, p.N)
        out = np.zeros((cts.shape[0], (p.k + 1) * p.N), dtype=np.uint64)
        li = np.ascontiguousarray(np.asarray(lut_index, dtype=np.uint32)) if lut_index is not None else None
        _check(lib().tfhe_hip_blind_rotate(self._h, _u64(cts), cts.shape[0], _u64(luts), luts.shape[0],
                                           li.ctypes.data_as(_U32P) if li is not None else None, _u64(out)))
        return out

    def sample_extract(self, acc: np.ndarray) -> np.ndarray:
        p = self.params
        acc = _c_u64(acc).reshape(-1, (p.k + 1) * p.N)
        out = np.zeros((acc.shape[0], p.k * p.N + 1), dtype=np.uint64)
        _check(lib().tfhe_hip_sample_extract(self._h, _u64(acc), acc.shape[0], _u64(out)))
        return out

    def keyswitch(self, big: np.ndarray) -> np.ndarray:
        p = self.params
        big = _c_u64(big).reshape(-1, p.k * p.N + 1)
        out = np.zeros((big.shape[0], p.n + 1), dtype=np.uint64)
        _check(lib().tfhe_hip_keyswitch(self._h, _u64(big), big.shape[0], _u64(out)))
        return out

    def ntt_fwd(self, polys: np.ndarray) -> np.ndarray:
        x = _c_u64(polys).copy()
        _check(lib().tfhe_hip_ntt_fwd(self._h, _u64(x), x.size // self.params.N))
        return x

    def ntt_inv(self, polys: np.ndarray) -> np.ndarray:
        x = _c_u64(polys).copy()
        _check(lib().tfhe_hip_ntt_inv(self._h, _u64(x), x.size // self.params.N))
        return x

    def fft_fwd(self, polys: np.ndarray) -> np.ndarray:
        """FFT64 ctx: N torus values (read as int64) per polynomial -> N/2 complex128, natural order."""
        x = _c_u64(polys).reshape(-1, self.params.N)
        out = np.zeros((x.shape[0], self.params.N // 2), dtype=np.complex128)
        _check(lib().tfhe_hip_fft_fwd(self._h, _u64(x), x.shape[0], ctypes.c_void_p(out.ctypes.data)))
        return out

    def fft_inv(self, spec: np.ndarray) -> np.ndarray:
        """FFT64 ctx: N/2 complex -> N doubles (no 1/M, no rounding)."""
        z = np.ascontiguousarray(spec, dtype=np.complex128).reshape(-1, self.params.N // 2)
        out = np.zeros((z.shape[0], self.params.N), dtype=np.float64)
        _check(lib().tfhe_hip_fft_inv(self._h, ctypes.c_void_p(z.ctypes.data), z.shape[0],
                                      ctypes.c_void_p(out.ctypes.data)))
        return out

    def nand(self, c1: np.ndarray, c2: np.ndarray) -> np.ndarray:
        dim = self.params.n + 1
        c1, c2 = _c_u64(c1).reshape(-1, dim), _c_u64(c2).reshape(-1, dim)
        out = np.zeros_like(c1)
        _check(lib().tfhe_hip_nand(self._h, _u64(c1), _u64(c2), c1.shape[0], _u64(out)))
        return out

    def sync(self) -> None:
        _check(lib().tfhe_hip_sync(self._h))

    def set_latency_batch(self, max_batch: int) -> None:
        """Batches up to ``max_batch`` use the latency blind-rotate kernel (0: always the batch kernel)."""
        _check(lib().tfhe_hip_set_latency_batch(self._h, ctypes.c_size_t(max_batch)))

    def br_kernel(self, batch: int) -> str:
        """Name of the blind-rotate kernel the dispatch launches for a per-shard batch of ``batch``."""
        return lib().tfhe_hip_br_kernel(self._h, ctypes.c_size_t(batch)).decode()

    # -- timing (HIP events around each kernel launch) -----------------------------------------
    def timing(self, enable: bool = True) -> None:
        _check(lib().tfhe_hip_timing_enable(self._h, 1 if enable else 0))

    def timing_reset(self) -> None:
        _check(lib().tfhe_hip_timing_reset(self._h))

    def timing_stats(self, which: int = 0):
        ms, cnt = ctypes.c_double(), ctypes.c_int()
        _check(lib().tfhe_hip_timing_stats(self._h, which, ctypes.byref(ms), ctypes.byref(cnt)))
        return ms.value, cnt.value


# ------------------------------------------------------------------------------ FheBool / FheUint8
def _gate_lin(c1: np.ndarray, c2: Optional[np.ndarray], k1: int, k2: int, const: int) -> np.ndarray:
    """(0, const) + k1*c1 + k2*c2 over Z_2^64 (TFHE-lib gate linear parts)."""
    with np.errstate(over="ignore"):
        out = c1 * np.uint64(k1 % (1 << 64))
        if c2 is not None:
            out = out + c2 * np.uint64(k2 % (1 << 64))
        out[..., -1] = out[..., -1] + np.uint64(const % (1 << 64))
    return out


class FheBool:
    """Encrypted booleans (a batch), gate-bootstrapped on the GPU.  NOT is free (negation)."""

    def __init__(self, engine: Engine, ct: np.ndarray):
        self.engine, self.ct = engine, _c_u64(ct).reshape(-1, engine.params.n + 1)

    @classmethod
    def encrypt(cls, values, ck: ClientKey, engine: Engine, seed: Optional[int] = None, stream0: int = 0) -> "FheBool":
        return cls(engine, ck.encrypt_bool(np.atleast_1d(values), seed, stream0))

    def decrypt(self, ck: ClientKey) -> np.ndarray:
        return ck.decrypt_bool(self.ct)

    def _boot(self, lin: np.ndarray) -> "FheBool":
        return FheBool(self.engine, self.engine.pbs(lin, self.engine.gate_lut()))

    def nand(self, other: "FheBool") -> "FheBool":
        return FheBool(self.engine, self.engine.nand(self.ct, other.ct))

    def __and__(self, other: "FheBool") -> "FheBool":
        return self._boot(_gate_lin(self.ct, other.ct, 1, 1, -MU))

    def __or__(self, other: "FheBool") -> "FheBool":
        return self._boot(_gate_lin(self.ct, other.ct, 1, 1, MU))

    def __xor__(self, other: "FheBool") -> "FheBool":
        return self._boot(_gate_lin(self.ct, other.ct, 2, 2, 2 * MU))

    def __invert__(self) -> "FheBool":
        with np.errstate(over="ignore"):
            return FheBool(self.engine, (np.uint64(0) - self.ct).astype(np.uint64))


class FheUint8:
    """Encrypted 8-bit unsigned integers as 8 gate-encoded bits (LSB first): shape (B, 8, n+1)."""

    def __init__(self, engine: Engine, bits: np.ndarray):
        self.engine = engine
        self.bits = _c_u64(bits).reshape(-1, 8, engine.params.n + 1)

    @classmethod
    def encrypt(cls, values, ck: ClientKey, engine: Engine, seed: Optional[int] = None, stream0: int = 0) -> "FheUint8":
        v = np.atleast_1d(np.asarray(values, dtype=np.uint64))
        bits = ((v[:, None] >> np.arange(8, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
        return cls(engine, ck.encrypt_bool(bits.reshape(-1), seed, stream0))

    def decrypt(self, ck: ClientKey) -> np.ndarray:
        b = ck.decrypt_bool(self.bits.reshape(-1, self.engine.params.n + 1)).reshape(-1, 8).astype(np.uint64)
        return (b << np.arange(8, dtype=np.uint64)[None, :]).sum(axis=1).astype(np.uint64)

    def map_bits(self, luts: np.ndarray) -> "FheUint8":
        """Bootstrap every bit with its own LUT (luts: 8 x N; bit j uses LUT j): 8 PBS per value."""
        B = self.bits.shape[0]
        idx = np.tile(np.arange(8, dtype=np.uint32), B)
        out = self.engine.pbs(self.bits.reshape(B * 8, -1), luts, idx)
        return FheUint8(self.engine, out)

    def refresh(self) -> "FheUint8":
        """Identity bootstrap of every bit (noise refresh)."""
        return self.map_bits(np.tile(self.engine.gate_lut(), (8, 1)))
