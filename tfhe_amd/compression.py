"""LWE -> GLWE packing keyswitch and modulus-switched ciphertext compression on the MI355X
(include/tfhe_hip.h tfhe_hip_pks_*; kernels tfhe_amd/csrc/pks.hip).

Mirrors the reference's compression surface (ml/extensions/rust/src/compression.rs):
  CompressionKey.new(input_lwe_secret_key, params) -> (post-packing GLWE key, key)   :159-187
  compress_ciphertexts_into_list(lwes) -> [CompressedGlwe]                           :246-291
  CompressedGlwe.extract() -> GLWE                                                   :134-156
with the packing keyswitch on the GPU (one integer GEMM + negacyclic shift-sum per chunk of GLWEs)
and the modulus switch / bit packing on the host.  Parameters: the reference's PARAMS_8B_2048_NEW
(ml/extensions/rust/src/fhext_classes.rs:98-112).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np

from . import RngKey, _c_u64, _check, _stream_handle, _u64, lib, rng_key

PKS_PRESET_ML2048 = 0
_U64P = ctypes.POINTER(ctypes.c_uint64)


class PksParams(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_uint32), ("out_k", ctypes.c_uint32), ("out_N", ctypes.c_uint32),
                ("base_log", ctypes.c_uint32), ("level", ctypes.c_uint32), ("lwe_per_glwe", ctypes.c_uint32),
                ("storage_log", ctypes.c_uint32), ("noise_log2", ctypes.c_int32)]

    @classmethod
    def preset(cls, which: int = PKS_PRESET_ML2048) -> "PksParams":
        p = cls()
        _check(_lib().tfhe_hip_pks_params_preset(which, ctypes.byref(p)))
        return p

    @property
    def glwe_len(self) -> int:
        return (self.out_k + 1) * self.out_N


_BOUND = None


def _lib():
    global _BOUND
    L = lib()
    if _BOUND is None:
        P = ctypes.POINTER(PksParams)
        L.tfhe_hip_pks_params_preset.argtypes = [ctypes.c_int, P]
        L.tfhe_hip_pksk_len.argtypes = [P]
        L.tfhe_hip_pksk_len.restype = ctypes.c_size_t
        L.tfhe_hip_pks_keygen.argtypes = [P, ctypes.c_uint64, _U64P, _U64P, _U64P]
        L.tfhe_hip_pks_keygen_k.argtypes = [P, ctypes.POINTER(RngKey), _U64P, _U64P, _U64P]
        L.tfhe_hip_pks_create.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.tfhe_hip_pks_destroy.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_pks_load_key.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t]
        L.tfhe_hip_pks_pack.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, _U64P]
        L.tfhe_hip_pks_pack_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                              ctypes.c_void_p]
        L.tfhe_hip_pks_packed_words.argtypes = [P, ctypes.c_uint32]
        L.tfhe_hip_pks_packed_words.restype = ctypes.c_size_t
        L.tfhe_hip_pks_compress.argtypes = [P, _U64P, ctypes.c_uint32, _U64P]
        L.tfhe_hip_pks_extract.argtypes = [P, _U64P, ctypes.c_uint32, _U64P]
        L.tfhe_hip_glwe_phase.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _U64P, _U64P, _U64P]
        _BOUND = True
    return L


class CompressionKey:
    """Packing keyswitching key from an input LWE key (e.g. a GLWE key read as an LWE key) to a fresh
    binary GLWE key (`post_packing_key`, held by the client for decryption)."""

    def __init__(self, params: PksParams, seed: Optional[int], in_key: np.ndarray, with_key: bool = True):
        L = _lib()
        self.params, self.seed = params, seed
        self.in_key = _c_u64(in_key)
        self.post_packing_key = np.zeros(params.out_k * params.out_N, dtype=np.uint64)
        self.pksk = np.zeros(L.tfhe_hip_pksk_len(ctypes.byref(params)), dtype=np.uint64) if with_key else None
        rk = rng_key(seed)  # None: 192 bits of OS entropy (production); an int: the public test stream
        _check(L.tfhe_hip_pks_keygen_k(ctypes.byref(params), ctypes.byref(rk), _u64(self.in_key), _u64(self.post_packing_key),
                                     _u64(self.pksk) if with_key else None))


class CompressedGlwe:
    """A modulus-switched, bit-packed GLWE holding `bodies` ciphertexts (compression.rs:134-156)."""

    def __init__(self, params: PksParams, packed: np.ndarray, bodies: int):
        self.params, self.packed, self.bodies = params, packed, bodies

    def extract(self) -> np.ndarray:
        out = np.zeros(self.params.glwe_len, dtype=np.uint64)
        _check(_lib().tfhe_hip_pks_extract(ctypes.byref(self.params), _u64(self.packed), self.bodies, _u64(out)))
        return out

    @property
    def nbytes(self) -> int:
        return self.packed.nbytes


def compress_glwe(params: PksParams, glwe: np.ndarray, bodies: int) -> CompressedGlwe:
    L = _lib()
    g = _c_u64(glwe)
    out = np.zeros(L.tfhe_hip_pks_packed_words(ctypes.byref(params), bodies), dtype=np.uint64)
    _check(L.tfhe_hip_pks_compress(ctypes.byref(params), _u64(g), bodies, _u64(out)))
    return CompressedGlwe(params, out, bodies)


def glwe_phase(k: int, N: int, key: np.ndarray, glwe: np.ndarray) -> np.ndarray:
    out = np.zeros(N, dtype=np.uint64)
    kk, g = _c_u64(key), _c_u64(glwe)
    _check(_lib().tfhe_hip_glwe_phase(k, N, _u64(kk), _u64(g), _u64(out)))
    return out


class Packer:
    """Device context for the packing keyswitch (one GPU)."""

    def __init__(self, params: PksParams, device: int = 0):
        self.params, self.device = params, device
        h = ctypes.c_void_p()
        _check(_lib().tfhe_hip_pks_create(ctypes.byref(params), device, ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib().tfhe_hip_pks_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_key(self, key: CompressionKey) -> "Packer":
        k = _c_u64(key.pksk)
        _check(_lib().tfhe_hip_pks_load_key(self._h, _u64(k), k.size))
        return self

    def pack(self, lwes: np.ndarray) -> np.ndarray:
        """count LWEs -> (ceil(count / lwe_per_glwe), (k+1)N) GLWEs."""
        p = self.params
        x = _c_u64(lwes).reshape(-1, p.in_dim + 1)
        groups = -(-x.shape[0] // p.lwe_per_glwe)
        out = np.zeros((groups, p.glwe_len), dtype=np.uint64)
        _check(_lib().tfhe_hip_pks_pack(self._h, _u64(x), x.shape[0], _u64(out)))
        return out

    def pack_async(self, d_lwes, count: int, d_glwes, stream=None) -> None:
        """torch device tensors (int64/uint64), enqueued on `stream` (torch.cuda.Stream, raw handle, or None =
        torch's current stream)."""
        _check(_lib().tfhe_hip_pks_pack_async(self._h, ctypes.c_void_p(d_lwes.data_ptr()), count,
                                              ctypes.c_void_p(d_glwes.data_ptr()),
                                              ctypes.c_void_p(_stream_handle(stream, self.device))))

    def compress_ciphertexts_into_list(self, lwes: np.ndarray) -> List[CompressedGlwe]:
        """compression.rs:246-291: pack chunks of lwe_per_glwe, then modulus-switch + bit-pack each."""
        p = self.params
        x = _c_u64(lwes).reshape(-1, p.in_dim + 1)
        glwes = self.pack(x)
        out = []
        for g in range(glwes.shape[0]):
            bodies = min(p.lwe_per_glwe, x.shape[0] - g * p.lwe_per_glwe)
            out.append(compress_glwe(p, glwes[g], bodies))
        return out


def extract_lwe(params: PksParams, glwe: np.ndarray, index: int) -> np.ndarray:
    """LWE (dim k*N, native q) of coefficient `index` of a GLWE (tfhe-rs extract_lwe_sample_from_glwe_
    ciphertext at MonomialDegree(index); the decompression path before its PBS)."""
    k, N = params.out_k, params.out_N
    g = np.asarray(glwe, dtype=np.uint64).reshape(k + 1, N)
    out = np.zeros(k * N + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for c in range(k):
            a = g[c]
            # a'_{cN + j} = a_c[index - j] for j <= index, -a_c[N + index - j] otherwise
            j = np.arange(N)
            src = index - j
            val = np.where(src >= 0, a[np.where(src >= 0, src, 0)], np.uint64(0) - a[np.where(src < 0, src + N, 0)])
            out[c * N:(c + 1) * N] = val
    out[-1] = g[k][index]
    return out
