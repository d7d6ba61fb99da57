"""Switch-and-squash: noise squashing of P-FHEVM ciphertexts into 128-bit LWEs on the MI355X
(include/tfhe_hip.h tfhe_hip_sns_*; kernels tfhe_amd/csrc/sns.hip).

fhEVM's sns-worker (coprocessor-docker-compose.yml:124-140) squashes each 64-bit ciphertext before
threshold decryption.  Here: `squash_noise(engine, squasher, cts)` = keyswitch to the small key and
modulus-switch noise reduction on the P-FHEVM engine, then the 128-bit bootstrap with the identity
LUT on the squasher; `SquashedKey.decrypt` recovers the message from the (k*N+1) x 128-bit LWE.
The GLWE ring is the native 2^128 torus, as in tfhe-rs: a coefficient is one u128 word, held as
(lo, hi) u64 pairs in the LWEs and as [lo][N], [hi][N] planes in keys and accumulators.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import RngKey, _c_u64, _check, _stream_handle, _u64, lib, rng_key

SNS_PRESET_FHEVM = 0
_U64P = ctypes.POINTER(ctypes.c_uint64)


class SnsParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("k", ctypes.c_uint32), ("N", ctypes.c_uint32), ("base_log", ctypes.c_uint32),
                ("level", ctypes.c_uint32), ("noise_log2", ctypes.c_int32)]

    @classmethod
    def preset(cls, which: int = SNS_PRESET_FHEVM) -> "SnsParams":
        p = cls()
        _check(_lib().tfhe_hip_sns_params_preset(which, ctypes.byref(p)))
        return p

    @property
    def out_dim(self) -> int:
        return self.k * self.N


_BOUND = None


def _lib():
    global _BOUND
    L = lib()
    if _BOUND is None:
        P = ctypes.POINTER(SnsParams)
        L.tfhe_hip_sns_params_preset.argtypes = [ctypes.c_int, P]
        L.tfhe_hip_sns_bsk_len.argtypes = [P]
        L.tfhe_hip_sns_bsk_len.restype = ctypes.c_size_t
        L.tfhe_hip_sns_keygen.argtypes = [P, ctypes.c_uint64, _U64P, _U64P, _U64P]
        L.tfhe_hip_sns_keygen_k.argtypes = [P, ctypes.POINTER(RngKey), _U64P, _U64P, _U64P]
        L.tfhe_hip_sns_create.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.tfhe_hip_sns_destroy.argtypes = [ctypes.c_void_p]
        L.tfhe_hip_sns_load_key.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t]
        L.tfhe_hip_sns_squash.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, ctypes.c_uint32, _U64P]
        L.tfhe_hip_sns_squash_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                ctypes.c_void_p, ctypes.c_void_p]
        L.tfhe_hip_sns_blind_rotate.argtypes = [ctypes.c_void_p, _U64P, ctypes.c_size_t, ctypes.c_uint32, _U64P]
        L.tfhe_hip_sns_phase.argtypes = [P, _U64P, _U64P, ctypes.c_size_t, _U64P]
        _BOUND = True
    return L


class SquashedKey:
    """128-bit GLWE key (client side) and the squashing BSK (server side) for a small LWE key."""

    def __init__(self, params: SnsParams, seed: Optional[int], lwe_key: np.ndarray, with_bsk: bool = True):
        L = _lib()
        self.params, self.seed = params, seed
        self.lwe_key = _c_u64(lwe_key)
        self.glwe_key = np.zeros(params.k * params.N, dtype=np.uint64)
        self.bsk = np.zeros(L.tfhe_hip_sns_bsk_len(ctypes.byref(params)), dtype=np.uint64) if with_bsk else None
        rk = rng_key(seed)  # None: 192 bits of OS entropy (production); an int: the public test stream
        _check(L.tfhe_hip_sns_keygen_k(ctypes.byref(params), ctypes.byref(rk), _u64(self.lwe_key), _u64(self.glwe_key),
                                     _u64(self.bsk) if with_bsk else None))

    def phase(self, cts: np.ndarray) -> list:
        p = self.params
        c = _c_u64(cts).reshape(-1, p.out_dim + 1, 2)
        out = np.zeros((c.shape[0], 2), dtype=np.uint64)
        _check(_lib().tfhe_hip_sns_phase(ctypes.byref(p), _u64(self.glwe_key), _u64(c), c.shape[0], _u64(out)))
        return [int(o[0]) | (int(o[1]) << 64) for o in out]

    def decrypt(self, cts: np.ndarray, msg_modulus: int = 16) -> np.ndarray:
        """round(phase / (2^127 / msg_modulus)) mod msg_modulus (one padding bit)."""
        delta = (1 << 127) // msg_modulus
        return np.array([((ph + delta // 2) // delta) % msg_modulus for ph in self.phase(cts)], dtype=np.uint64)


class Squasher:
    """Device context for noise squashing (one GPU)."""

    def __init__(self, params: SnsParams, device: int = 0):
        self.params, self.device = params, device
        h = ctypes.c_void_p()
        _check(_lib().tfhe_hip_sns_create(ctypes.byref(params), device, ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            _lib().tfhe_hip_sns_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_key(self, key: SquashedKey) -> "Squasher":
        b = _c_u64(key.bsk)
        _check(_lib().tfhe_hip_sns_load_key(self._h, _u64(b), b.size))
        return self

    def squash(self, small: np.ndarray, msg_modulus: int = 16) -> np.ndarray:
        """small-key ciphertexts (B x (n+1)) -> B x (k N + 1) x 2 u64 (128-bit LWEs, (lo, hi))."""
        p = self.params
        x = _c_u64(small).reshape(-1, p.n + 1)
        out = np.zeros((x.shape[0], p.out_dim + 1, 2), dtype=np.uint64)
        _check(_lib().tfhe_hip_sns_squash(self._h, _u64(x), x.shape[0], msg_modulus, _u64(out)))
        return out

    def squash_async(self, d_small, B: int, d_out, msg_modulus: int = 16, stream=None) -> None:
        _check(_lib().tfhe_hip_sns_squash_async(self._h, ctypes.c_void_p(d_small.data_ptr()), B, msg_modulus,
                                                ctypes.c_void_p(d_out.data_ptr()),
                                                ctypes.c_void_p(_stream_handle(stream, self.device))))

    def blind_rotate(self, small: np.ndarray, msg_modulus: int = 16) -> np.ndarray:
        p = self.params
        x = _c_u64(small).reshape(-1, p.n + 1)
        out = np.zeros((x.shape[0], p.k + 1, 2, p.N), dtype=np.uint64)
        _check(_lib().tfhe_hip_sns_blind_rotate(self._h, _u64(x), x.shape[0], msg_modulus, _u64(out)))
        return out


def squash_noise(engine, squasher: Squasher, cts: np.ndarray, msg_modulus: Optional[int] = None) -> np.ndarray:
    """P-FHEVM big-key ciphertexts -> squashed 128-bit LWEs: keyswitch + modulus-switch noise
    reduction (engine, KS -> PBS parameter set) then the 128-bit bootstrap (squasher)."""
    mm = msg_modulus or 16
    small = engine.keyswitch(cts)
    small, _ = engine.ms_reduce(small)
    return squasher.squash(small, mm)
