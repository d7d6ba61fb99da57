"""ctypes binding for the CPU oracle (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product (tfhe_amd/, js/).  See tfhe_oracle.h for the
reference file:line each function restates and the "parity unpinned" statement.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P = 0xFFFFFFFF00000001
U64P = ctypes.POINTER(ctypes.c_uint64)
U32P = ctypes.POINTER(ctypes.c_uint32)
I64P = ctypes.POINTER(ctypes.c_int64)


class Params(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32), ("k", ctypes.c_uint32), ("N", ctypes.c_uint32),
        ("pbs_base_log", ctypes.c_uint32), ("pbs_level", ctypes.c_uint32),
        ("ks_base_log", ctypes.c_uint32), ("ks_level", ctypes.c_uint32),
        ("lwe_noise_log2", ctypes.c_int32), ("glwe_noise_log2", ctypes.c_int32),
        ("order", ctypes.c_uint32), ("transform", ctypes.c_uint32),
    ]


class MsKey(ctypes.Structure):
    _fields_ = [("zeros", ctypes.c_void_p), ("count", ctypes.c_uint32), ("bound", ctypes.c_double),
                ("r_sigma", ctypes.c_double), ("input_variance", ctypes.c_double)]


# P-FHEVM modulus-switch noise reduction (tfhe_oracle.h: or_ms_key)
MS_FHEVM = dict(count=1449, bound=2.0 ** 58, r_sigma=13.179852282053789, input_variance=2.63039184094559e-07)


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.or_rng_u64.restype = ctypes.c_uint64
        L.or_rng_mod_p.restype = ctypes.c_uint64
        L.or_rng_gauss.restype = ctypes.c_int64
        L.or_add.restype = ctypes.c_uint64
        L.or_sub.restype = ctypes.c_uint64
        L.or_mul.restype = ctypes.c_uint64
        L.or_mul.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_pow.restype = ctypes.c_uint64
        L.or_pow.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_psi.restype = ctypes.c_uint64
        L.or_tor_to_p.restype = ctypes.c_uint64
        L.or_tor_to_p.argtypes = [ctypes.c_uint64]
        L.or_p_to_tor.restype = ctypes.c_uint64
        L.or_p_to_tor.argtypes = [ctypes.c_uint64]
        L.or_mod_switch.restype = ctypes.c_uint32
        L.or_mod_switch.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
        L.or_ms_measure.restype = ctypes.c_double
        L.or_ms_measure.argtypes = [ctypes.c_void_p, ctypes.c_void_p, U64P, U64P]
        L.or_ms_reduce.restype = ctypes.c_int
        L.or_bsk_len.restype = ctypes.c_size_t
        L.or_ksk_len.restype = ctypes.c_size_t
        L.or_f64_to_torus.restype = ctypes.c_uint64
        L.or_f64_to_torus.argtypes = [ctypes.c_double]
        L.or_f64_to_torus_dev.restype = ctypes.c_uint64
        L.or_f64_to_torus_dev.argtypes = [ctypes.c_double]
        if os.environ.get("ORACLE_FFT2K_SPLIT") == "1":  # A/B of the N = 2048 MAC order (fft_oracle.c)
            L.or_set_fft2k_mac_split(1)
        _LIB = L
    return _LIB


def _p(a: np.ndarray, t=U64P):
    return a.ctypes.data_as(t)


def params(preset: int = 0) -> Params:
    p = Params()
    assert lib().or_params_preset(preset, ctypes.byref(p)) == 0
    return p


class Rng:
    def __init__(self, seed: int, stream: int):
        self.buf = (ctypes.c_uint8 * 128)()
        lib().or_rng_init(self.buf, ctypes.c_uint64(seed), ctypes.c_uint64(stream))

    def u64(self) -> int:
        return lib().or_rng_u64(self.buf)


def ntt_fwd(a: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(a, dtype=np.uint64).copy()
    for row in x.reshape(-1, x.shape[-1]):
        lib().or_ntt_fwd(_p(row), ctypes.c_uint32(x.shape[-1]))
    return x


def ntt_inv(a: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(a, dtype=np.uint64).copy()
    for row in x.reshape(-1, x.shape[-1]):
        lib().or_ntt_inv(_p(row), ctypes.c_uint32(x.shape[-1]))
    return x


def poly_mul_schoolbook(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros_like(a)
    lib().or_poly_mul_schoolbook(_p(out), _p(a), _p(b), ctypes.c_uint32(a.shape[0]))
    return out


def poly_mul_ntt(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros_like(a)
    lib().or_poly_mul_ntt(_p(out), _p(a), _p(b), ctypes.c_uint32(a.shape[0]))
    return out


def decompose(x: int, base_log: int, level: int) -> list[int]:
    d = np.zeros(64, dtype=np.int64)
    lib().or_decompose(ctypes.c_uint64(x), ctypes.c_uint32(base_log), ctypes.c_uint32(level), _p(d, I64P))
    return [int(v) for v in d[:level]]


def psi(N: int) -> int:
    return lib().or_psi(ctypes.c_uint32(N))


class Keys:
    """Oracle key material generated from a seed (same ChaCha20 streams as the product keygen)."""

    def __init__(self, prm: Params, seed: int, with_bsk: bool = True, with_ksk: bool = True):
        L = lib()
        self.prm = prm
        self.seed = seed
        self.lwe_key = np.zeros(prm.n, dtype=np.uint64)
        self.glwe_key = np.zeros(prm.k * prm.N, dtype=np.uint64)
        self.bsk = np.zeros(L.or_bsk_len(ctypes.byref(prm)), dtype=np.uint64) if with_bsk else None
        self.ksk = np.zeros(L.or_ksk_len(ctypes.byref(prm)), dtype=np.uint64) if with_ksk else None
        L.or_keygen(ctypes.byref(prm), ctypes.c_uint64(seed), _p(self.lwe_key), _p(self.glwe_key),
                    _p(self.bsk) if with_bsk else None, _p(self.ksk) if with_ksk else None)
        self._bsk_ntt = None
        self._ms_zeros_keygen()

    def _ms_zeros_keygen(self):
        """P-FHEVM (KS -> PBS) server keys carry the modulus-switch zeros; P-GATE none."""
        self.ms_zeros = None
        if self.prm.order == 1:
            self.ms_zeros = np.zeros((MS_FHEVM["count"], self.prm.n + 1), dtype=np.uint64)
            lib().or_ms_zeros_keygen(ctypes.byref(self.prm), ctypes.c_uint64(self.seed), _p(self.lwe_key),
                                     ctypes.c_uint32(MS_FHEVM["count"]), _p(self.ms_zeros))

    def ms_key(self, enabled: bool = True):
        if not enabled or self.ms_zeros is None:
            return None
        k = MsKey(self.ms_zeros.ctypes.data, self.ms_zeros.shape[0], MS_FHEVM["bound"], MS_FHEVM["r_sigma"],
                  MS_FHEVM["input_variance"])
        k._keep = self.ms_zeros
        return k

    @classmethod
    def from_secret(cls, prm: Params, seed: int, lwe_key: np.ndarray, glwe_key: np.ndarray) -> "Keys":
        """Server keys for given secret keys (or_server_keygen; same streams as the seeded keygen)."""
        k = cls.__new__(cls)
        k.prm, k.seed = prm, seed
        k.lwe_key = np.ascontiguousarray(lwe_key, dtype=np.uint64).copy()
        k.glwe_key = np.ascontiguousarray(glwe_key, dtype=np.uint64).copy()
        L = lib()
        k.bsk = np.zeros(L.or_bsk_len(ctypes.byref(prm)), dtype=np.uint64)
        k.ksk = np.zeros(L.or_ksk_len(ctypes.byref(prm)), dtype=np.uint64)
        L.or_server_keygen(ctypes.byref(prm), ctypes.c_uint64(seed), _p(k.lwe_key), _p(k.glwe_key), _p(k.bsk),
                           _p(k.ksk))
        k._bsk_ntt = None
        k._ms_zeros_keygen()
        return k

    @property
    def bsk_ntt(self) -> np.ndarray:
        if self._bsk_ntt is None:
            self._bsk_ntt = np.zeros_like(self.bsk)
            lib().or_bsk_to_ntt(ctypes.byref(self.prm), _p(self.bsk), _p(self._bsk_ntt))
        return self._bsk_ntt

    @property
    def bsk_fourier(self) -> np.ndarray:
        """FFT64 transform: Fourier-domain BSK, complex128 [polys][N/2] (or_bsk_to_fourier)."""
        if getattr(self, "_bsk_f", None) is None:
            self._bsk_f = np.zeros((self.bsk.size // self.prm.N, self.prm.N // 2), dtype=np.complex128)
            lib().or_bsk_to_fourier(ctypes.byref(self.prm), _p(self.bsk), _p(self._bsk_f, ctypes.c_void_p))
        return self._bsk_f

    # --- encryption under the input-side key (small key for PBS_KS order, big for KS_PBS) ---
    def in_key(self):
        return (self.lwe_key, self.prm.n) if self.prm.order == 0 else (self.glwe_key, self.prm.k * self.prm.N)

    def out_key(self):
        return self.in_key()

    def encrypt(self, msgs_torus, seed: int, stream0: int = 0) -> np.ndarray:
        key, dim = self.in_key()
        noise = self.prm.lwe_noise_log2 if self.prm.order == 0 else self.prm.glwe_noise_log2
        m = np.ascontiguousarray(np.asarray(msgs_torus, dtype=np.uint64))
        out = np.zeros((m.shape[0], dim + 1), dtype=np.uint64)
        lib().or_lwe_encrypt(ctypes.c_uint32(dim), _p(key), ctypes.c_int32(noise), ctypes.c_uint64(seed),
                             ctypes.c_uint64(stream0), _p(m), ctypes.c_size_t(m.shape[0]), _p(out))
        return out

    def phase(self, cts: np.ndarray, key=None, dim=None) -> np.ndarray:
        if key is None:
            key, dim = self.out_key()
        cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, dim + 1)
        out = np.zeros(cts.shape[0], dtype=np.uint64)
        lib().or_lwe_phase(ctypes.c_uint32(dim), _p(key), _p(cts), ctypes.c_size_t(cts.shape[0]), _p(out))
        return out


def blind_rotate(prm: Params, keys: Keys, lwe_in: np.ndarray, lut: np.ndarray, schoolbook=False) -> np.ndarray:
    acc = np.zeros((prm.k + 1) * prm.N, dtype=np.uint64)
    bsk = keys.bsk if schoolbook else keys.bsk_ntt
    lib().or_blind_rotate(ctypes.byref(prm), _p(bsk), ctypes.c_int(1 if schoolbook else 0),
                          _p(np.ascontiguousarray(lwe_in, dtype=np.uint64)),
                          _p(np.ascontiguousarray(lut, dtype=np.uint64)), _p(acc))
    return acc


def sample_extract(prm: Params, acc: np.ndarray) -> np.ndarray:
    out = np.zeros(prm.k * prm.N + 1, dtype=np.uint64)
    lib().or_sample_extract(ctypes.byref(prm), _p(np.ascontiguousarray(acc, dtype=np.uint64)), _p(out))
    return out


def keyswitch(prm: Params, keys: Keys, lwe_big: np.ndarray) -> np.ndarray:
    out = np.zeros(prm.n + 1, dtype=np.uint64)
    lib().or_keyswitch(ctypes.byref(prm), _p(keys.ksk), _p(np.ascontiguousarray(lwe_big, dtype=np.uint64)), _p(out))
    return out


def ms_measure(prm: Params, keys: Keys, ct: np.ndarray, zero_index=None) -> float:
    ms = keys.ms_key()
    ct = np.ascontiguousarray(ct, dtype=np.uint64)
    z = None if zero_index is None else _p(np.ascontiguousarray(keys.ms_zeros[zero_index]))
    return lib().or_ms_measure(ctypes.byref(prm), ctypes.byref(ms), _p(ct), z)


def ms_reduce(prm: Params, keys: Keys, small: np.ndarray):
    """-> (reduced ciphertexts, chosen zero index per ciphertext or -1)"""
    ms = keys.ms_key()
    out = np.ascontiguousarray(small, dtype=np.uint64).reshape(-1, prm.n + 1).copy()
    picks = np.array([lib().or_ms_reduce(ctypes.byref(prm), ctypes.byref(ms), _p(out[i])) for i in range(out.shape[0])],
                     dtype=np.int64)
    return out, picks


def pbs_batch(prm: Params, keys: Keys, lwe_in: np.ndarray, luts: np.ndarray, lut_index=None,
              threads: int = 0, ms: bool = True) -> np.ndarray:
    if prm.transform == 1:
        return pbs_batch_fft(prm, keys, lwe_in, luts, lut_index, threads, ms)
    lwe_in = np.ascontiguousarray(lwe_in, dtype=np.uint64)
    luts = np.ascontiguousarray(luts, dtype=np.uint64).reshape(-1, prm.N)
    B = lwe_in.shape[0]
    dout = (prm.n if prm.order == 0 else prm.k * prm.N) + 1
    out = np.zeros((B, dout), dtype=np.uint64)
    li = None
    if lut_index is not None:
        li = np.ascontiguousarray(lut_index, dtype=np.uint32)
    msk = keys.ms_key(ms)
    lib().or_pbs_batch_ex(ctypes.byref(prm), _p(keys.bsk_ntt), _p(keys.ksk), ctypes.byref(msk) if msk else None,
                       _p(lwe_in), ctypes.c_size_t(B),
                       _p(luts), ctypes.c_size_t(luts.shape[0]), _p(li, U32P) if li is not None else None,
                       _p(out), ctypes.c_int(threads))
    return out


# ---- FFT64 transform (fft_oracle.c) -----------------------------------------------------------------
def fft_fwd(a) -> np.ndarray:
    """N real values (exact doubles, e.g. digits or int64 torus values) -> N/2 complex128."""
    a = np.ascontiguousarray(a, dtype=np.float64).reshape(-1, np.shape(a)[-1])
    N = a.shape[1]
    out = np.zeros((a.shape[0], N // 2), dtype=np.complex128)
    for i in range(a.shape[0]):
        lib().or_fft_fwd(_p(a[i], ctypes.c_void_p), ctypes.c_uint32(N), _p(out[i], ctypes.c_void_p))
    return out


def fft_inv(z) -> np.ndarray:
    """N/2 complex -> N doubles, without the 1/M factor and without rounding."""
    z = np.ascontiguousarray(z, dtype=np.complex128).reshape(-1, np.shape(z)[-1])
    N = 2 * z.shape[1]
    out = np.zeros((z.shape[0], N), dtype=np.float64)
    for i in range(z.shape[0]):
        lib().or_fft_inv(_p(z[i], ctypes.c_void_p), ctypes.c_uint32(N), _p(out[i], ctypes.c_void_p))
    return out


def f64_to_torus(x: float) -> int:
    return int(lib().or_f64_to_torus(float(x)))


def f64_to_torus_dev(x: float) -> int:
    """the device's accumulator increment (fft512.h torus_acc_add): rint(x) mod 2^64 but for tiny negative x"""
    return int(lib().or_f64_to_torus_dev(float(x)))


def fft_twiddle(t: int, M: int) -> tuple:
    c, s = ctypes.c_double(), ctypes.c_double()
    lib().or_fft_twiddle(ctypes.c_uint32(t), ctypes.c_uint32(M), ctypes.byref(c), ctypes.byref(s))
    return c.value, s.value


def poly_mul_torus_schoolbook(a_small, b) -> np.ndarray:
    a = np.ascontiguousarray(a_small, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros(b.shape[0], dtype=np.uint64)
    lib().or_poly_mul_torus_schoolbook(_p(out), _p(a, I64P), _p(b), ctypes.c_uint32(b.shape[0]))
    return out


def blind_rotate_fft(prm: Params, keys: Keys, lwe_in: np.ndarray, lut: np.ndarray) -> np.ndarray:
    acc = np.zeros((prm.k + 1) * prm.N, dtype=np.uint64)
    lib().or_blind_rotate_fft(ctypes.byref(prm), _p(keys.bsk_fourier, ctypes.c_void_p),
                              _p(np.ascontiguousarray(lwe_in, dtype=np.uint64)),
                              _p(np.ascontiguousarray(lut, dtype=np.uint64)), _p(acc))
    return acc


def sample_extract_torus(prm: Params, acc: np.ndarray) -> np.ndarray:
    out = np.zeros(prm.k * prm.N + 1, dtype=np.uint64)
    lib().or_sample_extract_torus(ctypes.byref(prm), _p(np.ascontiguousarray(acc, dtype=np.uint64)), _p(out))
    return out


def pbs_batch_fft(prm: Params, keys: Keys, lwe_in: np.ndarray, luts: np.ndarray, lut_index=None,
                  threads: int = 0, ms: bool = True) -> np.ndarray:
    """FFT64 PBS (or_pbs_batch_fft_ex): P-GATE BR -> SE -> KS, P-FHEVM KS -> MS -> BR -> SE."""
    lwe_in = np.ascontiguousarray(lwe_in, dtype=np.uint64)
    luts = np.ascontiguousarray(luts, dtype=np.uint64).reshape(-1, prm.N)
    B = lwe_in.shape[0]
    dout = (prm.n if prm.order == 0 else prm.k * prm.N) + 1
    out = np.zeros((B, dout), dtype=np.uint64)
    li = np.ascontiguousarray(lut_index, dtype=np.uint32) if lut_index is not None else None
    msk = keys.ms_key(ms)
    lib().or_pbs_batch_fft_ex(ctypes.byref(prm), _p(keys.bsk_fourier, ctypes.c_void_p), _p(keys.ksk),
                              ctypes.byref(msk) if msk else None, _p(lwe_in),
                              ctypes.c_size_t(B), _p(luts), ctypes.c_size_t(luts.shape[0]),
                              _p(li, U32P) if li is not None else None, _p(out), ctypes.c_int(threads))
    return out


def pbs_batch_fft_simd(prm: Params, keys: Keys, lwe_in: np.ndarray, luts: np.ndarray, lut_index=None,
                       threads: int = 0, ms: bool = True) -> np.ndarray:
    """FFT64 PBS with 8 (AVX-512) or 4 (AVX2) ciphertexts per vector (fft_batch.c): bit-identical to pbs_batch_fft
    at P-GATE (BR -> SE -> KS) and P-FHEVM (KS -> MS -> BR -> SE); the CPU port bench.py times.  Other parameter sets
    raise ValueError."""
    lwe_in = np.ascontiguousarray(lwe_in, dtype=np.uint64)
    luts = np.ascontiguousarray(luts, dtype=np.uint64).reshape(-1, prm.N)
    B = lwe_in.shape[0]
    dout = (prm.n if prm.order == 0 else prm.k * prm.N) + 1
    out = np.zeros((B, dout), dtype=np.uint64)
    li = np.ascontiguousarray(lut_index, dtype=np.uint32) if lut_index is not None else None
    msk = keys.ms_key(ms)
    rc = lib().or_pbs_batch_fft_simd_ex(ctypes.byref(prm), _p(keys.bsk_fourier, ctypes.c_void_p), _p(keys.ksk),
                                        ctypes.byref(msk) if msk else None, _p(lwe_in), ctypes.c_size_t(B), _p(luts),
                                        ctypes.c_size_t(luts.shape[0]), _p(li, U32P) if li is not None else None,
                                        _p(out), ctypes.c_int(threads))
    if rc != 0:
        raise ValueError("or_pbs_batch_fft_simd_ex: the FFT64 presets (P-GATE, P-FHEVM) only")
    return out


def simd_lanes() -> int:
    """Ciphertexts per vector of pbs_batch_fft_simd on this CPU: 8 (AVX-512F) or 4 (AVX2 / ORACLE_SIMD_LANES=4)."""
    return int(lib().or_fft_batch_lanes())


def lut_constant(N: int, torus_value: int) -> np.ndarray:
    out = np.zeros(N, dtype=np.uint64)
    lib().or_lut_constant(ctypes.c_uint32(N), ctypes.c_uint64(torus_value), _p(out))
    return out


def lut_from_table(N: int, msg_modulus: int, table, delta_out: int) -> np.ndarray:
    t = np.ascontiguousarray(np.asarray(table, dtype=np.uint64))
    out = np.zeros(N, dtype=np.uint64)
    lib().or_lut_from_table(ctypes.c_uint32(N), ctypes.c_uint32(msg_modulus), _p(t), ctypes.c_uint64(delta_out), _p(out))
    return out


def nand(prm: Params, keys: Keys, c1: np.ndarray, c2: np.ndarray) -> np.ndarray:
    out = np.zeros(prm.n + 1, dtype=np.uint64)
    lib().or_nand(ctypes.byref(prm), _p(keys.bsk_ntt), _p(keys.ksk), _p(np.ascontiguousarray(c1, dtype=np.uint64)),
                  _p(np.ascontiguousarray(c2, dtype=np.uint64)), _p(out))
    return out


MU = 1 << 61  # gate encoding: true = +1/8, false = -1/8 (2^64 torus)


def encode_bit(b: int) -> int:
    return MU if b else (1 << 64) - MU


def decode_bit(phase: int) -> int:
    return 1 if phase < (1 << 63) else 0


# ---- packing keyswitch + compression (tfhe_oracle.h: or_pks_params) ----------------------------
class PksParams(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_uint32), ("out_k", ctypes.c_uint32), ("out_N", ctypes.c_uint32),
                ("base_log", ctypes.c_uint32), ("level", ctypes.c_uint32), ("lwe_per_glwe", ctypes.c_uint32),
                ("storage_log", ctypes.c_uint32), ("noise_log2", ctypes.c_int32)]


def pks_params(preset: int = 0) -> PksParams:
    p = PksParams()
    assert lib().or_pks_params_preset(preset, ctypes.byref(p)) == 0
    return p


class PksKeys:
    def __init__(self, pp: PksParams, seed: int, in_key: np.ndarray, with_pksk: bool = True):
        L = lib()
        L.or_pksk_len.restype = ctypes.c_size_t
        self.pp, self.seed = pp, seed
        self.in_key = np.ascontiguousarray(in_key, dtype=np.uint64)
        self.out_key = np.zeros(pp.out_k * pp.out_N, dtype=np.uint64)
        self.pksk = np.zeros(L.or_pksk_len(ctypes.byref(pp)), dtype=np.uint64) if with_pksk else None
        L.or_pks_keygen(ctypes.byref(pp), ctypes.c_uint64(seed), _p(self.in_key), _p(self.out_key),
                        _p(self.pksk) if with_pksk else None)


def pks_pack(pp: PksParams, keys: PksKeys, lwes: np.ndarray) -> np.ndarray:
    lwes = np.ascontiguousarray(lwes, dtype=np.uint64).reshape(-1, pp.in_dim + 1)
    out = np.zeros((pp.out_k + 1) * pp.out_N, dtype=np.uint64)
    lib().or_pks_pack(ctypes.byref(pp), _p(keys.pksk), _p(lwes), ctypes.c_uint32(lwes.shape[0]), _p(out))
    return out


def glwe_phase_native(k: int, N: int, key: np.ndarray, glwe: np.ndarray) -> np.ndarray:
    out = np.zeros(N, dtype=np.uint64)
    lib().or_glwe_phase_native(ctypes.c_uint32(k), ctypes.c_uint32(N), _p(np.ascontiguousarray(key, dtype=np.uint64)),
                               _p(np.ascontiguousarray(glwe, dtype=np.uint64)), _p(out))
    return out


def pks_compress(pp: PksParams, glwe: np.ndarray, bodies: int) -> np.ndarray:
    L = lib()
    L.or_pks_packed_words.restype = ctypes.c_size_t
    out = np.zeros(L.or_pks_packed_words(ctypes.byref(pp), ctypes.c_uint32(bodies)), dtype=np.uint64)
    L.or_pks_compress(ctypes.byref(pp), _p(np.ascontiguousarray(glwe, dtype=np.uint64)), ctypes.c_uint32(bodies), _p(out))
    return out


def pks_extract(pp: PksParams, packed: np.ndarray, bodies: int) -> np.ndarray:
    out = np.zeros((pp.out_k + 1) * pp.out_N, dtype=np.uint64)
    lib().or_pks_extract(ctypes.byref(pp), _p(np.ascontiguousarray(packed, dtype=np.uint64)), ctypes.c_uint32(bodies),
                         _p(out))
    return out


# ---- switch-and-squash / noise squashing (sns_oracle.c) ----------------------------------------
class SnsParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("k", ctypes.c_uint32), ("N", ctypes.c_uint32), ("base_log", ctypes.c_uint32),
                ("level", ctypes.c_uint32), ("noise_log2", ctypes.c_int32)]


def sns_params(preset: int = 0) -> SnsParams:
    p = SnsParams()
    assert lib().or_sns_params_preset(preset, ctypes.byref(p)) == 0
    return p


class SnsKeys:
    def __init__(self, sp: SnsParams, seed: int, lwe_key: np.ndarray, with_bsk: bool = True):
        L = lib()
        L.or_sns_bsk_len.restype = ctypes.c_size_t
        L.or_sns_limb_ntt_len.restype = ctypes.c_size_t
        self.sp, self.seed = sp, seed
        self.lwe_key = np.ascontiguousarray(lwe_key, dtype=np.uint64)
        self.glwe_key = np.zeros(sp.k * sp.N, dtype=np.uint64)
        self.bsk = np.zeros(L.or_sns_bsk_len(ctypes.byref(sp)), dtype=np.uint64) if with_bsk else None
        L.or_sns_keygen(ctypes.byref(sp), ctypes.c_uint64(seed), _p(self.lwe_key), _p(self.glwe_key),
                        _p(self.bsk) if with_bsk else None)
        self._bsk_limb = None

    @property
    def bsk_limb(self) -> np.ndarray:
        """The key as the blind rotation consumes it: rounded to multiples of 2^16 at load (or_sns_bsk_round,
        as the device does), then its five limb polynomials: the low 48-bit limb as the device's f64 spectrum
        (bits in the u64 words), the four 16-bit limbs as NTTs (2.0 GB at n = 918)."""
        if self._bsk_limb is None:
            rounded = np.zeros_like(self.bsk)
            lib().or_sns_bsk_round(ctypes.byref(self.sp), _p(self.bsk), _p(rounded))
            self._bsk_limb = np.zeros(lib().or_sns_limb_ntt_len(ctypes.byref(self.sp)), dtype=np.uint64)
            lib().or_sns_bsk_to_limb_ntt(ctypes.byref(self.sp), _p(rounded), _p(self._bsk_limb))
        return self._bsk_limb


def sns_squash(sp: SnsParams, keys: SnsKeys, small: np.ndarray, msg_modulus: int = 16, threads: int = 0) -> np.ndarray:
    small = np.ascontiguousarray(small, dtype=np.uint64).reshape(-1, sp.n + 1)
    out = np.zeros((small.shape[0], sp.k * sp.N + 1, 2), dtype=np.uint64)
    lib().or_sns_squash(ctypes.byref(sp), _p(keys.bsk_limb), _p(small), ctypes.c_size_t(small.shape[0]),
                        ctypes.c_uint32(msg_modulus), _p(out), ctypes.c_int(threads))
    return out


def sns_blind_rotate(sp: SnsParams, keys: SnsKeys, small: np.ndarray, lut: np.ndarray) -> np.ndarray:
    acc = np.zeros((sp.k + 1, 2, sp.N), dtype=np.uint64)
    lib().or_sns_blind_rotate(ctypes.byref(sp), _p(keys.bsk_limb), _p(np.ascontiguousarray(small, dtype=np.uint64)),
                              _p(np.ascontiguousarray(lut, dtype=np.uint64)), _p(acc))
    return acc


def sns_lut_identity(sp: SnsParams, msg_modulus: int = 16) -> np.ndarray:
    lut = np.zeros((2, sp.N), dtype=np.uint64)
    lib().or_sns_lut_identity(ctypes.byref(sp), ctypes.c_uint32(msg_modulus), _p(lut))
    return lut


def sns_sample_extract(sp: SnsParams, acc: np.ndarray) -> np.ndarray:
    out = np.zeros((sp.k * sp.N + 1, 2), dtype=np.uint64)
    lib().or_sns_sample_extract(ctypes.byref(sp), _p(np.ascontiguousarray(acc, dtype=np.uint64)), _p(out))
    return out


def sns_phase(sp: SnsParams, glwe_key: np.ndarray, cts: np.ndarray) -> list:
    cts = np.ascontiguousarray(cts, dtype=np.uint64).reshape(-1, sp.k * sp.N + 1, 2)
    out = np.zeros((cts.shape[0], 2), dtype=np.uint64)
    lib().or_sns_phase(ctypes.byref(sp), _p(np.ascontiguousarray(glwe_key, dtype=np.uint64)), _p(cts),
                       ctypes.c_size_t(cts.shape[0]), _p(out))
    return [int(o[0]) | (int(o[1]) << 64) for o in out]


def sns_ntt(which: int, a: np.ndarray, inverse: bool = False) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64).copy()
    f = lib().or_sns_ntt_inv if inverse else lib().or_sns_ntt_fwd
    f(ctypes.c_int(which), _p(a), ctypes.c_uint32(a.size))
    return a


# ---- exact integer arithmetic over Z_2^64 (exact_oracle.c): the arbiter of the FFT64 path --------------------
def poly_mul_torus_exact(a_small, b) -> np.ndarray:
    """The limb / Goldilocks-NTT exact wrapping product (or_poly_mul_torus_exact)."""
    a = np.ascontiguousarray(a_small, dtype=np.int64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    out = np.zeros(b.shape[0], dtype=np.uint64)
    lib().or_poly_mul_torus_exact(_p(out), _p(a, I64P), _p(b), ctypes.c_uint32(b.shape[0]))
    return out


class ExactKey:
    """or_exact_key: the standard-domain torus BSK as NTT-domain limb polynomials (3 x the BSK's size)."""

    def __init__(self, prm: Params, bsk: np.ndarray):
        L = lib()
        L.or_exact_key_new.restype = ctypes.c_void_p
        L.or_exact_key_free.argtypes = [ctypes.c_void_p]
        self.prm = prm
        self._bsk = np.ascontiguousarray(bsk, dtype=np.uint64)
        self.h = L.or_exact_key_new(ctypes.byref(prm), _p(self._bsk))
        assert self.h, "or_exact_key_new refused the parameters"

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_exact_key_free(ctypes.c_void_p(self.h))
            self.h = None

    def cmux(self, key_index, a_tilde, acc_in, threads: int = 0):
        """-> (acc_out, s1, s2): acc_out[q] = acc_in[q] + ExtProd(BSK_i, X^a acc - acc) exactly, with the norm sums of
        the FFT error bound (s1 = sum_r ||d_r|| ||w_r||, s2 = sum_r ||d_r||^2 ||w_r||^2, per output column)."""
        prm = self.prm
        row = (prm.k + 1) * prm.N
        acc_in = np.ascontiguousarray(acc_in, dtype=np.uint64).reshape(-1, row)
        cnt = acc_in.shape[0]
        ki = np.ascontiguousarray(np.broadcast_to(np.asarray(key_index, dtype=np.uint32), (cnt,)))
        at = np.ascontiguousarray(np.broadcast_to(np.asarray(a_tilde, dtype=np.uint32), (cnt,)))
        assert int(ki.max(initial=0)) < prm.n and int(at.max(initial=0)) < 2 * prm.N
        out = np.zeros_like(acc_in)
        s1 = np.zeros((cnt, prm.k + 1), dtype=np.float64)
        s2 = np.zeros((cnt, prm.k + 1), dtype=np.float64)
        lib().or_cmux_exact_batch(ctypes.c_void_p(self.h), ctypes.c_size_t(cnt), _p(ki, U32P), _p(at, U32P),
                                  _p(acc_in), _p(out), _p(s1, ctypes.c_void_p), _p(s2, ctypes.c_void_p),
                                  ctypes.c_int(threads))
        return out, s1, s2

    def blind_rotate(self, lwe_in: np.ndarray, lut: np.ndarray) -> np.ndarray:
        acc = np.zeros((self.prm.k + 1) * self.prm.N, dtype=np.uint64)
        lib().or_blind_rotate_exact(ctypes.c_void_p(self.h), _p(np.ascontiguousarray(lwe_in, dtype=np.uint64)),
                                    _p(np.ascontiguousarray(lut, dtype=np.uint64)), _p(acc))
        return acc


def blind_rotate_fft_trace(prm: Params, keys: Keys, lwe_in: np.ndarray, lut: np.ndarray) -> np.ndarray:
    """(n + 1) x (k+1)N: the FFT64 oracle's accumulator before CMUX 0 and after each CMUX."""
    tr = np.zeros((prm.n + 1, (prm.k + 1) * prm.N), dtype=np.uint64)
    lib().or_blind_rotate_fft_trace(ctypes.byref(prm), _p(keys.bsk_fourier, ctypes.c_void_p),
                                    _p(np.ascontiguousarray(lwe_in, dtype=np.uint64)),
                                    _p(np.ascontiguousarray(lut, dtype=np.uint64)), _p(tr))
    return tr


def mod_switch(x, two_n: int) -> np.ndarray:
    """round(x 2N / 2^64) mod 2N (or_mod_switch), vectorised."""
    x = np.asarray(x, dtype=np.uint64)
    lg = int(two_n).bit_length() - 1
    return ((((x >> np.uint64(64 - lg - 1)) + np.uint64(1)) >> np.uint64(1)) & np.uint64(two_n - 1)).astype(np.uint32)
