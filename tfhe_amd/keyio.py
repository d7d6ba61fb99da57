"""tfhe-rs key ingest (the packages/kms key-loader role).

Reads the `safe_serialize` files the reference's relayer SDK ships and generates
(sdk/relayer/generateKeys.js:20-31; fixtures sdk/relayer/src/test/keys/{privateKey,publicKey}.bin):

    u64 len | "0.5"   (safe-serialization header version)
    u32               (versioning mode tag)
    u64 len | "0.1"   (versioning scheme)
    u64 len | type name ("high_level_api::ClientKey" / "high_level_api::CompactPublicKey")
    versioned bincode payload (little endian; enum/version tags are u32)

ClientKey payload (tfhe-rs 1.x, PARAM_MESSAGE_2_CARRY_2_KS_PBS_TUNIFORM_2M128):
    GLWE secret key  Vec<u64> (k*N binary words)
    LWE secret key   Vec<u64> (n binary words)
    shortint parameters: version-tagged fields at fixed offsets from the end of the LWE key
      (+0x1c lwe_dimension, +0x28 glwe_dimension, +0x34 polynomial_size, +0x48 lwe TUniform bound,
       +0x58 glwe TUniform bound, +0x60 pbs_base_log, +0x6c pbs_level, +0x78 ks_base_log,
       +0x84 ks_level, +0x90 message_modulus, +0x9c carry_modulus, +0xa8 max_noise_level,
       +0xb0 log2_p_fail (f64), +0xe5 modulus-switch zeros count, +0xf1 ms bound (f64),
       +0xfd ms r_sigma (f64), +0x109 ms input variance (f64))
    compact public-key encryption secret key Vec<u64> (binary) + its parameters
CompactPublicKey payload: Vec<u64> of 2N words = (mask polynomial | body polynomial) with
    body = mask (*) reverse(s_pke) + e    (negacyclic; tfhe-rs' semi-reverse convolution)
which `compact_public_key_noise` checks against the ingested PKE secret key: on the reference's own
fixtures the residual is bounded by 2^17, the TUniform(17) bound of the PKE parameters — a direct
pin of this parser and of the negacyclic conventions against real tfhe-rs output.

Only raw bytes are read (no deserializer that executes anything).  `to_engine_keys` maps the
ingested secret keys onto this engine's P-FHEVM parameter set and generates the server keys for
them (tfhe_hip_server_keygen), so fhEVM client keys flow through the GPU path.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, Tuple, Union

import numpy as np

SAFE_SERIALIZATION_VERSION = "0.5"
VERSIONING_VERSION = "0.1"


class KeyFormatError(ValueError):
    pass


class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.o = 0

    def u64(self, at: int = None) -> int:
        o = self.o if at is None else at
        if o + 8 > len(self.d):
            raise KeyFormatError(f"truncated at {o:#x}")
        v = struct.unpack_from("<Q", self.d, o)[0]
        if at is None:
            self.o += 8
        return v

    def u32_at(self, o: int) -> int:
        return struct.unpack_from("<I", self.d, o)[0]

    def f64_at(self, o: int) -> float:
        return struct.unpack_from("<d", self.d, o)[0]

    def string(self) -> str:
        n = self.u64()
        if n > 256:
            raise KeyFormatError(f"implausible string length {n} at {self.o - 8:#x}")
        s = self.d[self.o:self.o + n]
        self.o += n
        return s.decode("ascii", errors="replace")

    def vec_u64_at(self, o: int) -> Tuple[np.ndarray, int]:
        n = self.u64(o)
        end = o + 8 + 8 * n
        if n > (1 << 24) or end > len(self.d):
            raise KeyFormatError(f"bad Vec<u64> length {n} at {o:#x}")
        return np.frombuffer(self.d, dtype="<u8", count=n, offset=o + 8).astype(np.uint64), end


def _read_header(r: _Reader, type_name: str) -> None:
    ser = r.string()
    mode = r.u32_at(r.o)
    r.o += 4
    ver, ty = r.string(), r.string()
    if mode > 4:
        raise KeyFormatError(f"unknown versioning mode tag {mode}")
    if ser != SAFE_SERIALIZATION_VERSION or ver != VERSIONING_VERSION:
        raise KeyFormatError(f"unsupported safe_serialize versions {ser!r}/{ver!r}")
    if ty != type_name:
        raise KeyFormatError(f"expected {type_name!r}, file holds {ty!r}")


def _find_binary_vec(r: _Reader, start: int, length: int, window: int = 64) -> Tuple[np.ndarray, int]:
    """The Vec<u64> of `length` binary words whose length prefix lies in [start, start + window)."""
    for o in range(start, min(start + window, len(r.d) - 8)):
        if r.u64(o) == length:
            v, end = r.vec_u64_at(o)
            if np.all(v <= 1):
                return v, end
    raise KeyFormatError(f"no binary Vec<u64> of length {length} near {start:#x}")


@dataclass
class TfhersClientKey:
    params: Dict[str, Union[int, float, str]]
    glwe_key: np.ndarray            # k*N binary words (the big LWE key of KS->PBS ciphertexts)
    lwe_key: np.ndarray             # n binary words
    pke_key: np.ndarray             # compact public-key encryption secret key
    pke_params: Dict[str, int] = field(default_factory=dict)


def load_client_key(src: Union[str, bytes], N: int = 2048, n: int = 918) -> TfhersClientKey:
    """Parse a tfhe-rs `high_level_api::ClientKey` (safe_serialize 0.5 / versioning 0.1)."""
    data = open(src, "rb").read() if isinstance(src, str) else bytes(src)
    r = _Reader(data)
    _read_header(r, "high_level_api::ClientKey")
    glwe, end_g = _find_binary_vec(r, r.o, N)
    lwe, E = _find_binary_vec(r, end_g, n)
    P = {
        "lwe_dimension": r.u64(E + 0x1c), "glwe_dimension": r.u64(E + 0x28), "polynomial_size": r.u64(E + 0x34),
        "lwe_noise": f"TUniform({r.u32_at(E + 0x48)})" if r.u32_at(E + 0x40) == 1 else "Gaussian",
        "glwe_noise": f"TUniform({r.u32_at(E + 0x58)})" if r.u32_at(E + 0x50) == 1 else "Gaussian",
        "lwe_noise_bound_log2": r.u32_at(E + 0x48), "glwe_noise_bound_log2": r.u32_at(E + 0x58),
        "pbs_base_log": r.u64(E + 0x60), "pbs_level": r.u64(E + 0x6c),
        "ks_base_log": r.u64(E + 0x78), "ks_level": r.u64(E + 0x84),
        "message_modulus": r.u64(E + 0x90), "carry_modulus": r.u64(E + 0x9c),
        "max_noise_level": r.u64(E + 0xa8), "log2_p_fail": r.f64_at(E + 0xb0),
        "ms_noise_reduction_zeros": r.u64(E + 0xe5), "ms_bound": r.f64_at(E + 0xf1),
        "ms_r_sigma": r.f64_at(E + 0xfd), "ms_input_variance": r.f64_at(E + 0x109),
    }
    if P["lwe_dimension"] != n or P["glwe_dimension"] * P["polynomial_size"] != N:
        raise KeyFormatError(f"parameter block does not match the key sizes: {P}")
    pke, end_p = _find_binary_vec(r, E + 0x110, N, window=128)
    pke_params = {"lwe_dimension": r.u64(end_p + 8), "noise_bound_log2": r.u32_at(end_p + 0x1c)}
    return TfhersClientKey(P, glwe, lwe, pke, pke_params)


def load_compact_public_key(src: Union[str, bytes], N: int = 2048) -> Tuple[np.ndarray, np.ndarray]:
    """Parse a tfhe-rs `high_level_api::CompactPublicKey`: returns (mask, body) polynomials."""
    data = open(src, "rb").read() if isinstance(src, str) else bytes(src)
    r = _Reader(data)
    _read_header(r, "high_level_api::CompactPublicKey")
    for o in range(r.o, r.o + 64):
        if r.u64(o) == 2 * N:
            v, _ = r.vec_u64_at(o)
            return v[:N].copy(), v[N:].copy()
    raise KeyFormatError("no 2N-word key vector found")


def negacyclic_mul_binary(a: np.ndarray, s: np.ndarray) -> np.ndarray:
    """a (*) s mod (X^N + 1, 2^64) for a binary polynomial s."""
    N = a.shape[0]
    acc = np.zeros(N, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for j in np.nonzero(s)[0]:
            r = np.roll(a, int(j))
            r[:j] = np.uint64(0) - r[:j]
            acc += r
    return acc


def compact_public_key_noise(mask: np.ndarray, body: np.ndarray, pke_key: np.ndarray) -> int:
    """max |body - mask (*) reverse(s)| over the torus (signed); small iff the key pair matches."""
    with np.errstate(over="ignore"):
        e = (body - negacyclic_mul_binary(mask, pke_key[::-1].copy())).view(np.int64)
    return int(np.abs(e.astype(object)).max())


def to_engine_keys(tk: TfhersClientKey, seed=None, with_server_key: bool = True):
    """(ClientKey, ServerKey) of this engine over the ingested secret keys (P-FHEVM preset, checked).

    The server-key randomness (BSK / KSK masks and noise, the modulus-switch zeros) comes from 192 bits of
    OS entropy unless a test seed is given: with a public seed anyone holding the published evaluation
    keys could regenerate every mask and noise term and solve the KSK rows for the secret key."""
    import tfhe_amd
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM)
    P = tk.params
    want = {"lwe_dimension": p.n, "glwe_dimension": p.k, "polynomial_size": p.N, "pbs_base_log": p.pbs_base_log,
            "pbs_level": p.pbs_level, "ks_base_log": p.ks_base_log, "ks_level": p.ks_level}
    bad = {k: (P[k], v) for k, v in want.items() if P[k] != v}
    if bad:
        raise KeyFormatError(f"ingested parameters differ from the engine's P-FHEVM preset: {bad}")
    ck = tfhe_amd.ClientKey(p, seed, tk.lwe_key.copy(), tk.glwe_key.copy())
    return ck, (tfhe_amd.server_keygen(ck, seed) if with_server_key else None)
