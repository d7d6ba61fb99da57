"""tfhe-rs compact ciphertext lists -> the GPU engine (ciphertext ingest).

The reference's SDK encrypts every user input as ONE compact list under the network's CompactPublicKey
and ships it with a ZK proof: sdk/relayer/src/sdk/encrypt.ts:97-148,185 (`build_with_proof_packed`),
fixtures sdk/relayer/src/test/v1/ciphertext.ts:1 and src/test/assets/input-proof-payload-{1,2,3}.json
(`ciphertextWithInputVerification`, with the declared fheTypeEncryptionBitwidths and, for payload 2,
the clear values).  This module reads that format, expands it to LWE ciphertexts and casts them into
the engine's key set:

    safe_serialize header "0.5" / "0.1" / "high_level_api::ProvenCompactCiphertextList"
    Vec<(list, proof)> (one entry)
      LWE compact list: data Vec<u64> = bins x lwe_dim mask words, then count body words
                        (each bin of <= lwe_dim ciphertexts shares one mask polynomial), lwe_size, count
      degree, message_modulus 4, carry_modulus 4, packing -- then the CompactPkeProof (not verified here:
      there is no ZK proof system on this path; the relayer / KMS verifies proofs)
    info: Vec<DataKind> = Unsigned(num_blocks) | Signed(num_blocks) | Boolean, one per encrypted value

Packed lists ("build_with_proof_packed") hold two 2-bit radix blocks per LWE: v = lo + 4 hi, encoded
as v * 2^63 / 16 (message x carry space with one padding bit).

Encryption convention (tfhe-rs core_crypto, semi-reverse negacyclic convolution conv(a, rev(b))):
    CPK:   body = mask (*) rev(s) + e                       (verified on the reference's key pair,
                                                             tfhe_amd/keyio.compact_public_key_noise)
    list:  M = pk_mask (*) rev(r) + e1,   b_i = (pk_body (*) rev(r))[i] + e2_i + Delta v_i
so b_i - (M (*) rev(s))[i] = Delta v_i + small, i.e. expanded ciphertext i has the LWE mask
    a_i[k] = M[k - (N-1-i)]     for k >= N-1-i,      a_i[k] = -M[k + i + 1]   for k < N-1-i.
tests/test_ctlist.py pins this against the reference's own CompactPublicKey / ClientKey pair.

Casting: expanded ciphertexts live under the compact-PKE secret key (dimension 2048).  A P-FHEVM engine
whose keyswitch key is the CASTING key pke -> small LWE key (same 2^4 x 4 decomposition) and whose
bootstrapping key is the normal one turns them, with the "low block" / "high block" LUTs, into radix
blocks under the computation key -- unpacking and refreshing in one PBS each (tfhe-rs does KS with its
KeySwitchingKey then a PBS per block).  No other engine change is needed: KS -> PBS is that engine's order.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .keyio import KeyFormatError, _read_header, _Reader, negacyclic_mul_binary

TYPE_NAME = "high_level_api::ProvenCompactCiphertextList"
KIND_UNSIGNED, KIND_SIGNED, KIND_BOOLEAN = 0, 1, 2
PACKED_MM = 16                         # message_modulus x carry_modulus of a packed LWE
DELTA_PACKED = (1 << 63) // PACKED_MM  # 2^59


@dataclass
class CompactList:
    lwe_dim: int
    count: int
    masks: np.ndarray                  # (bins, lwe_dim) u64
    bodies: np.ndarray                 # (count,) u64
    message_modulus: int = 4
    carry_modulus: int = 4
    kinds: List[Tuple[int, int]] = field(default_factory=list)   # (kind, num_blocks)

    @property
    def blocks(self) -> int:
        return sum(1 if k == KIND_BOOLEAN else n for k, n in self.kinds)


def _parse_kinds(d: bytes) -> List[Tuple[int, int]]:
    """The trailing Vec<DataKind>: u32 2 | u64 L | L x (u32 1, u32 tag[, u64 blocks]) | 12 zero bytes."""
    if d[-12:] != bytes(12):
        raise KeyFormatError("unexpected compact-list trailer")
    end = len(d) - 12
    for start in range(end - 16, max(0, end - 8192), -4):
        if struct.unpack_from("<I", d, start)[0] != 2:
            continue
        L = struct.unpack_from("<Q", d, start + 4)[0]
        if not 1 <= L <= 4096:
            continue
        o, out, ok = start + 12, [], True
        for _ in range(L):
            if o + 8 > end or struct.unpack_from("<I", d, o)[0] != 1:
                ok = False
                break
            tag = struct.unpack_from("<I", d, o + 4)[0]
            o += 8
            if tag in (KIND_UNSIGNED, KIND_SIGNED):
                if o + 8 > end:
                    ok = False
                    break
                out.append((tag, struct.unpack_from("<Q", d, o)[0]))
                o += 8
            elif tag == KIND_BOOLEAN:
                out.append((tag, 1))
            else:
                ok = False
                break
        if ok and o == end:
            return out
    raise KeyFormatError("no DataKind list found at the end of the compact list")


def load_compact_list(src) -> CompactList:
    """Parse a tfhe-rs `high_level_api::ProvenCompactCiphertextList` (safe_serialize 0.5 / 0.1): the LWE
    compact list, its message / carry moduli and the data kinds.  The proof is skipped, not verified."""
    data = open(src, "rb").read() if isinstance(src, str) else bytes(src)
    r = _Reader(data)
    _read_header(r, TYPE_NAME)
    for o in range(r.o, min(r.o + 128, len(data) - 8)):
        L = r.u64(o)
        if not 0 < L < (1 << 26) or o + 8 + 8 * L + 28 > len(data):
            continue
        e = o + 8 + 8 * L
        lwe_size = r.u64(e + 4)
        count = r.u64(e + 16)
        dim = lwe_size - 1
        if dim < 1 or count < 1 or r.u32_at(e) != 0 or r.u32_at(e + 12) != 0:
            continue
        bins = -(-count // dim)
        if L != bins * dim + count:
            continue
        words = np.frombuffer(data, dtype="<u8", count=L, offset=o + 8).astype(np.uint64)
        masks = words[:bins * dim].reshape(bins, dim).copy()
        bodies = words[bins * dim:].copy()
        tail = data[e + 28:e + 160]
        pat = struct.pack("<QIQ", 4, 0, 4)
        at = tail.find(pat)
        mm = cm = 4
        if at >= 0:
            mm = struct.unpack_from("<Q", tail, at)[0]
            cm = struct.unpack_from("<Q", tail, at + 12)[0]
        return CompactList(int(dim), int(count), masks, bodies, int(mm), int(cm), _parse_kinds(data))
    raise KeyFormatError("no LWE compact list found after the header")


def expand(cl: CompactList) -> np.ndarray:
    """(count, lwe_dim + 1) LWE ciphertexts under the compact-PKE secret key (tfhe-rs expansion)."""
    N = cl.lwe_dim
    out = np.zeros((cl.count, N + 1), dtype=np.uint64)
    with np.errstate(over="ignore"):
        for q in range(cl.count):
            M = cl.masks[q // N]
            i = q % N
            k0 = N - 1 - i
            out[q, k0:N] = M[:i + 1]
            out[q, :k0] = np.uint64(0) - M[i + 1:]
            out[q, N] = cl.bodies[q]
    return out


def unpack_values(blocks: Sequence[int], kinds: Sequence[Tuple[int, int]]) -> List[int]:
    """Radix blocks (2 bits each, least significant first) -> one integer per DataKind."""
    vals, o = [], 0
    for kind, n in kinds:
        v = sum(int(blocks[o + j]) << (2 * j) for j in range(n))
        vals.append(v)
        o += n
    return vals


# ---- client side: compact public key and compact encryption (tfhe-rs conventions above) -------------
def _tuniform(rng: np.random.Generator, bound_log2: int, size) -> np.ndarray:
    b = 1 << bound_log2
    return (rng.integers(-b, b + 1, size=size, dtype=np.int64)).astype(np.uint64)


def gen_compact_public_key(pke_key: np.ndarray, rng: Optional[np.random.Generator] = None,
                           noise_bound_log2: int = 17) -> Tuple[np.ndarray, np.ndarray]:
    """(mask, body) with body = mask (*) rev(s) + e, TUniform noise (the reference's PKE parameters)."""
    rng = rng or np.random.default_rng(np.random.SeedSequence())
    N = pke_key.shape[0]
    mask = rng.integers(0, 1 << 64, N, dtype=np.uint64)
    with np.errstate(over="ignore"):
        body = negacyclic_mul_binary(mask, pke_key[::-1].copy()) + _tuniform(rng, noise_bound_log2, N)
    return mask, body


def encrypt_compact(cpk: Tuple[np.ndarray, np.ndarray], packed_values: Sequence[int],
                    kinds: Sequence[Tuple[int, int]], rng: Optional[np.random.Generator] = None,
                    noise_bound_log2: int = 17) -> CompactList:
    """A compact list of 4-bit packed values (lo + 4 hi) under the compact public key, in the layout
    load_compact_list returns (the client half of build_with_proof_packed, without the proof)."""
    rng = rng or np.random.default_rng(np.random.SeedSequence())
    pk_mask, pk_body = cpk
    N = pk_mask.shape[0]
    v = np.asarray([int(x) % PACKED_MM for x in packed_values], dtype=np.uint64)
    count = v.shape[0]
    bins = -(-count // N)
    masks = np.zeros((bins, N), dtype=np.uint64)
    bodies = np.zeros(count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for g in range(bins):
            r = rng.integers(0, 2, N).astype(np.uint64)
            rr = r[::-1].copy()
            masks[g] = negacyclic_mul_binary(pk_mask, rr) + _tuniform(rng, noise_bound_log2, N)
            cb = negacyclic_mul_binary(pk_body, rr)
            sl = slice(g * N, min(count, (g + 1) * N))
            n = sl.stop - sl.start
            bodies[sl] = cb[:n] + _tuniform(rng, noise_bound_log2, n) + v[sl] * np.uint64(DELTA_PACKED)
    return CompactList(N, count, masks, bodies, 4, 4, list(kinds))


def pack_blocks(blocks: Sequence[int]) -> List[int]:
    """Pairs of 2-bit blocks -> packed 4-bit values lo + 4 hi (an odd count leaves hi = 0)."""
    b = list(blocks) + ([0] if len(blocks) % 2 else [])
    return [int(b[2 * j]) + 4 * int(b[2 * j + 1]) for j in range(len(b) // 2)]


def value_blocks(values: Sequence[int], kinds: Sequence[Tuple[int, int]]) -> List[int]:
    out = []
    for v, (kind, n) in zip(values, kinds):
        out += [(int(v) >> (2 * j)) & 3 for j in range(n)]
    return out


# ---- casting into the engine ---------------------------------------------------------------------------
def casting_keys(ck, pke_key: np.ndarray, seed: Optional[int] = None):
    """(BSK small -> computation key, casting KSK pke key -> small key, MS zeros) for a P-FHEVM engine that
    bootstraps expanded compact ciphertexts into radix blocks under ck's computation (GLWE) key."""
    import tfhe_amd
    p = ck.params
    if pke_key.shape[0] != p.k * p.N:
        raise ValueError(f"compact-PKE key dimension {pke_key.shape[0]} != k*N = {p.k * p.N}")
    sk = tfhe_amd.server_keygen(ck, seed)
    return tfhe_amd.ServerKey(p, sk.bsk, casting_ksk(ck, pke_key, seed), sk.ms_zeros)


# seeded test streams of the casting KSK are offset from the server key's seed, so the two KSKs never share
# a mask or noise term (their row difference would otherwise expose glwe_key XOR pke_key)
CAST_SEED_TAG = 0xCA57_1E5D_0000_0000


def casting_ksk(ck, pke_key: np.ndarray, seed: Optional[int] = None) -> np.ndarray:
    """The casting KSK alone (compact-PKE key -> small LWE key, P-FHEVM KS 2^4 x 4): no BSK is generated.
    seed None: its own 192 bits of OS entropy; an int: a test stream independent of ``server_keygen(ck,
    seed)``'s."""
    import ctypes
    import tfhe_amd
    p = ck.params
    L = tfhe_amd.lib()
    ksk = np.zeros(L.tfhe_hip_ksk_len(ctypes.byref(p)), dtype=np.uint64)
    rk = tfhe_amd.rng_key(None if seed is None else (int(seed) ^ CAST_SEED_TAG) & (2**64 - 1))
    lwe, pke = tfhe_amd._c_u64(ck.lwe_key), tfhe_amd._c_u64(np.asarray(pke_key, dtype=np.uint64))
    tfhe_amd._check(L.tfhe_hip_server_keygen_k(ctypes.byref(p), ctypes.byref(rk), tfhe_amd._u64(lwe),
                                               tfhe_amd._u64(pke), None, tfhe_amd._u64(ksk)))
    return ksk


T_LO = tuple(v % 4 for v in range(PACKED_MM))
T_HI = tuple(v // 4 for v in range(PACKED_MM))


def cast_to_blocks(cast_engine, expanded: np.ndarray, n_blocks: int) -> np.ndarray:
    """Expanded packed LWEs (count, 2049) -> (n_blocks, 2049) radix blocks under the computation key:
    one PBS per block with the low / high LUT (unpack + refresh), through the casting engine."""
    from . import lut_from_table
    N = cast_engine.params.N
    luts = np.stack([lut_from_table(N, PACKED_MM, list(T_LO), DELTA_PACKED),
                     lut_from_table(N, PACKED_MM, list(T_HI), DELTA_PACKED)])
    src = np.repeat(np.arange(expanded.shape[0]), 2)[:n_blocks]
    idx = (np.arange(n_blocks) % 2).astype(np.uint32)
    return cast_engine.pbs(expanded[src], luts, idx)
