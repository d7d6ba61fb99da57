"""Compressed (seeded) server keys on CPU (tfhe_amd/csrc/seeded.cpp, tfhe_amd/keyio.py).

Pins: AES-128 against the FIPS-197 known answers; the mask stream against its definition (AES blocks of a
little-endian counter, from byte 1 of block 0); every checked row of a decompressed key decrypts under the secret
key to the plaintext tfhe-rs puts there; the container round-trips; the decompressed keys bootstrap correctly on the
CPU oracle, also for the reference's own tfhe-rs client key (read in place when /root/reference is present).  The
byte layout of a real tfhe-rs CompressedServerKey is PARITY UNPINNED: the reference holds no such file."""
import ctypes
import os

import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import keyio
from oracle import oracle as O

KEYS = "/root/reference/sdk/relayer/src/test/keys"


def _aes(key_hex: str, pt_hex: str) -> str:
    out = ctypes.create_string_buffer(16)
    tfhe_amd._check(tfhe_amd.lib().tfhe_hip_aes128_block(bytes.fromhex(key_hex), bytes.fromhex(pt_hex), out))
    return out.raw.hex()


def test_aes128_fips197_known_answers():
    assert _aes("000102030405060708090a0b0c0d0e0f", "00112233445566778899aabbccddeeff") == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"  # FIPS-197 Appendix C.1
    assert _aes("2b7e151628aed2a6abf7158809cf4f3c", "3243f6a8885a308d313198a2e0370734") == \
        "3925841d02dc09fbdc118597196a0b32"  # FIPS-197 Appendix B


def _words(seed: int, first: int, count: int) -> np.ndarray:
    out = np.zeros(count, dtype=np.uint64)
    tfhe_amd._check(tfhe_amd.lib().tfhe_hip_csprng_words(tfhe_amd._u64(keyio._seed2(seed)), first, count,
                                                          tfhe_amd._u64(out)))
    return out


def test_mask_stream_definition():
    seed = 0x0123456789ABCDEF_FEDCBA9876543210
    key = seed.to_bytes(16, "little").hex()
    blocks = b"".join(bytes.fromhex(_aes(key, b.to_bytes(16, "little").hex())) for b in range(40))
    want = np.frombuffer(blocks[1:1 + 8 * 70], dtype="<u8")
    assert np.array_equal(_words(seed, 0, 70), want)
    assert np.array_equal(_words(seed, 13, 40), want[13:53])           # any window of the same stream
    assert not np.array_equal(_words(seed + 1, 0, 70), want)


def _rows_decrypt(p, ck, sk, csk, rows=((0, 0), (1, 0), (5, 1), (629, 1)), tol_log2=45):
    """(GGSW i, row c) at level 0 of the decompressed BSK and a few KSK rows decrypt to tfhe-rs's plaintexts."""
    N, k, L = p.N, p.k, p.pbs_level
    row_len = (k + 1) * N
    bsk = sk.bsk.reshape(p.n, k + 1, L, row_len)   # this engine's [i][c * L + l][j]
    S = ck.glwe_key.reshape(k, N)
    for i, c in rows:
        i = min(i, p.n - 1)
        for l in range(L):
            r = bsk[i, c, l]
            assert np.array_equal(r[k * N:], csk.bsk_bodies[i, l, c])   # the stored body, untouched
            phase = r[k * N:].copy()
            with np.errstate(over="ignore"):
                for cc in range(k):
                    phase -= keyio.negacyclic_mul_binary(r[cc * N:(cc + 1) * N], S[cc])
                g = np.uint64(1 << (64 - p.pbs_base_log * (l + 1)))
                want = np.zeros(N, dtype=np.uint64)
                if ck.lwe_key[i]:
                    if c < k:
                        want -= g * S[c]
                    else:
                        want[0] = g
                e = (phase - want).view(np.int64)
            assert int(np.abs(e).max()) < 2 ** tol_log2, (i, c, l)
    ksk = sk.ksk.reshape(k * N, p.ks_level, p.n + 1)
    for j in (0, 7, k * N - 1):
        for l in range(p.ks_level):
            a, b = ksk[j, l, :p.n], ksk[j, l, p.n]
            with np.errstate(over="ignore"):
                ph = b - np.sum(a * ck.lwe_key, dtype=np.uint64) - (ck.glwe_key[j] << np.uint64(64 - p.ks_base_log * (l + 1)))
            assert abs(int(np.int64(ph.view(np.int64)))) < 2 ** (tol_log2 + 8)
            # tfhe-rs stores a keyswitch block least significant level first: storage row s = engine row L - 1 - s
            assert int(b) == int(csk.ksk_bodies[j, p.ks_level - 1 - l]), (j, l)


@pytest.fixture(scope="module")
def gate():
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT)
    ck, _ = tfhe_amd.gen_keys(p, 0x5EED0001, with_server_key=False)
    csk = keyio.compress_server_key(ck, seed=0x5EED0002)
    p2, sk = keyio.decompress_server_key(csk)
    return p, ck, csk, sk


def test_decompressed_rows_decrypt(gate):
    p, ck, csk, sk = gate
    assert csk.bsk_bodies.shape == (630, 3, 2, 1024) and csk.ksk_bodies.shape == (1024, 8)
    _rows_decrypt(p, ck, sk, csk)


def test_container_roundtrip(gate):
    p, ck, csk, sk = gate
    blob = keyio.dumps_compressed_server_key(csk)
    # 8 bytes a body word: the compressed key is 1/(k+1) of the BSK and 1/(n+1) of the KSK
    assert len(blob) < 8 * (csk.bsk_bodies.size + csk.ksk_bodies.size) + 1024
    back = keyio.loads_compressed_server_key(blob)
    assert back.params == csk.params and (back.bsk_seed, back.ksk_seed) == (csk.bsk_seed, csk.ksk_seed)
    assert np.array_equal(back.bsk_bodies, csk.bsk_bodies) and np.array_equal(back.ksk_bodies, csk.ksk_bodies)
    with pytest.raises(keyio.KeyFormatError):
        keyio.loads_compressed_server_key(blob[:len(blob) // 2])
    with pytest.raises(keyio.KeyFormatError):
        keyio.loads_compressed_server_key(blob.replace(b"CompressedServerKey", b"CompressedServerKez"))


def test_decompressed_keys_bootstrap_on_oracle(gate):
    p, ck, csk, sk = gate
    prm = O.params(tfhe_amd.PRESET_GATE_FFT)
    keys = O.Keys.__new__(O.Keys)
    keys.prm, keys.seed, keys.lwe_key, keys.glwe_key = prm, 0, ck.lwe_key, ck.glwe_key
    keys.bsk, keys.ksk, keys._bsk_ntt, keys.ms_zeros = sk.bsk, sk.ksk, None, None
    bits = np.array([1, 0, 0, 1], dtype=bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE)
    out = O.pbs_batch_fft(prm, keys, cts, O.lut_constant(1024, O.MU)[None])
    assert np.array_equal(ck.decrypt_bool(out), bits)   # the gate LUT (+-1/8 by the sign of the phase)


@pytest.mark.skipif(not os.path.exists(os.path.join(KEYS, "privateKey.bin")),
                    reason="reference key fixtures not present (read in place, never copied)")
def test_reference_client_key_seeded_server_key():
    """Seeded server keys for the reference's own tfhe-rs ClientKey (P-FHEVM): rows decrypt under the real
    secret keys, the modulus-switch zeros decompress to encryptions of zero, and a KS -> MS -> PBS on the oracle
    with the decompressed keys decrypts."""
    tk = keyio.load_client_key(os.path.join(KEYS, "privateKey.bin"))
    ck, _ = keyio.to_engine_keys(tk, with_server_key=False)
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT)
    ck.params = p
    csk = keyio.compress_server_key(ck, seed=0xF1E5, ms_count=32)
    back = keyio.loads_compressed_server_key(keyio.dumps_compressed_server_key(csk))
    p2, sk = keyio.decompress_server_key(back)
    assert (p2.N, p2.n, p2.transform) == (2048, 918, tfhe_amd.TRANSFORM_FFT64)
    _rows_decrypt(p, ck, sk, csk, rows=((0, 0), (1, 1), (917, 0)), tol_log2=50)
    with np.errstate(over="ignore"):
        ph = sk.ms_zeros[:, -1] - (sk.ms_zeros[:, :-1] * tk.lwe_key).sum(axis=1, dtype=np.uint64)
    assert int(np.abs(ph.view(np.int64)).max()) < 2 ** 50
    prm = O.params(tfhe_amd.PRESET_FHEVM_FFT)
    keys = O.Keys.__new__(O.Keys)
    keys.prm, keys.seed, keys.lwe_key, keys.glwe_key = prm, 0, tk.lwe_key, tk.glwe_key
    keys.bsk, keys.ksk, keys._bsk_ntt, keys.ms_zeros = sk.bsk, sk.ksk, None, sk.ms_zeros
    m = np.array([1, 3, 12], dtype=np.uint64)          # message x carry space 16, Delta = 2^63 / 16
    cts = ck.encrypt(m, 16, seed=0xABC)
    lut = O.lut_from_table(2048, 16, [(3 * v + 1) % 16 for v in range(16)], (1 << 63) // 16)
    out = O.pbs_batch_fft(prm, keys, cts, lut[None])
    assert np.array_equal(ck.decrypt(out, 16), (3 * m + 1) % 16)
