"""Compressed (seeded) server keys on the MI355X: a P-FHEVM key set issued in seeded form, moved
through the safe_serialize container, decompressed (tfhe_hip_decompress_*) and loaded into an engine; its KS -> MS
noise reduction -> PBS batch is bit-exact with the CPU oracle on the same decompressed keys and decrypts.  The byte
layout of a real tfhe-rs CompressedServerKey is parity unpinned (tests/test_seeded.py)."""
import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import keyio

pytestmark = pytest.mark.gpu
MM = 16
DELTA = (1 << 63) // MM


def test_seeded_fhevm_key_bootstraps_bit_exact(oracle_mod):
    p = tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT)
    ck, _ = tfhe_amd.gen_keys(p, 0x5EED5EED, with_server_key=False)
    csk = keyio.compress_server_key(ck, seed=0x5EED0003, ms_count=tfhe_amd.MS_FHEVM["count"])
    csk = keyio.loads_compressed_server_key(keyio.dumps_compressed_server_key(csk))
    p2, sk = keyio.decompress_server_key(csk)
    assert sk.ms_zeros.shape == (1449, 919)
    msgs = np.arange(37, dtype=np.uint64) % MM
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE70)
    lut = oracle_mod.lut_from_table(2048, MM, [(5 * m + 3) % MM for m in range(MM)], DELTA)
    with tfhe_amd.Engine(p2, 0) as eng:
        eng.load_keys(sk)
        out = eng.pbs(cts, lut[None])
    assert np.array_equal(ck.decrypt(out, MM), (5 * msgs + 3) % MM)
    prm = oracle_mod.params(tfhe_amd.PRESET_FHEVM_FFT)
    keys = oracle_mod.Keys.__new__(oracle_mod.Keys)
    keys.prm, keys.seed, keys.lwe_key, keys.glwe_key = prm, 0, ck.lwe_key, ck.glwe_key
    keys.bsk, keys.ksk, keys._bsk_ntt, keys.ms_zeros = sk.bsk, sk.ksk, None, sk.ms_zeros
    ref = oracle_mod.pbs_batch_fft(prm, keys, cts[:6], lut[None])
    assert np.array_equal(out[:6], ref)
