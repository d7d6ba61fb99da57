"""Packing keyswitch + compression (tfhe_amd/compression.py) on CPU: the product's
host pieces (key generation, modulus switch + bit packing, extraction, GLWE decryption) against the
oracle (oracle/tfhe_oracle.h or_pks_params), and the oracle's packing rule against decryption.
The device packing keyswitch is tests/test_gpu_compression.py."""
import ctypes

import numpy as np
import pytest

from tfhe_amd import compression as C

SEED = 0x7F4E0001


@pytest.fixture(scope="module")
def pks(oracle_mod):
    pp = C.PksParams.preset(C.PKS_PRESET_ML2048)
    opp = oracle_mod.pks_params(0)
    in_key = np.random.default_rng(5).integers(0, 2, pp.in_dim).astype(np.uint64)
    return pp, opp, C.CompressionKey(pp, SEED, in_key), oracle_mod.PksKeys(opp, SEED, in_key)


def encrypt_lwes(oracle_mod, key, msgs, seed=9, noise_log2=-48):
    msgs = np.ascontiguousarray(msgs, dtype=np.uint64)
    out = np.zeros((msgs.size, key.size + 1), dtype=np.uint64)
    oracle_mod.lib().or_lwe_encrypt(ctypes.c_uint32(key.size), oracle_mod._p(key), ctypes.c_int32(noise_log2),
                                    ctypes.c_uint64(seed), ctypes.c_uint64(0), oracle_mod._p(msgs),
                                    ctypes.c_size_t(msgs.size), oracle_mod._p(out))
    return out


def test_preset_is_reference_params(pks):
    pp = pks[0]
    assert (pp.in_dim, pp.out_k, pp.out_N, pp.base_log, pp.level, pp.lwe_per_glwe, pp.storage_log) == \
        (2048, 1, 2048, 14, 2, 2048, 26)


def test_keygen_matches_oracle(pks):
    pp, opp, ck, ok = pks
    assert np.array_equal(ck.post_packing_key, ok.out_key)
    assert np.array_equal(ck.pksk, ok.pksk)
    assert ck.pksk.size == 2048 * 2 * 2 * 2048


@pytest.mark.parametrize("bodies", [0, 1, 100, 2048])
def test_compress_extract_match_oracle(pks, oracle_mod, bodies):
    pp, opp, _, _ = pks
    g = np.random.default_rng(bodies).integers(0, 2 ** 64 - 1, pp.glwe_len, dtype=np.uint64)
    c = C.compress_glwe(pp, g, bodies)
    assert np.array_equal(c.packed, oracle_mod.pks_compress(opp, g, bodies))
    assert c.packed.size == -(-(2048 + bodies) * 26 // 64)
    x = c.extract()
    assert np.array_equal(x, oracle_mod.pks_extract(opp, c.packed, bodies))
    n = 2048 + bodies
    err = (x[:n] - g[:n]).view(np.int64)                  # modulus-switch rounding only
    assert np.abs(err).max() <= 2 ** 37
    assert not x[n:].any()


def test_oracle_pack_decrypts_and_extracts(pks, oracle_mod):
    pp, opp, ck, ok = pks
    msgs = (np.arange(6, dtype=np.uint64) * 37 + 5) << np.uint64(40)
    lwes = encrypt_lwes(oracle_mod, ok.in_key, msgs)
    g = oracle_mod.pks_pack(opp, ok, lwes)
    ph = C.glwe_phase(1, 2048, ck.post_packing_key, g)
    err = (ph[:6] - msgs).view(np.int64)
    assert np.abs(err).max() < 2 ** 43                      # decomposition 2 x 2^14 -> ~2^40 noise
    assert np.abs(ph[6:].view(np.int64)).max() < 2 ** 43   # unused coefficients carry noise only
    for i in (0, 3, 5):                                    # LWE extraction at degree i
        lwe = C.extract_lwe(pp, g, i)
        s = int(lwe[-1]) - sum(int(a) * int(b) for a, b in zip(lwe[:-1], ck.post_packing_key))
        assert (s - int(ph[i])) % (1 << 64) == 0
    comp = C.compress_glwe(pp, g, 6)
    ph2 = C.glwe_phase(1, 2048, ck.post_packing_key, comp.extract())
    assert np.abs((ph2[:6] - msgs).view(np.int64)).max() < 2 ** 45
    assert comp.nbytes == 8 * -(-(2048 + 6) * 26 // 64)
