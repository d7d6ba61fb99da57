"""Noise squashing on the MI355X (tfhe_amd/csrc/sns.hip) against the oracle: the 128-bit blind
rotation accumulator and the squashed LWE bit-exact, and the full path from P-FHEVM big-key
ciphertexts (engine keyswitch + MS noise reduction + squash) decrypting every message."""
import numpy as np
import pytest

from conftest import KEY_SEED
from tfhe_amd import sns as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sns_setup(fhevm_keys, oracle_mod):
    ck, _ = fhevm_keys
    sp = S.SnsParams.preset(0)
    key = S.SquashedKey(sp, KEY_SEED, ck.lwe_key)
    osp = oracle_mod.sns_params(0)
    okey = oracle_mod.SnsKeys(osp, KEY_SEED, ck.lwe_key)
    assert np.array_equal(key.bsk, okey.bsk)
    sq = S.Squasher(sp, 0).load_key(key)
    yield sp, osp, key, okey, sq
    sq.close()


def test_squash_vs_oracle(sns_setup, fhevm_engine, fhevm_keys, oracle_mod):
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = np.array([1, 7, 14], dtype=np.uint64)
    small = fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE71))
    small, _ = fhevm_engine.ms_reduce(small)
    acc = sq.blind_rotate(small[:1])
    lut = oracle_mod.sns_lut_identity(osp, 16)
    assert np.array_equal(acc[0], oracle_mod.sns_blind_rotate(osp, okey, small[0], lut))
    out = sq.squash(small)
    assert np.array_equal(out, oracle_mod.sns_squash(osp, okey, small, 16, threads=16))
    assert np.array_equal(key.decrypt(out), msgs)


def test_squash_noise_batch(sns_setup, fhevm_engine, fhevm_keys):
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    B = 300
    msgs = (np.arange(B) % 16).astype(np.uint64)
    out = S.squash_noise(fhevm_engine, sq, ck.encrypt(msgs, 16, seed=0xC0FFEE72))
    assert out.shape == (B, 4097, 2)
    assert np.array_equal(key.decrypt(out), msgs)
    delta = 1 << 123
    noise = [((v - int(m) * delta + (1 << 127)) % (1 << 128)) - (1 << 127) for v, m in zip(key.phase(out), msgs)]
    assert max(abs(e) for e in noise) < 2 ** 72


def test_squash_arbitrary_words_vs_oracle(sns_setup, oracle_mod):
    """Arithmetic parity beyond valid encryptions: uniform random 64-bit input words (every mask
    coefficient a rotation, worst-case digits), a trivial ciphertext (zero mask: no CMUX moves the
    accumulator) and one whose mask is all 2^63 (rotation by N): squashed LWEs bit-exact."""
    sp, osp, key, okey, sq = sns_setup
    rng = np.random.default_rng(0x5A5)
    small = rng.integers(0, 2 ** 64 - 1, size=(4, sp.n + 1), dtype=np.uint64)
    small[2, :-1] = 0
    small[3, :-1] = np.uint64(1 << 63)
    out = sq.squash(small)
    assert np.array_equal(out, oracle_mod.sns_squash(osp, okey, small, 16, threads=16))


def test_mac_slot_walk_vs_oracle(sns_setup, fhevm_engine, fhevm_keys, oracle_mod):
    """300 ciphertexts = 10 MAC groups of 32 over 8 group slots (slots 0 and 1 walk a second group, the last
    one ragged): every message decrypts, and ciphertexts of the first and the walked groups are bit-exact."""
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = (np.arange(300) * 7 % 16).astype(np.uint64)
    small, _ = fhevm_engine.ms_reduce(fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE75)))
    out = sq.squash(small)
    assert np.array_equal(key.decrypt(out), msgs)
    sel = np.array([0, 31, 256, 290, 299])
    assert np.array_equal(out[sel], oracle_mod.sns_squash(osp, okey, small[sel], 16, threads=16))
