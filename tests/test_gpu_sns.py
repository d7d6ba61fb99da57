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


def test_ntt_path_agrees_with_fft_path(sns_setup, fhevm_engine, fhevm_keys, monkeypatch):
    """The default f64 FFT external product (exact limb convolutions) and the Z_p NTT one
    (TFHE_HIP_SNS_NTT=1) compute the same Z_Q product of the load-time rounded key: equal accumulators."""
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = np.array([0, 3, 9, 15, 6], dtype=np.uint64)
    small, _ = fhevm_engine.ms_reduce(fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE73)))
    monkeypatch.setenv("TFHE_HIP_SNS_NTT", "1")
    sq_ntt = S.Squasher(sp, 0).load_key(key)
    try:
        assert np.array_equal(sq_ntt.blind_rotate(small), sq.blind_rotate(small))
        assert np.array_equal(key.decrypt(sq_ntt.squash(small)), msgs)
    finally:
        sq_ntt.close()


@pytest.mark.parametrize("switch", ["TFHE_HIP_SNS_FUSED2", "TFHE_HIP_SNS_INVW"])
def test_fft_variants_agree(sns_setup, fhevm_engine, fhevm_keys, monkeypatch, switch):
    """The measured alternatives of the FFT path (one-kernel step 2; one wave per limb inverse) give the
    default path's accumulators bit for bit."""
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = np.array([2, 11], dtype=np.uint64)
    small, _ = fhevm_engine.ms_reduce(fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE74)))
    ref = sq.blind_rotate(small)
    monkeypatch.setenv(switch, "1")
    assert np.array_equal(sq.blind_rotate(small), ref)


@pytest.mark.parametrize("slots", ["1", "3"])
def test_mac_slot_walk_agrees(sns_setup, fhevm_engine, fhevm_keys, monkeypatch, slots):
    """The MAC grid with fewer ciphertext-group slots than groups (each workgroup stages its key tile
    once and walks groups g, g + G, ...; 100 ciphertexts = 3 full groups of 32 + a ragged one) gives
    the one-group-per-workgroup accumulators bit for bit."""
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = (np.arange(100) % 16).astype(np.uint64)
    small, _ = fhevm_engine.ms_reduce(fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE75)))
    monkeypatch.setenv("TFHE_HIP_SNS_MACG", "0")
    ref = sq.blind_rotate(small)
    monkeypatch.setenv("TFHE_HIP_SNS_MACG", slots)
    assert np.array_equal(sq.blind_rotate(small), ref)
    assert np.array_equal(key.decrypt(sq.squash(small)), msgs)


@pytest.mark.parametrize("occ", ["3", "4", "5", "13", "14"])
def test_inverse_occupancy_variants_agree(sns_setup, fhevm_engine, fhevm_keys, monkeypatch, occ):
    """The inverse kernel's measured forms (all five stages through LDS, unrolled at 3 waves/SIMD or
    rolled at 4 and 5; twiddles from an LDS table at 3 and 4) give the default (register-ended stages)
    accumulators bit for bit."""
    sp, osp, key, okey, sq = sns_setup
    ck, _ = fhevm_keys
    msgs = np.array([5, 14, 1], dtype=np.uint64)
    small, _ = fhevm_engine.ms_reduce(fhevm_engine.keyswitch(ck.encrypt(msgs, 16, seed=0xC0FFEE76)))
    ref = sq.blind_rotate(small)
    monkeypatch.setenv("TFHE_HIP_SNS_INVOCC", occ)
    assert np.array_equal(sq.blind_rotate(small), ref)
