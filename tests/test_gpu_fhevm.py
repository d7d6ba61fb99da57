"""P-FHEVM on the MI355X: n=918, k=1, N=2048, PBS 2^23 x 1, KS 2^4 x 4, KS -> PBS
(PARAM_MESSAGE_2_CARRY_2_KS_PBS_TUNIFORM_2M128, sdk/relayer/src/tfhe.ts:14-19).

Bit-exact against the C oracle at every stage (N=2048 NTT, blind rotation, sample extraction,
keyswitch 2048 -> 918, full PBS) and message-level checks with the shortint encoding
(message 2 bits + carry 2 bits, one padding bit: delta = 2^63 / 16).  TUniform noise of the real
parameter set is modelled by a Gaussian of the same order (oracle header)."""
import numpy as np
import pytest

from conftest import KEY_SEED

pytestmark = pytest.mark.gpu
P = 0xFFFFFFFF00000001
MM = 16                      # message x carry space of P-FHEVM
DELTA = (1 << 63) // MM


@pytest.fixture(scope="module")
def fprm(oracle_mod):
    return oracle_mod.params(1)


@pytest.fixture(scope="module")
def fkeys_oracle(oracle_mod, fprm):
    return oracle_mod.Keys(fprm, KEY_SEED)


@pytest.fixture(scope="module")
def fkeys(fhevm_keys):
    return fhevm_keys


@pytest.fixture(scope="module")
def fengine(fhevm_engine):
    return fhevm_engine


def test_ntt2048_vs_oracle(fengine, oracle_mod):
    rng = np.random.default_rng(2048)
    x = rng.integers(0, P, size=(9, 2048), dtype=np.uint64)
    X = fengine.ntt_fwd(x)
    assert np.array_equal(X, oracle_mod.ntt_fwd(x))
    assert np.array_equal(fengine.ntt_inv(X), x)
    assert np.array_equal(fengine.ntt_inv(x), oracle_mod.ntt_inv(x))
    e = np.zeros((1, 2048), dtype=np.uint64)
    e[0, 1] = 1                                   # X -> psi^(2j+1)
    assert np.array_equal(fengine.ntt_fwd(e), oracle_mod.ntt_fwd(e))


def test_blind_rotate2048_vs_oracle(fengine, oracle_mod, fprm, fkeys_oracle):
    rng = np.random.default_rng(7)
    small = rng.integers(0, 2**64 - 1, size=(5, 919), dtype=np.uint64)   # 5: pads a 4-ciphertext workgroup
    lut = oracle_mod.lut_from_table(2048, MM, [(3 * m + 1) % MM for m in range(MM)], DELTA)
    acc = fengine.blind_rotate(small, lut)
    for i in (0, 3, 4):
        assert np.array_equal(acc[i], oracle_mod.blind_rotate(fprm, fkeys_oracle, small[i], lut)), i


def test_sample_extract2048_and_keyswitch_vs_oracle(fengine, oracle_mod, fprm, fkeys_oracle):
    rng = np.random.default_rng(8)
    acc = rng.integers(0, P, size=(3, 4096), dtype=np.uint64)
    se = fengine.sample_extract(acc)
    for i in range(3):
        assert np.array_equal(se[i], oracle_mod.sample_extract(fprm, acc[i]))
    big = rng.integers(0, 2**64 - 1, size=(70, 2049), dtype=np.uint64)
    ks = fengine.keyswitch(big)
    for i in (0, 1, 63, 64, 69):
        assert np.array_equal(ks[i], oracle_mod.keyswitch(fprm, fkeys_oracle, big[i])), i


def test_pbs2048_vs_oracle_and_messages(fengine, fkeys, oracle_mod, fprm, fkeys_oracle):
    ck, _ = fkeys
    rng = np.random.default_rng(21)
    B = 9
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE21)
    luts = np.stack([oracle_mod.lut_from_table(2048, MM, [(m * (s + 1) + s) % MM for m in range(MM)], DELTA)
                     for s in range(3)])
    idx = (np.arange(B) % 3).astype(np.uint32)
    out = fengine.pbs(cts, luts, idx)
    ref = oracle_mod.pbs_batch(fprm, fkeys_oracle, cts, luts, idx)
    assert np.array_equal(out, ref)
    want = (msgs * (idx.astype(np.uint64) + 1) + idx.astype(np.uint64)) % MM
    assert np.array_equal(ck.decrypt(out, MM), want)


def test_pbs2048_all_messages_and_batch(fengine, fkeys):
    ck, _ = fkeys
    f = lambda m: (m * m + 3) % MM                # noqa: E731
    acc = fengine.generate_accumulator(f, MM)
    B = 1000                                      # 250 workgroups, crosses KS tiles
    msgs = (np.arange(B) % MM).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE22)
    out = fengine.keyswitch_programmable_bootstrap(cts, acc)
    assert np.array_equal(ck.decrypt(out, MM), np.array([f(int(m)) for m in msgs], dtype=np.uint64))
    # chained: f(f(m))
    out2 = fengine.pbs(out, acc)
    assert np.array_equal(ck.decrypt(out2, MM), np.array([f(f(int(m))) for m in msgs], dtype=np.uint64))


@pytest.mark.parametrize("B", [1, 6, 130])
def test_latency_and_batch_kernels_agree_2048(fengine, fkeys, oracle_mod, fprm, fkeys_oracle, B):
    ck, _ = fkeys
    rng = np.random.default_rng(B + 2048)
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE40 + B)
    lut = oracle_mod.lut_from_table(2048, MM, [(7 * m + 2) % MM for m in range(MM)], DELTA)
    small = fengine.keyswitch(cts)
    try:
        fengine.set_latency_batch(0)
        acc_b = fengine.blind_rotate(small, lut)
        out_b = fengine.pbs(cts, lut)
        fengine.set_latency_batch(1 << 20)
        acc_l = fengine.blind_rotate(small, lut)
        out_l = fengine.pbs(cts, lut)
    finally:
        fengine.set_latency_batch(512)
    assert np.array_equal(acc_l, acc_b)
    assert np.array_equal(out_l, out_b)
    i = B // 2
    assert np.array_equal(acc_l[i], oracle_mod.blind_rotate(fprm, fkeys_oracle, small[i], lut))
    assert np.array_equal(ck.decrypt(out_l, MM), (7 * msgs + 2) % MM)


@pytest.mark.parametrize("B", [1, 9, 300])
def test_ms_noise_reduction_vs_oracle(fengine, fkeys, oracle_mod, fprm, fkeys_oracle, B):
    """Modulus-switch noise reduction kernel (ms_reduce.hip) == oracle: same zero chosen, same
    ciphertext, on real keyswitch outputs (early exit after 1-2 tiles of zeros) and on uniformly
    random ciphertexts (no zero reaches the bound: full scan of all 1449 + argmin)."""
    ck, _ = fkeys
    rng = np.random.default_rng(B + 31)
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    small = fengine.keyswitch(ck.encrypt(msgs, MM, seed=0xC0FFEE50 + B))
    small[: max(1, B // 10)] = rng.integers(0, 2 ** 64 - 1, size=(max(1, B // 10), 919), dtype=np.uint64)
    out, picks = fengine.ms_reduce(small)
    ref, rpicks = oracle_mod.ms_reduce(fprm, fkeys_oracle, small)
    assert np.array_equal(picks, rpicks)
    assert np.array_equal(out, ref)
    if B >= 9:
        assert (picks >= 0).mean() > 0.5


def test_ms_noise_reduction_in_pbs(fengine, fkeys, oracle_mod, fprm, fkeys_oracle):
    """The full P-FHEVM PBS applies the reduction (KS -> MS -> BR): bit-exact with the oracle with it,
    different from the oracle without it, and decrypting correctly either way."""
    ck, _ = fkeys
    B = 40
    msgs = (np.arange(B) % MM).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE60)
    lut = oracle_mod.lut_from_table(2048, MM, [(5 * m + 3) % MM for m in range(MM)], DELTA)
    out = fengine.pbs(cts, lut)
    assert np.array_equal(out, oracle_mod.pbs_batch(fprm, fkeys_oracle, cts, lut))
    plain = oracle_mod.pbs_batch(fprm, fkeys_oracle, cts, lut, ms=False)
    assert not np.array_equal(out, plain)
    want = (5 * msgs + 3) % MM
    assert np.array_equal(ck.decrypt(out, MM), want) and np.array_equal(ck.decrypt(plain, MM), want)
    try:
        fengine.load_ms_key(None)                     # disabled: the plain path
        assert np.array_equal(fengine.pbs(cts, lut), plain)
    finally:
        fengine.load_ms_key(fkeys[1].ms_zeros)


def test_ms_key_refused_for_pbs_ks_order(engine):
    import tfhe_amd
    z = np.zeros((4, 631), dtype=np.uint64)
    with pytest.raises(tfhe_amd.TfheError, match="EUNSUPPORTED"):
        engine.load_ms_key(z)


def test_ms_key_refuses_keys_beyond_the_scan_window(fengine, fkeys):
    """The scan reads the key's element-major transpose through a buffer resource with 32-bit offsets: a key with
    (n + 1) x pitch x 8 >= 2^31 bytes is refused up front, not scanned with silently zeroed loads.
    Called through the C ABI with a one-row buffer: the size check comes before anything is read."""
    import ctypes
    import tfhe_amd
    one = np.zeros(919, dtype=np.uint64)
    big = (2**31 // (919 * 8)) // 64 * 64 + 64           # the first 64-multiple past the window at n = 918
    rc = tfhe_amd.lib().tfhe_hip_load_ms_key(fengine._h, one.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                              big, 2.0**58, 13.18, 2.63e-7)
    assert rc == -1                                      # TFHE_HIP_EINVAL
    assert "2 GiB scan window" in tfhe_amd.lib().tfhe_hip_last_error().decode()
    fengine.load_ms_key(fkeys[1].ms_zeros)                 # the real key still loads afterwards
