"""GPU parity of the FFT64 engine at N = 2048 (P-FHEVM, the one-wave 1024-point transform of fft1k.h and
pbs_fft2k.hip) against oracle/fft_oracle.c, bit-exact through the C ABI: the transform both ways, blind-rotation
accumulators, the full KS -> MS noise reduction -> BR -> SE PBS with multiple LUTs on ragged batches (padding in the
last workgroup), the latency (2 ciphertexts per workgroup) and batch (4) kernels against each other, and a 4096
batch by decryption plus a sampled bit-exact subset.
"""
import numpy as np
import pytest

from conftest import KEY_SEED

import tfhe_amd

pytestmark = pytest.mark.gpu
N = 2048
MM = 16
DELTA = (1 << 63) // MM


@pytest.fixture(scope="module")
def f2_keys():
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_FHEVM_FFT), KEY_SEED)


@pytest.fixture(scope="module")
def f2_engine(f2_keys):
    ck, sk = f2_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def f2_prm(oracle_mod):
    return oracle_mod.params(3)


@pytest.fixture(scope="module")
def f2_okeys(oracle_mod, f2_prm):
    return oracle_mod.Keys(f2_prm, KEY_SEED)


def test_fft2k_forward_inverse_bitexact(f2_engine, oracle_mod):
    assert f2_engine.br_kernel(4096) == "blind_rotate_fft2k_kernel"
    rng = np.random.default_rng(41)
    x = rng.integers(0, 2**64, size=(11, N), dtype=np.uint64)
    x[0] = 0
    x[1] = np.uint64(2**63)
    x[2] = rng.integers(0, 2**23 + 1, N).astype(np.uint64) - np.uint64(2**22)  # digit-sized values
    Z = f2_engine.fft_fwd(x)
    Zo = oracle_mod.fft_fwd(x.view(np.int64).astype(np.float64))
    assert np.array_equal(Z.view(np.uint64), Zo.view(np.uint64)), "forward FFT differs from the oracle"
    y = f2_engine.fft_inv(Zo)
    yo = oracle_mod.fft_inv(Zo)
    assert np.array_equal(y.view(np.uint64), yo.view(np.uint64)), "inverse FFT differs from the oracle"
    assert np.max(np.abs(y[3] / 1024 - x[3].view(np.int64).astype(np.float64))) <= 2.0**24


def test_blind_rotate2k_accumulators_bitexact(f2_engine, f2_keys, oracle_mod, f2_prm, f2_okeys):
    ck, _ = f2_keys
    rng = np.random.default_rng(42)
    msgs = rng.integers(0, MM, 6).astype(np.uint64)
    small = f2_engine.keyswitch(ck.encrypt(msgs, MM, seed=0xC0FFEE61))
    luts = np.stack([oracle_mod.lut_from_table(N, MM, [(m * 5 + 3) % MM for m in range(MM)], DELTA),
                     oracle_mod.lut_from_table(N, MM, list(range(MM)), DELTA)])
    idx = np.array([0, 1, 0, 1, 1, 0], dtype=np.uint32)
    acc = f2_engine.blind_rotate(small, luts, idx)
    for i in range(6):
        ref = oracle_mod.blind_rotate_fft(f2_prm, f2_okeys, small[i], luts[idx[i]])
        assert np.array_equal(acc[i], ref), f"accumulator {i} differs from the oracle"
    big = f2_engine.sample_extract(acc)
    for i in range(6):
        assert np.array_equal(big[i], oracle_mod.sample_extract_torus(f2_prm, acc[i]))


@pytest.mark.parametrize("B", [1, 5, 23])
def test_pbs2k_bitexact_ragged_multi_lut(f2_engine, f2_keys, oracle_mod, f2_prm, f2_okeys, B):
    ck, _ = f2_keys
    rng = np.random.default_rng(43 + B)
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE70 + B)
    luts = np.stack([oracle_mod.lut_from_table(N, MM, [(m * (s + 1) + s) % MM for m in range(MM)], DELTA)
                     for s in range(3)])
    idx = rng.integers(0, 3, B).astype(np.uint32)
    out = f2_engine.pbs(cts, luts, idx)
    ref = oracle_mod.pbs_batch_fft(f2_prm, f2_okeys, cts, luts, idx)
    assert np.array_equal(out, ref)
    want = (msgs * (idx.astype(np.uint64) + 1) + idx.astype(np.uint64)) % MM
    assert np.array_equal(ck.decrypt(out, MM), want)


def test_pbs2k_batch_4096_decrypts_and_sampled_bitexact(f2_engine, f2_keys, oracle_mod, f2_prm, f2_okeys):
    ck, _ = f2_keys
    f = lambda m: (m * m + 3) % MM  # noqa: E731
    acc = f2_engine.generate_accumulator(f, MM)
    msgs = (np.arange(4096) % MM).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEE80)
    out = f2_engine.pbs(cts, acc)
    assert np.array_equal(ck.decrypt(out, MM), np.array([f(int(m)) for m in msgs], dtype=np.uint64))
    # batch ends plus the workgroup boundaries where the wave priority (blockIdx bit 8, 2 ciphertexts per workgroup)
    # switches: ciphertexts 512 and 1024
    sample = np.r_[0:8, 510:514, 1022:1026, 4088:4096]
    assert np.array_equal(out[sample], oracle_mod.pbs_batch_fft(f2_prm, f2_okeys, cts[sample], acc[None]))
    out2 = f2_engine.pbs(out[:512], acc)  # chained: f(f(m))
    assert np.array_equal(ck.decrypt(out2, MM), np.array([f(f(int(m))) for m in msgs[:512]], dtype=np.uint64))


@pytest.mark.parametrize("B", [1, 7, 100, 513])
def test_latency_and_batch_kernels_agree_2k(f2_engine, f2_keys, oracle_mod, f2_prm, f2_okeys, B):
    ck, _ = f2_keys
    rng = np.random.default_rng(B + 4096)
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEEA0 + B)
    lut = oracle_mod.lut_from_table(N, MM, [(7 * m + 2) % MM for m in range(MM)], DELTA)
    small = f2_engine.keyswitch(cts)
    try:
        f2_engine.set_latency_batch(0)
        acc_b = f2_engine.blind_rotate(small, lut)
        out_b = f2_engine.pbs(cts, lut)
        f2_engine.set_latency_batch(1 << 20)
        acc_l = f2_engine.blind_rotate(small, lut)
        out_l = f2_engine.pbs(cts, lut)
    finally:
        f2_engine.set_latency_batch(512)  # the N = 2048 FFT64 default
    assert np.array_equal(acc_l, acc_b)
    assert np.array_equal(out_l, out_b)
    i = B // 2
    assert np.array_equal(acc_l[i], oracle_mod.blind_rotate_fft(f2_prm, f2_okeys, small[i], lut))
    assert np.array_equal(ck.decrypt(out_l, MM), (7 * msgs + 2) % MM)


def test_pbs2k_batch_kernel_ragged_multi_lut_1027(f2_engine, f2_keys, oracle_mod, f2_prm, f2_okeys):
    """Above the latency crossover (512) with a ragged last workgroup (1027 = 4 * 256 + 3) and three
    LUTs: every output decrypts to its LUT's value, a sample across the padding edge is bit-exact."""
    ck, _ = f2_keys
    B = 1027
    rng = np.random.default_rng(1027)
    msgs = rng.integers(0, MM, B).astype(np.uint64)
    cts = ck.encrypt(msgs, MM, seed=0xC0FFEEB0)
    luts = np.stack([oracle_mod.lut_from_table(N, MM, [(m * (s + 2) + 1) % MM for m in range(MM)], DELTA)
                     for s in range(3)])
    idx = rng.integers(0, 3, B).astype(np.uint32)
    out = f2_engine.pbs(cts, luts, idx)
    want = (msgs * (idx.astype(np.uint64) + 2) + 1) % MM
    assert np.array_equal(ck.decrypt(out, MM), want)
    sample = np.r_[0:4, 1020:1027]
    ref = oracle_mod.pbs_batch_fft(f2_prm, f2_okeys, cts[sample], luts, idx[sample])
    assert np.array_equal(out[sample], ref)
