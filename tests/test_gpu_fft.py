"""GPU parity of the FFT64 transform (pbs_fft.hip) against oracle/fft_oracle.c, bit-exact, through the
C ABI: the transform itself, the blind rotation accumulators, full PBS (multi-LUT, ragged batches that
leave padding waves in the last workgroup), gate bootstrapping, and a 4096 batch by decryption plus a
sampled bit-exact subset.
"""
import numpy as np
import pytest

from conftest import KEY_SEED

import tfhe_amd

pytestmark = pytest.mark.gpu
N = 1024


@pytest.fixture(scope="module")
def fft_keys():
    return tfhe_amd.gen_keys(tfhe_amd.Params.preset(tfhe_amd.PRESET_GATE_FFT), KEY_SEED)


@pytest.fixture(scope="module")
def fft_engine(fft_keys):
    ck, sk = fft_keys
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield eng
    eng.close()


@pytest.fixture(scope="module")
def fft_params(oracle_mod):
    return oracle_mod.params(2)


@pytest.fixture(scope="module")
def fft_okeys(oracle_mod, fft_params):
    return oracle_mod.Keys(fft_params, KEY_SEED)


def test_fft_forward_inverse_bitexact(fft_engine, oracle_mod):
    rng = np.random.default_rng(31)
    x = rng.integers(0, 2**64, size=(19, N), dtype=np.uint64)
    x[0] = 0
    x[1] = np.uint64(2**63)                       # most negative int64
    x[2] = rng.integers(0, 129, N).astype(np.uint64) - np.uint64(64)  # digit-sized values
    Z = fft_engine.fft_fwd(x)
    Zo = oracle_mod.fft_fwd(x.view(np.int64).astype(np.float64))
    assert np.array_equal(Z.view(np.uint64), Zo.view(np.uint64)), "forward FFT differs from the oracle"
    y = fft_engine.fft_inv(Zo)
    yo = oracle_mod.fft_inv(Zo)
    assert np.array_equal(y.view(np.uint64), yo.view(np.uint64)), "inverse FFT differs from the oracle"
    # and it is a transform: inverse(forward(x)) / M == x up to f64 rounding (2^-40 of 2^63 values)
    assert np.max(np.abs(y[3] / 512 - x[3].view(np.int64).astype(np.float64))) <= 2.0**23


def test_blind_rotate_accumulators_bitexact(fft_engine, fft_keys, oracle_mod, fft_params, fft_okeys):
    ck, _ = fft_keys
    rng = np.random.default_rng(32)
    cts = ck.encrypt_torus(rng.integers(0, 2**63, 5, dtype=np.uint64), seed=0xC0FFEE31)
    luts = np.stack([oracle_mod.lut_from_table(N, 8, [(m * 5 + 3) % 8 for m in range(8)], (1 << 63) // 8),
                     oracle_mod.lut_constant(N, 1 << 61)])
    idx = np.array([0, 1, 0, 1, 1], dtype=np.uint32)
    acc = fft_engine.blind_rotate(cts, luts, idx)
    for i in range(5):
        ref = oracle_mod.blind_rotate_fft(fft_params, fft_okeys, cts[i], luts[idx[i]])
        assert np.array_equal(acc[i], ref), f"accumulator {i} differs from the oracle"
    big = fft_engine.sample_extract(acc)
    for i in range(5):
        assert np.array_equal(big[i], oracle_mod.sample_extract_torus(fft_params, acc[i]))


@pytest.mark.parametrize("B", [1, 13, 37])
def test_pbs_bitexact_ragged(fft_engine, fft_keys, oracle_mod, fft_params, fft_okeys, B):
    ck, _ = fft_keys
    rng = np.random.default_rng(33 + B)
    msgs = rng.integers(0, 8, B).astype(np.uint64) * np.uint64((1 << 63) // 8)
    cts = ck.encrypt_torus(msgs, seed=0xC0FFEE40 + B)
    luts = np.stack([oracle_mod.lut_from_table(N, 8, [(m + s) % 8 for m in range(8)], (1 << 63) // 8)
                     for s in range(3)])
    idx = rng.integers(0, 3, B).astype(np.uint32)
    out = fft_engine.pbs(cts, luts, idx)
    ref = oracle_mod.pbs_batch_fft(fft_params, fft_okeys, cts, luts, idx)
    assert np.array_equal(out, ref)
    m = np.array([int(v) for v in msgs]) // ((1 << 63) // 8)
    dec = [((int(p) + (1 << 59)) >> 60) % 16 for p in ck.phase(out)]
    assert dec == [int((mm + idx[q]) % 8) for q, mm in enumerate(m)]


def test_gates_on_fft_engine(fft_engine, fft_keys):
    ck, _ = fft_keys
    rng = np.random.default_rng(34)
    a, b = rng.integers(0, 2, 64).astype(bool), rng.integers(0, 2, 64).astype(bool)
    ca, cb = ck.encrypt_bool(a, seed=0xC0FFEE51), ck.encrypt_bool(b, seed=0xC0FFEE52)
    assert np.array_equal(ck.decrypt_bool(fft_engine.nand(ca, cb)), ~(a & b))
    x = tfhe_amd.FheBool(fft_engine, ca)
    y = tfhe_amd.FheBool(fft_engine, cb)
    assert np.array_equal((x ^ y).decrypt(ck), a ^ b)
    assert np.array_equal((x & y).decrypt(ck), a & b)


def test_batch_4096_decrypts_and_sampled_bitexact(fft_engine, fft_keys, oracle_mod, fft_params, fft_okeys):
    ck, _ = fft_keys
    rng = np.random.default_rng(35)
    bits = rng.integers(0, 2, 4096).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE03)
    out = fft_engine.pbs(cts, fft_engine.gate_lut())
    assert np.array_equal(ck.decrypt_bool(out), bits)
    # ends of the batch, plus the workgroup boundaries where the pair kernel's wave priority (blockIdx bit 8) and
    # its start stagger (workgroups 256..511) switch: 2 ciphertexts per workgroup, so ciphertexts 512, 1024, 2048
    sample = np.r_[0:16, 510:514, 1022:1026, 2046:2050, 4080:4096]
    ref = oracle_mod.pbs_batch_fft(fft_params, fft_okeys, cts[sample], oracle_mod.lut_constant(N, 1 << 61)[None])
    assert np.array_equal(out[sample], ref)


def test_batch_kernel_ragged_workgroups_agree(fft_engine, fft_keys):
    """The component-pair batch kernel runs 2 ciphertexts x 2 component waves per workgroup at any batch size above
    the latency range: a ragged batch (1025 = 512 full workgroups + one with a padding ciphertext) gives every
    ciphertext the same output as its first 1024 alone, and every output decrypts."""
    ck, _ = fft_keys
    bits = np.random.default_rng(0x4A8).integers(0, 2, 1025).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE4A)
    lut = fft_engine.gate_lut()
    out_r = fft_engine.pbs(cts, lut)
    out_f = fft_engine.pbs(cts[:1024], lut)
    assert np.array_equal(out_r[:1024], out_f)
    assert np.array_equal(ck.decrypt_bool(out_r), bits)


@pytest.mark.parametrize("B", [1, 9, 300])
def test_latency_and_batch_kernels_agree(fft_engine, fft_keys, oracle_mod, fft_params, fft_okeys, B):
    """The latency-mode kernel (one ciphertext per workgroup, 6 transforms in parallel) and the component-pair
    batch kernel (2 ciphertexts x 2 component waves per workgroup) produce identical accumulators and PBS outputs."""
    ck, _ = fft_keys
    rng = np.random.default_rng(B + 1024)
    msgs = rng.integers(0, 8, B).astype(np.uint64) * np.uint64((1 << 63) // 8)
    cts = ck.encrypt_torus(msgs, seed=0xC0FFEE90 + B)
    lut = oracle_mod.lut_from_table(N, 8, [(3 * m + 1) % 8 for m in range(8)], (1 << 63) // 8)
    try:
        fft_engine.set_latency_batch(0)
        acc_b = fft_engine.blind_rotate(cts, lut)
        out_b = fft_engine.pbs(cts, lut)
        fft_engine.set_latency_batch(1 << 20)
        acc_l = fft_engine.blind_rotate(cts, lut)
        out_l = fft_engine.pbs(cts, lut)
    finally:
        fft_engine.set_latency_batch(256)  # the P-GATE FFT64 default
    assert np.array_equal(acc_l, acc_b)
    assert np.array_equal(out_l, out_b)
    i = B // 2
    assert np.array_equal(acc_l[i], oracle_mod.blind_rotate_fft(fft_params, fft_okeys, cts[i], lut))


def test_fft_edge_cases(fft_engine, oracle_mod, fft_params, fft_okeys):
    """Empty batch, trivial ciphertexts (every CMUX skipped by the oracle, all-zero digits on the
    device), mask values on the modulus-switch rounding boundaries, and a bad lut_index (EINVAL)."""
    gate = fft_engine.gate_lut()
    lut = oracle_mod.lut_constant(N, 1 << 61)[None]
    assert fft_engine.pbs(np.zeros((0, 631), dtype=np.uint64), gate).shape == (0, 631)
    triv = np.zeros((3, 631), dtype=np.uint64)
    triv[:, 630] = [1 << 61, (1 << 64) - (1 << 61), (1 << 63) - 1]
    edge = np.zeros((2, 631), dtype=np.uint64)
    edge[0, :630] = np.uint64((1 << 52) - 1)
    edge[1, :630] = np.uint64((1 << 64) - (1 << 52))
    edge[:, 630] = 1 << 61
    for lat in (0, 1024):  # batch kernel and latency kernel
        fft_engine.set_latency_batch(lat)
        assert np.array_equal(fft_engine.pbs(triv, gate), oracle_mod.pbs_batch_fft(fft_params, fft_okeys, triv, lut))
        assert np.array_equal(fft_engine.pbs(edge, gate), oracle_mod.pbs_batch_fft(fft_params, fft_okeys, edge, lut))
    fft_engine.set_latency_batch(256)
    with pytest.raises(tfhe_amd.TfheError) as e:
        fft_engine.pbs(triv, gate, lut_index=[0, 1, 0])
    assert e.value.code == -1


def test_fft_large_batch_decrypts(fft_engine, fft_keys, oracle_mod, fft_params, fft_okeys):
    """C4-sized shard on one GPU (16,384 PBS = 4 rounds of the batch kernel's grid): every output
    decrypts, a sampled subset is bit-exact (size-independent properties)."""
    ck, _ = fft_keys
    B = 16384
    bits = np.random.default_rng(36).integers(0, 2, B).astype(bool)
    cts = ck.encrypt_bool(bits, seed=0xC0FFEE04)
    out = fft_engine.pbs(cts, fft_engine.gate_lut())
    assert np.array_equal(ck.decrypt_bool(out), bits)
    sample = np.r_[0:4, 8190:8194, B - 4:B]
    ref = oracle_mod.pbs_batch_fft(fft_params, fft_okeys, cts[sample], oracle_mod.lut_constant(N, 1 << 61)[None])
    assert np.array_equal(out[sample], ref)
