"""The exact arbiter of the FFT64 path (oracle/exact_oracle.c) on CPU.

* the limb / Goldilocks-NTT exact product equals the O(N^2) wrapping schoolbook (computations.rs:50-54 semantics)
  at both N, on random and edge operands;
* the exact CMUX / blind rotation decrypt to the LUT value (message level, main.rs:65-77 pattern);
* every CMUX of the FFT64 oracle's blind rotation (fft_oracle.c, the device's bit-exact twin) lands within the
  derived worst-case bound of the exact CMUX of the same input state, with an rms error matching the variance
  model (tests/fft_error_model.py), at P-GATE and P-FHEVM;
* the twiddle tables' accuracy the bound assumes.
The same checks against the GPU's states are tests/test_gpu_exact.py.
"""
import math

import numpy as np
import pytest

from conftest import KEY_SEED
import fft_error_model as fem


def test_exact_product_equals_schoolbook(oracle_mod):
    rng = np.random.default_rng(0xE1)
    for N, dmax in ((1024, 64), (2048, 2 ** 22)):
        for t in range(3):
            d = rng.integers(-dmax, dmax + 1, N)
            b = rng.integers(0, 2 ** 64, N, dtype=np.uint64)
            if t == 0:   # extreme operands: every key word at the wrap points, digits at +-max
                b[:] = np.uint64(2 ** 63)
                b[1::3] = np.uint64(2 ** 64 - 1)
                d[:] = dmax
                d[::2] = -dmax
            assert np.array_equal(oracle_mod.poly_mul_torus_exact(d, b), oracle_mod.poly_mul_torus_schoolbook(d, b))


def test_twiddle_accuracy(oracle_mod):
    """mu of the worst-case bound: every twiddle of the oracle's (= the device's) tables within 4 u of e^{2 pi i t/M}."""
    two_pi = np.longdouble("6.283185307179586476925286766559")
    worst = 0.0
    for M in (512, 2048, 4096):
        t = np.arange(M)
        x = two_pi * t.astype(np.longdouble) / np.longdouble(M)
        got = np.array([oracle_mod.fft_twiddle(int(i), M) for i in t], dtype=np.float64).astype(np.longdouble)
        worst = max(worst, float(np.sqrt((got[:, 0] - np.cos(x)) ** 2 + (got[:, 1] - np.sin(x)) ** 2).max()))
    assert worst <= fem.MU_BOUND, f"twiddle error {worst / fem.U:.2f} u"
    assert 0.5 <= fem.twiddle_rms(oracle_mod) <= 1.5


def _small_cts(oracle_mod, prm, okeys, msgs_torus, seed):
    """LWE encryptions under the small key (the blind rotation's input at both presets)."""
    m = np.ascontiguousarray(np.asarray(msgs_torus, dtype=np.uint64))
    out = np.zeros((m.shape[0], prm.n + 1), dtype=np.uint64)
    L = oracle_mod.lib()
    c = oracle_mod.ctypes
    L.or_lwe_encrypt(c.c_uint32(prm.n), oracle_mod._p(okeys.lwe_key), c.c_int32(prm.lwe_noise_log2), c.c_uint64(seed),
                     c.c_uint64(0), oracle_mod._p(m), c.c_size_t(m.shape[0]), oracle_mod._p(out))
    return out


PRESETS = {2: dict(mm=8, lut=lambda O, N: O.lut_constant(N, 1 << 61)),
           3: dict(mm=16, lut=lambda O, N: O.lut_from_table(N, 16, [(3 * v + 1) % 16 for v in range(16)],
                                                           (1 << 63) // 16))}


@pytest.fixture(scope="module", params=[2, 3], ids=["pgate", "pfhevm"])
def setup(request, oracle_mod):
    prm = oracle_mod.params(request.param)
    keys = oracle_mod.Keys(prm, KEY_SEED)
    return request.param, prm, keys, oracle_mod.ExactKey(prm, keys.bsk)


def test_exact_blind_rotation_decrypts(oracle_mod, setup):
    preset, prm, keys, K = setup
    N, mm = prm.N, PRESETS[preset]["mm"]
    delta = (1 << 63) // mm
    table = [(3 * v + 1) % mm for v in range(mm)]
    lut = oracle_mod.lut_from_table(N, mm, table, delta)
    msgs = [0, 1, mm // 2, mm - 1]
    cts = _small_cts(oracle_mod, prm, keys, [v * delta for v in msgs], seed=0xE2 + preset)
    for v, ct in zip(msgs, cts):
        acc = K.blind_rotate(ct, lut)
        big = oracle_mod.sample_extract_torus(prm, acc)
        ph = int(keys.phase(big, keys.glwe_key, N)[0])
        assert ((ph + delta // 2) // delta) % (2 * mm) == table[v]


def test_fft_oracle_every_cmux_within_bound_of_exact(oracle_mod, setup):
    """Teacher-forced chain: for every CMUX i of a full FFT64 blind rotation (fft_oracle.c), the state after it vs
    the exact CMUX of the state before it.  Also the accumulated FFT noise in the phase, against its model."""
    preset, prm, keys, K = setup
    N = prm.N
    lut = PRESETS[preset]["lut"](oracle_mod, N)
    ct = _small_cts(oracle_mod, prm, keys, [(1 << 61)], seed=0xE3 + preset)[0]
    tr = oracle_mod.blind_rotate_fft_trace(prm, keys, ct, lut)
    a = oracle_mod.mod_switch(ct[:prm.n], 2 * N)
    ex, s1, s2 = K.cmux(np.arange(prm.n), a, tr[:-1])
    st = fem.check_steps(oracle_mod, prm, tr[1:], ex, s1, s2)
    assert st["steps"] >= prm.n * 2 * 0.99
    # phase-domain FFT noise accumulated over the whole rotation: sum_i (D_B,i - D_A,i (*) S)
    d = fem.signed(tr[1:] - ex).reshape(prm.n, 2, N)
    e = d[:, 1].sum(axis=0) - fem.negacyclic_mul_key(d[:, 0].sum(axis=0), keys.glwe_key)
    m = fem.twiddle_rms(oracle_mod)
    sig = fem.sigma_model(N, 2 * prm.pbs_level, s2, m)
    h = int(keys.glwe_key.sum())
    var_model = float((sig[:, 1] ** 2 + h * sig[:, 0] ** 2).sum())
    ratio = math.sqrt(float((e ** 2).mean()) / var_model)
    assert 0.5 <= ratio <= 2.0, ratio
