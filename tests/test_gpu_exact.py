"""The device's FFT64 blind rotation against EXACT integer arithmetic (oracle/exact_oracle.c), at P-GATE and P-FHEVM.

The FFT64 kernels are bit-exact against oracle/fft_oracle.c (tests/test_gpu_fft.py, test_gpu_fft2k.py), which
restates their f64 operation order.  These tests judge them with an arbiter that shares no operation order: the
exact wrapping product of the reference's computations.rs:50-54, applied to SignedDecomposer digits
(encryption.rs:152-166) in the CMUX of keyswitch_programmable_bootstrap (main.rs:71).

How a device state is obtained after exactly m CMUXes: a ciphertext whose masks a_i are zeroed for i >= m (a zero
mask switches to a~ = 0, whose CMUX is an exact identity on the device and in the oracle).  So the device's
accumulator for ct_{m+1} is the device's CMUX m applied to its accumulator for ct_m, and the exact CMUX of the
latter is the arbiter.  Checked (tests/fft_error_model.py): every compared coefficient within the derived
worst-case bound, the rms error within [0.5, 2] x the variance model, and -- over whole teacher-forced chains --
the FFT noise accumulated in the phase against its model.  Plus the committed FFT64 fixtures.
"""
import math

import numpy as np
import pytest

from conftest import KEY_SEED, load_golden
import fft_error_model as fem
from test_exact import PRESETS, _small_cts

import tfhe_amd

pytestmark = pytest.mark.gpu
LAT_DEFAULT = {2: 256, 3: 512}


@pytest.fixture(scope="module", params=[2, 3], ids=["pgate", "pfhevm"])
def env(request, oracle_mod):
    preset = request.param
    prm = oracle_mod.params(preset)
    okeys = oracle_mod.Keys(prm, KEY_SEED)
    K = oracle_mod.ExactKey(prm, okeys.bsk)
    ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(preset), KEY_SEED)
    assert np.array_equal(sk.bsk, okeys.bsk)
    eng = tfhe_amd.Engine(ck.params, 0)
    eng.load_keys(sk)
    yield preset, prm, okeys, K, eng, fem.twiddle_rms(oracle_mod)
    eng.close()


def _truncated(ct: np.ndarray, ms) -> np.ndarray:
    """copies of ct with masks a_i, i >= m, set to 0 (body kept)"""
    ms = np.asarray(ms)
    n = ct.shape[-1] - 1
    out = np.repeat(ct[None], len(ms), axis=0)
    out[:, :n][np.arange(n)[None, :] >= ms[:, None]] = 0
    return out


def test_one_cmux_64_ciphertexts_within_bound(env, oracle_mod):
    preset, prm, okeys, K, eng, m_tw = env
    N, mm = prm.N, PRESETS[preset]["mm"]
    rng = np.random.default_rng(0xE50 + preset)
    delta = (1 << 63) // mm
    cts = _small_cts(oracle_mod, prm, okeys, rng.integers(0, mm, 64).astype(np.uint64) * np.uint64(delta),
                     seed=0xE5A0 + preset)
    half = np.uint64(1 << (64 - (4 * N).bit_length() + 1))   # 2^64 / 4N: the modulus switch's rounding boundary
    for q in range(8):   # 8 ciphertexts with every mask on a boundary (odd multiple of the half step, or one below)
        t = rng.integers(0, 2 * N, prm.n).astype(np.uint64)
        cts[q, :prm.n] = (np.uint64(2) * t + np.uint64(1)) * half - np.uint64(q & 1)
    a_all = oracle_mod.mod_switch(cts[:, :prm.n], 2 * N)
    ms = np.array([rng.choice(np.nonzero(a_all[q])[0]) for q in range(64)])
    for q in range(4):                                         # include the last CMUXes of a full rotation
        ms[q] = np.nonzero(a_all[q])[0][-1 - q]
    batch = np.concatenate([_truncated(cts[q], [ms[q], ms[q] + 1]) for q in range(64)])
    lut = PRESETS[preset]["lut"](oracle_mod, N)
    try:
        for lat in (0, 1 << 20):                               # the batch kernel, then the latency kernel
            eng.set_latency_batch(lat)
            acc = eng.blind_rotate(batch, lut)
            ex, s1, s2 = K.cmux(ms, a_all[np.arange(64), ms], acc[0::2])
            st = fem.check_steps(oracle_mod, prm, acc[1::2], ex, s1, s2, m_tw)
            assert st["steps"] == 128
            print(f"preset {preset} lat {lat}: {st}")
    finally:
        eng.set_latency_batch(LAT_DEFAULT[preset])


def test_full_rotation_teacher_forced_every_cmux(env, oracle_mod):
    """Every CMUX of whole device blind rotations (4 ciphertexts at P-GATE, 2 at P-FHEVM) vs the exact CMUX of the
    device's own previous state; the device chain equals the FFT64 oracle's trace word for word; the FFT noise
    accumulated in the phase over the rotation matches its model (its size against the decision margin is the
    FFT's share of the failure probability)."""
    preset, prm, okeys, K, eng, m_tw = env
    N, mm = prm.N, PRESETS[preset]["mm"]
    nct = 4 if preset == 2 else 2
    delta = (1 << 63) // mm
    cts = _small_cts(oracle_mod, prm, okeys, [(v * delta) for v in range(nct)], seed=0xE6A0 + preset)
    lut = PRESETS[preset]["lut"](oracle_mod, N)
    ms = np.arange(prm.n + 1)
    acc = eng.blind_rotate(np.concatenate([_truncated(c, ms) for c in cts]), lut).reshape(nct, prm.n + 1, -1)
    assert np.array_equal(acc[0], oracle_mod.blind_rotate_fft_trace(prm, okeys, cts[0], lut))
    full = eng.blind_rotate(cts, lut)
    assert np.array_equal(full, acc[:, -1])
    h = int(okeys.glwe_key.sum())
    for q in range(nct):
        a = oracle_mod.mod_switch(cts[q, :prm.n], 2 * N)
        ex, s1, s2 = K.cmux(np.arange(prm.n), a, acc[q, :-1])
        st = fem.check_steps(oracle_mod, prm, acc[q, 1:], ex, s1, s2, m_tw)
        d = fem.signed(acc[q, 1:] - ex).reshape(prm.n, 2, N)
        e = d[:, 1].sum(axis=0) - fem.negacyclic_mul_key(d[:, 0].sum(axis=0), okeys.glwe_key)
        sig = fem.sigma_model(N, 2 * prm.pbs_level, s2, m_tw)
        ratio = math.sqrt(float((e ** 2).mean()) / float((sig[:, 1] ** 2 + h * sig[:, 0] ** 2).sum()))
        assert 0.5 <= ratio <= 2.0, ratio
        margin = math.log2(delta // 2) - 0.5 * math.log2(float((e ** 2).mean()))
        print(f"preset {preset} ct {q}: {st}; phase FFT noise rms 2^{0.5 * math.log2(float((e ** 2).mean())):.2f} "
              f"(model ratio {ratio:.2f}), decision half-interval / rms = 2^{margin:.1f}")


@pytest.mark.parametrize("name", ["fft64_gate.npz", "fft64_fhevm.npz"])
def test_golden_fft64_fixtures(name):
    """The device against the committed FFT64 fixtures (tests/golden/make_golden_fft64.py)."""
    g = load_golden(name)
    preset = int(g["preset"])
    ck, sk = tfhe_amd.gen_keys(tfhe_amd.Params.preset(preset), int(g["key_seed"]))
    with tfhe_amd.Engine(ck.params, 0) as eng:
        eng.load_keys(sk)
        bri = g["small"] if "small" in g else g["lwe_in"]
        if "small" in g:
            assert np.array_equal(eng.keyswitch(g["lwe_in"]), bri)
        for lat in (0, 1 << 20):
            eng.set_latency_batch(lat)
            assert np.array_equal(eng.blind_rotate(bri, g["luts"], g["lut_index"]), g["acc"])
            assert np.array_equal(eng.pbs(g["lwe_in"], g["luts"], g["lut_index"]), g["lwe_out"])
