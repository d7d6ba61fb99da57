"""Switch-and-squash / noise squashing (tfhe_amd/sns.py) on CPU: product key
generation and decryption against the oracle (oracle/sns_oracle.c), the oracle's limb-convolution NTT
against a schoolbook product, the load-time key rounding and its limb split on the native 2^128 torus,
and the oracle pipeline end to end at the full parameter set (keyswitch -> modulus-switch noise
reduction -> 128-bit bootstrap) decrypting every message with ~2^-63 noise."""
import numpy as np
import pytest

from conftest import KEY_SEED
from tfhe_amd import sns as S


def test_preset():
    sp = S.SnsParams.preset(S.SNS_PRESET_FHEVM)
    assert (sp.n, sp.k, sp.N, sp.base_log, sp.level) == (918, 2, 2048, 24, 3)


def test_keygen_and_phase_match_oracle(oracle_mod):
    sp = S.SnsParams.preset(0)
    osp = oracle_mod.sns_params(0)
    sp.n = osp.n = 12                              # key structure at a reduced input dimension
    key = np.random.default_rng(2).integers(0, 2, 12).astype(np.uint64)
    a = S.SquashedKey(sp, KEY_SEED, key)
    b = oracle_mod.SnsKeys(osp, KEY_SEED, key)
    assert np.array_equal(a.glwe_key, b.glwe_key) and np.array_equal(a.bsk, b.bsk)
    assert a.bsk.size == 12 * 9 * 3 * 2 * 2048
    cts = np.random.default_rng(3).integers(0, 2 ** 64 - 1, size=(3, 4097, 2), dtype=np.uint64)
    assert a.phase(cts) == oracle_mod.sns_phase(osp, b.glwe_key, cts)


@pytest.mark.parametrize("which", [0, 1])
def test_oracle_ntt_is_negacyclic_product(oracle_mod, which):
    N = 64
    p = [0xFFFFFFFF00000001, 0xFFFFFFFC00000001][which]
    rng = np.random.default_rng(which)
    x = rng.integers(0, 2 ** 40, N).astype(object)
    y = rng.integers(0, 2 ** 40, N).astype(object)
    want = [0] * N
    for i in range(N):
        for j in range(N):
            t = x[i] * y[j]
            if i + j < N:
                want[i + j] += t
            else:
                want[i + j - N] -= t
    X = oracle_mod.sns_ntt(which, np.array(x, dtype=np.uint64))
    Y = oracle_mod.sns_ntt(which, np.array(y, dtype=np.uint64))
    Z = np.array([(int(a) * int(b)) % p for a, b in zip(X, Y)], dtype=np.uint64)
    got = oracle_mod.sns_ntt(which, Z, inverse=True)
    assert [int(v) for v in got] == [w % p for w in want]


def test_oracle_squash_end_to_end(oracle_mod):
    prm = oracle_mod.params(1)
    ok = oracle_mod.Keys(prm, KEY_SEED, with_bsk=False)
    osp = oracle_mod.sns_params(0)
    sk = oracle_mod.SnsKeys(osp, KEY_SEED, ok.lwe_key)
    msgs = np.array([0, 5, 10, 15], dtype=np.uint64)
    big = ok.encrypt(msgs * np.uint64((1 << 63) // 16), seed=0xC0FFEE70)
    small = np.stack([oracle_mod.keyswitch(prm, ok, c) for c in big])
    small, _ = oracle_mod.ms_reduce(prm, ok, small)
    out = oracle_mod.sns_squash(osp, sk, small, 16, threads=8)
    ph = oracle_mod.sns_phase(osp, sk.glwe_key, out)
    delta = 1 << 123
    assert [((v + delta // 2) // delta) % 16 for v in ph] == [int(m) for m in msgs]
    noise = [((v - int(m) * delta + (1 << 127)) % (1 << 128)) - (1 << 127) for v, m in zip(ph, msgs)]
    assert max(abs(e) for e in noise) < 2 ** 70      # squashed: ~2^65 of the 2^128 torus


def _words(a):
    """(lo, hi) planes [..][2][N] -> python ints [..][N]"""
    a = a.reshape(-1, 2, a.shape[-1])
    return [[int(lo) | (int(hi) << 64) for lo, hi in zip(p[0], p[1])] for p in a]


def _digitrev4(p, digits=5):
    r = 0
    for _ in range(digits):
        r, p = 4 * r + (p & 3), p >> 2
    return r


def test_key_rounding_and_limbs(oracle_mod):
    """or_sns_bsk_round (the device's load-time rounding): every key word, read as a signed 128-bit
    integer, becomes the nearest multiple of 2^16 (moved by at most 2^15), so a rounded word is 2^16 x a
    112-bit integer.  or_sns_bsk_to_limb_ntt splits it into the balanced low 48 bits (limb 0, stored as the
    device's f64 spectrum / M: numpy's transform of the twisted fold, in base-4 digit-reversed order) and
    four balanced 16-bit limbs (NTTs; the inverse NTT returns the signed limbs); they recombine to the
    rounded word mod 2^128."""
    import ctypes
    osp = oracle_mod.sns_params(0)
    osp.n = 1
    keys = oracle_mod.SnsKeys(osp, KEY_SEED, np.array([1], dtype=np.uint64))
    out = np.zeros_like(keys.bsk)
    oracle_mod.lib().or_sns_bsk_round(ctypes.byref(osp), oracle_mod._p(keys.bsk), oracle_mod._p(out))
    words, rounded = _words(keys.bsk.reshape(-1, 2, 2048)), _words(out.reshape(-1, 2, 2048))
    limb = keys.bsk_limb.reshape(-1, 5, 2048)
    p1 = 0xFFFFFFFF00000001
    rng = np.random.default_rng(5)
    signed = lambda v: v - (1 << 128) if v >> 127 else v
    order = np.array([_digitrev4(q) for q in range(1024)])
    psi = np.exp(1j * np.pi * np.arange(1024) / 2048)
    for pp in rng.integers(0, len(words), 4):
        lv = [oracle_mod.sns_ntt(0, limb[pp, t].copy(), inverse=True) for t in range(1, 5)]
        low = np.zeros(2048)
        for t in range(2048):
            x, y = signed(words[pp][t]), signed(rounded[pp][t])
            assert y % 65536 == 0 and abs(y - x) <= 32768 and abs(y >> 16) < 2 ** 111
            ls = [int(v[t]) - p1 if int(v[t]) > p1 // 2 else int(v[t]) for v in lv]
            assert all(abs(v) <= 32768 for v in ls)
            up = sum(v << (64 + 16 * u) for u, v in enumerate(ls))
            m = signed((rounded[pp][t] - up) % (1 << 128))
            assert m % 65536 == 0 and abs(m >> 16) <= 2 ** 47
            low[t] = m >> 16
        spec = limb[pp, 0].view(np.float64).reshape(1024, 2)
        spec = spec[:, 0] + 1j * spec[:, 1]
        want = np.fft.ifft((low[:1024] + 1j * low[1024:]) * psi)   # sum_m z_m e^{+2 pi i m k / M} / M
        assert np.max(np.abs(spec - want[order])) <= 2 ** -40 * np.max(np.abs(want))


def test_lut_identity_native(oracle_mod):
    """The oracle's identity LUT on the 2^128 torus (one padding bit, delta = 2^127 / 16, half-box
    rotation: coefficient i holds the message of box (i + box/2) / box, the wrapped half negated); the
    device's copy (client library) is checked through the accumulators of tests/test_gpu_sns.py."""
    osp = oracle_mod.sns_params(0)
    w = _words(oracle_mod.sns_lut_identity(osp, 16).reshape(1, 2, 2048))[0]
    box, delta = 2048 // 16, (1 << 127) // 16
    for i in range(2048):
        src = i + box // 2
        want = (src // box) * delta if src < 2048 else (-(((src - 2048) // box) * delta)) % (1 << 128)
        assert w[i] == want
    assert w[box // 2] == delta and w[2047 - box // 2] == 15 * delta


def test_fft_limb_product_exactness(tmp_path):
    """tools/sns_fft_check.cpp runs the device's FFT stage functions (tfhe_amd/csrc/sns_fft.h) on the
    host: 9-term digit x 16-bit limb products (limbs 1..4; the low 48-bit limb is inexact by design and
    restated by the oracle) at N = 2048 with uniform and extreme-magnitude random operands
    land within 0.07 of the exact integers (rint() exact with margin), and the adversarial all-maximum
    operand (|value| = 2^52.2, no f64 headroom) is reported as the one inexact case."""
    import subprocess
    root = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
    exe = tmp_path / "sns_fft_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", f"{root}/tfhe_amd/csrc", f"{root}/tools/sns_fft_check.cpp",
                    "-o", str(exe)], check=True)
    for form in ("s", "w"):  # the 256-thread stage form (inverse, key conversion) and the one-wave form (step 1)
        out = subprocess.run([str(exe), "6", form], capture_output=True, text=True).stdout
        assert "stage form vs wave form spectra: max |diff| = 0.000e+00" in out
        errs = [(int(l.split()[3].rstrip(":")), float(l.split("=")[1].split(",")[0])) for l in out.splitlines()
                if l.startswith("trial")]
        assert len(errs) == 6
        assert all(e < 0.07 for mode, e in errs if mode != 2)
    out = subprocess.run([str(exe), "3", "s", "48"], capture_output=True, text=True)   # the low 48-bit limb
    assert out.returncode == 0 and "OK: below 2^34" in out.stdout, out.stdout


def test_device_arithmetic_replay_matches_oracle(tmp_path):
    """tools/sns_native_check.cpp replays the squash blind rotation on the host with the device's own
    shared code (sns_fft.h: key rounding + limb split, 128-bit decomposition, Horner recombination, the
    one-wave forward passes of step 1, the stage-form key / inverse transforms, the MAC order) and
    compares every accumulator word with oracle/sns_oracle.c (exact Goldilocks NTTs for limbs 1..4, its own
    restatement of the f64 operation order for the low limb): arbitrary 64-bit input words and a
    trivial-mask ciphertext at n = 24."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "sns_native_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", f"{root}/tfhe_amd/csrc", "-I", f"{root}/oracle",
                    f"{root}/tools/sns_native_check.cpp", "-L", f"{root}/oracle", "-loracle",
                    f"-Wl,-rpath,{root}/oracle", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "24", "3"], capture_output=True, text=True)
    assert out.returncode == 0 and "OK: device arithmetic == oracle" in out.stdout, out.stdout + out.stderr
